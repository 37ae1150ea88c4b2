"""REST prediction service with request micro-batching.

Reference: Flask services ``rfsvc.py`` / ``gbtsvc.py`` / ``svmsvc.py`` (P/app/rfsvc.py:36-70):
``GET /<model>/predict/<recs>`` (records separated by ``,,``) and ``GET|POST /<model>/predict/batch``
(``{"recs": "..."}``) returning ``{"predictions": "p1,p2,..."}`` = predictProb[:, 1]; the model is
built lazily from its config and cached; clients in rfclnt.py / gbtclnt.py and the Spark ICE job
(S/interpret/IndividualConditionalExpectation.scala:112-134).

MI355X design: models stay resident on the device; concurrent requests for the same model are
coalesced by a batcher thread (up to ``max_batch`` records or ``max_wait_ms``) into ONE device
inference call, then scattered back to the waiting requests.  Also exposes the online bandit
service (``/bandit/event``, ``/bandit/reward``, ``/bandit/actions``) in place of the Redis queues.
Standard library HTTP server, JSON wire format unchanged.
"""
from __future__ import annotations

import json
import queue
import threading
import time
from concurrent.futures import Future
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable
from urllib.parse import unquote

import numpy as np
import torch


class MicroBatcher:
    """Coalesce predict calls: ``submit(rows [n, F]) -> Future`` of ``probs [n]``."""

    def __init__(self, predict_proba: Callable, max_batch: int = 4096, max_wait_ms: float = 2.0):
        self.fn = predict_proba
        self.max_batch, self.max_wait = max_batch, max_wait_ms / 1000.0
        self.q: queue.Queue = queue.Queue()
        self.batches = 0
        self._t = threading.Thread(target=self._loop, daemon=True)
        self._t.start()

    def submit(self, rows: np.ndarray) -> Future:
        f: Future = Future()
        self.q.put((rows, f))
        return f

    def _loop(self):
        while True:
            first = self.q.get()
            if first is None:
                return
            items = [first]
            n = first[0].shape[0]
            deadline = time.monotonic() + self.max_wait
            while n < self.max_batch:
                rem = deadline - time.monotonic()
                if rem <= 0:
                    break
                try:
                    it = self.q.get(timeout=rem)
                except queue.Empty:
                    break
                if it is None:
                    self.q.put(None)
                    break
                items.append(it)
                n += it[0].shape[0]
            try:
                X = np.concatenate([r for r, _ in items], 0)
                P = torch.as_tensor(self.fn(X)).float().cpu()
                p1 = P[:, 1] if P.dim() == 2 and P.shape[1] > 1 else P.view(-1)
                o = 0
                for r, f in items:
                    f.set_result(p1[o:o + r.shape[0]].tolist())
                    o += r.shape[0]
                self.batches += 1
            except Exception as e:  # noqa: BLE001
                for _, f in items:
                    if not f.done():
                        f.set_exception(e)

    def close(self):
        self.q.put(None)


def parse_recs(recs: str, feature_fields: list[int] | None = None) -> np.ndarray:
    rows = [r.split(",") for r in recs.split(",,") if r.strip()]
    if feature_fields:
        return np.array([[float(r[i]) for i in feature_fields] for r in rows], dtype=np.float32)
    return np.array([[float(v) for v in r] for r in rows], dtype=np.float32)


class PredictionServer:
    """``register(name, predict_proba, feature_fields)``; ``serve(port)`` blocks, ``start(port)``
    runs in a background thread and returns the bound port."""

    def __init__(self, max_batch: int = 4096, max_wait_ms: float = 2.0):
        self.models: dict[str, tuple[MicroBatcher, list[int] | None]] = {}
        self.lazy: dict[str, Callable] = {}
        self.bandit = None
        self.max_batch, self.max_wait = max_batch, max_wait_ms
        self.httpd: ThreadingHTTPServer | None = None
        self._lock = threading.Lock()

    def register(self, name: str, predict_proba: Callable, feature_fields: list[int] | None = None):
        self.models[name] = (MicroBatcher(predict_proba, self.max_batch, self.max_wait), feature_fields)

    def register_lazy(self, name: str, factory: Callable[[], tuple[Callable, list[int] | None]]):
        """Model built on first request (the reference's getClassifier cache)."""
        self.lazy[name] = factory

    def register_bandit(self, service):
        self.bandit = service

    def _model(self, name):
        with self._lock:
            if name not in self.models and name in self.lazy:
                fn, ff = self.lazy.pop(name)()
                self.register(name, fn, ff)
        return self.models[name]

    def predict(self, name: str, recs: str) -> dict:
        mb, ff = self._model(name)
        probs = mb.submit(parse_recs(recs, ff)).result(timeout=60)
        return {"predictions": ",".join(f"{p:.3f}" for p in probs)}

    def _handler(self):
        server = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, obj):
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _route(self, payload: dict | None):
                parts = [unquote(p) for p in self.path.split("?")[0].strip("/").split("/")]
                try:
                    if parts[0] == "bandit" and server.bandit is not None:
                        return self._bandit(parts, payload or {})
                    if len(parts) >= 3 and parts[1] == "predict":
                        name = parts[0]
                        if parts[2] == "batch":
                            recs = (payload or {}).get("recs")
                            if recs is None and "?" in self.path:
                                q = dict(kv.split("=", 1) for kv in self.path.split("?", 1)[1].split("&"))
                                recs = unquote(q.get("recs", ""))
                        else:
                            recs = "/".join(parts[2:])
                        return self._send(200, server.predict(name, recs))
                    return self._send(404, {"error": "not found"})
                except KeyError as e:
                    return self._send(404, {"error": f"unknown model {e}"})
                except Exception as e:  # noqa: BLE001
                    return self._send(500, {"error": str(e)})

            def _bandit(self, parts, payload):
                svc = server.bandit
                if parts[1] == "event":
                    ok = svc.submit_event(int(payload["eventID"]), int(payload.get("group", 0)))
                    return self._send(200, {"accepted": bool(ok)})
                if parts[1] == "reward":
                    ok = svc.submit_reward(payload["action"], float(payload["reward"]), int(payload.get("group", 0)))
                    return self._send(200, {"accepted": bool(ok)})
                if parts[1] == "actions":
                    svc.step()
                    return self._send(200, {"actions": [f"{e},{a}" for e, a in svc.actions()]})
                return self._send(404, {"error": "unknown bandit route"})

            def do_GET(self):
                self._route(None)

            def do_POST(self):
                n = int(self.headers.get("Content-Length", 0) or 0)
                payload = json.loads(self.rfile.read(n) or b"{}") if n else {}
                self._route(payload)

        return H

    def start(self, port: int = 0, host: str = "127.0.0.1") -> int:
        self.httpd = ThreadingHTTPServer((host, port), self._handler())
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return self.httpd.server_address[1]

    def serve(self, port: int, host: str = "127.0.0.1"):
        self.httpd = ThreadingHTTPServer((host, port), self._handler())
        self.httpd.serve_forever()

    def shutdown(self):
        if self.httpd is not None:
            self.httpd.shutdown()
            self.httpd.server_close()
        for mb, _ in self.models.values():
            mb.close()


def classifier_factory(kind: str, config):
    """Lazy factory for a config-driven classifier (rf | gbt | svm | lr) -> (predict_proba, features)."""
    from ..models import supervised as SV

    def make():
        cls = {"rf": SV.RandomForest, "gbt": SV.GradientBoostedTrees, "svm": SV.SupportVectorMachine,
               "lr": SV.LogisticRegressionDiscriminant}[kind]
        c = cls(config)
        c._ensure_model()
        return c.model.predict_proba, c._ints("predict.data.feature.fields")
    return make
