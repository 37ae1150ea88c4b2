"""Serving: micro-batched REST prediction service, online bandit service over SPSC rings."""
import json
import threading
import urllib.request

import numpy as np
import torch

from avenir_amd.models.bandit import BanditBank
from avenir_amd.serve import BanditService, MicroBatcher, PredictionServer, parse_recs, simulate_lead_generation


def _get(url):
    with urllib.request.urlopen(url, timeout=30) as r:
        return json.loads(r.read())


def _post(url, obj):
    req = urllib.request.Request(url, data=json.dumps(obj).encode(), headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=30) as r:
        return json.loads(r.read())


def test_parse_recs():
    X = parse_recs("a,1,2,,b,3,4", [1, 2])
    assert X.tolist() == [[1.0, 2.0], [3.0, 4.0]]


def test_micro_batcher_coalesces():
    calls = []

    def fn(X):
        calls.append(X.shape[0])
        p = torch.sigmoid(torch.as_tensor(X).sum(1))
        return torch.stack([1 - p, p], 1)
    mb = MicroBatcher(fn, max_batch=1000, max_wait_ms=50)
    futs = [mb.submit(np.full((2, 3), i, dtype=np.float32)) for i in range(20)]
    res = [f.result(timeout=10) for f in futs]
    assert len(res) == 20 and all(len(r) == 2 for r in res)
    assert len(calls) < 20 and sum(calls) == 40
    mb.close()


def test_prediction_server_routes():
    srv = PredictionServer(max_wait_ms=5)
    w = torch.tensor([1.0, -1.0])
    srv.register("rf", lambda X: torch.stack([1 - torch.sigmoid(torch.as_tensor(X) @ w),
                                              torch.sigmoid(torch.as_tensor(X) @ w)], 1), [1, 2])
    port = srv.start(0)
    base = f"http://127.0.0.1:{port}"
    r = _get(f"{base}/rf/predict/x,2,0,,y,0,2")
    p = [float(v) for v in r["predictions"].split(",")]
    assert p[0] > 0.8 and p[1] < 0.2
    r2 = _post(f"{base}/rf/predict/batch", {"recs": "x,2,0,,y,0,2"})
    assert r2 == r
    # concurrent clients share device batches
    out = []
    ths = [threading.Thread(target=lambda: out.append(_get(f"{base}/rf/predict/x,1,1"))) for _ in range(16)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    assert len(out) == 16 and srv.models["rf"][0].batches < 18
    try:
        _get(f"{base}/nope/predict/1,2")
        raise AssertionError("expected 404")
    except urllib.error.HTTPError as e:
        assert e.code == 404
    bank = BanditBank("randomGreedy", ["a", "b"], config={"random.selection.prob": 0.1})
    srv.register_bandit(BanditService(bank))
    assert _post(f"{base}/bandit/event", {"eventID": 7})["accepted"]
    acts = _get(f"{base}/bandit/actions")["actions"]
    assert acts[0].startswith("7,")
    assert _post(f"{base}/bandit/reward", {"action": "a", "reward": 5.0})["accepted"]
    srv.shutdown()


def test_bandit_service_learns_best_arm(tmp_path):
    bank = BanditBank("upperConfidenceBoundOne", ["p1", "p2", "p3"], config={"reward.scale": 100.0})
    svc = BanditService(bank)
    res = simulate_lead_generation(svc, {"p1": 0.05, "p2": 0.30, "p3": 0.10}, n_rounds=60, events_per_round=40)
    assert res["shown"]["p2"] > res["shown"]["p1"] and res["shown"]["p2"] > res["shown"]["p3"]
    assert svc.stats["events"] == 2400 and svc.stats["batches"] == 60
    p = tmp_path / "bandit.txt"
    svc.checkpoint(p)
    bank2 = BanditBank("upperConfidenceBoundOne", ["p1", "p2", "p3"], config={"reward.scale": 100.0})
    svc2 = BanditService(bank2)
    svc2.restore(p)
    assert torch.equal(bank2.trials, bank.trials)


def test_bandit_service_groups_and_thread():
    bank = BanditBank("softMax", ["x", "y"], n_groups=4, config={"temp.constant": 10})
    svc = BanditService(bank).start()
    for i in range(200):
        assert svc.submit_event(i, i % 4)
    import time
    t0 = time.time()
    got = []
    while len(got) < 200 and time.time() - t0 < 10:
        got += svc.actions()
        time.sleep(0.01)
    svc.stop()
    assert sorted(e for e, _ in got) == list(range(200))
