#!/usr/bin/env python3
"""Flagship benchmark: distributed Naive Bayes training throughput (rows/s summed over all GPUs).

BASELINE.json names no metric (the reference publishes no numbers), so the
headline is the one BASELINE.md lists first and SURVEY.md §7.3 names as the minimum end-to-end
slice: Naive Bayes churn-model training (``BayesianDistribution``) on the ``resource/churn.json``
schema — 5 categorical features, 2 classes.

One step = one complete training pass over this rank's shard: the K2 class-conditional histogram
(HIP joint-table kernel: one LDS atomic per record, marginals per block) + class counts over
``rows_per_gpu`` records, ONE RCCL
all-reduce of the [C, TB+1] count table, and the model finalisation (log-probability tables for
the predictor).  Weak scaling: every GPU owns ``rows_per_gpu`` synthetic records (same
distributions as the reference's ``usage.rb``), generated on device before timing.

The records are held on device packed once at load time, losslessly (``--layout rowpacked``: the
5 codes + one-hot class of a record in 13 bits, streamed as a dense 13-bit record stream; the
16-bit word form is kept too) or as uint8 code columns (``--layout columns``).
CSV parsing and packing are NOT in the timed steps (the headline is the on-device training pass);
``extra`` reports them separately:

* ``columns_rows_per_s_per_gpu`` — the same training step over the uint8 code columns.
* ``ingest`` (``--ingest-rows``; default 2^26 records on one GPU, 2^24 per rank on more) — the
  end-to-end job time for a CSV file written beforehand: native K1 parse -> device -> fit -> model
  text lines; on several GPUs every rank ingests its own file and ``job_rows_per_s`` is the total
  over the slowest rank's time.
* ``rccl_all_reduce`` (more than one GPU) — all-reduce latency at 8 KB and bus bandwidth at
  1 MB / 64 MB over the job's GPUs, next to the deterministic all-gather path and the hand-written
  peer-mapped one-shot / two-shot kernels (``algo="p2p"``, csrc/kernels/comm.hip).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--rows-per-gpu R] [--layout L]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def _timed(fn, dev) -> float:
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return time.perf_counter() - t0


def _allreduce_probe(comm, dev) -> list:
    """RCCL all-reduce over this job's GPUs (outside the timed steps): latency of a KB-scale
    count-table-sized message and bus bandwidth (algbw x 2(n-1)/n) at 1 MB and 64 MB."""
    import torch.distributed as dist
    out = []
    W = comm.world
    for nbytes, iters in ((8 << 10, 50), (1 << 20, 20), (64 << 20, 10)):
        x = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
        for _ in range(3):
            dist.all_reduce(x)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()
        t = _timed(lambda: [dist.all_reduce(x) for _ in range(iters)], dev) / iters
        t = comm.reduce_max_scalar(t)
        alg = nbytes / t / 1e9
        out.append({"bytes": nbytes, "us": t * 1e6, "algbw_GBps": alg, "busbw_GBps": alg * 2 * (W - 1) / W})
    # deterministic small-message path (RCCL all-gather + rank-ordered local sum) at the count-table size
    for nbytes, iters in ((8 << 10, 50), (64 << 10, 50)):
        x = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
        for _ in range(3):
            comm.all_reduce(x, algo="oneshot")
        comm.barrier()
        t = _timed(lambda: [comm.all_reduce(x, algo="oneshot") for _ in range(iters)], dev) / iters
        t = comm.reduce_max_scalar(t)
        out.append({"bytes": nbytes, "algo": "allgather_ordered_sum", "us": t * 1e6})
    # hand-written peer-mapped kernels (csrc/kernels/comm.hip): one-shot / two-shot over xGMI
    # (construction agrees over ranks and raises on all of them together; the kernels' waits are
    # bounded, so a rank out of step shows as a status word, and every rank reaches every collective)
    p = comm.p2p()                  # collective; None on every rank together when unavailable
    if p is None:
        out.append({"algo": "p2p", "error": "peer-mapped all-reduce unavailable on this node"})
        return out
    for nbytes, iters in ((8 << 10, 100), (64 << 10, 100), (1 << 20, 50)):
        x = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
        for _ in range(5):
            comm.all_reduce(x, algo="p2p")
        f = torch.tensor([1 if p.ok() else 0], device=dev)
        comm.all_reduce(f, "min", algo="ring")
        if not bool(f.item()):                      # out of step: every later call would wait out its bound
            out.append({"bytes": nbytes, "algo": "p2p", "error": "a bounded wait timed out on some rank"})
            break
        comm.barrier()
        t = _timed(lambda: [comm.all_reduce(x, algo="p2p") for _ in range(iters)], dev) / iters
        x.fill_(float(comm.rank + 1))
        comm.all_reduce(x, algo="p2p")
        exact = bool((x == float(W * (W + 1) // 2)).all().item()) and p.ok()
        t = comm.reduce_max_scalar(t)
        out.append({"bytes": nbytes, "algo": "p2p_" + ("oneshot" if nbytes <= p.oneshot_max else "twoshot"),
                    "us": t * 1e6, "exact": exact})
    return out


def _pick_small_allreduce(comm, like: torch.Tensor, mode: str) -> dict:
    """Choose the algorithm of the model's count-table all-reduce on this job's GPUs, before the
    timed steps: the hand-written peer-mapped kernel (``p2p``) is taken only if it is exact on an
    integer probe, its status is clean on every rank, and it is faster than RCCL at the table's
    size (max over ranks).  ``mode``: auto | rccl | p2p."""
    info = {"mode": mode, "bytes": like.numel() * like.element_size()}
    if mode == "rccl" or comm.world == 1 or like.device.type != "cuda":
        info["chosen"] = "rccl"
        comm.small_allreduce = None
        return info
    if mode == "auto":
        # the communicator's own default selection (Comm._auto_small_allreduce), made at the
        # first count-table all-reduce of the sizing fit — the same probe every job runs
        info.update(comm.small_allreduce_probe or {})
        info["chosen"] = "p2p" if comm.small_allreduce == "p2p" else "rccl"
        return info
    W = comm.world
    x = torch.empty_like(like)

    def agree(ok: bool) -> bool:                      # every rank takes the same branch
        f = torch.tensor([1 if ok else 0], device=like.device)
        comm.all_reduce(f, "min", algo="ring")
        return bool(f.item())

    # Every step below is either a kernel (bounded waits: a peer that is out of step sets a status
    # word, never hangs) or a collective that ALL ranks reach: a failure on one rank is carried by
    # the agreement all-reduces, never by an exception that would skip a collective on that rank.
    use = False
    p = comm.p2p()                                    # collective; None on every rank together
    if p is None:
        info["p2p_error"] = "peer-mapped all-reduce unavailable on this node"
    else:
        ok = True
        for i in range(20):
            x.fill_(comm.rank + 1 + i)
            comm.all_reduce(x, algo="p2p")
            ok &= bool((x == W * (W + 1) // 2 + W * i).all().item())
            if i == 0 and not agree(ok and p.ok()):   # out of step: stop before 19 more bounded waits
                ok = False
                break
        info["p2p_exact"] = agree(ok and p.ok())
        if info["p2p_exact"]:
            times = {}
            for name, fn in (("rccl", lambda: comm.all_reduce(x, algo="ring")),
                             ("p2p", lambda: comm.all_reduce(x, algo="p2p"))):
                for _ in range(5):
                    fn()
                comm.barrier()
                times[name] = comm.reduce_max_scalar(_timed(lambda: [fn() for _ in range(50)], like.device) / 50)
            info.update({f"{k}_us": v * 1e6 for k, v in times.items()})
            use = agree(p.ok()) and (mode == "p2p" or times["p2p"] < times["rccl"])
    info["chosen"] = "p2p" if use else "rccl"
    comm.small_allreduce = "p2p" if info["chosen"] == "p2p" else None
    return info


def _comm_selftest(comm, dev) -> dict:
    """The library collectives other than all-reduce that the framework's jobs use, run on THIS
    job's GPUs (RCCL over xGMI when the driver launches several ranks), checked for content and
    timed (max over ranks): the systolic ring of recordSimilarity / the kNN joins
    (``ring_pass_start`` = one ``batch_isend_irecv`` group, and ``ring_iter``), the uneven
    ``all_to_all_single`` of ``all_to_all_v`` / ``fetch_rows``, ``all_gather_v`` and
    ``barrier(device_ids=...)``.  Runs after the timed steps."""
    W, r = comm.world, comm.rank
    out = {}
    # ring: 64 MiB per rank -> per-link bandwidth of the neighbour exchange
    n = 16 << 20
    x = torch.full((n,), float(r), device=dev)
    y = comm.ring_pass_finish(comm.ring_pass_start(x, n))
    ok = bool((y == float((r - 1) % W)).all().item())
    comm.barrier()
    t = comm.reduce_max_scalar(_timed(lambda: [comm.ring_pass_finish(comm.ring_pass_start(x, n)) for _ in range(5)], dev) / 5)
    out["ring_batch_isend_irecv"] = {"ok": ok, "bytes": 4 * n, "ms": t * 1e3, "GBps": 4 * n / t / 1e9}
    del x, y
    # ring_iter over two tensors of rank-dependent length
    blocks = [torch.full((r + 3, 4), r, dtype=torch.int64, device=dev), torch.full((r + 3,), 2.0 * r, device=dev)]
    seen, ok = [], True
    for owner, blk in comm.ring_iter(blocks):
        seen.append(owner)
        ok &= blk[0].shape[0] == owner + 3 and bool((blk[0] == owner).all().item()) and bool((blk[1] == 2.0 * owner).all().item())
    out["ring_iter"] = {"ok": bool(ok and seen == [(r - s) % W for s in range(W)])}
    # uneven all-to-all: rank a sends cnt(a, b) rows [a, b, i] to rank b; large uneven pass timed
    cnt = lambda a, b: 1 + (7 * a + 3 * b) % 11
    chunks = [torch.stack([torch.full((cnt(r, b),), r), torch.full((cnt(r, b),), b), torch.arange(cnt(r, b))], 1).to(dev)
              for b in range(W)]
    got = comm.all_to_all_v(chunks)
    ok = all(g.shape[0] == cnt(a, r) and bool((g[:, 0] == a).all().item()) and bool((g[:, 1] == r).all().item())
             and bool((g[:, 2] == torch.arange(cnt(a, r), device=dev)).all().item()) for a, g in enumerate(got))
    big = [torch.full(((1 << 18) * (1 + (r + b) % 3), 16), float(r), device=dev) for b in range(W)]
    comm.all_to_all_v(big)
    comm.barrier()
    t = comm.reduce_max_scalar(_timed(lambda: [comm.all_to_all_v(big) for _ in range(3)], dev) / 3)
    sent = sum(c.numel() * 4 for c in big)
    out["all_to_all_v"] = {"ok": bool(ok), "bytes_sent_per_rank": sent, "ms": t * 1e3, "GBps_per_rank": sent / t / 1e9}
    del big
    g = comm.all_gather_v(torch.full((r + 1, 3), r, dtype=torch.int32, device=dev))
    ref = torch.cat([torch.full((a + 1, 3), a, dtype=torch.int32) for a in range(W)])
    out["all_gather_v"] = {"ok": bool(torch.equal(g.cpu(), ref))}
    comm.barrier()
    t = comm.reduce_max_scalar(_timed(lambda: [comm.barrier() for _ in range(20)], dev) / 20)
    out["barrier"] = {"ok": True, "us": t * 1e6}
    out["ok"] = all(v.get("ok", False) for v in out.values() if isinstance(v, dict))
    return out


def _ingest(rows: int, schema, dev, comm) -> dict:
    """CSV file -> ``load_csv`` (native K1 parse, device upload) -> fit -> model lines, every rank on
    its own file of ``rows`` records (written before timing, outside the clock)."""
    import tempfile

    from avenir_amd.data import synth
    from avenir_amd.data.table import load_csv
    from avenir_amd.models.bayes import NaiveBayes

    d = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    path = os.path.join(d, f"avmi_bench_churn_{os.getpid()}_{comm.rank}.csv")
    try:
        nbytes = synth.write_churn_native(path, rows, seed=99 + comm.rank)
        # page cache warm, as for a file just produced by the previous stage of a pipeline
        with open(path, "rb") as fh:
            while fh.read(1 << 26):
                pass
        out = {}
        t = None

        def load():
            nonlocal t
            t = load_csv(path, schema, device=dev, rank=0, world=1)
        # the first load of a process also allocates the pinned staging ring (one-time, reported
        # apart); the job rate is a full re-parse + upload of the file on a warm process
        out["first_load_s"] = _timed(load, dev)
        t = None
        out["load_s"] = _timed(load, dev)
        nb = NaiveBayes(schema, comm=comm)        # one distributed job: the fit all-reduces the counts
        out["fit_s"] = _timed(lambda: nb.fit(t), dev)
        lines = []
        out["model_lines_s"] = _timed(lambda: lines.extend(nb.model_lines()), dev)
        assert int(nb.class_n.sum().item()) == rows * comm.world
        total = out["load_s"] + out["fit_s"] + out["model_lines_s"]
        cold = out["first_load_s"] + out["fit_s"] + out["model_lines_s"]
        out.update(rows=rows, file_bytes=nbytes, total_s=total, rows_per_s=rows / total,
                   cold_total_s=cold, cold_rows_per_s=rows / cold,
                   parse_gbps=nbytes / out["load_s"] / 1e9, model_lines=len(lines),
                   parser=str((getattr(t, "meta", None) or {}).get("parser", "unknown")))
        return out
    finally:
        if os.path.exists(path):
            os.remove(path)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows-per-gpu", type=int, default=1 << 30)
    ap.add_argument("--predict", action="store_true", help="also time batched inference")
    ap.add_argument("--layout", choices=["rowpacked", "columns"], default="rowpacked",
                    help="device layout of the encoded records: one 16-bit word per record "
                         "(2 B/record) or one uint8 column per feature + label (6 B/record)")
    ap.add_argument("--small-allreduce", choices=["auto", "rccl", "p2p"], default="auto",
                    help="algorithm of the count-table all-reduce on >1 GPU: auto = the communicator's "
                         "default selection (the faster of RCCL and the hand-written peer-mapped "
                         "kernel if it is exact, probed on the job's GPUs at the first such all-reduce)")
    ap.add_argument("--probe-allreduce", action="store_true",
                    help="run the all-reduce probe on any device (it runs by default on >1 GPU)")
    ap.add_argument("--ingest-rows", type=int, default=-1,
                    help="rows per rank of the ingest-inclusive CSV measurement (0 = skip; default 2^26 "
                         "on a single GPU, 2^24 per rank on more)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE",
              file=sys.stderr)

    import avenir_amd
    from avenir_amd.data.synth import CHURN_SCHEMA, churn_device
    from avenir_amd.data.table import Table
    from avenir_amd.models.bayes import NaiveBayes
    from avenir_amd.parallel.comm import get_comm
    from avenir_amd.utils.schema import FeatureSchema

    avenir_amd.freeze_startup_objects()
    comm = get_comm()
    dev = comm.device
    if dev.type != "cuda":
        print("[bench] no GPU visible: running on CPU with a tiny problem", file=sys.stderr)
        args.rows_per_gpu = min(args.rows_per_gpu, 1 << 16)
    n = int(args.rows_per_gpu)
    schema = FeatureSchema.from_json(CHURN_SCHEMA)
    codes, labels = churn_device(n, seed=1234 + comm.rank, device=dev)
    feats = schema.feature_fields
    table = Table(schema, n, codes, feats, torch.zeros((0, codes.shape[1]), device=dev), [],
                  labels, schema.find_class_attr_field())
    bytes_per_row = codes.shape[0] + 1  # 5 feature codes + 1 label byte
    if args.layout == "rowpacked":
        # lossless re-encoding done once at load time, like the dictionary encoding itself
        table.pack_rows()
        if table.rowpack is None:
            print("[bench] schema does not fit 16-bit records: using code columns", file=sys.stderr)
            args.layout = "columns"
        else:
            rp = table.rowpack
            bytes_per_row = rp.bits / 8.0 if getattr(rp, "dense", None) is not None else 2
    nb = NaiveBayes(schema, comm=comm)

    def step():
        # one training step = count + (multi-GPU) all-reduce + fused finalize into the log-prob
        # tables; a GPU fit builds the tables itself, and with >1 rank the all-reduce + finalize
        # run on a side stream that overlaps the next step's histogram (models/bayes.py)
        nb.fit(table)

    allreduce_choice = None
    if comm.world > 1:
        nb.fit(table)                     # sizes the count table
        allreduce_choice = _pick_small_allreduce(comm, nb._both, args.small_allreduce)
    for _ in range(args.warmup):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    comm.check()                          # a failed peer-mapped sum in the timed steps raises here
    dt = comm.reduce_max_scalar(dt)

    # sanity: the model must have counted every record of every rank in the last step
    total_rows = int(nb.class_n.sum().item())
    assert total_rows == n * comm.world, (total_rows, n * comm.world)

    ms = dt * 1000.0 / args.steps
    rows_per_s = n * comm.world * args.steps / dt
    extra = {"layout": args.layout, "ms_per_step": ms, "count_allreduce": allreduce_choice, "hbm_gbps_per_gpu": n * bytes_per_row / (ms / 1000.0) / 1e9}
    if args.layout == "rowpacked" and table.rowpack is not None:
        rp, table.rowpack = table.rowpack, None
        k = max(1, min(args.steps, 5))
        step()
        t1 = _timed(lambda: [step() for _ in range(k)], dev)
        extra["columns_rows_per_s_per_gpu"] = n * k / t1
        extra["columns_hbm_gbps_per_gpu"] = n * (codes.shape[0] + 1) * k / t1 / 1e9
        table.rowpack = rp
    if comm.world > 1 and (dev.type == "cuda" or args.probe_allreduce):
        try:
            extra["rccl_all_reduce"] = _allreduce_probe(comm, dev)
        except Exception as e:      # a probe failure must not lose the measured headline
            extra["rccl_all_reduce"] = {"error": repr(e)}
        if os.environ.get("AVMI_BENCH_COMM_SELFTEST", "1") != "0":
            try:
                extra["comm_selftest"] = _comm_selftest(comm, dev)
            except Exception as e:
                extra["comm_selftest"] = {"error": repr(e)}
    # every rank ingests its own file (2^26 records on one GPU; 2^24 per rank on more, so 8 ranks'
    # files fit /dev/shm together); the job's rate is the sum of records over the SLOWEST rank's time
    ingest_rows = args.ingest_rows if args.ingest_rows >= 0 else ((1 << 26) if comm.world == 1 else (1 << 24))
    if ingest_rows > 0 and (dev.type == "cuda" or args.ingest_rows > 0):
        try:
            comm.barrier()
            ing = _ingest(ingest_rows, schema, dev, comm)
            if comm.world > 1:
                for k in ("total_s", "cold_total_s", "load_s", "first_load_s"):
                    ing[k] = comm.reduce_max_scalar(float(ing[k]))
                ing["job_rows"] = ingest_rows * comm.world
                ing["job_rows_per_s"] = ingest_rows * comm.world / ing["total_s"]
                ing["job_cold_rows_per_s"] = ingest_rows * comm.world / ing["cold_total_s"]
            extra["ingest"] = ing
        except Exception as e:      # the ingest extra must never cost the measured headline
            extra["ingest"] = {"error": repr(e)}
    if args.predict:
        pr_n = min(n, 1 << 26)
        sub = Table(schema, pr_n, codes[:, : ((pr_n + 15) // 16) * 16].contiguous(), feats,
                    torch.zeros((0, 16), device=dev), [], labels[: ((pr_n + 15) // 16) * 16].contiguous(),
                    schema.find_class_attr_field())
        nb.predict(sub, with_prob=True)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(5):
            nb.predict(sub, with_prob=True)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        extra["predict_rows_per_s_per_gpu"] = pr_n * 5 / (time.perf_counter() - t1)

    if comm.rank == 0:
        out = {
            "metric": "naive_bayes_train_rows_per_s",
            "value": rows_per_s,
            "unit": "rows/s",
            "n_gpus": comm.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": (f"row-packed categorical records ({bytes_per_row * 8:g}-bit records, lossless)/int64 counts (exact)"
                      if args.layout == "rowpacked" else "uint8-codes/int64-counts (exact integer counting)"),
            "data": "synthetic (device-generated, resource/usage.rb distributions)",
            "config": {
                "model": "NaiveBayes(resource/churn.json: 5 categorical features, 2 classes)",
                "global_batch": n * comm.world,
                "rows_per_gpu": n,
                "seq_len": None,
                "parallelism": f"dp{comm.world}",
            },
            "extra": extra,
        }
        print(json.dumps(out))
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
