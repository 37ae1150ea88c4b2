#!/usr/bin/env python3
"""Measurements for the kernel rows of README's table that had none: K17 Apriori support
(assoc.hip), K18 GSP candidate join (gsp.hip), K20 bandit selection (bandit.hip), K24 streaming PCA
(pca.hip).  Each is timed against the framework's own non-kernel path of the same op (the torch /
host oracle the tests compare it with), on the same box; one JSON line per case.

    python benchmarks/bench_r5_kernels.py [apriori gsp bandit spirit]
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn, reps=5, dev=True):
    fn()
    if dev:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    if dev:
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def emit(**kw):
    print(json.dumps(kw), flush=True)


def apriori():
    """Support of 8,192 candidate 2-sets over 2^22 transactions (65,536 words per bit row): every
    candidate ANDs two 512 KiB rows and popcounts them."""
    from avenir_amd.models.association import _POP8, itemset_support
    g = torch.Generator(device="cuda").manual_seed(0)
    n_items, W, C = 512, (1 << 22) // 64, 8192
    bits = torch.randint(-(1 << 62), 1 << 62, (n_items, W), generator=g, device="cuda", dtype=torch.int64)
    pre = torch.randint(0, n_items, (C,), generator=g, device="cuda", dtype=torch.int32)
    it = torch.randint(0, n_items, (C,), generator=g, device="cuda", dtype=torch.int32)
    got = itemset_support(bits, bits, pre, it)
    t_k = _t(lambda: itemset_support(bits, bits, pre, it))
    pop = _POP8.to("cuda")

    def torch_path():            # the same AND + byte-table popcount in torch ops, bounded chunks
        out = torch.empty(C, dtype=torch.int64, device="cuda")
        for a in range(0, C, 64):
            x = bits[pre[a:a + 64].long()] & bits[it[a:a + 64].long()]
            out[a:a + 64] = pop[x.view(torch.uint8).long()].view(x.shape[0], -1).sum(1)
        return out
    want = torch_path()
    t_ref = _t(torch_path, reps=2)
    nbytes = 2 * C * W * 8
    emit(kernel="K17 itemset_support", candidates=C, transactions=W * 64, ms=t_k * 1e3, GBps=nbytes / t_k / 1e9,
         torch_ms=t_ref * 1e3, speedup=t_ref / t_k, exact=bool(torch.equal(got, want)))


def gsp():
    """GSP self-join of 2^20 distinct 4-token sequences over 24 tokens."""
    from avenir_amd.ops.sequence_ops import gsp_join
    g = torch.Generator().manual_seed(1)
    X = torch.randint(0, 24, (1 << 20, 4), generator=g, dtype=torch.int32)
    Xd = X.cuda()
    out = gsp_join(Xd)
    t_k = _t(lambda: gsp_join(Xd), reps=3)
    t0 = time.perf_counter()
    ref = gsp_join(X)
    t_ref = time.perf_counter() - t0
    same = out.shape == ref.shape and bool(torch.equal(out.cpu(), ref))
    emit(kernel="K18 gsp_join", rows=X.shape[0], candidates=int(out.shape[0]), ms=t_k * 1e3,
         candidates_per_s=out.shape[0] / t_k, host_torch_ms=t_ref * 1e3, speedup=t_ref / t_k, exact=same)


def bandit():
    """One decision round of 65,536 learner groups x 64 arms for three policies."""
    from avenir_amd.models.bandit import BanditBank
    G, A = 1 << 16, 64
    acts = [f"a{i}" for i in range(A)]
    for algo in ("upperConfidenceBoundOne", "softMax", "thompsonSampler"):
        cfg = {"min.trial": 1, "max.reward": 100, "bin.width": 5}
        gb = BanditBank(algo, acts, G, cfg, device="cuda", seed=3)
        g = torch.Generator(device="cuda").manual_seed(2)
        grp = torch.arange(G, device="cuda").repeat_interleave(8)
        gb.set_rewards(grp, torch.randint(0, A, grp.shape, generator=g, device="cuda"),
                       torch.rand(grp.shape, generator=g, device="cuda") * 100)
        t_k = _t(lambda: gb.next_actions(1), reps=20)
        # the host reference of the same round (same Philox streams; a per-group numpy loop) on
        # 1/16 of the groups, scaled
        cb = BanditBank(algo, acts, G // 16, cfg, device="cpu", seed=3)
        cb.trials, cb.rsum, cb.hist = gb.trials[: G // 16].cpu(), gb.rsum[: G // 16].cpu(), gb.hist[: G // 16].cpu()
        t0 = time.perf_counter()
        cb.next_actions(1)
        t_ref = (time.perf_counter() - t0) * 16
        emit(kernel="K20 bandit_select", algo=algo, groups=G, arms=A, us=t_k * 1e6, decisions_per_s=G / t_k,
             host_ref_ms=t_ref * 1e3, speedup=t_ref / t_k)


def spirit():
    """Streaming PCA of 2,048 keyed streams x 256 records x 16 dims (up to 16 hidden units)."""
    from avenir_amd.analytics.pca import IncrementalPCA
    g = torch.Generator().manual_seed(4)
    K, T, D = 2048, 256, 16
    base = torch.randn(K, 3, D, generator=g, dtype=torch.float64)
    streams = {f"k{k}": (torch.randn(T, 3, generator=g, dtype=torch.float64) @ base[k]
                         + 0.05 * torch.randn(T, D, generator=g, dtype=torch.float64)) for k in range(K)}

    def run(dev):
        m = IncrementalPCA(D, device=dev)
        m.update(streams)
        return m

    t_k = _t(lambda: run("cuda"), reps=3)
    # the torch path of the same update (batched over keys, stepping records and hidden units)
    t0 = time.perf_counter()
    run("cpu")
    t_ref = time.perf_counter() - t0
    emit(kernel="K24 spirit_update", keys=K, records_per_key=T, dim=D, ms=t_k * 1e3,
         records_per_s=K * T / t_k, host_torch_ms=t_ref * 1e3, speedup=t_ref / t_k)


CASES = {"apriori": apriori, "gsp": gsp, "bandit": bandit, "spirit": spirit}

if __name__ == "__main__":
    for name in (sys.argv[1:] or list(CASES)):
        CASES[name]()
