#!/usr/bin/env python3
"""Small driver programs for hardware-counter passes (scripts/gpu_pmc.sh): each target runs a
handful of launches of ONE hot kernel at a roofline-relevant size, so a ``rocprofv3 --pmc`` pass
over it is short and its counters belong to that kernel.

    python benchmarks/pmc_targets.py {rowpack,columns,knn16,knn64,knn256,smo_ws,forest}
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rowpack():
    from avenir_amd.data.synth import churn_device
    from avenir_amd.ops import histogram as H
    n = 1 << 30
    codes, labels = churn_device(n, seed=1, device="cuda")
    rp = H.pack_rows(codes, n, [4, 3, 3, 3, 5], labels, 2)
    del codes, labels
    for _ in range(4):
        H.class_histogram_packed(rp)
    torch.cuda.synchronize()


def columns():
    from avenir_amd.data.synth import churn_device
    from avenir_amd.ops import histogram as H
    n = 1 << 29
    codes, labels = churn_device(n, seed=1, device="cuda")
    bins = [4, 3, 3, 3, 5]
    out = torch.zeros((2, sum(bins) + 1), dtype=torch.int64, device="cuda")
    for _ in range(4):
        out.zero_()
        H.class_histogram(codes, n, bins, labels, 2, out=out, mode=0, count_labels=True)
    torch.cuda.synchronize()


def _knn(D):
    from avenir_amd.ops import distance as Dm
    g = torch.Generator(device="cuda").manual_seed(0)
    Q = torch.randn((16384, D), device="cuda", generator=g)
    R = torch.randn((1 << 18, D), device="cuda", generator=g)
    for _ in range(3):
        Dm.knn(Q, R, 10)
    torch.cuda.synchronize()


def smo_ws():
    from avenir_amd.models.svm import kernel_matrix, smo_batch
    g = torch.Generator(device="cuda").manual_seed(9)
    X = torch.randn((8192, 8), device="cuda", generator=g)
    y = torch.where(X[:, 0] * X[:, 1] > 0, 1.0, -1.0)
    K = kernel_matrix(X, X, "rbf", 0.5).unsqueeze(0).contiguous()
    smo_batch(K, y.view(1, -1), 1.0, 1e-3, solver="ws")
    torch.cuda.synchronize()


def forest():
    import numpy as np
    from avenir_amd.models.forest import ForestBuilder
    from avenir_amd.ops import forest_ops as FO
    dev = torch.device("cuda")
    R, F, A = 1 << 25, 16, 256
    g = torch.Generator(device=dev).manual_seed(0)
    codes = torch.randint(0, 32, (F, R), generator=g, device=dev, dtype=torch.uint8)
    lab = torch.randint(0, 2, (R,), generator=g, device=dev, dtype=torch.uint8)
    wt = torch.randint(1, 4, (R,), generator=g, device=dev, dtype=torch.uint8)
    dc, dl, dw = torch.empty_like(codes), torch.empty_like(lab), torch.empty_like(wt)
    cnt = np.full(A, R // A, dtype=np.int64)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    feat = torch.randint(0, F, (A,), generator=g, device=dev, dtype=torch.int32)
    thr = torch.full((A,), 15, dtype=torch.int32, device=dev)
    bins = [32] * F
    bd = torch.tensor(bins, dtype=torch.int32, device=dev)
    od = torch.tensor(list(np.cumsum([0] + bins[:-1])), dtype=torch.int32, device=dev)
    inode, istart, ilen, nch = ForestBuilder(None, 1, None)._chunks(np.arange(A), start, cnt, 26000)
    il = FO.forest_part_count(codes, inode, istart, ilen, feat, thr).cpu().numpy().astype(np.int64)
    ends = np.cumsum(nch)
    first = ends - nch
    csum = np.concatenate([[0], np.cumsum(il)])
    nleft = csum[ends] - csum[first]
    rsum = np.concatenate([[0], np.cumsum(ilen.astype(np.int64) - il)])
    owner = inode.astype(np.int64)
    lbase = start[owner] + (csum[:-1] - csum[first[owner]])
    rbase = start[owner] + nleft[owner] + (rsum[:-1] - rsum[first[owner]])
    hist = torch.zeros((A, 2, sum(bins) + 1), dtype=torch.int64, device=dev)
    for _ in range(3):
        FO.forest_part_scatter(codes, lab, wt, dc, dl, dw, inode, istart, ilen, lbase, rbase, il, feat, thr)
        FO.forest_hist(codes, lab, wt, inode, istart, ilen, bd, od, bins, sum(bins) + 1, 2, hist)
        FO.forest_bootstrap(codes[:, : R // 4].contiguous(), lab, R // 4, list(range(4)), 0, 1, 0)
    torch.cuda.synchronize()


def kmeans():
    """K16 Lloyd pass at 16.7 M rows x 16 dims x 16 centroids."""
    from avenir_amd.models.cluster import kmeans_step
    g = torch.Generator(device="cuda").manual_seed(0)
    n, D, k = 1 << 24, 16, 16
    X = torch.randn((n, D), device="cuda", generator=g)
    C = X[torch.randint(0, n, (k,), device="cuda", generator=g)].clone()
    for _ in range(6):
        kmeans_step(X, [C])
    torch.cuda.synchronize()


def fmt():
    """format.hip (fmt_len_kernel / fmt_write_kernel): 2^24 rows of int / float / string-table columns
    formatted on the device into a file."""
    import tempfile
    from avenir_amd.data.records import format_lines
    n = 1 << 24
    g = torch.Generator(device="cuda").manual_seed(0)
    ids = torch.randint(0, 1 << 30, (n,), generator=g, device="cuda")
    v = torch.randn(n, generator=g, device="cuda", dtype=torch.float64) * 100
    cls = torch.randint(0, 3, (n,), generator=g, device="cuda", dtype=torch.int32)
    path = os.path.join(tempfile.gettempdir(), f"avmi_fmt_{os.getpid()}.txt")
    try:
        for _ in range(3):
            format_lines([("i", ids), ("f", v, 3), ("s", ["low", "mid", "high"], cls)], n, ",", path=path)
        torch.cuda.synchronize()
    finally:
        if os.path.exists(path):
            os.remove(path)


def pairs():
    """distance.hip pairs_within_kernel: the recordSimilarity self-join of 2^17 x 8 rows."""
    from avenir_amd import _native
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.rand((1 << 17, 8), generator=g, device="cuda")
    for _ in range(3):
        _native.C().pairs_within(A, A, 8 ** 0.5, 1000.0, 100.0, True, 0, 0)
    torch.cuda.synchronize()


def split():
    """split.hip ref_split_score_kernel (K7): a reference-split random forest level-wise build."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from bench_models import _numeric_table
    from avenir_amd.models.tree import RandomForest, TreeParams
    t = _numeric_table(1 << 20, 16, 2)
    for f in t.schema.feature_fields:
        f.max_split = 3
    p = TreeParams(binary=False, stopping="maxDepth", max_depth=5, sub_sampling="withReplace",
                   attr_selection="randomNotUsedYet", random_attr_count=4, split_selection="randomAmongTop",
                   top_split_count=3, max_bins=8)
    RandomForest(t.schema, 10, p, "all").fit(t)
    torch.cuda.synchronize()


def lstm():
    """rnn_f32.hip lstm_fwd_f32_kernel / lstm_bwd_f32_kernel: training steps of the reference's
    contact-tracing LSTM shape scaled to 65,536 sequences (input 5, hidden 100, 2 layers, T 5)."""
    from avenir_amd.ops.rnn import FusedLSTM
    torch.manual_seed(0)
    m = FusedLSTM(5, 100, 2, precision="fp32").cuda()
    x = torch.randn(65536, 5, 5, device="cuda")
    for _ in range(4):
        out, _ = m(x)
        out[:, -1].sum().backward()
    torch.cuda.synchronize()


def gemm_tn():
    """gemm.hip gemm_tn_partial_kernel / gemm_tn_reduce_kernel: the LSTM weight gradient of 65,536
    sequences x T 5 (K = 327,680 rows, M = 4H = 400, N = H + I + 1 = 106)."""
    from avenir_amd import _native
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn((327680, 400), generator=g, device="cuda")
    B = torch.randn((327680, 106), generator=g, device="cuda")
    for _ in range(4):
        _native.C().gemm_tn(A, B)
    torch.cuda.synchronize()


def k27():
    """mlp.hip linear_act_fwd (K27) at 4,096 x 3,072 x 768 + GELU, the BERT FFN-up shape at 32 x 128
    tokens; the arithmetic mode from AVMI_F32_GEMM."""
    from avenir_amd import _native
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn((4096, 768), generator=g, device="cuda")
    W = torch.randn((3072, 768), generator=g, device="cuda") / 768 ** 0.5
    b = torch.randn(3072, generator=g, device="cuda")
    for _ in range(6):
        _native.C().linear_act_fwd(X, W, b, 6)
    torch.cuda.synchronize()


def bert():
    """transformer.hip add_layernorm / embed_layernorm and mlp.hip's GELU tile epilogue: 12 encoder
    passes of the bert-base shape at B 1 x S 128 (the query path of semantic search)."""
    from avenir_amd.nn.bert import BertConfig, BertEncoder
    torch.manual_seed(0)
    m = BertEncoder(BertConfig()).cuda()
    ids = torch.randint(0, 30522, (1, 128), device="cuda")
    mask = torch.ones_like(ids)
    for _ in range(12):
        m(ids, mask)
    torch.cuda.synchronize()


def bert32():
    """The bert-base encoder at B 32 x S 128 (4,096 token rows: the planes path for Q/K/V and FFN-up,
    the in-loop split tiles for the 768-column projections): 6 passes."""
    from avenir_amd.nn.bert import BertConfig, BertEncoder
    torch.manual_seed(0)
    m = BertEncoder(BertConfig()).cuda()
    ids = torch.randint(0, 30522, (32, 128), device="cuda")
    mask = torch.ones_like(ids)
    for _ in range(6):
        m(ids, mask)
    torch.cuda.synchronize()


def dqn():
    """DQNAgent.learn (hiddens [128, 128, 128], batch 256, the reference sizes) replayed as its HIP
    graph: 50 updates after a short fill of the replay ring."""
    from avenir_amd.nn.rl import DQNAgent, PricingEnv
    torch.manual_seed(0)
    env = PricingEnv(64, device="cuda", seed=1)
    ag = DQNAgent(env, batch=256, seed=1)
    s = env.reset()
    for _ in range(8):
        a = ag.act(s)
        s2, r, done = env.step(a)
        ag._store(s, a, r, s2, done)
        s = s2
    for _ in range(50):
        ag.learn()
    torch.cuda.synchronize()


def svm_select():
    """svm.hip smo_ws_topk_stream_kernel + the rank merge: the working-set selection at 1,048,576 rows."""
    from avenir_amd import _native
    g = torch.Generator(device="cuda").manual_seed(7)
    N, C = 1 << 20, 1.0
    y = torch.where(torch.rand(1, N, generator=g, device="cuda") < 0.5, 1.0, -1.0)
    a = torch.rand(1, N, generator=g, device="cuda") * C
    G = torch.randn(1, N, generator=g, device="cuda")
    ws = torch.zeros((1, 128), dtype=torch.long, device="cuda")
    ok = torch.zeros((1, 128), dtype=torch.bool, device="cuda")
    gap = torch.full((1,), float("inf"), device="cuda")
    for _ in range(20):
        _native.C().smo_ws_select(a, G, y, C, 64, ws, ok, gap)
    torch.cuda.synchronize()


TARGETS = {"kmeans": kmeans, "fmt": fmt, "pairs": pairs, "split": split, "lstm": lstm, "rowpack": rowpack, "columns": columns, "knn16": lambda: _knn(16), "knn64": lambda: _knn(64),
           "knn256": lambda: _knn(256), "smo_ws": smo_ws, "forest": forest,
           "gemm_tn": gemm_tn, "k27": k27, "bert": bert, "bert32": bert32, "dqn": dqn, "svm_select": svm_select}

if __name__ == "__main__":
    TARGETS[sys.argv[1]]()
