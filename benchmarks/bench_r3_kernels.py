#!/usr/bin/env python3
"""Round-3 kernel families against their alternatives on one MI355X (JSON lines):

* K26r rank statistics (stats.hip) — Spearman / Mann-Whitney / Wilcoxon / Kendall on the device vs
  scipy.stats on the host arrays (the reference's daexp.py calls);
* K28 text (text.hip) — CSR TF-IDF rows vs scikit-learn's TfidfTransformer, the persistent
  TextRank power iteration vs networkx.pagerank (the reference's summariser), SGNS word2vec
  mini-batches as kernels vs the same batches as torch tensor ops on the GPU;
* mixed-type kNN (distance.hip) vs the one-hot embedding + GEMM distance path.
Timings take the best of a few repetitions after a warm-up; host baselines run once (they are
seconds long)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn, reps=3, sync=True):
    fn()
    if sync:
        torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        if sync:
            torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def _host(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def emit(**kw):
    print(json.dumps(kw), flush=True)


def ranks():
    from scipy import stats

    from avenir_amd.ops import stats_ops as S
    rng = np.random.default_rng(0)
    for n in (1 << 20, 1 << 22):
        x = np.round(rng.normal(size=n), 3)
        y = np.round(0.5 * x + rng.normal(size=n), 3)
        gx, gy = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
        dev = _t(lambda: S.spearman(gx, gy))
        ref = _host(lambda: stats.spearmanr(x, y))
        emit(bench="spearman", n=n, gpu_s=dev, scipy_s=ref, speedup=ref / dev)
        h = n // 2
        dev = _t(lambda: S.mann_whitney_u(gx[:h], gy[h:]))
        ref = _host(lambda: stats.mannwhitneyu(x[:h], y[h:]))
        emit(bench="mann_whitney", n=n, gpu_s=dev, scipy_s=ref, speedup=ref / dev)
        dev = _t(lambda: S.wilcoxon_signed_rank(gx, gy))
        ref = _host(lambda: stats.wilcoxon(x, y))
        emit(bench="wilcoxon", n=n, gpu_s=dev, scipy_s=ref, speedup=ref / dev)
        dev = _t(lambda: S.cvm_2samp(gx[:h], gy[h:]))
        ref = _host(lambda: stats.cramervonmises_2samp(x[:h], y[h:]))
        emit(bench="cvm_2samp", n=n, gpu_s=dev, scipy_s=ref, speedup=ref / dev)
    for n in (1 << 16, 1 << 18):   # exact O(n^2) pair counts vs scipy's O(n log n) merge count
        x = np.round(rng.normal(size=n), 2)
        y = np.round(0.5 * x + rng.normal(size=n), 2)
        gx, gy = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
        dev = _t(lambda: S.kendall_tau_b(gx, gy), reps=2)
        ref = _host(lambda: stats.kendalltau(x, y))
        emit(bench="kendall_tau_b", n=n, pairs=n * (n - 1) // 2, gpu_s=dev, scipy_s=ref, speedup=ref / dev,
             pairs_per_s=n * (n - 1) / 2 / dev)


def tfidf():
    import scipy.sparse as sp
    from sklearn.feature_extraction.text import TfidfTransformer

    from avenir_amd.text.preprocess import tfidf_csr
    rng = np.random.default_rng(1)
    D, V, per = 200_000, 1 << 16, 120
    cols = np.minimum(rng.zipf(1.3, size=D * per) - 1, V - 1).astype(np.int64)
    rows = np.repeat(np.arange(D), per)
    M = sp.csr_matrix((np.ones(D * per, dtype=np.float32), (rows, cols)), shape=(D, V))
    M.sum_duplicates()
    G = torch.sparse_csr_tensor(torch.tensor(M.indptr, dtype=torch.long), torch.tensor(M.indices, dtype=torch.long),
                                torch.tensor(M.data), size=(D, V)).to("cuda")
    for sub in (False, True):
        dev = _t(lambda: tfidf_csr(G, sublinear=sub))
        ref = _host(lambda: TfidfTransformer(sublinear_tf=sub).fit_transform(M))
        emit(bench="tfidf_csr", docs=D, vocab=V, nnz=int(M.nnz), sublinear=sub, gpu_s=dev, sklearn_s=ref,
             speedup=ref / dev)


def pagerank():
    import networkx as nx

    from avenir_amd.text.models import pagerank as pr
    rng = np.random.default_rng(2)
    for n in (512, 2048):
        S = rng.random((n, n)) * (rng.random((n, n)) < 0.1)
        S = (S + S.T) / 2
        np.fill_diagonal(S, 0)
        g = torch.tensor(S, device="cuda")
        dev = _t(lambda: pr(g), reps=5)
        G = nx.from_numpy_array(S)
        ref = _host(lambda: nx.pagerank(G, alpha=0.85, tol=1e-10, max_iter=100))
        emit(bench="textrank_pagerank", n=n, gpu_s=dev, networkx_s=ref, speedup=ref / dev)


def sgns():
    from avenir_amd.text import models as T
    rng = np.random.default_rng(3)
    V, n_sent, L = 20_000, 50_000, 20
    toks = np.minimum(rng.zipf(1.2, size=(n_sent, L)) - 1, V - 1)
    ids = [list(map(int, r)) for r in toks]
    for dim in (128,):
        m = T.Word2Vec(dim=dim, window=5, negative=5, epochs=1, batch=4096, device="cuda")
        cen, ctx = m._pairs(ids)
        cnt = torch.bincount(torch.tensor(toks.reshape(-1)), minlength=V).double()
        m.noise = (cnt ** 0.75 / (cnt ** 0.75).sum()).float().cuda()
        dp = T._sgns_dim(dim)

        def kern():
            Win = torch.zeros((V, dp), device="cuda")
            Wout = torch.zeros((V, dp), device="cuda")
            m._fit_kernel(Win, Wout, cen, ctx)
        k = _t(kern, reps=2)
        # the same batches as tensor ops on the GPU (Word2Vec.fit's non-kernel branch)
        cg, og = cen.cuda(), ctx.cuda()

        def tensors():
            g = torch.Generator(device="cuda").manual_seed(0)
            W = torch.rand((V, dim), device="cuda", generator=g)
            C = torch.zeros((V, dim), device="cuda")
            n = cg.numel()
            perm = torch.randperm(n, device="cuda", generator=g)
            for b in range(0, n, 4096):
                idx = perm[b:b + 4096]
                c, o = cg[idx], og[idx]
                negs = torch.multinomial(m.noise, idx.numel() * 5, True, generator=g).view(-1, 5)
                wc = W[c]
                tgt = torch.cat([o.view(-1, 1), negs], 1)
                ct = C[tgt]
                lab = torch.zeros(tgt.shape, device="cuda")
                lab[:, 0] = 1
                gsc = (lab - torch.sigmoid((ct * wc.unsqueeze(1)).sum(2))) * 0.5
                T._row_mean_add(W, c, (gsc.unsqueeze(2) * ct).sum(1))
                T._row_mean_add(C, tgt.reshape(-1), (gsc.unsqueeze(2) * wc.unsqueeze(1)).reshape(-1, dim))
        t = _t(tensors, reps=1)
        emit(bench="sgns_word2vec_epoch", vocab=V, pairs=int(cen.numel()), dim=dim, negative=5, kernel_s=k,
             tensor_ops_s=t, speedup=t / k, pairs_per_s=cen.numel() / k)


def mixed_knn():
    from avenir_amd.ops.distance import knn_mixed
    g = torch.Generator(device="cuda").manual_seed(4)
    nr, nq, Dn, Dc, card, k = 200_000, 20_000, 8, 8, 64, 10
    Rn = torch.rand((nr, Dn), device="cuda", generator=g)
    Qn = torch.rand((nq, Dn), device="cuda", generator=g)
    Rc = torch.randint(0, card, (nr, Dc), device="cuda", generator=g, dtype=torch.int32)
    Qc = torch.randint(0, card, (nq, Dc), device="cuda", generator=g, dtype=torch.int32)
    wc = torch.ones(Dc, device="cuda")
    dev = _t(lambda: knn_mixed(Qn, Qc, Rn, Rc, wc, k))
    # one-hot embedding (categorical mismatch = half the squared distance of one-hots) + GEMM top-k
    Ro = torch.cat([Rn] + [torch.nn.functional.one_hot(Rc[:, j].long(), card).float() * (0.5 ** 0.5)
                           for j in range(Dc)], 1)
    Qo = torch.cat([Qn] + [torch.nn.functional.one_hot(Qc[:, j].long(), card).float() * (0.5 ** 0.5)
                           for j in range(Dc)], 1)

    def onehot():
        for s in range(0, nq, 4096):
            q = Qo[s:s + 4096]
            d = (q * q).sum(1, keepdim=True) + (Ro * Ro).sum(1) - 2 * q @ Ro.T
            torch.topk(d, k, 1, largest=False)
    t = _t(onehot, reps=2)
    emit(bench="mixed_knn", refs=nr, queries=nq, numeric=Dn, categorical=Dc, cardinality=card, k=k, kernel_s=dev,
         onehot_gemm_s=t, onehot_width=Dn + Dc * card, speedup=t / dev, pairs_per_s=nr * nq / dev)


if __name__ == "__main__":
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else ["ranks", "tfidf", "pagerank", "sgns", "mixed_knn"]
    for name in only:
        globals()[name]()
