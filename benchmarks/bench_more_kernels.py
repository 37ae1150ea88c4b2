"""Throughput of the K-family kernels that had no micro-benchmark line yet: K3 pair histograms,
K4 Markov bigrams, K9 level-wise node histograms, K10 Viterbi, K11 Markov log-odds, K16 the fused
k-means Lloyd pass.  One JSON line each: median ms over the repetitions, bytes the kernel must
read, and the implied GB/s (or rows/s), on device-resident synthetic inputs.
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    from avenir_amd.models.cluster import kmeans_step
    from avenir_amd.ops import histogram as H
    from avenir_amd.ops import sequence_ops as SQ
    from avenir_amd.ops import tree_ops as TO
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    # K3: mutual-information pair tables, 6 features of 8 bins, all 15 pairs, 2 classes
    n, F = 1 << 27, 6
    codes = torch.randint(0, 8, (F, n), device=dev, dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 2, (n,), device=dev, dtype=torch.uint8, generator=g)
    pairs = [(a, b) for a in range(F) for b in range(a + 1, F)]
    ms = timeit(lambda: H.pair_histogram(codes, n, [8] * F, pairs, labels, 2))
    emit(kernel="pair_hist", rows=n, features=F, pairs=len(pairs), ms=ms, rows_per_s=n / ms * 1e3,
         gbps=n * (F + 1) / ms / 1e6)
    del codes, labels
    # K4: Markov bigrams over int16 state sequences [N, L]
    N, L, S = 1 << 22, 32, 12
    st = torch.randint(0, S, (N, L), device=dev, dtype=torch.int16, generator=g)
    lab = torch.randint(0, 2, (N,), device=dev, dtype=torch.uint8, generator=g)
    ms = timeit(lambda: H.bigram_histogram(st, S, lab, 2))
    emit(kernel="bigram", sequences=N, length=L, states=S, ms=ms, transitions_per_s=N * (L - 1) / ms * 1e3,
         gbps=N * L * 2 / ms / 1e6)
    # K11: Markov log-odds classifier
    lr = torch.randn((S, S), device=dev, generator=g)
    ms = timeit(lambda: SQ.markov_logodds(st, lr))
    emit(kernel="markov_logodds", sequences=N, length=L, ms=ms, gbps=N * L * 2 / ms / 1e6)
    # K10: Viterbi, 8 hidden states, 16 symbols, sequences of 64
    Nv, T, Sh, V = 1 << 20, 64, 8, 16
    obs = torch.randint(0, V, (Nv, T), device=dev, dtype=torch.int16, generator=g)
    logA = torch.log_softmax(torch.randn((Sh, Sh), device=dev, generator=g), 1)
    logB = torch.log_softmax(torch.randn((Sh, V), device=dev, generator=g), 1)
    logpi = torch.log_softmax(torch.randn((Sh,), device=dev, generator=g), 0)
    ms = timeit(lambda: SQ.viterbi(obs, logA, logB, logpi))
    emit(kernel="viterbi", sequences=Nv, length=T, states=Sh, ms=ms, steps_per_s=Nv * T / ms * 1e3,
         state_updates_per_s=Nv * T * Sh * Sh / ms * 1e3)
    del obs, st, lab
    # K9: level-wise node histograms, 16 features x 32 bins, 2 classes, 64 frontier nodes
    n, F, B, A = 1 << 25, 16, 32, 64
    codes = torch.randint(0, B, (F + 1, n), device=dev, dtype=torch.uint8, generator=g)
    codes[F] = 0
    labels = torch.randint(0, 2, (n,), device=dev, dtype=torch.uint8, generator=g)
    node = torch.randint(0, A, (n,), device=dev, dtype=torch.int32, generator=g)
    ms = timeit(lambda: TO.node_histogram(codes, n, labels, node, None, [B] * F + [1], 2, A))
    emit(kernel="node_hist", rows=n, features=F, nodes=A, ms=ms, rows_per_s=n / ms * 1e3,
         gbps=n * (F + 1 + 1 + 4) / ms / 1e6)
    del codes, labels, node
    # K16: fused Lloyd pass, 16.7 M x 16, k = 16
    n, D, k = 1 << 24, 16, 16
    X = torch.randn((n, D), device=dev, generator=g)
    C = X[torch.randint(0, n, (k,), device=dev, generator=g)].clone()
    ms = timeit(lambda: kmeans_step(X, [C]))
    emit(kernel="kmeans_step", rows=n, dim=D, k=k, ms=ms, rows_per_s=n / ms * 1e3, gbps=n * D * 4 / ms / 1e6)


if __name__ == "__main__":
    main()
