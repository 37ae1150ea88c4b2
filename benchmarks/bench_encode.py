"""Throughput of the K26 column-moments and K23 leave-one-out kernels (encode.hip) on one GPU,
with the equivalent PyTorch-op chains as the comparison; one JSON line per case."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from avenir_amd.ops import encode_ops as E


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def torch_moments(x):
    m = x.mean(1, keepdim=True)
    d = x - m
    d2 = d * d
    return torch.stack([x.sum(1), x.amin(1), x.amax(1), d2.mean(1), (d2 * d).mean(1), (d2 * d2).mean(1)], 1)


def main():
    dev = torch.device("cuda")
    for F, n in [(1, 1 << 28), (16, 1 << 24), (64, 1 << 22)]:
        x = torch.randn(F, n, device=dev)
        t = timeit(lambda: E.column_moments(x))
        tt = timeit(lambda: torch_moments(x.double()))
        print(json.dumps({"op": "col_moments_f32", "F": F, "n": n, "ms": t * 1e3,
                          "hbm_gbps": 2 * x.numel() * 4 / t / 1e9, "torch_f64_chain_ms": tt * 1e3,
                          "speedup": tt / t}), flush=True)
    for F, n, wide in [(8, 1 << 24, False), (32, 1 << 22, False), (4, 1 << 24, True)]:
        hi = 10_000 if wide else 200
        codes = torch.randint(0, hi, (F, n), device=dev).to(torch.uint16 if wide else torch.uint8)
        y = torch.rand(n, device=dev, dtype=torch.float64)
        gm = y.mean().view(1)

        def run():
            s, k = E.loo_stats(codes, n, y)
            return E.loo_apply(codes, n, y, s, k, gm, reg=1.0)

        def run_torch():
            m = 65536 if wide else 256
            c = codes.long() + torch.arange(F, device=dev).view(-1, 1) * m
            s = torch.zeros(F * m, device=dev, dtype=torch.float64).index_add_(0, c.view(-1), y.repeat(F))
            k = torch.zeros(F * m, device=dev, dtype=torch.float64).index_add_(0, c.view(-1),
                                                                               torch.ones(F * n, device=dev, dtype=torch.float64))
            return ((s[c] - y + gm) / (k[c] - 1 + 1.0).clamp_min(1e-12)).float().T.contiguous()

        t, tt = timeit(run), timeit(run_torch, reps=5)
        byts = F * n * codes.element_size() * 2 + n * 8 * 2 + F * n * 4
        print(json.dumps({"op": "loo_encode", "F": F, "n": n, "wide": wide, "ms": t * 1e3,
                          "hbm_gbps": byts / t / 1e9, "torch_chain_ms": tt * 1e3, "speedup": tt / t}), flush=True)


if __name__ == "__main__":
    main()
