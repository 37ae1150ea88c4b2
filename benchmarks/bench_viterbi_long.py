#!/usr/bin/env python3
"""One long HMM sequence: the sequential one-wavefront Viterbi kernel vs the chunked max-plus
scan (sequence_ops.viterbi_long).  Prints one JSON line per configuration."""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from avenir_amd.ops import sequence_ops as SO


def _timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def main() -> int:
    Ts = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["262144", "1048576"])]
    for S in (8, 32):
        g = torch.Generator().manual_seed(S)
        norm = lambda m: torch.log(m / m.sum(-1, keepdim=True))
        lA = norm(torch.rand(S, S, generator=g) + 0.05).cuda()
        lB = norm(torch.rand(S, 32, generator=g) + 0.05).cuda()
        lp = norm(torch.rand(S, generator=g) + 0.05).cuda()
        for T in Ts:
            obs = torch.randint(0, 32, (T,), generator=g).to(torch.int16).cuda()
            t_seq, (p_seq, s_seq) = _timed(lambda: SO.viterbi(obs.view(1, -1), lA, lB, lp), reps=1)
            for chunk in (256, 1024):
                t_chk, (p_chk, s_chk) = _timed(lambda: SO.viterbi_long(obs, lA, lB, lp, chunk=chunk))
                agree = (p_chk == p_seq[0]).float().mean().item()
                print(json.dumps({"S": S, "T": T, "chunk": chunk, "sequential_ms": t_seq * 1e3,
                                  "chunked_ms": t_chk * 1e3, "speedup": t_seq / t_chk,
                                  "score_seq": float(s_seq[0]), "score_chunked": s_chk,
                                  "path_agreement": agree}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
