#!/usr/bin/env python3
"""Island GA throughput (islands x generations per second) on one GPU: the one-launch island kernel
(optimize/ga.py, csrc/kernels/optim.hip::ga_assign_kernel) against the per-island torch path of
round 5 (GeneticAlgorithm(use_kernel=False): ~12 small launches per island per generation), at 8,
64 and 512 islands; task-schedule-sized assignment domain (L 24 positions, V 9 values, conflicts),
pool 20, mating 8, replacement 6, 50 generations.  One JSON line each."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from avenir_amd.optimize.domain import AssignmentDomain
    from avenir_amd.optimize.search import GeneticAlgorithm
    g = torch.Generator().manual_seed(3)
    cost = torch.rand((24, 9), generator=g) * 100
    conf = torch.rand((24, 24), generator=g) < 0.1
    d = AssignmentDomain(cost.cuda(), (conf | conf.T).cuda(), invalid_cost=150.0)
    G = 50
    for islands in (8, 64, 512):
        for name, uk in (("island_kernel", True), ("per_island_torch", False)):
            if not uk and islands > 64:
                continue                                   # minutes of launches; the trend is clear by 64
            ga = GeneticAlgorithm(d, islands=islands, pool=20, mating=8, replacement=6, generations=G, seed=1,
                                  use_kernel=uk)
            ga.run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = ga.run()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"bench": "genetic_algorithm", "impl": name, "islands": islands, "generations": G,
                              "pool": 20, "L": 24, "s": dt, "island_generations_per_s": islands * G / dt,
                              "best_cost": r.best_cost}), flush=True)


if __name__ == "__main__":
    main()
