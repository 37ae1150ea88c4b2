#!/usr/bin/env python3
"""Per-step time of the DQN update, the autoencoder mini-batch step and the RBM PCD step at the
reference sizes (P/app/price_rl.py:175-217: hiddens [128, 128, 128], train batch 256;
P/unsupv/ae.py:233-275 hidden 100; P/unsupv/rbm.py:82-158 100 components), three ways: the eager
``torch.nn`` twin, the fused kernels eager, and the fused kernels replayed as one HIP graph per
step.  Also the DQN learning curve: greedy return before and after training.  One JSON line each.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def dqn():
    from avenir_amd.nn.rl import DQNAgent, PricingEnv
    for name, fused, graph in (("torch_eager", False, False), ("fused_eager", True, False), ("fused_graph", True, True)):
        env = PricingEnv(64, device="cuda", seed=0)
        ag = DQNAgent(env, batch=256, seed=0, fused=fused, graph=graph)
        ag.train(iterations=4)                        # fills the replay ring (4 x 19 x 64 transitions)
        t = timed(ag.learn, 200)
        print(json.dumps({"bench": "dqn_learn", "impl": name, "batch": 256, "hiddens": [128, 128, 128],
                          "us_per_update": t * 1e6}), flush=True)
    # learning curve (4 updates per environment step) and the best CONSTANT price as a yardstick
    torch.manual_seed(0)
    env = PricingEnv(64, device="cuda", seed=1)
    ag = DQNAgent(env, batch=256, seed=1)
    before = ag.evaluate(4)
    curve = []
    for it in range(6):
        ag.train(iterations=10, updates_per_step=4)
        curve.append(ag.evaluate(4))
    consts = []
    for a in range(env.n_actions):
        e2 = PricingEnv(64, device="cuda", seed=7)
        tot, done = torch.zeros(64, device="cuda"), False
        e2.reset()
        while not done:
            _, r, done = e2.step(torch.full((64,), a, device="cuda"))
            tot += r
        consts.append(float(tot.mean()))
    best = max(range(len(consts)), key=consts.__getitem__)
    print(json.dumps({"bench": "dqn_learning", "envs": 64, "updates_per_step": 4, "greedy_return_before": before,
                      "greedy_return_every_10_iterations": curve, "best_constant_price": float(env.grid[best]),
                      "best_constant_return": consts[best], "worst_constant_return": min(consts)}), flush=True)


def autoencoder():
    from avenir_amd.nn.unsupervised import AutoEncoder
    torch.manual_seed(0)
    x = torch.rand(8192, 400, device="cuda")
    for name, fused, graph in (("torch_eager", False, False), ("fused_eager", True, False), ("fused_graph", True, True)):
        torch.manual_seed(0)
        ae = AutoEncoder(400, [100], ["sigmoid"], ["sigmoid"], batch_size=256, num_iter=1, device="cuda", fused=fused,
                         graph=graph)
        ae.fit(x, num_iter=1)
        t = timed(lambda: ae.fit(x, num_iter=1), 5) / (8192 // 256)
        print(json.dumps({"bench": "autoencoder_step", "impl": name, "n_in": 400, "hidden": 100, "batch": 256,
                          "us_per_step": t * 1e6, "last_loss": ae.losses[-1]}), flush=True)


def rbm():
    from avenir_amd.nn.unsupervised import RestrictedBoltzmannMachine
    x = (torch.rand(8192, 784, device="cuda") < 0.3).float()
    for name, graph in (("eager", False), ("graph", True)):
        m = RestrictedBoltzmannMachine(784, 100, lr=0.1, batch_size=64, num_iter=1, device="cuda")
        m.fit(x, graph=graph)
        t = timed(lambda: m.fit(x, graph=graph), 3) / (8192 // 64)
        print(json.dumps({"bench": "rbm_pcd_step", "impl": name, "visible": 784, "hidden": 100, "batch": 64,
                          "us_per_step_incl_epoch_score": t * 1e6}), flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["dqn", "autoencoder", "rbm"]
    for w in which:
        globals()[w]()
