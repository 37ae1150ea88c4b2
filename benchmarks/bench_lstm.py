#!/usr/bin/env python3
"""K27 fused LSTM vs PyTorch-ROCm nn.LSTM (MIOpen) — training step and inference on one MI355X.

Configs: the reference's contact-tracing LSTM (R/lstm_ct.properties: input 5, hidden 100, 2
layers, seq_len 5, 1000 sequences from R/viral_infection_prediction_with_lstm_tutorial.txt:14) and
two larger batch/sequence shapes.  A training step = forward + CE loss + backward + Adam on the
whole model (LSTM + linear head).  Prints one JSON line per (config, implementation).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from avenir_amd.nn.common import GraphedStep  # noqa: E402
from avenir_amd.ops.rnn import FusedLSTM  # noqa: E402

CONFIGS = [
    dict(name="reference_ct", B=1000, T=5, I=5, H=100, L=2, O=2),
    dict(name="b8k_t16_h64", B=8192, T=16, I=32, H=64, L=2, O=2),
    # MIOpen's graph capture at this size aborts the process inside hipBLASLt ("operation not
    # permitted when stream is capturing" -> core dump), so that one arm is not run
    dict(name="b64k_t32_h128", B=65536, T=32, I=16, H=128, L=2, O=2, skip=("miopen_graph",)),
]


class Net(torch.nn.Module):
    def __init__(self, lstm, H, O):
        super().__init__()
        self.lstm = lstm
        self.head = torch.nn.Linear(H, O)

    def forward(self, x):
        out, _ = self.lstm(x)
        return self.head(out[:, -1])


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


def run(cfg, impl, steps, warmup):
    torch.manual_seed(0)
    dev = torch.device("cuda")
    B, T, I, H, L, O = (cfg[k] for k in "BTIHLO")
    ref = torch.nn.LSTM(I, H, L, batch_first=True)
    if impl.startswith("fused"):
        lstm = FusedLSTM(I, H, L, precision="bf16" if "bf16" in impl else "fp32")
        lstm.load_state_dict(ref.state_dict())
    else:
        lstm = ref
    net = Net(lstm, H, O).to(dev)
    # miopen_bf16: the whole model in bf16 on MIOpen — the like-for-like precision comparison for
    # the fused kernel's bf16 GEMM operands (miopen = fp32, the reference's numerics)
    xdt = torch.bfloat16 if impl.startswith("miopen_bf16") else torch.float32
    if impl.startswith("miopen_bf16"):
        net = net.to(torch.bfloat16)
    graph = impl.endswith("graph")
    opt = torch.optim.Adam(net.parameters(), lr=2e-3, capturable=graph)
    x = torch.randn(B, T, I, device=dev, dtype=xdt)
    y = torch.randint(0, O, (B,), device=dev)
    lossf = torch.nn.CrossEntropyLoss()
    losses = []

    def train_step():
        opt.zero_grad(set_to_none=True)
        loss = lossf(net(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.detach())

    def infer():
        with torch.no_grad():
            net(x)

    if graph:   # whole step (forward, loss, backward, Adam) as one HIP graph
        def step_fn(xx, yy):
            opt.zero_grad(set_to_none=False)
            loss = lossf(net(xx), yy)
            loss.backward()
            opt.step()
            return loss.detach()
        gs = GraphedStep(step_fn, x, y, model=net, optimizer=opt)

        def train_step():
            losses.append(gs(x, y).clone())

    ms_train = timed(train_step, steps, warmup)
    ms_inf = timed(infer, steps, warmup)
    flops = 2 * B * T * 4 * H * (I + H) * L  # forward GEMM flops (input + recurrent)
    return {"bench": "lstm", "config": cfg["name"], "impl": impl, "B": B, "T": T, "I": I, "H": H, "L": L,
            "train_ms": ms_train, "infer_ms": ms_inf,
            "train_seq_per_s": B / (ms_train * 1e-3), "infer_seq_per_s": B / (ms_inf * 1e-3),
            "fwd_tflops": flops / (ms_inf * 1e-3) / 1e12,
            "loss_first": float(losses[0]), "loss_last": float(losses[-1])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--configs", default="all")
    ap.add_argument("--impls", default="fused,fused_graph,fused_bf16,miopen,miopen_graph,miopen_bf16")
    args = ap.parse_args()
    names = None if args.configs == "all" else set(args.configs.split(","))
    for cfg in CONFIGS:
        if names and cfg["name"] not in names:
            continue
        res = {}
        for impl in args.impls.split(","):
            if impl in cfg.get("skip", ()):
                print(json.dumps({"bench": "lstm", "config": cfg["name"], "impl": impl,
                                  "skipped": "library graph capture aborts the process at this size"}), flush=True)
                continue
            try:
                res[impl] = run(cfg, impl, args.steps, args.warmup)
            except Exception as e:           # e.g. a library LSTM that refuses graph capture
                print(json.dumps({"bench": "lstm", "config": cfg["name"], "impl": impl, "error": str(e)[:200]}),
                      flush=True)
                res[impl] = None
                continue
            print(json.dumps(res[impl]), flush=True)
        # like-for-like pairs: eager vs eager and graph vs graph at fp32 (the reference's numerics),
        # and the bf16 fused kernel vs bf16 MIOpen
        for impl, base in (("fused", "miopen"), ("fused_graph", "miopen_graph"), ("fused_bf16", "miopen_bf16"),
                           ("fused_graph", "miopen")):
            if impl in res and base in res and res[base] and res[impl]:
                print(json.dumps({"bench": "lstm_speedup", "config": cfg["name"], "impl": impl, "vs": base,
                                  "train_x": res[base]["train_ms"] / res[impl]["train_ms"],
                                  "infer_x": res[base]["infer_ms"] / res[impl]["infer_ms"]}), flush=True)


if __name__ == "__main__":
    main()
