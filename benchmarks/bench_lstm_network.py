#!/usr/bin/env python3
"""LstmNetwork.fit (nn/sequence.py) at the reference's contact-tracing configuration
(R/lstm_ct.properties: input 5, hidden 100, 2 layers, seq_len 5, 1,000 sequences, batch = all,
Adam lr 0.002, 100 iterations): wall time per iteration of the framework's own training loop
(fused LSTM kernels, fused optimiser, the whole step captured as a HIP graph)."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avenir_amd.nn.sequence import LstmNetwork  # noqa: E402


def main():
    torch.manual_seed(0)
    B, T, I = 1000, 5, 5
    x = torch.randn(B, T, I)
    y = (x[:, :, 0].sum(1) > 0).float().view(-1, 1)
    for graph in (False, True):
        net = LstmNetwork(I, 100, 1, num_layers=2, seq_len=T, batch_size=B, out_sequence=False,
                          out_activation="sigmoid", loss="bce", optimizer="adam", lr=0.002, num_iter=10,
                          device="cuda", graph=graph)
        net.fit(x, y)                                     # warm-up (and the graph capture)
        torch.cuda.synchronize()
        net.num_iter = 100
        t0 = time.perf_counter()
        net.fit(x, y)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 100
        print(json.dumps({"bench": "lstm_network_fit", "graph": graph, "ms_per_iter": dt * 1e3,
                          "optimizer": type(net.optimizer).__name__,
                          "fused_optimizer": bool(net.optimizer.defaults.get("fused")),
                          "loss_last": net.losses[-1] if net.losses else None}), flush=True)


if __name__ == "__main__":
    main()
