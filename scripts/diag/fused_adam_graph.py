"""Diagnostic: LstmNetwork weights after 3 steps — graphed vs eager, fused vs foreach optimiser."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(graph, fused):
    os.environ["AVMI_FUSED_OPT"] = "1" if fused else "0"
    from avenir_amd.nn.sequence import LstmNetwork
    g = torch.Generator().manual_seed(3)
    x = torch.rand(64, 10, generator=g)
    y = (x.sum(1) > 5).float()
    torch.manual_seed(100)
    net = LstmNetwork(2, 8, 1, num_layers=2, seq_len=5, batch_size=1 << 20, lr=0.01, num_iter=3, device="cuda",
                      out_sequence=False, graph=graph)
    net.fit(net.to_sequences(x), y, num_iter=3)
    return {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}, net.losses


res = {(gr, fu): run(gr, fu) for gr in (False, True) for fu in (False, True)}
base = res[(False, False)][0]
for key, (sd, losses) in res.items():
    d = max(float((sd[k] - base[k]).abs().max()) for k in base)
    print(key, "max |w - eager foreach| =", d, "losses", losses)
