"""Diagnostic: torch's fused Adam in eager mode vs foreach, on plain parameters and on the fused LSTM."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def plain(fused, capturable):
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(37, 11, device="cuda")), torch.nn.Parameter(torch.randn(5, device="cuda"))]
    opt = torch.optim.Adam(ps, lr=0.01, fused=fused, capturable=capturable)
    for i in range(3):
        opt.zero_grad(set_to_none=False)
        loss = sum((p ** 2).sum() * (i + 1) for p in ps)
        loss.backward()
        opt.step()
    return [p.detach().cpu() for p in ps]


base = plain(False, False)
for f, c in ((True, False), (True, True), (False, True)):
    r = plain(f, c)
    print("plain fused", f, "capturable", c, "max diff", max(float((a - b).abs().max()) for a, b in zip(r, base)))


def lstm(fused, capturable, contig_check=False):
    from avenir_amd.nn.sequence import LstmNetwork
    g = torch.Generator().manual_seed(3)
    x = torch.rand(64, 10, generator=g)
    y = (x.sum(1) > 5).float()
    torch.manual_seed(100)
    net = LstmNetwork(2, 8, 1, num_layers=2, seq_len=5, batch_size=1 << 20, lr=0.01, num_iter=3, device="cuda",
                      out_sequence=False, graph=False)
    net.optimizer = torch.optim.Adam(net.parameters(), lr=0.01, fused=fused, capturable=capturable)
    xs = net.to_sequences(x).cuda()
    tgt = net._target(y.cuda())
    for _ in range(3):
        net._step(xs, tgt)
        if contig_check:
            print("grad contiguity:", [(n, p.grad.is_contiguous(), tuple(p.grad.stride())) for n, p in net.named_parameters()][:6])
            print("grad aliasing b_ih/b_hh:", net.lstm.bias_ih_l0.grad.data_ptr() == net.lstm.bias_hh_l0.grad.data_ptr())
            contig_check = False
    return {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}


b = lstm(False, False, True)
for f, c in ((True, False), (True, True), (False, True)):
    r = lstm(f, c)
    print("lstm fused", f, "capturable", c, "max diff", max(float((r[k] - b[k]).abs().max()) for k in b))
