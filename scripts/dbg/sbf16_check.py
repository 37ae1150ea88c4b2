import os, sys, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from avenir_amd import _native
C = _native.C()
g = torch.Generator(device="cuda").manual_seed(0)
for M, N, K in ((20000, 48, 64), (1025, 33, 64), (20000, 64, 48), (300, 130, 64), (4097, 1031, 1028), (64, 64, 32), (65, 65, 36)):
    for zero in (False, True):
        X = torch.randn(M, K, generator=g, device="cuda")
        if zero:
            X = X * (torch.rand(M, K, generator=g, device="cuda") > 0.5)
        W = torch.randn(N, K, generator=g, device="cuda") / K ** 0.5
        Y = C.linear_act_fwd(X, W, None, 0) if True else None
        ref = X.double() @ W.double().t()
        e = (Y.double() - ref).abs()
        i = int(e.argmax())
        print(json.dumps({"M": M, "N": N, "K": K, "zero": zero, "max_err": float(e.max()), "at": [i // N, i % N],
                          "got": float(Y.view(-1)[i]), "ref": float(ref.view(-1)[i]), "nan": bool(torch.isnan(Y).any())}), flush=True)
