import torch, sys
sys.path.insert(0, ".")
from avenir_amd.ops.mlp_ops import _act_torch, ACT_CODES, linear_act
cuda = torch.device("cuda")
for M, K, N in [(20000, 48, 64), (20000, 200, 96), (1025, 33, 64)]:
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g, dtype=torch.float64)
    W = torch.randn(N, K, generator=g, dtype=torch.float64) / K ** 0.5
    b = torch.randn(N, generator=g, dtype=torch.float64)
    gy = torch.randn(M, N, generator=g, dtype=torch.float64)
    xr, Wr, br = (t.clone().requires_grad_() for t in (x, W, b))
    yr = _act_torch(torch.nn.functional.linear(xr, Wr, br), ACT_CODES["relu"])
    yr.backward(gy)
    xg, Wg, bg = (t.float().to(cuda).requires_grad_() for t in (x, W, b))
    yg = linear_act(xg, Wg, bg, "relu")
    yg.backward(gy.float().to(cuda))
    for nm, a, r in (("y", yg.detach(), yr.detach()), ("dx", xg.grad, xr.grad), ("dW", Wg.grad, Wr.grad), ("db", bg.grad, br.grad)):
        d = (a.cpu().double() - r).abs()
        rel = d / (r.abs() * 1e-3 + 1e-3)
        print(M, K, N, nm, "maxabs", float(d.max()), "worst allclose ratio", float(rel.max()))
