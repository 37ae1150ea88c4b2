"""K26 column moments and K23 leave-one-out encoding (encode.hip) against their fp64 PyTorch
oracles; CPU cases check the oracles against plain formulas (and the old per-column loop)."""
import math

import pytest
import torch

from avenir_amd.ops import encode_ops as E


def _loo_loop(codes, n, y, reg, u, amp):
    """The pre-kernel per-column formulation of models.explore.leave_one_out_encoding."""
    y = y[:n].double()
    gm = y.mean()
    cols = []
    for j in range(codes.shape[0]):
        c = codes[j, :n].long()
        m = 65536 if codes.dtype == torch.uint16 else 256
        s = torch.zeros(m, dtype=torch.float64).index_add_(0, c, y)
        k = torch.zeros(m, dtype=torch.float64).index_add_(0, c, torch.ones_like(y))
        v = (s[c] - y + reg * gm) / (k[c] - 1 + reg).clamp_min(1e-12)
        if u is not None:
            v = v * (1 + amp * (2 * u[j] - 1))
        cols.append(v.float())
    return torch.stack(cols, 1)


def test_column_moments_cpu_oracle():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 1001, generator=g, dtype=torch.float64) * 2 + 5
    x[1, 7] = float("nan")
    r = E.column_moments(x)
    for f in range(3):
        v = x[f][~torch.isnan(x[f])]
        assert r[f, 0] == v.numel()
        assert torch.isclose(r[f, 7], v.mean())
        assert torch.isclose(r[f, 4], ((v - v.mean()) ** 2).mean())
        assert r[f, 2] == v.min() and r[f, 3] == v.max()
    d = E.moments_dict(r[0])
    v = x[0]
    sd = ((v - v.mean()) ** 2).mean().sqrt()
    assert math.isclose(d["skew"], float(((v - v.mean()) ** 3).mean() / sd ** 3), rel_tol=1e-9)


@pytest.mark.parametrize("wide", [False, True])
def test_loo_cpu_matches_loop(wide):
    g = torch.Generator().manual_seed(1)
    n, F = 777, 3
    hi = 3000 if wide else 40
    codes = torch.randint(0, hi, (F, 800), generator=g).to(torch.uint16 if wide else torch.uint8)
    y = torch.rand(n, generator=g, dtype=torch.float64)
    u = torch.rand(F, n, generator=g, dtype=torch.float64)
    s, k = E.loo_stats(codes, n, y)
    out = E.loo_apply(codes, n, y, s, k, y.mean().view(1), reg=2.0, noise=u, amp=0.1)
    assert torch.allclose(out, _loo_loop(codes, n, y, 2.0, u, 0.1))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,n,F", [(torch.float32, 1 << 20, 3), (torch.float32, 1001, 1),
                                       (torch.float64, 300_000, 5), (torch.float32, 5, 2)])
def test_column_moments_gpu(cuda, dtype, n, F):
    g = torch.Generator().manual_seed(2)
    ld = (n + 3) // 4 * 4
    x = (torch.randn(F, ld, generator=g, dtype=torch.float64).exp() * 3 - 1).to(dtype)
    x[0, n // 2] = float("nan")
    ref = E.column_moments(x[:, :n].double())
    got = E.column_moments(x.to(cuda), n).cpu()
    assert torch.equal(got[:, 0], ref[:, 0])
    assert torch.equal(got[:, 2:4], ref[:, 2:4])
    assert torch.allclose(got, ref, rtol=1e-9, atol=1e-9)
    # deterministic: a second run gives the same bits
    assert torch.equal(got, E.column_moments(x.to(cuda), n).cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("wide,n,F", [(False, 1 << 20, 4), (False, 1000, 40), (True, 200_000, 3)])
def test_loo_gpu_matches_cpu(cuda, wide, n, F):
    g = torch.Generator().manual_seed(3)
    hi = 10_000 if wide else 200
    codes = torch.randint(0, hi, (F, n + 16), generator=g).to(torch.uint16 if wide else torch.uint8)
    y = torch.rand(n, generator=g, dtype=torch.float64)
    u = torch.rand(F, n, generator=g, dtype=torch.float64)
    s, k = E.loo_stats(codes, n, y)
    sg, kg = E.loo_stats(codes.to(cuda), n, y.to(cuda))
    assert torch.equal(kg.cpu(), k)
    assert torch.allclose(sg.cpu(), s, rtol=1e-12, atol=1e-9)
    ref = E.loo_apply(codes, n, y, s, k, y.mean().view(1), reg=1.5, noise=u, amp=0.05)
    got = E.loo_apply(codes.to(cuda), n, y.to(cuda), sg, kg, y.mean().view(1).to(cuda), reg=1.5,
                      noise=u.to(cuda), amp=0.05).cpu()
    assert got.shape == (n, F)
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_explorer_getstats_gpu(cuda):
    from avenir_amd.analytics.explorer import DataExplorer
    g = torch.Generator().manual_seed(4)
    x = torch.randn(50_001, generator=g, dtype=torch.float64).exp()
    dc, dg = DataExplorer(device="cpu"), DataExplorer(device=cuda)
    dc.addListNumericData(x.tolist(), "x")
    dg.addListNumericData(x.tolist(), "x")
    a, b = dc.getStats("x"), dg.getStats("x")
    for key in ("mean", "std", "skew", "kurtosis", "min", "max", "median"):
        assert math.isclose(a[key], b[key], rel_tol=1e-9), key


@pytest.mark.gpu
def test_incremental_pca_kernel_matches_cpu(cuda):
    """K24 spirit_kernel (one wave per key) == the torch recurrence on the CPU, across two update
    calls (state carried), keys of different lengths and unit growth / shrink."""
    from avenir_amd.analytics import IncrementalPCA
    g = torch.Generator().manual_seed(5)
    D = 12
    mix = torch.randn(D, D, generator=g, dtype=torch.float64)
    streams = [{f"k{j}": (torch.randn(40 + 7 * j, D, generator=g, dtype=torch.float64) * torch.linspace(3, 0.1, D,
                dtype=torch.float64)) @ mix for j in range(5)} for _ in range(2)]
    a, b = IncrementalPCA(D, init_hidden=1, forget=0.97), IncrementalPCA(D, init_hidden=1, forget=0.97, device=cuda)
    for i, s in enumerate(streams):     # host streams, then device streams (padded on the device)
        sa, sb = a.update(s), b.update(s if i == 0 else {k: v.to(cuda) for k, v in s.items()})
    for key in sa:
        assert sa[key].num_hidden == sb[key].num_hidden and sa[key].count == sb[key].count
        assert torch.allclose(sa[key].components, sb[key].components.cpu(), rtol=1e-8, atol=1e-9)
        assert all(math.isclose(x, y, rel_tol=1e-8, abs_tol=1e-12)
                   for x, y in zip(sa[key].hidden_unit_energy, sb[key].hidden_unit_energy))
