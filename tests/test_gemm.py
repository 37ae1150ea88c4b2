"""gemm.hip: split-K fp32 Aᵀ·B (the LSTM weight-gradient product) against an fp64 torch oracle."""
import pytest
import torch

from avenir_amd import _native


@pytest.mark.gpu
@pytest.mark.parametrize("K,M,N", [(5000, 400, 106), (5000, 400, 201), (777, 33, 65), (64, 1, 1), (100_000, 64, 64), (40_000, 400, 106),
                                   (31, 130, 70), (3, 5, 7)])
def test_gemm_tn_vs_fp64(cuda, K, M, N):
    g = torch.Generator().manual_seed(K + M + N)
    A, B = torch.randn(K, M, generator=g), torch.randn(K, N, generator=g)
    C = _native.C().gemm_tn(A.to(cuda), B.to(cuda)).cpu()
    ref = A.double().t() @ B.double()
    err = (C.double() - ref).abs().max().item()
    assert err <= 1e-5 * (K ** 0.5) * 4, err        # fp32 accumulation over K products
    # deterministic: the slices are summed in a fixed order
    C2 = _native.C().gemm_tn(A.to(cuda), B.to(cuda)).cpu()
    assert torch.equal(C, C2)


@pytest.mark.gpu
@pytest.mark.parametrize("prec", [0, 3, 6])
@pytest.mark.parametrize("K,M,N", [(5000, 400, 106), (777, 33, 65), (100_000, 64, 64), (31, 130, 70)])
def test_gemm_tn_every_mode_vs_fp64(cuda, K, M, N, prec):
    """fp32 MFMA (0) and the split-bf16 x3 / x6 paths (3 / 6) all within the fp32 tolerance."""
    g = torch.Generator().manual_seed(K + M + N + prec)
    A, B = torch.randn(K, M, generator=g), torch.randn(K, N, generator=g)
    C = _native.C().gemm_tn(A.to(cuda), B.to(cuda), prec=prec).cpu()
    err = (C.double() - A.double().t() @ B.double()).abs().max().item()
    assert err <= 1e-5 * (K ** 0.5) * 4, err
    assert torch.equal(C, _native.C().gemm_tn(A.to(cuda), B.to(cuda), prec=prec).cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(128, 768, 3072), (128, 2304, 768), (1, 3072, 768), (37, 200, 1000), (130, 130, 4099)])
@pytest.mark.parametrize("act", [0, 1, 6])
def test_linear_act_fwd_split_k_vs_fp64(cuda, M, N, K, act):
    """mlp.hip's split-K path (few output tiles over a long K: slices of K summed in order, then
    bias + activation) against fp64; deterministic across calls."""
    g = torch.Generator().manual_seed(M + N + K + act)
    X, W, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) / K ** 0.5, torch.randn(N, generator=g)
    Y = _native.C().linear_act_fwd(X.to(cuda), W.to(cuda), b.to(cuda), act).cpu()
    z = X.double() @ W.double().t() + b.double()
    ref = {0: z, 1: torch.relu(z), 6: torch.nn.functional.gelu(z)}[act]
    assert (Y.double() - ref).abs().max().item() <= 2e-5 * (K ** 0.5)
    assert torch.equal(Y, _native.C().linear_act_fwd(X.to(cuda), W.to(cuda), b.to(cuda), act).cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(700, 650, 96), (4096, 3072, 64), (65, 4100, 32), (1030, 1100, 100), (2048, 2304, 768)])
def test_linear_act_fwd_xcd_tile_order(cuda, M, N, K):
    """The XCD-aware grouped tile order (>= 64 output tiles, counts not a multiple of 8, a partial
    last group of tile rows) still covers every output tile exactly once."""
    g = torch.Generator().manual_seed(M + N)
    X, W, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) / K ** 0.5, torch.randn(N, generator=g)
    Y = _native.C().linear_act_fwd(X.to(cuda), W.to(cuda), b.to(cuda), 1).cpu()
    ref = torch.relu(X.double() @ W.double().t() + b.double())
    assert (Y.double() - ref).abs().max().item() <= 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("prec", [3, 6])
@pytest.mark.parametrize("M,N,K", [(4100, 2600, 100), (4096, 2560, 768), (3000, 3500, 1), (2600, 4100, 33),
                                   (3300, 3200, 1027)])
def test_linear_act_fwd_planes_vs_fp64(cuda, M, N, K, prec):
    """The pre-split term-plane path (outputs >= 1,024 x 1,024 in the split-bf16 modes: bf16 term
    planes with K zero-padded to 32, LDS-DMA ring): ragged tile edges (clamped source rows), K not a
    multiple of 32 or of 4, against fp64 at the mode's tolerance; deterministic across calls."""
    g = torch.Generator().manual_seed(M + N + K + prec)
    X, W, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) / K ** 0.5, torch.randn(N, generator=g)
    C = _native.C()
    assert C.linear_act_fwd_planes_bytes(M, N, K, prec) > 0          # the shape takes the planes path
    Y = C.linear_act_fwd(X.to(cuda), W.to(cuda), b.to(cuda), 6, prec).cpu()
    ref = torch.nn.functional.gelu(X.double() @ W.double().t() + b.double())
    err = (Y.double() - ref).abs().max().item()
    assert err <= (2e-5 if prec == 6 else 1.5e-4) * max(1.0, K ** 0.25), err
    assert torch.equal(Y, C.linear_act_fwd(X.to(cuda), W.to(cuda), b.to(cuda), 6, prec).cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("prec", [3, 6])
def test_linear_act_fwd_cached_weight_planes(cuda, prec):
    """w_planes (the weight's bf16 term planes, split once) gives the bit-identical result of the
    per-call split; a mismatched planes tensor is refused."""
    g = torch.Generator().manual_seed(prec)
    M, N, K = 4096, 2600, 200
    X, W, b = (torch.randn(M, K, generator=g).to(cuda), (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda),
               torch.randn(N, generator=g).to(cuda))
    C = _native.C()
    assert C.linear_act_fwd_planes_bytes(M, N, K, prec) > 0
    P = C.sbf16_weight_planes(W, prec)
    assert torch.equal(C.linear_act_fwd(X, W, b, 1, prec, P), C.linear_act_fwd(X, W, b, 1, prec))
    with pytest.raises(RuntimeError):
        C.linear_act_fwd(X, W, b, 1, prec, P[:-2])
    assert C.sbf16_weight_planes(W, 0) is None


@pytest.mark.gpu
def test_linear_act_fwd_beyond_the_row_grid_limit(cuda):
    """More than 2^22 rows (65,535 row tiles of 64): the forward runs in row chunks."""
    g = torch.Generator().manual_seed(5)
    M, N, K = (1 << 22) + 4100, 8, 4
    X, W, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g), torch.randn(N, generator=g)
    Y = _native.C().linear_act_fwd(X.to(cuda), W.to(cuda), b.to(cuda), 1).cpu()
    ref = torch.relu(X.double() @ W.double().t() + b.double())
    # any process mode (x3's ~2^-17 per product included); a mis-offset chunk is off by O(1)
    assert (Y.double() - ref).abs().max().item() <= 5e-4


@pytest.mark.gpu
@pytest.mark.parametrize("prec", [3, 6])
def test_linear_act_fwd_random_shapes_every_path(cuda, prec):
    """Seeded random shapes across the dispatcher's paths (split-K for few tiles, 64 / 128 in-loop
    tiles, the planes path from 513 / 640 tiles; ragged edges, odd K, K = 1): fp64 oracle at the
    mode's tolerance and bit-identical repeats."""
    import random
    rnd = random.Random(prec)
    C = _native.C()
    seen_planes = seen_split = 0
    for _ in range(24):
        M = rnd.choice([1, 7, 129, 1000, 2049, 4097, 6000])
        N = rnd.choice([3, 64, 130, 767, 1025, 2500, 3100])
        K = rnd.choice([1, 5, 33, 96, 257, 768, 1500])
        if M * N * K > 3e9:                 # keep the fp64 oracle on the host quick
            K = 33
        g = torch.Generator().manual_seed(M * 7 + N * 13 + K)
        X, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) / K ** 0.5
        b = torch.randn(N, generator=g)
        seen_planes += C.linear_act_fwd_planes_bytes(M, N, K, prec) > 0
        seen_split += C.linear_act_fwd_planes_bytes(M, N, K, prec) == 0 and M * N < 256 * 4096
        Y = C.linear_act_fwd(X.to(cuda), W.to(cuda), b.to(cuda), 1, prec)
        ref = torch.relu(X.double() @ W.double().t() + b.double())
        err = (Y.cpu().double() - ref).abs().max().item()
        assert err <= (2e-5 if prec == 6 else 1.5e-4) * max(1.0, K ** 0.25), (M, N, K, err)
        assert torch.equal(Y, C.linear_act_fwd(X.to(cuda), W.to(cuda), b.to(cuda), 1, prec)), (M, N, K)
    assert seen_planes and seen_split
