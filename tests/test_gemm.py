"""gemm.hip: split-K fp32 Aᵀ·B (the LSTM weight-gradient product) against an fp64 torch oracle."""
import pytest
import torch

from avenir_amd import _native


@pytest.mark.gpu
@pytest.mark.parametrize("K,M,N", [(5000, 400, 106), (5000, 400, 201), (777, 33, 65), (64, 1, 1), (100_000, 64, 64),
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
