"""SVM without the N x N matrix: the implicit-kernel working-set solver.

GPU: the implicit K[ws, ws] gather and gradient update (VALU for d <= 64, f32 MFMA beyond) against
torch fp32 oracles for every kernel kind; the MFMA kernel matrix (any d) against fp64; the
production path at N = 8192 (implicit kernel, native loop) against an fp64 ``smo_reference`` dual
objective (rel 1e-4) and sklearn's support-vector count (within 1 %); one-vs-rest and cascade
batches on the implicit kernel against the dense one.  CPU: the implicit kernel materialises to
the same matrices."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from avenir_amd import _native
from avenir_amd.models import svm as S

KINDS = ["linear", "poly", "rbf", "sigmoid"]


def _x(n, d, seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, d, generator=g) / d ** 0.5).to(device)


def _k64(A, B, kind, gamma, coef0=0.5, degree=3):
    A, B = A.double().cpu(), B.double().cpu()
    dot = A @ B.T
    if kind == "linear":
        return dot
    if kind == "poly":
        return (gamma * dot + coef0) ** degree
    if kind == "sigmoid":
        return torch.tanh(gamma * dot + coef0)
    d2 = (A * A).sum(1).view(-1, 1) + (B * B).sum(1).view(1, -1) - 2 * dot
    return torch.exp(-gamma * d2.clamp_min(0))


def test_implicit_kernel_dense_equals_kernel_matrix():
    X = _x(300, 7)
    for kind in KINDS:
        ik = S.ImplicitKernel(X, kind, 0.7, 0.5, 3)
        K = ik.dense()
        assert K.shape == (1, 300, 300)
        assert torch.allclose(K[0].double(), _k64(X, X, kind, 0.7), atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("d", [5, 16, 100, 300])
@pytest.mark.parametrize("kind", KINDS)
def test_kernel_matrix_any_d(cuda, d, kind):
    A, B = _x(777, d, 1, cuda), _x(515, d, 2, cuda)
    K = S.kernel_matrix(A, B, kind, 0.8, 3, 0.5).double().cpu()
    ref = _k64(A, B, kind, 0.8)
    assert torch.allclose(K, ref, atol=2e-5 * max(1.0, float(ref.abs().max())), rtol=1e-4)


def _ws(B, N, seed):
    g = torch.Generator().manual_seed(seed)
    ws = torch.stack([torch.randperm(N, generator=g)[:128] for _ in range(B)])
    ok = torch.rand(B, 128, generator=g) > 0.2
    dA = torch.randn(B, 128, generator=g) * ok
    dA[:, 5] = 0.0                         # zero changes are skipped by the compaction
    return ws, ok, dA


@pytest.mark.gpu
@pytest.mark.parametrize("d", [3, 16, 64, 100])
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("mfma", [False, True])
def test_implicit_gather_and_update_match_oracle(cuda, d, kind, mfma, monkeypatch):
    if mfma:
        monkeypatch.setenv("AVMI_SVM_MFMA_UPDATE", "1")
    B, N = 2, 3001
    X = _x(N, d, 3, cuda)
    ik = S.ImplicitKernel(X, kind, 0.6, 0.5, 3)
    ws, ok, dA = _ws(B, N, 4)
    Kd = _k64(X, X, kind, 0.6)
    C = _native.C()
    Kws = C.smo_ws_gather_x(*ik.args(), ws.to(cuda), ok.to(cuda), N).double().cpu()
    for b in range(B):
        ref = Kd[ws[b]][:, ws[b]]
        m = ok[b].view(-1, 1) & ok[b].view(1, -1)
        assert torch.allclose(Kws[b][m], ref[m], atol=3e-5 * max(1.0, float(ref.abs().max())), rtol=1e-4)
    y = torch.where(torch.rand(B, N) > 0.5, 1.0, -1.0)
    G0 = torch.randn(B, N + 1)
    G = G0.clone().to(cuda)
    C.smo_ws_update_x(*ik.args(), ws.to(cuda), dA.to(cuda), ok.to(cuda), y.to(cuda), G)
    for b in range(B):
        sel = ok[b] & (dA[b] != 0)
        ref = G0[b, :N].double() + y[b].double() * (dA[b][sel].double() @ Kd[ws[b][sel]])
        scale = float(dA[b].abs().sum()) * max(1.0, float(Kd.abs().max()))
        assert torch.allclose(G[b, :N].double().cpu(), ref, atol=2e-5 * scale)


def _blobs(n, d=16, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)).astype(np.float32)
    w = rng.normal(size=d)
    y = np.where(X @ w + 0.8 * rng.normal(size=n) > 0, 1, 0)
    return X, y


def _dual(alpha, y, X, gamma):
    K = _k64(torch.tensor(X), torch.tensor(X), "rbf", gamma).numpy()
    ys = np.where(y > 0, 1.0, -1.0)
    a = alpha.astype(np.float64)
    v = a * ys
    return 0.5 * v @ K @ v - a.sum(), K, ys


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["implicit", "dense"])
def test_production_path_n8192_matches_fp64_dual_and_sklearn(cuda, monkeypatch, path):
    """The production working-set paths at N = 8192 x 16 RBF (native C++ outer loop, two-level
    selection with the rank merge, graph-captured step blocks): the implicit kernel (rows from X,
    the path above DENSE_MAX_N rows) and the dense kernel matrix."""
    from sklearn.svm import SVC as SKSVC
    monkeypatch.setattr(S, "DENSE_MAX_N", 0 if path == "implicit" else 1 << 30)
    X, y = _blobs(8192)
    m = S.SVC(kernel="rbf", C=1.0, gamma=0.05, eps=1e-3).fit(torch.tensor(X, device=cuda), torch.tensor(y, device=cuda))
    assert S.LAST_SOLVE.get("solver") == ("ws-implicit" if path == "implicit" else "ws")
    alpha = np.zeros(len(y))
    dc = m.dual_coef[0].double().cpu().numpy()
    alpha[m.support_.cpu().numpy()] = np.abs(dc)
    f_gpu, K, ys = _dual(alpha, y, X, 0.05)
    a_ref, _, _ = S.smo_reference(K, ys, 1.0, 1e-3, max_iter=2_000_000)
    f_ref = 0.5 * (a_ref * ys) @ K @ (a_ref * ys) - a_ref.sum()
    assert abs(f_gpu - f_ref) <= 1e-4 * abs(f_ref)
    sk = SKSVC(C=1.0, kernel="rbf", gamma=0.05, tol=1e-3).fit(X, y)
    n_sk = int(sk.n_support_.sum())
    assert abs(int(m.support_.numel()) - n_sk) <= 0.01 * n_sk + 1
    assert float((m.predict(torch.tensor(X, device=cuda)).cpu().numpy() == sk.predict(X)).mean()) > 0.995


@pytest.mark.gpu
def test_implicit_one_vs_rest_and_cascade_equal_dense(cuda, monkeypatch):
    rng = np.random.default_rng(5)
    X = rng.normal(size=(3000, 24)).astype(np.float32)
    y = (X[:, 0] > 0.5).astype(int) + (X[:, 1] > 0).astype(int) * (X[:, 0] <= 0.5)
    Xt, yt = torch.tensor(X, device=cuda), torch.tensor(y, device=cuda)
    yb = torch.tensor((y > 0).astype(int), device=cuda)
    dense = S.SVC(kernel="rbf", C=2.0, gamma=0.1).fit(Xt, yt)
    c_dense = S.CascadeSVM(shards=3, kernel="rbf", C=1.0, gamma=0.1).fit(Xt, yb)
    monkeypatch.setattr(S, "DENSE_MAX_N", 0)
    imp = S.SVC(kernel="rbf", C=2.0, gamma=0.1).fit(Xt, yt)
    assert S.LAST_SOLVE.get("solver") == "ws-implicit"
    agree = float((dense.predict(Xt) == imp.predict(Xt)).float().mean())
    assert agree > 0.995
    assert abs(int(dense.support_.numel()) - int(imp.support_.numel())) <= 0.02 * int(dense.support_.numel()) + 2
    c_imp = S.CascadeSVM(shards=3, kernel="rbf", C=1.0, gamma=0.1).fit(Xt, yb)
    assert float((c_dense.predict(Xt) == c_imp.predict(Xt)).float().mean()) > 0.99


@pytest.mark.gpu
def test_large_n_fits_without_the_matrix(cuda, monkeypatch):
    """N = 65 536 x 16 RBF through the implicit kernel: peak device memory stays O(N D), far below
    the 17 GB a dense N x N fp32 matrix would take."""
    X, y = _blobs(65536, seed=7)
    Xt, yt = torch.tensor(X, device=cuda), torch.tensor(y, device=cuda)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    m = S.SVC(kernel="rbf", C=1.0, gamma=0.05).fit(Xt, yt)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    assert S.LAST_SOLVE.get("solver") == "ws-implicit"
    assert peak < 2e9                      # the dense matrix alone: 17.2 GB
    acc = float((m.predict(Xt) == yt).float().mean())
    assert acc > 0.9
