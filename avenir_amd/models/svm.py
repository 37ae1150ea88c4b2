"""Kernel support vector machines: SMO (K12) and the cascade SVM.

Reference: ``SequentialMinimalOptimization`` (J/discriminant/SequentialMinimalOptimization.java:77-556;
linear kernel only — and ``LinearKernel.compute`` returns 0, J/discriminant/LinearKernel.java:36,
so the reference SVM cannot train at all), the cascade ``SupportVectorMachine`` MR job
(J/discriminant/SupportVectorMachine.java:97-196: SMO per mapper split, final SMO over the union
of support vectors), and the sklearn wrapper ``SupportVectorMachine`` (P/supv/svm.py:83-121:
svc with linear / poly / rbf / sigmoid kernels, C, gamma).

MI355X design: small problems build K = kernel(X X^T) once (the fused RBF pass for d <= 64, f32
MFMA for any other d / kernel) and run SMO inside one persistent workgroup per problem (svm.hip);
larger ones run the working-set decomposition, either over that dense K or — above
``DENSE_MAX_N`` rows, or when K would not fit — over an IMPLICIT kernel: every outer step
recomputes the Q x Q sub-problem block and the Q x N gradient-update rows from the rows of X
(``smo_ws_run_x``; VALU from squared differences for d <= 64, f32 MFMA beyond), so memory is
O(N D): N = 262 144 x 16 needs ~30 MB instead of the 275 GB N x N matrix.  For wide rows (D >= 256
by default) an HBM LRU cache of kernel rows (``row_cache_slots``) serves the rows the working
sets revisit and only the misses are recomputed.  There is no row cap: the working-set selection
streams any N (the streaming top-k parts of svm.hip).  B problems — one-vs-rest
classes or cascade shards — are B workgroups of ONE launch.  The CPU path runs the same algorithm
in numpy.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import _native
from ..parallel.comm import Comm, get_comm
from ..utils.tracing import traced


KERNEL_KIND = {"linear": 0, "poly": 1, "rbf": 2, "sigmoid": 3}


def kernel_matrix(A: torch.Tensor, B: torch.Tensor, kernel: str = "rbf", gamma: float = 1.0, degree: int = 3,
                  coef0: float = 0.0) -> torch.Tensor:
    """K(A, B) [na, nb] float32.  GPU: RBF with d <= 64 is one fused pass of the ``rbf_matrix``
    kernel from squared differences; every other (kernel, d) is the f32-MFMA tile kernel
    (``svm_kernel_matrix``, v_mfma_f32_16x16x4_f32) with the kernel applied in its epilogue.
    CPU: one GEMM + the elementwise kernel."""
    A, B = A.float(), B.float()
    if A.is_cuda and A.shape[0] and B.shape[0] and kernel in KERNEL_KIND:
        if kernel == "rbf" and 1 <= A.shape[1] <= 64:
            return _native.C().rbf_matrix(A.contiguous(), B.contiguous(), float(gamma))
        return _native.C().svm_kernel_matrix(A.contiguous(), B.contiguous(), KERNEL_KIND[kernel], float(gamma),
                                             float(coef0), int(degree))
    dot = A @ B.T
    if kernel == "linear":
        return dot
    if kernel == "poly":
        return (gamma * dot + coef0) ** degree
    if kernel == "sigmoid":
        return torch.tanh(gamma * dot + coef0)
    if kernel == "rbf":
        na, nb = (A * A).sum(1), (B * B).sum(1)
        return torch.exp(-gamma * (na.view(-1, 1) + nb.view(1, -1) - 2 * dot).clamp_min(0))
    raise ValueError(f"unknown kernel {kernel}")


class ImplicitKernel:
    """The kernel of B problems as the rows of X instead of an N x N matrix: X [N, D] (shared by all
    problems) or [B, N, D] (one row set per problem, e.g. cascade shards), squared norms, kernel
    parameters.  ``dense()`` materialises K for small problems and the CPU path."""

    def __init__(self, X: torch.Tensor, kernel: str = "rbf", gamma: float = 1.0, coef0: float = 0.0, degree: int = 3):
        self.X = X.float().contiguous()
        self.xn = (self.X * self.X).sum(-1).contiguous()
        self.kernel, self.kind = kernel, KERNEL_KIND[kernel]
        self.gamma, self.coef0, self.degree = float(gamma), float(coef0), int(degree)

    @property
    def device(self) -> torch.device:
        return self.X.device

    @property
    def N(self) -> int:
        return int(self.X.shape[-2])

    def dense(self) -> torch.Tensor:
        """[B or 1, N, N]."""
        Xs = self.X if self.X.dim() == 3 else self.X.unsqueeze(0)
        return torch.stack([kernel_matrix(x, x, self.kernel, self.gamma, self.degree, self.coef0) for x in Xs])

    def args(self) -> tuple:
        return (self.X, self.xn, self.kind, self.gamma, self.coef0, self.degree)


#: above this many rows (or when the dense matrices would not fit in free memory) the working-set
#: solver runs on the implicit kernel
DENSE_MAX_N = int(__import__("os").environ.get("AVMI_SVM_DENSE_MAX_N", "16384"))


def use_implicit(n: int, n_mats: int, device) -> bool:
    """Whether a problem of ``n`` rows (``n_mats`` dense N x N matrices) takes the implicit kernel."""
    if torch.device(device).type != "cuda":
        return False
    if n > DENSE_MAX_N:
        return True
    free, _ = torch.cuda.mem_get_info(torch.device(device))
    return 4.0 * n * n * n_mats > 0.5 * free


#: kernel-row cache of the implicit solver: "auto" (on when recomputing a row costs more than
#: reading it back, D >= AVMI_SVM_CACHE_MIN_D (default 256), AND the cache holds at least a quarter
#: of the rows), "0" (off) or a slot count.  Measured (profiles/r5_svm_cache_*): 16,384 rows at
#: d = 512, 73 % hits: 0.140 s vs 0.158 s; at d = 128, 77 % hits: 0.072 s vs 0.065 s (the f32-MFMA
#: row recompute is cheaper than the cache traffic); 4,096 slots for 65,536-262,144 rows: 0.01-4 %
#: hits, up to 5x slower — hence the quarter-of-the-rows rule
ROW_CACHE = __import__("os").environ.get("AVMI_SVM_CACHE", "auto")
ROW_CACHE_MIN_D = int(__import__("os").environ.get("AVMI_SVM_CACHE_MIN_D", "256"))


def row_cache_slots(K: "ImplicitKernel", B: int) -> int:
    """Slots of the HBM kernel-row cache (svm.hip svm_cache_lookup_kernel) for an implicit-kernel
    solve: 0 when off (several problems, per-problem X; under "auto" small D or fewer than N / 4
    slots); else up to 16,384 rows ("auto": N / 2), within a quarter of the device's free memory
    (one slot = N fp32 values).  Every outer
    step the working set's rows come from the cache (LRU within 8-way sets) and only the misses are
    recomputed from X — the reference's SMO memoises kernel values the same way
    (J/discriminant/SequentialMinimalOptimization.java:511-524)."""
    if B != 1 or K.X.dim() == 3 or K.device.type != "cuda":
        return 0
    mode = str(ROW_CACHE)
    if mode in ("0", "off", "false"):
        return 0
    D = int(K.X.shape[-1])
    if mode == "auto" and D < ROW_CACHE_MIN_D:
        return 0
    N = K.N
    want = (N + 1) // 2 if mode in ("auto", "on", "1", "true") else int(mode)
    free, _ = torch.cuda.mem_get_info(K.device)
    fit = int(0.25 * free // (4 * N)) - 128
    slots = max(0, min(want, fit, 16384)) // 8 * 8
    if mode == "auto" and 4 * slots < N:
        return 0
    return slots


def smo_reference(K: np.ndarray, y: np.ndarray, C: float, eps: float = 1e-3, max_iter: int = 100000,
                  alpha0: np.ndarray | None = None, G0: np.ndarray | None = None):
    """Host SMO with the same working-set selection and update as ``smo_kernel`` (and, from a
    given (alpha0, G0), as the working-set kernel ``smo_ws_kernel``).  Returns (alpha, G, iterations)."""
    K = np.asarray(K, np.float64)
    y = np.asarray(y, np.float64)
    N = y.size
    valid = y != 0
    alpha = np.zeros(N) if alpha0 is None else np.asarray(alpha0, np.float64).copy()
    G = np.where(valid, -1.0, 0.0) if G0 is None else np.asarray(G0, np.float64).copy()
    QD = np.diag(K).copy()
    it = 0
    for it in range(max_iter):
        up = valid & np.where(y > 0, alpha < C, alpha > 0)
        low = valid & np.where(y > 0, alpha > 0, alpha < C)
        if not up.any():
            break
        v = np.where(up, -y * G, -np.inf)
        i = int(np.argmax(v))
        gmax = v[i]
        yg = np.where(low, y * G, -np.inf)
        gmax2 = yg.max() if low.any() else -np.inf
        bd = gmax + yg
        a = QD[i] + QD - 2 * K[i]
        a = np.where(a > 0, a, 1e-12)
        gain = np.where(low & (bd > 0), bd * bd / a, -np.inf)
        j = int(np.argmax(gain))
        if gmax + gmax2 < eps or not np.isfinite(gain[j]):
            break
        yi, yj, oi, oj = y[i], y[j], alpha[i], alpha[j]
        ai, aj = oi, oj
        quad = QD[i] + QD[j] - 2 * K[i, j]
        quad = quad if quad > 0 else 1e-12
        if yi != yj:
            delta = (-G[i] - G[j]) / quad
            diff = ai - aj
            ai += delta
            aj += delta
            if diff > 0:
                if aj < 0:
                    aj, ai = 0.0, diff
            elif ai < 0:
                ai, aj = 0.0, -diff
            if diff > 0:
                if ai > C:
                    ai, aj = C, C - diff
            elif aj > C:
                aj, ai = C, C + diff
        else:
            delta = (G[i] - G[j]) / quad
            s = ai + aj
            ai -= delta
            aj += delta
            if s > C:
                if ai > C:
                    ai, aj = C, s - C
            elif aj < 0:
                aj, ai = 0.0, s
            if s > C:
                if aj > C:
                    aj, ai = C, s - C
            elif ai < 0:
                ai, aj = 0.0, s
        alpha[i], alpha[j] = ai, aj
        G += np.where(valid, y * (K[i] * (ai - oi) * yi + K[j] * (aj - oj) * yj), 0.0)
    return alpha, G, it


def _rho(alpha: torch.Tensor, G: torch.Tensor, y: torch.Tensor, C: float) -> torch.Tensor:
    """Bias per problem (LIBSVM-style): mean of y*G over free SVs, else the midpoint of bounds."""
    yg = y * G
    valid = y != 0
    at_ub = valid & (alpha >= C)
    at_lb = valid & (alpha <= 0)
    free = valid & ~at_ub & ~at_lb
    inf = torch.full_like(yg, float("inf"))
    ub_mask = (at_ub & (y < 0)) | (at_lb & (y > 0))
    lb_mask = (at_ub & (y > 0)) | (at_lb & (y < 0))
    ub = torch.where(ub_mask, yg, inf).min(-1).values
    lb = torch.where(lb_mask, yg, -inf).max(-1).values
    nf = free.sum(-1)
    sf = torch.where(free, yg, torch.zeros_like(yg)).sum(-1)
    return torch.where(nf > 0, sf / nf.clamp_min(1), (ub + lb) / 2)


class _WorkingSetSMO:
    """State and one outer step of the working-set solver, written with static shapes so that a
    block of steps can be captured as one HIP graph (see ``smo_decomposition``)."""

    def __init__(self, K, y, C, eps, inner_iter, Q, fused=True, rel_tol=0.1):
        self.K, self.C, self.eps, self.inner_iter = K, float(C), float(eps), int(inner_iter)
        self.rel_tol = float(rel_tol)
        B, N = y.shape
        dev = K.device
        self.gpu = dev.type == "cuda"
        self.B, self.N, self.Q, self.h = B, N, Q, min(Q // 2, N)
        self.yf = y.float().contiguous()
        self.yp = torch.cat([self.yf, torch.zeros((B, 1), device=dev)], 1)     # slot N = unused
        self.alpha = torch.zeros((B, N + 1), device=dev)
        self.G = torch.where(self.yp != 0, -torch.ones_like(self.yp), torch.zeros_like(self.yp))
        self.rows = torch.arange(B, device=dev)
        self.inner_total = torch.zeros(B, dtype=torch.long, device=dev)
        self.gap = torch.full((B,), float("inf"), device=dev)
        self.ninf = torch.tensor(-float("inf"), device=dev)
        # fused selection / update kernels (one launch each instead of ~25 torch ops per step)
        self.fused = (fused and self.gpu and K.dtype == torch.float32 and K.is_contiguous() and N <= (1 << 18)
                      and Q == 128)
        if K.shape[0] == 1 and B > 1 and not self.fused:   # one shared K: a broadcast view for indexing
            self.K = K.expand(B, -1, -1)
        if self.fused:
            self.ws_buf = torch.zeros((B, Q), dtype=torch.long, device=dev)
            self.ok_buf = torch.zeros((B, Q), dtype=torch.bool, device=dev)
            self.dA_buf = torch.zeros((B, Q), device=dev)

    def refresh_gap(self):
        a, g, yf = self.alpha[:, :self.N], self.G[:, :self.N], self.yf
        up = (yf > 0) & (a < self.C) | (yf < 0) & (a > 0)
        low = (yf > 0) & (a > 0) | (yf < 0) & (a < self.C)
        vu = torch.where(up, -yf * g, self.ninf)
        vl = torch.where(low, yf * g, self.ninf)
        self.gap.copy_(vu.max(1).values + vl.max(1).values)
        return vu, vl

    def step(self):
        B, N, Q, h, dev = self.B, self.N, self.Q, self.h, self.K.device
        if self.fused:  # three launches: select, solve (gathers / scatter folded in), gradient update
            C_ = _native.C()
            C_.smo_ws_select(self.alpha, self.G, self.yf, self.C, Q // 2, self.ws_buf, self.ok_buf, self.gap)
            C_.smo_ws_solve_fused(self.K, self.ws_buf, self.ok_buf, self.alpha, self.G, self.yf, self.gap, self.C,
                                  self.eps, self.inner_iter, self.dA_buf, self.inner_total, self.rel_tol)
            C_.smo_ws_update(self.K, self.ws_buf, self.dA_buf, self.ok_buf, self.yf, self.G)
            return
        vu, vl = self.refresh_gap()
        vu_v, iu = torch.topk(vu, h, 1)
        vl_v, il = torch.topk(vl, h, 1)
        ws = torch.cat([iu, il], 1)
        ok = torch.cat([vu_v > -float("inf"),
                        (vl_v > -float("inf")) & ~(il.unsqueeze(2) == iu.unsqueeze(1)).any(2)], 1)
        if ws.shape[1] < Q:                                                # N < Q/2: pad the set
            pad = Q - ws.shape[1]
            ws = torch.cat([ws, torch.zeros((B, pad), dtype=ws.dtype, device=dev)], 1)
            ok = torch.cat([ok, torch.zeros((B, pad), dtype=torch.bool, device=dev)], 1)
        wsg = torch.where(ok, ws, torch.zeros_like(ws))
        yws = (self.yp.gather(1, wsg) * ok).contiguous()
        aws = self.alpha.gather(1, wsg).contiguous()
        gws = self.G.gather(1, wsg).contiguous()
        Kws = self.K[self.rows.view(-1, 1, 1), wsg.unsqueeze(2), wsg.unsqueeze(1)].float().contiguous()
        a_old = aws.clone()
        gap = torch.where(torch.isfinite(self.gap), self.gap, torch.zeros_like(self.gap)).contiguous()
        if self.gpu:
            it = _native.C().smo_ws_solve(Kws, yws, aws, gws, gap, self.C, self.eps, self.inner_iter)
        else:
            its = []
            for b in range(B):
                an, _, ib = smo_reference(Kws[b].double().numpy(), yws[b].double().numpy(), self.C,
                                          max(self.eps, 0.1 * float(gap[b])), self.inner_iter,
                                          aws[b].double().numpy(), gws[b].double().numpy())
                aws[b] = torch.from_numpy(an).float()
                its.append(ib)
            it = torch.tensor(its)
        self.inner_total += it.to(dev).long()
        dA = (aws - a_old) * yws
        self.alpha.scatter_(1, torch.where(ok, ws, torch.full_like(ws, N)), torch.where(ok, aws, torch.zeros_like(aws)))
        if self.fused:
            _native.C().smo_ws_update(self.K, ws, dA.contiguous(), ok, self.yf, self.G)
        else:
            Krows = self.K[self.rows.view(-1, 1), wsg].float()                 # [B, Q, N]
            self.G[:, :N] += self.yf * torch.bmm(dA.unsqueeze(1), Krows).squeeze(1)


def smo_decomposition(K: torch.Tensor, y: torch.Tensor, C: float, eps: float = 1e-3, max_outer: int = 100_000,
                      inner_iter: int = 2048, check_every: int = 16, Q: int | None = None, graph: bool = True,
                      fused: bool = True, rel_tol: float | None = None):
    """Working-set SMO for B problems (K [B, N, N], y [B, N] in {-1, 0, +1}).

    Each outer step picks the Q/2 largest violators of the "up" set and the Q/2 largest of the
    "low" set (the maximal violating pair is always among them), solves that Q-variable
    sub-problem to a relaxed tolerance max(eps, 0.1 gap) — on the GPU in ``smo_ws_kernel``, one
    wavefront per problem with the Q x Q kernel block in LDS — and applies the alpha changes to
    the full gradient with one batched GEMV.  On the GPU with the fused kernels the whole loop runs
    in C++ (``smo_ws_run``: blocks of 8 steps queued back to back, the gap of the previous block
    tested while the next one runs, steps past convergence are no-op launches); otherwise (or with
    AVMI_SMO_LOOP=graph) ``check_every`` steps are one captured HIP graph (static shapes; steps
    after convergence are no-ops because the sub-problem solver stops at once), and the host reads
    the global violation gap once per replay.  Stops when the gap < eps.  ``fused`` (GPU, float32 K, N <= 2^18): the working-set selection and the
    gradient update are one kernel each (``smo_ws_select`` / ``smo_ws_update``) instead of ~25
    torch ops.  Returns (alpha, G, outer steps, inner steps).
    """
    Q = Q or (_native.C().smo_ws_size() if K.device.type == "cuda" else 128)
    if rel_tol is None:   # sub-problem tolerance max(eps, rel_tol * gap) of the fused GPU solver
        import os
        rel_tol = float(os.environ.get("AVMI_SMO_REL_TOL", "0.3"))
    if isinstance(K, ImplicitKernel):
        if K.device.type != "cuda":
            return smo_decomposition(K.dense(), y, C, eps, max_outer, inner_iter, check_every, Q, graph, fused,
                                     rel_tol)
        # the native loop over the implicit kernel: K[ws, ws] and the Q x N update rows from X
        B, N = y.shape
        dev = K.device
        yf = y.float().contiguous()
        alpha = torch.zeros((B, N + 1), device=dev)
        G = torch.where(torch.cat([yf, torch.zeros((B, 1), device=dev)], 1) != 0, -1.0, 0.0).contiguous()
        ws = torch.zeros((B, Q), dtype=torch.long, device=dev)
        ok = torch.zeros((B, Q), dtype=torch.bool, device=dev)
        dA = torch.zeros((B, Q), device=dev)
        inner_total = torch.zeros(B, dtype=torch.long, device=dev)
        gap = torch.full((B,), float("inf"), device=dev)
        slots = row_cache_slots(K, B)
        stats = torch.zeros(2, dtype=torch.long, device=dev)
        outer = int(_native.C().smo_ws_run_x(*K.args(), alpha, G, yf, float(C), float(eps), int(inner_iter),
                                             float(rel_tol), int(max_outer), 8, ws, ok, dA, inner_total, gap,
                                             cache_slots=slots, cache_stats=stats))
        if slots:
            h, m = (int(v) for v in stats.tolist())
            LAST_SOLVE.update(cache_slots=slots, cache_hits=h, cache_misses=m,
                              cache_hit_rate=h / max(1, h + m))
        return alpha[:, :N].contiguous(), G[:, :N].contiguous(), outer, inner_total
    st = _WorkingSetSMO(K, y, C, eps, inner_iter, Q, fused, rel_tol)
    outer = 0
    import os
    mode = os.environ.get("AVMI_SMO_LOOP", "native")   # native | graph | eager
    if st.fused and graph and mode == "native":
        # the step loop in C++ (smo_ws_run): no capture, no per-step Python; queued steps past
        # convergence are no-op launches
        outer = int(_native.C().smo_ws_run(K, st.alpha, st.G, st.yf, st.C, st.eps, st.inner_iter, st.rel_tol,
                                           int(max_outer), 8, st.ws_buf, st.ok_buf, st.dA_buf, st.inner_total,
                                           st.gap))
    elif st.gpu and graph and mode != "eager":
        st.step()                                # eager warm-up: allocator pool, kernel caches
        outer = 1
        from ..utils.hipgraph import capturing
        g = torch.cuda.CUDAGraph()
        with capturing(g, device=st.K.device):
            for _ in range(check_every):
                st.step()
            st.refresh_gap()
        # capture records without executing: replay the block until converged (the captured block
        # ends with refresh_gap, so the gap read after a replay is current)
        st.refresh_gap()
        while outer < max_outer:
            if bool((~(st.gap >= eps)).all()):
                break
            g.replay()
            outer += check_every
    else:
        while outer < max_outer:
            st.refresh_gap()
            if outer % check_every == 0 and bool((~(st.gap >= eps)).all()):
                break
            st.step()
            outer += 1
    N = st.N
    return st.alpha[:, :N].contiguous(), st.G[:, :N].contiguous(), outer, st.inner_total


WS_MIN_N = 4096   # above this the working-set solver beats the single-workgroup full SMO (bench_svm.py)
LAST_SOLVE: dict = {}   # outer-step count of the last working-set solve (benchmarks / diagnostics)


@traced("svm.smo", nbytes=lambda K, *a, **k: K.numel() * K.element_size(), device=lambda K, *a, **k: K.device)
def smo_batch(K: torch.Tensor, y: torch.Tensor, C: float, eps: float = 1e-3, max_iter: int = 1_000_000,
              solver: str = "auto"):
    """Solve B SVM duals: K [B, N, N] (or [1, N, N] shared by all B problems — one-vs-rest classes
    — which the working-set kernels read in place instead of B copies) or an :class:`ImplicitKernel`
    (rows of X, no N x N matrix), y [B, N] in {-1, 0 (padding), +1}.  Returns (alpha, rho, iters).
    ``solver``: "full" (one persistent workgroup runs plain SMO over all N), "ws" (working-set
    decomposition, ``smo_decomposition``) or "auto" (ws on the GPU for N > WS_MIN_N, always for an
    implicit kernel).

    Iteration caps: the full solver stops after ``max_iter`` two-variable steps.  The working-set
    solver stops after ``max(1, max_iter // 64)`` OUTER steps, each solving its sub-problem with
    at most ``min(2048, max_iter)`` two-variable steps — so its total two-variable step count can
    exceed ``max_iter`` (by up to 32x); ``max_iter`` is a bound on the outer work there, not on the
    inner steps (a cap of ``max_iter // inner_iter`` outer steps stopped large problems before
    convergence).  ``iters`` is the number of two-variable steps taken per problem in both cases
    (for the working-set path: the inner steps summed over the outer steps)."""
    B, N = y.shape
    if isinstance(K, ImplicitKernel):
        if K.device.type != "cuda":      # CPU: the same solvers over the materialised matrix
            return smo_batch(K.dense(), y, C, eps, max_iter, solver)
        inner_iter = min(2048, max(1, max_iter))
        alpha, G, outer, inner = smo_decomposition(K, y, C, eps, max_outer=max(1, max_iter // 64),
                                                   inner_iter=inner_iter)
        LAST_SOLVE.update(solver="ws-implicit", outer=outer)
        return alpha, _rho(alpha, G, y.float(), C), inner.int()
    if solver == "ws" or (solver == "auto" and K.device.type == "cuda" and N > WS_MIN_N):
        inner_iter = min(2048, max(1, max_iter))
        alpha, G, outer, inner = smo_decomposition(K, y, C, eps, max_outer=max(1, max_iter // 64),
                                                   inner_iter=inner_iter)
        LAST_SOLVE.update(solver="ws", outer=outer)
        return alpha, _rho(alpha, G, y.float(), C), inner.int()
    if K.shape[0] == 1 and B > 1:
        K = K.expand(B, -1, -1)
    if K.device.type == "cuda":
        Kc = K.float().contiguous()
        yc = y.float().contiguous()
        diag = torch.diagonal(Kc, dim1=1, dim2=2).contiguous()
        alpha = torch.zeros((B, N), dtype=torch.float32, device=K.device)
        G = torch.where(yc != 0, -torch.ones_like(yc), torch.zeros_like(yc)).contiguous()
        iters = _native.C().smo_solve(Kc, yc, diag, alpha, G, float(C), float(eps), int(max_iter))
        return alpha, _rho(alpha, G, yc, C), iters
    al, gs, its = [], [], []
    for b in range(B):
        a, g, it = smo_reference(K[b].double().numpy(), y[b].double().numpy(), C, eps, max_iter)
        al.append(torch.from_numpy(a).float())
        gs.append(torch.from_numpy(g).float())
        its.append(it)
    alpha, G = torch.stack(al), torch.stack(gs)
    return alpha, _rho(alpha, G, y.float(), C), torch.tensor(its, dtype=torch.int32)


class SVC:
    """Binary or one-vs-rest multi-class kernel SVM.  All classes' duals are solved in one launch."""

    def __init__(self, kernel: str = "rbf", C: float = 1.0, gamma: float | str = "scale", degree: int = 3,
                 coef0: float = 0.0, eps: float = 1e-3, max_iter: int = 1_000_000):
        self.kernel, self.C, self.gamma, self.degree, self.coef0 = kernel, C, gamma, degree, coef0
        self.eps, self.max_iter = eps, max_iter

    @classmethod
    def from_config(cls, conf) -> "SVC":
        """``train.*`` keys of P/supv/svm.py:83-121 (a :class:`~avenir_amd.utils.config.Configuration`)."""
        g = conf.get_string("train.gamma")[0] if "train.gamma" in conf.configs else "scale"
        try:
            g = float(g)
        except (TypeError, ValueError):
            pass
        return cls(kernel=conf.get_string("train.kernel.function")[0] or "rbf",
                   C=conf.get_float("train.penalty")[0] or 1.0, gamma=g,
                   degree=conf.get_int("train.poly.degree")[0] or 3)

    def _gamma(self, X):
        if isinstance(self.gamma, (int, float)):
            return float(self.gamma)
        if self.gamma == "auto":
            return 1.0 / X.shape[1]
        var = float(X.float().var())
        return 1.0 / (X.shape[1] * var) if var > 0 else 1.0

    def fit(self, X, y) -> "SVC":
        X = torch.as_tensor(X).float()
        y = torch.as_tensor(y, device=X.device).long().view(-1)
        self.classes = torch.unique(y).tolist()
        self.g = self._gamma(X)
        if use_implicit(X.shape[0], 1, X.device):
            K = ImplicitKernel(X, self.kernel, self.g, self.coef0, self.degree)
        else:
            K = kernel_matrix(X, X, self.kernel, self.g, self.degree, self.coef0)
        if len(self.classes) == 2:
            ys = torch.where(y == self.classes[1], 1.0, -1.0).view(1, -1)
        else:
            ys = torch.stack([torch.where(y == c, 1.0, -1.0) for c in self.classes])
        # one K for all one-vs-rest problems (smo_batch broadcasts it where a solver needs copies)
        alpha, rho, iters = smo_batch(K if isinstance(K, ImplicitKernel) else K.unsqueeze(0), ys.to(X.device),
                                      self.C, self.eps, self.max_iter)
        self.iters = iters.tolist()
        sv = (alpha > 0).any(0)
        self.support_ = sv.nonzero().view(-1)
        self.sv_X = X[self.support_]
        self.dual_coef = (alpha * ys.to(alpha.device))[:, self.support_]          # [B, nsv]
        self.rho = rho
        return self

    def decision_function(self, X) -> torch.Tensor:
        X = torch.as_tensor(X).float().to(self.sv_X.device)
        # blocks of query rows: [nsv, block] kernel tiles stay bounded for any number of queries
        blk = max(1, (1 << 28) // max(1, self.sv_X.shape[0]))
        outs = []
        for s in range(0, X.shape[0], blk):
            Kx = kernel_matrix(self.sv_X, X[s:s + blk], self.kernel, self.g, self.degree, self.coef0)   # [nsv, n]
            outs.append(self.dual_coef @ Kx - self.rho.view(-1, 1))
        f = torch.cat(outs, 1) if outs else torch.zeros((self.dual_coef.shape[0], 0), device=X.device)
        return f[0] if f.shape[0] == 1 else f.T

    def predict(self, X) -> torch.Tensor:
        f = self.decision_function(X)
        cls = torch.tensor(self.classes, device=f.device)
        if f.dim() == 1:
            return cls[(f > 0).long()]
        return cls[f.argmax(1)]

    def support_indexes(self) -> list[int]:
        """Support-vector row indexes (getSupVecIndexes, SequentialMinimalOptimization.java:545-556)."""
        return self.support_.tolist()


class CascadeSVM:
    """Cascade SVM (SupportVectorMachine.java:97-196): the rows are split into ``shards`` per rank,
    every shard's dual is solved in one batched launch, the support vectors of all shards and ranks
    are gathered (one all-gather-v), and a final SMO over that union gives the model."""

    def __init__(self, shards: int = 4, comm: Comm | None = None, **svc_kw):
        self.shards, self.comm, self.kw = shards, comm, svc_kw

    def fit(self, X, y) -> "CascadeSVM":
        comm = self.comm or get_comm()
        X = torch.as_tensor(X).float()
        y = torch.as_tensor(y, device=X.device).long().view(-1)
        base = SVC(**self.kw)
        classes = sorted(set(sum(comm.all_gather_object(sorted(torch.unique(y).tolist())), [])))
        assert len(classes) == 2, "cascade SVM is binary"
        g = base._gamma(X) if not isinstance(base.gamma, (int, float)) else float(base.gamma)
        if comm.is_distributed:
            g = float(comm.all_reduce(torch.tensor([g], dtype=torch.float64)) / comm.world)
        n = X.shape[0]
        S = max(1, min(self.shards, n))
        m = (n + S - 1) // S
        yb = torch.zeros((S, m), dtype=torch.float32, device=X.device)
        ys = torch.where(y == classes[1], 1.0, -1.0)
        if use_implicit(m, S, X.device):
            # every shard's rows as one padded [S, m, D] block: B problems of ONE implicit solve
            Xb = torch.zeros((S, m, X.shape[1]), dtype=torch.float32, device=X.device)
            for s in range(S):
                lo, hi = s * m, min(n, (s + 1) * m)
                Xb[s, : hi - lo] = X[lo:hi]
                yb[s, : hi - lo] = ys[lo:hi]
            Kb = ImplicitKernel(Xb, base.kernel, g, base.coef0, base.degree)
        else:
            Kb = torch.zeros((S, m, m), dtype=torch.float32, device=X.device)
            for s in range(S):
                lo, hi = s * m, min(n, (s + 1) * m)
                Kb[s, : hi - lo, : hi - lo] = kernel_matrix(X[lo:hi], X[lo:hi], base.kernel, g, base.degree,
                                                            base.coef0)
                yb[s, : hi - lo] = ys[lo:hi]
        alpha, _, _ = smo_batch(Kb, yb, base.C, base.eps, base.max_iter)
        keep = torch.cat([(alpha[s, : min(n, (s + 1) * m) - s * m] > 0) for s in range(S)])
        Xs, yv = X[keep], y[keep]
        if comm.is_distributed:
            dev = comm.device if comm.backend == "nccl" else torch.device("cpu")
            Xs = comm.all_gather_v(Xs.to(dev)).to(X.device)
            yv = comm.all_gather_v(yv.to(dev)).to(X.device)
        self.n_cascade_sv = int(Xs.shape[0])
        final = SVC(**{**self.kw, "gamma": g})
        self.model = final.fit(Xs, yv)
        return self

    def predict(self, X):
        return self.model.predict(X)

    def decision_function(self, X):
        return self.model.decision_function(X)


class OneClassSVM:
    """nu one-class SVM (Schölkopf et al.; P/app/ocsvm.py uses sklearn's OneClassSVM) on the same
    K12 SMO kernel: all labels +1, linear term 0, box [0, 1] with sum(alpha) = nu * n (LIBSVM's
    scaling), initial alphas = the first nu*n points and gradient G = K alpha."""

    def __init__(self, kernel: str = "rbf", nu: float = 0.1, gamma: float | str = "scale", degree: int = 3,
                 coef0: float = 0.0, eps: float = 1e-3, max_iter: int = 1_000_000):
        self.kernel, self.nu, self.gamma, self.degree, self.coef0 = kernel, nu, gamma, degree, coef0
        self.eps, self.max_iter = eps, max_iter

    def fit(self, X) -> "OneClassSVM":
        X = torch.as_tensor(X).float()
        n = X.shape[0]
        self.g = SVC(gamma=self.gamma)._gamma(X) if not isinstance(self.gamma, (int, float)) else float(self.gamma)
        K = kernel_matrix(X, X, self.kernel, self.g, self.degree, self.coef0)
        m = self.nu * n
        k = int(m)
        alpha = torch.zeros(n, dtype=torch.float32, device=X.device)
        alpha[:k] = 1.0
        if k < n:
            alpha[k] = m - k
        G = (K @ alpha).contiguous()
        y = torch.ones(n, dtype=torch.float32, device=X.device)
        if X.device.type == "cuda":
            a = alpha.view(1, -1).contiguous()
            g = G.view(1, -1).contiguous()
            Kc = K.unsqueeze(0).contiguous()
            diag = torch.diagonal(Kc, dim1=1, dim2=2).contiguous()
            _native.C().smo_solve(Kc, y.view(1, -1).contiguous(), diag, a, g, 1.0, float(self.eps), int(self.max_iter))
            alpha, G = a[0], g[0]
        else:
            alpha, G = _smo_from(K.double().numpy(), np.ones(n), alpha.double().numpy(), G.double().numpy(), 1.0,
                                 self.eps, self.max_iter)
            alpha, G = torch.from_numpy(alpha).float(), torch.from_numpy(G).float()
        self.rho = _rho(alpha.view(1, -1), G.view(1, -1), y.view(1, -1).cpu() if alpha.device.type == "cpu"
                        else y.view(1, -1), 1.0)[0]
        sv = alpha > 0
        self.sv_X, self.coef = X[sv], alpha[sv]
        return self

    def decision_function(self, X):
        X = torch.as_tensor(X).float().to(self.sv_X.device)
        Kx = kernel_matrix(self.sv_X, X, self.kernel, self.g, self.degree, self.coef0)
        return self.coef @ Kx - self.rho

    def predict(self, X):
        return torch.where(self.decision_function(X) >= 0, 1, -1)


def _smo_from(K, y, alpha, G, C, eps, max_iter):
    """Host SMO continuing from a given (alpha, G) — same selection / update as smo_reference."""
    N = y.size
    QD = np.diag(K).copy()
    for _ in range(max_iter):
        up = np.where(y > 0, alpha < C, alpha > 0)
        low = np.where(y > 0, alpha > 0, alpha < C)
        if not up.any():
            break
        v = np.where(up, -y * G, -np.inf)
        i = int(np.argmax(v))
        gmax = v[i]
        yg = np.where(low, y * G, -np.inf)
        gmax2 = yg.max()
        bd = gmax + yg
        a = np.where(QD[i] + QD - 2 * K[i] > 0, QD[i] + QD - 2 * K[i], 1e-12)
        gain = np.where(low & (bd > 0), bd * bd / a, -np.inf)
        j = int(np.argmax(gain))
        if gmax + gmax2 < eps or not np.isfinite(gain[j]):
            break
        oi, oj = alpha[i], alpha[j]
        quad = max(QD[i] + QD[j] - 2 * K[i, j], 1e-12)
        delta = (G[i] - G[j]) / quad          # y_i == y_j == 1
        s = oi + oj
        ai, aj = oi - delta, oj + delta
        if s > C:
            if ai > C:
                ai, aj = C, s - C
        elif aj < 0:
            aj, ai = 0.0, s
        if s > C:
            if aj > C:
                aj, ai = C, s - C
        elif ai < 0:
            ai, aj = 0.0, s
        alpha[i], alpha[j] = ai, aj
        G += K[i] * (ai - oi) + K[j] * (aj - oj)
    return alpha, G
