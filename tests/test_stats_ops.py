"""K26 rank statistics (csrc/kernels/stats.hip, ops/stats_ops.py) against scipy.stats.

CPU: the host twins (ranks, tie terms, pair counts) and the statistic / p-value formulas match
scipy on tied and tie-free samples.  GPU: the kernels equal the twins exactly (integer pair counts,
half-integer rank sums) and the explorer methods equal scipy."""
import numpy as np
import pytest
import torch
from scipy import stats

from avenir_amd.ops import stats_ops as S


def _samples(n=700, seed=0, ties=True):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=n)
    y = 0.6 * x + rng.normal(size=n)
    if ties:
        x, y = np.round(x, 1), np.round(y, 1)
    return x, y


@pytest.mark.parametrize("ties", [True, False])
def test_rank_avg_matches_scipy(ties):
    x, _ = _samples(ties=ties)
    r, tie, _ = S.rank_avg(torch.tensor(x))
    assert np.allclose(r.numpy(), stats.rankdata(x))
    _, cnt = np.unique(x, return_counts=True)
    t = cnt.astype(float)
    assert np.allclose(tie.numpy(), [(t ** 3 - t).sum(), (t * (t - 1)).sum(), (t * (t - 1) * (t - 2)).sum(),
                                     (t * (t - 1) * (2 * t + 5)).sum()])


@pytest.mark.parametrize("ties", [True, False])
def test_rank_statistics_match_scipy(ties):
    x, y = _samples(ties=ties)
    rho, p = S.spearman(torch.tensor(x), torch.tensor(y))
    ref = stats.spearmanr(x, y)
    assert rho == pytest.approx(ref.statistic, rel=1e-12) and p == pytest.approx(ref.pvalue, rel=1e-6, abs=1e-300)
    tau, p = S.kendall_tau_b(torch.tensor(x), torch.tensor(y))
    ref = stats.kendalltau(x, y)
    assert tau == pytest.approx(ref.statistic, rel=1e-12) and p == pytest.approx(ref.pvalue, rel=1e-6, abs=1e-300)
    a, b = x[:300], y[300:] + 0.2
    u, p = S.mann_whitney_u(torch.tensor(a), torch.tensor(b))
    ref = stats.mannwhitneyu(a, b)
    assert u == pytest.approx(ref.statistic) and p == pytest.approx(ref.pvalue, rel=1e-6)
    h, p = S.kruskal_h(torch.tensor(a), torch.tensor(b), torch.tensor(x[100:250] - 0.1))
    ref = stats.kruskal(a, b, x[100:250] - 0.1)
    assert h == pytest.approx(ref.statistic, rel=1e-10) and p == pytest.approx(ref.pvalue, rel=1e-6)


def test_kendall_nan_propagates():
    x, y = _samples(50, seed=1)
    x[7] = np.nan
    tau, p = S.kendall_tau_b(torch.tensor(x), torch.tensor(y))
    ref = stats.kendalltau(x, y)
    assert np.isnan(tau) and np.isnan(p) and np.isnan(ref.statistic)


def test_small_samples_use_exact_paths():
    x = np.array([3.1, 1.2, 5.5, 4.0, 2.2, 9.1, 7.3])
    y = np.array([2.0, 1.0, 6.0, 3.0, 2.5, 8.0, 9.0])
    tau, p = S.kendall_tau_b(torch.tensor(x), torch.tensor(y))
    ref = stats.kendalltau(x, y)
    assert tau == pytest.approx(ref.statistic) and p == pytest.approx(ref.pvalue)
    u, p = S.mann_whitney_u(torch.tensor(x[:4]), torch.tensor(y[:5]))
    ref = stats.mannwhitneyu(x[:4], y[:5])
    assert u == pytest.approx(ref.statistic) and p == pytest.approx(ref.pvalue)


@pytest.mark.parametrize("n1,n2", [(5, 200), (200, 8), (9, 9)])
def test_mann_whitney_unbalanced_matches_scipy_method_choice(n1, n2):
    """scipy's method='auto' takes the exact null when either tie-free sample has <= 8 values."""
    rng = np.random.default_rng(n1 * 1000 + n2)
    a, b = rng.normal(size=n1), rng.normal(size=n2) + 0.1
    u, p = S.mann_whitney_u(torch.tensor(a), torch.tensor(b))
    ref = stats.mannwhitneyu(a, b)
    assert u == pytest.approx(ref.statistic) and p == pytest.approx(ref.pvalue, rel=1e-9)


def test_explorer_uses_rank_kernels():
    from avenir_amd.analytics.explorer import DataExplorer
    x, y = _samples(400, seed=3)
    ex = DataExplorer()
    ex.addListNumericData(x.tolist(), "x")
    ex.addListNumericData(y.tolist(), "y")
    r = ex.getKendalRankCorr("x", "y")
    assert r["stat"] == pytest.approx(stats.kendalltau(x, y).statistic, rel=1e-12)
    r = ex.testTwoSampleMw("x", "y")
    assert r["stat"] == pytest.approx(stats.mannwhitneyu(x, y).statistic)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 255, 256, 1000, 70_001])
def test_rank_kernels_match_twins(cuda, n):
    rng = np.random.default_rng(n)
    x = np.round(rng.normal(size=n), 2)
    y = np.round(0.3 * x + rng.normal(size=n), 2)
    grp = torch.tensor(rng.integers(0, 3, n), dtype=torch.int32)
    rc, tc, gc = S.rank_avg(torch.tensor(x), grp, 3)
    rg, tg, gg = S.rank_avg(torch.tensor(x, device=cuda), grp.to(cuda), 3)
    assert torch.equal(rg.cpu(), rc) and torch.allclose(tg.cpu(), tc, rtol=1e-12) and torch.equal(gg.cpu(), gc)
    if n <= 20_000:
        assert torch.equal(S.kendall_counts(torch.tensor(x, device=cuda), torch.tensor(y, device=cuda)).cpu(),
                           S.kendall_counts(torch.tensor(x), torch.tensor(y)))
    else:
        tau, p = S.kendall_tau_b(torch.tensor(x, device=cuda), torch.tensor(y, device=cuda))
        ref = stats.kendalltau(x, y)
        assert tau == pytest.approx(ref.statistic, rel=1e-12) and p == pytest.approx(ref.pvalue, rel=1e-6, abs=1e-300)


def _edf_checks(x, y, dev="cpu"):
    import warnings
    tx, ty = torch.tensor(x, device=dev), torch.tensor(y, device=dev)
    w, p = S.wilcoxon_signed_rank(tx, ty)
    ref = stats.wilcoxon(x, y)
    assert w == pytest.approx(ref.statistic) and p == pytest.approx(ref.pvalue, rel=1e-9, abs=1e-300)
    a, b = x, y[: len(y) // 2 + 3] + 0.1
    t, p = S.cvm_2samp(torch.tensor(a, device=dev), torch.tensor(b, device=dev))
    ref = stats.cramervonmises_2samp(a, b)
    assert t == pytest.approx(ref.statistic, rel=1e-10) and p == pytest.approx(ref.pvalue, rel=1e-8, abs=1e-300)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a2, crit, p = S.anderson_ksamp(torch.tensor(a, device=dev), torch.tensor(b, device=dev),
                                       torch.tensor(x[:90] - 0.05, device=dev))
        ref = stats.anderson_ksamp([a, b, x[:90] - 0.05])
    assert a2 == pytest.approx(ref.statistic, rel=1e-10) and np.allclose(crit, ref.critical_values)
    assert p == pytest.approx(ref.pvalue, rel=1e-9)


@pytest.mark.parametrize("ties", [True, False])
def test_edf_and_signed_rank_tests_match_scipy(ties):
    x, y = _samples(ties=ties)
    _edf_checks(x, y)
    # small samples: scipy's exact / permutation nulls on the host values
    w, p = S.wilcoxon_signed_rank(torch.tensor(x[:30]), torch.tensor(y[:30]))
    ref = stats.wilcoxon(x[:30], y[:30])
    assert w == pytest.approx(ref.statistic) and p == pytest.approx(ref.pvalue)


def test_explorer_two_sample_edf_tests():
    import warnings
    from avenir_amd.analytics.explorer import DataExplorer
    x, y = _samples(300, seed=5)
    ex = DataExplorer()
    ex.addListNumericData(x.tolist(), "x")
    ex.addListNumericData(y.tolist(), "y")
    assert ex.testTwoSampleWilcox("x", "y")["stat"] == pytest.approx(stats.wilcoxon(x, y).statistic)
    assert ex.testTwoSampleCvm("x", "y")["stat"] == pytest.approx(stats.cramervonmises_2samp(x, y).statistic)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        assert ex.testTwoSampleAnderson("x", "y")["stat"] == pytest.approx(stats.anderson_ksamp([x, y]).statistic)


@pytest.mark.gpu
def test_edf_and_signed_rank_tests_on_device(cuda):
    x, y = _samples(5000, seed=7)
    _edf_checks(x, y, cuda)


@pytest.mark.parametrize("ties", [True, False])
def test_kendall_merge_count_equals_pair_count(ties):
    x, y = _samples(3000, seed=9, ties=ties)
    a = S.kendall_counts(torch.tensor(x), torch.tensor(y), method="pairs")
    b = S.kendall_counts(torch.tensor(x), torch.tensor(y), method="merge")
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_kendall_merge_count_on_device(cuda):
    x, y = _samples(100_000, seed=10)
    g = S.kendall_counts(torch.tensor(x, device=cuda), torch.tensor(y, device=cuda), method="merge")
    c = S.kendall_counts(torch.tensor(x), torch.tensor(y), method="merge")
    assert torch.equal(g.cpu(), c)
    small = S.kendall_counts(torch.tensor(x[:20000], device=cuda), torch.tensor(y[:20000], device=cuda), method="pairs")
    assert torch.equal(small.cpu(), S.kendall_counts(torch.tensor(x[:20000]), torch.tensor(y[:20000]), method="merge"))
    # the merge-path kernels at sizes around the 1,024-value LDS block, against the all-pairs kernel
    for n in (2, 3, 1000, 1024, 1025, 2048, 5000):
        gx, gy = torch.tensor(x[:n], device=cuda), torch.tensor(y[:n], device=cuda)
        assert torch.equal(S.kendall_counts(gx, gy, method="merge").cpu(),
                           S.kendall_counts(gx, gy, method="pairs").cpu()), n
