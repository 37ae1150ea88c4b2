"""K21 samplers (host Philox mirror + device kernel) and the batched Monte-Carlo simulator."""
import math

import numpy as np
import pytest
import torch

from avenir_amd.models.montecarlo import MonteCarloSimulator, geweke_z, raftery_lewis
from avenir_amd.ops import samplers as S

N = 200_000


@pytest.mark.parametrize("dist,params,mean,var", [
    (S.UNIFORM, [2.0, 6.0], 4.0, 16 / 12),
    (S.NORMAL, [1.5, 2.0], 1.5, 4.0),
    (S.EXPONENTIAL, [0.5], 2.0, 4.0),
    (S.LOGNORMAL, [0.0, 0.5], math.exp(0.125), (math.exp(0.25) - 1) * math.exp(0.25)),
    (S.GAMMA, [2.5, 2.0], 5.0, 10.0),
    (S.POISSON, [4.0], 4.0, 4.0),
    (S.POISSON, [60.0], 60.0, 60.0),
    (S.PARETO, [5.0, 1.0], 1.25, 5 / (16 * 3)),
    (S.TRIANGULAR, [0.0, 1.0, 4.0], 5 / 3, (0 + 1 + 16 - 0 - 0 - 4) / 18),
    (S.BERNOULLI, [0.3], 0.3, 0.21),
    (S.UNIFORM_INT, [1, 6], 3.5, 35 / 12),
])
def test_distribution_moments_cpu(dist, params, mean, var):
    v = S.device_sample(dist, N, params, "cpu", seed=5).double()
    assert float(v.mean()) == pytest.approx(mean, rel=0.02, abs=0.01)
    assert float(v.var()) == pytest.approx(var, rel=0.05, abs=0.005)


def test_table_sampler_and_specs():
    s = S.create_sampler("0:10:0.1:0.3:0.6:nonparam:float")
    v = s.sample_n(N)
    # 3 bins of width 10 from 0: probabilities .1/.3/.6
    h = torch.histc(v, bins=3, min=0, max=30) / N
    assert torch.allclose(h, torch.tensor([0.1, 0.3, 0.6]), atol=0.01)
    d = S.create_sampler("1:3:1:20:30:50:discrete:int")
    x = d.sample_n(50_000)
    f = torch.bincount(x.long(), minlength=4)[1:].double() / 50_000
    assert torch.allclose(f, torch.tensor([0.2, 0.3, 0.5], dtype=torch.float64), atol=0.01)
    c = S.create_sampler("a:1:b:3:categorical:string")
    vals = c.sample_n(20_000)
    assert abs(vals.count("b") / 20_000 - 0.75) < 0.02
    u = S.create_sampler("red:green:blue:uniform:string")
    assert set(u.sample_n(300)) == {"red", "green", "blue"}
    i = S.create_sampler("3:9:uniform:int").sample_n(10_000)
    assert int(i.min()) == 3 and int(i.max()) == 9
    n = S.create_sampler("10:2:normal:int").sample_n(1000)
    assert torch.equal(n, torch.round(n))
    for spec in ("2:exponential:float", "0:1:lognormal:float", "2:3:gamma:float", "3:poisson:int",
                 "2:1:pareto:float", "0:1:3:triangular:float", "0.4:bernoulli:int"):
        assert S.create_sampler(spec).sample_n(10).numel() == 10


def test_composite_samplers():
    mv = S.MultiVarNormalSampler([1.0, -1.0], [[2.0, 0.8], [0.8, 1.0]])
    x = mv.sample_n(100_000).double()
    cov = torch.cov(x.T)
    assert torch.allclose(cov, torch.tensor([[2.0, 0.8], [0.8, 1.0]], dtype=torch.float64), atol=0.05)
    mix = S.DistrMixtureSampler([S.NormalSampler(-5, 1), S.NormalSampler(5, 1)], [1, 3])
    v = mix.sample_n(40_000)
    assert float((v > 0).float().mean()) == pytest.approx(0.75, abs=0.02)
    cl = S.ClusterSampler([[0, 0], [10, 10]], 0.5)
    assert cl.sample_n(100).shape == (100, 2)
    jp = S.JointNonParamRejectSampler([0, 0], [1, 1], [2, 2], [1, 0, 0, 1])
    j = jp.sample_n(1000)
    assert bool(((j[:, 0] == j[:, 1])).all())
    perm = S.PermutationSampler([1, 2, 3, 4]).sample_n(5)
    assert all(sorted(p) == [1, 2, 3, 4] for p in perm)
    tr = S.NormalSamplerWithTrendCycle(0, 0.001, trend=1.0, cycle=[0, 10])
    y = tr.sample_n(4)
    assert torch.allclose(y, torch.tensor([0.0, 11.0, 2.0, 13.0]), atol=0.05)
    sp = S.SpikeyDataSampler(0, 1, 0.05, 50).sample_n(20_000)
    assert 0.03 < float((sp > 20).float().mean()) < 0.07
    ms = S.MetropolitanSampler(lambda x: -0.5 * (x - 2) ** 2, 1.0, chains=256, burn_in=200)
    m = ms.sample_n(200)
    assert float(m.mean()) == pytest.approx(2.0, abs=0.1)
    assert 0.2 < ms.acceptance_rate < 0.95


def test_philox_stream_reproducible():
    a = S.device_sample(S.NORMAL, 1000, [0, 1], "cpu", seed=3, offset=17)
    b = S.device_sample(S.NORMAL, 1000, [0, 1], "cpu", seed=3, offset=17)
    c = S.device_sample(S.NORMAL, 1000, [0, 1], "cpu", seed=3, offset=18)
    assert torch.equal(a, b) and not torch.equal(a, c)


def test_monte_carlo_simulator():
    # project cost: sum of a triangular and a normal (pccb-style), vectorised callback
    mc = MonteCarloSimulator(50_000, lambda X: X[:, 0] + X[:, 1], seed=1)
    mc.registerTriangularSampler(0, 4, 1).registerNormalSampler(10, 1)
    out = mc.run()
    assert out.numel() == 50_000
    assert mc.getMean() == pytest.approx(5 / 3 + 10, abs=0.03)
    assert mc.getStdDev() == pytest.approx(math.sqrt(13 / 18 + 1), abs=0.03)
    assert mc.getMin() < mc.getMedian() < mc.getMax()
    assert mc.getPercentile(mc.getMedian()) == pytest.approx(50, abs=1)
    assert mc.getUpperTailStat(5) > mc.getLowerTailStat(5)
    # scalar reference-style callback (args list + simulator + iteration)
    mc2 = MonteCarloSimulator(500, lambda args: args[0] * 2, vectorized=False, seed=2)
    mc2.registerUniformSampler(0.0, 1.0)
    mc2.run()
    assert 0.8 < mc2.getMean() < 1.2


def test_mcmc_diagnostics():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(20_000, generator=g)
    assert abs(geweke_z(x)) < 3
    drift = x + torch.linspace(0, 5, 20_000)
    assert abs(geweke_z(drift)) > 5
    rl = raftery_lewis(x)
    assert rl["n_min"] > 0 and rl["dependence"] < 5


@pytest.mark.gpu
def test_device_samplers_match_host_stream(cuda):
    # transform-based distributions: the kernel draws the same Philox stream as the host mirror
    for dist, params in [(S.UNIFORM, [2.0, 6.0]), (S.NORMAL, [1.0, 2.0]), (S.EXPONENTIAL, [0.5]),
                         (S.PARETO, [3.0, 1.0]), (S.TRIANGULAR, [0, 1, 4]), (S.BERNOULLI, [0.3]),
                         (S.UNIFORM_INT, [1, 6])]:
        h = S.device_sample(dist, 100_000, params, "cpu", seed=9, offset=3)
        d = S.device_sample(dist, 100_000, params, cuda, seed=9, offset=3).cpu()
        close = torch.isclose(h, d, rtol=2e-3, atol=2e-3).float().mean()
        assert close > 0.999, (dist, float(close))
    tab = torch.cumsum(torch.tensor([0.1, 0.3, 0.6]), 0)
    h = S.device_sample(S.TABLE, 50_000, [0.0, 10.0], "cpu", seed=1, offset=2, table=tab)
    d = S.device_sample(S.TABLE, 50_000, [0.0, 10.0], cuda, seed=1, offset=2, table=tab).cpu()
    assert torch.isclose(h, d, atol=1e-3).float().mean() > 0.999
    # rejection samplers: moments
    for dist, params, mean, var in [(S.GAMMA, [2.5, 2.0], 5.0, 10.0), (S.GAMMA, [0.5, 1.0], 0.5, 0.5),
                                    (S.POISSON, [4.0], 4.0, 4.0), (S.POISSON, [80.0], 80.0, 80.0)]:
        v = S.device_sample(dist, 1_000_000, params, cuda, seed=4).double()
        assert float(v.mean()) == pytest.approx(mean, rel=0.01), dist
        assert float(v.var()) == pytest.approx(var, rel=0.03), dist


@pytest.mark.gpu
def test_monte_carlo_on_device(cuda):
    mc = MonteCarloSimulator(4_000_000, lambda X: X[:, 0] * X[:, 1], device=cuda, seed=3)
    mc.registerUniformSampler(0.0, 2.0).registerGaussianSampler(3.0, 1.0)
    out = mc.run()
    assert out.device.type == "cuda"
    assert mc.getMean() == pytest.approx(3.0, rel=0.005)
