"""The island GA as one K22 launch (csrc/kernels/optim.hip::ga_assign_kernel):
bit-equal to its numpy twin (optimize/ga.py) for 1 and 256 islands, both replacement policies,
with conflicts and mutation; chunked launches (migration intervals) continue the Philox streams."""
import numpy as np
import pytest
import torch


def _domain(L=24, V=9, seed=3, device="cpu"):
    from avenir_amd.optimize.domain import AssignmentDomain
    g = torch.Generator().manual_seed(seed)
    cost = torch.rand((L, V), generator=g) * 100
    conf = torch.rand((L, L), generator=g) < 0.1
    return AssignmentDomain(cost.to(device), (conf | conf.T).to(device), invalid_cost=150.0)


def test_twin_chunks_equal_one_run():
    from avenir_amd.optimize.ga import ga_assign_reference, ga_init_population, ga_price
    d = _domain()
    cost, conf = d.cost_table.numpy(), d.conflict.numpy()
    pop = ga_init_population(5, 16, d.L, d.V, 7, 11, conf)
    pc = ga_price(cost, conf, 150.0, pop.astype(np.int64))
    one = ga_assign_reference(cost, conf, 150.0, pop, pc, 12, 6, 5, True, True, 7, 11)
    a = ga_assign_reference(cost, conf, 150.0, pop, pc, 5, 6, 5, True, True, 7, 11)
    b = ga_assign_reference(cost, conf, 150.0, a[0], a[1], 7, 6, 5, True, True, 7, 11, gen_base=5)
    assert np.array_equal(one[0], b[0]) and np.array_equal(one[1], b[1])
    assert np.array_equal(one[2], np.concatenate([a[2], b[2]], 1))
    assert (np.diff(one[2], axis=1) <= 0).all()                     # elitism: the best never gets worse


@pytest.mark.gpu
@pytest.mark.parametrize("islands", [1, 256])
@pytest.mark.parametrize("purge_first,mutate", [(True, True), (False, True), (True, False)])
def test_kernel_bit_equal_to_twin(cuda, islands, purge_first, mutate):
    from avenir_amd.optimize.ga import ga_assign_reference, ga_assign_run, ga_init_population, ga_price
    d = _domain()
    dg = _domain(device="cuda")
    P, m, r, G = 20, 8, 6, 30
    pop = ga_init_population(islands, P, d.L, d.V, 5, 100, d.conflict.numpy())
    pc = ga_price(d.cost_table.numpy(), d.conflict.numpy(), 150.0, pop.astype(np.int64))
    want = ga_assign_reference(d.cost_table.numpy(), d.conflict.numpy(), 150.0, pop, pc, G, m, r, purge_first, mutate,
                               5, 100, swap=d.swap_moves)
    got = ga_assign_run(dg, pop, pc, G, m, r, purge_first, mutate, 5, 100, torch.device("cuda"))
    for w, g_ in zip(want, got):
        assert w.dtype == g_.dtype and np.array_equal(w, g_)


@pytest.mark.gpu
def test_genetic_algorithm_gpu_equals_cpu(cuda):
    """The GeneticAlgorithm class takes the kernel on the GPU and the twin on the CPU: same result,
    migration included."""
    from avenir_amd.optimize.search import GeneticAlgorithm
    kw = dict(islands=8, pool=16, mating=6, replacement=6, generations=24, migrate_every=6, seed=9)
    rc = GeneticAlgorithm(_domain(), **kw).run()
    rg = GeneticAlgorithm(_domain(device="cuda"), **kw).run()
    assert rg.stats["engine"] == "ga_assign_kernel" and rc.stats["engine"] == "ga_twin"
    assert rg.best_cost == rc.best_cost and rg.history == rc.history
    assert torch.equal(rg.best.cpu(), rc.best.cpu())
