"""Collective layer (parallel/comm.py): the one-shot small-message all-reduce (all-gather + rank-ordered
local reduction) equals the library all-reduce, is bit-identical on every rank, and
the env switch routes small sum reductions through it (gloo ranks on the CPU; the RCCL path is
the same code with device tensors)."""
import pytest
import torch

from _dist import run_world


def _oneshot(rank, world):
    from avenir_amd.parallel.comm import get_comm
    comm = get_comm()
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(2048, generator=g, dtype=torch.float64)
    counts = torch.randint(0, 1000, (37, 5), generator=g)
    a, b = x.clone(), x.clone()
    comm.all_reduce(a)
    comm.all_reduce(b, algo="oneshot")
    c = counts.clone()
    comm.all_reduce(c, algo="oneshot")
    m = x.clone()
    comm.all_reduce(m, "max", algo="oneshot")
    ref_c = counts.clone()
    comm.all_reduce(ref_c)
    return a.tolist(), b.tolist(), torch.equal(c, ref_c), m.tolist()


@pytest.mark.parametrize("world", [2, 4])
def test_oneshot_all_reduce(world):
    res = run_world(_oneshot, world, timeout=300)
    for a, b, counts_equal, m in res:
        assert counts_equal
        assert max(abs(u - v) for u, v in zip(a, b)) < 1e-12
        assert b == res[0][1]                 # bit-identical on every rank (rank-ordered sum)
        assert m == res[0][3]


def _p2p_fallback(rank, world):
    from avenir_amd.parallel.comm import get_comm
    comm = get_comm()
    x = torch.arange(64, dtype=torch.float64) * (rank + 1)
    a, b = x.clone(), x.clone()
    comm.all_reduce(a)
    comm.all_reduce(b, algo="p2p")        # gloo / host tensors: the library collective
    return torch.equal(a, b)


def test_p2p_all_reduce_falls_back_off_rccl():
    assert all(run_world(_p2p_fallback, 2, timeout=300))
