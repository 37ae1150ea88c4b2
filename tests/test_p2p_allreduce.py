"""Hand-written peer-mapped all-reduce (csrc/kernels/comm.hip, parallel/p2p.py).

GPU tests: 2 and 4 processes share cuda:0 (the ``gloo:cuda`` harness of ``_dist.py``: gloo only
carries the one-time IPC handle exchange and barriers).  Each rank maps its peers' staging buffers
with hipIpcOpenMemHandle and runs 1,000 back-to-back all-reduces of CHANGING data with no host sync
in between; every result must be bit-equal to the rank-ordered host sum ((x0 + x1) + x2) + ...
(fp32 random values, so another summation order would differ), for 8 KB and 64 KB (one-shot) and
1 MB / odd-sized (two-shot) messages of float32 / float64 / int64.  The reference's counterpart
is the combiner + reducer shuffle of a count table
(src/main/java/org/avenir/bayesian/BayesianDistribution.java:72-79).
"""
import time

import pytest
import torch

from _dist import run_world

POOL = 8


def _pool(world, n, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    if dtype.is_floating_point:
        return torch.randn(POOL, world, n, generator=g, dtype=dtype)
    return torch.randint(-(1 << 40), 1 << 40, (POOL, world, n), generator=g, dtype=dtype)


def _scale(i, dtype):
    # float: powers of two keep the rank-ordered sum's bits exact under scaling; int: any factor
    return float(2.0 ** (i % 5 - 2)) if dtype.is_floating_point else (i % 7) - 3


def _ordered_sum(rows):
    acc = rows[0].clone()
    for k in range(1, rows.shape[0]):
        acc += rows[k]
    return acc


def _p2p_world(rank, world, cases, iters):
    from avenir_amd.parallel.comm import get_comm
    comm = get_comm()
    dev = comm.device
    out = {}
    for (n, dtype_name, algo) in cases:
        dtype = getattr(torch, dtype_name)
        pool = _pool(world, n, dtype, seed=1000 + n)
        mine = pool[:, rank].to(dev)                             # [POOL, n] this rank's operands
        res = torch.empty((iters, n), dtype=dtype, device=dev)
        x = torch.empty(n, dtype=dtype, device=dev)
        for i in range(iters):                                    # back to back: no host sync
            torch.mul(mine[i % POOL], _scale(i, dtype), out=x)
            comm.p2p().all_reduce(x, algo=algo)
            res[i].copy_(x)
        comm.p2p().check()
        got = res.cpu()
        bad = 0
        for j in range(POOL):
            ref = _ordered_sum(pool[j])
            for i in range(j, iters, POOL):
                if not torch.equal(got[i], ref * _scale(i, dtype)):
                    bad += 1
        out[(n, dtype_name, algo)] = (bad, got[-1].numpy().tobytes())
    # latency at 8 KB (one-shot) and 1 MB (two-shot), fp32, after the correctness runs
    lat = {}
    for nbytes in (8 << 10, 64 << 10, 1 << 20):
        x = torch.ones(nbytes // 4, device=dev)
        for _ in range(20):
            comm.p2p().all_reduce(x)
        torch.cuda.synchronize()
        comm.barrier()
        k = 200
        t0 = time.perf_counter()
        for _ in range(k):
            comm.p2p().all_reduce(x)
        torch.cuda.synchronize()
        lat[nbytes] = (time.perf_counter() - t0) / k * 1e6
    comm.p2p().check()
    return out, lat, dict(comm.p2p().calls)


CASES = [(2048, "float32", None), (16384, "float32", None), (1024, "int64", None), (8192, "int64", None),
         (262144, "float32", None), (12345, "float64", "twoshot"), (4097, "float32", "oneshot")]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_p2p_all_reduce_multiprocess_gpu(world):
    res = run_world(_p2p_world, world, CASES, 1000, timeout=600, comm="gloo:cuda")
    for rank, (out, lat, calls) in enumerate(res):
        for key, (bad, last) in out.items():
            assert bad == 0, f"rank {rank} case {key}: {bad} of 1000 results differ from the rank-ordered sum"
            assert last == res[0][0][key][1]                      # bit-identical on every rank
        assert calls["oneshot"] > 0 and calls["twoshot"] > 0
    lat0 = res[0][1]
    print(f"p2p all-reduce, {world} processes on one GPU: " +
          ", ".join(f"{b >> 10} KiB {us:.1f} us" for b, us in lat0.items()))


def _p2p_small_world(rank, world):
    """Comm.all_reduce(algo="p2p") routes device sums to the kernel and anything else (max, bool)
    to the library collective; results match the library all-reduce exactly for integers."""
    from avenir_amd.parallel.comm import get_comm
    comm = get_comm()
    dev = comm.device
    c = torch.arange(37 * 5, device=dev, dtype=torch.int64).view(37, 5) * (rank + 1)
    a = c.clone()
    comm.all_reduce(a, algo="p2p")
    m = torch.full((3,), float(rank), device=dev)
    comm.all_reduce(m, "max", algo="p2p")
    strided = torch.arange(64, device=dev, dtype=torch.float64).view(8, 8).t() * (rank + 1)
    s = strided.clone()
    comm.all_reduce(s, algo="p2p")                              # non-contiguous operand
    comm.p2p().check()
    tot = sum(range(1, world + 1))
    return (torch.equal(a.cpu(), torch.arange(37 * 5).view(37, 5) * tot),
            m.cpu().tolist() == [float(world - 1)] * 3,
            torch.equal(s.cpu(), torch.arange(64, dtype=torch.float64).view(8, 8).t() * tot))


@pytest.mark.gpu
def test_comm_routes_p2p_gpu():
    for ok in run_world(_p2p_small_world, 2, timeout=300, comm="gloo:cuda"):
        assert all(ok), ok


def _host_fallback(rank, world):
    from avenir_amd.parallel.comm import get_comm
    comm = get_comm()
    x = torch.arange(64, dtype=torch.float64) * (rank + 1)
    a, b = x.clone(), x.clone()
    comm.all_reduce(a)
    comm.all_reduce(b, algo="p2p")          # host tensors: the library collective
    return torch.equal(a, b) and comm._p2p is None


def test_p2p_host_tensors_fall_back():
    assert all(run_world(_host_fallback, 2, timeout=300))


def test_p2p_reference_sum_is_order_sensitive():
    """The oracle must be able to tell summation orders apart (else the GPU test proves nothing)."""
    pool = _pool(4, 16384, torch.float32, seed=1)
    fwd = _ordered_sum(pool[0])
    rev = _ordered_sum(pool[0].flip(0))
    assert not torch.equal(fwd, rev)


class _FakeHandle:
    """Stands in for the native P2PComm on CPU: rank 1 fails to map its peers."""
    released = False

    def __init__(self, dev, cap, uncached):
        self.cap_bytes = cap

    def set_timeout(self, s):
        pass

    def handles(self):
        return b"h"

    def open(self, handles, rank, world):
        if rank == 1:
            raise RuntimeError("ipc open (data): invalid argument")

    def close_peers(self):
        pass

    def release(self):
        _FakeHandle.released = True


def _p2p_open_fails_on_one_rank(rank, world):
    from avenir_amd import _native
    from avenir_amd.parallel import comm as C
    from avenir_amd.parallel.p2p import P2PAllReduce, P2PError

    class _Lib:
        P2PComm = _FakeHandle
    _native.C = lambda: _Lib
    c = C.get_comm()
    with pytest.raises(P2PError):
        P2PAllReduce(c, torch.device("cuda", 0))
    # the collective sequence is still aligned on every rank after the failure
    x = torch.tensor([float(rank + 1)])
    c.all_reduce(x)
    return float(x.item()), _FakeHandle.released


def test_p2p_construction_failure_on_one_rank_raises_everywhere():
    """A peer mapping that fails on ONE rank makes every rank raise (agreement all-reduce), frees
    every rank's region after a common barrier, and leaves the ranks' collectives in step."""
    out = run_world(_p2p_open_fails_on_one_rank, 2)
    assert out == [(3.0, True), (3.0, True)]


# ---- round 6: the peer-mapped path as the safe default ------------------------------------------

def _auto_choices(rank, world):
    """The agreed verdict of the selection probe, with this rank's measurements injected."""
    from avenir_amd.parallel import comm as C
    c = C.get_comm()
    like = torch.zeros(16, dtype=torch.int64)
    c.p2p = lambda: object()                        # stands in for a constructed P2PAllReduce
    out = []
    for exact, tp, tl in ((rank != 1, 1e-6, 2e-6),                       # rank 1 not exact
                          (True, 3e-6 if rank == 1 else 1e-6, 2e-6),      # slower on rank 1's clock
                          (True, 1e-6, 2e-6)):                            # exact and faster everywhere
        c._probe_p2p = lambda p, l, _r=(exact, tp, tl): _r
        c.small_allreduce = "auto"
        out.append(c._auto_small_allreduce(like))
        out.append(c.small_allreduce_probe["chosen"])
    return out


def test_auto_selection_is_agreed_over_ranks():
    """One rank that finds the kernel inexact (or slower) keeps EVERY rank on the library
    collective; the kernel is taken only when all ranks found it exact and faster."""
    for got in run_world(_auto_choices, 2):
        assert got == [None, "library", None, "library", "p2p", "p2p"]


class _FailingP2P:
    """A constructed peer-mapped state whose waits stop delivering after two good rounds: rank 1
    times out, rank 0 then sees the poisoned flag — both raise P2PError from inside the probe."""

    def __init__(self, comm):
        self.comm, self.timeout_s, self.timeouts, self.calls, self.closed = comm, 600.0, [], 0, False

    def set_timeout(self, s):
        self.timeout_s = s
        self.timeouts.append(s)

    def all_reduce(self, t, checked=True):
        from avenir_amd.parallel.p2p import P2PError
        self.calls += 1
        if self.calls > 2:
            raise P2PError(f"rank {self.comm.rank}: injected")
        return self.comm.all_reduce(t, algo="ring")

    def close(self):
        self.comm.barrier()
        self.closed = True


def _probe_fails(rank, world):
    from avenir_amd.parallel import comm as C
    c = C.get_comm()
    fake = _FailingP2P(c)
    c._p2p = fake
    c.small_allreduce = "auto"
    choice = c._auto_small_allreduce(torch.zeros(16, dtype=torch.int64))
    x = torch.full((8,), rank + 1, dtype=torch.int64)
    c.all_reduce(x)                                 # later small sums: the library collective
    return (choice, c.small_allreduce, c._p2p, fake.closed, fake.timeouts[0], c.small_allreduce_probe["chosen"],
            x.tolist())


def test_probe_failure_retires_the_kernel_on_every_rank():
    """A peer mapping that stops delivering fails the selection probe under its short wait bound
    (not the job's 600 s one); exactness is agreed before the timing rounds, so the ranks stay in
    step, close the kernel state together and take the library collective from then on."""
    from avenir_amd.parallel import comm as C
    for got in run_world(_probe_fails, 2):
        assert got == (None, None, False, True, C._PROBE_TIMEOUT_S, "library", [3] * 8)


def _p2p_unavailable(rank, world):
    from avenir_amd import _native
    from avenir_amd.parallel import comm as C

    class _Lib:
        P2PComm = _FakeHandle
    _native.C = lambda: _Lib
    c = C.get_comm()
    c.device = torch.device("cuda", 0)              # as on a GPU node; nothing is launched
    c.small_allreduce = "p2p"
    first = c.p2p()                                 # agreed failure: None on every rank, no raise
    n0 = c.stats["calls"]
    second = c.p2p()                                # remembered: no second construction round
    x = torch.tensor([float(rank + 1)])
    c.all_reduce(x)                                 # the library collective
    return first is None, second is None, c._p2p is False, c.small_allreduce, c.stats["calls"] - n0, float(x)


def test_p2p_unavailable_degrades_to_library():
    """a node without peer mapping degrades to the library collective (once, on every
    rank together) instead of raising from every later all-reduce."""
    for got in run_world(_p2p_unavailable, 2):
        assert got == (True, True, True, None, 1, 3.0)


def _default_path(rank, world):
    """No algorithm named, no env: the first small device sum runs the probe; the kernel must win
    over the gloo-carried library path here, and every later small sum takes it (counted)."""
    from avenir_amd.parallel.comm import get_comm
    comm = get_comm()
    dev = comm.device
    assert comm.small_allreduce == "auto"
    res = []
    for i in range(50):
        x = torch.full((513,), rank + 1 + i, dtype=torch.int64, device=dev)
        comm.all_reduce(x)
        res.append(bool((x == world * (world + 1) // 2 + world * i).all().item()))
    comm.check()
    return all(res), comm.small_allreduce, comm.p2p_calls, comm.small_allreduce_probe


@pytest.mark.gpu
def test_default_small_allreduce_takes_p2p_gpu():
    for ok, chosen, calls, probe in run_world(_default_path, 2, timeout=300, comm="gloo:cuda"):
        assert ok and chosen == "p2p", probe
        assert calls >= 50, calls


def _run_rank_procs(args, world, env_extra, timeout=240):
    import os
    import subprocess
    import sys
    from _dist import free_port
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PYTHONPATH=root, **env_extra)
        procs.append(subprocess.Popen([sys.executable, "-m", "avenir_amd"] + args, env=env, cwd=root,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    out = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            o, e = p.communicate()
        out.append((p.returncode, o.decode(errors="replace"), e.decode(errors="replace")))
    return out


@pytest.mark.gpu
def test_p2p_timeout_fails_the_job_on_every_rank(tmp_path):
    """Fault injection: in a 2-rank bayesianDistribution job on one GPU, rank 1
    reaches the count all-reduce 6 s late, past the 2 s wait bound.  Rank 0's wait times out
    (status 1; it poisons the flag it raised for rank 1), rank 1's kernel then finds the poison
    (status 2): BOTH ranks exit non-zero with P2PError, and no model file is written."""
    from avenir_amd.data import synth
    data, schema = tmp_path / "churn.csv", tmp_path / "churn.json"
    synth.write_churn(data, 5001, seed=3, schema_path=schema)
    model = tmp_path / "nb_model.txt"
    res = _run_rank_procs(["bayesianDistribution", "-i", str(data), "-o", str(model), "--schema", str(schema),
                           "--device", "cuda"], 2,
                          {"AVENIR_COMM_BACKEND": "gloo", "AVMI_SMALL_ALLREDUCE": "p2p", "AVMI_P2P_TIMEOUT_S": "2",
                           "AVMI_FAULT_P2P_SLEEP_RANK": "1", "AVMI_FAULT_P2P_SLEEP_S": "6"})
    for rank, (rc, _o, err) in enumerate(res):
        assert rc != 0, f"rank {rank} exited 0:\n{err[-3000:]}"
        assert "P2PError" in err, f"rank {rank}:\n{err[-3000:]}"
    assert not model.exists()


@pytest.mark.gpu
def test_p2p_healthy_job_writes_the_single_rank_model(tmp_path):
    """The same job without the fault: the default selection, exit 0 on both ranks, and the model
    equal to the one-process job's."""
    from avenir_amd.cli import main
    from avenir_amd.data import synth
    data, schema = tmp_path / "churn.csv", tmp_path / "churn.json"
    synth.write_churn(data, 5001, seed=3, schema_path=schema)
    one, two = tmp_path / "nb1.txt", tmp_path / "nb2.txt"
    assert main(["bayesianDistribution", "-i", str(data), "-o", str(one), "--schema", str(schema), "--device", "cuda"]) == 0
    res = _run_rank_procs(["bayesianDistribution", "-i", str(data), "-o", str(two), "--schema", str(schema),
                           "--device", "cuda"], 2, {"AVENIR_COMM_BACKEND": "gloo"})
    for rank, (rc, _o, err) in enumerate(res):
        assert rc == 0, f"rank {rank}:\n{err[-3000:]}"
    assert two.read_text() == one.read_text()
