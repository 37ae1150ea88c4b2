"""Long-sequence Viterbi as a chunked max-plus scan: equal to the sequential
decoder on CPU (fp64), across 3 gloo ranks each holding one segment, and on the GPU (chunk +
back-track kernels vs the one-wave sequential kernel)."""
import pytest
import torch

from _dist import run_world
from avenir_amd.ops import sequence_ops as SO


def _hmm(S, O, seed):
    g = torch.Generator().manual_seed(seed)
    norm = lambda m: torch.log(m / m.sum(-1, keepdim=True))
    A = torch.rand(S, S, generator=g, dtype=torch.float64) + 0.05
    B = torch.rand(S, O, generator=g, dtype=torch.float64) + 0.05
    pi = torch.rand(S, generator=g, dtype=torch.float64) + 0.05
    return norm(A), norm(B), norm(pi)


def _obs(T, O, seed):
    g = torch.Generator().manual_seed(seed + 100)
    return torch.randint(0, O, (T,), generator=g).to(torch.int16)


def _logprob(path, obs, lA, lB, lp):
    p, o = path.long().cpu(), obs.long().cpu()
    lA, lB, lp = lA.double().cpu(), lB.double().cpu(), lp.double().cpu()
    return float(lp[p[0]] + lB[p, o].sum() + lA[p[:-1], p[1:]].sum())


@pytest.mark.parametrize("T,chunk", [(1500, 64), (40, 64), (512, 64), (777, 2)])
def test_chunked_equals_sequential_cpu(T, chunk):
    lA, lB, lp = _hmm(5, 6, T)
    obs = _obs(T, 6, T)
    ref_path, ref_score = SO.viterbi(obs.view(1, -1), lA, lB, lp)
    path, score = SO.viterbi_long(obs, lA, lB, lp, chunk=chunk)
    assert abs(score - float(ref_score[0])) <= 1e-5 * abs(score)
    assert torch.equal(path, ref_path[0])
    assert abs(_logprob(path, obs, lA, lB, lp) - score) <= 1e-9 * abs(score)


def test_end_marker_cpu():
    lA, lB, lp = _hmm(4, 3, 1)
    obs = torch.cat([_obs(300, 3, 1), torch.full((20,), -1, dtype=torch.int16)])
    path, _ = SO.viterbi_long(obs, lA, lB, lp, chunk=32)
    ref, _ = SO.viterbi(obs.view(1, -1), lA, lB, lp)
    assert torch.equal(path, ref[0]) and (path[300:] == -1).all()


_CUTS = [0, 500, 1130, 1800]


def _segment_worker(rank, world):
    lA, lB, lp = _hmm(6, 5, 9)
    obs = _obs(_CUTS[-1], 5, 9)
    return SO.viterbi_long(obs[_CUTS[rank]:_CUTS[rank + 1]], lA, lB, lp, chunk=64)


def test_sequence_parallel_three_ranks():
    res = run_world(_segment_worker, 3)
    lA, lB, lp = _hmm(6, 5, 9)
    obs = _obs(_CUTS[-1], 5, 9)
    ref, sc = SO.viterbi(obs.view(1, -1), lA, lB, lp)
    assert torch.equal(torch.cat([r[0] for r in res]), ref[0])
    assert all(abs(r[1] - float(sc[0])) <= 1e-5 * abs(r[1]) for r in res)


@pytest.mark.gpu
@pytest.mark.parametrize("S,chunk", [(4, 256), (16, 1024), (70, 512)])
def test_chunked_gpu_matches_sequential_kernel(S, chunk):
    T = 20000
    lA, lB, lp = _hmm(S, 8, S)
    obs = _obs(T, 8, S)
    dA, dB, dp = lA.float().cuda(), lB.float().cuda(), lp.float().cuda()
    ref_path, ref_score = SO.viterbi(obs.view(1, -1).cuda(), dA, dB, dp)
    path, score = SO.viterbi_long(obs.cuda(), dA, dB, dp, chunk=chunk)
    torch.cuda.synchronize()
    rs = float(ref_score[0])
    assert abs(score - rs) <= 1e-4 * abs(rs)
    # the returned path is optimal up to fp32 rounding and (near-)identical to the sequential one
    assert abs(_logprob(path, obs, lA, lB, lp) - rs) <= 1e-4 * abs(rs)
    agree = (path.cpu() == ref_path[0].cpu()).double().mean().item()
    assert agree > 0.98, agree
