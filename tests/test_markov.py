"""Markov / HMM / Viterbi / PST / CTMC / sequence-mining tests."""
import math

import numpy as np
import pytest
import torch

from avenir_amd.data import synth
from avenir_amd.models import markov as M
from avenir_amd.ops import sequence_ops as SO


def test_normalize_rows_reference_semantics():
    c = torch.tensor([[2, 0, 2], [1, 1, 2]])
    p = M.normalize_rows(c, 1000)
    assert p[0].tolist() == [3000 // 7, 1000 // 7, 3000 // 7]
    assert p[1].tolist() == [250, 250, 500]


def test_transition_model_and_classifier(tmp_path):
    st, lab, trans = synth.markov_sequences(4000, 5, 20, 2, seed=1)
    model = M.MarkovStateTransitionModel([str(i) for i in range(5)], ["a", "b"], scale=1).fit(st, lab)
    P = model.probabilities()
    assert torch.allclose(P.float(), trans.float(), atol=0.03)
    f = tmp_path / "mm.txt"
    M.MarkovStateTransitionModel([str(i) for i in range(5)], ["a", "b"], scale=1000).fit(st, lab).save(f)
    states, mats = M.MarkovStateTransitionModel.load_matrices(f)
    assert set(mats) == {"a", "b"} and len(states) == 5
    clf = M.MarkovModelClassifier(P[0], P[1], ["a", "b"])
    pred, lo = clf.predict(st)
    assert float((pred == lab.long()).float().mean()) > 0.9
    # oracle for one row
    r = 7
    exp = sum(math.log(float(P[0, st[r, j], st[r, j + 1]]) / float(P[1, st[r, j], st[r, j + 1]])) for j in range(19))
    assert float(lo[r]) == pytest.approx(exp, rel=1e-4)


def _np_viterbi(obs, A, B, pi):
    T = len(obs)
    S = A.shape[0]
    d = np.log(pi) + np.log(B[:, obs[0]])
    bp = np.zeros((T, S), dtype=int)
    for t in range(1, T):
        c = d[:, None] + np.log(A)
        bp[t] = c.argmax(0)
        d = c.max(0) + np.log(B[:, obs[t]])
    s = [int(d.argmax())]
    for t in range(T - 1, 0, -1):
        s.append(int(bp[t, s[-1]]))
    return s[::-1], float(d.max())


def test_hmm_builder_and_viterbi():
    rng = np.random.default_rng(0)
    S, O = 3, 4
    A = rng.dirichlet(np.ones(S), S)
    B = rng.dirichlet(np.ones(O), S)
    pi = rng.dirichlet(np.ones(S))
    tagged = []
    for _ in range(500):
        s = rng.choice(S, p=pi)
        seq = []
        for _ in range(12):
            o = rng.choice(O, p=B[s])
            seq.append(f"o{o}:s{s}")
            s = rng.choice(S, p=A[s])
        tagged.append(seq)
    b = M.HiddenMarkovModelBuilder([f"s{i}" for i in range(S)], [f"o{i}" for i in range(O)])
    obs, st = b.encode(tagged)
    hmm = b.fit(obs, st)
    assert torch.allclose(hmm.A.float(), torch.tensor(A, dtype=torch.float32), atol=0.06)
    lines = hmm.to_lines()
    hmm2 = M.HiddenMarkovModel.from_lines(lines)
    assert torch.allclose(hmm2.A, hmm.A, atol=1e-5)
    dec = M.ViterbiDecoder(hmm)
    obs2 = obs[:20].clone()
    obs2[3, 8:] = -1
    path, score = dec.decode(obs2)
    Ah, Bh, ph = hmm.A.numpy(), hmm.B.numpy(), hmm.pi.numpy()
    for r in (0, 3, 11):
        L = 8 if r == 3 else 12
        ref, sc = _np_viterbi(obs2[r, :L].numpy().astype(int), Ah, Bh, ph)
        assert path[r, :L].tolist() == ref
        assert float(score[r]) == pytest.approx(sc, rel=1e-4)
    ll = dec.log_likelihood(obs2)
    assert bool((ll >= score - 1e-4).all())


def test_pst_and_ngrams():
    st = torch.tensor([[0, 1, 2, 0, 1], [0, 1, 1, -1, -1]], dtype=torch.int16)
    c = SO.ngram_counts(st, 3, 2, 3)
    keys, cnt = c[2]
    got = {tuple(SO.decode_ngram(int(k), 2, 3)[1]): int(n) for k, n in zip(keys, cnt)}
    assert got == {(0, 1): 3, (1, 2): 1, (2, 0): 1, (1, 1): 1}
    pst = M.ProbabilisticSuffixTree(3, 3).fit(st)
    assert pst.find([0, 1]).count == 3
    p = pst.next_prob([0, 1])
    assert float(p.sum()) == pytest.approx(1.0)


def test_ctmc():
    Q = torch.tensor([[-0.5, 0.3, 0.2], [0.1, -0.4, 0.3], [0.2, 0.2, -0.4]], dtype=torch.float64)
    stats = M.ContTimeStateTransitionStats(Q)
    P = stats.future_state_prob(2.0)
    ref = torch.linalg.matrix_exp(Q * 2.0)
    assert torch.allclose(P, ref, atol=1e-8)
    dw = stats.state_dwell_time(2.0)
    assert torch.allclose(dw.sum(1), torch.full((3,), 2.0, dtype=torch.float64), atol=1e-6)
    ent = torch.tensor([0, 0, 0, 1, 1])
    tm = torch.tensor([0, 10, 30, 0, 5])
    s = torch.tensor([0, 1, 0, 1, 0])
    Qh = M.StateTransitionRate(2).fit(ent, tm, s)
    assert float(Qh[0, 1]) == pytest.approx(1 / 10) and float(Qh[1, 0]) == pytest.approx(2 / 25)


def test_sequence_mining():
    assert M.gsp_candidates([(1, 2), (2, 3), (2, 4)]) == [(1, 2, 3), (1, 2, 4)]
    A = torch.tensor([[1, 2, 3, 4], [4, 3, 2, 1]])
    sim = M.dot_matrix_similarity(A, A, 2)
    assert sim[0, 0] > sim[0, 1]
    ks, vals, starts = M.sequence_generator(torch.tensor([2, 1, 2, 1]), torch.tensor([5, 9, 1, 3]),
                                            torch.tensor([10, 20, 30, 40]))
    assert vals.tolist() == [40, 20, 30, 10] and starts.tolist() == [0, 2]
    m = M.positional_event_clusters(torch.tensor([0.0, 1, 2, 50]), torch.tensor([1, 1, 1, 1]), 1.5, 2)
    assert m.tolist() == [True, True, True, False]


@pytest.mark.gpu
def test_sequence_kernels_gpu(cuda):
    st, lab, trans = synth.markov_sequences(20000, 7, 30, 2, seed=3)
    st[::7, 20:] = -1
    P = M.MarkovStateTransitionModel([str(i) for i in range(7)], ["a", "b"], scale=1).fit(st, lab).probabilities()
    clf = M.MarkovModelClassifier(P[0], P[1], ["a", "b"])
    lc = clf.log_odds(st)
    lg = clf.log_odds(st.to(cuda)).cpu()
    assert torch.allclose(lc, lg, atol=1e-3)
    for S, O in ((5, 6), (70, 9)):
        rng = np.random.default_rng(S)
        A = torch.tensor(rng.dirichlet(np.ones(S), S))
        B = torch.tensor(rng.dirichlet(np.ones(O), S))
        pi = torch.tensor(rng.dirichlet(np.ones(S)))
        hmm = M.HiddenMarkovModel([str(i) for i in range(S)], [str(i) for i in range(O)], A, B, pi)
        obs = torch.tensor(rng.integers(0, O, (300, 25)), dtype=torch.int16)
        obs[5, 10:] = -1
        obs[6, 0] = -1                      # an invalid first observation: an empty path
        obs[7, 3] = O                       # an out-of-range observation ends the sequence
        dec = M.ViterbiDecoder(hmm)
        pc, sc = dec.decode(obs)
        pg, sg = M.ViterbiDecoder(hmm).decode(obs.to(cuda))
        assert torch.allclose(sc, sg.cpu(), rtol=1e-4, atol=1e-3)
        assert float((pc == pg.cpu()).float().mean()) > 0.999
        assert bool((pg[6] == -1).all()) and bool((pc[6] == -1).all())
        assert bool((pg[7, 3:] == -1).all()) and bool((pg[7, :3] >= 0).all())
        fc = dec.log_likelihood(obs)
        fg = dec.log_likelihood(obs.to(cuda)).cpu()
        assert torch.allclose(fc, fg, rtol=1e-4, atol=1e-3)


def test_ctmc_batched_sums_and_dot_matrix_oracle():
    Q = torch.tensor([[-0.5, 0.3, 0.2], [0.1, -0.4, 0.3], [0.2, 0.2, -0.4]], dtype=torch.float64)
    stats = M.ContTimeStateTransitionStats(Q)
    A, B = stats.sums([0.5, 2.0, 7.0])
    for b, t in enumerate([0.5, 2.0, 7.0]):
        assert torch.allclose(A[b], torch.linalg.matrix_exp(Q * t), atol=1e-8)
        assert torch.allclose(B[b].sum(1), torch.full((3,), t, dtype=torch.float64), atol=1e-6)
    ida = torch.tensor([[0, 1, 2, -1], [3, 3, 0, 1]], dtype=torch.int32)
    idb = torch.tensor([[1, 1, 9], [-1, -1, -1]], dtype=torch.int32)
    assert SO.dot_matrix_hits(ida, idb).tolist() == [[2, 0], [2, 0]]


@pytest.mark.gpu
def test_seqmine_kernels_gpu(cuda):
    # K5: n-gram hash counting (hot short n-grams collide in the LDS table; many distinct long ones)
    gen = torch.Generator().manual_seed(0)
    for S, N, L, lo, hi in ((4, 20000, 24, 2, 5), (40, 3000, 50, 1, 4)):
        st = torch.randint(0, S, (N, L), generator=gen, dtype=torch.int16)
        st[::5, L - 7:] = -1
        st[3::11, 4] = -1
        grp = torch.randint(0, 3, (N,), generator=gen, dtype=torch.int32)
        for g in (None, grp):
            ref = SO.ngram_counts(st, S, lo, hi, g)
            got = SO.ngram_counts(st.to(cuda), S, lo, hi, None if g is None else g.to(cuda))
            assert sorted(ref) == sorted(got)
            for k in ref:
                assert torch.equal(ref[k][0], got[k][0].cpu()) and torch.equal(ref[k][1], got[k][1].cpu())
    # K16: uniformisation power chain against matrix_exp / the CPU chain
    rng = np.random.default_rng(1)
    for S in (3, 17, 64):
        R = torch.tensor(rng.uniform(0.05, 1.0, (S, S)))
        R.fill_diagonal_(0)
        Q = R - torch.diag(R.sum(1))
        cpu = M.ContTimeStateTransitionStats(Q)
        gpu = M.ContTimeStateTransitionStats(Q.to(cuda))
        ts = [0.1, 1.0, 3.0]
        Ac, Bc = cpu.sums(ts)
        Ag, Bg = gpu.sums(ts)
        assert torch.allclose(Ac, Ag.cpu(), atol=1e-10) and torch.allclose(Bc, Bg.cpu(), atol=1e-9)
        assert torch.allclose(Ag[1].cpu(), torch.linalg.matrix_exp(Q), atol=1e-8)
    # K19: dot-matrix window matching, window ids longer than one LDS chunk
    for n, m, Wa, Wb in ((37, 50, 20, 33), (20, 18, 300, 270)):
        ida = torch.randint(-1, 40, (n, Wa), generator=gen, dtype=torch.int32)
        idb = torch.randint(-1, 40, (m, Wb), generator=gen, dtype=torch.int32)
        assert torch.equal(SO.dot_matrix_hits(ida, idb), SO.dot_matrix_hits(ida.to(cuda), idb.to(cuda)).cpu())
    A = torch.randint(0, 4, (64, 40), generator=gen)
    assert torch.allclose(M.dot_matrix_similarity(A, A[:9], 3), M.dot_matrix_similarity(A.to(cuda), A[:9].to(cuda), 3).cpu())
