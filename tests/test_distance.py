"""Distance / kNN / k-means / similarity tests (CPU oracles + gpu numerics)."""
import math

import numpy as np

import pytest
import torch

from avenir_amd.data import synth
from avenir_amd.models.cluster import KMeans, categorical_modes, dbscan, hopkins
from avenir_amd.models.knn import NearestNeighbor
from avenir_amd.models.similarity import NearestRecords, RecordSimilarity, top_matches_by_class
from avenir_amd.ops import distance as D

from _dist import run_world


def _brute(Q, R, k):
    d = torch.cdist(Q.double(), R.double())
    v, i = torch.topk(d, k, dim=1, largest=False)
    return v.float(), i


def test_knn_cpu_matches_bruteforce():
    g = torch.Generator().manual_seed(0)
    Q, R = torch.randn(50, 7, generator=g), torch.randn(300, 7, generator=g)
    d, i = D.knn(Q, R, 5)
    bd, bi = _brute(Q, R, 5)
    assert torch.allclose(d, bd, atol=1e-5) and torch.equal(i, bi)
    d2, i2 = D.knn(R[:40], R, 3, exclude_self=True)
    assert not bool((i2 == torch.arange(40).view(-1, 1)).any())


def test_knn_classifier_and_kernels():
    x, y = synth.supervised(1200, 5, 2, seed=1)
    nn_ = NearestNeighbor(k=7, kernel="gaussian", kernel_param=300.0).fit(x[:1000], y[:1000], 2)
    r = nn_.predict(x[1000:])
    assert float((r.pred == y[1000:]).float().mean()) > 0.85
    live = r.class_scores.sum(1) > 0
    assert bool(live.any())
    assert torch.allclose(r.class_prob[live].sum(1), torch.full((int(live.sum()),), 100.0), atol=1e-3)
    for kern in ("none", "linearMultiplicative", "linearAdditive"):
        r2 = NearestNeighbor(k=5, kernel=kern).fit(x[:1000], y[:1000], 2).predict(x[1000:])
        assert r2.pred.shape == (200,)
    reg = NearestNeighbor(k=5, regression="average").fit(x[:1000], y[:1000].float() * 10, 2).predict(x[1000:1010])
    assert reg.pred.shape == (10,)


def test_kmeans_recovers_blobs():
    g = torch.Generator().manual_seed(3)
    centers = torch.tensor([[0.0, 0.0], [10.0, 10.0], [-10.0, 8.0]])
    lab = torch.randint(0, 3, (3000,), generator=g)
    X = centers[lab] + 0.5 * torch.randn(3000, 2, generator=g)
    km = KMeans([2, 3, 4, 5], n_init=2, seed=1).fit(X)
    C = km.best[3].centroids
    for c in centers:
        assert float(((C - c) ** 2).sum(1).min()) < 0.1
    assert km.knuckle_k() == 3
    pred = km.predict(X, 3)
    # purity
    agree = 0
    for k in range(3):
        m = pred == k
        agree += int(torch.bincount(lab[m], minlength=3).max())
    assert agree / 3000 > 0.99


def _rank_kmeans(rank, world, X):
    from avenir_amd.parallel.comm import get_comm
    n = X.shape[0]
    s, e = rank * n // world, (rank + 1) * n // world
    km = KMeans(3, seed=5, comm=get_comm()).fit(X[s:e])
    return km.best[3].centroids, km.best[3].sse


def test_kmeans_world_size_equivalence():
    g = torch.Generator().manual_seed(4)
    X = torch.randn(2000, 3, generator=g) + torch.randint(0, 3, (2000, 1), generator=g) * 6.0
    ref = KMeans(3, seed=5).fit(X)
    res = run_world(_rank_kmeans, 2, X)
    for C, sse in res:
        assert sse == pytest.approx(ref.best[3].sse, rel=1e-4)


def test_distributed_knn_ring():
    g = torch.Generator().manual_seed(5)
    R = torch.randn(400, 4, generator=g)
    Q = torch.randn(30, 4, generator=g)
    res = run_world(_rank_knn, 2, Q, R)
    bd, bi = _brute(Q, R, 4)
    for d, i in res:
        assert torch.equal(i, bi) and torch.allclose(d, bd, atol=1e-5)


def _rank_knn(rank, world, Q, R):
    from avenir_amd.parallel.comm import get_comm
    n = R.shape[0]
    s, e = rank * n // world, (rank + 1) * n // world
    return D.distributed_knn(Q, R[s:e].contiguous(), 4, get_comm(), r_base=s)


def test_similarity_helpers():
    g = torch.Generator().manual_seed(6)
    X = torch.randn(100, 3, generator=g)
    y = torch.randint(0, 2, (100,), generator=g)
    d, i = top_matches_by_class(X, y, 3)
    ok = i >= 0
    assert bool((y[i[ok]] == y.view(-1, 1).expand_as(i)[ok]).all())
    d2, i2 = top_matches_by_class(X, y, 3, same_class=False)
    assert bool((y[i2[i2 >= 0]] != y.view(-1, 1).expand_as(i2)[i2 >= 0]).all())
    pairs = list(RecordSimilarity().all_pairs(X[:10]))
    assert sum(p[0].numel() for p in pairs) == 45
    nd, ni = NearestRecords(k=2, max_distance=0.5)(X)
    assert bool((nd[ni >= 0] <= 0.5).all())


def test_dbscan_and_hopkins():
    g = torch.Generator().manual_seed(7)
    X = torch.cat([torch.randn(100, 2, generator=g) * 0.2, torch.randn(100, 2, generator=g) * 0.2 + 5])
    lab = dbscan(X, eps=0.5, min_samples=4)
    assert int(lab.max()) == 1
    assert hopkins(X, 50) > 0.8


def test_categorical_modes():
    codes = torch.full((2, 16), 255, dtype=torch.uint8)
    codes[0, :6] = torch.tensor([0, 0, 1, 2, 2, 2], dtype=torch.uint8)
    codes[1, :6] = torch.tensor([1, 1, 0, 0, 0, 1], dtype=torch.uint8)
    m = categorical_modes(codes, 6, [3, 2], torch.tensor([0, 0, 0, 1, 1, 1]), 2)
    assert m.tolist() == [[0, 1], [2, 0]]


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,Dm,k", [(1000, 5000, 16, 5), (77, 3001, 3, 1), (513, 1000, 70, 32),
                                       (4096, 20000, 33, 8), (257, 2000, 200, 10), (100, 1500, 300, 5),
                                       (130, 999, 256, 64)])
def test_knn_mfma_gpu(cuda, M, N, Dm, k):
    g = torch.Generator().manual_seed(M)
    Q, R = torch.randn(M, Dm, generator=g), torch.randn(N, Dm, generator=g)
    d, i = D.knn(Q.to(cuda), R.to(cuda), k)
    bd, bi = _brute(Q, R, k)
    assert torch.allclose(d.cpu(), bd, atol=2e-3, rtol=1e-4)
    agree = float((i.cpu() == bi).float().mean())
    assert agree > 0.995
    d2, i2 = D.knn(R[:300].to(cuda), R.to(cuda), 4, exclude_self=True)
    assert not bool((i2.cpu() == torch.arange(300).view(-1, 1)).any())


@pytest.mark.gpu
@pytest.mark.parametrize("prec", [0, 3, 6])
@pytest.mark.parametrize("M,N,Dm,k", [(1000, 5000, 16, 5), (513, 1000, 70, 32), (257, 2000, 200, 10),
                                       (100, 1500, 300, 5)])
def test_knn_every_mode_gpu(cuda, M, N, Dm, k, prec):
    """The squared-euclidean dot products on fp32 MFMA (0) and on split-bf16 x3 / x6 (3 / 6)
    against the fp64 oracle at the same tolerances."""
    g = torch.Generator().manual_seed(M + prec)
    Q, R = torch.randn(M, Dm, generator=g), torch.randn(N, Dm, generator=g)
    d, i = D.knn(Q.to(cuda), R.to(cuda), k, prec=prec)
    bd, bi = _brute(Q, R, k)
    assert torch.allclose(d.cpu(), bd, atol=2e-3, rtol=1e-4)
    assert float((i.cpu() == bi).float().mean()) > 0.995
    d2, i2 = D.knn(R[:300].to(cuda), R.to(cuda), 4, exclude_self=True, prec=prec)
    assert not bool((i2.cpu() == torch.arange(300).view(-1, 1)).any())


@pytest.mark.gpu
@pytest.mark.parametrize("metric,p,k", [("manhattan", 1.0, 5), ("minkowski", 3.0, 7), ("euclidean", 2.0, 50),
                                        ("manhattan", 1.0, 64), ("minkowski", 1.5, 1), ("cosine", 2.0, 40)])
def test_knn_metrics_and_large_k_gpu(cuda, metric, p, k):
    """L1 / Lp on the VALU tile and k up to 64 in the fused kernel, against a float64 oracle."""
    g = torch.Generator().manual_seed(k)
    Q, R = torch.randn(700, 19, generator=g), torch.randn(4003, 19, generator=g)
    d, i = D.knn(Q.to(cuda), R.to(cuda), k, metric=metric, p=p)
    if metric == "cosine":
        ref = 1 - torch.nn.functional.normalize(Q.double(), dim=1) @ torch.nn.functional.normalize(R.double(), dim=1).T
    else:
        ref = torch.cdist(Q.double(), R.double(), p=p)
    bd, bi = torch.topk(ref, k, dim=1, largest=False)
    assert torch.allclose(d.cpu().double(), bd, atol=2e-3, rtol=1e-4)
    agree = float((i.cpu() == bi).float().mean())
    assert agree > 0.99
    d2, i2 = D.knn(R[:200].to(cuda), R.to(cuda), 3, metric=metric, p=p, exclude_self=True)
    assert not bool((i2.cpu() == torch.arange(200).view(-1, 1)).any())


@pytest.mark.gpu
def test_kmeans_gpu_matches_cpu(cuda):
    g = torch.Generator().manual_seed(8)
    X = torch.randn(20000, 6, generator=g) + torch.randint(0, 4, (20000, 1), generator=g) * 5.0
    kc = KMeans(4, seed=2, max_iter=50).fit(X)
    kg = KMeans(4, seed=2, max_iter=50).fit(X.to(cuda))
    assert kg.best[4].sse == pytest.approx(kc.best[4].sse, rel=1e-3)
    s, c = D.cluster_accumulate(X.to(cuda), torch.randint(0, 4, (20000,), generator=g).int().to(cuda), 4)
    assert int(c.sum()) == 20000


@pytest.mark.gpu
def test_kmeans_step_kernel_matches_oracle(cuda):
    from avenir_amd.models.cluster import KMeans, kmeans_step
    # (D, k): MFMA variant with 1, 2 and 4 centroid blocks, odd k (pair padding), D padding,
    # and a group large enough for the LDS fallback variant (k 300 at D 16: 32 centroid blocks)
    # (D, k) in {(4, 16), (8, 20), (16, 16), (32, 10)}: the MFMA-scoring kernel (kmeans_score_kernel)
    for D, k in ((2, 3), (16, 16), (5, 40), (33, 7), (16, 300), (4, 16), (8, 20), (32, 10)):
        g = torch.Generator().manual_seed(D + k)
        X = torch.randn((50_000, D), generator=g)
        C = torch.randn((k, D), generator=g)
        Dp = next(p for p in (2, 4, 8, 16, 32, 64) if p >= D)
        Xp = torch.zeros((X.shape[0], Dp))
        Xp[:, :D] = X
        sums, counts, sse, assign = kmeans_step(Xp.to(cuda), [C.to(cuda)], True)[0]
        d2 = torch.cdist(X.double(), C.double()) ** 2
        ref_a = d2.argmin(1)
        a = assign.cpu().long()
        # equal to the fp64 argmin except where the chosen centroid ties it within fp32 rounding of
        # the ||c||^2 - 2 x.c scores (no fixed disagreement allowance)
        gap = (d2.gather(1, a.view(-1, 1)) - d2.gather(1, ref_a.view(-1, 1))).view(-1)
        tol = 1e-5 * (1 + (X.double() ** 2).sum(1) + (C.double() ** 2).sum(1).max())
        assert bool(((a == ref_a) | (gap.abs() <= tol)).all())
        ref_sums = torch.zeros((k, D), dtype=torch.float64).index_add_(0, a, X.double())
        assert torch.allclose(sums.cpu()[:, :D], ref_sums, atol=1e-2, rtol=1e-4)
        assert torch.equal(counts.cpu().round().long(), torch.bincount(a, minlength=k))
        assert float(sse) == pytest.approx(float(d2.gather(1, a.view(-1, 1)).sum()), rel=1e-4)
    X = torch.randn((20_000, 3), generator=torch.Generator().manual_seed(1))
    cpu = KMeans([3, 4, 5], n_init=2, max_iter=10, seed=3).fit(X)
    gpu = KMeans([3, 4, 5], n_init=2, max_iter=10, seed=3).fit(X.to(cuda))     # 6 runs, one launch / iter
    for k in (3, 4, 5):
        assert gpu.best[k].sse == pytest.approx(cpu.best[k].sse, rel=1e-3)
        assert len(gpu.best[k].history) == gpu.best[k].iterations
    # multi-run launch equals single-run launches
    C1 = torch.randn((3, 4), generator=torch.Generator().manual_seed(5)).to(cuda)
    C2 = torch.randn((7, 4), generator=torch.Generator().manual_seed(6)).to(cuda)
    X4 = torch.randn((30_000, 4), generator=torch.Generator().manual_seed(7)).to(cuda)
    both = kmeans_step(X4, [C1, C2], True)
    one = kmeans_step(X4, [C1], True) + kmeans_step(X4, [C2], True)
    for (s_a, c_a, e_a, a_a), (s_b, c_b, e_b, a_b) in zip(both, one):
        assert torch.equal(a_a, a_b) and torch.equal(c_a, c_b)
        assert torch.allclose(s_a, s_b, rtol=1e-5, atol=1e-3)
        assert float(e_a) == pytest.approx(float(e_b), rel=1e-6)


def _grouped_oracle(X, groups):
    out = []
    for g in sorted(set(groups.tolist())):
        idx = [i for i in range(len(groups)) if int(groups[i]) == g]
        for a in range(len(idx)):
            for b in range(a + 1, len(idx)):
                out.append((idx[a], idx[b], float(torch.dist(X[idx[a]].double(), X[idx[b]].double()))))
    return out


@pytest.mark.parametrize("seed", [0, 1])
def test_grouped_similarity_batched_equals_per_group(seed):
    from avenir_amd.models.similarity import GroupedRecordSimilarity
    g = torch.Generator().manual_seed(seed)
    sizes = [1, 2, 3, 5, 8, 9, 17, 1, 33, 4]
    groups = torch.cat([torch.full((s,), 7 * k + 3) for k, s in enumerate(sizes)])
    perm = torch.randperm(groups.numel(), generator=g)
    groups = groups[perm]
    X = torch.randn(groups.numel(), 4, generator=g)
    i, j, d = GroupedRecordSimilarity().pairs(X, groups)
    ref = _grouped_oracle(X, groups)
    assert [(a, b) for a, b, _ in ref] == list(zip(i.tolist(), j.tolist()))
    assert torch.allclose(d.double(), torch.tensor([v for _, _, v in ref], dtype=torch.float64), atol=1e-5)


@pytest.mark.gpu
def test_grouped_similarity_gpu(cuda):
    from avenir_amd.models.similarity import GroupedRecordSimilarity
    g = torch.Generator().manual_seed(3)
    groups = torch.randint(0, 500, (6000,), generator=g)
    X = torch.randn(6000, 5, generator=g)
    ic, jc, dc = GroupedRecordSimilarity().pairs(X, groups)
    ig, jg, dg = GroupedRecordSimilarity().pairs(X.to(cuda), groups.to(cuda))
    assert torch.equal(ic, ig.cpu()) and torch.equal(jc, jg.cpu())
    assert torch.allclose(dc, dg.cpu(), atol=1e-4)


def test_kmeans_sklearn_tolerance_mode():
    """tol_mode='sklearn': converged when the summed squared centroid shift <= tol x the mean
    feature variance (scikit-learn's rule, P/unsupv/cluster.py); 'shift' keeps the Java
    per-centroid movement threshold.  The relative rule stops no later than the absolute one."""
    g = torch.Generator().manual_seed(3)
    X = torch.randn(4000, 3, generator=g) * 3 + torch.randint(0, 5, (4000, 1), generator=g) * 4.0
    a = KMeans(5, seed=1, tol=1e-4, tol_mode="shift").fit(X)
    b = KMeans(5, seed=1, tol=1e-4, tol_mode="sklearn").fit(X)
    assert b.best[5].iterations <= a.best[5].iterations
    assert b._tol_eff == pytest.approx(1e-4 * float(X.double().var(0, unbiased=False).mean()), rel=1e-9)
    assert b.best[5].sse == pytest.approx(a.best[5].sse, rel=1e-2)
    with pytest.raises(ValueError):
        KMeans(3, tol_mode="bogus")


@pytest.mark.gpu
@pytest.mark.parametrize("kern,C,ccw,thr", [("none", 2, False, -1.0), ("gaussian", 2, True, -1.0),
                                            ("linearMultiplicative", 5, False, -1.0),
                                            ("linearAdditive", 2, False, 1.5), ("gaussian", 37, True, -1.0)])
def test_knn_vote_kernel_matches_torch_vote(cuda, kern, C, ccw, thr):
    """K10 knn_vote_kernel (one launch) == the torch vote on the same neighbour lists, including
    class-conditional weights ([R] and [R, C] posteriors) and the decision-threshold rule."""
    g = torch.Generator().manual_seed(C)
    X = torch.randn(3000, 8, generator=g)
    y = torch.randint(0, C, (3000,), generator=g)
    post = torch.rand(3000, C, generator=g) if C > 2 else torch.rand(3000, generator=g)
    m = NearestNeighbor(k=9, kernel=kern, kernel_param=300.0, class_cond_weighted=ccw,
                        inverse_distance_weighted=(kern == "none"), decision_threshold=thr)
    m.fit(X.to(cuda), y.to(cuda), C, feature_post_prob=post.to(cuda) if ccw else None)
    got = m.predict(X[:500].to(cuda), exclude_self=True)
    # torch vote: same object with the kernel path disabled (an unknown-to-K10 kernel name forces it)
    import avenir_amd.models.knn as K
    saved = dict(K._VOTE_KERNELS)
    K._VOTE_KERNELS.clear()
    try:
        ref = m.predict(X[:500].to(cuda), exclude_self=True)
    finally:
        K._VOTE_KERNELS.update(saved)
    assert torch.equal(got.neighbors, ref.neighbors)
    assert torch.allclose(got.class_scores, ref.class_scores, rtol=1e-5, atol=1e-3)
    assert torch.allclose(got.class_prob, ref.class_prob, rtol=1e-5, atol=1e-3)
    close = (ref.class_scores.topk(2, 1).values.diff(dim=1).abs().squeeze(1) > 1e-3 * ref.class_scores.abs().max())
    assert torch.equal(got.pred.long()[close], ref.pred.long()[close])


def test_knn_class_cond_weight_per_class_posterior():
    """[R, C] posteriors weight each neighbour by ITS OWN class column (torch vote path)."""
    g = torch.Generator().manual_seed(5)
    C, k = 6, 4
    X = torch.randn(400, 5, generator=g)
    y = torch.randint(0, C, (400,), generator=g)
    post = torch.rand(400, C, generator=g)
    m = NearestNeighbor(k=k, class_cond_weighted=True).fit(X, y, C, feature_post_prob=post)
    r = m.predict(X[:50], exclude_self=True)
    exp = torch.zeros(50, C)
    for q in range(50):
        for j in range(k):
            i = int(r.neighbors[q, j])
            exp[q, y[i]] += post[i, y[i]]
    assert torch.allclose(r.class_scores, exp, atol=1e-5)


# ---------------------------------------------------------------------------------------------
# mixed-type distance without one-hot expansion (distance.hip mixed_knn_kernel)
# ---------------------------------------------------------------------------------------------
def _mixed_table(n, seed, device="cpu", card=300):
    from avenir_amd.data.table import from_arrays
    from avenir_amd.utils.schema import FeatureSchema
    rng = np.random.default_rng(seed)
    sj = {"fields": [
        {"name": "x", "ordinal": 0, "dataType": "double", "feature": True, "weight": 1.0},
        {"name": "z", "ordinal": 1, "dataType": "double", "feature": True, "weight": 0.5},
        {"name": "c", "ordinal": 2, "dataType": "categorical", "feature": True, "weight": 2.0,
         "cardinality": [f"v{i}" for i in range(card)]},
        {"name": "e", "ordinal": 3, "dataType": "categorical", "feature": True, "cardinality": ["a", "b", "c"]}]}
    cols = {0: rng.normal(size=n).round(3), 1: rng.uniform(0, 5, n).round(3),
            2: [f"v{v}" if v < card else "zz" for v in rng.integers(0, card + 5, n)],   # some unknown values
            3: [("a", "b", "c")[v] for v in rng.integers(0, 3, n)]}
    return from_arrays(FeatureSchema.from_json(sj), cols, device=device)


def test_split_mixed_equals_onehot_embedding_distances():
    from avenir_amd.ops.distance import encode_mixed, knn, knn_mixed, split_mixed
    tr, te = _mixed_table(500, 1), _mixed_table(80, 2)
    ranges = {0: (-4.0, 4.0), 1: (0.0, 5.0)}
    A, B = encode_mixed(tr, ranges=ranges), encode_mixed(te, ranges=ranges)
    An, Ac, wc = split_mixed(tr, ranges=ranges)
    Bn, Bc, _ = split_mixed(te, ranges=ranges)
    assert Ac.shape[1] == 2 and A.shape[1] > 300          # the one-hot width the kernel avoids
    d1, i1 = knn(B, A, 7, "euclidean")
    d2, i2 = knn_mixed(Bn, Bc, An, Ac, wc, 7)
    assert torch.allclose(d1, d2, atol=1e-5)


@pytest.mark.gpu
def test_mixed_knn_kernel_matches_cpu(cuda):
    from avenir_amd.ops.distance import knn_mixed, split_mixed
    tr, te = _mixed_table(3000, 3), _mixed_table(700, 4)
    ranges = {0: (-4.0, 4.0), 1: (0.0, 5.0)}
    An, Ac, wc = split_mixed(tr, ranges=ranges)
    Bn, Bc, _ = split_mixed(te, ranges=ranges)
    for k in (1, 5, 20):
        dc, ic = knn_mixed(Bn, Bc, An, Ac, wc, k)
        dg, ig = knn_mixed(Bn.to(cuda), Bc.to(cuda), An.to(cuda), Ac.to(cuda), wc.to(cuda), k, r_base=0)
        assert torch.allclose(dg.cpu(), dc, atol=1e-5)
        # neighbour sets agree wherever distances are not tied
        ok = (dc[:, 1:] - dc[:, :-1]).abs().min(1).values > 1e-4 if k > 1 else torch.ones(dc.shape[0], dtype=torch.bool)
        assert torch.equal(ig.cpu()[ok], ic[ok])


@pytest.mark.gpu
@pytest.mark.parametrize("D", [3, 8, 20, 64])
def test_pairs_within_kernel_vs_fp64(cuda, D):
    """distance.hip pairs_within_kernel: every pair with round(|a - b| / nf * scale) <= thr (and
    j > i in global order for a self-join), sorted by (i, j), against an fp64 brute force."""
    import math
    from avenir_amd import _native
    g = torch.Generator().manual_seed(D)
    A, B = torch.rand(700, D, generator=g), torch.rand(900, D, generator=g)
    nf, scale = math.sqrt(D), 1000.0
    ref = torch.round(torch.cdist(A.double(), B.double()) / nf * scale)
    thr = float(torch.quantile(ref.flatten(), 0.01))
    for tri, a_base, b_base in ((False, 0, 0), (True, 100, 50)):
        i, j, d = _native.C().pairs_within(A.to(cuda), B.to(cuda), nf, scale, thr, tri, a_base, b_base)
        i, j, d = i.cpu(), j.cpu(), d.cpu()
        keep = ref <= thr
        if tri:
            keep &= (torch.arange(900).view(1, -1) + b_base) > (torch.arange(700).view(-1, 1) + a_base)
        ri, rj = torch.nonzero(keep, as_tuple=True)
        got = set(zip(i.tolist(), j.tolist()))
        exp = set(zip(ri.tolist(), rj.tolist()))
        assert (i * 900 + j).diff().gt(0).all()                 # sorted by (i, j)
        assert len(got ^ exp) <= 0.002 * len(exp) + 2           # fp32 vs fp64 at the threshold edge
        for a, b, dd in zip(i.tolist()[:500], j.tolist()[:500], d.tolist()[:500]):
            assert abs(dd - ref[a, b]) <= 1
    # every pair kept: 4 M pairs overflow the first segment sizing -> the one re-run; all present, sorted
    A2, B2 = torch.rand(2000, D, generator=g), torch.rand(2000, D, generator=g)
    i, j, d = _native.C().pairs_within(A2.to(cuda), B2.to(cuda), nf, scale, 1e9, False, 0, 0)
    assert i.numel() == 2000 * 2000
    assert bool(((i * 2000 + j) == torch.arange(2000 * 2000, device=i.device)).all())
