"""TPE search (optimize/tpe.py, reference python/app/autosupv.py with hyperopt's tpe.suggest).
Parity unpinned (hyperopt is not installed and its RNG stream cannot be reproduced): the tests pin
optimiser behaviour on objectives with known optima and the conditional (tree) structure."""
import json

import numpy as np
import pytest

from avenir_amd.optimize import tpe


def test_tpe_beats_random_on_quadratic():
    space = {"x": tpe.uniform("x", -5.0, 5.0), "y": tpe.uniform("y", -5.0, 5.0)}
    f = lambda a: (a["x"] - 2.0) ** 2 + (a["y"] + 1.0) ** 2
    best, t = tpe.fmin(f, space, 100, seed=1)
    assert (best["x"] - 2.0) ** 2 + (best["y"] + 1.0) ** 2 < 0.3
    rng = np.random.default_rng(1)
    rand = [f({"x": rng.uniform(-5, 5), "y": rng.uniform(-5, 5)}) for _ in range(100)]
    late_tpe = np.median([tr.loss for tr in t.trials[60:]])
    assert late_tpe < np.median(rand[60:]) / 3


def test_conditional_space_and_choice():
    space = tpe.choice("branch", [
        {"kind": "a", "x": tpe.uniform("a:x", 0.0, 1.0)},
        {"kind": "b", "y": tpe.choice("b:y", [0, 1, 2, 3, 4])},
    ])

    def f(v):
        return 1.0 + v["x"] if v["kind"] == "a" else abs(v["y"] - 2) * 0.4

    best, t = tpe.fmin(f, space, 60, seed=3)
    assert best["branch"] == 1 and best["b:y"] == 2 and "a:x" not in best
    for tr in t.trials:      # a label is recorded only when its branch was taken
        assert ("a:x" in tr.assign) == (tr.assign["branch"] == 0)
        assert ("b:y" in tr.assign) == (tr.assign["branch"] == 1)
    # after the random start-up, TPE samples the better branch most of the time
    assert sum(tr.assign["branch"] == 1 for tr in t.trials[20:]) >= 30


def test_pchoice_prior():
    t = tpe.TPE(tpe.pchoice("c", [(0.9, "a"), (0.1, "b")]), seed=0)
    picks = [t.suggest()["c"] for _ in range(2000)]
    assert 0.86 < picks.count(0) / 2000 < 0.94


def _props(path, d):
    path.write_text("\n".join(f"{k}={v}" for k, v in d.items()) + "\n")


def test_autosupv_cli(tmp_path, capsys):
    from avenir_amd.cli import main
    rng = np.random.default_rng(0)
    X = rng.normal(size=(300, 4))
    y = ((X[:, 0] + 0.8 * X[:, 1]) > 0).astype(int)
    data = tmp_path / "train.csv"
    data.write_text("\n".join(f"id{i}," + ",".join(f"{v:.5f}" for v in X[i]) + f",{y[i]}" for i in range(300)) + "\n")
    common = {"train.data.file": data, "train.data.fields": "0,1,2,3,4,5", "train.data.feature.fields": "1,2,3,4",
              "train.data.class.field": 5, "train.num.folds": 3, "common.device": "cpu"}
    _props(tmp_path / "lr.properties", dict(common, **{
        "train.search.params": "train.search.reg.strength:float,train.search.penalty:string",
        "train.search.reg.strength": "0.01,2.0", "train.search.penalty": "l2,l1"}))
    _props(tmp_path / "rf.properties", dict(common, **{
        "train.num.trees": 5, "train.search.params": "train.search.max.depth:int",
        "train.search.max.depth": "2,5"}))
    assert main(["autoSupervisedLearning", "--gen-args",
                 f"8,lr:{tmp_path / 'lr.properties'}:0.7,rf:{tmp_path / 'rf.properties'}:0.3",
                 "--device", "cpu"]) == 0
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["evals"] == 8 and 0 <= out["loss"] < 0.3 and "classifier" in out["best"]


def _tpe_ranks(rank, world, max_evals):
    from avenir_amd.optimize.search import parameter_search
    from avenir_amd.optimize.tpe import choice, fmin, uniform
    from avenir_amd.parallel.comm import get_comm
    comm = get_comm()
    evaluated = []

    def loss(v):
        evaluated.append(v)
        return (v["x"] - 0.3) ** 2 + (0.0 if v["kind"] == "b" else 0.5)
    space = {"x": uniform("x", -2.0, 2.0), "kind": choice("kind", ["a", "b", "c"])}
    best, t = fmin(loss, space, max_evals, seed=7, comm=comm, n_startup=8)
    ps_evals = []

    def score(p):
        ps_evals.append(p)
        return abs(p["a"] - 3) + abs(p["b"] - 1)
    pbest, pscore, _ = parameter_search({"a": list(range(8)), "b": list(range(4))}, score, "random",
                                        n_iter=12, seed=3, comm=comm)
    return best, [tr.loss for tr in t.trials], len(evaluated), pbest, pscore, len(ps_evals)


@pytest.mark.parametrize("world", [2, 4])
def test_tpe_and_random_search_trial_parallel(world):
    """every rank evaluates its share of each TPE batch / of the random candidates;
    the result equals the single-process run with the same batch size, and no trial is evaluated
    twice across ranks."""
    from _dist import run_world
    from avenir_amd.optimize.tpe import choice, fmin, uniform
    res = run_world(_tpe_ranks, world, 24, timeout=300)
    space = {"x": uniform("x", -2.0, 2.0), "kind": choice("kind", ["a", "b", "c"])}
    ref_best, ref_t = fmin(lambda v: (v["x"] - 0.3) ** 2 + (0.0 if v["kind"] == "b" else 0.5), space, 24,
                           seed=7, batch=world, n_startup=8)
    for best, losses, _, pbest, pscore, _ in res:
        assert best == ref_best and losses == [tr.loss for tr in ref_t.trials]
        assert pbest == res[0][3] and pscore == res[0][4]
    assert sum(r[2] for r in res) == 24                    # each TPE proposal trained once
    assert sum(r[5] for r in res) <= 12                    # random candidates split, duplicates once
