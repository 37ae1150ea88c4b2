"""Tree-structured Parzen Estimator search over conditional spaces (hyperopt's ``tpe.suggest``),
and the multi-classifier hyper-parameter search of ``autosupv``.

Reference: ``python/app/autosupv.py:32-137`` builds an ``hp.choice`` (or ``hp.pchoice`` with
per-classifier probabilities) over classifiers, each branch a dict of ``hp.choice`` (string / int
range) and ``hp.uniform`` (float) parameters named from ``train.search.params``, and minimises
``clf.trainValidate()`` with ``fmin(algo=tpe.suggest)``.  hyperopt is not available here, so the
estimator is implemented directly (Bergstra et al., NIPS 2011), following hyperopt's defaults:
20 random start-up trials, good set = the ``ceil(gamma * sqrt(n))`` lowest losses (gamma 0.25,
at most 25 points), 24 candidates drawn from the good-set density l(x) per parameter, the one
maximising l(x) / g(x) kept; categorical densities are smoothed counts (prior weight 1), uniform
densities are truncated-gaussian Parzen mixtures with a prior component and neighbour-distance
bandwidths.  A parameter's observations come only from trials in which it was active (its
branch was chosen), which is what makes the estimator tree-structured.

Parity unpinned: hyperopt's RNG stream cannot be reproduced; tests check the optimiser
behaviour (convergence on known objectives, conditional activity) instead.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Callable, Sequence

import numpy as np


# ---- search-space nodes (hp.choice / hp.pchoice / hp.uniform / hp.randint-style ranges) ---------
@dataclass
class Choice:
    label: str
    options: list                       # values or nested spaces (dict / node)
    probs: list[float] | None = None    # hp.pchoice


@dataclass
class Uniform:
    label: str
    low: float
    high: float


def choice(label: str, options: Sequence) -> Choice:
    return Choice(label, list(options))


def pchoice(label: str, weighted: Sequence[tuple[float, Any]]) -> Choice:
    ps = [float(p) for p, _ in weighted]
    return Choice(label, [o for _, o in weighted], [p / sum(ps) for p in ps])


def uniform(label: str, low: float, high: float) -> Uniform:
    return Uniform(label, float(low), float(high))


def _labels(space, out: dict):
    if isinstance(space, (Choice, Uniform)):
        if space.label in out and out[space.label] is not space:
            raise ValueError(f"duplicate label {space.label}")
        out[space.label] = space
        if isinstance(space, Choice):
            for o in space.options:
                _labels(o, out)
    elif isinstance(space, dict):
        for v in space.values():
            _labels(v, out)
    elif isinstance(space, (list, tuple)):
        for v in space:
            _labels(v, out)
    return out


def _materialise(space, assign: dict):
    """Concrete value of ``space`` under the label -> (index | float) assignment."""
    if isinstance(space, Choice):
        return _materialise(space.options[assign[space.label]], assign)
    if isinstance(space, Uniform):
        return assign[space.label]
    if isinstance(space, dict):
        return {k: _materialise(v, assign) for k, v in space.items()}
    if isinstance(space, (list, tuple)):
        return type(space)(_materialise(v, assign) for v in space)
    return space


@dataclass
class Trial:
    assign: dict            # active label -> choice index / float value
    loss: float
    value: Any = None


@dataclass
class TPE:
    space: Any
    n_startup: int = 20
    gamma: float = 0.25
    n_candidates: int = 24
    prior_weight: float = 1.0
    seed: int = 0
    trials: list[Trial] = field(default_factory=list)

    def __post_init__(self):
        self.rng = np.random.default_rng(self.seed)
        self.nodes = _labels(self.space, {})

    # -- sampling ---------------------------------------------------------------------------------
    def _walk(self, space, pick: Callable, assign: dict):
        if isinstance(space, Choice):
            i = pick(space)
            assign[space.label] = i
            self._walk(space.options[i], pick, assign)
        elif isinstance(space, Uniform):
            assign[space.label] = pick(space)
        elif isinstance(space, dict):
            for v in space.values():
                self._walk(v, pick, assign)
        elif isinstance(space, (list, tuple)):
            for v in space:
                self._walk(v, pick, assign)

    def _random(self, node):
        if isinstance(node, Choice):
            return int(self.rng.choice(len(node.options), p=node.probs))
        return float(self.rng.uniform(node.low, node.high))

    def _split(self, label: str):
        obs = [(t.assign[label], t.loss) for t in self.trials if label in t.assign and math.isfinite(t.loss)]
        if not obs:
            return [], []
        order = sorted(range(len(obs)), key=lambda i: obs[i][1])
        n_good = max(1, min(int(math.ceil(self.gamma * math.sqrt(len(obs)))), 25))
        good = [obs[i][0] for i in order[:n_good]]
        bad = [obs[i][0] for i in order[n_good:]]
        return good, bad

    def _cat_density(self, node: Choice, xs):
        k = len(node.options)
        prior = np.asarray(node.probs if node.probs else [1.0 / k] * k)
        c = np.bincount(np.asarray(xs, dtype=np.int64), minlength=k).astype(np.float64) if xs else np.zeros(k)
        w = c + self.prior_weight * prior * k
        return w / w.sum()

    def _parzen(self, node: Uniform, xs):
        """Mixture (weights, mus, sigmas) of the observations plus a prior component, sigmas from
        the distances to the sorted neighbours, clipped to [range / min(100, n + 1), range]."""
        lo, hi = node.low, node.high
        rng_w = hi - lo
        mus = np.asarray(list(xs) + [0.5 * (lo + hi)], dtype=np.float64)
        order = np.argsort(mus)
        sm = mus[order]
        if sm.size > 1:
            left = np.diff(sm, prepend=lo)
            right = np.diff(sm, append=hi)
            sig_sorted = np.maximum(left, right)
        else:
            sig_sorted = np.asarray([rng_w])
        sig = np.empty_like(sig_sorted)
        sig[order] = sig_sorted
        sig[-1] = rng_w                                    # prior component
        sig = np.clip(sig, rng_w / min(100.0, mus.size + 1.0), rng_w)
        w = np.ones(mus.size)
        w[-1] = self.prior_weight
        return w / w.sum(), mus, sig

    @staticmethod
    def _trunc_logpdf(x, w, mus, sig, lo, hi):
        from scipy.stats import norm
        mass = norm.cdf(hi, mus, sig) - norm.cdf(lo, mus, sig)
        p = (w / np.maximum(mass, 1e-12))[None, :] * norm.pdf(np.asarray(x)[:, None], mus[None, :], sig[None, :])
        return np.log(np.maximum(p.sum(1), 1e-300))

    def _sample_parzen(self, w, mus, sig, lo, hi, n):
        out = []
        while len(out) < n:
            k = self.rng.choice(w.size, p=w)
            v = self.rng.normal(mus[k], sig[k])
            if lo <= v <= hi:
                out.append(v)
        return np.asarray(out)

    def _suggest_node(self, node):
        good, bad = self._split(node.label)
        if not good:
            return self._random(node)
        if isinstance(node, Choice):
            lg, lb = self._cat_density(node, good), self._cat_density(node, bad)
            cand = self.rng.choice(len(node.options), size=self.n_candidates, p=lg)
            score = np.log(lg[cand]) - np.log(lb[cand])
            return int(cand[int(np.argmax(score))])
        wl, ml, sl = self._parzen(node, good)
        wg, mg, sg = self._parzen(node, bad)
        cand = self._sample_parzen(wl, ml, sl, node.low, node.high, self.n_candidates)
        score = (self._trunc_logpdf(cand, wl, ml, sl, node.low, node.high)
                 - self._trunc_logpdf(cand, wg, mg, sg, node.low, node.high))
        return float(cand[int(np.argmax(score))])

    def suggest(self) -> dict:
        assign: dict = {}
        pick = self._random if len(self.trials) < self.n_startup else self._suggest_node
        self._walk(self.space, pick, assign)
        return assign

    # -- driver -----------------------------------------------------------------------------------
    def minimize(self, fn: Callable[[Any], float], max_evals: int, batch: int | None = None,
                 comm=None) -> tuple[Any, float]:
        """Sequential TPE (batch 1), or batches of ``batch`` proposals drawn from the same
        posterior and evaluated concurrently: with a distributed ``comm`` every rank draws the
        same batch (identical RNG and trial history), evaluates proposal ``rank`` on its own GPU
        and the losses are all-gathered, so all ranks keep one trial list (one trial
        per GPU).  ``batch`` defaults to the world size."""
        world = comm.world if comm is not None and comm.is_distributed else 1
        rank = comm.rank if world > 1 else 0
        batch = max(1, int(batch or world))
        done = 0
        while done < max_evals:
            nb = min(batch, max_evals - done)
            props = [self.suggest() for _ in range(nb)]
            vals = [_materialise(self.space, a) for a in props]
            if world > 1:
                mine = {i: float(fn(vals[i])) for i in range(rank, nb, world)}
                losses: dict = {}
                for part in comm.all_gather_object(mine):
                    losses.update(part)
            else:
                losses = {i: float(fn(v)) for i, v in enumerate(vals)}
            for i in range(nb):
                self.trials.append(Trial(props[i], losses[i], vals[i]))
            done += nb
        best = min(self.trials, key=lambda t: t.loss)
        return best.value, best.loss

    def best_assignment(self) -> dict:
        """hyperopt's ``fmin`` return form: label -> index (choices) or value (floats)."""
        return dict(min(self.trials, key=lambda t: t.loss).assign)


def fmin(fn: Callable[[Any], float], space, max_evals: int, seed: int = 0, batch: int | None = None,
         comm=None, **kw) -> tuple[dict, TPE]:
    t = TPE(space, seed=seed, **kw)
    t.minimize(fn, max_evals, batch=batch, comm=comm)
    return t.best_assignment(), t


# ---- autosupv: classifier + hyper-parameter search -------------------------------------------
def classifier_space(config, name: str) -> dict:
    """Space of one classifier from its config (autosupv.py:75-121): ``train.search.params`` =
    ``train.search.<a>.<b>:<type>,...``; the values of each come from that key itself — a list for
    ``string``, ``lo,hi`` (exclusive hi) for ``int``, ``lo,hi`` uniform for ``float``; the searched
    name drops the ``search`` component (``train.search.num.trees`` -> ``train.num.trees``)."""
    items = str(config.get_string("train.search.params")[0]).split(",")
    params = {}
    for it in items:
        ext, typ = it.split(":")[0], it.split(":")[1]
        parts = ext.split(".")
        pname = ".".join(parts[:1] + parts[2:])
        vals = str(config.configs[ext]).split(",")
        if ext == "train.search.data.feature.fields":
            vals = [v.replace(":", ",") for v in vals]
        if typ == "string":
            params[pname] = choice(f"{name}:{pname}", vals)
        elif typ == "int":
            if len(vals) != 2:
                raise ValueError("only 2 values needed for parameter range space")
            params[pname] = choice(f"{name}:{pname}", list(range(int(vals[0]), int(vals[1]))))
        elif typ == "float":
            if len(vals) != 2:
                raise ValueError("only 2 values needed for parameter uniform space")
            params[pname] = uniform(f"{name}:{pname}", float(vals[0]), float(vals[1]))
        else:
            raise ValueError("invalid paramter type")
    return {"model": name, "param": params}


def auto_supervised(classifiers: dict, max_evals: int, probs: Sequence[float] | None = None, seed: int = 0,
                    comm=None):
    """Pick the classifier and its hyper-parameters minimising ``trainValidate()`` by TPE
    (autosupv.py:124-137).  ``classifiers``: name -> BaseClassifier.  Returns (best assignment,
    best loss, the TPE object with every trial)."""
    branches = [classifier_space(c.config, n) for n, c in classifiers.items()]
    space = pchoice("classifier", list(zip(probs, branches))) if probs else choice("classifier", branches)

    def evaluate(args):
        clf = classifiers[args["model"]]
        for k, v in args["param"].items():
            clf.setConfigParam(k, str(v))
        return clf.trainValidate()

    best, t = fmin(evaluate, space, max_evals, seed=seed, comm=comm)
    return best, min(tr.loss for tr in t.trials), t
