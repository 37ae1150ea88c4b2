"""The remaining P/app drivers as CLI verbs (VERDICT r5 missing item 1): ``python -m avenir_amd
<verb> <args...>`` with the scripts' positional arguments, output on stdout (or ``-o``) in the
scripts' print formats.

* ``invSim <props> samp_size|burinin_size|gweke_conv|mean|percentile``  P/app/inv_sim.py:199-250
* ``tsstat <numIter> ks|and|cvm|zk|za|zc <nsamp>``                       P/app/tsstat.py:93-111
* ``fesel eo|sa <optConf> rf|gbt|svm|lr <clfConf>``                       P/app/fesel.py:78-95
* ``mesched <optConf> <numMeeting> <numPeople>``                          P/app/mesched.py:240-272
* ``pccb <numIter>``                                                      P/app/pccb.py:123-162
* ``ocsvm <trainSize> <nu> <kernel> <gamma>``                              P/app/ocsvm.py:24-63
* ``compLearn <featureCards> <classCard> terms|dnf|cnf [cSize] [dSize]``  P/app/comp_learn.py:82-109
* ``priceRl serve [--port P] [--train N]`` / ``priceRl client <url> ...`` (jobs/app_jobs.py) put
  the DQN pricing policy behind HTTP (P/app/price_rl_srv.py:35-60, price_rl_clnt.py:40-76):
  :class:`PolicyHTTPServer` below.

The work runs on the framework's device paths: the inventory chains advance together
(apps/inventory.py), the two-sample statistics of all ``numIter`` simulated pairs are computed in
ONE batch of sorted-label tensors (the reference runs one DataExplorer call per iteration), the
meeting schedules and feature subsets are populations of the batched optimisers
(optimize/search.py), the project-cost model prices every sampled scenario at once.
"""
from __future__ import annotations

import json
import math
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np
import torch

from .app_jobs import _Out, _dev, _props, _rest
from .common import job


# ---------------------------------------------------------------------------------------------
# invSim
# ---------------------------------------------------------------------------------------------
def _int_list(conf, key, step_key, num_key):
    """``a,b,c`` or start + step x count (inv_sim.py:176-197 get_sample_size_list / build_array)."""
    v = str(conf[key])
    if "," in v:
        return [int(x) for x in v.split(",")]
    s, st, n = int(v), int(conf[step_key]), int(conf[num_key])
    return [s + i * st for i in range(n)]


@job("invSim", "inventory MCMC app (P/app/inv_sim.py): invSim <props> samp_size | burinin_size | gweke_conv | "
     "mean | percentile")
def inv_sim(args):
    from ..apps.inventory import InventorySimulation
    rest = _rest(args, 2, "invSim <props> <op>")
    conf, op, out = _props(rest[0], rest[2:]), rest[1], _Out(args)
    sim = InventorySimulation.from_config(conf, device=_dev(args), seed=args.seed or 0)
    inv = int(str(conf["inv.size"]).split(",")[0])
    if op == "samp_size":
        out("sample size analysis")
        burn = int(conf["burn.in.sample.size"])
        for n in _int_list(conf, "sample.size", "sample.size.step", "num.sample.size"):
            r = sim.run([inv], n, burn)
            out(f"sample size {n} earning mean {r['mean'][0]:.2f}  earning mean std dev {r['stderr'][0]:.3f}")
    elif op == "burinin_size":
        out("burn sample size analysis")
        n = int(conf["sample.size"])
        prev = -1
        for b in _int_list(conf, "burn.in.sample.size", "burn.in.sample.size.step", "burn.in.num.sample.size"):
            if prev > 0:
                n += b - prev          # the reference grows the chain with the burn-in (inv_sim.py:112-114)
            r = sim.run([inv], n, b)
            out(f"sample size {n} earning mean {r['mean'][0]:.3f}  earning mean std dev {r['stderr'][0]:.3f}")
            prev = b
    elif op == "gweke_conv":
        out("running gweke convergence analysis")
        sizes = _int_list(conf, "sample.size", "sample.size.step", "num.sample.size")
        burns = _int_list(conf, "burn.in.sample.size", "burn.in.sample.size.step", "burn.in.num.sample.size")
        for s, b, z in sim.geweke(inv, sizes, burns):
            out(f"sample size {s}  burn in size {b}  z score {z:.3f}")
    elif op in ("mean", "percentile"):
        invs = _int_list(conf, "inv.size", "inv.step", "num.inv")
        n, burn = int(conf["sample.size"]), int(conf["burn.in.sample.size"])
        verbose = str(conf.get("output.verbose", "false")).lower() == "true"
        if op == "mean":
            out("mean earning for different inventory")
            r = sim.run(invs, n, burn)
            for i, v in enumerate(invs):
                if verbose:
                    out(f"inventory {v} average earning {r['mean'][i]:.2f} error {r['stderr'][i]:.3f} excess count "
                        f"{r['excess_count'][i]} deficit count {r['deficit_count'][i]}")
                else:
                    out(f"inventory {v} average earning {r['mean'][i]:.2f} ")
        else:
            out("percentile earning for different inventory")
            pct = float(conf.get("earning.precentile", conf.get("earning.percentile", 0.6)))
            for v, e in zip(invs, sim.percentile(invs, n, burn, pct)):
                out(f"inventory {v}  earning {e:.2f} ")
    else:
        raise ValueError(f"invalid op {op}")
    out.close()


# ---------------------------------------------------------------------------------------------
# tsstat: Monte-Carlo distribution of a two-sample statistic
# ---------------------------------------------------------------------------------------------
def two_sample_stats(a: torch.Tensor, b: torch.Tensor, kind: str) -> torch.Tensor:
    """Statistic of every row pair (a [B, n1], b [B, n2]) at once: ``ks`` (sup |F1 - F2|), ``cvm``
    (two-sample Cramér-von Mises T, scipy's definition), ``and`` (k = 2 Anderson-Darling A2 without
    ties, Scholz-Stephens), ``zk`` / ``za`` / ``zc`` (Zhang's likelihood-ratio EDF statistics, the
    definitions of DataExplorer._zhang).  One sort of the pooled rows; the rest are cumulative sums
    and reductions over the [B, N] sorted-label tensor."""
    B, n1 = a.shape
    n2 = b.shape[1]
    N = n1 + n2
    z = torch.cat([a, b], 1).double()
    lab = torch.cat([torch.ones_like(a, dtype=torch.bool), torch.zeros_like(b, dtype=torch.bool)], 1)
    order = z.argsort(1)
    lab = lab.gather(1, order)                                                # True = sample 1
    c1 = lab.double().cumsum(1)
    c2 = (~lab).double().cumsum(1)
    F1, F2 = c1 / n1, c2 / n2
    i = torch.arange(1, N + 1, dtype=torch.float64, device=z.device).view(1, -1)
    if kind == "ks":
        return (F1 - F2).abs().max(1).values
    if kind == "cvm":
        # ranks of each sample's members in the pooled order: U = n1 sum (r_i - i)^2 + n2 sum (s_j - j)^2
        r1 = torch.where(lab, i, torch.zeros_like(i))
        r2 = torch.where(~lab, i, torch.zeros_like(i))
        U = n1 * ((r1 - c1) ** 2 * lab).sum(1) + n2 * ((r2 - c2) ** 2 * ~lab).sum(1)
        return U / (n1 * n2 * N) - (4.0 * n1 * n2 - 1) / (6.0 * N)
    if kind == "and":
        j = i[:, :-1]
        M1 = c1[:, :-1]
        M2 = c2[:, :-1]
        s = ((N * M1 - j * n1) ** 2 / n1 + (N * M2 - j * n2) ** 2 / n2) / (j * (N - j))
        return s.sum(1) / N
    if kind in ("zk", "za", "zc"):
        F = i / N
        eps = 1e-12

        def lr(Fk, nk):
            return nk * (Fk * torch.log((Fk + eps) / (F + eps)) + (1 - Fk) * torch.log((1 - Fk + eps) / (1 - F + eps)))
        t = lr(F1, n1) + lr(F2, n2)
        if kind == "zk":
            return t.max(1).values
        if kind == "za":
            return (t / ((i - 0.5) * (N - i + 0.5))).sum(1)
        return (t / (i * (N - i + 1))).sum(1)
    raise ValueError("invalid 2 sample statistic")


def _nonparam_samples(w: torch.Tensor, n: int, g: torch.Generator) -> torch.Tensor:
    """``NonParamRejectSampler(0, 10, w).sampleAsFloat()`` for every row of weights w [B, 10]: a
    bin by weight, a uniform position inside it."""
    B = w.shape[0]
    k = torch.multinomial(w, n, replacement=True, generator=g).double()
    return (k + torch.rand((B, n), dtype=torch.float64, generator=g, device=w.device)) * 10.0


@job("tsstat", "two-sample statistic Monte-Carlo app (P/app/tsstat.py): tsstat <numIter> <ks|and|cvm|zk|za|zc> <nsamp>")
def tsstat(args):
    rest = _rest(args, 3, "tsstat <numIter> <stat> <nsamp>")
    n_iter, kind, nsamp = int(rest[0]), rest[1], int(rest[2])
    if kind not in ("ks", "and", "cvm", "zk", "za", "zc"):
        raise ValueError("invalid 2 sample statistic")
    out, dev = _Out(args), torch.device(_dev(args))
    g = torch.Generator(device=dev).manual_seed(args.seed or 0)
    # genStat (tsstat.py:39-87) for all iterations: 10 uniform(10, 100) weights, the second
    # distribution mutated (10 %: half extreme 100 - v, half unchanged; else 0..6 entries redrawn)
    w1 = 10.0 + 90.0 * torch.rand((n_iter, 10), dtype=torch.float64, generator=g, device=dev)
    w2 = w1.clone()
    u = torch.rand((n_iter, 2), dtype=torch.float64, generator=g, device=dev)
    rare, extreme = u[:, 0] < 0.10, u[:, 1] < 0.50
    nmut = torch.randint(0, 8, (n_iter,), generator=g, device=dev)
    pos = torch.rand((n_iter, 10), generator=g, device=dev).argsort(1).argsort(1)     # random ranks of positions
    redraw = (pos < nmut.view(-1, 1)) & ~rare.view(-1, 1)
    w2 = torch.where(redraw, 10.0 + 90.0 * torch.rand((n_iter, 10), dtype=torch.float64, generator=g, device=dev), w2)
    w2 = torch.where((rare & extreme).view(-1, 1), 100.0 - w1, w2)
    s1 = _nonparam_samples(w1, nsamp, g)
    s2 = _nonparam_samples(w2, nsamp, g)
    stat = two_sample_stats(s1, s2, kind).cpu()
    out(f"mean {float(stat.mean()):.3f}  sd {float(stat.std(unbiased=False)):.3f}  min {float(stat.min()):.3f}")
    # getUpperTailStat(0.5): (percentile, value) pairs of the upper half (mcsim.py)
    srt = stat.sort().values
    for p in range(50, 100, 5):
        out(f"{p:.3f}  {float(torch.quantile(srt, p / 100.0)):.3f}")
    out.close()


# ---------------------------------------------------------------------------------------------
# fesel: feature selection by an optimiser scored with a classifier
# ---------------------------------------------------------------------------------------------
_OPT_DEFAULTS = {
    "opti.solution.size": ("1", None), "opti.solution.data.distr": ("0:9:uniform:int", None),
    "opti.solution.data.groups": (None, None), "opti.pool.size": (10, None), "opti.pool.select.size": (3, None),
    "opti.mating.size": (5, None), "opti.replacement.size": (5, None), "opti.num.iter": (20, None),
    "opti.purge.cost.weight": (0.7, None), "opti.purge.age.scale": (1.0, None), "opti.purge.first": (True, None),
    "opti.temp": (10.0, None), "opti.temp.reduction.rate": (0.95, None), "opti.temp.adjust.num.iter": (2, None),
    "opti.local.search.num.iter": (20, None), "opti.performance.track.on": (False, None),
}


def _opt_config(path):
    from ..utils.config import Configuration
    return Configuration(str(path), dict(_OPT_DEFAULTS))


def _classifier(name: str, conf_path: str, device):
    from ..models import supervised as S
    kinds = {"rf": S.RandomForest, "gbt": S.GradientBoostedTrees, "svm": S.SupportVectorMachine,
             "lr": S.LogisticRegressionDiscriminant}
    if name not in kinds:
        raise ValueError("unsupported classifier")
    return kinds[name](conf_path, device=device)


class FeatureSelector:
    """The solution is an include mask over the candidate columns ``lo..hi`` of
    ``opti.solution.data.distr``; its cost is the classifier's ``trainValidate`` (k-fold) error
    with ``train.data.feature.fields`` set to the chosen columns (fesel.py:36-62).  Subsets already
    scored are memoised (the optimisers revisit them)."""

    def __init__(self, clf, columns: list[int]):
        self.clf, self.columns = clf, columns
        self.memo: dict[tuple, float] = {}

    def features(self, mask) -> list[int]:
        return [c for c, m in zip(self.columns, mask) if m]

    def score(self, mask) -> float:
        key = tuple(int(v) for v in mask)
        if key not in self.memo:
            cols = self.features(key)
            self.clf.setConfigParam("train.data.feature.fields", ",".join(map(str, cols)))
            self.memo[key] = float(self.clf.trainValidate())
        return self.memo[key]

    def __call__(self, sols: torch.Tensor) -> list[float]:
        return [self.score(r) for r in sols.cpu().tolist()]


@job("fesel", "feature selection app (P/app/fesel.py): fesel <eo|sa> <optConf> <rf|gbt|svm|lr> <clfConf>")
def fesel(args):
    from ..optimize.domains import FeatureSubsetDomain
    from ..optimize.search import EvolutionaryOptimizer, SimulatedAnnealing
    rest = _rest(args, 4, "fesel <eo|sa> <optConf> <clfName> <clfConf>")
    opt_name, conf = rest[0], _opt_config(rest[1])
    out, dev = _Out(args), _dev(args)
    lo, hi = (int(x) for x in conf.get_string("opti.solution.data.distr")[0].split(":")[:2])
    columns = list(range(lo, hi + 1))
    sizes = [int(x) for x in str(conf.get_string("opti.solution.size")[0]).split(",")]
    min_size, max_size = (sizes[0], sizes[-1]) if len(sizes) > 1 else (1, sizes[0])
    gs = conf.get_string("opti.solution.data.groups")[0]
    groups = None
    if gs and gs != "_":
        groups = [[columns.index(int(x)) for x in grp.split(":") if int(x) in columns] for grp in gs.split(",")]
        groups = [grp for grp in groups if len(grp) > 1] or None
    sel = FeatureSelector(_classifier(rest[2], rest[3], "cpu"), columns)
    dom = FeatureSubsetDomain(len(columns), min_size=min_size, max_size=min(max_size, len(columns)), groups=groups,
                              cost_fn=sel, device="cpu")
    seed = args.seed or 0
    if opt_name == "eo":
        res = EvolutionaryOptimizer(dom, islands=1, pool=conf.get_int("opti.pool.size")[0],
                                    select=conf.get_int("opti.pool.select.size")[0], iters=conf.get_int("opti.num.iter")[0],
                                    purge_cost_weight=conf.get_float("opti.purge.cost.weight")[0],
                                    purge_age_scale=conf.get_float("opti.purge.age.scale")[0], seed=seed).run()
    elif opt_name == "sa":
        res = SimulatedAnnealing(dom, n_chains=1, iters=conf.get_int("opti.num.iter")[0],
                                 t0=conf.get_float("opti.temp")[0], cooling=conf.get_float("opti.temp.reduction.rate")[0],
                                 interval=conf.get_int("opti.temp.adjust.num.iter")[0], seed=seed, use_kernel=False).run()
    else:
        raise ValueError("invalid optimizer name")
    best = res.best.view(-1).tolist()
    out("best soln found")
    out(f"features {','.join(map(str, sel.features(best)))}  cost {float(res.best_cost):.3f}")
    if conf.get_boolean("opti.performance.track.on")[0]:
        out("soln history")
        out(" ".join(f"{c:.3f}" for c in res.history))
    out(f"subsets evaluated {len(sel.memo)}")
    out.close()


# ---------------------------------------------------------------------------------------------
# mesched: meeting schedule by the genetic algorithm
# ---------------------------------------------------------------------------------------------
@job("mesched", "meeting schedule app (P/app/mesched.py): mesched <optConf> <numMeeting> <numPeople>")
def mesched(args):
    from ..optimize.domains import MeetingScheduleDomain
    from ..optimize.search import GeneticAlgorithm, local_focussed
    rest = _rest(args, 3, "mesched <optConf> <numMeeting> <numPeople>")
    conf = _opt_config(rest[0])
    n_meet, n_people = int(rest[1]), int(rest[2])
    out, dev, seed = _Out(args), _dev(args), args.seed or 0
    dom = MeetingScheduleDomain.random_instance(n_meet, n_people, seed=seed, device=dev)
    ga = GeneticAlgorithm.from_properties(dom, conf, islands=1, seed=seed)
    res = ga.run()
    out("optimizer started, check log file for output details...")

    def print_soln(sol, cost):
        out(f"cost {cost:.3f}")
        dec = dom.decode(sol.view(1, -1))[0].tolist()
        durs = (dom.dur / dom.SEC_MIN).tolist()
        for m in range(n_meet):
            out(f"meeting: day {int(dec[3 * m])} hour {int(dec[3 * m + 1])} min {int(dec[3 * m + 2])} "
                f"duration {int(durs[m])}")
    out("")
    out("best solution found")
    best, bc = res.best.view(1, -1), float(res.best_cost)
    print_soln(best, bc)
    if conf.get_boolean("opti.performance.track.on")[0]:
        out("")
        out("best solution history")
        out(" ".join(f"{c:.3f}" for c in res.history))
    lsol, lcost = local_focussed(dom, best, torch.tensor([bc], device=best.device),
                                 conf.get_int("opti.local.search.num.iter")[0],
                                 torch.Generator(device=best.device).manual_seed(seed + 1))
    lc = float(lcost.view(-1)[0])
    out("")
    out("best solution after local search of global best solution")
    print_soln(lsol.view(1, -1), lc)
    out("")
    out("locally search solution is best overall" if lc < bc else "local search failed to find a better solution")
    out.close()


# ---------------------------------------------------------------------------------------------
# pccb: project cost confidence bounds
# ---------------------------------------------------------------------------------------------
@job("pccb", "project cost Monte-Carlo app (P/app/pccb.py): pccb <numIter>")
def pccb(args):
    from ..apps.project_cost import project_cost_simulation
    rest = _rest(args, 1, "pccb <numIter>")
    out = _Out(args)
    sim = project_cost_simulation(int(rest[0]), device=_dev(args), seed=args.seed or 0)
    out(f"mean {sim.getMean():.2f}")
    out(f"std dev {sim.getStdDev():.2f}")
    out("upper critical values")
    srt = sim.output.sort().values
    n = srt.numel()
    for p in (0.90, 0.95, 0.99):       # getUpperTailStat(1.0): (value, percentile) pairs
        out(f"{float(torch.quantile(srt, p)):.3f}  {int(round(p * 100))}")
    out(f"iterations {n}")
    out.close()


# ---------------------------------------------------------------------------------------------
# ocsvm: one-class SVM outlier detection on the script's synthetic clusters
# ---------------------------------------------------------------------------------------------
@job("ocsvm", "one-class SVM app (P/app/ocsvm.py): ocsvm <trainSize> <nu> <kernel> <gamma>")
def ocsvm(args):
    from ..models.svm import OneClassSVM
    rest = _rest(args, 4, "ocsvm <trainSize> <nu> <kernel> <gamma>")
    n, nu, kernel, gamma = int(rest[0]), float(rest[1]), rest[2], float(rest[3])
    out, dev = _Out(args), torch.device(_dev(args))
    g = torch.Generator().manual_seed(args.seed or 0)
    X = 0.3 * torch.randn((n, 2), generator=g)
    X_train = torch.cat([X + 2, X - 2])
    X = 0.3 * torch.randn((20, 2), generator=g)
    X_test = torch.cat([X + 2, X - 2])
    X_out = torch.rand((20, 2), generator=g) * 8.0 - 4.0
    out("X_outliers")
    out(np.array2string(X_out.numpy(), precision=8))
    clf = OneClassSVM(kernel=kernel, nu=nu, gamma=gamma).fit(X_train.to(dev))
    p_train, p_test, p_out = (clf.predict(x.to(dev)).cpu() for x in (X_train, X_test, X_out))
    out("n_error_train")
    out(str(int((p_train == -1).sum())))
    out("n_error_test")
    out(str(int((p_test == -1).sum())))
    out("y_pred_outliers")
    out(np.array2string(p_out.numpy()))
    out("n_error_outliers")
    out(str(int((p_out == 1).sum())))
    out.close()


# ---------------------------------------------------------------------------------------------
# compLearn: PAC sample complexity
# ---------------------------------------------------------------------------------------------
@job("compLearn", "PAC sample complexity app (P/app/comp_learn.py): compLearn <featureCards> <classCard> "
     "<terms|dnf|cnf> [cSize] [dSize]")
def comp_learn(args):
    from ..utils import misc as M
    rest = _rest(args, 3, "compLearn <card,card,...> <classCard> <terms|dnf|cnf> [cSize] [dSize]")
    cards = [int(x) for x in rest[0].split(",")]
    ccard, space = int(rest[1]), rest[2]
    out = _Out(args)
    errors = [0.01, 0.02, 0.03, 0.04, 0.05]
    probs = [0.01, 0.02, 0.03, 0.04, 0.05]
    ln = None
    if space == "terms":
        out("all terms:")
        hyp = M.terms_hyp_space(cards, ccard)
    elif space == "dnf":
        out("k term dnf:")
        c_size, d_size = (int(rest[3]), int(rest[4])) if len(rest) >= 5 else (len(cards), int(rest[3]))
        hyp = M.disjunctive_hyp_space(cards, ccard, c_size, d_size)
    elif space == "cnf":
        out("k cnf:")
        ln = M.conjunctive_hyp_space_ln(cards, ccard, int(rest[3]))
    else:
        raise ValueError("invalid hypothesis space")
    for e in errors:
        for p in probs:
            m = M.pac_num_samples_ln(ln, e, p) if ln is not None else M.pac_num_samples(hyp, e, p)
            out(f"{e:.3f},{p:.3f},{m}")
    out.close()


# ---------------------------------------------------------------------------------------------
# the DQN pricing policy over HTTP (price_rl_srv.py / price_rl_clnt.py)
# ---------------------------------------------------------------------------------------------
class PolicyHTTPServer:
    """HTTP front of :class:`~avenir_amd.nn.rl.PolicyServer` — the RLlib ``PolicyServerInput`` of
    price_rl_srv.py reduced to its protocol: ``POST /start_episode`` -> ``{"episode_id"}``,
    ``POST /get_action {"episode_id", "observation"}`` -> ``{"action", "price"}`` (greedy, or
    epsilon-greedy while the episode trains), ``POST /log_returns {"episode_id", "reward"}``,
    ``POST /end_episode {"episode_id"}`` -> the episode's total reward, ``GET /stats``.  With
    ``train`` on, logged transitions go into the agent's replay buffer and every ``learn_every``
    returns trigger one DQN update (the server-side training of the reference)."""

    def __init__(self, agent, train: bool = False, learn_every: int = 8):
        from ..nn.rl import PolicyServer
        self.policy = PolicyServer(agent)
        self.agent, self.train, self.learn_every = agent, train, learn_every
        self.episodes: dict[int, dict] = {}
        self._next = 0
        self._lock = threading.Lock()
        self.httpd: ThreadingHTTPServer | None = None
        self.updates = 0

    # -- protocol ---------------------------------------------------------------------------
    def start_episode(self, training: bool = True) -> int:
        with self._lock:
            eid = self._next
            self._next += 1
            self.episodes[eid] = {"reward": 0.0, "steps": 0, "train": training and self.train, "last": None}
        return eid

    def get_action(self, eid: int, obs) -> dict:
        with self._lock:
            ep = self.episodes[eid]
            s = torch.as_tensor(obs, dtype=torch.float32, device=self.agent.device).view(1, -1)
            a = int(self.agent.act(s, greedy=not ep["train"])[0])
            ep["last"] = (obs, a)
        return {"action": a, "price": float(self.agent.env.grid[a])}

    def log_returns(self, eid: int, reward: float, next_obs=None) -> None:
        with self._lock:
            ep = self.episodes[eid]
            ep["reward"] += float(reward)
            ep["steps"] += 1
            self.policy.log_returns(reward)
            if ep["train"] and ep["last"] is not None and next_obs is not None:
                dev = self.agent.device
                s = torch.as_tensor(ep["last"][0], dtype=torch.float32, device=dev).view(1, -1)
                s2 = torch.as_tensor(next_obs, dtype=torch.float32, device=dev).view(1, -1)
                self.agent._store(s, torch.tensor([ep["last"][1]], device=dev), torch.tensor([float(reward)], device=dev),
                                  s2, False)
                if ep["steps"] % self.learn_every == 0:
                    self.agent.learn()
                    self.updates += 1

    def end_episode(self, eid: int) -> float:
        with self._lock:
            return self.episodes.pop(eid)["reward"]

    # -- HTTP -------------------------------------------------------------------------------
    def _handler(self):
        srv = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, obj):
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):
                if self.path.strip("/") == "stats":
                    return self._send(200, {"episodes_open": len(srv.episodes), "updates": srv.updates,
                                            "returns_logged": len(srv.policy.returns)})
                return self._send(404, {"error": "not found"})

            def do_POST(self):
                n = int(self.headers.get("Content-Length", 0) or 0)
                p = json.loads(self.rfile.read(n) or b"{}") if n else {}
                route = self.path.strip("/")
                try:
                    if route == "start_episode":
                        return self._send(200, {"episode_id": srv.start_episode(bool(p.get("training_enabled", True)))})
                    if route == "get_action":
                        return self._send(200, srv.get_action(int(p["episode_id"]), p["observation"]))
                    if route == "log_returns":
                        srv.log_returns(int(p["episode_id"]), float(p["reward"]), p.get("next_observation"))
                        return self._send(200, {"ok": True})
                    if route == "end_episode":
                        return self._send(200, {"total_reward": srv.end_episode(int(p["episode_id"]))})
                    return self._send(404, {"error": "not found"})
                except KeyError as e:
                    return self._send(400, {"error": f"missing or unknown {e}"})
                except Exception as e:  # noqa: BLE001
                    return self._send(500, {"error": str(e)})
        return H

    def start(self, port: int = 0, host: str = "127.0.0.1") -> int:
        self.httpd = ThreadingHTTPServer((host, port), self._handler())
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return self.httpd.server_address[1]

    def serve(self, port: int, host: str = "127.0.0.1"):
        self.httpd = ThreadingHTTPServer((host, port), self._handler())
        self.httpd.serve_forever()

    def shutdown(self):
        if self.httpd is not None:
            self.httpd.shutdown()
            self.httpd.server_close()


def _post(url: str, route: str, obj: dict) -> dict:
    import urllib.request
    req = urllib.request.Request(url.rstrip("/") + "/" + route, data=json.dumps(obj).encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=30) as r:
        return json.loads(r.read())


def policy_client(url: str, n_episodes: int, train: bool, off_policy: bool, stop_at_reward: float, out,
                  seed: int = 0, device="cpu") -> list[float]:
    """price_rl_clnt.py's loop: the client owns the pricing environment, asks the server for each
    action (or takes a random one and logs it), reports the rewards, prints each episode's total."""
    from ..nn.rl import PricingEnv
    env = PricingEnv(1, device=device, seed=seed)
    rng = np.random.default_rng(seed)
    totals = []
    for _ in range(n_episodes):
        eid = _post(url, "start_episode", {"training_enabled": train})["episode_id"]
        obs = env.reset()
        done, rewards = False, 0.0
        while not done:
            if off_policy:
                a = int(rng.integers(0, env.n_actions))
            else:
                a = int(_post(url, "get_action", {"episode_id": eid, "observation": obs.view(-1).tolist()})["action"])
            obs, r, done = env.step(torch.tensor([a], device=env.device))
            rewards += float(r.view(-1)[0])
            _post(url, "log_returns", {"episode_id": eid, "reward": float(r.view(-1)[0]),
                                       "next_observation": obs.view(-1).tolist()})
        _post(url, "end_episode", {"episode_id": eid})
        out(f"Total reward: {rewards:.3f}")
        totals.append(rewards)
        if rewards >= stop_at_reward:
            out("target reward achieved, exiting")
            break
    else:
        out("completed all episodes, exiting")
    return totals
