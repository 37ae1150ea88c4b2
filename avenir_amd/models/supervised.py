"""Estimator layer: array-based classifiers / regressors and the config-driven ``BaseClassifier``
workflow (train / trainValidate / trainValidateSearch / validate / predict / predictProb /
autoTrain).

Reference: ``BaseClassifier`` (P/supv/bacl.py:38-445) and its sklearn wrappers ``RandomForest``
(P/supv/rf.py:86-116), ``GradientBoostedTrees`` (P/supv/gbt.py:41-477), ``SupportVectorMachine``
(P/supv/svm.py:83-121), ``LogisticRegressionDiscriminant`` (P/supv/lrd.py:37-109) and
``BaseRegressor`` / ``LinearRegressor`` / ``ElasticNetRegressor`` (P/supv/regress.py:38-253);
``PredictiveModel`` / ``ProbabilisticPredictiveModel`` / ``EnsemblePredictiveModel``
(J/model/*.java: error counting, cost-based threshold fpCost/(fpCost+fnCost), weighted majority
vote with minimum odds ratio).

MI355X design: every estimator is one of the framework's device models (histogram RF / GBT on the
tree kernels, SMO SVM, K13 logistic regression, Gram-matrix regression); k-fold CV trains the k
fold models on device-resident data (no host copies); models persist as ``torch.save`` state
dicts of plain tensors / lists loaded with ``weights_only=True`` (no joblib pickles).
"""
from __future__ import annotations

import math
from pathlib import Path
from typing import Callable, Sequence

import numpy as np
import torch

from ..data.table import Table, from_arrays
from ..optimize.search import parameter_search
from ..utils.config import Configuration
from ..utils.logging import get_logger
from ..utils.metrics import perf_metric
from ..utils.schema import FeatureSchema
from . import linear as L
from . import svm as S
from . import tree as T


# ================================================================================================
# array adapters
# ================================================================================================
def array_schema(n_features: int, class_values: Sequence) -> FeatureSchema:
    fields = [{"name": f"f{i}", "ordinal": i, "dataType": "double", "feature": True} for i in range(n_features)]
    fields.append({"name": "class", "ordinal": n_features, "dataType": "categorical",
                   "cardinality": [str(c) for c in class_values]})
    return FeatureSchema.from_json({"fields": fields})


def array_table(X, y, schema: FeatureSchema, device="cpu") -> Table:
    X = np.asarray(torch.as_tensor(X).cpu(), dtype=np.float32)
    cols = {i: X[:, i] for i in range(X.shape[1])}
    if y is not None:
        cols[X.shape[1]] = [str(v) for v in np.asarray(torch.as_tensor(y).cpu()).tolist()]
    return from_arrays(schema, cols, device=device)


class _TreeClassifierBase:
    def __init__(self, device=None):
        self.device = torch.device(device) if device else torch.device("cuda" if torch.cuda.is_available() else "cpu")

    def _prep(self, X, y):
        ys = np.asarray(torch.as_tensor(y).cpu()).tolist()
        self.classes_ = sorted(set(ys))
        self.schema = array_schema(np.shape(X)[1], self.classes_)
        return array_table(X, ys, self.schema, self.device)

    def _table(self, X):
        return array_table(X, None, self.schema, self.device)

    def predict(self, X):
        idx = self.predict_proba(X).argmax(1).cpu()
        return torch.tensor(self.classes_)[idx] if not isinstance(self.classes_[0], str) else \
            [self.classes_[i] for i in idx.tolist()]

    def score(self, X, y) -> float:
        p = self.predict(X)
        yt = np.asarray(torch.as_tensor(y).cpu()) if not isinstance(y, list) else np.asarray(y)
        return float(np.mean(np.asarray(p if isinstance(p, list) else p.numpy()) == yt))


class RandomForestClassifier(_TreeClassifierBase):
    def __init__(self, n_estimators: int = 100, max_depth: int | None = None, criterion: str = "gini",
                 max_features="sqrt", min_samples_split: int = 2, bootstrap: bool = True, max_bins: int = 32,
                 random_state: int = 0, device=None, comm=None):
        super().__init__(device)
        self.n_estimators, self.max_depth, self.criterion = n_estimators, max_depth or 12, criterion
        self.max_features, self.min_samples_split, self.bootstrap = max_features, min_samples_split, bootstrap
        self.max_bins, self.random_state, self.comm = max_bins, random_state, comm

    def fit(self, X, y):
        t = self._prep(X, y)
        p = T.TreeParams(algorithm="entropy" if self.criterion == "entropy" else "giniIndex", binary=True,
                         stopping="maxDepth", max_depth=self.max_depth, min_population=self.min_samples_split,
                         sub_sampling="withReplace" if self.bootstrap else "none", attr_selection="randomAll",
                         seed=self.random_state, max_bins=self.max_bins)
        self.model = T.RandomForest(self.schema, self.n_estimators, p, self.max_features, comm=self.comm).fit(t)
        return self

    def predict_proba(self, X):
        return self.model.predict_proba(self._table(X))

    def state(self) -> dict:
        return {"kind": "rf", "classes": [str(c) for c in self.classes_], "numeric": not isinstance(self.classes_[0], str),
                "F": len(self.schema.feature_fields), "trees": [t.state() for t in self.model.trees]}

    @classmethod
    def from_state(cls, st, device=None):
        m = cls(device=device)
        m.classes_ = [type_cast(c, st["numeric"]) for c in st["classes"]]
        m.schema = array_schema(st["F"], m.classes_)
        rf = T.RandomForest(m.schema, len(st["trees"]))
        rf.trees = [T.DecisionTree.from_state(s, m.schema) for s in st["trees"]]
        m.model = rf
        return m


def type_cast(v: str, numeric: bool):
    if not numeric:
        return v
    f = float(v)
    return int(f) if f.is_integer() else f


class GradientBoostingClassifier(_TreeClassifierBase):
    def __init__(self, n_estimators: int = 100, learning_rate: float = 0.1, max_depth: int = 3,
                 subsample: float = 1.0, min_samples_leaf: int = 1, max_bins: int = 64, random_state: int = 0,
                 device=None, comm=None):
        super().__init__(device)
        self.p = T.GBTParams(n_estimators=n_estimators, learning_rate=learning_rate, max_depth=max_depth,
                             min_samples_leaf=min_samples_leaf, subsample=subsample, max_bins=max_bins,
                             seed=random_state)
        self.comm = comm

    def fit(self, X, y):
        t = self._prep(X, y)
        self.model = T.GradientBoostedTrees(self.schema, self.p, self.comm).fit(t)
        return self

    def predict_proba(self, X):
        return self.model.predict_proba(self._table(X))


class SupportVectorClassifier:
    def __init__(self, kernel="rbf", C=1.0, gamma="scale", degree=3, coef0=0.0, device=None):
        self.svc = S.SVC(kernel, C, gamma, degree, coef0)
        self.device = torch.device(device) if device else torch.device("cuda" if torch.cuda.is_available() else "cpu")

    def fit(self, X, y):
        Xs = torch.as_tensor(np.asarray(X, dtype=np.float32), device=self.device)
        self.svc.fit(Xs, torch.as_tensor(np.asarray(y), device=self.device))
        return self

    def decision_function(self, X):
        return self.svc.decision_function(torch.as_tensor(np.asarray(X, dtype=np.float32), device=self.device))

    def predict_proba(self, X):
        f = self.decision_function(X)
        if f.dim() == 1:
            p = torch.sigmoid(2 * f)
            return torch.stack([1 - p, p], 1)
        return torch.softmax(f, 1)

    def predict(self, X):
        return self.svc.predict(torch.as_tensor(np.asarray(X, dtype=np.float32), device=self.device)).cpu()

    def score(self, X, y):
        return float((self.predict(X).numpy() == np.asarray(y)).mean())


class LogisticRegressionClassifier:
    def __init__(self, C: float = 1.0, penalty: str = "l2", max_iter: int = 50, device=None):
        self.C, self.penalty, self.max_iter = C, penalty, max_iter
        self.device = torch.device(device) if device else torch.device("cuda" if torch.cuda.is_available() else "cpu")

    def fit(self, X, y):
        y = np.asarray(y)
        self.classes_ = sorted(set(y.tolist()))
        Xs = torch.as_tensor(np.asarray(X, dtype=np.float32), device=self.device)
        n = Xs.shape[0]
        l2 = 0.0 if self.penalty == "none" else 1.0 / (self.C * n)
        self.models = []
        targets = [self.classes_[1]] if len(self.classes_) == 2 else self.classes_
        for c in targets:
            yy = torch.as_tensor((y == c).astype(np.float32), device=self.device)
            self.models.append(L.LogisticRegression(max_iter=self.max_iter, l2=l2).fit(Xs, yy, pos_class=1))
        return self

    def predict_proba(self, X):
        Xs = torch.as_tensor(np.asarray(X, dtype=np.float32), device=self.device)
        if len(self.models) == 1:
            return self.models[0].predict_proba(Xs)
        s = torch.stack([m.decision_function(Xs) for m in self.models], 1)
        return torch.softmax(s, 1)

    def predict(self, X):
        return torch.tensor(self.classes_)[self.predict_proba(X).argmax(1).cpu()]

    def score(self, X, y):
        return float((self.predict(X).numpy() == np.asarray(y)).mean())


# ================================================================================================
# cross validation
# ================================================================================================
def kfold_indices(n: int, k: int, seed: int = 0, shuffle: bool = True):
    idx = np.random.default_rng(seed).permutation(n) if shuffle else np.arange(n)
    folds = np.array_split(idx, k)
    for i in range(k):
        test = folds[i]
        train = np.concatenate([folds[j] for j in range(k) if j != i])
        yield train, test


def cross_val_score(make: Callable, X, y, k: int = 5, scoring: str = "accuracy", seed: int = 0) -> list[float]:
    X, y = np.asarray(X), np.asarray(y)
    scores = []
    for tr, te in kfold_indices(len(y), k, seed):
        m = make().fit(X[tr], y[tr])
        pred = m.predict(X[te])
        pred = np.asarray(pred if isinstance(pred, list) else torch.as_tensor(pred).cpu().numpy())
        scores.append(float(perf_metric(scoring, y[te].tolist(), pred.tolist())))
    return scores


# ================================================================================================
# config-driven workflow (BaseClassifier)
# ================================================================================================
_COMMON_DEFAULTS = {
    "common.mode": ("training", None), "common.model.directory": ("model", None), "common.model.file": (None, None),
    "common.preprocessing": (None, None), "common.verbose": (False, None), "common.logging.file": (None, None),
    "common.logging.level": ("info", None), "common.device": (None, None),
    "train.data.file": (None, None), "train.data.fields": (None, None), "train.data.feature.fields": (None, None),
    "train.data.class.field": (None, None), "train.validation": ("kfold", None), "train.num.folds": (5, None),
    "train.success.criterion": ("error", None), "train.model.save": (False, None),
    "train.score.method": ("accuracy", None), "train.search.param.strategy": (None, None),
    "train.search.params": (None, None), "train.search.max.iterations": (10, None),
    "train.search.sa.temp": (10.0, None), "train.search.sa.temp.red.rate": (0.9, None),
    "predict.data.file": (None, None), "predict.data.fields": (None, None),
    "predict.data.feature.fields": (None, None), "predict.use.saved.model": (False, None),
    "validate.data.file": (None, None), "validate.data.fields": (None, None),
    "validate.data.feature.fields": (None, None), "validate.data.class.field": (None, None),
    "validate.use.saved.model": (False, None), "validate.score.method": ("accuracy", None),
    "train.auto.max.test.error": (0.1, None), "train.auto.max.error": (0.05, None),
    "train.auto.max.error.diff": (0.02, None),
}


class BaseClassifier:
    """Reference workflow over a properties config.  Subclasses implement ``build_model``."""

    extra_defaults: dict = {}

    def __init__(self, config, device=None):
        d = dict(_COMMON_DEFAULTS)
        d.update(self.extra_defaults)
        self.config = config if isinstance(config, Configuration) else Configuration(config, d)
        for k, v in d.items():
            self.config.defaults.setdefault(k, v)
            self.config.configs.setdefault(k, "_")
        self.device = device or self.config.get_string("common.device")[0]
        self.logger = get_logger("avenir.supv")
        self.model = None
        self.feat = self.cls = None

    # -- config helpers ------------------------------------------------------------------------
    def setConfigParam(self, name, value):
        self.config.set_param(name, value)

    def getMode(self):
        return self.config.get_string("common.mode")[0]

    def _ints(self, key):
        v = self.config.get_string(key)[0]
        return [int(x) for x in str(v).split(",")] if v else None

    def _load(self, prefix: str, with_class: bool = True):
        path = self.config.get_string(f"{prefix}.data.file")[0]
        fields = self._ints(f"{prefix}.data.fields")
        feats = self._ints(f"{prefix}.data.feature.fields")
        rows = [l.rstrip("\n").split(",") for l in Path(path).read_text().splitlines() if l.strip()]
        sel = [[r[i] for i in fields] for r in rows] if fields else rows
        X = np.array([[float(r[i]) for i in feats] for r in sel], dtype=np.float32)
        if self.config.get_string("common.preprocessing")[0] == "scale":
            X = (X - X.mean(0)) / np.where(X.std(0) > 0, X.std(0), 1)
        if not with_class:
            return X, None
        ci = self.config.get_int(f"{prefix}.data.class.field")[0]
        y = np.array([_num(r[ci]) for r in sel])
        return X, y

    def prepTrainingData(self):
        return self._load("train")

    def prepValidationData(self):
        return self._load("validate")

    def build_model(self):
        raise NotImplementedError

    def _model_path(self) -> Path:
        d = Path(self.config.get_string("common.model.directory")[0] or "model")
        f = self.config.get_string("common.model.file")[0] or "model.pt"
        return d / f

    # -- modes ---------------------------------------------------------------------------------
    def train(self):
        self.model = self.build_model()
        if self.feat is None:
            self.feat, self.cls = self.prepTrainingData()
        self.model.fit(self.feat, self.cls)
        score = self.model.score(self.feat, self.cls)
        crit = self.config.get_string("train.success.criterion")[0]
        res = score if crit == "accuracy" else 1.0 - score
        if self.config.get_boolean("train.model.save")[0]:
            self.save_model()
        return res

    def trainValidate(self):
        X, y = self.prepTrainingData()
        k = self.config.get_int("train.num.folds")[0]
        scoring = self.config.get_string("train.score.method")[0]
        scores = cross_val_score(self.build_model, X, y, k, scoring)
        av = float(np.mean(scores))
        crit = self.config.get_string("train.success.criterion")[0]
        return av if crit == "accuracy" else 1.0 - av

    def trainValidateSearch(self):
        """Search ``train.search.params`` = ``train.search.<name>:<type>,...``; each searched key's
        values come from the config key itself (bacl.py:134-207); the reference name form
        ``train.search.x.y`` maps onto ``train.x.y``."""
        strategy = self.config.get_string("train.search.param.strategy")[0]
        items = self.config.get_string("train.search.params")[0].split(",")
        space = {}
        for it in items:
            ext = it.split(":")[0]
            parts = ext.split(".")
            name = ".".join(parts[:1] + parts[2:])
            space[name] = [v for v in self.config.configs[ext].split(",")]
        strat = {"grid": "guided", "random": "random", "simuan": "sa"}[strategy]

        def score(params):
            for k2, v in params.items():
                self.setConfigParam(k2, v)
            return self.trainValidate()
        best, cost, hist = parameter_search(space, score, strat, self.config.get_int("train.search.max.iterations")[0])
        return best, cost

    def validate(self):
        if self.config.get_boolean("validate.use.saved.model")[0]:
            self.load_model()
        else:
            self.train()
        X, y = self.prepValidationData()
        pred = self.model.predict(X)
        pred = np.asarray(pred if isinstance(pred, list) else torch.as_tensor(pred).cpu().numpy())
        method = self.config.get_string("validate.score.method")[0]
        if method == "confusionMatrix":
            return perf_metric("confusion", y.tolist(), pred.tolist())
        return perf_metric(method, y.tolist(), pred.tolist())

    def _predict_input(self, recs):
        if recs is None:
            X, _ = self._load("predict", with_class=False)
            return X
        if isinstance(recs, str):
            # REST form: records separated by ",," with comma-separated fields
            recs = [r.split(",") for r in recs.split(",,") if r]
        feats = self._ints("predict.data.feature.fields")
        arr = np.array([[float(r[i]) for i in feats] if feats else [float(v) for v in r] for r in recs], np.float32)
        return arr

    def _ensure_model(self):
        if self.model is None:
            if self.config.get_boolean("predict.use.saved.model")[0]:
                self.load_model()
            else:
                self.train()

    def predict(self, recs=None):
        self._ensure_model()
        return self.model.predict(self._predict_input(recs))

    def predictProb(self, recs=None):
        self._ensure_model()
        return self.model.predict_proba(self._predict_input(recs))

    def autoTrain(self):
        """Learning-curve driven check (bacl.py:380-442): train error vs CV error against the
        configured thresholds -> 'high bias' / 'high variance' / 'ok' diagnosis."""
        train_err = self.train()
        if self.config.get_string("train.success.criterion")[0] == "accuracy":
            train_err = 1 - train_err
        cv = self.trainValidate()
        test_err = cv if self.config.get_string("train.success.criterion")[0] != "accuracy" else 1 - cv
        max_test = self.config.get_float("train.auto.max.test.error")[0]
        max_err = self.config.get_float("train.auto.max.error")[0]
        max_diff = self.config.get_float("train.auto.max.error.diff")[0]
        if train_err > max_err:
            status = "high bias"
        elif test_err - train_err > max_diff:
            status = "high variance"
        elif test_err > max_test:
            status = "high error"
        else:
            status = "ok"
        return {"trainError": train_err, "testError": test_err, "status": status}

    # -- persistence ---------------------------------------------------------------------------
    def save_model(self):
        p = self._model_path()
        p.parent.mkdir(parents=True, exist_ok=True)
        st = self.model.state() if hasattr(self.model, "state") else None
        if st is None:
            raise NotImplementedError(f"{type(self.model).__name__} does not support saving")
        torch.save(st, p)

    def load_model(self):
        st = torch.load(self._model_path(), map_location="cpu", weights_only=True)
        if st.get("kind") == "rf":
            self.model = RandomForestClassifier.from_state(st, self.device)
        else:
            raise ValueError(f"unknown model kind {st.get('kind')}")


def _num(v: str):
    try:
        f = float(v)
        return int(f) if f.is_integer() else f
    except ValueError:
        return v


class RandomForest(BaseClassifier):
    extra_defaults = {"train.num.trees": (100, None), "train.split.criterion": ("gini", None),
                      "train.max.depth": (None, None), "train.min.samples.split": (4, None),
                      "train.max.features": ("auto", None), "train.bootstrap": (True, None),
                      "train.random.state": (None, None)}

    def build_model(self):
        c = self.config
        md = c.get_int("train.max.depth")[0]
        mf = c.get_string("train.max.features")[0]
        mf = "sqrt" if mf in ("auto", None) else (int(mf) if str(mf).isdigit() else mf)
        return RandomForestClassifier(c.get_int("train.num.trees")[0], md, c.get_string("train.split.criterion")[0],
                                      mf, c.get_int("train.min.samples.split")[0], c.get_boolean("train.bootstrap")[0],
                                      random_state=c.get_int("train.random.state")[0] or 0, device=self.device)


class GradientBoostedTrees(BaseClassifier):
    extra_defaults = {"train.learning.rate": (0.1, None), "train.num.estimators.gb": (100, None),
                      "train.max.depth.gb": (3, None), "train.subsample": (1.0, None),
                      "train.min.samples.leaf.gb": (1, None), "train.random.state": (None, None)}

    def build_model(self):
        c = self.config
        return GradientBoostingClassifier(c.get_int("train.num.estimators.gb")[0], c.get_float("train.learning.rate")[0],
                                          c.get_int("train.max.depth.gb")[0], c.get_float("train.subsample")[0],
                                          int(c.get_int("train.min.samples.leaf.gb")[0]),
                                          random_state=c.get_int("train.random.state")[0] or 0, device=self.device)


class SupportVectorMachine(BaseClassifier):
    extra_defaults = {"train.algorithm": ("svc", None), "train.kernel.function": ("rbf", None),
                      "train.poly.degree": (3, None), "train.penalty": (1.0, None), "train.gamma": ("scale", None)}

    def build_model(self):
        c = self.config
        g = c.get_string("train.gamma")[0]
        try:
            g = float(g)
        except (TypeError, ValueError):
            pass
        return SupportVectorClassifier(c.get_string("train.kernel.function")[0], c.get_float("train.penalty")[0], g,
                                       c.get_int("train.poly.degree")[0], device=self.device)


class LogisticRegressionDiscriminant(BaseClassifier):
    extra_defaults = {"train.penalty": ("l2", None), "train.reg.strength": (1.0, None), "train.max.iter": (50, None)}

    def build_model(self):
        c = self.config
        return LogisticRegressionClassifier(c.get_float("train.reg.strength")[0], c.get_string("train.penalty")[0],
                                            c.get_int("train.max.iter")[0], device=self.device)


class BaseRegressor:
    """``LinearRegressor`` / ``ElasticNetRegressor`` workflow (P/supv/regress.py): train,
    validate (rmse / mae / r2), predict."""

    def __init__(self, kind: str = "linear", alpha: float = 0.0, l1_ratio: float = 0.5):
        self.kind, self.alpha, self.l1_ratio = kind, alpha, l1_ratio
        self.model = None

    def fit(self, X, y):
        X = torch.as_tensor(np.asarray(X, dtype=np.float64))
        y = torch.as_tensor(np.asarray(y, dtype=np.float64))
        self.model = (L.LinearRegression(self.alpha) if self.kind == "linear" else
                      L.ElasticNet(self.alpha, self.l1_ratio)).fit(X, y)
        return self

    def predict(self, X):
        return self.model.predict(torch.as_tensor(np.asarray(X, dtype=np.float64)))

    def validate(self, X, y, metric: str = "rmse") -> float:
        p = self.predict(X).cpu().numpy()
        y = np.asarray(y, dtype=np.float64)
        if metric == "r2":
            return 1 - float(((y - p) ** 2).sum() / ((y - y.mean()) ** 2).sum())
        if metric == "mae":
            return float(np.abs(y - p).mean())
        return float(np.sqrt(((y - p) ** 2).mean()))


LinearRegressor = lambda **kw: BaseRegressor("linear", **kw)                      # noqa: E731
ElasticNetRegressor = lambda alpha=1.0, l1_ratio=0.5: BaseRegressor("elasticNet", alpha, l1_ratio)  # noqa: E731


# ================================================================================================
# J/model: predictive model wrappers
# ================================================================================================
class PredictiveModel:
    """Error counting and cost-based prediction around a probabilistic classifier
    (J/model/PredictiveModel.java:65-171, ProbabilisticPredictiveModel.java:41-59)."""

    def __init__(self, model, pos_class=1):
        self.model, self.pos = model, pos_class
        self.error_counting = False
        self.cost_based = False
        self.threshold = 0.5
        self.total = self.errors = self.fp = self.fn = 0

    def enableErrorCounting(self):
        self.error_counting = True
        return self

    def enableCostBasedPrediction(self, fp_cost: float, fn_cost: float):
        self.cost_based = True
        self.threshold = fp_cost / (fp_cost + fn_cost)
        return self

    def predict(self, X, actual=None):
        proba = torch.as_tensor(self.model.predict_proba(X)).cpu()
        if self.cost_based and proba.shape[1] == 2:
            pred = (proba[:, 1] >= self.threshold).long()
        else:
            pred = proba.argmax(1)
        if self.error_counting and actual is not None:
            a = torch.as_tensor(np.asarray(actual)).long()
            self.total += len(a)
            self.errors += int((pred != a).sum())
            self.fp += int(((pred == 1) & (a == 0)).sum())
            self.fn += int(((pred == 0) & (a == 1)).sum())
        return pred

    def getError(self):
        return self.errors / max(self.total, 1)

    def getFalsePosError(self):
        return self.fp / max(self.total, 1)

    def getFalseNegError(self):
        return self.fn / max(self.total, 1)


class EnsemblePredictiveModel:
    """Weighted majority vote of an odd number of member models; rows whose top / second vote
    ratio is below ``min_odds_ratio`` are ambiguous (-1) (EnsemblePredictiveModel.java:54-127).
    Votes are one scatter-add over [N, M] -> [N, C]."""

    def __init__(self, min_odds_ratio: float | None = None):
        self.models, self.weights = [], []
        self.min_odds = min_odds_ratio

    def addModel(self, model, weight: float = 1.0):
        self.models.append(model)
        self.weights.append(weight)
        return self

    def predict(self, X, n_classes: int = 2) -> torch.Tensor:
        if len(self.models) % 2 == 0:
            raise ValueError("ensemble needs an odd number of models")
        preds = torch.stack([torch.as_tensor(np.asarray(m.predict(X))).long().view(-1) for m in self.models], 1)
        w = torch.tensor(self.weights, dtype=torch.float64).view(1, -1).expand_as(preds)
        votes = torch.zeros((preds.shape[0], n_classes), dtype=torch.float64).scatter_add_(1, preds, w)
        top2 = torch.topk(votes, min(2, n_classes), 1).values
        out = votes.argmax(1)
        if self.min_odds is not None and n_classes > 1:
            ratio = top2[:, 0] / top2[:, 1].clamp_min(1e-12)
            out = torch.where(ratio >= self.min_odds, out, torch.full_like(out, -1))
        return out


class DeterministicPredictiveModel(PredictiveModel):
    """Label-only predictor (J/model/DeterministicPredictiveModel.java:41-49)."""

    def predict(self, X, actual=None):
        pred = torch.as_tensor(np.asarray(self.model.predict(X))).long().view(-1)
        if self.error_counting and actual is not None:
            a = torch.as_tensor(np.asarray(actual)).long()
            self.total += len(a)
            self.errors += int((pred != a).sum())
            self.fp += int(((pred == 1) & (a == 0)).sum())
            self.fn += int(((pred == 0) & (a == 1)).sum())
        return pred


class ModelPredictor:
    """Decision-tree model predictor (J/model/ModelPredictor.java:49-254): one or more tree models
    (decision-path JSON or native state); several models form a voting ensemble; output modes
    ``withRecord`` (record + prediction), ``withKId`` (id + prediction), ``withActualClassAttr``
    (id + actual + prediction); error rate reported at the end.  Batched inference = the K8
    forest kernel over all trees at once."""

    def __init__(self, trees: list, schema: FeatureSchema, output_mode: str = "withRecord", delim: str = ",",
                 min_odds_ratio: float | None = None):
        self.ens = T.TreeEnsemble(trees)
        self.schema, self.mode, self.delim, self.min_odds = schema, output_mode, delim, min_odds_ratio
        self.errors = self.total = 0

    @classmethod
    def from_state_files(cls, paths, schema: FeatureSchema, **kw):
        import json as _json
        trees = [T.DecisionTree.from_state(_json.loads(Path(p).read_text()), schema) for p in paths]
        return cls(trees, schema, **kw)

    def predict_lines(self, t: Table) -> list[str]:
        pred = self.ens.predict(t, self.min_odds).cpu().tolist()
        vals = self.ens.class_values
        ids = t.ids or [str(i) for i in range(t.n)]
        act = t.labels[: t.n].cpu().tolist() if t.labels is not None else None
        out = []
        d = self.delim
        for i, p in enumerate(pred):
            pv = vals[p] if 0 <= p < len(vals) else "ambiguous"
            if act is not None and act[i] < len(vals):
                self.total += 1
                self.errors += int(vals[act[i]] != pv)
            if self.mode == "withKId":
                out.append(f"{ids[i]}{d}{pv}")
            elif self.mode == "withActualClassAttr":
                out.append(f"{ids[i]}{d}{vals[act[i]] if act is not None else ''}{d}{pv}")
            else:
                out.append(f"{t.lines[i] if t.lines else ids[i]}{d}{pv}")
        return out

    def error_rate(self) -> float:
        return self.errors / max(self.total, 1)
