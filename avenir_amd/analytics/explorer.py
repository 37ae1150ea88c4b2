"""Data exploration workspace (``DataExplorer``, P/mlextra/daexp.py:70-1899).

Named data sets (numeric, binary, categorical) from files, arrays or lists, notes, save/restore,
and ~70 analysis methods returning result dicts with the reference's key names.  The numeric
core (moments, histograms, percentiles, extremes, correlations, auto/cross correlation via FFT,
regressions, outlier scores, trend/seasonality) runs as torch reductions on the workspace device;
the long tail of classical hypothesis tests delegates the p-value to scipy.stats on the host (the
reference does the same); Zhang's tests use device permutation sampling.

Differences: plotting methods render with matplotlib's Agg backend into ``plot_dir`` (PNG files,
one per call) when it is set and otherwise only return the plotted data (no display here);
``save``/``restore`` write JSON + .npz (no pickle).  The isolation-forest outliers use
``models/outlier.py`` (level-synchronous device trees) and the one-class-SVM outliers the K12 SMO
kernel (``models/svm.py::OneClassSVM``); both agree with scikit-learn statistically (random draws
differ).  kNN-distance, LOF and Mahalanobis scores are extra detectors.
"""
from __future__ import annotations

import json
import math
from pathlib import Path
from typing import Sequence

import numpy as np
import torch

from ..ops import distance as Dm


def _np(x):
    return x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


class DataExplorer:
    def __init__(self, verbose: bool = False, device="cpu", plot_dir: str | None = None):
        self.plot_dir = plot_dir
        self._nplots = 0
        self.data: dict[str, tuple[str, object]] = {}
        self.notes: dict[str, list[str]] = {}
        self.verbose = verbose
        self.device = torch.device(device)

    # ------------------------------------------------------------------------------------------
    # workspace
    # ------------------------------------------------------------------------------------------
    def _add(self, name, kind, values):
        if kind == "cat":
            self.data[name] = (kind, list(values))
        else:
            self.data[name] = (kind, torch.as_tensor(np.asarray(values, dtype=np.float64), device=self.device))
        self.notes.setdefault(name, [])

    def addListNumericData(self, values, name):
        self._add(name, "num", values)

    def addListBinaryData(self, values, name):
        self._add(name, "bin", values)

    def addListData(self, values, name):
        self._add(name, "num", values)

    def addCatListData(self, values, name):
        self._add(name, "cat", values)

    def addFileNumericData(self, path, *cols_names, delim=","):
        cols = cols_names[: len(cols_names) // 2]
        names = cols_names[len(cols_names) // 2:]
        arr = np.loadtxt(path, delimiter=delim, usecols=[int(c) for c in cols], ndmin=2)
        for j, n in enumerate(names):
            self._add(n, "num", arr[:, j])

    addFileData = addFileNumericData

    def addFileBinaryData(self, path, *cols_names, delim=","):
        cols = cols_names[: len(cols_names) // 2]
        names = cols_names[len(cols_names) // 2:]
        arr = np.loadtxt(path, delimiter=delim, usecols=[int(c) for c in cols], ndmin=2)
        for j, n in enumerate(names):
            self._add(n, "bin", arr[:, j])

    def addFileCatData(self, path, *cols_names, delim=","):
        cols = [int(c) for c in cols_names[: len(cols_names) // 2]]
        names = cols_names[len(cols_names) // 2:]
        rows = [l.rstrip("\n").split(delim) for l in Path(path).read_text().splitlines() if l.strip()]
        for c, n in zip(cols, names):
            self._add(n, "cat", [r[c] for r in rows])

    def addDataFrameData(self, df, *columns):
        """``addDataFrameData(df, numeric, *columns)`` as in the reference (``numeric`` True for
        numeric, False for binary; columns = indexes followed by names, or names), or
        ``addDataFrameData(df, *names)`` which infers numeric vs categorical per column."""
        if columns and isinstance(columns[0], (bool, np.bool_)):
            numeric, cols = bool(columns[0]), list(columns[1:])
            for name, col in self._df_columns(df, cols):
                arr = col.to_numpy()
                if numeric:
                    assert self.inferDataType(arr) in ("binary", "integer", "float"), "data is not numeric"
                else:
                    assert self.inferDataType(arr) == "binary", "data is not binary"
                self._add(str(name), "num" if numeric else "bin", arr)
            return
        for n in (columns or df.columns):
            kind = "cat" if df[n].dtype == object else "num"
            self._add(str(n), kind, df[n].tolist() if kind == "cat" else df[n].to_numpy())

    @staticmethod
    def _df_columns(df, cols):
        """(name, column) pairs for 'indexes followed by names' or plain column names."""
        if cols and isinstance(cols[0], (int, np.integer)):
            k = len(cols) // 2
            for ci, name in zip(cols[:k], cols[k:]):
                assert ci < len(df.columns), f"col index {ci} outside range"
                yield name, df.iloc[:, ci]
        else:
            for c in cols:
                yield c, df[c]

    def addDataFrameNumericData(self, df, *columns):
        self.addDataFrameData(df, True, *columns)

    def addDataFrameBinaryData(self, df, *columns):
        self.addDataFrameData(df, False, *columns)

    def addDataFrameCatData(self, df, *columns):
        for name, col in self._df_columns(df, list(columns)):
            self._add(str(name), "cat", [str(v) for v in col.tolist()])

    @staticmethod
    def _read_df(path, cols):
        import pandas as pd
        return pd.read_csv(path, header=None if cols and isinstance(cols[0], (int, np.integer)) else 0)

    def addFileData(self, path, numeric, *columns):
        """Reference form: ``addFileData(path, numeric, *columns)`` through a pandas frame (a
        header row when the columns are given by name)."""
        if not isinstance(numeric, (bool, np.bool_)):     # older form: numeric columns only
            return self.addFileNumericData(path, numeric, *columns)
        self.addDataFrameData(self._read_df(path, list(columns)), bool(numeric), *columns)

    def queryDataFrameData(self, df, *columns):
        """Inferred data type of each column: binary / integer / float / categorical / mixed."""
        return {"columns and data types": [(str(n), self.inferDataType(c.to_numpy()))
                                           for n, c in self._df_columns(df, list(columns))]}

    def queryFileData(self, path, *columns):
        return self.queryDataFrameData(self._read_df(path, list(columns)), *columns)

    def loadCatFloatDataFrame(self, ds1, ds2):
        """A frame with the categorical data set in column 0 and the numeric one in column 1."""
        import pandas as pd
        a, b = self.getCatData(ds1), _np(self.getNumericData(ds2))
        a, b = self.ensureSameSize([a, b])
        return pd.DataFrame({0: a, 1: b})

    def remData(self, name):
        self.data.pop(name, None)
        self.notes.pop(name, None)

    def addNote(self, name, note):
        self.notes.setdefault(name, []).append(note)

    def getNotes(self, name):
        return self.notes.get(name, [])

    def showNames(self):
        return sorted(self.data)

    def getDataType(self, name):
        """Workspace kind (num / bin / cat) of a data set name, or the inferred type of an array."""
        if isinstance(name, str) and name in self.data:
            return self.data[name][0]
        return self.inferDataType(name)

    @staticmethod
    def inferDataType(col) -> str:
        """binary / integer / float / categorical / mixed, the reference's order of checks."""
        a = np.asarray(col, dtype=object).ravel()
        if a.size == 0:
            return "mixed"
        nums = [isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool) for v in a]
        if all(nums):
            f = a.astype(np.float64)
            if np.all((f == 0) | (f == 1)):
                return "binary"
            if np.all(np.floor(f) == f):
                return "integer"
            return "float"
        if all(isinstance(v, str) for v in a):
            return "categorical"
        return "mixed"

    def print(self, ds):
        """First 50 values of a data set (and its size); returned as well as printed when verbose."""
        kind, v = self.data[ds]
        vals = v[:50] if kind == "cat" else _np(v[:50]).tolist()
        n = len(v) if kind == "cat" else int(v.numel())
        if self.verbose:
            print(f"size {n}")
            print("showing first 50 elements")
            print(vals)
        return {"size": n, "head": vals}

    def getNumericData(self, ds) -> torch.Tensor:
        if isinstance(ds, str):
            kind, v = self.data[ds]
            if kind == "cat":
                raise ValueError(f"{ds} is categorical")
            return v
        return torch.as_tensor(np.asarray(ds, dtype=np.float64), device=self.device)

    def getCatData(self, ds) -> list:
        if isinstance(ds, str):
            return list(self.data[ds][1])
        return list(ds)

    def save(self, path):
        p = Path(path)
        arrays = {k: _np(v) for k, (kind, v) in self.data.items() if kind != "cat"}
        meta = {"kinds": {k: kind for k, (kind, _) in self.data.items()},
                "cat": {k: v for k, (kind, v) in self.data.items() if kind == "cat"}, "notes": self.notes}
        np.savez(p.with_suffix(".npz"), **arrays)
        p.with_suffix(".json").write_text(json.dumps(meta))

    def restore(self, path):
        p = Path(path)
        meta = json.loads(p.with_suffix(".json").read_text())
        with np.load(p.with_suffix(".npz"), allow_pickle=False) as z:
            for k, kind in meta["kinds"].items():
                self._add(k, kind, meta["cat"][k] if kind == "cat" else z[k])
        self.notes = meta["notes"]

    # ------------------------------------------------------------------------------------------
    # distributions and summary statistics
    # ------------------------------------------------------------------------------------------
    def isMonotonicallyChanging(self, ds):
        d = torch.diff(self.getNumericData(ds))
        return {"monotonic increasing": bool((d >= 0).all()), "monotonic decreasing": bool((d <= 0).all())}

    def getFreqDistr(self, ds, nbins: int = 20):
        x = self.getNumericData(ds)
        lo, hi = float(x.min()), float(x.max())
        # scipy.stats.relfreq limits: extend the range by half a bin on each side
        width = (hi - lo) / (nbins - 1) if nbins > 1 and hi > lo else 1.0
        lo2 = lo - width / 2
        h = torch.histc(x.double(), bins=nbins, min=lo2, max=lo2 + width * nbins)
        return {"frequency": _np(h / x.numel()), "lowLimit": lo2, "binsize": width, "extraPoints": 0}

    def getCumFreqDistr(self, ds, nbins: int = 20):
        r = self.getFreqDistr(ds, nbins)
        r["cumFrequency"] = np.cumsum(r.pop("frequency"))
        return r

    def getExtremeValue(self, ds, ensamp: int, nsamp: int, polarity: str = "max", doPlotDistr=False, nbins=20):
        x = self.getNumericData(ds)
        g = torch.Generator(device=x.device).manual_seed(0)
        idx = torch.randint(0, x.numel(), (ensamp, nsamp), device=x.device, generator=g)
        s = x[idx]
        ev = s.max(1).values if polarity == "max" else s.min(1).values
        return {"extremes": _np(ev), "mean": float(ev.mean()), "std": float(ev.std())}

    def getEntropy(self, ds, nbins: int = 20):
        f = torch.as_tensor(self.getFreqDistr(ds, nbins)["frequency"])
        f = f[f > 0]
        return {"entropy": float(-(f * torch.log(f)).sum())}

    def getRelEntropy(self, ds1, ds2, nbins: int = 20):
        x1, x2 = self.getNumericData(ds1), self.getNumericData(ds2)
        lo, hi = float(min(x1.min(), x2.min())), float(max(x1.max(), x2.max()))
        p = torch.histc(x1, nbins, lo, hi) / x1.numel()
        q = torch.histc(x2, nbins, lo, hi) / x2.numel()
        m = (p > 0) & (q > 0)
        return {"relEntropy": float((p[m] * torch.log(p[m] / q[m])).sum())}

    def getMutualInfo(self, ds1, ds2, nbins: int = 20):
        x1, x2 = self.getNumericData(ds1), self.getNumericData(ds2)
        b1 = ((x1 - x1.min()) / (x1.max() - x1.min()).clamp_min(1e-300) * (nbins - 1e-9)).long()
        b2 = ((x2 - x2.min()) / (x2.max() - x2.min()).clamp_min(1e-300) * (nbins - 1e-9)).long()
        j = torch.bincount(b1 * nbins + b2, minlength=nbins * nbins).view(nbins, nbins).double() / x1.numel()
        p1, p2 = j.sum(1), j.sum(0)
        m = j > 0
        mi = (j[m] * torch.log(j[m] / (p1.view(-1, 1) * p2.view(1, -1))[m])).sum()
        return {"mutInfo": float(mi)}

    def getPercentile(self, ds, value):
        x = self.getNumericData(ds)
        # scipy percentileofscore(kind="rank"): mean of strict and weak percentiles
        lt, le = float((x < value).double().mean()), float((x <= value).double().mean())
        return {"value": value, "percentile": 50.0 * (lt + le)}

    def getValueRangePercentile(self, ds, value1, value2):
        return {"valueFirst": value1, "valueSecond": value2,
                "percentile": self.getPercentile(ds, value2)["percentile"] - self.getPercentile(ds, value1)["percentile"]}

    def getValueAtPercentile(self, ds, percent):
        return {"value": float(torch.quantile(self.getNumericData(ds), percent / 100.0)), "percentile": percent}

    def getLessThanValues(self, ds, cvalue):
        x = self.getNumericData(ds)
        sel = x < cvalue
        return {"count": int(sel.sum()), "values": _np(x[sel]), "indexes": _np(sel.nonzero().view(-1))}

    def getGreaterThanValues(self, ds, cvalue):
        x = self.getNumericData(ds)
        sel = x > cvalue
        return {"count": int(sel.sum()), "values": _np(x[sel]), "indexes": _np(sel.nonzero().view(-1))}

    def getUniqueValueCounts(self, ds, maxCnt: int = 10):
        u, c = torch.unique(self.getNumericData(ds), return_counts=True)
        o = torch.argsort(c, descending=True)[:maxCnt]
        return {"unique values": _np(u[o]), "counts": _np(c[o])}

    def getCatUniqueValueCounts(self, ds, maxCnt: int = 10):
        from collections import Counter
        c = Counter(self.getCatData(ds)).most_common(maxCnt)
        return {"unique values": [k for k, _ in c], "counts": [v for _, v in c]}

    def getStats(self, ds, nextreme: int = 5):
        from ..ops.encode_ops import column_moments, moments_dict
        x = self.getNumericData(ds).double()
        n = x.numel()
        mo = moments_dict(column_moments(x)[0])  # K26: moments in two streaming passes
        u, c = torch.unique(x, return_counts=True)
        xs = torch.sort(x).values
        med = torch.quantile(x, 0.5)
        return {"length": n, "min": mo["min"], "max": mo["max"],
                "n smallest": _np(xs[:nextreme]).tolist(),
                "n largest": _np(xs.flip(0)[:nextreme]).tolist(),
                "mean": mo["mean"], "median": float(med), "mode": float(u[c.argmax()]), "mode count": int(c.max()),
                "std": mo["std"], "skew": mo["skew"],
                "kurtosis": mo["kurtosis"], "mad": float((x - med).abs().median() * 1.4826)}

    def getNullCount(self, ds):
        x = self.getNumericData(ds)
        return {"nullCount": int(torch.isnan(x).sum())}

    def getDifference(self, ds, order: int = 1):
        x = self.getNumericData(ds)
        return _np(x[order:] - x[:-order])

    # ------------------------------------------------------------------------------------------
    # trend, seasonality, regression
    # ------------------------------------------------------------------------------------------
    def getTrend(self, ds, doPlot=False):
        y = self.getNumericData(ds).double()
        n = y.numel()
        t = torch.arange(n, dtype=torch.float64, device=y.device)
        A = torch.stack([t, torch.ones_like(t)], 1)
        coef = torch.linalg.lstsq(A, y.view(-1, 1)).solution.view(-1)
        trend = A @ coef
        r2 = 1 - float(((y - trend) ** 2).sum() / ((y - y.mean()) ** 2).sum().clamp_min(1e-300))
        return {"coeff": [float(coef[0])], "intercept": float(coef[1]), "r square error": r2, "trend": _np(trend)}

    def deTrend(self, ds, trend, doPlot=False):
        return _np(self.getNumericData(ds) - torch.as_tensor(np.asarray(trend), device=self.device))

    def getTimeSeriesComponents(self, ds, model: str, freq: int, summaryOnly: bool = True, doPlot=False):
        """Classical decomposition (centred moving-average trend, period-mean seasonal, residue)."""
        x = self.getNumericData(ds).double()
        n = x.numel()
        if freq % 2 == 0:
            w = torch.ones(freq + 1, dtype=torch.float64, device=x.device)
            w[0] = w[-1] = 0.5
            w /= freq
        else:
            w = torch.ones(freq, dtype=torch.float64, device=x.device) / freq
        h = (w.numel() - 1) // 2
        tr = torch.full_like(x, float("nan"))
        tr[h:n - h] = torch.nn.functional.conv1d(x.view(1, 1, -1), w.view(1, 1, -1)).view(-1)
        det = x - tr if model == "additive" else x / tr
        idx = torch.arange(n, device=x.device) % freq
        ok = ~torch.isnan(det)
        per = torch.zeros(freq, dtype=torch.float64, device=x.device).index_add_(0, idx[ok], det[ok])
        cnt = torch.bincount(idx[ok], minlength=freq).double()
        per = per / cnt.clamp_min(1)
        per = per - per.mean() if model == "additive" else per / per.mean()
        seas = per[idx]
        resid = x - tr - seas if model == "additive" else x / (tr * seas)
        trv, rv = tr[~torch.isnan(tr)], resid[~torch.isnan(resid)]
        res = {"trendMean": float(trv.mean()), "trendSlope": float((trv[-1] - trv[0]) / (trv.numel() - 1)),
               "seasonalAmp": float((seas.max() - seas.min()) / 2), "residueMean": float(rv.mean()),
               "residueStdDev": float(rv.std(unbiased=False))}
        if not summaryOnly:
            res.update({"trend": _np(tr), "seasonal": _np(seas), "residual": _np(resid)})
        return res

    def fitLinearReg(self, dsx, dsy, doPlot=False):
        x, y = self.getNumericData(dsx).double(), self.getNumericData(dsy).double()
        A = torch.stack([x, torch.ones_like(x)], 1)
        c = torch.linalg.lstsq(A, y.view(-1, 1)).solution.view(-1)
        pred = A @ c
        r2 = 1 - float(((y - pred) ** 2).sum() / ((y - y.mean()) ** 2).sum())
        return {"coeff": float(c[0]), "intercept": float(c[1]), "r square error": r2}

    def fitSiegelRobustLinearReg(self, dsx, dsy, doPlot=False):
        """Repeated medians: slope = median_i median_{j!=i} slope(i, j) — one [n, n] device tensor."""
        x, y = self.getNumericData(dsx).double(), self.getNumericData(dsy).double()
        dx = x.view(1, -1) - x.view(-1, 1)
        dy = y.view(1, -1) - y.view(-1, 1)
        s = torch.where(dx != 0, dy / dx, torch.full_like(dx, float("nan")))
        slope = float(torch.nanmedian(torch.nanmedian(s, 1).values))
        return {"slope": slope, "intercept": float(torch.median(y - slope * x))}

    def fitTheilSenRobustLinearReg(self, dsx, dsy, doPlot=False):
        x, y = self.getNumericData(dsx).double(), self.getNumericData(dsy).double()
        i, j = torch.triu_indices(x.numel(), x.numel(), 1, device=x.device)
        dx = x[j] - x[i]
        ok = dx != 0
        slope = float(torch.median((y[j] - y[i])[ok] / dx[ok]))
        return {"slope": slope, "intercept": float(torch.median(y) - slope * torch.median(x))}

    # ------------------------------------------------------------------------------------------
    # outliers
    # ------------------------------------------------------------------------------------------
    def _matrix(self, dss):
        return torch.stack([self.getNumericData(d).float() for d in dss], 1)

    def getOutliersWithKnnDistance(self, dss, k: int = 5, contamination: float = 0.05):
        X = self._matrix(dss if isinstance(dss, (list, tuple)) else [dss])
        d, _ = Dm.knn(X, X, k, exclude_self=True)
        sc = d[:, -1]
        thr = torch.quantile(sc, 1 - contamination)
        return {"scores": _np(sc), "outliers": _np((sc > thr).nonzero().view(-1))}

    def _outlier_result(self, X, is_out):
        m = _np(is_out).astype(bool)
        Xn = _np(X)
        return {"numOutliers": int(m.sum()), "outliers": Xn[m], "dataWithoutOutliers": Xn[~m],
                "outlierIndexes": np.nonzero(m)[0]}

    def getOutliersWithIsoForest(self, contamination, *dsl, seed: int = 0):
        """Isolation forest over the named numeric data sets (P/mlextra/daexp.py:921-941)."""
        from ..models.outlier import IsolationForest
        assert 0 <= contamination <= 0.5, "contamination outside valid range"
        X = self._matrix(dsl)
        iso = IsolationForest(contamination=contamination if contamination > 0 else "auto", seed=seed)
        return self._outlier_result(X, iso.fit_predict(X) == -1)

    def getOutliersWithLocalFactor(self, dss, k: int = 10, contamination: float = 0.05):
        """Local outlier factor from the k-NN graph (reachability distances)."""
        X = self._matrix(dss if isinstance(dss, (list, tuple)) else [dss])
        d, idx = Dm.knn(X, X, k, exclude_self=True)
        kd = d[:, -1]
        reach = torch.maximum(d, kd[idx])
        lrd = 1.0 / reach.mean(1).clamp_min(1e-12)
        lof = lrd[idx].mean(1) / lrd
        thr = torch.quantile(lof, 1 - contamination)
        return {"scores": _np(lof), "outliers": _np((lof > thr).nonzero().view(-1))}

    def getOutliersWithCovarDeterminant(self, dss, contamination: float = 0.05):
        X = self._matrix(dss if isinstance(dss, (list, tuple)) else [dss]).double()
        mu = X.mean(0)
        C = torch.cov(X.T).view(X.shape[1], X.shape[1])
        Ci = torch.linalg.pinv(C)
        d = X - mu
        md = (d @ Ci * d).sum(1)
        thr = torch.quantile(md, 1 - contamination)
        return {"scores": _np(md), "outliers": _np((md > thr).nonzero().view(-1))}

    def getOutliersWithSupVecMach(self, nu, *dsl):
        """One-class SVM (RBF, gamma 'scale') outliers (P/mlextra/daexp.py:965-985)."""
        from ..models.svm import OneClassSVM
        assert 0 <= nu <= 0.5, "error upper bound outside valid range"
        X = self._matrix(dsl)
        svm = OneClassSVM(nu=nu).fit(X)
        return self._outlier_result(X, svm.predict(X) == -1)

    # ------------------------------------------------------------------------------------------
    # correlation
    # ------------------------------------------------------------------------------------------
    def getCovar(self, *dss):
        return _np(torch.cov(self._matrix(dss).double().T))

    def getPearsonCorr(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        x, y = self.getNumericData(ds1).double(), self.getNumericData(ds2).double()
        xc, yc = x - x.mean(), y - y.mean()
        r = float((xc @ yc) / (xc.norm() * yc.norm()))
        n = x.numel()
        t = r * math.sqrt((n - 2) / max(1e-300, 1 - r * r))
        return {"stat": r, "pvalue": float(2 * stats.t.sf(abs(t), n - 2))}

    def _rank(self, x):
        """Average ranks over ties (K26 rank_avg kernel on the GPU)."""
        from ..ops.stats_ops import rank_avg
        return rank_avg(x)[0]

    def getSpearmanRankCorr(self, ds1, ds2, sigLev=0.05):
        from ..ops.stats_ops import spearman
        rho, p = spearman(self.getNumericData(ds1), self.getNumericData(ds2))
        return {"stat": rho, "pvalue": p}

    def getKendalRankCorr(self, ds1, ds2, sigLev=0.05):
        """tau-b from exact device pair counts (K26 kendall_pairs) + tie terms of the ranks."""
        from ..ops.stats_ops import kendall_tau_b
        tau, p = kendall_tau_b(self.getNumericData(ds1), self.getNumericData(ds2))
        return {"stat": tau, "pvalue": p}

    def getPointBiserialCorr(self, ds1, ds2, sigLev=0.05):
        return self.getPearsonCorr(ds1, ds2)

    def getConTab(self, ds1, ds2):
        a, b = self.getCatData(ds1), self.getCatData(ds2)
        ra, rb = sorted(set(a)), sorted(set(b))
        ia = torch.tensor([ra.index(v) for v in a])
        ib = torch.tensor([rb.index(v) for v in b])
        t = torch.bincount(ia * len(rb) + ib, minlength=len(ra) * len(rb)).view(len(ra), len(rb))
        return {"rowValues": ra, "colValues": rb, "table": _np(t)}

    def getChiSqCorr(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        t = self.getConTab(ds1, ds2)["table"]
        chi2, p, dof, _ = stats.chi2_contingency(t)
        return {"stat": float(chi2), "pvalue": float(p), "dof": int(dof)}

    def getAnovaCorr(self, ds1, ds2, sigLev=0.05):
        """One-way ANOVA of numeric ds1 grouped by categorical ds2."""
        from scipy import stats
        x = _np(self.getNumericData(ds1))
        g = self.getCatData(ds2)
        groups = [x[[i for i, v in enumerate(g) if v == k]] for k in sorted(set(g))]
        f, p = stats.f_oneway(*groups)
        return {"stat": float(f), "pvalue": float(p)}

    # ------------------------------------------------------------------------------------------
    # time-series correlation and spectra
    # ------------------------------------------------------------------------------------------
    def getAutoCorr(self, ds, nlags: int = 40):
        x = self.getNumericData(ds).double()
        n = x.numel()
        xc = x - x.mean()
        f = torch.fft.rfft(xc, n=2 * n)
        ac = torch.fft.irfft(f * f.conj(), n=2 * n)[: nlags + 1]
        return {"autoCorr": _np(ac / ac[0])}

    def getParAutoCorr(self, ds, nlags: int = 40):
        """Durbin-Levinson recursion on the sample autocorrelation."""
        r = self.getAutoCorr(ds, nlags)["autoCorr"]
        pacf = [1.0]
        phi = np.zeros((nlags + 1, nlags + 1))
        for k in range(1, nlags + 1):
            num = r[k] - sum(phi[k - 1, j] * r[k - j] for j in range(1, k))
            den = 1 - sum(phi[k - 1, j] * r[j] for j in range(1, k))
            phi[k, k] = num / den if den != 0 else 0.0
            for j in range(1, k):
                phi[k, j] = phi[k - 1, j] - phi[k, k] * phi[k - 1, k - j]
            pacf.append(phi[k, k])
        return {"partAutoCorr": np.array(pacf)}

    def getCrossCorr(self, ds1, ds2, nlags: int = 40):
        x, y = self.getNumericData(ds1).double(), self.getNumericData(ds2).double()
        n = x.numel()
        xc, yc = x - x.mean(), y - y.mean()
        c = torch.fft.irfft(torch.fft.rfft(xc, n=2 * n) * torch.fft.rfft(yc, n=2 * n).conj(), n=2 * n)
        c = c / (n * xc.std(unbiased=False) * yc.std(unbiased=False))
        return {"crossCorr": _np(c[: nlags + 1])}

    def getFourierTransform(self, ds, slen: int | None = None):
        x = self.getNumericData(ds).double()
        f = torch.fft.rfft(x - x.mean(), n=slen)
        return {"amplitude": _np(f.abs()), "frequency": _np(torch.fft.rfftfreq(slen or x.numel()))}

    # ------------------------------------------------------------------------------------------
    # stationarity and normality
    # ------------------------------------------------------------------------------------------
    def testStationaryAdf(self, ds, regression: str = "c", autolag=None, sigLev=0.05):
        """Augmented Dickey-Fuller statistic with 1 lag (constant) and MacKinnon 5% critical value
        -2.86 (p-value approximate: parity unpinned without statsmodels)."""
        x = self.getNumericData(ds).double()
        dx = torch.diff(x)
        y = dx[1:]
        A = torch.stack([x[1:-1], dx[:-1], torch.ones_like(y)], 1)
        sol = torch.linalg.lstsq(A, y.view(-1, 1)).solution.view(-1)
        res = y - A @ sol
        s2 = (res @ res) / (y.numel() - 3)
        cov = s2 * torch.linalg.inv(A.T @ A)
        stat = float(sol[0] / cov[0, 0].sqrt())
        return {"stat": stat, "critical values": {"1%": -3.43, "5%": -2.86, "10%": -2.57},
                "stationary": stat < -2.86}

    def testStationaryKpss(self, ds, regression: str = "c", nlags: int | None = None, sigLev=0.05):
        x = self.getNumericData(ds).double()
        n = x.numel()
        e = x - x.mean()
        S = torch.cumsum(e, 0)
        L = nlags if nlags is not None else int(math.ceil(12 * (n / 100) ** 0.25))
        s2 = float(e @ e) / n
        for l in range(1, L + 1):
            w = 1 - l / (L + 1)
            s2 += 2 * w * float(e[l:] @ e[:-l]) / n
        stat = float((S @ S) / (n * n * s2))
        return {"stat": stat, "critical values": {"10%": 0.347, "5%": 0.463, "1%": 0.739}, "stationary": stat < 0.463}

    def _scipy_test(self, fn, *arrs, **kw):
        r = fn(*[_np(a) for a in arrs], **kw)
        stat = getattr(r, "statistic", r[0])
        pv = getattr(r, "pvalue", r[1] if len(r) > 1 else None)
        return {"stat": float(stat) if np.ndim(stat) == 0 else _np(stat),
                "pvalue": None if pv is None or np.ndim(pv) else float(pv)}

    def testNormalJarqBera(self, ds, sigLev=0.05):
        from scipy import stats
        return self._scipy_test(stats.jarque_bera, self.getNumericData(ds))

    def testNormalShapWilk(self, ds, sigLev=0.05):
        from scipy import stats
        return self._scipy_test(stats.shapiro, self.getNumericData(ds))

    def testNormalDagast(self, ds, sigLev=0.05):
        from scipy import stats
        return self._scipy_test(stats.normaltest, self.getNumericData(ds))

    def testDistrAnderson(self, ds, dist: str = "norm", sigLev=0.05):
        from scipy import stats
        r = stats.anderson(_np(self.getNumericData(ds)), dist)
        return {"stat": float(r.statistic), "critical values": r.critical_values.tolist(),
                "significance levels": r.significance_level.tolist()}

    def testSkew(self, ds, sigLev=0.05):
        from scipy import stats
        return self._scipy_test(stats.skewtest, self.getNumericData(ds))

    # ------------------------------------------------------------------------------------------
    # two-sample tests
    # ------------------------------------------------------------------------------------------
    def _two(self, fn, ds1, ds2, **kw):
        return self._scipy_test(fn, self.getNumericData(ds1), self.getNumericData(ds2), **kw)

    def testTwoSampleStudent(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        return self._two(stats.ttest_ind, ds1, ds2)

    def testTwoSampleKs(self, ds1, ds2, sigLev=0.05):
        """KS statistic on device (merged-sample ECDF difference), p-value from scipy."""
        from scipy import stats
        a, b = torch.sort(self.getNumericData(ds1)).values, torch.sort(self.getNumericData(ds2)).values
        allv = torch.cat([a, b])
        cdf1 = torch.searchsorted(a, allv, right=True).double() / a.numel()
        cdf2 = torch.searchsorted(b, allv, right=True).double() / b.numel()
        d = float((cdf1 - cdf2).abs().max())
        return {"stat": d, "pvalue": float(stats.ks_2samp(_np(a), _np(b)).pvalue)}

    def testTwoSampleMw(self, ds1, ds2, sigLev=0.05):
        """U from device rank sums of the merged sample (K26 rank_avg), scipy's p-value formula."""
        from ..ops.stats_ops import mann_whitney_u
        u, p = mann_whitney_u(self.getNumericData(ds1), self.getNumericData(ds2))
        return {"stat": u, "pvalue": p}

    def testTwoSampleWilcox(self, ds1, ds2, sigLev=0.05):
        """Signed-rank statistic from device ranks of |x - y| (K26 rank_avg), scipy's formulas."""
        from ..ops.stats_ops import wilcoxon_signed_rank
        w, p = wilcoxon_signed_rank(self.getNumericData(ds1), self.getNumericData(ds2))
        return {"stat": w, "pvalue": p}

    def testTwoSampleKw(self, ds1, ds2, sigLev=0.05):
        from ..ops.stats_ops import kruskal_h
        h, p = kruskal_h(self.getNumericData(ds1), self.getNumericData(ds2))
        return {"stat": h, "pvalue": p}

    def testTwoSampleFriedman(self, ds1, ds2, ds3, sigLev=0.05):
        from scipy import stats
        return self._scipy_test(stats.friedmanchisquare, self.getNumericData(ds1), self.getNumericData(ds2),
                                self.getNumericData(ds3))

    def testTwoSampleEs(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        return self._two(stats.epps_singleton_2samp, ds1, ds2)

    def testTwoSampleAnderson(self, ds1, ds2, sigLev=0.05):
        """k-sample Anderson-Darling (midrank) with the A2 sums on the samples' device."""
        from ..ops.stats_ops import anderson_ksamp
        a2, _, p = anderson_ksamp(self.getNumericData(ds1), self.getNumericData(ds2))
        return {"stat": a2, "pvalue": p}

    def testTwoSampleScaleAb(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        return self._two(stats.ansari, ds1, ds2)

    def testTwoSampleScaleMood(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        return self._two(stats.mood, ds1, ds2)

    def testTwoSampleVarBartlet(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        return self._two(stats.bartlett, ds1, ds2)

    def testTwoSampleVarLevene(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        return self._two(stats.levene, ds1, ds2)

    def testTwoSampleVarFk(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        return self._two(stats.fligner, ds1, ds2)

    def testTwoSampleMedMood(self, ds1, ds2, sigLev=0.05):
        from scipy import stats
        r = stats.median_test(_np(self.getNumericData(ds1)), _np(self.getNumericData(ds2)))
        return {"stat": float(r[0]), "pvalue": float(r[1])}

    def testTwoSampleCvm(self, ds1, ds2, sigLev=0.05):
        """Two-sample Cramer-von Mises from device pooled ranks (K26 rank_avg)."""
        from ..ops.stats_ops import cvm_2samp
        t, p = cvm_2samp(self.getNumericData(ds1), self.getNumericData(ds2))
        return {"stat": t, "pvalue": p}

    # Zhang (2002, 2006) likelihood-ratio EDF tests with device permutation p-values
    def _zhang(self, ds1, ds2, kind: str, nperm: int = 500, seed: int = 0):
        a, b = self.getNumericData(ds1).double(), self.getNumericData(ds2).double()
        z = torch.cat([a, b])
        n1, N = a.numel(), z.numel()
        g = torch.Generator(device=z.device).manual_seed(seed)
        perms = torch.stack([torch.randperm(N, device=z.device, generator=g) for _ in range(nperm)])
        labels = torch.zeros((nperm + 1, N), dtype=torch.bool, device=z.device)
        labels[0, :n1] = True
        labels[1:] = perms < n1
        order = torch.argsort(z)
        lab = labels[:, order]                                     # [P, N] in sorted order
        c1 = torch.cumsum(lab.double(), 1)
        c2 = torch.cumsum((~lab).double(), 1)
        n2 = N - n1
        i = torch.arange(1, N + 1, dtype=torch.float64, device=z.device)
        F1, F2 = c1 / n1, c2 / n2
        F = i / N
        eps = 1e-12

        def lr(Fk, nk):
            return nk * (Fk * torch.log((Fk + eps) / (F + eps)) + (1 - Fk) * torch.log((1 - Fk + eps) / (1 - F + eps)))
        if kind == "Zk":
            s = (lr(F1, n1) + lr(F2, n2)).max(1).values
        elif kind == "Za":
            s = ((lr(F1, n1) + lr(F2, n2)) / ((i - 0.5) * (N - i + 0.5))).sum(1)
        else:  # Zc
            s = ((lr(F1, n1) + lr(F2, n2)) / (i * (N - i + 1))).sum(1)
        stat = s[0]
        p = float((s[1:] >= stat).double().mean())
        return {"stat": float(stat), "pvalue": p}

    def testTwoSampleZc(self, ds1, ds2, sigLev=0.05):
        return self._zhang(ds1, ds2, "Zc")

    def testTwoSampleZa(self, ds1, ds2, sigLev=0.05):
        return self._zhang(ds1, ds2, "Za")

    def testTwoSampleZk(self, ds1, ds2, sigLev=0.05):
        return self._zhang(ds1, ds2, "Zk")

    def ensureSameSize(self, dlist):
        m = min(len(d) for d in dlist)
        return [d[:m] for d in dlist]

    # ------------------------------------------------------------------------------------------
    # plots (P/mlextra/daexp.py:488-560, 1080-1090, 1230-1300): Agg-rendered PNGs in plot_dir
    # ------------------------------------------------------------------------------------------
    def _render(self, tag: str, draw) -> str | None:
        """Run ``draw(ax)`` on a fresh Agg figure and save it as ``<plot_dir>/<n>_<tag>.png``;
        nothing is drawn without a plot_dir (or without matplotlib)."""
        if not self.plot_dir:
            return None
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except ImportError:
            return None
        Path(self.plot_dir).mkdir(parents=True, exist_ok=True)
        fig, ax = plt.subplots()
        try:
            draw(ax)
            self._nplots += 1
            path = str(Path(self.plot_dir) / f"{self._nplots:03d}_{tag}.png")
            fig.savefig(path)
        finally:
            plt.close(fig)
        return path

    def plot(self, ds, yscale=None):
        y = _np(self.getNumericData(ds))

        def draw(ax):
            ax.plot(y)
            if yscale:
                ax.set_yscale(yscale)
        return {"data": y, "file": self._render("plot", draw)}

    def plotZoomed(self, ds, beg, end, yscale=None):
        y = _np(self.getNumericData(ds))[beg:end]

        def draw(ax):
            ax.plot(np.arange(beg, beg + len(y)), y)
            if yscale:
                ax.set_yscale(yscale)
        return {"data": y, "file": self._render("zoomed", draw)}

    def scatterPlot(self, ds1, ds2):
        a, b = self.ensureSameSize([_np(self.getNumericData(ds1)), _np(self.getNumericData(ds2))])
        x = np.arange(1, len(a) + 1)

        def draw(ax):
            ax.scatter(x, a, color="red")
            ax.scatter(x, b, color="blue")
        return {"data": (a, b), "file": self._render("scatter", draw)}

    def plotHist(self, ds, cumulative=False, density=False, nbins=20):
        x = self.getNumericData(ds).double()
        lo, hi = float(x.min()), float(x.max())
        cnt = torch.histc(x, bins=nbins, min=lo, max=hi if hi > lo else lo + 1.0)
        edges = np.linspace(lo, hi if hi > lo else lo + 1.0, nbins + 1)
        h = _np(cnt)
        if density:
            h = h / max(h.sum() * (edges[1] - edges[0]), 1e-300)
        if cumulative:
            h = np.cumsum(h)

        def draw(ax):
            ax.stairs(h, edges, fill=True)
        return {"counts": h, "edges": edges, "file": self._render("hist", draw)}

    def plotRegFit(self, x, y, slope, intercept):
        x, y = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)

        def draw(ax):
            ax.plot(x, y, "b.")
            ax.plot(x, intercept + slope * x, "r-")
        return {"fit": intercept + slope * x, "file": self._render("regfit", draw)}

    def _bars(self, tag, vals, alpha_band=None):
        def draw(ax):
            ax.stem(np.arange(len(vals)), vals)
            if alpha_band is not None:
                ax.axhline(alpha_band, ls="--")
                ax.axhline(-alpha_band, ls="--")
        return self._render(tag, draw)

    def plotAutoCorr(self, ds, lags, alpha=0.05, diffOrder=0):
        """Autocorrelation bars with the +-z/sqrt(n) band (the reference's statsmodels plot_acf)."""
        x = self.getNumericData(ds)
        if diffOrder > 0:
            for _ in range(diffOrder):
                x = x[1:] - x[:-1]
            ds = x
        ac = self.getAutoCorr(ds, lags)["autoCorr"]
        band = self._z(alpha) / math.sqrt(max(int(x.numel()), 1))
        return {"autoCorr": ac, "file": self._bars("acf", ac, band)}

    def plotParAcf(self, ds, lags, alpha=0.05):
        pac = self.getParAutoCorr(ds, lags)
        vals = np.asarray(pac["partAutoCorr"])
        band = self._z(alpha) / math.sqrt(max(int(self.getNumericData(ds).numel()), 1))
        return {"partAutoCorr": vals, "file": self._bars("pacf", vals, band)}

    def plotCrossCorr(self, ds1, ds2, normed=True, lags=10):
        cc = self.getCrossCorr(ds1, ds2, lags)["crossCorr"]
        return {"crossCorr": cc, "file": self._bars("xcorr", cc)}

    @staticmethod
    def _z(alpha):
        from scipy.stats import norm
        return float(norm.ppf(1 - alpha / 2))
