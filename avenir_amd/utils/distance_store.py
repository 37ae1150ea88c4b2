"""Persisted entity -> [(entity, distance)] store (J/util/EntityDistanceMapFileAccessor.java:70-123).

The reference writes a Hadoop ``MapFile`` from text lines ``key<delim>value`` and reads one key's
neighbour list per lookup (a sorted-file binary search each time).  Here the store is a CSR matrix
in three ``.npy`` files plus the entity list, opened with ``numpy.load(mmap_mode="r")``: a lookup is
two index reads and a slice of the memory-mapped column/value arrays, and the whole store can be
moved to the device as one sparse matrix for batched gathers (the agglomerative clusterer
scatter-adds a whole neighbour row into per-cluster sums in one op).

Text form accepted by :meth:`EntityDistanceStore.write_text`: ``entity,e1:d1,e2:d2,...`` (outer
delimiter ``delim``, inner ``sub_delim``) — the reference's reader splits both levels on the same
delimiter, which cannot parse its own writer's format; the two-level form is used here.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Iterable

import numpy as np
import torch


class EntityDistanceStore:
    def __init__(self, path: str | Path):
        p = Path(path)
        self.path = p
        self.entities: list[str] = json.loads((p / "entities.json").read_text())
        self.index = {e: i for i, e in enumerate(self.entities)}
        self.indptr = np.load(p / "indptr.npy", mmap_mode="r")
        self.cols = np.load(p / "cols.npy", mmap_mode="r")
        self.vals = np.load(p / "vals.npy", mmap_mode="r")

    # -- writing ---------------------------------------------------------------------------------
    @staticmethod
    def write_text(lines: Iterable[str], path: str | Path, delim: str = ",", sub_delim: str = ":") -> "EntityDistanceStore":
        rows: dict[str, list[tuple[str, float]]] = {}
        for ln in lines:
            parts = ln.split(delim)
            key = parts[0]
            lst = rows.setdefault(key, [])
            for p in parts[1:]:
                if not p:
                    continue
                e, d = p.rsplit(sub_delim, 1)
                lst.append((e, float(d)))
        return EntityDistanceStore.write_rows(rows, path)

    @staticmethod
    def write_pairs(src: Iterable[str], dst: Iterable[str], dist: Iterable[float], path: str | Path,
                    symmetric: bool = True) -> "EntityDistanceStore":
        rows: dict[str, list[tuple[str, float]]] = {}
        for a, b, d in zip(src, dst, dist):
            rows.setdefault(a, []).append((b, float(d)))
            if symmetric:
                rows.setdefault(b, []).append((a, float(d)))
        return EntityDistanceStore.write_rows(rows, path)

    @staticmethod
    def write_codes(src: "torch.Tensor", dst: "torch.Tensor", dist: "torch.Tensor", vocab: list[str], path: str | Path,
                    symmetric: bool = True) -> "EntityDistanceStore":
        """``write_pairs`` from dictionary codes (a native token table): entities are the vocabulary
        entries that occur, in string order; the CSR rows come from one stable sort of the (row,
        column) pairs — the same store as ``write_pairs`` without a Python object per pair."""
        import torch
        src, dst, dist = src.long().cpu(), dst.long().cpu(), dist.double().cpu()
        if symmetric:
            a = torch.stack([src, dst], 1).reshape(-1)
            b = torch.stack([dst, src], 1).reshape(-1)
            w = torch.stack([dist, dist], 1).reshape(-1)
        else:
            a, b, w = src, dst, dist
        used = torch.zeros(max(1, len(vocab)), dtype=torch.bool)
        used[a] = True
        used[b] = True
        ids = torch.nonzero(used).view(-1).tolist()
        order = sorted(ids, key=lambda c: vocab[c])
        ents = [vocab[c] for c in order]
        rank = torch.full((max(1, len(vocab)),), -1, dtype=torch.long)
        rank[torch.tensor(order, dtype=torch.long)] = torch.arange(len(order))
        ra, rb = rank[a], rank[b]
        o = torch.argsort(rb, stable=True)
        o = o[torch.argsort(ra[o], stable=True)]
        ra, rb, w = ra[o], rb[o], w[o]
        indptr = torch.zeros(len(ents) + 1, dtype=torch.long)
        if ra.numel():
            indptr[1:] = torch.cumsum(torch.bincount(ra, minlength=len(ents)), 0)
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        np.save(p / "indptr.npy", indptr.numpy())
        np.save(p / "cols.npy", rb.numpy().astype(np.int64))
        np.save(p / "vals.npy", w.numpy().astype(np.float64))
        (p / "entities.json").write_text(json.dumps(ents))
        return EntityDistanceStore(p)

    @staticmethod
    def write_rows(rows: dict[str, list[tuple[str, float]]], path: str | Path) -> "EntityDistanceStore":
        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        ents = sorted(set(rows) | {e for lst in rows.values() for e, _ in lst})
        idx = {e: i for i, e in enumerate(ents)}
        indptr = np.zeros(len(ents) + 1, dtype=np.int64)
        cols, vals = [], []
        for i, e in enumerate(ents):
            lst = sorted(rows.get(e, []), key=lambda x: idx[x[0]])
            cols += [idx[x] for x, _ in lst]
            vals += [d for _, d in lst]
            indptr[i + 1] = len(cols)
        np.save(p / "indptr.npy", indptr)
        np.save(p / "cols.npy", np.asarray(cols, dtype=np.int64))
        np.save(p / "vals.npy", np.asarray(vals, dtype=np.float64))
        (p / "entities.json").write_text(json.dumps(ents))
        return EntityDistanceStore(p)

    # -- reading ---------------------------------------------------------------------------------
    def read(self, key: str) -> dict[str, float]:
        """Neighbour map of one entity (the reference's ``read(key)``)."""
        i = self.index.get(key)
        if i is None:
            return {}
        a, b = int(self.indptr[i]), int(self.indptr[i + 1])
        return {self.entities[int(c)]: float(v) for c, v in zip(self.cols[a:b], self.vals[a:b])}

    def row(self, i: int) -> tuple[np.ndarray, np.ndarray]:
        a, b = int(self.indptr[i]), int(self.indptr[i + 1])
        return np.asarray(self.cols[a:b]), np.asarray(self.vals[a:b])

    def to_sparse(self, device="cpu") -> torch.Tensor:
        n = len(self.entities)
        return torch.sparse_csr_tensor(torch.from_numpy(np.asarray(self.indptr)), torch.from_numpy(np.asarray(self.cols)),
                                       torch.from_numpy(np.asarray(self.vals)), size=(n, n)).to(device)


def agglomerative_graphical(store: EntityDistanceStore, entities: list[str], threshold: float,
                            dist_scale: float | None = None) -> list[tuple[list[str], float]]:
    """Greedy edge-weighted clustering (J/cluster/AgglomerativeGraphical.java:108-131,
    EdgeWeightedCluster.java:58-77): each entity joins the cluster that maximises the new average
    edge weight ``(avg * E + sum_w) / (E + size)`` (E = size(size-1)/2) when that exceeds
    ``threshold``, else starts a new cluster.  Weights are similarities, or ``dist_scale - d`` for
    distances.  For an incoming entity the per-cluster weight sums come from ONE scatter-add of its
    neighbour row by the neighbours' cluster ids.  (The reference's new cluster never receives the
    entity that created it; here it does.)"""
    cl_of = np.full(len(store.entities), -1, dtype=np.int64)
    sizes: list[int] = []
    avg: list[float] = []
    members: list[list[str]] = []
    for e in entities:
        i = store.index.get(e)
        best, best_w = -1, -np.inf
        if i is not None and sizes:
            cols, vals = store.row(i)
            w = (dist_scale - vals) if dist_scale is not None else vals
            cid = cl_of[cols]
            ok = cid >= 0
            sums = np.bincount(cid[ok], weights=w[ok], minlength=len(sizes))
            sz = np.asarray(sizes, dtype=np.float64)
            E = sz * (sz - 1) / 2
            new_avg = (np.asarray(avg) * E + sums) / (E + sz)
            best = int(np.argmax(new_avg))
            best_w = float(new_avg[best])
        if best >= 0 and best_w > threshold:
            sizes[best] += 1
            avg[best] = best_w
            members[best].append(e)
            if i is not None:
                cl_of[i] = best
        else:
            sizes.append(1)
            avg.append(0.0)
            members.append([e])
            if i is not None:
                cl_of[i] = len(sizes) - 1
    return list(zip(members, avg))
