"""Device-resident random-forest builder: all trees grow together, level-synchronously, with their
bootstrap rows partitioned in HBM (kernels and design notes in ``csrc/kernels/forest.hip``).

Reference: random forest = ``DecisionTreeBuilder`` repeated per tree with sub-sampling and random
attribute subsets (J/tree/DecisionTreeBuilder.java:137-193 sampling, :365-381 attribute selection,
:499-616 expandTree, R/rafo.sh), each level one MapReduce job.  Per level here, for ALL trees:

1. histogram of the smaller child of every split (one chunked launch over contiguous segments;
   the larger child = parent - sibling, one batched tensor op); all-reduced when data-parallel;
2. K6/K7 split scoring of every frontier node (one launch; random feature subsets as masks drawn
   by one device RNG call; ``best`` or ``randomAmongTop``);
3. stopping rules (maxDepth / minPopulation / minInfoGain / pure) as tensor ops;
4. ONE device->host copy: decisions + per-chunk left-row counts;
5. numpy (vectorised, no per-node Python loop) child segments, build/derive slots, next work lists;
6. stable partition of every splitting node's rows into [left | right] (double buffer).

The trees come back as :class:`models.tree.DecisionTree` (same predicates, decision-path JSON,
flattening for the K8 inference kernel).  Binary threshold splits over the split space's ordered
fine bins (numeric and categorical), like ``TreeParams(binary=True)``.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass

import numpy as np
import torch

from ..data.table import Table
from ..ops import forest_ops as FO
from ..parallel.comm import Comm, get_comm
from ..utils.schema import FeatureSchema
from . import tree as T


@dataclass
class _Frontier:
    node: np.ndarray      # global node id (into the node table)
    start: np.ndarray     # int64 local row offset of the node's segment in the buffer
    count: np.ndarray     # int64 local row count
    depth: np.ndarray     # int64
    key: np.ndarray       # int64 holding a uint32 per-node random key (see _h32)


_M32 = 0xFFFFFFFF


def _h32(x):
    """32-bit integer mixer (two multiply-xorshift rounds) on int64 arrays / tensors holding uint32
    values; every product stays below 2^59, so numpy, torch CPU and torch GPU agree bit for bit."""
    x = x & _M32
    x = (((x >> 16) ^ x) * 0x45D9F3B) & _M32
    x = (((x >> 16) ^ x) * 0x45D9F3B) & _M32
    return (x >> 16) ^ x


def _child_keys(key: np.ndarray) -> np.ndarray:
    """Keys of the (left, right) children, interleaved: a node's random stream depends only on the
    seed, its tree id and its path, never on which other trees / ranks grow alongside it."""
    return np.stack([_h32(key ^ 0x5BD1E995), _h32(key ^ 0x1B873593)], 1).reshape(-1)


class ForestBuilder:
    """Grow ``n_trees`` binary-split trees at once.

    ``params``: a :class:`models.tree.TreeParams` (algorithm, stopping, max_depth,
    min_population, min_info_gain, attr_selection + random_attr_count, split_selection +
    top_split_count, sub_sampling + sampling_rate, seed, max_bins).  ``comm``: data-parallel over
    row shards (histograms all-reduced per level); ``tree_parallel`` distributes whole trees over
    ranks instead (no per-level collective)."""

    def __init__(self, schema: FeatureSchema, n_trees: int, params: T.TreeParams, comm: Comm | None = None,
                 chunk: int | None = None):
        self.schema = schema
        self.n_trees = n_trees
        self.p = params
        self.comm = comm
        self.chunk = chunk
        self.level_times: list[float] = []
        self.stats: dict = {}

    # ------------------------------------------------------------------------------------------
    def _boot_keys(self, tree_ids: list[int]) -> np.ndarray:
        """One 64-bit bootstrap key per tree from (seed, tree id): the sample of a tree depends on
        nothing else (not the rank, the device or the world size — rows are keyed globally)."""
        p = self.p
        k = (np.asarray(tree_ids, dtype=np.uint64) + np.uint64(1)) * np.uint64(0xD1B54A32D192ED03)
        with np.errstate(over="ignore"):
            k ^= np.uint64((p.seed * 1000003 + 17) & 0xFFFFFFFFFFFFFFFF)
        return k.view(np.int64)

    def _weights(self, n: int, row_off: int, tree_ids: list[int]) -> np.ndarray:
        """uint8 [T, n] bootstrap multiplicities of this rank's rows (host; the builder draws them
        on the device inside ``forest_bootstrap``): Poisson(1) = with replacement, Bernoulli
        (without replacement, rate %), or ones."""
        mode, rate32 = self._boot_mode()
        rows = np.arange(row_off, row_off + n, dtype=np.int64)
        return np.stack([FO.boot_weights(int(k), rows, mode, rate32) for k in self._boot_keys(tree_ids)])

    def _boot_mode(self) -> tuple[int, int]:
        p = self.p
        if p.sub_sampling not in FO.BOOT_MODES:
            raise ValueError(f"unknown sub sampling strategy {p.sub_sampling}")
        rate32 = int(min(max(p.sampling_rate, 0.0), 100.0) / 100.0 * 4294967296.0)
        return FO.BOOT_MODES[p.sub_sampling], min(rate32, 0xFFFFFFFF)

    def _chunks(self, node_idx: np.ndarray, start: np.ndarray, count: np.ndarray, chunk: int):
        """Split segments into <= chunk-row work items: (item node index, item start, item len)."""
        nch = np.maximum(1, -(-count // chunk))
        item_node = np.repeat(node_idx, nch)
        first = np.repeat(np.cumsum(nch) - nch, nch)
        k = np.arange(item_node.size) - first
        seg_start = np.repeat(start, nch)
        seg_cnt = np.repeat(count, nch)
        istart = seg_start + k * chunk
        ilen = np.clip(seg_cnt - k * chunk, 0, chunk)
        return item_node.astype(np.int32), istart.astype(np.int64), ilen.astype(np.int32), nch

    def _mask(self, A: int, F: int, key: torch.Tensor, dev) -> torch.Tensor:
        """Random feature subset per node from its key: the k features with the smallest
        h32(key ^ f * golden) (ties broken by feature index)."""
        p = self.p
        if p.attr_selection in ("all", "notUsedYet") or A == 0:
            return torch.ones((A, F), dtype=torch.uint8, device=dev)
        k = max(1, min(p.random_attr_count, F))
        fk = (torch.arange(F, device=dev, dtype=torch.int64) * 0x9E3779B9) & _M32
        r = _h32(key.view(-1, 1) ^ fk.view(1, -1)) * F + torch.arange(F, device=dev).view(1, -1)
        idx = torch.topk(r, k, dim=1, largest=False).indices
        m = torch.zeros((A, F), dtype=torch.uint8, device=dev)
        m.scatter_(1, idx, 1)
        return m

    # ------------------------------------------------------------------------------------------
    def fit(self, t: Table, space: list | None = None, codes: torch.Tensor | None = None,
            tree_ids: list[int] | None = None, weights: torch.Tensor | None = None) -> list[T.DecisionTree]:
        """``weights``: optional explicit uint8 [T, n] bootstrap multiplicities (tests)."""
        comm = self.comm or get_comm()
        p = self.p
        dev = t.device
        if space is None:
            space = T.build_split_space(self.schema, t, binary=True, max_bins=p.max_bins, comm=comm)
        if codes is None:
            codes = T.encode_for_tree(space, t)
        n = t.n
        F = len(space)
        bins = [fs.n_bins for fs in space]
        offs = list(np.cumsum([0] + bins[:-1]))
        TB = sum(bins) + 1
        C = t.n_classes
        algo = 1 if p.algorithm == "entropy" else 0
        topk = p.top_split_count if p.split_selection == "randomAmongTop" else 1
        tree_ids = list(range(self.n_trees)) if tree_ids is None else tree_ids
        Tn = len(tree_ids)
        if Tn == 0:        # tree-parallel with more ranks than trees
            return []
        bins_d = torch.tensor(bins, dtype=torch.int32, device=dev)
        offs_d = torch.tensor(offs, dtype=torch.int32, device=dev)
        t0 = time.perf_counter()

        # ---- per-tree bootstrap row buffers (one gather) ----------------------------------
        if weights is None:        # fused on-device draw + compaction (one pass per tree tile)
            mode, rate32 = self._boot_mode()
            cb, lb, wb, cnt_t = FO.forest_bootstrap(codes.contiguous(), t.labels.to(dev).contiguous(), n,
                                                    self._boot_keys(tree_ids), t.row_offset, mode, rate32)
            R = int(cnt_t.sum())
        else:
            w = weights.to(dev, torch.uint8)                        # [T, n] explicit multiplicities
            keep = w > 0
            cnt_t = keep.sum(1)
            rows = torch.nonzero(keep.view(-1)).view(-1)            # flat (tree, row) ids, tree-major
            src_row = rows % n
            R = int(rows.numel())
            ldb = max(16, (R + 15) // 16 * 16)    # 8-byte lane loads need a multiple of 8 rows
            cb = torch.empty((F, ldb), dtype=torch.uint8, device=dev)
            cb[:, :R] = codes[:, :n].index_select(1, src_row)
            lb = torch.empty(ldb, dtype=torch.uint8, device=dev)
            lb[:R] = t.labels[:n].to(dev).index_select(0, src_row)
            wb = torch.zeros(ldb, dtype=torch.uint8, device=dev)
            wb[:R] = w.view(-1)[rows]
            del rows, src_row, keep, w
        cb2, lb2, wb2 = torch.empty_like(cb), torch.empty_like(lb), torch.zeros_like(wb)
        cnt_h = cnt_t.cpu().numpy().astype(np.int64)
        starts_h = np.concatenate([[0], np.cumsum(cnt_h)[:-1]]).astype(np.int64)
        chunk = self.chunk or int(max(2048, min(65536, R // 4096 if R else 2048)))

        # ---- node table (host, numpy growing arrays) ---------------------------------------
        cap = 1024
        tbl = {k: np.zeros(cap, dtype=np.int64) for k in ("tree", "depth", "feat", "thr", "left", "right", "parent")}
        tbl["counts"] = np.zeros((cap, C), dtype=np.int64)
        tbl["imp"] = np.zeros(cap, dtype=np.float64)
        for k in ("feat", "thr", "left", "right", "parent"):
            tbl[k][:] = -1
        n_nodes = 0

        def add_nodes(tree, depth, parent, counts):
            nonlocal n_nodes, cap
            m = len(tree)
            while n_nodes + m > cap:
                for k in tbl:
                    a = tbl[k]
                    b = np.zeros((cap * 2,) + a.shape[1:], dtype=a.dtype)
                    if k in ("feat", "thr", "left", "right", "parent"):
                        b[:] = -1
                    b[:cap] = a
                    tbl[k] = b
                cap *= 2
            ids = np.arange(n_nodes, n_nodes + m)
            tbl["tree"][ids], tbl["depth"][ids], tbl["parent"][ids] = tree, depth, parent
            tbl["counts"][ids] = counts
            n_nodes += m
            return ids

        # ---- root histograms ---------------------------------------------------------------
        root_ids = add_nodes(np.arange(Tn), np.zeros(Tn, np.int64), np.full(Tn, -1), np.zeros((Tn, C), np.int64))
        root_key = _h32((np.int64(p.seed) * 1000003 + 7) ^ (np.asarray(tree_ids, np.int64) * 2654435761))
        fr = _Frontier(root_ids, starts_h.copy(), cnt_h.copy(), np.zeros(Tn, np.int64), root_key)
        hist = torch.zeros((Tn, C, TB), dtype=torch.int64, device=dev)
        inode, istart, ilen, _ = self._chunks(np.arange(Tn), fr.start, fr.count, chunk)
        FO.forest_hist(cb, lb, wb, inode, istart, ilen, bins_d, offs_d, bins, TB, C, hist)
        if comm.is_distributed:
            comm.all_reduce(hist)
        level = 0
        n_hist_rows = int(fr.count.sum())
        from ..parallel.comm import maybe_inject_fault
        from ..utils.tracing import TRACER
        while fr.node.size:
            tl = time.perf_counter()
            maybe_inject_fault(level, comm.rank)            # env-driven fault injection per level
            A = fr.node.size
            key_d = torch.as_tensor(fr.key, device=dev)
            fmask = self._mask(A, F, key_d, dev)
            rnd = (_h32(key_d ^ 0x2545F491).double() / 4294967296.0).float()
            with TRACER.range("forest.split", 0.0, float(A) * sum(bins) * C * 8, dev):
                feat, thr, score, imp, left = FO.forest_split(hist, fmask, bins_d, offs_d, bins, algo, topk, rnd)
            tot = hist[:, :, TB - 1]
            pop = tot.sum(1).double()
            depth_d = torch.as_tensor(fr.depth, device=dev)
            stop = ~torch.isfinite(score) | (imp <= 0)
            if p.stopping == "maxDepth":
                stop |= depth_d >= p.max_depth
            elif p.stopping == "minPopulation":
                stop |= pop < p.min_population
            elif p.stopping == "minInfoGain":
                stop |= (imp.double() - score.double()) < p.min_info_gain
            feat_eff = torch.where(stop, torch.full_like(feat, -1), feat).int().contiguous()
            thr = thr.int().contiguous()
            inode, istart, ilen, nch = self._chunks(np.arange(A), fr.start, fr.count, chunk)
            # last level (every child at max depth): children are leaves, rows need no partition
            last = p.stopping == "maxDepth" and bool((fr.depth + 1 >= p.max_depth).all())
            item_left = (torch.zeros(inode.size, dtype=torch.int32) if last
                         else FO.forest_part_count(cb, inode, istart, ilen, feat_eff, thr))
            # ---- the ONE host copy of the level: every per-node result packed as int64 words ----
            parts = [feat_eff.long().view(-1), thr.long().view(-1), left.long().reshape(-1), tot.long().reshape(-1),
                     imp.double().view(torch.int64).view(-1), item_left.to(dev).long().view(-1)]
            sizes = [x.numel() for x in parts]
            flat = torch.cat(parts).cpu().numpy()
            segs = np.split(flat, np.cumsum(sizes)[:-1])
            f_h, t_h = segs[0], segs[1]
            l_h, tot_h = segs[2].reshape(A, C), segs[3].reshape(A, C)
            imp_h = segs[4].view(np.float64)
            il_h = segs[5]
            ids = fr.node
            tbl["counts"][ids] = tot_h
            tbl["imp"][ids] = imp_h
            split = f_h >= 0
            if not split.any():
                break
            # per-node local left / right row counts from the chunk counts
            il_h = il_h.astype(np.int64)
            ends = np.cumsum(nch)
            first = ends - nch
            csum = np.concatenate([[0], np.cumsum(il_h)])
            nleft = csum[ends] - csum[first]
            nright = fr.count - nleft
            sp = np.nonzero(split)[0]
            tbl["feat"][ids[sp]] = f_h[sp]
            tbl["thr"][ids[sp]] = t_h[sp]
            lc = l_h[sp]
            rc = tot_h[sp] - lc
            d1 = fr.depth[sp] + 1
            kids = add_nodes(np.repeat(tbl["tree"][ids[sp]], 2), np.repeat(d1, 2), np.repeat(ids[sp], 2),
                             np.stack([lc, rc], 1).reshape(-1, C))
            lk, rk = kids[0::2], kids[1::2]
            tbl["left"][ids[sp]], tbl["right"][ids[sp]] = lk, rk
            # ---- next frontier: children that can still split -------------------------------
            ch_node = np.stack([lk, rk], 1).reshape(-1)
            ch_start = np.stack([fr.start[sp], fr.start[sp] + nleft[sp]], 1).reshape(-1)
            ch_count = np.stack([nleft[sp], nright[sp]], 1).reshape(-1)
            ch_depth = np.repeat(d1, 2)
            ch_w = np.stack([lc.sum(1), rc.sum(1)], 1).reshape(-1)          # global weighted populations
            ch_pure = (np.stack([lc, rc], 1).reshape(-1, C) > 0).sum(1) <= 1
            go = (ch_w >= 2) & ~ch_pure
            if p.stopping == "maxDepth":
                go &= ch_depth < p.max_depth
            elif p.stopping == "minPopulation":
                go &= ch_w >= p.min_population
            if last:
                go[:] = False
            # partition: only the rows of nodes with a continuing child move (leaf rows are done)
            need = np.zeros(A, dtype=bool)
            need[sp] = go.reshape(-1, 2).any(1)
            if need.any():
                item_right = ilen.astype(np.int64) - il_h
                rsum = np.concatenate([[0], np.cumsum(item_right)])
                owner = inode.astype(np.int64)
                lbase = fr.start[owner] + (csum[:-1] - csum[first[owner]])
                rbase = fr.start[owner] + nleft[owner] + (rsum[:-1] - rsum[first[owner]])
                fs_h = np.where(need, f_h, -1).astype(np.int32)
                feat_sc = torch.from_numpy(fs_h).to(dev) if need.sum() < sp.size else feat_eff
                with TRACER.range("forest.partition", 2.0 * int(fr.count[need].sum()) * (F + 2), 0.0, dev):
                    FO.forest_part_scatter(cb, lb, wb, cb2, lb2, wb2, inode, istart, ilen, lbase, rbase, il_h,
                                           feat_sc, thr)
                cb, cb2, lb, lb2, wb, wb2 = cb2, cb, lb2, lb, wb2, wb
            parent_slot = np.repeat(sp, 2)
            sib = np.arange(ch_node.size) ^ 1
            both = go & go[sib]
            # of a live pair the lighter child is built, the heavier derived (ties: left built)
            lighter = np.where(np.arange(ch_node.size) % 2 == 0, ch_w <= ch_w[sib], ch_w < ch_w[sib])
            build = go & (~both | lighter)
            derive = go & both & ~lighter
            order = np.concatenate([np.nonzero(build)[0], np.nonzero(derive)[0]])
            nb = int(build.sum())
            newA = order.size
            slot_of = np.full(ch_node.size, -1, np.int64)
            slot_of[order] = np.arange(newA)
            hist_new = torch.zeros((newA, C, TB), dtype=torch.int64, device=dev)
            bidx = order[:nb]
            if nb:
                inode2, istart2, ilen2, _ = self._chunks(np.arange(nb), ch_start[bidx], ch_count[bidx], chunk)
                with TRACER.range("forest.hist", float(ch_count[bidx].sum()) * (F + 2), 0.0, dev):
                    FO.forest_hist(cb, lb, wb, inode2, istart2, ilen2, bins_d, offs_d, bins, TB, C, hist_new)
                n_hist_rows += int(ch_count[bidx].sum())
            if comm.is_distributed and newA:
                comm.all_reduce(hist_new)
            if newA > nb:
                didx = order[nb:]
                ps = torch.as_tensor(parent_slot[didx], device=dev)
                ss = torch.as_tensor(slot_of[sib[didx]], device=dev)
                hist_new[nb:] = hist[ps] - hist_new[ss]
            hist = hist_new
            ch_key = _child_keys(fr.key[sp])
            fr = _Frontier(ch_node[order], ch_start[order], ch_count[order], ch_depth[order], ch_key[order])
            level += 1
            self.level_times.append(time.perf_counter() - tl)
        self.stats = {"rows_buffered": R, "levels": level, "nodes": n_nodes, "hist_rows": n_hist_rows,
                      "chunk": chunk, "seconds": time.perf_counter() - t0}
        # thousands of small node objects: keep the cyclic GC from pausing in the middle (a gen-2
        # pass over every live object cost 50-100 ms here, more than the whole device build)
        import gc
        was = gc.isenabled()
        gc.disable()
        try:
            return self._to_trees(tbl, n_nodes, Tn, space, t)
        finally:
            if was:
                gc.enable()

    # ------------------------------------------------------------------------------------------
    def _to_trees(self, tbl, n_nodes, Tn, space, t: Table) -> list[T.DecisionTree]:
        cls = list(t.class_field.cardinality) if t.class_field else ["_"]
        algo = self.p.algorithm
        trees = []
        tree_of = tbl["tree"][:n_nodes]
        cnts = tbl["counts"][:n_nodes].astype(np.float64)
        pops = cnts.sum(1)
        pr_all = cnts / np.maximum(pops, 1.0)[:, None]
        if algo == "entropy":
            with np.errstate(divide="ignore", invalid="ignore"):
                info_all = -np.where(pr_all > 0, pr_all * np.log2(np.where(pr_all > 0, pr_all, 1.0)), 0.0).sum(1)
        else:
            info_all = 1.0 - (pr_all * pr_all).sum(1)
        info_all = np.where(pops > 0, info_all, 0.0)
        # host-side node assembly over plain lists (numpy scalar access per node dominated):
        # predicate strings and segment maps are shared per (feature, threshold)
        par_l = tbl["parent"][:n_nodes].tolist()
        feat_l = tbl["feat"][:n_nodes].tolist()
        thr_l = tbl["thr"][:n_nodes].tolist()
        left_l = tbl["left"][:n_nodes].tolist()
        right_l = tbl["right"][:n_nodes].tolist()
        depth_l = tbl["depth"][:n_nodes].tolist()
        pops_l = pops.astype(np.int64).tolist()
        info_l = info_all.tolist()
        pr_l = pr_all.tolist()
        pred_cache: dict[tuple[int, int], tuple[str, str]] = {}
        seg_cache: dict[tuple[int, int], list[int]] = {}

        def preds_for(f: int, s: int) -> tuple[str, str]:
            key = (f, s)
            if key not in pred_cache:
                fs = space[f]
                o = fs.field.ordinal
                if fs.kind == "num":
                    pv = fs.pred_value(fs.points[s])
                    pred_cache[key] = (f"{o} le {pv}", f"{o} gt {pv}")
                else:
                    card = fs.field.cardinality
                    pred_cache[key] = (f"{o} in {':'.join(card[: s + 1])}", f"{o} in {':'.join(card[s + 1:])}")
            return pred_cache[key]

        order = np.argsort(tree_of[:n_nodes], kind="stable")
        bounds = np.searchsorted(tree_of[:n_nodes][order], np.arange(Tn + 1))
        for ti in range(Tn):
            gids = order[bounds[ti]:bounds[ti + 1]].tolist()
            local = {g: i for i, g in enumerate(gids)}
            nodes: list[T.Node] = []
            preds_of: dict[int, list[str]] = {}
            used_of: dict[int, frozenset] = {}
            for g in gids:
                par = par_l[g]
                if par < 0:
                    preds, used = [], frozenset()
                else:
                    lp, rp = preds_for(feat_l[par], thr_l[par])
                    preds = preds_of[par] + [lp if left_l[par] == g else rp]
                    used = used_of[par] | {feat_l[par]}
                preds_of[g], used_of[g] = preds, used
                f = feat_l[g]
                nd = T.Node(preds, pops_l[g], info_l[g], pr_l[g], depth_l[g], stopped=f < 0, used_attrs=used)
                if f >= 0:
                    thr = thr_l[g]
                    nd.feature, nd.split = f, thr
                    sm = seg_cache.get((f, thr))
                    if sm is None:
                        sm = seg_cache[(f, thr)] = [0 if b <= thr else 1 for b in range(space[f].n_bins)]
                    nd.segmap = sm
                    nd.children = [local[left_l[g]], local[right_l[g]]]
                nodes.append(nd)
            trees.append(T.DecisionTree(nodes, space, cls))
        return trees
