"""Co-visitation counting on MI355X behind the reference's function signatures.

Mirrors model/count_co_events.py:
  count_co_events(df)                         :60-77  (here: raw events in, fused GPU path)
  count_co_events_all_files(dir_sessions, dir_stats, skip_if_exists=True)   :80-100
  concat_files_w_stats(name, dir_stats, files_stats=None)                   :103-181
plus the fused build used by the benchmark:
  count_co_events_fused(events, file_bounds) -> CovisTable   (count + cross-file merge in one pass)

All compute goes through libottohip.so (include/ottohip.h); there is no CPU path.
"""
from __future__ import annotations

import ctypes
import glob
import os
from pathlib import Path
from typing import Dict

import numpy as np

from . import _lib
from . import config
from .synth import Events


def reference_rules(names=None):
    """config.MAP_NAME_COUNT_TYPE + MAP_MAX_TIME_TO_NEXT as C-ABI rules (config.py:43-49,81-88)."""
    names = list(names or config.CO_EVENTS_TO_COUNT)
    arr = (_lib.Rule * len(names))()
    for i, n in enumerate(names):
        this, nxt = config.MAP_NAME_COUNT_TYPE[n]
        arr[i].this_type = this
        arr[i].next_type_mask = sum(1 << t for t in nxt)
        arr[i].max_abs_dt = config.MAP_MAX_TIME_TO_NEXT[n]
    return names, arr


class DeviceEvents:
    """Events resident in HBM (torch tensors as device buffers) + host file bounds."""

    def __init__(self, offsets, aid, ts, type_, file_bounds, n_sessions, n_events):
        self.offsets, self.aid, self.ts, self.type = offsets, aid, ts, type_
        self.file_bounds = np.ascontiguousarray(file_bounds, dtype=np.int64)
        self.n_sessions, self.n_events = int(n_sessions), int(n_events)

    @staticmethod
    def from_host(ev: Events, file_bounds=None, device=None) -> "DeviceEvents":
        import torch
        _lib.require_gpu()
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        off = np.ascontiguousarray(ev.session_offsets - ev.session_offsets[0], np.int64)
        if file_bounds is None:
            file_bounds = np.array([0, ev.n_sessions], np.int64)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=False)
        return DeviceEvents(t(off), t(ev.aid), t(ev.ts), t(ev.type), file_bounds, ev.n_sessions, ev.n_events)

    @staticmethod
    def from_columns(session, aid, ts, type_, file_rows=None, device=None, ctx=None, stream=None) -> "DeviceEvents":
        """Raw event rows (session, aid, ts, type; numpy or device tensors) -> device CSR built by
        ottohip_events_csr_files (file_rows: rows per file, the reference's 100k-session files;
        None = one file). A file's first row always starts a session."""
        import torch
        _lib.require_gpu()
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        ctx = ctx or _lib.context()
        up = lambda a, dt: (a.to(dev).contiguous() if torch.is_tensor(a) else
                            torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev))
        sess, aid_d, ts_d, ty_d = (up(session, np.int32), up(aid, np.int32), up(ts, np.int32), up(type_, np.int8))
        n = int(sess.numel())
        if not (aid_d.numel() == ts_d.numel() == ty_d.numel() == n):
            raise ValueError("events: columns of different lengths")
        if (sess.dtype, aid_d.dtype, ts_d.dtype, ty_d.dtype) != (torch.int32, torch.int32, torch.int32, torch.int8):
            raise TypeError("events: columns must be session:int32, aid:int32, ts:int32, type:int8")
        file_rows = [n] if file_rows is None else [int(r) for r in file_rows]
        if sum(file_rows) != n:
            raise ValueError("events: file_rows do not add up to the rows")
        off = torch.empty(n + len(file_rows), dtype=torch.int64, device=dev)
        # columns uploaded here are rewritten in place (no copy); a caller's device columns are kept
        owned = not any(torch.is_tensor(x) for x in (aid, ts, type_))
        aid_o, ts_o, ty_o = ((aid_d, ts_d, ty_d) if owned else
                             (torch.empty_like(aid_d), torch.empty_like(ts_d), torch.empty_like(ty_d)))
        starts = np.zeros(len(file_rows) + 1, np.int64)
        starts[1:] = np.cumsum(file_rows)
        bounds = np.zeros(len(file_rows) + 1, np.int64)
        _lib.check(_lib.load().ottohip_events_csr_files(
            ctx.h, _lib.ptr(sess), _lib.ptr(aid_d), _lib.ptr(ts_d), _lib.ptr(ty_d), len(file_rows),
            starts.ctypes.data, _lib.ptr(off), None, _lib.ptr(aid_o), _lib.ptr(ts_o), _lib.ptr(ty_o),
            bounds.ctypes.data, None, _lib.stream_handle(stream)))
        S = int(bounds[-1])
        return DeviceEvents(off[:S + 1].contiguous(), aid_o, ts_o, ty_o, bounds, S, n)

    @staticmethod
    def from_parquet(paths, device=None, ctx=None, stream=None) -> "DeviceEvents":
        """Reference-schema session files (etl/jsonl_to_parquet.py:23-29, one file = one
        file_session_bounds entry, as read at model/count_co_events.py:81,91): columns decoded on
        the host, uploaded raw, grouped into the CSR on the device."""
        import pyarrow.parquet as pq
        paths = [paths] if isinstance(paths, (str, os.PathLike)) else list(paths)
        cols = {k: [] for k in ("session", "aid", "ts", "type")}
        rows = []
        for p in paths:
            t = pq.read_table(p, columns=list(cols))
            rows.append(t.num_rows)
            for k, dt in (("session", np.int32), ("aid", np.int32), ("ts", np.int32), ("type", np.int8)):
                cols[k].append(t.column(k).to_numpy().astype(dt, copy=False))
        cat = {k: (np.concatenate(v) if v else np.zeros(0, np.int8 if k == "type" else np.int32)) for k, v in cols.items()}
        return DeviceEvents.from_columns(cat["session"], cat["aid"], cat["ts"], cat["type"], rows or None,
                                         device, ctx, stream)

    def subset_files(self, f0: int, f1: int) -> "DeviceEvents":
        """Files [f0, f1) as a device view (offsets rebased; event columns are views)."""
        s0, s1 = int(self.file_bounds[f0]), int(self.file_bounds[f1])
        off = self.offsets[s0:s1 + 1]
        e0, e1 = int(off[0].item()), int(off[-1].item())
        return DeviceEvents((off - e0).contiguous(), self.aid[e0:e1], self.ts[e0:e1], self.type[e0:e1],
                            self.file_bounds[f0:f1 + 1] - self.file_bounds[f0], s1 - s0, e1 - e0)

    def subset_file_list(self, files) -> "DeviceEvents":
        """Files `files` (any order, no repeats) as one device event set, one file per entry (columns copied)."""
        import torch
        parts = [self.subset_files(int(f), int(f) + 1) for f in files]
        base, offs, fb = 0, [], [0]
        for v in parts:
            offs.append(v.offsets[:-1] + base)
            base += v.n_events
            fb.append(fb[-1] + v.n_sessions)
        dev = self.offsets.device
        offs.append(torch.tensor([base], dtype=torch.int64, device=dev))
        cat = lambda k: torch.cat([getattr(v, k) for v in parts]) if parts else getattr(self, k)[:0].clone()
        return DeviceEvents(torch.cat(offs).contiguous(), cat("aid"), cat("ts"), cat("type"), np.asarray(fb, np.int64),
                            fb[-1], base)

    def abi(self) -> _lib.Events:
        e = _lib.Events()
        e.session_offsets = _lib.ptr(self.offsets)
        e.n_sessions = self.n_sessions
        e.aid, e.ts, e.type = _lib.ptr(self.aid), _lib.ptr(self.ts), _lib.ptr(self.type)
        e.n_events = self.n_events
        e.file_session_bounds = self.file_bounds.ctypes.data
        e.n_files = len(self.file_bounds) - 1
        return e


class CovisTable:
    """Device-resident result of ottohip_covis_count: per rule (aid, aid_next, count, count_ge2)."""

    def __init__(self, handle, names, ctx):
        self.h = handle
        self.names = list(names)
        self.ctx = ctx

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def free(self):
        if self.h:
            _lib.load().ottohip_table_free(self.h)
            self.h = ctypes.c_void_p()

    def _rule(self, name) -> int:
        return self.names.index(name) if isinstance(name, str) else int(name)

    def stats(self, name) -> dict:
        st = _lib.RuleStats()
        _lib.check(_lib.load().ottohip_table_stats(self.h, self._rule(name), ctypes.byref(st)))
        return {"n_rows": st.n_rows, "n_pairs": st.n_pairs, "file_rows": st.file_rows,
                "file_rows_ge2": st.file_rows_ge2}

    def to_torch(self, name, stream=None):
        import torch
        n = self.stats(name)["n_rows"]
        dev = torch.device("cuda", self.ctx.device)
        a = torch.empty(n, dtype=torch.int32, device=dev)
        b = torch.empty(n, dtype=torch.int32, device=dev)
        c = torch.empty(n, dtype=torch.int32, device=dev)   # u32 bits
        c2 = torch.empty(n, dtype=torch.int32, device=dev)
        _lib.check(_lib.load().ottohip_table_copy(self.h, self._rule(name), _lib.ptr(a), _lib.ptr(b), _lib.ptr(c),
                                                  _lib.ptr(c2), _lib.stream_handle(stream)))
        return a, b, c, c2

    def to_numpy(self, name, sort=True):
        """(aid:int32, aid_next:int32, count:uint32, count_ge2:uint32), sorted by (aid, aid_next)."""
        a, b, c, c2 = (x.cpu().numpy() for x in self.to_torch(name))
        c, c2 = c.view(np.uint32), c2.view(np.uint32)
        if sort:
            o = np.lexsort((b, a))
            a, b, c, c2 = a[o], b[o], c[o], c2[o]
        return a, b, c, c2

    def digest(self, name, stream=None) -> dict:
        """ottohip_table_digest: order-independent checksums of one rule's rows."""
        out = (ctypes.c_uint64 * 5)()
        _lib.check(_lib.load().ottohip_table_digest(self.ctx.h, self.h, self._rule(name), out,
                                                    _lib.stream_handle(stream)))
        return {"d_count": int(out[0]), "d_count_ge2": int(out[1]), "pairs": int(out[2]), "pairs_ge2": int(out[3]),
                "rows": int(out[4])}

    def finalize(self, name, stream=None, max_rows=None, params: dict | None = None):
        """concat_files_w_stats' final step (:131-175) on the device for one rule:
        returns torch (aid, aid_next, count:int32) in (count desc, aid, aid_next) order.
        params overrides ottohip_merge_params fields (click_rule, min_count, max_rows,
        filter_rows, max_rows_groupby); the default is the reference's configuration. Raises
        OttoHipError(ELIMIT) where the reference takes its part-wise branch (:135-166): use
        concat_files_w_stats_fused for that case."""
        import torch
        rname = self.names[self._rule(name)]
        mp = _lib.MergeParams()
        mp.click_rule = 1 if "click_to" in rname else 0
        mp.min_count_in_part = config.MIN_COUNT_IN_PART.get(rname, 1)
        mp.min_count = config.MIN_COUNT_TO_SAVE.get(rname, 1)
        mp.max_rows = config.MAX_CO_EVENT_PAIRS_TO_SAVE_DISK if max_rows is None else int(max_rows)
        mp.filter_rows = config.CLICK_FILTER_ROWS
        mp.max_rows_groupby = config.MAX_ROWS_POLARS_GROUPBY
        for k, v in (params or {}).items():
            setattr(mp, k, int(v))
        n = min(self.stats(name)["n_rows"], mp.max_rows)
        dev = torch.device("cuda", self.ctx.device)
        a = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        b = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        c = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        n_out = ctypes.c_int64(0)
        _lib.check(_lib.load().ottohip_table_finalize(self.ctx.h, self.h, self._rule(name), ctypes.byref(mp),
                                                      _lib.ptr(a), _lib.ptr(b), _lib.ptr(c), ctypes.byref(n_out),
                                                      _lib.stream_handle(stream)))
        k = int(n_out.value)
        return a[:k], b[:k], c[:k]


def _bits_for(n: int) -> int:
    """bits needed to store values in [0, n) (common.h bits_for)."""
    return max(0, int(n - 1).bit_length()) if n > 1 else 0


def max_files_per_call(names=None, n_items: int = config.N_ITEMS_OTTO) -> int:
    """Files one device pass can count: a pair word holds rule-within-type | aid_next | file in 31
    bits (csrc/abi.hip setup_rules), so 2^(31 - rule bits - aid bits) files (512 at 1.86 M items)."""
    names, rules = reference_rules(names)
    per_type = max(sum(1 for r in rules if r.this_type == t) for t in range(3))
    return min(1 << (31 - _bits_for(per_type) - max(1, _bits_for(int(n_items)))), 65535)


class FileCuts:
    """Per-file options of one rule for a count (ottohip_file_opts): `lo` = (file, key) drops the
    rule's pairs of that file with key < key, `hi` = (file, key) those with key >= key (key =
    aid << 32 | aid_next; file = index among the call's files, or global id in the sharded calls);
    per_file=True reports every file's rows of the rule (file_rows / file_rows_ge2 per file)."""

    def __init__(self, rule: str, lo=None, hi=None, per_file: bool = False, keep_words: bool = False):
        self.rule, self.lo, self.hi, self.per_file, self.keep_words = rule, lo, hi, per_file, keep_words

    def shifted(self, f0: int, f1: int) -> "FileCuts":
        """The options of the files [f0, f1) renumbered from 0 (a batch of whole files)."""
        mv = lambda c: (c[0] - f0, c[1]) if c is not None and f0 <= c[0] < f1 else None
        return FileCuts(self.rule, mv(self.lo), mv(self.hi), self.per_file, self.keep_words)

    def abi(self, names, n_files: int):
        o = _lib.FileOpts()
        o.rule = list(names).index(self.rule)
        o.lo_file, o.lo_key = (int(self.lo[0]), int(self.lo[1])) if self.lo is not None else (-1, 0)
        o.hi_file, o.hi_key = (int(self.hi[0]), int(self.hi[1])) if self.hi is not None else (-1, 0)
        o.n_files = int(n_files)
        o.keep_words = 1 if self.keep_words else 0
        rows = rows2 = None
        if self.per_file:
            rows, rows2 = np.zeros(max(n_files, 1), np.int64), np.zeros(max(n_files, 1), np.int64)
            o.file_rows, o.file_rows_ge2 = rows.ctypes.data, rows2.ctypes.data
        return o, rows, rows2


def count_co_events_fused(events: DeviceEvents, names=None, n_items: int = config.N_ITEMS_OTTO, dedup: bool = True,
                          stream=None, ctx=None, max_files: int | None = None, cuts: FileCuts | None = None,
                          per_file_rule: str | None = None, keep_words: bool = False) -> CovisTable:
    """All rules over all files of `events` in one device pass (per-file counts folded into
    count / count_ge2): count_co_events_all_files + the groupby of concat_files_w_stats.
    More files than one pass can tell apart (max_files_per_call) are counted in batches of
    whole files and the batch tables merge-summed: count, count_ge2 and the per-file row
    statistics are sums over disjoint file sets. cuts: per-file options of one rule (FileCuts);
    with per_file=True the table carries file_rows_per_file / file_rows_ge2_per_file (numpy).
    per_file_rule: the same per-file row statistics of one rule from this count (the reduce leaves
    histogram every per-file row of the rule), so that concat_files_w_stats_fused's part-wise branch (2)
    needs no count of its own to plan its row slices (model/count_co_events.py:136-153).
    keep_words: the table keeps the count's pair words (one pass of files only), so that branch (2)'s part-tagged
    table is re-folded from them (ottohip_table_count_parts) instead of counted again."""
    ctx = ctx or _lib.context()
    nf = len(events.file_bounds) - 1
    pfr = per_file_rule if per_file_rule in (names or config.CO_EVENTS_TO_COUNT) else None
    # words are kept only by a count of one pass: per-file statistics cap a pass at 1024 files (below)
    keep = keep_words and nf <= min(max_files or max_files_per_call(names, n_items), 1024 if pfr else 1 << 62)
    if cuts is None and (keep or pfr is not None):
        tab = count_co_events_fused(events, names, n_items, dedup, stream, ctx, max_files,
                                    FileCuts(pfr or list(names or config.CO_EVENTS_TO_COUNT)[0], per_file=pfr is not None,
                                             keep_words=keep))
        if pfr is not None:
            tab.per_file_rule = pfr
        tab.kept_words = keep and getattr(tab, "kept_words", False)  # a batched merge keeps none
        return tab
    cap = max_files or max_files_per_call(names, n_items)
    if cuts is not None and cuts.per_file:
        cap = min(cap, 1024)  # the per-file histogram's file range (ottohip_file_opts), as in dist.py
    nf = len(events.file_bounds) - 1
    if nf > cap:
        import torch
        from . import dist as gd
        recs, fs, pf, pf2 = [], None, [], []
        for f0 in range(0, nf, cap):
            f1 = min(nf, f0 + cap)
            t = count_co_events_fused(events.subset_files(f0, f1), names, n_items, dedup, stream, ctx,
                                      max_files=cap, cuts=cuts.shifted(f0, f1) if cuts is not None else None)
            st = [(t.stats(r)["file_rows"], t.stats(r)["file_rows_ge2"]) for r in range(len(t.names))]
            fs = st if fs is None else [(a + c, b + d) for (a, b), (c, d) in zip(fs, st)]
            if cuts is not None and cuts.per_file:
                pf.append(t.file_rows_per_file); pf2.append(t.file_rows_ge2_per_file)
            r, _ = gd.pack_by_owner(t, 1, stream)
            recs.append(r.clone())
            names = t.names
            t.free()
        merged = gd.table_from_records(torch.cat(recs).contiguous(), names, n_items, fs, ctx=ctx, stream=stream)
        if pf:
            merged.file_rows_per_file, merged.file_rows_ge2_per_file = np.concatenate(pf), np.concatenate(pf2)
        return merged
    names, rules = reference_rules(names)
    p = _lib.CovisParams()
    p.min_dt, p.max_dt, p.n_items, p.dedup = config.MIN_TIME_TO_NEXT, config.MAX_TIME_TO_NEXT, int(n_items), int(dedup)
    ev = events.abi()
    h = ctypes.c_void_p()
    lib = _lib.load()
    if cuts is None:
        _lib.check(lib.ottohip_covis_count(ctx.h, ctypes.byref(ev), rules, len(names), ctypes.byref(p),
                                           ctypes.byref(h), _lib.stream_handle(stream)))
        return CovisTable(h, names, ctx)
    o, rows, rows2 = cuts.abi(names, nf)
    _lib.check(lib.ottohip_covis_count_opts(ctx.h, ctypes.byref(ev), rules, len(names), ctypes.byref(p),
                                            ctypes.byref(o), ctypes.byref(h), _lib.stream_handle(stream)))
    tab = CovisTable(h, names, ctx)
    if cuts.per_file:
        tab.file_rows_per_file, tab.file_rows_ge2_per_file = rows[:nf], rows2[:nf]
    tab.kept_words = bool(cuts.keep_words)
    return tab


def part_plan(file_rows, n_parts: int):
    """Row slices of concat_files_w_stats' branch (2) (model/count_co_events.py:136-153) over the
    per-file row counts of the concatenation: part i = rows [i * rows_part, (i + 1) * rows_part),
    rows_part = ceil(N / n_parts). Returns [(fa, lo, fb, hi)]: the part starts at row lo of file fa
    and ends before row hi of file fb (fa <= fb; files strictly between are whole)."""
    import math
    R = np.asarray(file_rows, np.int64)
    N = int(R.sum())
    C = np.concatenate([[0], np.cumsum(R)])
    rows_part = math.ceil(N / n_parts) if n_parts else 0
    plan = []
    for i in range(n_parts):
        g0, g1 = i * rows_part, min((i + 1) * rows_part, N)
        if g1 <= g0:
            continue
        fa = int(np.searchsorted(C, g0, side="right")) - 1
        fb = int(np.searchsorted(C, g1 - 1, side="right")) - 1
        plan.append((fa, int(g0 - C[fa]), fb, int(g1 - C[fb])))
    return plan


def part_assignment(plan, file_rows, keys):
    """Per-file part map of one ottohip_covis_count_parts call for the row slices `plan`: the first part
    of every file and the cuts (file, key): a pair of file f with key >= key belongs to the next part.
    None when some file holds two cuts (a file longer than a part) or the map does not fit the call."""
    nf = len(file_rows)
    first = np.full(nf, -1, np.int64)
    cuts = {}
    for p, (fa, lo, fb, hi) in enumerate(plan):
        for f in range(fa, fb + 1):
            if first[f] < 0:
                first[f] = p
        if hi < int(file_rows[fb]):
            if fb in cuts:
                return None
            cuts[fb] = int(keys[(fb, hi)])
    # files without rows between parts: any part (they hold no row of the sliced column)
    last = 0
    for f in range(nf):
        if first[f] < 0:
            first[f] = last
        last = first[f]
    if len(plan) > 254 or len(cuts) > 64 or nf > 1024:
        return None
    return first.astype(np.int32), sorted(cuts.items())


def count_co_events_parts(events: DeviceEvents, name: str, first_part, cuts, n_parts: int,
                          n_items: int = config.N_ITEMS_OTTO, dedup: bool = True, stream=None, ctx=None) -> CovisTable:
    """ottohip_covis_count_parts: one count of rule `name` whose rows are (part, aid, aid_next), every
    pair in the part of its file (first_part[f], or the next part from the file's cut key on). The
    returned table's rule index is the part (names = [name] * n_parts)."""
    ctx = ctx or _lib.context()
    names, rules = reference_rules([name])
    p = _lib.CovisParams()
    p.min_dt, p.max_dt, p.n_items, p.dedup = config.MIN_TIME_TO_NEXT, config.MAX_TIME_TO_NEXT, int(n_items), int(dedup)
    fp = np.ascontiguousarray(first_part, np.int32)
    cf = np.ascontiguousarray([f for f, _ in cuts] or [0], np.int32)
    ck = np.ascontiguousarray([k for _, k in cuts] or [0], np.uint64)
    po = _lib.PartOpts()
    po.n_files, po.n_parts, po.first_part = len(fp), int(n_parts), fp.ctypes.data
    po.n_cuts, po.cut_file, po.cut_key = len(cuts), cf.ctypes.data, ck.ctypes.data
    ev = events.abi()
    h = ctypes.c_void_p()
    _lib.check(_lib.load().ottohip_covis_count_parts(ctx.h, ctypes.byref(ev), rules, 1, ctypes.byref(p), ctypes.byref(po),
                                                     ctypes.byref(h), _lib.stream_handle(stream)))
    return CovisTable(h, [name] * int(n_parts), ctx)


def table_count_parts(table: CovisTable, name: str, first_part, cuts, n_parts: int, stream=None) -> CovisTable:
    """ottohip_table_count_parts: count_co_events_parts re-folded from the words `table` kept (its count's files and
    file ids): rows (part, aid, aid_next) of rule `name`, a symmetric rule's mirrors as explicit rows."""
    fp = np.ascontiguousarray(first_part, np.int32)
    cf = np.ascontiguousarray([f for f, _ in cuts] or [0], np.int32)
    ck = np.ascontiguousarray([k for _, k in cuts] or [0], np.uint64)
    po = _lib.PartOpts()
    po.n_files, po.n_parts, po.first_part = len(fp), int(n_parts), fp.ctypes.data
    po.n_cuts, po.cut_file, po.cut_key = len(cuts), cf.ctypes.data, ck.ctypes.data
    h = ctypes.c_void_p()
    _lib.check(_lib.load().ottohip_table_count_parts(table.ctx.h, table.h, table._rule(name), ctypes.byref(po),
                                                     ctypes.byref(h), _lib.stream_handle(stream)))
    return CovisTable(h, [name] * int(n_parts), table.ctx)


def part_heads(table: CovisTable, n_parts: int, use_ge2: bool, min_count: int, max_rows_part: int, stream=None):
    """ottohip_table_part_heads: the head(max_rows_part) of every part of a count_co_events_parts table as
    int32 records [m, 4] (aid, aid_next, count, 0), or None where the device selection does not apply (a
    part's cut count >= 65535): the caller then finalizes part by part."""
    import torch
    cap = max(1, int(n_parts) * int(max_rows_part))
    rec = torch.empty((cap, 4), dtype=torch.int32, device=torch.device("cuda", table.ctx.device))
    n = ctypes.c_int64(0)
    rc = _lib.load().ottohip_table_part_heads(table.ctx.h, table.h, int(n_parts), 1 if use_ge2 else 0, int(min_count),
                                              int(max_rows_part), _lib.ptr(rec), cap, ctypes.byref(n),
                                              _lib.stream_handle(stream))
    if rc == _lib.OTTOHIP_ELIMIT:
        return None
    _lib.check(rc)
    return rec[:int(n.value)]


def table_keys_at(table: CovisTable, name, use_ge2: bool, idx, stream=None) -> np.ndarray:
    """ottohip_table_keys_at: keys (aid << 32 | aid_next) of rows idx of one rule's rows in (aid,
    aid_next) order (use_ge2: rows with count >= 2 only)."""
    idx = np.ascontiguousarray(idx, np.int64)
    keys = np.zeros(max(len(idx), 1), np.uint64)
    _lib.check(_lib.load().ottohip_table_keys_at(table.ctx.h, table.h, table._rule(name), 1 if use_ge2 else 0,
                                                 idx.ctypes.data, len(idx), keys.ctypes.data,
                                                 _lib.stream_handle(stream)))
    return keys[:len(idx)]


def table_keys_at_parts(table: CovisTable, use_ge2: bool, idx_per_part, stream=None) -> list:
    """ottohip_table_keys_at_parts: for parts 0 .. len(idx_per_part) - 1 of a part-mode table, the keys (aid << 32 |
    aid_next) of rows idx_per_part[p] of part p's rows in (aid, aid_next) order, all parts in one pass."""
    n_idx = np.ascontiguousarray([len(r) for r in idx_per_part], np.int32)
    idx = np.ascontiguousarray(np.concatenate([np.asarray(r, np.int64).reshape(-1) for r in idx_per_part] +
                                              [np.zeros(0, np.int64)]), np.int64)
    keys = np.zeros(max(len(idx), 1), np.uint64)
    _lib.check(_lib.load().ottohip_table_keys_at_parts(table.ctx.h, table.h, len(idx_per_part), 1 if use_ge2 else 0,
                                                       idx.ctypes.data, n_idx.ctypes.data, keys.ctypes.data,
                                                       _lib.stream_handle(stream)))
    return np.split(keys[:len(idx)], np.cumsum(n_idx)[:-1])


def boundary_keys(events: DeviceEvents, name: str, plan, file_rows, use_ge2: bool, n_items: int, ctx=None) -> dict:
    """{(file, row): key} for every part boundary of `plan` that falls inside a file: the key of that row of
    the file's own (aid, aid_next)-ordered (use_ge2: count >= 2) table, as count_co_events.py:94 writes it.
    The boundary files are counted together, one part per file (ottohip_covis_count_parts: rows carry
    their file's part), where the part machinery applies (n_items < 2^24, < 255 files); else each file
    alone."""
    need = {}
    for fa, lo, fb, hi in plan:
        if lo > 0:
            need.setdefault(fa, set()).add(lo)
        if hi < int(file_rows[fb]):
            need.setdefault(fb, set()).add(hi)
    out = {}
    files = sorted(need)
    # the part machinery: aid_next < 2^24, < 255 parts, and the call's files within a pair word's file bits
    if files and n_items <= (1 << 24) and len(files) <= min(254, max_files_per_call([name], n_items)):
        sub = events.subset_file_list(files)
        try:
            t = count_co_events_parts(sub, name, np.arange(len(files), dtype=np.int32), [], len(files), n_items,
                                      ctx=ctx)
        except _lib.OttoHipError as e:
            if e.rc != _lib.OTTOHIP_ELIMIT:
                raise
            t = None  # a layout limit of the one-count form: each file alone below
        if t is not None:
            # every boundary file's keys from one pass over the table (ottohip_table_keys_at_parts)
            rows_of = [sorted(need[f]) for f in files]
            for f, rows, keys in zip(files, rows_of, table_keys_at_parts(t, use_ge2, rows_of)):
                for r, k in zip(rows, keys.tolist()):
                    out[(f, r)] = int(k)
            t.free()
            return out
    for f, rows in sorted(need.items()):
        rows = sorted(rows)
        t = count_co_events_fused(events.subset_files(f, f + 1), [name], n_items=n_items, ctx=ctx)
        for r, k in zip(rows, table_keys_at(t, name, use_ge2, rows)):
            out[(f, r)] = int(k)
        t.free()
    return out


def a6_refold() -> bool:
    """OTTOHIP_A6_REFOLD=1: branch (2)'s part table re-folded from the count's kept words (ottohip_table_count_parts)
    instead of a part-tagged recount. Exact (tests/test_covis_gpu.py::test_part_branch_from_kept_words) but measured
    slower at 220 M events (A6 193.6 vs 141.8 ms, gpurun_out/r5e): a symmetric rule's mirrors become explicit rows
    outside aid order, so the part heads' tie cut and the merge of the heads lose their ordered fast paths."""
    return os.environ.get("OTTOHIP_A6_REFOLD", "0") == "1"


def concat_files_w_stats_fused(events: DeviceEvents, name: str, table: CovisTable | None = None,
                               n_items: int = config.N_ITEMS_OTTO, max_rows_groupby: int = config.MAX_ROWS_POLARS_GROUPBY,
                               optim_rows: int = config.OPTIM_ROWS_POLARS_GROUPBY,
                               max_pairs: int = config.MAX_CO_EVENT_PAIRS_TO_SAVE_DISK,
                               click_filter_rows: int = config.CLICK_FILTER_ROWS, ctx=None, timings: dict | None = None,
                               one_count: bool = True):
    """model/count_co_events.py:103-181 for one rule over the files of `events`, all branches:
    (1) per-file count >= 2 for click_to_* tables when N > 1e8 (count_ge2), (2) when still
    N > max_rows_groupby, part-wise groupby -> keep count >= MIN_COUNT_IN_PART -> count desc
    -> head(int(max_rows_groupby / N * optim_rows)) per part, (3) groupby, MIN_COUNT_TO_SAVE,
    count desc, head(max_pairs). Branch (2) slices rows as the reference does (:136-153):
    ceil(N / n_parts) consecutive rows of the files' concatenated per-file tables, each file's
    table in (aid, aid_next) order (polars leaves it unspecified). One pass
    gives every file's row count; a part is the count of its files with the boundary files cut
    to the key range of their row slice; with one_count (default) all parts come from ONE count whose
    rows carry their part (ottohip_covis_count_parts), else one count per part (FileCuts). Returns torch
    (aid, aid_next, count:int32) in (count desc, aid, aid_next) order. timings: per-stage seconds are added to this dict
    (device-synchronised; a profiling aid)."""
    import math
    import time
    import torch
    from . import dist as gd
    ctx = ctx or _lib.context()
    t_last = [time.perf_counter()]

    def mark(stage):
        if timings is not None:
            torch.cuda.synchronize()
            t = time.perf_counter()
            timings[stage] = timings.get(stage, 0.0) + t - t_last[0]
            t_last[0] = t
    own = table is None
    tab = table if table is not None else count_co_events_fused(events, [name], n_items=n_items, ctx=ctx,
                                                                per_file_rule=name, keep_words=a6_refold())
    st = tab.stats(name)
    use_ge2 = "click_to" in name and st["file_rows"] > click_filter_rows
    N = st["file_rows_ge2"] if use_ge2 else st["file_rows"]
    base = {"filter_rows": click_filter_rows, "max_rows_groupby": max_rows_groupby}
    if N <= max_rows_groupby:
        out = tab.finalize(name, max_rows=max_pairs, params=base)
        if own:
            tab.free()
        return out
    if own and not getattr(tab, "kept_words", False):
        tab.free()
    n_parts = math.ceil(N / optim_rows)
    max_rows_part = int(max_rows_groupby / N * optim_rows)
    mark("prelude")
    if getattr(tab, "per_file_rule", None) == name:  # the table's own count histogrammed every file's rows
        R = tab.file_rows_ge2_per_file if use_ge2 else tab.file_rows_per_file
    else:
        t = count_co_events_fused(events, [name], n_items=n_items, ctx=ctx, cuts=FileCuts(name, per_file=True))
        R = t.file_rows_ge2_per_file if use_ge2 else t.file_rows_per_file
        t.free()
    if int(R.sum()) != N:
        raise RuntimeError(f"{name}: per-file rows sum to {int(R.sum())}, the table's N is {N}")
    mark("file_rows")
    plan = part_plan(R, n_parts)
    keys = boundary_keys(events, name, plan, R, use_ge2, n_items, ctx)
    mark("boundary_keys")
    part = {"click_rule": 1 if use_ge2 else 0, "filter_rows": -1, "max_rows_groupby": 1 << 62,
            "min_count": config.MIN_COUNT_IN_PART.get(name, 1)}
    recs = []
    nf = len(events.file_bounds) - 1
    fits = one_count and n_items <= (1 << 24) and nf <= max_files_per_call([name], n_items)
    assign = part_assignment(plan, R, keys) if fits else None
    if assign is not None:  # every part from ONE count (its rows carry their part)
        refold = a6_refold()
        if refold and getattr(tab, "kept_words", False) and tab.h:  # re-folded from the words of the table's own count
            t = table_count_parts(tab, name, assign[0], assign[1], len(plan))
        else:
            t = count_co_events_parts(events, name, assign[0], assign[1], len(plan), n_items, ctx=ctx)
        if own:
            tab.free()
        mark("part_count")
        heads = part_heads(t, len(plan), use_ge2, part["min_count"], max_rows_part) if len(plan) <= 32 else None
        if heads is not None:  # every part's head at once (histogram cuts, no per-part sort)
            recs.append(heads)
        else:
            for p_ in range(len(plan)):
                a, b, c = t.finalize(p_, max_rows=max_rows_part, params=part)
                recs.append(torch.stack([a, b, c, torch.zeros_like(c)], 1))
        t.free()
        mark("part_finalize")
        plan = []
    if own:
        tab.free()
    for fa, lo, fb, hi in plan:
        cuts = FileCuts(name, lo=(0, keys[(fa, lo)]) if lo > 0 else None,
                        hi=(fb - fa, keys[(fb, hi)]) if hi < int(R[fb]) else None)
        t = count_co_events_fused(events.subset_files(fa, fb + 1), [name], n_items=n_items, ctx=ctx, cuts=cuts)
        mark("part_count")
        a, b, c = t.finalize(name, max_rows=max_rows_part, params=part)
        recs.append(torch.stack([a, b, c, torch.zeros_like(c)], 1))
        t.free()
        mark("part_finalize")
    # one part-heads tensor (the one-count path) is merged in place: torch.cat would copy its ~5 GB
    r = (recs[0] if len(recs) == 1 else torch.cat(recs)) if recs else torch.zeros((0, 4), dtype=torch.int32,
                                                                                 device=events.aid.device)
    merged = gd.table_from_records(r.contiguous(), [name], n_items, ctx=ctx)
    mark("merge_parts")
    out = merged.finalize(name, max_rows=max_pairs,
                          params={"click_rule": 0, "filter_rows": -1, "max_rows_groupby": 1 << 62,
                                  "min_count": config.MIN_COUNT_TO_SAVE.get(name, 1)})
    merged.free()
    mark("final")
    return out


def _merge_params(name: str, max_pairs: int, click_filter_rows: int, max_rows_groupby: int) -> "_lib.MergeParams":
    mp = _lib.MergeParams()
    mp.click_rule = 1 if "click_to" in name else 0
    mp.min_count_in_part = config.MIN_COUNT_IN_PART.get(name, 1)
    mp.min_count = config.MIN_COUNT_TO_SAVE.get(name, 1)
    mp.max_rows = int(max_pairs)
    mp.filter_rows = int(click_filter_rows)
    mp.max_rows_groupby = int(max_rows_groupby)
    return mp


def concat_tables_w_stats(name: str, tables, n_items: int = config.N_ITEMS_OTTO,
                          max_rows_groupby: int = config.MAX_ROWS_POLARS_GROUPBY,
                          optim_rows: int = config.OPTIM_ROWS_POLARS_GROUPBY,
                          max_pairs: int = config.MAX_CO_EVENT_PAIRS_TO_SAVE_DISK,
                          click_filter_rows: int = config.CLICK_FILTER_ROWS, loaded_from_cache: bool = False,
                          stream=None, ctx=None):
    """model/count_co_events.py:103-181 on finished tables [(aid, aid_next, count) device int32
    tensors, ...] concatenated in the given order (ottohip_concat_tables): the per-file tables of
    a folder, or -- the train+test merge of :218-226 (A7) -- the two thresholded folder tables.
    Branch (2) slices rows of the concatenation as the reference does (:146-155). Returns torch
    (aid, aid_next, count:int32) in (count desc, aid, aid_next) order."""
    import torch
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    cols = [tuple(torch.as_tensor(x, dtype=torch.int32).to(dev).contiguous() for x in t) for t in tables]
    nt = len(cols)
    n = [int(t[0].numel()) for t in cols]
    for t in cols:
        if not (t[0].numel() == t[1].numel() == t[2].numel()):
            raise ValueError("concat_tables_w_stats: ragged table columns")
    P = ctypes.c_void_p * max(nt, 1)
    pa, pb, pc = P(*[_lib.ptr(t[0]) for t in cols]), P(*[_lib.ptr(t[1]) for t in cols]), P(*[_lib.ptr(t[2]) for t in cols])
    nr = (ctypes.c_int64 * max(nt, 1))(*n)
    mp = _merge_params(name, max_pairs, click_filter_rows, max_rows_groupby)
    cap = max(1, min(sum(n), int(max_pairs)))
    a = torch.empty(cap, dtype=torch.int32, device=dev)
    b = torch.empty(cap, dtype=torch.int32, device=dev)
    c = torch.empty(cap, dtype=torch.int32, device=dev)
    n_out = ctypes.c_int64(0)
    _lib.check(_lib.load().ottohip_concat_tables(ctx.h, nt, pa, pb, pc, nr, int(n_items), ctypes.byref(mp),
                                                 int(optim_rows), 1 if loaded_from_cache else 0, _lib.ptr(a),
                                                 _lib.ptr(b), _lib.ptr(c), ctypes.byref(n_out),
                                                 _lib.stream_handle(stream)))
    k = int(n_out.value)
    return a[:k], b[:k], c[:k]


def merge_train_test(name: str, train, test, n_items: int = config.N_ITEMS_OTTO, ctx=None, **kw):
    """A7 (model/count_co_events.py:218-226): concat_files_w_stats on the two thresholded folder
    tables [train, test] (each the output of A6 over its own folder's files)."""
    return concat_tables_w_stats(name, [train, test], n_items=n_items, ctx=ctx, **kw)


def _n_items_for_device(aid) -> int:
    return max(config.N_ITEMS_OTTO, int(aid.max().item()) + 1 if aid.numel() else 1)


def count_co_events(df, names=None) -> Dict[str, "object"]:
    """model/count_co_events.py:60 on RAW events (session, aid, ts, type): unique + self-join +
    time filter + per-rule groupby count, fused on the GPU without materialising the join.
    Returns {name: pandas.DataFrame[aid:int32, aid_next:int32, count:uint32]} (row order unspecified,
    as in the reference). A pre-joined frame (with 'aid_next') is rejected: the device path
    never builds the Cartesian product."""
    import pandas as pd
    if "aid_next" in df.columns:
        raise ValueError("count_co_events() takes raw events; the joined frame of self_merge() is not materialised "
                         "on the device path")
    dev = DeviceEvents.from_columns(df["session"].to_numpy(), df["aid"].to_numpy(), df["ts"].to_numpy(),
                                    df["type"].to_numpy())
    tab = count_co_events_fused(dev, names, n_items=_n_items_for_device(dev.aid))
    out = {}
    for n in tab.names:
        a, b, c, _ = tab.to_numpy(n, sort=False)
        out[n] = pd.DataFrame({"aid": a, "aid_next": b, "count": c.astype(np.uint32)})
    return out


def _write_table(path, aid, aid_next, count, count_dtype):
    import pyarrow as pa
    import pyarrow.parquet as pq
    os.makedirs(os.path.dirname(path), exist_ok=True)
    pq.write_table(pa.table({"aid": np.asarray(aid, np.int32), "aid_next": np.asarray(aid_next, np.int32),
                             "count": np.asarray(count).astype(count_dtype)}), path)


def count_co_events_all_files(dir_sessions, dir_stats, skip_if_exists=True):
    """model/count_co_events.py:80-100: per parquet file of sessions, the 5 count tables
    written to {dir_stats}/{name}/{stem}.parquet as (aid:int32, aid_next:int32, count:uint32)."""
    files = sorted(glob.glob(f"{dir_sessions}/*.parquet"))
    for f in files:
        stem = Path(f).stem
        outs = {n: f"{dir_stats}/{n}/{stem}.parquet" for n in config.CO_EVENTS_TO_COUNT}
        if skip_if_exists and all(os.path.exists(p) for p in outs.values()):
            continue
        dev = DeviceEvents.from_parquet(f)
        tab = count_co_events_fused(dev, n_items=_n_items_for_device(dev.aid))
        for n, p in outs.items():
            a, b, c, _ = tab.to_numpy(n, sort=False)
            _write_table(p, a, b, c, np.uint32)
        tab.free()


def _read_table(path):
    import pyarrow.parquet as pq
    t = pq.read_table(path, columns=["aid", "aid_next", "count"])
    return tuple(np.ascontiguousarray(t.column(k).to_numpy().astype(dt, copy=False))
                 for k, dt in (("aid", np.int32), ("aid_next", np.int32), ("count", np.uint32)))


def _part_heads(name, tabs, n_items, max_rows_groupby, optim_rows, ctx=None):
    """Branch (2) of :135-166 on host tables (already through the :131-132 filter): per row slice of
    the concatenation, groupby-sum (device merge of records), count >= MIN_COUNT_IN_PART, count desc,
    head(int(max_rows_groupby / N * optim_rows)); returns the concatenation of the part heads (host)."""
    import math
    import torch
    from . import dist as gd
    ctx = ctx or _lib.context()
    cat = [np.concatenate([t[i] for t in tabs]) for i in range(3)]
    N = len(cat[0])
    n_parts = math.ceil(N / optim_rows)
    max_rows_part = int(max_rows_groupby / N * optim_rows)
    rows_part = math.ceil(N / n_parts)
    dev = torch.device("cuda", ctx.device)
    out = []
    for i in range(n_parts):
        sl = slice(i * rows_part, (i + 1) * rows_part)
        rec = torch.from_numpy(np.stack([cat[0][sl].astype(np.int32), cat[1][sl].astype(np.int32),
                                         cat[2][sl].view(np.int32), np.zeros(len(cat[0][sl]), np.int32)], 1)).to(dev)
        t = gd.table_from_records(rec.contiguous(), [name], n_items, ctx=ctx)
        a, b, c = t.finalize(name, max_rows=max_rows_part,
                             params={"click_rule": 0, "filter_rows": -1, "max_rows_groupby": 1 << 62,
                                     "min_count": config.MIN_COUNT_IN_PART.get(name, 1)})
        out.append((a.cpu().numpy(), b.cpu().numpy(), c.cpu().numpy().view(np.uint32)))
        t.free()
    return tuple(np.concatenate([o[i] for o in out]) if out else np.zeros(0, np.int32) for i in range(3))


def concat_files_w_stats(name, dir_stats, files_stats=None, n_items: int | None = None,
                         max_rows_groupby: int = config.MAX_ROWS_POLARS_GROUPBY,
                         optim_rows: int = config.OPTIM_ROWS_POLARS_GROUPBY,
                         click_filter_rows: int = config.CLICK_FILTER_ROWS, **kw):
    """model/count_co_events.py:103-181 with the reference's signature and files: reads
    {dir_stats}/tmp/{name}.parquet if present (loaded_from_cache, :106-110), else the tables listed
    in files_stats (:111-112), else every {dir_stats}/{name}/*.parquet in sorted order (:113-114);
    runs A6 on the device and writes {dir_stats}/{name}.parquet [aid:int32, aid_next:int32,
    count:int32] in count-desc order (:179). When the part-wise branch (2) runs, the concatenated
    part heads are written to {dir_stats}/tmp/{name}.parquet first (:164-166), as the reference does,
    so a second call takes the loaded_from_cache path on the same file."""
    import torch
    file_tmp = f"{dir_stats}/tmp/{name}.parquet"
    cached = os.path.exists(file_tmp)
    if cached:
        paths = [file_tmp]
    elif files_stats is not None:
        paths = list(files_stats)
    else:
        paths = sorted(glob.glob(f"{dir_stats}/{name}/*.parquet"))
    tabs = [_read_table(p) for p in paths]
    if n_items is None:
        n_items = max([config.N_ITEMS_OTTO] + [int(max(t[0].max(), t[1].max())) + 1 for t in tabs if len(t[0])])
    if any(len(t[2]) and int(t[2].max()) > 0x7FFFFFFF for t in tabs):
        raise ValueError("concat_files_w_stats: a per-file count exceeds int32")
    if not cached:
        n_rows = sum(len(t[0]) for t in tabs)
        if "click_to" in name and n_rows > click_filter_rows:  # :131-132, then :135's test on the filtered rows
            thr = config.MIN_COUNT_IN_PART.get(name, 1)
            tabs_f = [tuple(x[t[2] >= thr] for x in t) for t in tabs]
        else:
            tabs_f = tabs
        if sum(len(t[0]) for t in tabs_f) > max_rows_groupby:  # :135-166, the parts written to tmp (:164-166)
            parts = _part_heads(name, tabs_f, n_items, max_rows_groupby, optim_rows)
            os.makedirs(f"{dir_stats}/tmp", exist_ok=True)
            _write_table(file_tmp, *parts, np.uint32)
            tabs, cached = [parts], True
    dev_tabs = [tuple(torch.from_numpy(x.view(np.int32) if x.flags.writeable else x.view(np.int32).copy()) for x in t)
                for t in tabs]
    a, b, c = concat_tables_w_stats(name, dev_tabs, n_items=n_items, loaded_from_cache=cached,
                                    max_rows_groupby=max_rows_groupby, optim_rows=optim_rows,
                                    click_filter_rows=click_filter_rows, **kw)
    _write_table(f"{dir_stats}/{name}.parquet", a.cpu().numpy(), b.cpu().numpy(), c.cpu().numpy(), np.int32)


def count_co_events_build(dir_sessions, dir_stats, names=None, **kw):
    """Fused equivalent of `count_co_events_all_files` + `concat_files_w_stats` for one folder:
    reads every session file once, counts all files in one device pass and writes the merged
    tables {dir_stats}/{name}.parquet (aid:int32, aid_next:int32, count:int32), count desc. Every
    branch of :131-175 applies (concat_files_w_stats_fused: the part-wise branch (2) by rows where
    a rule's N exceeds MAX_ROWS_POLARS_GROUPBY, e.g. click_to_click at 220 M events). kw:
    concat_files_w_stats_fused thresholds (max_rows_groupby, optim_rows, max_pairs, click_filter_rows)."""
    files = sorted(glob.glob(f"{dir_sessions}/*.parquet"))
    dev = DeviceEvents.from_parquet(files)
    n_items = _n_items_for_device(dev.aid)
    tab = count_co_events_fused(dev, names, n_items=n_items, per_file_rule="click_to_click")
    for n in tab.names:
        a, b, c = (x.cpu().numpy() for x in concat_files_w_stats_fused(dev, n, table=tab, n_items=n_items, **kw))
        _write_table(f"{dir_stats}/{n}.parquet", a, b, c, np.int32)
    tab.free()
