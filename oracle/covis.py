"""CPU oracle for co-visitation counting and its merge (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline -- never as a product path.

Parity status: UNPINNED against the reference itself (polars is absent, the reference has
no tests). Anchors: the hand-derived known-answer test of SURVEY.md
Appendix A (tests/golden/kat_appendix_a.json) and the op-for-op pandas restatement in
oracle/covis_pandas.py, which follows model/count_co_events.py:17-77 line by line.

Contents
  REFERENCE_RULES           config.py:41-49,81-88 restated
  count_co_events_file()    C restatement (covis_oracle.c) of count_co_events.py:91-94, one file
  concat_files_w_stats()    numpy restatement of count_co_events.py:103-181 (merge semantics A6)
  merge_train_test()        count_co_events.py:209-226 (A6 per folder, then A6 on [train, test]) (A7)
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# OTTO_ORACLE_SO: another build of the same source (the sanitized one, tests/test_sanitize.py)
_SO = os.environ.get("OTTO_ORACLE_SO") or os.path.join(_HERE, "_build", "libcovis_oracle.so")

# config.py:41-42
MIN_TIME_TO_NEXT = -24 * 60 * 60
MAX_TIME_TO_NEXT = 24 * 60 * 60
# config.py:43-49 and 81-88: name -> (this type, next types, max |dt|)
REFERENCE_RULES = {
    "click_to_click": (0, (0,), 12 * 60 * 60),
    "click_to_cart_or_buy": (0, (1, 2), MAX_TIME_TO_NEXT),
    "cart_to_cart": (1, (1,), MAX_TIME_TO_NEXT),
    "cart_to_buy": (1, (2,), MAX_TIME_TO_NEXT),
    "buy_to_buy": (2, (2,), MAX_TIME_TO_NEXT),
}
# config.py:52-64
OPTIM_ROWS_POLARS_GROUPBY = 100_000_000
MAX_ROWS_POLARS_GROUPBY = 300_000_000
MIN_COUNT_TO_SAVE = {"click_to_click": 10, "click_to_cart_or_buy": 5, "cart_to_cart": 2,
                     "cart_to_buy": 2, "buy_to_buy": 2}
MIN_COUNT_IN_PART = {"click_to_click": 2, "click_to_cart_or_buy": 2}
MAX_CO_EVENT_PAIRS_TO_SAVE_DISK = 300_000_000


class _Table(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("aid", ctypes.c_void_p), ("aid_next", ctypes.c_void_p),
                ("count", ctypes.c_void_p)]


_LIB = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def _lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_SO):
            build()
        lib = ctypes.CDLL(_SO)
        lib.oracle_count_co_events.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [
            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
            ctypes.c_int32, ctypes.POINTER(_Table)]
        lib.oracle_free_table.argtypes = [ctypes.POINTER(_Table)]
        _LIB = lib
    return _LIB


def _rule_arrays(rules):
    names = list(rules)
    this = np.array([rules[n][0] for n in names], np.int32)
    mask = np.array([sum(1 << t for t in rules[n][1]) for n in names], np.uint32)
    wmax = np.array([rules[n][2] for n in names], np.int32)
    return names, this, mask, wmax


def count_co_events_file(offsets, aid, ts, type_, rules=REFERENCE_RULES,
                         min_dt=MIN_TIME_TO_NEXT, max_dt=MAX_TIME_TO_NEXT) -> dict:
    """One file: dedup -> self-join -> time filter -> per-rule groupby count.
    Returns {name: (aid:int32[], aid_next:int32[], count:uint32[])} sorted by (aid, aid_next)."""
    lib = _lib()
    offsets = np.ascontiguousarray(offsets, np.int64)
    aid = np.ascontiguousarray(aid, np.int32)
    ts = np.ascontiguousarray(ts, np.int32)
    type_ = np.ascontiguousarray(type_, np.int8)
    names, this, mask, wmax = _rule_arrays(rules)
    out = (_Table * len(names))()
    rc = lib.oracle_count_co_events(len(offsets) - 1, offsets.ctypes.data, aid.ctypes.data,
                                    ts.ctypes.data, type_.ctypes.data, len(names), this.ctypes.data,
                                    mask.ctypes.data, wmax.ctypes.data, min_dt, max_dt, out)
    if rc != 0:
        raise RuntimeError(f"oracle_count_co_events failed ({rc})")
    res = {}
    for r, name in enumerate(names):
        n = out[r].n
        if n:
            a = np.ctypeslib.as_array(ctypes.cast(out[r].aid, ctypes.POINTER(ctypes.c_int32)), (n,)).copy()
            b = np.ctypeslib.as_array(ctypes.cast(out[r].aid_next, ctypes.POINTER(ctypes.c_int32)), (n,)).copy()
            c = np.ctypeslib.as_array(ctypes.cast(out[r].count, ctypes.POINTER(ctypes.c_uint32)), (n,)).copy()
        else:
            a = np.zeros(0, np.int32); b = np.zeros(0, np.int32); c = np.zeros(0, np.uint32)
        lib.oracle_free_table(ctypes.byref(out[r]))
        res[name] = (a, b, c)
    return res


def count_co_events_files(offsets, aid, ts, type_, file_bounds, rules=REFERENCE_RULES) -> list:
    """Per-file tables for consecutive session ranges [file_bounds[f], file_bounds[f+1])."""
    offsets = np.asarray(offsets, np.int64)
    res = []
    for f in range(len(file_bounds) - 1):
        s0, s1 = int(file_bounds[f]), int(file_bounds[f + 1])
        e0, e1 = int(offsets[s0] - offsets[0]), int(offsets[s1] - offsets[0])
        res.append(count_co_events_file(offsets[s0:s1 + 1], aid[e0:e1], ts[e0:e1], type_[e0:e1], rules))
    return res


def _groupby_sum(a, b, c):
    key = (a.astype(np.int64) << 32) | b.astype(np.uint32).astype(np.int64)
    order = np.argsort(key, kind="stable")
    key = key[order]
    c = c[order].astype(np.int64)
    if len(key) == 0:
        return a[:0], b[:0], np.zeros(0, np.int64)
    start = np.concatenate([[True], key[1:] != key[:-1]])
    idx = np.flatnonzero(start)
    sums = np.add.reduceat(c, idx)
    k = key[idx]
    return (k >> 32).astype(np.int32), (k & 0xFFFFFFFF).astype(np.int32), sums


def _sort_count_desc(a, b, c):
    """count desc with the build's deterministic tie-break (aid asc, aid_next asc)."""
    order = np.lexsort((b, a, -c))
    return a[order], b[order], c[order]


def concat_files_w_stats(name: str, parts: list, loaded_from_cache: bool = False,
                         max_rows_groupby: int = MAX_ROWS_POLARS_GROUPBY,
                         optim_rows: int = OPTIM_ROWS_POLARS_GROUPBY,
                         max_pairs: int = MAX_CO_EVENT_PAIRS_TO_SAVE_DISK,
                         click_filter_rows: int = 100_000_000):
    """Restates model/count_co_events.py:103-181 on in-memory per-file tables
    [(aid, aid_next, count)...] concatenated in the given order. Branch (2) slices ceil(N/n_parts)
    consecutive rows of that concatenation (:136-153), so the row order inside each table decides
    the slices: the reference's per-file tables come out of polars' groupby in an unspecified order,
    which makes its branch (2) nondeterministic; the build fixes it as (aid, aid_next) ascending
    (count_co_events_file's order) and every sort's ties as (count desc, aid, aid_next).
    Returns (aid:int32, aid_next:int32, count:int32)."""
    nf = len(parts)
    cat = lambda k, dt, sel: (np.concatenate([parts[f][k] for f in sel]).astype(dt) if len(sel)
                              else np.zeros(0, dt))
    a, b, c = cat(0, np.int32, range(nf)), cat(1, np.int32, range(nf)), cat(2, np.int64, range(nf))
    n = len(a)
    # :131-132 lossy per-part filter for click_to tables
    if "click_to" in name and n > click_filter_rows and not loaded_from_cache:
        keep = c >= MIN_COUNT_IN_PART.get(name, 1)
        a, b, c = a[keep], b[keep], c[keep]
        n = len(a)
    # :135-166 groupby by parts
    if n > max_rows_groupby and not loaded_from_cache:
        rows_part = optim_rows
        n_parts = math.ceil(n / rows_part)
        max_rows_part = int(max_rows_groupby / n * rows_part)
        rows_part = math.ceil(n / n_parts)
        sel = [slice(i * rows_part, (i + 1) * rows_part) for i in range(n_parts)]
        pa, pb, pc = [], [], []
        for m in sel:
            sa, sb, sc = _groupby_sum(a[m], b[m], c[m])
            keep = sc >= MIN_COUNT_IN_PART.get(name, 1)
            sa, sb, sc = _sort_count_desc(sa[keep], sb[keep], sc[keep])
            pa.append(sa[:max_rows_part]); pb.append(sb[:max_rows_part]); pc.append(sc[:max_rows_part])
        a, b, c = np.concatenate(pa), np.concatenate(pb), np.concatenate(pc)
    # :168-175
    a, b, c = _groupby_sum(a, b, c)
    keep = c >= MIN_COUNT_TO_SAVE.get(name, 1)
    a, b, c = _sort_count_desc(a[keep], b[keep], c[keep])
    a, b, c = a[:max_pairs], b[:max_pairs], c[:max_pairs]
    return a, b, c.astype(np.int32)


def merge_train_test(name: str, train_parts: list, test_parts: list, **kw):
    """Restates the stage orchestration of model/count_co_events.py:209-226 (A7) for one rule:
    concat_files_w_stats per folder (:214-215), each with its OWN N for the :131 and :135
    triggers and its own MIN_COUNT_TO_SAVE cut, then concat_files_w_stats on the concatenation
    [train table, test table] of the two thresholded folder tables (:218-226). Branch (2) of the
    final merge slices rows of that concatenation, which is deterministic here: both inputs are
    in (count desc, aid, aid_next) order."""
    t = concat_files_w_stats(name, train_parts, **kw)
    s = concat_files_w_stats(name, test_parts, **kw)
    return concat_files_w_stats(name, [t, s], **kw)


def files_digest(offsets, aid, ts, type_, file_bounds, threads: int = 0, rules=REFERENCE_RULES) -> dict:
    """Per rule, the linear checksums of every file's table (oracle_count_files_omp): equal to
    ottohip_table_digest of the cross-file merged table (count / count_ge2) without a merge.
    {name: {d_count, d_count_ge2, pairs, pairs_ge2, file_rows, file_rows_ge2}}."""
    lib = _lib()
    names, this, mask, wmax = _rule_arrays(rules)
    f = lib.oracle_count_files_omp
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 5 + [ctypes.c_int] + [ctypes.c_void_p] * 3 + [
        ctypes.c_int32, ctypes.c_int32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    off = np.ascontiguousarray(offsets, np.int64)
    fb = np.ascontiguousarray(file_bounds, np.int64)
    aid = np.ascontiguousarray(aid, np.int32); ts = np.ascontiguousarray(ts, np.int32)
    type_ = np.ascontiguousarray(type_, np.int8)
    tot = np.zeros(2 * len(names), np.int64)
    dig = np.zeros(6 * len(names), np.uint64)
    rc = f(len(fb) - 1, fb.ctypes.data, off.ctypes.data, aid.ctypes.data, ts.ctypes.data, type_.ctypes.data,
           len(names), this.ctypes.data, mask.ctypes.data, wmax.ctypes.data, MIN_TIME_TO_NEXT, MAX_TIME_TO_NEXT,
           int(threads or os.cpu_count() or 1), tot.ctypes.data, dig.ctypes.data)
    if rc:
        raise RuntimeError(f"oracle_count_files_omp failed ({rc})")
    keys = ["d_count", "d_count_ge2", "pairs", "pairs_ge2", "file_rows", "file_rows_ge2"]
    return {n: {k: int(dig[r * 6 + i]) for i, k in enumerate(keys)} for r, n in enumerate(names)}


def canonical_digest(tables: dict) -> dict:
    """sha256 of the canonical (rule, aid, aid_next, count) stream, plus rows and Σcount."""
    import hashlib
    out = {}
    for name in sorted(tables):
        a, b, c = tables[name]
        order = np.lexsort((np.asarray(b), np.asarray(a)))
        blob = np.stack([np.asarray(a, np.int64)[order], np.asarray(b, np.int64)[order],
                         np.asarray(c, np.int64)[order]], axis=1)
        out[name] = {"rows": int(len(a)), "sum": int(np.asarray(c, np.int64).sum()),
                     "sha256": hashlib.sha256(blob.tobytes()).hexdigest()}
    return out
