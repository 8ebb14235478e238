"""Deterministic OTTO-shaped synthetic sessions ("otto-synth").

Produces the reference's event schema (``etl/jsonl_to_parquet.py:23-29``:
``session:i32, aid:i32, ts:i32 seconds, type:i8``) in CSR form, plus a writer for the
reference's 100k-sessions-per-file parquet layout (``etl/jsonl_to_parquet.py:59-84``).
Generation is a host C++/OpenMP library (``libottosynth.so``) driven by a counter-based
RNG, so any session range is reproducible independently (rank shards, file slices).
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class _Params(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("n_items", ctypes.c_int64),
        ("len_mu", ctypes.c_double), ("len_sigma", ctypes.c_double),
        ("len_min", ctypes.c_int32), ("len_max", ctypes.c_int32),
        ("p_type", ctypes.c_double * 3),
        ("ts0", ctypes.c_int64), ("ts_span", ctypes.c_int64),
        ("gap_mu", ctypes.c_double), ("gap_sigma", ctypes.c_double),
        ("p_long_gap", ctypes.c_double),
        ("long_gap_min", ctypes.c_int64), ("long_gap_max", ctypes.c_int64),
        ("zipf_offset", ctypes.c_double), ("zipf_exponent", ctypes.c_double),
        ("p_revisit", ctypes.c_double),
        ("p_dup", ctypes.c_double),
    ]


def _lib():
    global _LIB
    if _LIB is None:
        # OTTOSYNTH_SO: another build of synth.cpp (the sanitized one, tests/test_sanitize.py)
        path = os.environ.get("OTTOSYNTH_SO") or os.path.join(_HERE, "libottosynth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build() (make -C csrc)")
        lib = ctypes.CDLL(path)
        P = ctypes.POINTER(_Params)
        lib.otto_synth_default_params.argtypes = [P]
        lib.otto_synth_lengths.argtypes = [P, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        lib.otto_synth_sessions_for_events.argtypes = [P, ctypes.c_int64, ctypes.c_int64,
                                                       ctypes.POINTER(ctypes.c_int64)]
        lib.otto_synth_sessions_for_events.restype = ctypes.c_int64
        lib.otto_synth_fill.argtypes = [P, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 5
        lib.otto_synth_item_rank.argtypes = [P, ctypes.c_void_p]
        lib.otto_synth_embeddings.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_void_p]
        _LIB = lib
    return _LIB


def default_params(seed: int = 0, **overrides) -> _Params:
    p = _Params()
    _lib().otto_synth_default_params(ctypes.byref(p))
    p.seed = seed
    for k, v in overrides.items():
        if k == "p_type":
            for i in range(3):
                p.p_type[i] = v[i]
        else:
            setattr(p, k, v)
    return p


@dataclass
class Events:
    """Session-sorted CSR event table: sessions are contiguous, events in generation order."""
    session_offsets: np.ndarray  # int64[S+1]
    session: np.ndarray          # int32[E]
    aid: np.ndarray              # int32[E]
    ts: np.ndarray               # int32[E]
    type: np.ndarray             # int8[E]
    first_session: int = 0

    @property
    def n_sessions(self) -> int:
        return len(self.session_offsets) - 1

    @property
    def n_events(self) -> int:
        return int(self.session_offsets[-1] - self.session_offsets[0])

    def slice_sessions(self, a: int, b: int) -> "Events":
        o = self.session_offsets
        e0, e1 = int(o[a] - o[0]), int(o[b] - o[0])
        return Events(o[a:b + 1] - o[a], self.session[e0:e1], self.aid[e0:e1], self.ts[e0:e1],
                      self.type[e0:e1], self.first_session + a)

    def to_pandas(self):
        import pandas as pd
        return pd.DataFrame({"session": self.session, "aid": self.aid, "ts": self.ts, "type": self.type})


def session_lengths(n_sessions: int, first_session: int = 0, seed: int = 0, params: _Params | None = None) -> np.ndarray:
    """Event counts of sessions [first_session, first_session + n_sessions) without generating them."""
    p = params if params is not None else default_params(seed)
    lens = np.empty(n_sessions, dtype=np.int32)
    if _lib().otto_synth_lengths(ctypes.byref(p), first_session, n_sessions, lens.ctypes.data) != 0:
        raise RuntimeError("otto_synth_lengths failed")
    return lens


def generate(n_sessions: int, first_session: int = 0, seed: int = 0, params: _Params | None = None) -> Events:
    p = params if params is not None else default_params(seed)
    lib = _lib()
    lens = np.empty(n_sessions, dtype=np.int32)
    if lib.otto_synth_lengths(ctypes.byref(p), first_session, n_sessions, lens.ctypes.data) != 0:
        raise RuntimeError("otto_synth_lengths failed")
    off = np.zeros(n_sessions + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    E = int(off[-1])
    sess = np.empty(E, np.int32)
    aid = np.empty(E, np.int32)
    ts = np.empty(E, np.int32)
    ty = np.empty(E, np.int8)
    rc = lib.otto_synth_fill(ctypes.byref(p), first_session, n_sessions, off.ctypes.data,
                             sess.ctypes.data, aid.ctypes.data, ts.ctypes.data, ty.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"otto_synth_fill failed ({rc})")
    return Events(off, sess, aid, ts, ty, first_session)


def sessions_for_events(target_events: int, first_session: int = 0, seed: int = 0,
                        params: _Params | None = None) -> tuple[int, int]:
    p = params if params is not None else default_params(seed)
    n_ev = ctypes.c_int64(0)
    n = _lib().otto_synth_sessions_for_events(ctypes.byref(p), first_session, target_events,
                                              ctypes.byref(n_ev))
    return int(n), int(n_ev.value)


def generate_events(target_events: int, seed: int = 0) -> Events:
    """Config-2 style input: sessions from 0 until at least ``target_events`` events."""
    n, _ = sessions_for_events(target_events, 0, seed)
    return generate(n, 0, seed)


def item_rank(seed: int = 0, n_items: int = 1855603) -> np.ndarray:
    p = default_params(seed, n_items=n_items)
    r = np.empty(n_items, np.int32)
    _lib().otto_synth_item_rank(ctypes.byref(p), r.ctypes.data)
    return r


def item_words(seed: int = 0, n_items: int = 1855603) -> np.ndarray:
    """Synthetic vocabulary in gensim index_to_key order (frequency-sorted): words[rank] = aid."""
    r = item_rank(seed, n_items)
    words = np.empty(n_items, np.int32)
    words[r] = np.arange(n_items, dtype=np.int32)
    return words


def embeddings(n: int = 1855603, dim: int = 100, seed: int = 1, n_clusters: int = 1000) -> np.ndarray:
    """Config-3 item embeddings (float32 [n, dim]), row i = vocabulary rank i."""
    out = np.empty((n, dim), np.float32)
    if _lib().otto_synth_embeddings(seed, n, dim, n_clusters, out.ctypes.data) != 0:
        raise RuntimeError("otto_synth_embeddings failed")
    return out


SESSIONS_PER_FILE = 100_000  # etl/jsonl_to_parquet.py:59 (chunksize)


def file_session_bounds(n_sessions: int, per_file: int = SESSIONS_PER_FILE) -> np.ndarray:
    """Session index boundaries of the reference's 100k-session files."""
    nf = max(1, math.ceil(n_sessions / per_file))
    b = np.minimum(np.arange(nf + 1, dtype=np.int64) * per_file, n_sessions)
    return b


def write_parquet_files(ev: Events, out_dir: str, per_file: int = SESSIONS_PER_FILE) -> list[str]:
    """Write events as ``{start}_{end}.parquet`` zero-padded to ``len(str(n_lines))`` digits,
    exactly like etl/jsonl_to_parquet.py:81-84 (n_lines = number of sessions)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    os.makedirs(out_dir, exist_ok=True)
    nd = len(str(ev.n_sessions))
    paths = []
    bounds = file_session_bounds(ev.n_sessions, per_file)
    for i in range(len(bounds) - 1):
        part = ev.slice_sessions(int(bounds[i]), int(bounds[i + 1]))
        start = str(i * per_file).zfill(nd)
        end = str(i * per_file + per_file).zfill(nd)
        t = pa.table({"session": part.session, "aid": part.aid, "ts": part.ts, "type": part.type})
        path = os.path.join(out_dir, f"{start}_{end}.parquet")
        pq.write_table(t, path)
        paths.append(path)
    return paths


def read_parquet_events(path: str) -> Events:
    """Read one reference-schema parquet file into CSR form. Rows of a session must be
    contiguous (true for files produced by etl/jsonl_to_parquet.py)."""
    import pyarrow.parquet as pq
    t = pq.read_table(path, columns=["session", "aid", "ts", "type"])
    sess = t.column("session").to_numpy().astype(np.int32, copy=False)
    aid = t.column("aid").to_numpy().astype(np.int32, copy=False)
    ts = t.column("ts").to_numpy().astype(np.int32, copy=False)
    ty = t.column("type").to_numpy().astype(np.int8, copy=False)
    return events_from_columns(sess, aid, ts, ty)


def events_from_columns(sess, aid, ts, ty) -> Events:
    """Build CSR from row columns; rows are stably grouped by session if not contiguous."""
    sess = np.asarray(sess, np.int32)
    if len(sess) and np.any(np.diff(sess) != 0):
        starts = np.flatnonzero(np.diff(sess)) + 1
        seen = sess[np.concatenate([[0], starts])]
        if len(np.unique(seen)) != len(seen):  # a session split into several runs
            order = np.argsort(sess, kind="stable")
            sess, aid, ts, ty = sess[order], np.asarray(aid)[order], np.asarray(ts)[order], np.asarray(ty)[order]
    if len(sess):
        starts = np.concatenate([[0], np.flatnonzero(np.diff(sess)) + 1, [len(sess)]]).astype(np.int64)
    else:
        starts = np.zeros(1, np.int64)
    return Events(starts, sess, np.asarray(aid, np.int32), np.asarray(ts, np.int32),
                  np.asarray(ty, np.int8), int(sess[0]) if len(sess) else 0)


def _mix(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 arrays (counter-based draws for the test split)."""
    x = x.astype(np.uint64)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def split_test_labels(ev: Events, test_days: int = 7, seed: int = 2):
    """Config 5: sessions starting in the last `test_days` days become test
    sessions, truncated at a uniform cut in [1, n-1]; labels follow the OTTO protocol: the next
    click after the cut, and every cart / order after it (unique aids per type).
    Returns (train Events, test Events, labels DataFrame[session, aid, type])."""
    import pandas as pd
    off = ev.session_offsets - ev.session_offsets[0]
    lens = np.diff(off)
    start = ev.ts[off[:-1]]
    t_split = int(start.max()) - test_days * 24 * 3600  # the last week of session starts
    sid = ev.session[off[:-1]].astype(np.int64)
    is_test = (start >= t_split) & (lens >= 2)
    u = (_mix(sid.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed)) >> np.uint64(11)).astype(np.float64)
    u /= float(1 << 53)
    cut = np.where(is_test, 1 + np.floor(u * (lens - 1)).astype(np.int64), lens)  # events kept per session
    pos = np.arange(len(ev.aid)) - np.repeat(off[:-1], lens)
    keep_ev = pos < np.repeat(cut, lens)
    test_ev = np.repeat(is_test, lens)
    tr, te = keep_ev & ~test_ev, keep_ev & test_ev
    lab_ev = ~keep_ev

    def sub(mask, sess_mask):
        l2 = np.where(sess_mask, np.add.reduceat(mask.astype(np.int64), off[:-1]) if len(off) > 1 else 0, 0)
        l2 = l2[sess_mask]
        o = np.zeros(len(l2) + 1, np.int64)
        np.cumsum(l2, out=o[1:])
        return Events(o, ev.session[mask], ev.aid[mask], ev.ts[mask], ev.type[mask])

    train, test = sub(tr, ~is_test), sub(te, is_test)
    ls, la, lt = ev.session[lab_ev], ev.aid[lab_ev], ev.type[lab_ev]
    df = pd.DataFrame({"session": ls, "aid": la, "type": lt.astype(np.int8), "ts": ev.ts[lab_ev]})
    clicks = df[df["type"] == 0].sort_values(["session", "ts"], kind="stable").drop_duplicates("session")
    rest = df[df["type"] > 0].drop_duplicates(["session", "aid", "type"])
    labels = pd.concat([clicks, rest])[["session", "aid", "type"]].sort_values(["session", "type", "aid"])
    return train, test, labels.reset_index(drop=True)
