"""Candidate retrieval on MI355X behind model/retrieve.py's function signatures.

R1  get_df_count_for_co_event_type(count_type, dir_counts, first_n=None)   model/retrieve.py:18-63
    (device form: topk_per_aid(aid, aid_next, count, first_n) on torch columns)

All compute goes through libottohip.so (ottohip_topk_per_aid); polars is replaced by
pandas/pyarrow at the boundary with the reference's column names and dtypes.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from . import config


def topk_per_aid(aid, aid_next, count, first_n: int, n_items: int = config.N_ITEMS_OTTO, stream=None, ctx=None):
    """R1 on device columns in FILE order (int32 torch tensors). Returns a dict of torch
    columns aid, aid_next, count (int32), count_pop, perc_pop, rank (int16), count_rel (int8)
    in (aid asc, rank asc) order."""
    import torch
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    # (numpy columns read from parquet are read-only: torch wants a writable buffer to wrap)
    w = lambda x: x.copy() if isinstance(x, np.ndarray) and not x.flags.writeable else x
    a = torch.as_tensor(w(aid)).to(dev, torch.int32).contiguous()
    b = torch.as_tensor(w(aid_next)).to(dev, torch.int32).contiguous()
    c = torch.as_tensor(w(count)).to(dev, torch.int32).contiguous()
    n = int(a.numel())
    if not (b.numel() == n == c.numel()):
        raise ValueError("aid, aid_next and count must have the same length")
    cap = max(n, 1)
    out = {"aid": torch.empty(cap, dtype=torch.int32, device=dev),
           "aid_next": torch.empty(cap, dtype=torch.int32, device=dev),
           "count": torch.empty(cap, dtype=torch.int32, device=dev),
           "count_pop": torch.empty(cap, dtype=torch.int16, device=dev),
           "perc_pop": torch.empty(cap, dtype=torch.int16, device=dev),
           "rank": torch.empty(cap, dtype=torch.int16, device=dev),
           "count_rel": torch.empty(cap, dtype=torch.int8, device=dev)}
    n_out = ctypes.c_int64(0)
    p = _lib.ptr
    _lib.check(_lib.load().ottohip_topk_per_aid(
        ctx.h, p(a) if n else None, p(b) if n else None, p(c) if n else None, n, int(max(n_items, 1)), int(first_n),
        p(out["aid"]), p(out["aid_next"]), p(out["count"]), p(out["count_pop"]), p(out["perc_pop"]), p(out["rank"]),
        p(out["count_rel"]), ctypes.byref(n_out), _lib.stream_handle(stream)))
    k = int(n_out.value)
    return {name: t[:k] for name, t in out.items()}


def get_df_count_for_co_event_type(count_type: str, dir_counts: str, first_n: int | None = None):
    """model/retrieve.py:18-63: reads {dir_counts}/{count_type}.parquet (aid, aid_next, count)
    and returns pandas DataFrame[aid, aid_next, {t}_count:i32, {t}_count_pop:i16,
    {t}_perc_pop:i16, {t}_rank:i16, {t}_count_rel:i8], at most first_n rows per aid."""
    import pandas as pd
    import pyarrow.parquet as pq
    if first_n is None:
        first_n = config.RETRIEVAL_FIRST_N_CO_COUNTS[count_type]
    t = pq.read_table(f"{dir_counts}/{count_type}.parquet", columns=["aid", "aid_next", "count"])
    cols = [t.column(k).to_numpy().astype(np.int32, copy=False) for k in ("aid", "aid_next", "count")]
    n_items = max(config.N_ITEMS_OTTO, int(cols[0].max()) + 1 if len(cols[0]) else 1)
    res = topk_per_aid(*cols, first_n=first_n, n_items=n_items)
    out = {"aid": res["aid"], "aid_next": res["aid_next"]}
    for k in ("count", "count_pop", "perc_pop", "rank", "count_rel"):
        out[f"{count_type}_{k}"] = res[k]
    return pd.DataFrame({k: v.cpu().numpy() for k, v in out.items()})


def get_pairs_for_all_co_event_types(dir_counts):
    """model/retrieve.py:66-72."""
    return {t: get_df_count_for_co_event_type(t, dir_counts) for t in config.RETRIEVAL_CO_COUNTS_TO_JOIN}
