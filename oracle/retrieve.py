"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the candidate-retrieval rows of SURVEY.md §8(a).

R1  get_df_count_for_co_event_type  (model/retrieve.py:18-63), restated on numpy with the
    polars ≈0.15 semantics it relies on:
      * pl.quantile default interpolation 'nearest': sorted[round((n - 1) * q)], f64::round
        (half away from zero);
      * integer '/' is true division in f64; casts to Int16 / Int8 truncate toward zero;
      * rank('ordinal', reverse=True).over('aid') after sort(['aid']): ties in count are broken
        by row order within the aid, taken here as FILE order (the build's deterministic
        choice; polars' unstable sort leaves it unspecified).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import math

import numpy as np


def get_df_count_for_co_event_type(aid, aid_next, count, first_n: int) -> dict:
    aid = np.asarray(aid, np.int32)
    aid_next = np.asarray(aid_next, np.int32)
    count = np.asarray(count, np.int32)
    n = len(aid)
    if n == 0 or first_n == 0:
        z = np.zeros(0)
        return {"aid": z.astype(np.int32), "aid_next": z.astype(np.int32), "count": z.astype(np.int32),
                "count_pop": z.astype(np.int16), "perc_pop": z.astype(np.int16), "rank": z.astype(np.int16),
                "count_rel": z.astype(np.int8)}
    # :34-36 over the entire population
    srt = np.sort(count.astype(np.int64))
    cmin = int(srt[0])
    qi = int(math.floor((n - 1) * 0.9999 + 0.5))  # f64::round for a non-negative value
    q = int(srt[qi])
    with np.errstate(divide="ignore", invalid="ignore"):
        pop = (count.astype(np.int64) - cmin).astype(np.float64) / float(q - cmin)
    pop = np.minimum(pop, 1.0)
    pop = np.where(np.isnan(pop), 0.0, pop)
    count_pop = np.trunc(pop * 10000.0).astype(np.int16)
    # :37-38 row number in file order
    perc_pop = np.trunc(np.arange(1, n + 1, dtype=np.float64) / float(n) * 10000.0).astype(np.int16)
    # :42-49 rank within aid: count desc, ties by file order
    order = np.lexsort((np.arange(n), -count.astype(np.int64), aid))
    a_s = aid[order]
    start = np.concatenate([[True], a_s[1:] != a_s[:-1]])
    gstart = np.maximum.accumulate(np.where(start, np.arange(n), 0))
    rank = np.arange(n) - gstart + 1
    cmax = count[order][gstart]
    keep = rank <= first_n
    o = order[keep]
    rel = np.trunc(count[o].astype(np.float64) / cmax[keep].astype(np.float64) * 100.0).astype(np.int8)
    return {"aid": aid[o], "aid_next": aid_next[o], "count": count[o], "count_pop": count_pop[o],
            "perc_pop": perc_pop[o], "rank": rank[keep].astype(np.int16), "count_rel": rel}
