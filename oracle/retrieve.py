"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the candidate-retrieval rows of SURVEY.md §8(a).

R1  get_df_count_for_co_event_type  (model/retrieve.py:18-63), restated on numpy with the
    polars ≈0.15 semantics it relies on:
      * pl.quantile default interpolation 'nearest': sorted[round((n - 1) * q)], f64::round
        (half away from zero);
      * integer '/' is true division in f64; casts to Int16 / Int8 truncate toward zero;
      * rank('ordinal', reverse=True).over('aid') after sort(['aid']): ties in count are broken
        by row order within the aid, taken here as FILE order (the build's deterministic
        choice; polars' unstable sort leaves it unspecified).
R5  trim rule's horizontal minima (model/retrieve.py:498, 502, 505: pl.min([col, ...])) are taken as
    polars' horizontal min with nulls SKIPPED (a row's min over its non-null sources; null only when
    every source is null), restated as pandas DataFrame.min(axis=1) (skipna=True). The installed
    polars version is unpinned; this is the assumed semantics, parity unpinned.
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


# ---------------------------------------------------------------------------------------------
# R3-R6, R8 (candidate columns only) and R9, restated on pandas for small inputs.
# Deterministic choices where polars leaves the order unspecified:
#   * every ordinal rank 'desc within group' breaks ties by aid ascending;
#   * the final (session, ts_order_aid) sort breaks ties by aid_next ascending.
SRC_NAMES = ["src_self", "src_click_to_click", "src_click_to_cart_or_buy", "src_cart_to_cart", "src_cart_to_buy",
             "src_buy_to_buy", "src_w2vec_all", "src_w2vec_1_2", "src_pop_cl50"]
RULES = ["click_to_click", "click_to_cart_or_buy", "cart_to_cart", "cart_to_buy", "buy_to_buy"]
RULE_TYPE = {"click_to_click": 0, "click_to_cart_or_buy": 0, "cart_to_cart": 1, "cart_to_buy": 1, "buy_to_buy": 2}
N_LAST = 99  # RETRIEVE_N_LAST_* / RETRIEVE_N_MOST_FREQUENT (config.py:76-79)


def _rank_desc(df, by, col, mask=None):
    """ordinal rank of `col` descending within `by`, ties by aid ascending; NaN where mask is False."""
    import pandas as pd
    d = df if mask is None else df[mask]
    order = d.sort_values(by + [col, "aid"], ascending=[True] * len(by) + [False, True], kind="stable")
    r = order.groupby(by, sort=False).cumcount() + 1
    out = pd.Series(np.nan, index=df.index)
    out.loc[r.index] = r.values
    return out


def session_aid_pairs_unique(ev):
    """model/retrieve.py:138-232 (columns used by candidate retrieval). ev: DataFrame
    [session, aid, ts, type], raw rows (no dedup)."""
    import pandas as pd
    g = ev.groupby(["session", "aid"], sort=True)
    sa = pd.DataFrame({"n_aid": g.size()})
    for t, nm in enumerate(["clicks", "carts", "orders"]):
        sa[f"n_aid_{nm}"] = ev.assign(x=(ev["type"] == t).astype(np.int64)).groupby(["session", "aid"])["x"].sum()
        m = ev[ev["type"] == t].groupby(["session", "aid"])["ts"].max()
        sa[f"max_ts_aid_{nm}"] = m
    sa["max_ts_aid"] = g["ts"].max()
    sa = sa.reset_index()
    for nm in ["clicks", "carts", "orders"]:
        sa[f"ts_order_aid_{nm}"] = _rank_desc(sa, ["session"], f"max_ts_aid_{nm}", sa[f"max_ts_aid_{nm}"].notna())
    sa["ts_order_aid"] = _rank_desc(sa, ["session"], "max_ts_aid")
    sa["rank_by_n_aid"] = _rank_desc(sa, ["session"], "n_aid")
    sa["rank_by_n_aid_carts"] = _rank_desc(sa, ["session"], "n_aid_carts")
    sa["rank_by_n_aid_orders"] = _rank_desc(sa, ["session"], "n_aid_orders")
    keep = ((sa["ts_order_aid_clicks"] <= N_LAST) | (sa["ts_order_aid_carts"] <= N_LAST)
            | (sa["ts_order_aid_orders"] <= N_LAST) | (sa["rank_by_n_aid"] <= N_LAST)
            | (sa["rank_by_n_aid_carts"] <= N_LAST) | (sa["rank_by_n_aid_orders"] <= N_LAST))
    return sa[keep].reset_index(drop=True)


def candidates(ev, r1: dict, knn_all, knn_12, session_cl=None, pop_cl50=None):
    """Candidate rows of retrieve_and_gen_feats (model/retrieve.py:477-595, features dropped):
    r1[name] = DataFrame[aid, aid_next, {name}_rank] (R1 output); knn_* = DataFrame[aid, aid_next, rank];
    session_cl = DataFrame[session, cl50]; pop_cl50 = DataFrame[cl50, aid] (aids with min rank <= 20).
    Returns DataFrame[session, aid_next, ts_order_aid, src_*] sorted by (session, ts_order_aid, aid_next)."""
    import pandas as pd
    sa = session_aid_pairs_unique(ev)
    # R4 (:244-290): self + co-event pairs of the session's aids + all kNN pairs, unique
    lst = [pd.DataFrame({"aid": sa["aid"].unique(), "aid_next": sa["aid"].unique()})]
    for n in RULES:
        lst.append(r1[n][["aid", "aid_next"]][r1[n]["aid"].isin(sa["aid"].unique())])
    lst += [knn_all[["aid", "aid_next"]], knn_12[["aid", "aid_next"]]]
    pairs = pd.concat(lst).drop_duplicates()
    df = sa.merge(pairs, on="aid", how="left")
    for n in RULES:
        df = df.merge(r1[n][["aid", "aid_next", f"{n}_rank"]], on=["aid", "aid_next"], how="left")
    df = df.merge(knn_all[["aid", "aid_next", "rank"]].rename(columns={"rank": "rank_w2vec_all"}),
                  on=["aid", "aid_next"], how="left")
    df = df.merge(knn_12[["aid", "aid_next", "rank"]].rename(columns={"rank": "rank_w2vec_1_2"}),
                  on=["aid", "aid_next"], how="left")
    # R5 (:490-516)
    best_order = df[["rank_by_n_aid", "ts_order_aid", "ts_order_aid_clicks", "ts_order_aid_carts",
                     "ts_order_aid_orders"]].min(axis=1)
    th = np.maximum(20 - (20 - 3) / (20 - 1) * (best_order - 1), 3)
    best_co = df[[f"{n}_rank" for n in RULES]].min(axis=1)
    best_w2v = df[["rank_w2vec_all", "rank_w2vec_1_2"]].min(axis=1)
    df = df[(df["aid"] == df["aid_next"]) | (best_co <= th) | (best_w2v <= th)]
    # keep_sessions_aids_next (:293-403) + source flags (:549-559)
    d = df.assign(
        slf=(df["aid"] == df["aid_next"]).astype(np.int64),
        **{f"has_{n}": df[f"{n}_rank"].notna().astype(np.int64) for n in RULES},
        w_all=df["rank_w2vec_all"].notna().astype(np.int64), w_12=df["rank_w2vec_1_2"].notna().astype(np.int64))
    g = d.groupby(["session", "aid_next"])
    out = pd.DataFrame({
        "ts_order_aid": g["ts_order_aid"].min(),
        "src_self": (g["slf"].sum() > 0).astype(np.int8),
    })
    n_type = {0: g["n_aid_clicks"].sum(), 1: g["n_aid_carts"].sum(), 2: g["n_aid_orders"].sum()}
    for n in RULES:
        out[f"src_{n}"] = ((n_type[RULE_TYPE[n]] > 0) & (g[f"has_{n}"].sum() > 0)).astype(np.int8)
    out["src_w2vec_all"] = (g["w_all"].sum() > 0).astype(np.int8)
    out["src_w2vec_1_2"] = (g["w_12"].sum() > 0).astype(np.int8)
    out = out.reset_index()
    out["src_pop_cl50"] = np.int8(0)
    # R6 (:571-585): pop candidates of the session's cl50 cluster, outer join
    if session_cl is not None and pop_cl50 is not None:
        s_cl = pd.DataFrame({"session": out["session"].unique()}).merge(session_cl, on="session", how="inner")
        pop = s_cl.merge(pop_cl50.rename(columns={"aid": "aid_next"}), on="cl50")[["session", "aid_next"]]
        pop = pop.drop_duplicates().assign(src_pop_cl50=np.int8(1))
        out = out.drop(columns=["src_pop_cl50"]).merge(pop, on=["session", "aid_next"], how="outer")
        for c in SRC_NAMES:
            out[c] = out[c].fillna(0).astype(np.int8)
        out["ts_order_aid"] = out["ts_order_aid"].fillna(999)
    out["ts_order_aid"] = out["ts_order_aid"].astype(np.int64)
    out = out.sort_values(["session", "ts_order_aid", "aid_next"], kind="stable").reset_index(drop=True)
    return out[["session", "aid_next", "ts_order_aid"] + SRC_NAMES]


def recall(cands, labels, max_k: int = 20, src: str | None = None) -> dict:
    """model/eval_retrieved.py:45-118 for one source filter: rank = position within session in
    candidate order (:52), per session hit@k clipped at max_k, summed; recall = hit / true per
    type, total = 0.1 clicks + 0.3 carts + 0.6 orders. labels: DataFrame[session, aid, type]."""
    import pandas as pd
    c = cands if src is None else cands[cands[src] == 1]
    c = c[["session", "aid_next"]].copy()
    c["rank"] = c.groupby("session").cumcount() + 1
    res = {}
    for t, nm in enumerate(["clicks", "carts", "orders"]):
        lab = labels[labels["type"] == t][["session", "aid"]].drop_duplicates().rename(columns={"aid": "aid_next"})
        m = lab.merge(c, on=["session", "aid_next"], how="left")
        hit = lambda k: ((m["rank"] <= k) if k else m["rank"].notna()).astype(np.int64)
        per = pd.DataFrame({"session": m["session"], "h20": hit(20), "h100": hit(100), "h200": hit(200),
                            "hall": hit(None), "true": 1}).groupby("session").sum().clip(upper=max_k)
        tot = per.sum()
        res[nm] = {f"top{k}": (tot[f"h{k}"] / tot["true"] if tot["true"] else 0.0) for k in ("20", "100", "200", "all")}
    res["total"] = {k: 0.1 * res["clicks"][k] + 0.3 * res["carts"][k] + 0.6 * res["orders"][k]
                    for k in res["clicks"]}
    return res
