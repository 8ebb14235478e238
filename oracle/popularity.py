"""CPU oracle (TEST INFRASTRUCTURE ONLY) for SURVEY.md §8(a) C1-C3 and R7.

C1 compute_sessions_embeddings (model/kmeans_sessions.py:40-86) in f64 (the reference sums f32 in
   an unspecified polars order; tests use a stated tolerance);
C2 Lloyd KMeans with the sklearn 'random' init (RandomState(seed).permutation(n)[:k]) and tol
   scaled by the mean feature variance (model/kmeans_sessions.py:153-161);
C3 count_popularity (model/count_popularity.py:53-85), ordinal ranks with aid-ascending ties;
R7 session-item similarity (model/retrieve.py:604-625).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import numpy as np


def sessions_embeddings(offsets, aid, ts, type_, words, emb):
    offsets = np.asarray(offsets, np.int64)
    row = {int(w): i for i, w in enumerate(np.asarray(words))}
    S, dim = len(offsets) - 1, emb.shape[1]
    out = np.zeros((S, dim), np.float64)
    wt = np.array([0.1, 0.3, 0.6], np.float32)
    for s in range(S):
        a, t, y = aid[offsets[s]:offsets[s + 1]], ts[offsets[s]:offsets[s + 1]], type_[offsets[s]:offsets[s + 1]]
        mx = t.max()
        wtime = np.maximum(1 - (mx - t.astype(np.float64)) / 259200.0, 0.10)
        w = (wtime * wt[y].astype(np.float64)).astype(np.float32).astype(np.float64)
        acc = np.zeros(dim)
        for j in range(len(a)):
            r = row.get(int(a[j]), -1)
            if r >= 0:
                acc += w[j] * emb[r].astype(np.float64)
        out[s] = np.round(acc / w.sum(), 6)
    return out


def kmeans(X, k, max_iter=100, tol=1e-3, seed=42):
    X = np.asarray(X, np.float64)
    n = len(X)
    C = X[np.random.RandomState(seed).permutation(n)[:k]].copy()
    tol_abs = X.var(axis=0).mean() * tol
    it = 0
    for it in range(1, max_iter + 1):
        d = (X ** 2).sum(1)[:, None] - 2 * X @ C.T + (C ** 2).sum(1)[None, :]
        lab = d.argmin(1)
        Cn = C.copy()
        for c in range(k):
            m = lab == c
            if m.any():
                Cn[c] = X[m].mean(0)
        shift = ((Cn - C) ** 2).sum()
        C = Cn
        if shift <= tol_abs:
            break
    d = (X ** 2).sum(1)[:, None] - 2 * X @ C.T + (C ** 2).sum(1)[None, :]
    return d.argmin(1), C, it


def popularity_ranks(session, aid, ts, type_, session_cl: dict, keep_top_k=20, suffix="cl50"):
    import pandas as pd
    df = pd.DataFrame({"session": session, "aid": aid, "ts": ts, "type": type_})
    df["cl"] = df["session"].map(session_cl)
    ts_7d = df["ts"].max() - 7 * 24 * 60 * 60
    g = df.assign(**{f"n_{nm}": (df["type"] == t).astype(np.int64) for t, nm in enumerate(["clicks", "carts", "orders"])},
                  **{f"n_{nm}_7d": ((df["type"] == t) & (df["ts"] > ts_7d)).astype(np.int64)
                     for t, nm in enumerate(["clicks", "carts", "orders"])})
    agg = g.groupby(["cl", "aid"])[[c for c in g.columns if c.startswith("n_")]].sum().reset_index()
    cols = ["n_clicks", "n_carts", "n_orders", "n_clicks_7d", "n_carts_7d", "n_orders_7d"]
    for c in cols:
        o = agg.sort_values(["cl", c, "aid"], ascending=[True, False, True], kind="stable")
        r = o.groupby("cl").cumcount() + 1
        agg.loc[r.index, c.replace("n_", "rank_") + f"_{suffix}"] = np.minimum(r.values, 999)
    rc = [c.replace("n_", "rank_") + f"_{suffix}" for c in cols]
    agg = agg[agg[rc].min(axis=1) <= keep_top_k].rename(columns={"cl": suffix})
    agg[rc] = agg[rc].astype(np.int16)
    return agg[["aid", suffix] + rc].sort_values([suffix, "aid"]).reset_index(drop=True)


def similarity(sess_emb, item_emb):
    dot = (sess_emb * item_emb).sum(1)
    ns, na = np.sqrt((sess_emb ** 2).sum(1)), np.sqrt((item_emb ** 2).sum(1))
    return dot / (ns * na), np.sqrt(((sess_emb - item_emb) ** 2).sum(1))
