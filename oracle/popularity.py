"""CPU oracle (TEST INFRASTRUCTURE ONLY) for SURVEY.md §8(a) C1-C3 and R7.

C1 compute_sessions_embeddings (model/kmeans_sessions.py:40-86) in f64 (the reference sums f32 in
   an unspecified polars order; tests use a stated tolerance);
C2 KMeans of the reference's scikit-learn==1.2 branch (model/kmeans_sessions.py:152-159): sklearn
   1.2's KMeans.fit / _kmeans_single_lloyd restated in f64 (n_init runs from successive
   RandomState.permutation seeds, centring, relocation of empty clusters, strict convergence); each
   run is pinned against the installed scikit-learn (tests/test_oracle.py) given the same seeds;
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


def _lloyd(Xc, C, max_iter, tol_abs):
    """sklearn 1.2 _kmeans_single_lloyd (sklearn/cluster/_kmeans.py) in f64 on centred rows:
    E-step argmin (ties: lowest index), sums per label, empty clusters relocated to the rows
    farthest from their centroid (_relocate_empty_clusters_dense; among equal distances the
    lower row first), M-step; stop on unchanged labels (strict) or squared shift <= tol."""
    n, k = len(Xc), len(C)
    labels = np.full(n, -1, np.int64)
    strict = False
    it = 0
    xn = (Xc ** 2).sum(1)
    for it in range(1, max_iter + 1):
        new = (xn[:, None] - 2 * Xc @ C.T + (C ** 2).sum(1)[None, :]).argmin(1)
        counts = np.bincount(new, minlength=k).astype(np.int64)
        # per-label sums in row order (the order np.add.at takes; bincount is ~20x faster)
        d = Xc.shape[1]
        sums = np.bincount((new[:, None] * d + np.arange(d)).ravel(), weights=Xc.ravel(),
                           minlength=k * d).reshape(k, d)
        empty = np.flatnonzero(counts == 0)
        if len(empty):
            dist = ((Xc - C[new]) ** 2).sum(1)
            far = np.lexsort((np.arange(n), -dist))[:len(empty)]
            for e, f in zip(empty, far):
                sums[new[f]] -= Xc[f]
                counts[new[f]] -= 1
                sums[e] = Xc[f]
                counts[e] = 1
        Cn = C.copy()
        nz = counts > 0
        Cn[nz] = sums[nz] / counts[nz, None]
        shift = ((Cn - C) ** 2).sum()
        C = Cn
        if np.array_equal(new, labels):
            strict = True
            break
        labels = new
        if shift <= tol_abs:
            break
    if not strict:
        labels = (xn[:, None] - 2 * Xc @ C.T + (C ** 2).sum(1)[None, :]).argmin(1)
    inertia = float(((Xc - C[labels]) ** 2).sum())
    return labels, C, inertia, it


def kmeans_seeds(n, k, n_init, seed):
    """sklearn 1.2 _init_centroids(init='random'): successive RandomState(seed).permutation(n)[:k]."""
    rs = np.random.RandomState(seed)
    return [rs.permutation(n)[:k] for _ in range(n_init)]


def kmeans(X, k, max_iter=100, tol=1e-3, seed=42, n_init=10):
    """KMeans(init='random', n_init=n_init, max_iter, tol, random_state=seed).fit(X) of
    scikit-learn==1.2 (the reference's branch model/kmeans_sessions.py:152-159) restated in f64:
    tol scaled by the mean column variance, rows centred on the column means, the lowest-inertia
    run kept. Returns (labels, centers, n_iter, inertia)."""
    X = np.asarray(X, np.float64)
    tol_abs = float(np.mean(np.var(X, axis=0))) * tol
    mean = X.mean(0)
    Xc = X - mean
    best = None
    for seeds in kmeans_seeds(len(X), k, n_init, seed):
        lab, C, inertia, it = _lloyd(Xc, Xc[seeds].copy(), max_iter, tol_abs)
        if best is None or inertia < best[0]:
            best = (inertia, lab, C + mean, it)
    return best[1], best[2], best[3], best[0]


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
