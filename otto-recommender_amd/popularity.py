"""Pop-cluster source of config 5 and session-item similarity.

  compute_sessions_embeddings   model/kmeans_sessions.py:40-86
  KMeans (fit / labels_)        model/kmeans_sessions.py:140-171 (Lloyd, sklearn 'random' init
                                semantics: rows RandomState(random_state).permutation(n)[:k];
                                tol scaled by the mean feature variance; the reference's dask-ml
                                k-means|| init is not reproducible)
  count_popularity              model/count_popularity.py:53-85 (ranks_for_clusters)
  session_item_similarity       model/retrieve.py:604-625
All compute runs in libottohip.so (csrc/popularity.hip).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from . import config

RANK_COLS = ["rank_clicks", "rank_carts", "rank_orders", "rank_clicks_7d", "rank_carts_7d", "rank_orders_7d"]


def _t(x, dev, dtype):
    import torch
    return (x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))).to(dev, dtype).contiguous()


def row_of_aid_map(words, n_items: int, dev):
    """aid -> embedding row (vocabulary order), -1 for aids without an embedding."""
    import torch
    words = np.asarray(words, np.int64)
    n = max(int(n_items), int(words.max()) + 1 if len(words) else 1)
    m = np.full(n, -1, np.int32)
    m[words] = np.arange(len(words), dtype=np.int32)
    return torch.from_numpy(m).to(dev)


def compute_sessions_embeddings(offsets, aid, ts, type_, words, embeddings, n_items: int = config.N_ITEMS_OTTO,
                                ctx=None, stream=None):
    """C1 for a session-sorted event table: torch f32 [n_sessions, dim] on the device."""
    import torch
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    off = _t(offsets, dev, torch.int64)
    off = off - off[0]
    a, s_, y = _t(aid, dev, torch.int32), _t(ts, dev, torch.int32), _t(type_, dev, torch.int8)
    emb = _t(embeddings, dev, torch.float32)
    rmap = row_of_aid_map(words, n_items, dev)
    S = int(off.numel()) - 1
    dim = int(emb.shape[1])
    out = torch.empty((max(S, 1), dim), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().ottohip_session_embeddings(ctx.h, _lib.ptr(off), S, _lib.ptr(a), _lib.ptr(s_), _lib.ptr(y),
                                                      _lib.ptr(rmap), int(rmap.numel()), _lib.ptr(emb), dim,
                                                      _lib.ptr(out), _lib.stream_handle(stream)))
    return out[:S]


class KMeans:
    """KMeans(n_clusters, max_iter=100, tol=1e-3, random_state=42) on a device matrix."""

    def __init__(self, n_clusters: int = 50, max_iter: int = 100, tol: float = 1e-3, random_state: int = 42):
        self.n_clusters, self.max_iter, self.tol, self.random_state = n_clusters, max_iter, tol, random_state

    def fit(self, X, ctx=None, stream=None, group=None):
        import torch
        ctx = ctx or _lib.context()
        dev = torch.device("cuda", ctx.device)
        X = _t(X, dev, torch.float32)
        n, dim = (int(v) for v in X.shape)
        k = self.n_clusters
        seeds = np.random.RandomState(self.random_state).permutation(n)[:k]
        C = X[torch.from_numpy(seeds).to(dev)].clone().contiguous()
        tol_abs = float(torch.var(X.double(), dim=0, unbiased=False).mean().item()) * self.tol
        labels = torch.empty(n, dtype=torch.int32, device=dev)
        lib = _lib.load()
        sh, inr = ctypes.c_double(), ctypes.c_double()
        it = 0
        for it in range(1, self.max_iter + 1):
            _lib.check(lib.ottohip_kmeans_step(ctx.h, _lib.ptr(X), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                               ctypes.byref(sh), ctypes.byref(inr), _lib.stream_handle(stream)))
            if sh.value <= tol_abs:
                break
        _lib.check(lib.ottohip_kmeans_assign(ctx.h, _lib.ptr(X), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                             ctypes.byref(inr), _lib.stream_handle(stream)))
        self.cluster_centers_, self.labels_, self.inertia_, self.n_iter_ = C, labels, inr.value, it
        return self


def count_popularity(offsets, aid, ts, type_, session_cl, n_clusters: int, n_items: int = config.N_ITEMS_OTTO,
                     keep_top_k: int = config.KEEP_TOP_K, ts_max: int | None = None, suffix: str = "cl50",
                     ctx=None, stream=None):
    """C3 for one clustering (dense cluster index per session). Returns pandas
    DataFrame[aid, {suffix}, rank_*_{suffix} (6 columns)], rows sorted by (cluster, aid)."""
    import pandas as pd
    import torch
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    off = _t(offsets, dev, torch.int64)
    off = off - off[0]
    a, s_, y = _t(aid, dev, torch.int32), _t(ts, dev, torch.int32), _t(type_, dev, torch.int8)
    cl = _t(session_cl, dev, torch.int32)
    S = int(off.numel()) - 1
    if ts_max is None:
        ts_max = int(s_.max().item()) if s_.numel() else 0
    ts_7d = int(ts_max) - 7 * 24 * 60 * 60                     # count_popularity.py:54-55
    h = ctypes.c_void_p()
    nout = ctypes.c_int64()
    lib = _lib.load()
    _lib.check(lib.ottohip_popularity_ranks(ctx.h, _lib.ptr(off), S, _lib.ptr(a), _lib.ptr(s_), _lib.ptr(y), _lib.ptr(cl),
                                            int(n_items), int(n_clusters), ts_7d, int(keep_top_k), ctypes.byref(h),
                                            ctypes.byref(nout), _lib.stream_handle(stream)))
    n = int(nout.value)
    try:
        oa = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        oc = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        orr = torch.empty((max(n, 1), 6), dtype=torch.int16, device=dev)
        _lib.check(lib.ottohip_pop_copy(h, _lib.ptr(oa), _lib.ptr(oc), _lib.ptr(orr), _lib.stream_handle(stream)))
    finally:
        lib.ottohip_pop_free(h)
    r = orr[:n].cpu().numpy()
    out = {"aid": oa[:n].cpu().numpy(), suffix: oc[:n].cpu().numpy()}
    for i, c in enumerate(RANK_COLS):
        out[f"{c}_{suffix}"] = r[:, i]
    return pd.DataFrame(out)


def session_item_similarity(cand_off, aid_next, sess_emb, words, embeddings, sess_has=None,
                            n_items: int = config.N_ITEMS_OTTO, ctx=None, stream=None):
    """R7 for candidates in CSR (cand_off [S+1]): torch (cos_sim_ses_aid, eucl_dist_ses_aid) f32."""
    import torch
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    off = _t(cand_off, dev, torch.int64)
    nxt = _t(aid_next, dev, torch.int32)
    se = _t(sess_emb, dev, torch.float32)
    emb = _t(embeddings, dev, torch.float32)
    has = None if sess_has is None else _t(sess_has, dev, torch.uint8)
    rmap = row_of_aid_map(words, n_items, dev)
    S = int(off.numel()) - 1
    n = int(nxt.numel())
    cos = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    eu = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().ottohip_session_item_similarity(
        ctx.h, _lib.ptr(off), S, _lib.ptr(nxt) if n else None, _lib.ptr(se), _lib.ptr(has) if has is not None else None,
        _lib.ptr(rmap), int(rmap.numel()), _lib.ptr(emb), int(emb.shape[1]), _lib.ptr(cos), _lib.ptr(eu),
        _lib.stream_handle(stream)))
    return cos[:n], eu[:n]
