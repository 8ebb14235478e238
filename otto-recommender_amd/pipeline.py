"""Config-5 end-to-end candidate generation (BASELINE.json configs[4]) on the device:

  co-visitation per folder (count_co_events_fused) -> A6 per folder -> A7 train+test merge -> R1
  Word2Vec kNN of both models (first 600k vocabulary rows)   -> B3 lists
  session embeddings (C1) -> KMeans k=50 (C2) -> popularity ranks cl50 / cl1 (C3)
  candidates for the test sessions (R3-R6) -> recall@20 (R9)

Mirrors the order of the reference's scripts (model/count_co_events.py, model/w2vec_aids.py,
model/kmeans_sessions.py, model/count_popularity.py, model/retrieve.py, model/eval_retrieved.py)
with every stage on the GPU; tables stay resident in HBM between stages.
"""
from __future__ import annotations

import time

import numpy as np

from . import _lib, config
from . import covis as gc
from . import retrieve as gr
from . import candidates as gcand
from . import popularity as gp
from .w2vec import KnnIndex


def _concat(parts):
    from .synth import Events
    offs, base = [np.zeros(1, np.int64)], 0
    for p in parts:
        o = p.session_offsets - p.session_offsets[0]
        offs.append(o[1:] + base)
        base += int(o[-1])
    cat = lambda k: np.concatenate([getattr(p, k) for p in parts])
    return Events(np.concatenate(offs), cat("session"), cat("aid"), cat("ts"), cat("type"))


def run(train, test, labels, words_all, emb_all, words_12, emb_12, n_items: int = config.N_ITEMS_OTTO,
        n_clusters: int = 50, kmeans_iter: int = 100, knn_queries: int = config.W2VEC_SEARCH_SIMILAR_FOR_FIRST_N_AIDS,
        ctx=None, timings: dict | None = None, keep_tables: bool = False) -> dict:
    import torch
    from .synth import file_session_bounds
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    T = timings if timings is not None else {}
    tables = {}

    def mark(name, t0):
        torch.cuda.synchronize()
        T[name] = T.get(name, 0.0) + time.perf_counter() - t0
        return time.perf_counter()

    t = time.perf_counter()
    # ---- co-visitation (model/count_co_events.py:201-226): count each folder (:204-205), A6 per
    # folder with its own file statistics (:212-216), then A6 on [train, test] (A7, :218-226)
    allev = _concat([train, test])
    fb_tr = file_session_bounds(train.n_sessions)
    fb = np.concatenate([fb_tr, file_session_bounds(test.n_sessions)[1:] + train.n_sessions])
    n_tr_files = len(fb_tr) - 1
    dev_all = gc.DeviceEvents.from_host(allev, fb)
    t = mark("upload", t)
    folders = [dev_all.subset_files(0, n_tr_files), dev_all.subset_files(n_tr_files, len(fb) - 1)]
    merged = {n: [] for n in config.CO_EVENTS_TO_COUNT}
    pairs = 0
    for folder in folders:
        tab = gc.count_co_events_fused(folder, n_items=n_items, ctx=ctx)
        pairs += sum(tab.stats(n)["n_pairs"] for n in tab.names)
        t = mark("covis_count", t)
        for n in tab.names:
            merged[n].append(gc.concat_files_w_stats_fused(folder, n, table=tab, n_items=n_items, ctx=ctx))
            t = mark(f"merge_{n}", t)
        tab.free()
    r1 = {}
    for n in config.CO_EVENTS_TO_COUNT:
        a, b, c = gc.merge_train_test(n, merged[n][0], merged[n][1], n_items=n_items, ctx=ctx)
        merged[n] = None
        t = mark("merge_train_test", t)
        r = gr.topk_per_aid(a, b, c, config.RETRIEVAL_FIRST_N_CO_COUNTS[n], n_items=n_items, ctx=ctx)
        r1[n] = (r["aid"], r["aid_next"], r["rank"])
        if keep_tables:
            tables[n] = (a, b, c)
        t = mark("R1", t)
    # ---- kNN of both Word2Vec models (model/retrieve.py:683-687)
    knn = []
    for words, emb in ((words_all, emb_all), (words_12, emb_12)):
        idx = KnnIndex(emb, ctx)
        nq = min(knn_queries, idx.n_items)
        i, _ = idx.search(None, n_q=nq, k=config.W2VEC_K)
        w = torch.as_tensor(np.asarray(words, np.int32)).to(dev)
        valid = i >= 0
        q_aid = w[:nq].view(nq, 1).expand(nq, config.W2VEC_K)[valid]
        nb = w[i.clamp(min=0).long()][valid]
        rk = torch.arange(1, config.W2VEC_K + 1, device=dev, dtype=torch.int16).view(1, -1).expand(nq, -1)[valid]
        knn.append((q_aid.contiguous(), nb.contiguous(), rk.contiguous()))
        idx.free()
    t = mark("knn", t)
    # ---- pop-cluster source: C1 embeddings of all sessions, C2 KMeans, C3 ranks (cl50 and cl1)
    se = gp.compute_sessions_embeddings(dev_all.offsets, dev_all.aid, dev_all.ts, dev_all.type, words_all, emb_all,
                                        n_items, ctx)
    t = mark("C1_embeddings", t)
    km = gp.KMeans(n_clusters=n_clusters, max_iter=kmeans_iter).fit(se, ctx)
    labels_all = km.labels_
    t = mark("C2_kmeans", t)
    pop50 = gp.count_popularity(dev_all.offsets, dev_all.aid, dev_all.ts, dev_all.type, labels_all, n_clusters,
                                n_items, ctx=ctx)
    t = mark("C3_popularity", t)
    # ---- candidates for the test sessions + recall
    rk_cols = [c for c in pop50.columns if c.startswith("rank_")]
    p = pop50[pop50[rk_cols].min(axis=1) <= 20]
    src = gcand.CandidateSources(r1, knn[0], knn[1], (p["cl50"].to_numpy(), p["aid"].to_numpy()), n_clusters,
                                 n_items, ctx)
    t = mark("sources", t)
    test_cl = labels_all[train.n_sessions:]
    dev_test = dev_all.subset_files(len(fb) - 1 - (len(file_session_bounds(test.n_sessions)) - 1), len(fb) - 1)
    cands = gcand.generate(dev_test.offsets, dev_test.aid, dev_test.ts, dev_test.type, src, test_cl)
    t = mark("candidates", t)
    sess = test.session[test.session_offsets[:-1] - test.session_offsets[0]]
    lo, la = gcand.labels_csr(labels, sess)
    t = mark("labels_csr", t)
    rec = cands.recall(lo, la)
    t = mark("recall", t)
    out = {"pairs": int(pairs), "candidates": cands.n_cand, "test_sessions": int(test.n_sessions),
           "kmeans_iter": km.n_iter_, "recall": rec, "timings_s": T}
    if keep_tables:  # host copies of every stage's output, for the parity tests
        h = lambda x: x.cpu().numpy()
        out["intermediates"] = {
            "tables": {n: tuple(h(x) for x in v) for n, v in tables.items()},
            "r1": {n: tuple(h(x) for x in v) for n, v in r1.items()},
            "knn": [tuple(h(x) for x in v) for v in knn],
            "cluster_labels": h(labels_all), "pop": p[["cl50", "aid"]].reset_index(drop=True),
            "candidates": cands.to_pandas(sess)}
    cands.free()
    return out
