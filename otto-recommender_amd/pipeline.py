"""Config-5 end-to-end candidate generation (BASELINE.json configs[4]) on the device:

  co-visitation per folder (count_co_events_fused) -> A6 per folder -> A7 train+test merge -> R1
  Word2Vec kNN of both models (first 600k vocabulary rows)   -> B3 lists
  session embeddings (C1) -> KMeans k=50 (C2) -> popularity ranks cl50 / cl1 (C3)
  candidates for the test sessions (R3-R6) -> session-item similarity (R7) -> recall@20 (R9)

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


def _files_events(ev, fb, files):
    """the whole files `files` (indices into the bounds fb) of an Events table, concatenated."""
    parts = [ev.slice_sessions(int(fb[f]), int(fb[f + 1])) for f in files]
    sizes = [p.n_sessions for p in parts]
    if not parts:
        from .synth import Events
        z = lambda dt: np.zeros(0, dt)
        return Events(np.zeros(1, np.int64), z(np.int32), z(np.int32), z(np.int32), z(np.int8)), np.zeros(1, np.int64)
    return _concat(parts), np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)


def _deal(fb, rank, world):
    from .dist import deal_files
    n_files = len(fb) - 1
    return deal_files(n_files, rank, world, [float(fb[f + 1] - fb[f]) for f in range(n_files)])


def _knn_lists(words, emb, knn_queries, ctx, dev, group):
    """B3 for the first knn_queries vocabulary rows; with a group the queries are split in equal
    ranges over ranks (the item matrix is replicated) and the lists all-gathered."""
    import torch
    idx = KnnIndex(emb, ctx)
    nq = min(knn_queries, idx.n_items)
    q0, q1 = 0, nq
    if group is not None:
        import torch.distributed as dist
        r, g = dist.get_rank(group), dist.get_world_size(group)
        q0, q1 = (nq * r) // g, (nq * (r + 1)) // g
    rows = torch.arange(q0, q1, dtype=torch.int32, device=dev)
    i, _ = idx.search(rows, k=config.W2VEC_K) if q1 > q0 else (torch.empty((0, config.W2VEC_K), dtype=torch.int32,
                                                                            device=dev), None)
    idx.free()
    if group is not None:
        from .dist import all_gather_rows
        n = i.shape[0]
        flat = i.reshape(-1)
        a, _, _ = all_gather_rows((flat, flat, flat), group)
        i = a.view(-1, config.W2VEC_K)
    w = torch.as_tensor(np.asarray(words, np.int32)).to(dev)
    valid = i >= 0
    q_aid = w[:nq].view(nq, 1).expand(nq, config.W2VEC_K)[valid]
    nb = w[i.clamp(min=0).long()][valid]
    rk = torch.arange(1, config.W2VEC_K + 1, device=dev, dtype=torch.int16).view(1, -1).expand(nq, -1)[valid]
    return q_aid.contiguous(), nb.contiguous(), rk.contiguous()


def run(train, test, labels, words_all, emb_all, words_12, emb_12, n_items: int = config.N_ITEMS_OTTO,
        n_clusters: int = 50, kmeans_iter: int = 100, knn_queries: int = config.W2VEC_SEARCH_SIMILAR_FOR_FIRST_N_AIDS,
        ctx=None, timings: dict | None = None, keep_tables: bool = False, group=None, n_init="auto",
        per_file: int | None = None, keep_candidates: bool = True) -> dict:
    """Config 5 end to end. group (torch.distributed, one process per GPU): train and test files
    are dealt whole to ranks (count + sharded A6 per folder, replicated A7 and R1), kNN queries are
    split over ranks and all-gathered, KMeans rows (every session) are sharded with all-reduced
    sums, C3 counters are all-reduced, and each rank generates the candidates of its own test
    files; recall sums are all-reduced. Every rank returns the global numbers; 'candidates' is the
    whole job's candidate count and 'local_candidates' this rank's. keep_tables: host copies of every
    stage's output in 'intermediates' (the candidates as a DataFrame, or with keep_candidates=False
    as the device CSR 'candidates_csr' plus 'test_session_ids', for full-size runs)."""
    t_entry = time.perf_counter()
    import torch
    from .synth import file_session_bounds
    from . import dist as gd
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    T = timings if timings is not None else {}
    tables = {}
    rank, world = 0, 1
    if group is not None:
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)

    def mark(name, t0):
        torch.cuda.synchronize()
        T[name] = T.get(name, 0.0) + time.perf_counter() - t0
        return time.perf_counter()

    t = time.perf_counter()
    T["prelude"] = T.get("prelude", 0.0) + t - t_entry
    # ---- co-visitation (model/count_co_events.py:201-226): count each folder (:204-205), A6 per
    # folder with its own file statistics (:212-216), then A6 on [train, test] (A7, :218-226)
    from .synth import SESSIONS_PER_FILE
    pf = per_file or SESSIONS_PER_FILE  # the reference's 100k-session parquet files (etl/jsonl_to_parquet.py:59)
    fb_tr, fb_te = file_session_bounds(train.n_sessions, pf), file_session_bounds(test.n_sessions, pf)
    my_tr = list(range(len(fb_tr) - 1)) if group is None else _deal(fb_tr, rank, world)
    my_te = list(range(len(fb_te) - 1)) if group is None else _deal(fb_te, rank, world)
    ev_tr, b_tr = _files_events(train, fb_tr, my_tr)
    ev_te, b_te = _files_events(test, fb_te, my_te)
    allev = _concat([ev_tr, ev_te])
    fb = np.concatenate([b_tr, b_te[1:] + b_tr[-1]])
    n_tr_files = len(b_tr) - 1
    dev_all = gc.DeviceEvents.from_host(allev, fb)
    # the label rows of this rank's test sessions (input, resident like the events)
    sess = ev_te.session[ev_te.session_offsets[:-1] - ev_te.session_offsets[0]]
    lab_cols = [torch.from_numpy(np.ascontiguousarray(labels[k].to_numpy(), dt)).to(dev)
                for k, dt in (("session", np.int32), ("aid", np.int32), ("type", np.int8))]
    sess_dev = torch.from_numpy(np.ascontiguousarray(sess, np.int32)).to(dev)
    # the two Word2Vec embedding tables (inputs like the events): resident once for the kNN indexes (B3), the
    # session embeddings (C1) and R7, instead of one host->device copy of 0.74 GB per consumer
    emb_dev = {}

    def resident(e):
        if isinstance(e, torch.Tensor) and e.device == dev and e.dtype == torch.float32:
            return e.contiguous()
        if id(e) not in emb_dev:
            x = e if isinstance(e, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(e, np.float32))
            emb_dev[id(e)] = x.to(dev, torch.float32).contiguous()
        return emb_dev[id(e)]

    emb_all, emb_12 = resident(emb_all), resident(emb_12)
    del emb_dev
    # the host copies made for the upload are input preparation: released here, not at the step's end
    # (freeing ~2 GB of host arrays took ~0.25 s after the last stage)
    n_tr_sessions = ev_tr.n_sessions
    del ev_tr, ev_te, allev
    t = mark("upload", t)
    # C2's n_init seed draws (numpy's permutation heads over all sessions) start now, on a host thread, and are
    # ready when the clustering begins
    km_model = gp.KMeans(n_clusters=n_clusters, max_iter=kmeans_iter, n_init=n_init)
    km_seeds = gp.SeedHeads(km_model.random_state, train.n_sessions + test.n_sessions, n_clusters, km_model.n_init)
    folders = [(dev_all.subset_files(0, n_tr_files), my_tr, len(fb_tr) - 1),
               (dev_all.subset_files(n_tr_files, len(fb) - 1), my_te, len(fb_te) - 1)]
    merged = {n: [] for n in config.CO_EVENTS_TO_COUNT}
    pairs = 0
    for folder, mine, n_files in folders:
        if group is None:
            tab = gc.count_co_events_fused(folder, n_items=n_items, ctx=ctx, per_file_rule="click_to_click")
        else:
            tab = gd.count_co_events_sharded(folder, mine, n_files, group, n_items=n_items, ctx=ctx,
                                                 per_file_rule="click_to_click")
        pairs += sum(tab.stats(n)["n_pairs"] for n in tab.names)
        t = mark("covis_count", t)
        for n in tab.names:
            if group is None:
                merged[n].append(gc.concat_files_w_stats_fused(folder, n, table=tab, n_items=n_items, ctx=ctx))
            else:
                merged[n].append(gd.concat_files_w_stats_sharded(folder, mine, n_files, n, table=tab, group=group,
                                                                 n_items=n_items, ctx=ctx))
            t = mark(f"merge_{n}", t)
        tab.free()
    if group is not None:
        pairs = int(gd._allreduce_sum(torch.tensor([pairs], dtype=torch.int64), group).item())
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
    knn = [_knn_lists(w, e, knn_queries, ctx, dev, group) for w, e in ((words_all, emb_all), (words_12, emb_12))]
    t = mark("knn", t)
    # ---- pop-cluster source: C1 embeddings of all sessions, C2 KMeans, C3 ranks (cl50)
    rmap_all = gp.row_of_aid_map(words_all, n_items, dev)  # aid -> row of emb_all, for C1 and R7
    se = gp.compute_sessions_embeddings(dev_all.offsets, dev_all.aid, dev_all.ts, dev_all.type, words_all, emb_all,
                                        n_items, ctx, rmap=rmap_all)
    t = mark("C1_embeddings", t)
    grows = None  # one GPU: every session, in order (KMeans.fit takes local rows as the global ones)
    if group is not None:
        grows = np.concatenate([np.concatenate([np.arange(fb_tr[f], fb_tr[f + 1]) for f in my_tr] or [np.zeros(0)]),
                                train.n_sessions + np.concatenate([np.arange(fb_te[f], fb_te[f + 1]) for f in my_te]
                                                                  or [np.zeros(0)])]).astype(np.int64)
    km = km_model.fit(se, ctx, group=group, global_rows=grows, seed_heads=km_seeds)
    labels_all = km.labels_
    t = mark("C2_kmeans", t)
    pop50 = gp.count_popularity(dev_all.offsets, dev_all.aid, dev_all.ts, dev_all.type, labels_all, n_clusters,
                                n_items, ctx=ctx, group=group)
    t = mark("C3_popularity", t)
    # ---- candidates for this rank's test sessions + recall
    rk_cols = [c for c in pop50.columns if c.startswith("rank_")]
    p = pop50[pop50[rk_cols].min(axis=1) <= 20]
    src = gcand.CandidateSources(r1, knn[0], knn[1], (p["cl50"].to_numpy(), p["aid"].to_numpy()), n_clusters,
                                 n_items, ctx)
    t = mark("sources", t)
    test_cl = labels_all[n_tr_sessions:]
    dev_test = folders[1][0]
    cands = gcand.generate(dev_test.offsets, dev_test.aid, dev_test.ts, dev_test.type, src, test_cl)
    t = mark("candidates", t)
    # ---- R7: cosine similarity / Euclidean distance between each candidate and its session's C1
    # embedding (model/retrieve.py:604-625; candidates without an aid embedding: 0 / -1)
    se_test = se[n_tr_sessions:]  # the candidates' arrays read in place (no copy of 8 B per candidate)
    sim = gp.session_item_similarity(cands, None, se_test, words_all, emb_all, None, n_items, ctx, rmap=rmap_all)
    t = mark("R7_similarity", t)
    lo, la = gcand.labels_csr_device(*lab_cols, sess_dev, ctx=ctx)
    t = mark("labels_csr", t)
    sums = cands.recall_sums(lo, la)
    n_cand = cands.n_cand
    if group is not None:
        tt = gd._allreduce_sum(torch.tensor(list(sums) + [n_cand], dtype=torch.int64), group).tolist()
        sums, n_cand = tt[:-1], int(tt[-1])
    rec = gcand.recall_from_sums(sums)
    t = mark("recall", t)
    out = {"pairs": int(pairs), "candidates": int(n_cand), "local_candidates": cands.n_cand,
           "local_test_files": len(my_te),
           "test_sessions": int(test.n_sessions), "kmeans_iter": km.n_iter_, "kmeans_inertia": km.inertia_,
           "kmeans_runs": list(km.run_stats_), "kmeans_best_run": km.best_run_,
           "recall": rec, "timings_s": T}
    if keep_tables:  # host copies of every stage's output, for the parity tests
        h = lambda x: x.cpu().numpy()
        out["intermediates"] = {
            "tables": {n: tuple(h(x) for x in v) for n, v in tables.items()},
            "r1": {n: tuple(h(x) for x in v) for n, v in r1.items()},
            "knn": [tuple(h(x) for x in v) for v in knn],
            "cluster_labels": h(labels_all), "cluster_rows": grows if grows is not None else np.arange(int(labels_all.numel()), dtype=np.int64), "pop": p[["cl50", "aid"]].reset_index(drop=True),
            "n_clusters": n_clusters, "test_session_ids": sess}
        if keep_candidates:  # R7 of every candidate and the test sessions' C1 embeddings (small runs)
            out["intermediates"]["similarity"] = tuple(h(x) for x in sim)
            out["intermediates"]["test_session_embeddings"] = h(se_test)
            out["intermediates"]["session_embeddings"] = h(se)  # C1 of every session: C2's input rows
        else:
            out["intermediates"]["similarity"] = sim
        if keep_candidates:
            out["intermediates"]["candidates"] = cands.to_pandas(sess)
        else:
            out["intermediates"]["candidates_csr"] = cands.to_torch()
    cands.free()
    del sim, se_test
    mark("finish", t)
    return out
