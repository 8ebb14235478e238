"""Config-5 pipeline (otto-recommender_amd/pipeline.py) end to end on a small synthetic split:
every stage runs on the device and the candidates / recall of the pipeline equal the
candidates built from the same intermediate tables (no stage is skipped or cached)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_pipeline_small(gpu):
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import pipeline
    ev = synth.generate(60_000)
    train, test, labels = synth.split_test_labels(ev)
    words = synth.item_words()
    emb = synth.embeddings(len(words), seed=1)
    emb2 = synth.embeddings(len(words), seed=3)
    T = {}
    res = pipeline.run(train, test, labels, words, emb, words, emb2, n_clusters=8, kmeans_iter=20,
                       knn_queries=20_000, timings=T)
    assert res["test_sessions"] == test.n_sessions > 0
    assert res["candidates"] > 10 * res["test_sessions"]
    for t in ("clicks", "carts", "orders", "total"):
        for k in ("top20", "top100", "top200", "topall"):
            assert 0.0 <= res["recall"][t][k] <= 1.0
        assert res["recall"][t]["top20"] <= res["recall"][t]["top100"] <= res["recall"][t]["topall"]
    assert res["recall"]["total"]["topall"] > 0.1  # self + co-visit candidates recover revisits
    for stage in ("covis_count", "R1", "knn", "C1_embeddings", "C2_kmeans", "C3_popularity", "candidates",
                  "R7_similarity", "recall"):
        assert stage in T, stage


def test_pipeline_recall_parity(gpu):
    """Config 5 (BASELINE configs[4]) at test scale, stage by stage against the oracle on the same
    inputs: A7 tables (oracle.merge_train_test: A6 per folder, then A6 on [train, test]), R1
    (model/retrieve.py:18-63), C3 given the device clustering, candidates (R3-R6, R8) from the
    same R1 / kNN / pop lists, and recall@20/100/200/all per type (model/eval_retrieved.py:45-118)
    -- all exact. kNN sets are checked against the exact oracle in tests/test_knn.py."""
    import pandas as pd
    import covis as oracle
    import retrieve as oracle_retrieve
    import popularity as oracle_pop
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import pipeline, config
    ev = synth.generate(24_000, first_session=31)
    train, test, labels = synth.split_test_labels(ev)
    words = synth.item_words()
    emb = synth.embeddings(len(words), seed=1)
    emb2 = synth.embeddings(len(words), seed=3)
    res = pipeline.run(train, test, labels, words, emb, words, emb2, n_clusters=6, kmeans_iter=15,
                       knn_queries=30_000, keep_tables=True)
    im = res["intermediates"]
    per_tr = oracle.count_co_events_file(train.session_offsets, train.aid, train.ts, train.type)
    per_te = oracle.count_co_events_file(test.session_offsets, test.aid, test.ts, test.type)
    r1 = {}
    for n in config.CO_EVENTS_TO_COUNT:
        ref = oracle.merge_train_test(n, [per_tr[n]], [per_te[n]])
        for x, y in zip(im["tables"][n], ref):
            np.testing.assert_array_equal(x, y, err_msg=f"A7 {n}")
        t = oracle_retrieve.get_df_count_for_co_event_type(*ref, config.RETRIEVAL_FIRST_N_CO_COUNTS[n])
        for x, k in zip(im["r1"][n], ("aid", "aid_next", "rank")):
            np.testing.assert_array_equal(x, t[k], err_msg=f"R1 {n} {k}")
        r1[n] = pd.DataFrame({"aid": t["aid"], "aid_next": t["aid_next"], f"{n}_rank": t["rank"]})
    assert sum(len(im["tables"][n][0]) for n in r1) > 0
    # C3 on the device clustering of all (train + test) sessions
    allv = pipeline._concat([train, test])
    sess_all = allv.session[allv.session_offsets[:-1]]
    cl = im["cluster_labels"]
    pop_ref = oracle_pop.popularity_ranks(allv.session, allv.aid, allv.ts, allv.type,
                                          dict(zip(sess_all.tolist(), cl.tolist())))
    rk = [c for c in pop_ref.columns if c.startswith("rank_")]
    pop_ref = pop_ref[pop_ref[rk].min(axis=1) <= 20].sort_values(["cl50", "aid"])
    got_pop = im["pop"].sort_values(["cl50", "aid"])
    np.testing.assert_array_equal(got_pop["cl50"].to_numpy(), pop_ref["cl50"].to_numpy())
    np.testing.assert_array_equal(got_pop["aid"].to_numpy(), pop_ref["aid"].to_numpy())
    # candidates of the test sessions from the same sources
    knn = [pd.DataFrame({"aid": a, "aid_next": b, "rank": r}) for a, b, r in im["knn"]]
    sess_te = test.session[test.session_offsets[:-1] - test.session_offsets[0]]
    scl = pd.DataFrame({"session": sess_te, "cl50": cl[train.n_sessions:]})
    ref_c = oracle_retrieve.candidates(test.to_pandas(), r1, knn[0], knn[1], scl, im["pop"])
    got_c = im["candidates"]
    assert len(got_c) == len(ref_c) == res["candidates"]
    for c in ["session", "aid_next", "ts_order_aid"] + [c for c in ref_c.columns if c.startswith("src_")]:
        np.testing.assert_array_equal(got_c[c].to_numpy().astype(np.int64), ref_c[c].to_numpy().astype(np.int64),
                                      err_msg=c)
    # R7 (model/retrieve.py:604-625) of every candidate: cos / Euclidean to the session's C1 embedding in
    # f64 (candidates without an aid embedding: 0 / -1); fp32 on the device, rtol 1e-5
    cos, eu = im["similarity"]
    se = im["test_session_embeddings"]
    from otto_recommender_amd.w2vec import word_rows
    o_ = np.argsort(sess_te, kind="stable")
    sidx = o_[np.searchsorted(sess_te[o_], got_c["session"].to_numpy())]
    r_ = word_rows(words, got_c["aid_next"].to_numpy())
    ok = r_ >= 0
    rc, re = oracle_pop.similarity(se[sidx[ok]].astype(np.float64), emb[r_[ok]].astype(np.float64))
    np.testing.assert_allclose(cos[ok], rc, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(eu[ok], re, rtol=1e-5)
    assert np.all(cos[~ok] == 0) and np.all(eu[~ok] == -1)
    rec = oracle_retrieve.recall(ref_c, labels)
    for t in ("clicks", "carts", "orders", "total"):
        for k in ("top20", "top100", "top200", "topall"):
            assert abs(res["recall"][t][k] - rec[t][k]) < 1e-12, (t, k)


@pytest.mark.slow
def test_pipeline_config5_full_size(gpu):
    """BASELINE configs[4] at the bench's size (12.9 M sessions, 100k-session files, seed 0):
    - the A7 train+test tables of all five rules equal the C oracle's (tests/golden/digest_config5.json,
      make_golden.py --config5): click_to_click's train folder takes A6 branches (1) and (2) by rows
      (N = 500 M rows with count >= 2), the others (1) / (3);
    - the candidates of 20,000 sampled test sessions equal oracle/retrieve.candidates given the
      device's own R1 / kNN / pop lists and clustering (model/retrieve.py:477-595);
    - device recall sums (k_cand_recall) of those sessions equal model/eval_retrieved.py:45-118's."""
    import json
    import os
    import pandas as pd
    import torch
    import covis as oracle
    import retrieve as oracle_retrieve
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import pipeline, candidates as gcand, config
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "digest_config5.json")))
    ev = synth.generate(g["sessions"])
    train, test, labels = synth.split_test_labels(ev)
    del ev
    assert (train.n_sessions, test.n_sessions) == (g["train_sessions"], g["test_sessions"])
    words = synth.item_words()
    emb = synth.embeddings(len(words), seed=1)
    emb2 = synth.embeddings(len(words), seed=3)
    res = pipeline.run(train, test, labels, words, emb, words, emb2, keep_tables=True, keep_candidates=False)
    im = res["intermediates"]
    for n in config.CO_EVENTS_TO_COUNT:
        d = oracle.canonical_digest({n: im["tables"][n]})[n]
        ref = g["rules"][n]
        assert (d["rows"], d["sum"], d["sha256"]) == (ref["rows"], ref["sum"], ref["sha256"]), n
    # 20k sampled test sessions: candidates from the device run vs the oracle on the same sources
    rng = np.random.default_rng(55)
    S = test.n_sessions
    pick = np.sort(rng.choice(S, size=20_000, replace=False))
    csr = im["candidates_csr"]
    off = csr["off"].cpu().numpy()
    lens = off[pick + 1] - off[pick]
    rows = torch.from_numpy(np.repeat(off[pick] - np.cumsum(lens) + lens, lens) + np.arange(lens.sum())).to(
        csr["aid_next"].device)
    sess_ids = im["test_session_ids"]
    got = pd.DataFrame({"session": np.repeat(sess_ids[pick], lens),
                        "aid_next": csr["aid_next"][rows].cpu().numpy(),
                        "ts_order_aid": csr["ts_order_aid"][rows].cpu().numpy()})
    fl = csr["flags"][rows].cpu().numpy().view(np.uint16)
    for i, c in enumerate(gcand.SRC_NAMES):
        got[c] = ((fl >> i) & 1).astype(np.int8)
    parts = [test.slice_sessions(int(s), int(s) + 1) for s in pick]
    sub = pipeline._concat(parts)
    df = sub.to_pandas()
    aids = np.unique(df["aid"].to_numpy())
    f = lambda a, b, r, col: (lambda m: pd.DataFrame({"aid": a[m], "aid_next": b[m], col: r[m]}))(np.isin(a, aids))
    r1 = {n: f(*im["r1"][n], f"{n}_rank") for n in config.CO_EVENTS_TO_COUNT}
    knn = [f(*k, "rank") for k in im["knn"]]
    cl = im["cluster_labels"][train.n_sessions:][pick]
    scl = pd.DataFrame({"session": sess_ids[pick], "cl50": cl})
    ref = oracle_retrieve.candidates(df, r1, knn[0], knn[1], scl, im["pop"])
    assert len(got) == len(ref) > 20 * 20_000
    for c in ["session", "aid_next", "ts_order_aid"] + gcand.SRC_NAMES:
        np.testing.assert_array_equal(got[c].to_numpy().astype(np.int64), ref[c].to_numpy().astype(np.int64),
                                      err_msg=c)
    # recall sums of the sample: the device kernel on the sampled sessions vs the restatement
    p = im["pop"]
    src = gcand.CandidateSources(im["r1"], im["knn"][0], im["knn"][1], (p["cl50"].to_numpy(), p["aid"].to_numpy()),
                                 im["n_clusters"], config.N_ITEMS_OTTO)
    c = gcand.generate(sub.session_offsets, sub.aid, sub.ts, sub.type, src, cl.astype(np.int32))
    lab = labels[labels["session"].isin(sess_ids[pick])]
    lo, la = gcand.labels_csr(lab, sess_ids[pick])
    r = c.recall(lo, la)
    e = oracle_retrieve.recall(ref, lab)
    for t in ("clicks", "carts", "orders", "total"):
        for k in ("top20", "top100", "top200", "topall"):
            assert abs(r[t][k] - e[t][k]) < 1e-12, (t, k)
    assert c.n_cand == len(ref)
    c.free()


def _kmeans_reference_runs(X64, k, n_init, seed=42):
    """The f64 runs of the reference's scikit-learn branch (model/kmeans_sessions.py:134, 152-161: np.array of the
    embedding lists is float64): each run is the installed scikit-learn's Lloyd from the n_init seed rows
    RandomState(seed).permutation(n)[:k] (oracle/popularity.kmeans_seeds). tests/test_oracle.py pins these runs
    to the sklearn-1.2 restatement oracle/popularity._lloyd run by run (labels, inertia, n_iter); sklearn's Cython
    Lloyd is used here only because the numpy restatement needs ~5 min for 10 x 100 steps at 50 k rows."""
    import warnings
    import popularity as oracle_pop
    from sklearn.cluster import KMeans as SKKMeans
    runs = []
    for sd in oracle_pop.kmeans_seeds(len(X64), k, n_init, seed):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            km = SKKMeans(n_clusters=k, init=X64[sd], n_init=1, max_iter=100, tol=1e-3, algorithm="lloyd").fit(X64)
        runs.append((float(km.inertia_), int(km.n_iter_), km.labels_.astype(np.int64)))
    return runs


def test_kmeans_config5_sessions_vs_f64_reference(gpu):
    """C2 pinned on its real workload: KMeans(n_clusters=50, n_init=10, max_iter=100,
    tol=1e-3, random_state=42) on the config-5 session embeddings (C1 of every train + test session) of
    50 k synthetic sessions, the device fit (f32 rows, pipeline.run) against the reference's f64 fit
    (model/kmeans_sessions.py:134, 152-161) from the same seeds, run by run, and the recall@20 effect of
    the two clusterings on the same candidate sources (R1 / kNN from the same run; C3 and the pop-cluster
    candidates recomputed by the oracle from each clustering; model/retrieve.py:477-595,
    model/eval_retrieved.py:45-118).

    Measured on MI355X (round 6, DESIGN.md §3 "C2 on its real workload"): 7 of the 10 runs end within 1e-9
    relative inertia of the f64 runs with the same n_iter; three drift (1.7e-5, 5.0e-6 and 6.1e-4, one of them
    100 vs 98 steps); the kept run is the same seed on both sides, its labels agree on every row and recall@20 is
    identical. The thresholds: the same best run, >= 99.9 % label agreement on it (the blob test's bar), its
    inertia within 1e-6, every run within 2e-3 and 2 steps, |delta recall@20| <= 1e-4 per type."""
    import json
    import pandas as pd
    import popularity as oracle_pop
    import retrieve as oracle_retrieve
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import pipeline
    ev = synth.generate(50_000, first_session=7)
    train, test, labels = synth.split_test_labels(ev)
    words = synth.item_words()
    emb = synth.embeddings(len(words), seed=1)
    emb2 = synth.embeddings(len(words), seed=3)
    res = pipeline.run(train, test, labels, words, emb, words, emb2, n_clusters=50, kmeans_iter=100,
                       knn_queries=30_000, keep_tables=True)
    im = res["intermediates"]
    X = im["session_embeddings"].astype(np.float64)
    ref = _kmeans_reference_runs(X, 50, 10)
    dev = res["kmeans_runs"]
    assert len(dev) == len(ref) == 10
    ref_best = int(np.argmin([r[0] for r in ref]))
    dev_best = int(res["kmeans_best_run"])
    rel = [abs(d[0] - r[0]) / r[0] for d, r in zip(dev, ref)]
    dit = [d[1] - r[1] for d, r in zip(dev, ref)]
    lab_dev = im["cluster_labels"].astype(np.int64)
    agree_same_seed = float(np.mean(lab_dev == ref[dev_best][2]))
    agree_best = float(np.mean(lab_dev == ref[ref_best][2]))
    # recall@20 of the candidates built from each clustering (same R1 / kNN lists, the oracle on both sides)
    allv = pipeline._concat([train, test])
    sess_all = allv.session[allv.session_offsets[:-1]]
    r1 = {n: pd.DataFrame({"aid": a, "aid_next": b, f"{n}_rank": r}) for n, (a, b, r) in im["r1"].items()}
    knn = [pd.DataFrame({"aid": a, "aid_next": b, "rank": r}) for a, b, r in im["knn"]]
    sess_te = test.session[test.session_offsets[:-1] - test.session_offsets[0]]
    df_te = test.to_pandas()
    recall = {}
    for side, cl in (("device", lab_dev), ("reference", ref[ref_best][2])):
        pop = oracle_pop.popularity_ranks(allv.session, allv.aid, allv.ts, allv.type,
                                          dict(zip(sess_all.tolist(), cl.tolist())))
        rk = [c for c in pop.columns if c.startswith("rank_")]
        pop = pop[pop[rk].min(axis=1) <= 20][["cl50", "aid"]].reset_index(drop=True)
        scl = pd.DataFrame({"session": sess_te, "cl50": cl[train.n_sessions:]})
        cands = oracle_retrieve.candidates(df_te, r1, knn[0], knn[1], scl, pop)
        recall[side] = oracle_retrieve.recall(cands, labels)
    d20 = {t: recall["device"][t]["top20"] - recall["reference"][t]["top20"] for t in ("clicks", "carts", "orders", "total")}
    metrics = {"rows": len(X), "dev_runs": dev, "ref_runs": [(r[0], r[1]) for r in ref], "rel_inertia": rel,
               "n_iter_diff": dit, "dev_best": dev_best, "ref_best": ref_best, "agree_same_seed": agree_same_seed,
               "agree_ref_best": agree_best, "recall20_device": {t: recall["device"][t]["top20"] for t in d20},
               "recall20_reference": {t: recall["reference"][t]["top20"] for t in d20}, "delta_recall20": d20}
    print("KMEANS_PIN", json.dumps(metrics))
    # the pipeline's own recall (device candidates + k_cand_recall) equals the oracle's on the device clustering
    for t in ("clicks", "carts", "orders", "total"):
        assert abs(res["recall"][t]["top20"] - recall["device"][t]["top20"]) < 1e-12, t
    assert dev_best == ref_best, metrics
    assert agree_same_seed >= 0.999, metrics
    assert rel[dev_best] <= 1e-6, metrics
    assert max(rel) <= 2e-3, metrics
    assert max(abs(x) for x in dit) <= 2, metrics
    assert max(abs(x) for x in d20.values()) <= 1e-4, metrics
