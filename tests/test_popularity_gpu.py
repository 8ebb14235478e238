"""GPU parity of the pop-cluster source and R7 (csrc/popularity.hip) against oracle/popularity.py.

C3 popularity ranks: exact (integer). C1 session embeddings: fp32 sums vs f64 restatement,
tolerance 3e-6 absolute after round6 (one unit in the 6th decimal plus fp32 output rounding;
the reference's own polars f32 summation order is unspecified). C2 KMeans: sklearn 1.2's
algorithm as restated in the oracle (itself pinned against scikit-learn); labels agree on >= 99.9 %
of rows (fp32 vs f64 near-ties), centroids within 1e-3, inertia rel 1e-5. R7: rtol 1e-5 vs f64."""

import numpy as np
import pandas as pd
import pytest

import popularity as oracle_pop
import otto_recommender_amd.synth as synth

pytestmark = pytest.mark.gpu


def _events(n=3000, first=777):
    ev = synth.generate(n, first_session=first)
    return ev


def test_session_embeddings(gpu):
    from otto_recommender_amd import popularity as gp
    ev = _events(1500)
    uni = np.unique(ev.aid)
    rng = np.random.default_rng(1)
    words = uni[rng.random(len(uni)) < 0.9]  # ~10 % of aids have no embedding
    emb = rng.normal(size=(len(words), 100)).astype(np.float32)
    got = gp.compute_sessions_embeddings(ev.session_offsets, ev.aid, ev.ts, ev.type, words, emb).cpu().numpy()
    ref = oracle_pop.sessions_embeddings(ev.session_offsets, ev.aid, ev.ts, ev.type, words, emb)
    np.testing.assert_allclose(got, ref, atol=3e-6, rtol=0)


def _check_kmeans(X, k, n_init=10, agree=0.999, rel=1e-5):
    from otto_recommender_amd import popularity as gp
    km = gp.KMeans(n_clusters=k, max_iter=100, tol=1e-3, random_state=42, n_init=n_init).fit(X)
    lab_ref, C_ref, it_ref, inertia_ref = oracle_pop.kmeans(X, k, n_init=n_init)
    lab = km.labels_.cpu().numpy()
    assert np.mean(lab == lab_ref) >= agree, (np.mean(lab == lab_ref), km.inertia_, inertia_ref)
    if agree >= 0.999:  # (the relocation fixture ends a few boundary rows apart: inertia and labels only)
        np.testing.assert_allclose(km.cluster_centers_.cpu().numpy(), C_ref, atol=1e-3)
    assert abs(km.inertia_ - inertia_ref) <= rel * inertia_ref, (km.inertia_, inertia_ref)
    assert abs(km.n_iter_ - it_ref) <= 2


def test_kmeans_matches_restatement(gpu):
    """sklearn 1.2 KMeans(init='random', n_init='auto'=10) vs the oracle (pinned against the
    installed scikit-learn run by run in tests/test_oracle.py)."""
    rng = np.random.default_rng(2)
    centers = rng.normal(scale=3, size=(12, 100))
    X = (centers[rng.integers(0, 12, 20000)] + rng.normal(size=(20000, 100))).astype(np.float32)
    _check_kmeans(X, 10)


def test_kmeans_lloyd_step_batches_equal_single_steps(gpu, monkeypatch):
    """ottohip_kmeans_lloyd_steps: the device-side stop checks and gating of later steps give the
    same clustering as one step per call (labels, centres, inertia, iterations bit-identical)."""
    from otto_recommender_amd import popularity as gp
    rng = np.random.default_rng(7)
    centers = rng.normal(scale=2, size=(9, 100))
    X = (centers[rng.integers(0, 9, 30000)] + rng.normal(size=(30000, 100))).astype(np.float32)
    X[:4000] = X[0]  # duplicated rows: empty clusters on some seeds (relocation between batches)
    fits = []
    for batch in (1, 10):
        monkeypatch.setattr(gp, "LLOYD_BATCH", batch)
        km = gp.KMeans(n_clusters=9, random_state=42).fit(X)
        fits.append((km.labels_.cpu().numpy(), km.cluster_centers_.cpu().numpy(), km.inertia_, km.n_iter_))
    np.testing.assert_array_equal(fits[0][0], fits[1][0])
    np.testing.assert_array_equal(fits[0][1], fits[1][1])
    assert fits[0][2] == fits[1][2] and fits[0][3] == fits[1][3]


@pytest.mark.parametrize("case", ["sessions_k50", "relocation_k9"])
def test_kmeans_run_lanes_equal_sequential_runs(gpu, monkeypatch, case):
    """KMeans.fit's n_init runs on 2 or 3 host threads (OTTOHIP_KM_LANES: a context and a HIP stream per lane, run
    r on lane r % lanes) give the sequential loop's labels, centres, inertia and iterations bit for bit, incl. the
    empty-cluster relocations (relocation_k9) and the earlier-run rule for the best inertia."""
    from otto_recommender_amd import popularity as gp
    rng = np.random.default_rng(12)
    if case == "sessions_k50":
        ev = synth.generate(30_000, first_session=99)
        words = np.unique(ev.aid)
        emb = synth.embeddings(len(words), seed=1)
        X = gp.compute_sessions_embeddings(ev.session_offsets, ev.aid, ev.ts, ev.type, words, emb).cpu().numpy()
        k, n_init = 50, 5
    else:
        centers = rng.normal(scale=2, size=(9, 100))
        X = (centers[rng.integers(0, 9, 30000)] + rng.normal(size=(30000, 100))).astype(np.float32)
        X[:4000] = X[0]
        k, n_init = 9, 10
    monkeypatch.setenv("OTTOHIP_KM_GROUP", "1")
    fits = []
    for lanes in ("1", "2", "3"):
        monkeypatch.setenv("OTTOHIP_KM_LANES", lanes)
        km = gp.KMeans(n_clusters=k, random_state=7, n_init=n_init).fit(X)
        fits.append((km.labels_.cpu().numpy(), km.cluster_centers_.cpu().numpy(), km.inertia_, km.n_iter_))
    for f in fits[1:]:
        np.testing.assert_array_equal(fits[0][0], f[0])
        np.testing.assert_array_equal(fits[0][1], f[1])
        assert fits[0][2] == f[2] and fits[0][3] == f[3]


@pytest.mark.parametrize("case", ["sessions_k50", "relocation_k9", "blocks_k33"])
def test_kmeans_bounded_steps_equal_full_steps(gpu, monkeypatch, case):
    """The bounded Lloyd steps (rows whose distance bounds separate keep their label unscored,
    csrc/popularity.hip k_km_filter) give bit-identical labels, centres, inertia and iterations to
    scoring every row each step: k = 50 on session embeddings of synthetic sessions (the config-5
    clustering; runs go to max_iter), duplicated rows with empty clusters relocated between steps,
    and k = 33 (the last bound group holds one cluster)."""
    from otto_recommender_amd import popularity as gp
    rng = np.random.default_rng(11)
    if case == "sessions_k50":
        ev = synth.generate(40_000, first_session=4242)
        words = np.unique(ev.aid)
        emb = synth.embeddings(len(words), seed=1)
        X = gp.compute_sessions_embeddings(ev.session_offsets, ev.aid, ev.ts, ev.type, words, emb).cpu().numpy()
        k, n_init = 50, 2
    elif case == "relocation_k9":
        centers = rng.normal(scale=2, size=(9, 100))
        X = (centers[rng.integers(0, 9, 30000)] + rng.normal(size=(30000, 100))).astype(np.float32)
        X[:4000] = X[0]
        k, n_init = 9, 10
    else:
        centers = rng.normal(scale=3, size=(40, 100))
        X = (centers[rng.integers(0, 40, 20000)] + rng.normal(size=(20000, 100))).astype(np.float32)
        k, n_init = 33, 3
    fits = []
    monkeypatch.setenv("OTTOHIP_KM_GROUP", "1")  # the bounded single-run steps (lockstep groups carry no bounds)
    for bounds in ("0", "1"):
        monkeypatch.setenv("OTTOHIP_KM_BOUNDS", bounds)
        km = gp.KMeans(n_clusters=k, random_state=42, n_init=n_init).fit(X)
        fits.append((km.labels_.cpu().numpy(), km.cluster_centers_.cpu().numpy(), km.inertia_, km.n_iter_))
    np.testing.assert_array_equal(fits[0][0], fits[1][0])
    np.testing.assert_array_equal(fits[0][1], fits[1][1])
    assert fits[0][2] == fits[1][2] and fits[0][3] == fits[1][3]


@pytest.mark.parametrize("case", ["sessions_k50", "relocation_k9", "blocks_k33", "one_block_k20"])
def test_kmeans_split_precision_steps_equal_exact_steps(gpu, monkeypatch, case):
    """The split-precision E-step (bf16 hi/lo MFMA pass deciding every row whose two best scores are
    separated beyond the error bound, the exact f32 kernel on the near ties; csrc/popularity.hip
    k_km_assign_split) gives bit-identical labels, centres, inertia and iterations to the exact f32
    kernel on every row: k = 50 on session embeddings of synthetic sessions (the config-5 clustering,
    runs reach max_iter), duplicated rows with empty clusters relocated, k = 33 and k = 20."""
    from otto_recommender_amd import popularity as gp
    rng = np.random.default_rng(11)
    if case == "sessions_k50":
        ev = synth.generate(40_000, first_session=4242)
        words = np.unique(ev.aid)
        emb = synth.embeddings(len(words), seed=1)
        X = gp.compute_sessions_embeddings(ev.session_offsets, ev.aid, ev.ts, ev.type, words, emb).cpu().numpy()
        k, n_init = 50, 2
    elif case == "relocation_k9":
        centers = rng.normal(scale=2, size=(9, 100))
        X = (centers[rng.integers(0, 9, 30000)] + rng.normal(size=(30000, 100))).astype(np.float32)
        X[:4000] = X[0]
        k, n_init = 9, 10
    else:
        k = 33 if case == "blocks_k33" else 20
        centers = rng.normal(scale=3, size=(40, 100))
        X = (centers[rng.integers(0, 40, 20000)] + rng.normal(size=(20000, 100))).astype(np.float32)
        n_init = 3
    fits = []
    monkeypatch.setenv("OTTOHIP_KM_GROUP", "1")  # the single-run steps (lockstep groups always take the split pass)
    # the exact kernel on every row; the split pass + the exact kernel on near ties, the label changes through
    # the move lists (k_km_ties) and through the split pass's own LDS sums (OTTOHIP_KM_MV=0)
    for split, mv in (("0", "1"), ("1", "1"), ("1", "0")):
        monkeypatch.setenv("OTTOHIP_KM_SPLIT", split)
        monkeypatch.setenv("OTTOHIP_KM_MV", mv)
        km = gp.KMeans(n_clusters=k, random_state=42, n_init=n_init).fit(X)
        fits.append((km.labels_.cpu().numpy(), km.cluster_centers_.cpu().numpy(), km.inertia_, km.n_iter_))
    for f in fits[1:]:
        np.testing.assert_array_equal(fits[0][0], f[0])
        np.testing.assert_array_equal(fits[0][1], f[1])
        assert fits[0][2] == f[2] and fits[0][3] == f[3]


def test_kmeans_half_rows_refused_outside_f16_range(gpu, monkeypatch):
    """A feature scaled to ~1e5 is outside f16's range (65504): ottohip_kmeans_attach_half refuses the f16 copy
    (ELIMIT, not an inf score that fminf would drop), KMeans.fit then scores the f32 rows, and the result is
    bit-identical to OTTOHIP_KM_H16=0 and to the unbounded steps, fit after fit. (Both n_init runs reach one
    partition here: the run kept is decided by an exact inertia tie, so the inertia sum must be deterministic.)"""
    import torch
    from otto_recommender_amd import popularity as gp, _lib
    rng = np.random.default_rng(23)
    centers = rng.normal(scale=3, size=(12, 100))
    X = (centers[rng.integers(0, 12, 12000)] + rng.normal(size=(12000, 100))).astype(np.float32)
    X[:, 7] *= 4e4  # |x| up to ~1e5 in one column
    Xd = torch.from_numpy(X).cuda()
    ctx = _lib.context()
    rc = _lib.load().ottohip_kmeans_attach_half(ctx.h, _lib.ptr(Xd), X.shape[0], X.shape[1], None)
    assert rc == _lib.OTTOHIP_ELIMIT, rc
    assert b"f16" in _lib.load().ottohip_last_error()
    fits = []
    monkeypatch.setenv("OTTOHIP_KM_GROUP", "1")
    for h16, bounds in (("0", "0"), ("0", "1"), ("1", "1"), ("1", "1")):
        monkeypatch.setenv("OTTOHIP_KM_H16", h16)
        monkeypatch.setenv("OTTOHIP_KM_BOUNDS", bounds)
        km = gp.KMeans(n_clusters=10, random_state=42, n_init=2).fit(X)
        fits.append((km.labels_.cpu().numpy(), km.cluster_centers_.cpu().numpy(), km.inertia_, km.n_iter_))
    for f in fits[1:]:
        np.testing.assert_array_equal(fits[0][0], f[0])
        np.testing.assert_array_equal(fits[0][1], f[1])
        assert fits[0][2] == f[2] and fits[0][3] == f[3]
    assert len(np.unique(fits[0][0])) == 10


@pytest.mark.parametrize("case", ["sessions_k50", "relocation_k40", "blocks_k33"])
def test_kmeans_lockstep_equals_single_runs(gpu, monkeypatch, case):
    """n_init runs in lockstep over one read of X per Lloyd step (ottohip_kmeans_lloyd_steps_multi, groups of
    2, 3 and 4 runs) give bit-identical labels, centres, inertia and iterations to the runs one at a time
    (with distance bounds): k = 50 on session embeddings (runs reach max_iter; n_init = 5: groups of 4 + 1,
    3 + 2, 2 + 2 + 1), duplicated rows with empty clusters relocated in one run of a group while the others
    keep stepping (k = 40), and k = 33 with runs that converge at different steps."""
    from otto_recommender_amd import popularity as gp
    rng = np.random.default_rng(19)
    if case == "sessions_k50":
        ev = synth.generate(40_000, first_session=999)
        words = np.unique(ev.aid)
        emb = synth.embeddings(len(words), seed=1)
        X = gp.compute_sessions_embeddings(ev.session_offsets, ev.aid, ev.ts, ev.type, words, emb).cpu().numpy()
        k, n_init = 50, 5
    elif case == "relocation_k40":
        centers = rng.normal(scale=2, size=(40, 100))
        X = (centers[rng.integers(0, 40, 30000)] + rng.normal(size=(30000, 100))).astype(np.float32)
        X[:6000] = X[0]
        k, n_init = 40, 4
    else:
        centers = rng.normal(scale=3, size=(40, 100))
        X = (centers[rng.integers(0, 40, 20000)] + rng.normal(size=(20000, 100))).astype(np.float32)
        k, n_init = 33, 4
    fits = []
    for grp in ("1", "2", "3", "4"):
        monkeypatch.setenv("OTTOHIP_KM_GROUP", grp)
        km = gp.KMeans(n_clusters=k, random_state=42, n_init=n_init).fit(X)
        fits.append((km.labels_.cpu().numpy(), km.cluster_centers_.cpu().numpy(), km.inertia_, km.n_iter_))
    for f in fits[1:]:
        np.testing.assert_array_equal(fits[0][0], f[0])
        np.testing.assert_array_equal(fits[0][1], f[1])
        assert fits[0][2] == f[2] and fits[0][3] == f[3]


def test_kmeans_empty_cluster_relocation(gpu):
    """a third of the rows identical: seeds collide, clusters empty out and are relocated to the
    farthest rows (_relocate_empty_clusters_dense)"""
    rng = np.random.default_rng(4)
    centers = rng.normal(scale=3, size=(9, 100))
    X = (centers[rng.integers(0, 9, 6000)] + rng.normal(size=(6000, 100))).astype(np.float32)
    X[:2000] = X[0]
    # fp32 distances reorder near-equal candidates of the relocation against the f64 oracle: a few
    # boundary rows may follow (measured 9 of 6000)
    _check_kmeans(X, 12, agree=0.995, rel=1e-4)


def test_kmeans_two_centroid_blocks(gpu):
    """k > 32 (two 32-centroid blocks in the MFMA variant, 56 padded columns in the VALU one)."""
    rng = np.random.default_rng(5)
    centers = rng.normal(scale=3, size=(50, 100))
    X = (centers[rng.integers(0, 50, 12000)] + rng.normal(size=(12000, 100))).astype(np.float32)
    _check_kmeans(X, 45, n_init=2)


def test_popularity_ranks_exact(gpu):
    from otto_recommender_amd import popularity as gp
    ev = _events(4000, first=12345)
    sess = ev.session[ev.session_offsets[:-1]]
    rng = np.random.default_rng(3)
    cl = rng.integers(0, 5, len(sess)).astype(np.int32)
    got = gp.count_popularity(ev.session_offsets, ev.aid, ev.ts, ev.type, cl, 5, keep_top_k=20)
    ref = oracle_pop.popularity_ranks(ev.session, ev.aid, ev.ts, ev.type, dict(zip(sess.tolist(), cl.tolist())))
    assert list(got.columns) == list(ref.columns)
    assert len(got) == len(ref)
    for c in got.columns:
        np.testing.assert_array_equal(got[c].to_numpy().astype(np.int64), ref[c].to_numpy().astype(np.int64), err_msg=c)
    # one global cluster (cl1)
    g1 = gp.count_popularity(ev.session_offsets, ev.aid, ev.ts, ev.type, np.zeros(len(sess), np.int32), 1,
                             suffix="cl1")
    r1 = oracle_pop.popularity_ranks(ev.session, ev.aid, ev.ts, ev.type, {int(s): 0 for s in sess}, suffix="cl1")
    np.testing.assert_array_equal(g1["aid"].to_numpy(), r1["aid"].to_numpy())


@pytest.mark.parametrize("dim", [100, 128, 64, 30])  # 16-lane float4 kernel; 30: the one-lane kernel
def test_session_item_similarity(gpu, dim):
    from otto_recommender_amd import popularity as gp
    rng = np.random.default_rng(4)
    words = np.arange(0, 5000, 2, dtype=np.int32)
    emb = rng.normal(size=(len(words), dim)).astype(np.float32)
    S = 300
    off = np.concatenate([[0], np.cumsum(rng.integers(0, 40, S))]).astype(np.int64)
    nxt = rng.integers(0, 5000, off[-1]).astype(np.int32)
    se = rng.normal(size=(S, dim)).astype(np.float32)
    has = (rng.random(S) < 0.9).astype(np.uint8)
    cos, eu = (x.cpu().numpy() for x in gp.session_item_similarity(off, nxt, se, words, emb, has))
    sidx = np.repeat(np.arange(S), np.diff(off))
    ok = (nxt % 2 == 0) & (has[sidx] == 1)
    rc, re = oracle_pop.similarity(se[sidx].astype(np.float64), emb[np.minimum(nxt // 2, len(words) - 1)].astype(np.float64))
    np.testing.assert_allclose(cos[ok], rc[ok], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(eu[ok], re[ok], rtol=1e-5)
    assert np.all(cos[~ok] == 0) and np.all(eu[~ok] == -1)


def test_kmeans_bounds_invalidated_by_other_label_writers(gpu, monkeypatch):
    """The distance bounds carried between ottohip_kmeans_lloyd_steps calls (csrc/popularity.hip
    k_km_filter) are dropped when another entry point writes the labels (ottohip_kmeans_partial here)
    and when the centroids move outside the batched steps (ottohip_kmeans_update): the same call
    sequence gives bit-identical labels, centroids and stop reasons with and without the bounds."""
    import ctypes
    import torch
    from otto_recommender_amd import _lib
    rng = np.random.default_rng(21)
    centers = rng.normal(scale=2, size=(20, 64))
    X = torch.from_numpy((centers[rng.integers(0, 20, 50_000)] + rng.normal(size=(50_000, 64))).astype(np.float32)).cuda()
    n, dim, k = X.shape[0], X.shape[1], 20
    lib, ctx = _lib.load(), _lib.context()
    sh = _lib.stream_handle()
    runs = []
    for bounds in ("0", "1"):
        monkeypatch.setenv("OTTOHIP_KM_BOUNDS", bounds)
        perm = np.random.default_rng(5).permutation(n)[:k]
        C = X[torch.from_numpy(perm).cuda()].clone()
        labels = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        sums = torch.zeros(k * dim, dtype=torch.int64, device="cuda")
        counts = torch.zeros(k, dtype=torch.int64, device="cuda")
        out = (ctypes.c_double * 6)()
        trace = []
        for phase in range(4):
            _lib.check(lib.ottohip_kmeans_lloyd_steps(ctx.h, _lib.ptr(X), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                                      _lib.ptr(sums), _lib.ptr(counts), 3, 0.0, out, sh))
            trace.append((int(out[4]), int(out[5]), int(out[1])))
            if phase == 1:  # an outside label writer, then an outside centroid update
                inr, chg = ctypes.c_double(), ctypes.c_int64()
                _lib.check(lib.ottohip_kmeans_partial(ctx.h, _lib.ptr(X), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                                      _lib.ptr(sums), _lib.ptr(counts), ctypes.byref(inr),
                                                      ctypes.byref(chg), sh))
                shift = ctypes.c_double()
                _lib.check(lib.ottohip_kmeans_update(ctx.h, _lib.ptr(C), _lib.ptr(sums), _lib.ptr(counts), k, dim,
                                                     ctypes.byref(shift), sh))
        torch.cuda.synchronize()
        runs.append((labels.cpu().numpy(), C.cpu().numpy(), trace))
    np.testing.assert_array_equal(runs[0][0], runs[1][0])
    np.testing.assert_array_equal(runs[0][1], runs[1][1])
    assert runs[0][2] == runs[1][2]
