"""Multi-process GPU tests of the PRODUCT multi-GPU path (dist.py over torch.distributed):
2 fresh rank processes (tests/dist_rank.py, gloo backend, both on cuda:0), checked here against
the oracle. BASELINE configs[3] at test scale: each rank counts its dealt whole files, the pair
words go to owner(aid) in the all-to-all-v, and every shard must equal the oracle's cross-file
merge (model/count_co_events.py:168, count_ge2 of :131-132) restricted to owner(aid) == rank.
The sharded A6 (concat_files_w_stats, :103-181: filter, part-wise branch, threshold, global
head cut) must give every rank the single-GPU table; the per-rank slices must partition it."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import covis as oracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = list(oracle.REFERENCE_RULES)
SYM_RULES = {"click_to_click", "cart_to_cart", "buy_to_buy"}  # stored once per unordered pair in the shards


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(mode, cfg, tmp_path, world=2, timeout=240):
    port = _free_port()
    procs, outs = [], []
    for r in range(world):
        out = str(tmp_path / f"rank{r}.npz")
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_rank.py"), mode, out,
                                       json.dumps(cfg)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-4000:]
    return [dict(np.load(o)) for o in outs]


def _owner(aid, world):
    a = np.asarray(aid).astype(np.uint64)
    return (((a * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)) * np.uint64(world)) >> np.uint64(32)


def test_covis_sharded_two_ranks(gpu, tmp_path):
    cfg = {"sessions": 18_000, "per_file": 1_500, "first_session": 5150,
           "merges": {
               "reference": {},
               # (1) + (2) for click_to_click, global head cut with ties for every rule
               "scaled": {"click_filter_rows": 200_000, "max_rows_groupby": 250_000, "optim_rows": 150_000,
                          "max_pairs": 700}}}
    _check_covis_sharded(cfg, tmp_path, world=2)


def test_covis_sharded_four_ranks(gpu, tmp_path):
    """The same at world 4 (SURVEY.md §8(e) runs 1/2/4/8): 16 files dealt by weight, branch (2)
    parts of two to three files (ranks hold no file of some parts; the boundary keys come from
    the file's holder), the global head cut on a count whose ties live on >= 3 owners, and the
    exchange in 1 / 3 chunks and in global file batches of 2 (_count_sharded_batches)."""
    from otto_recommender_amd.covis import part_plan
    cfg = {"sessions": 24_000, "per_file": 1_500, "first_session": 31337,
           "merges": {
               "scaled": {"click_filter_rows": 10**9, "max_rows_groupby": 1_500_000, "optim_rows": 600_000,
                          "max_pairs": 2_000},
               "filtered": {"click_filter_rows": 100_000, "max_rows_groupby": 300_000, "optim_rows": 120_000,
                            "max_pairs": 5_000}}}
    res, per_file = _check_covis_sharded(cfg, tmp_path, world=4)
    files_of = [set(r["files"].tolist()) for r in res]
    kw = cfg["merges"]["scaled"]
    n = "click_to_click"
    R = np.array([len(p[n][0]) for p in per_file])
    plan = part_plan(R, -(-int(R.sum()) // kw["optim_rows"]))
    idle = sum(1 for fa, _, fb, _ in plan for f in files_of if not f & set(range(fa, fb + 1)))
    assert len(plan) > 1 and idle > 0, "no rank without files of a part"
    # ties at the global cut spread over >= 3 owners
    full = oracle.concat_files_w_stats(n, [p[n] for p in per_file], **dict(kw, max_pairs=10**9))
    cstar = int(full[2][kw["max_pairs"] - 1])
    assert len(set(_owner(full[0][full[2] == cstar], 4).tolist())) >= 3


def test_covis_sharded_eight_ranks(gpu, tmp_path):
    """BASELINE configs[3] at world 8 (8 fresh rank processes on cuda:0, gloo): the G = 8 owner hash,
    an 8-way all-to-all-v of pair words and row pieces, branch (2) parts of a few files each (most
    ranks hold no file of a given part; the boundary keys come from the file's holder), and the global
    head cut on a count whose ties live on >= 5 of the 8 owners; every shard, final table and slice
    set against the oracle (model/count_co_events.py:103-181)."""
    from otto_recommender_amd.covis import part_plan
    cfg = {"sessions": 32_000, "per_file": 1_000, "first_session": 424_242,
           "merges": {
               "scaled": {"click_filter_rows": 10**9, "max_rows_groupby": 1_500_000, "optim_rows": 700_000,
                          "max_pairs": 3_000},
               "filtered": {"click_filter_rows": 100_000, "max_rows_groupby": 250_000, "optim_rows": 120_000,
                            "max_pairs": 8_000}}}
    res, per_file = _check_covis_sharded(cfg, tmp_path, world=8, timeout=420)
    files_of = [set(r["files"].tolist()) for r in res]
    n = "click_to_click"
    for tag in ("scaled", "filtered"):
        kw = cfg["merges"][tag]
        use_ge2 = sum(len(p[n][0]) for p in per_file) > kw["click_filter_rows"]
        R = np.array([int((p[n][2] >= 2).sum()) if use_ge2 else len(p[n][0]) for p in per_file])
        assert R.sum() > kw["max_rows_groupby"], tag  # branch (2) is taken
        plan = part_plan(R, -(-int(R.sum()) // kw["optim_rows"]))
        idle = sum(1 for fa, _, fb, _ in plan for f in files_of if not f & set(range(fa, fb + 1)))
        assert len(plan) > 2 and idle > len(plan), tag
    # ties at the global cut spread over >= 5 owners
    kw = cfg["merges"]["scaled"]
    full = oracle.concat_files_w_stats(n, [p[n] for p in per_file], **dict(kw, max_pairs=10**9))
    cstar = int(full[2][kw["max_pairs"] - 1])
    assert len(set(_owner(full[0][full[2] == cstar], 8).tolist())) >= 5


@pytest.mark.slow
def test_covis_sharded_full_size_config4(gpu, tmp_path):
    """BASELINE configs[3] at its real size: the 220 M-event stream (135 files of 100k sessions) session-sharded
    over 8 fresh rank processes on cuda:0 (gloo), files dealt by Σ n_s², the sharded count of all five rules
    (owner all-to-all-v of pair words in 2 event-balanced chunks) and the sharded A6 of every rule, including
    branch (2) of click_to_click at N = 694 M split over the owners (model/count_co_events.py:80-181).
    The shard digests are wrapping u64 sums over rows, so they add over the owners to the single-table digests
    of tests/golden/digest_220m.json (C oracle, make_golden.py --full); every rank's A6 output equals the
    golden rows / sum / sha256 and is identical on all ranks; the exchange's per-peer sizes stay below 2^31."""
    import torch
    g = json.load(open(os.path.join(HERE, "golden", "digest_220m.json")))
    gpu.trim()  # this process's cached device buffers (earlier full-size tests) are not needed by the ranks
    torch.cuda.empty_cache()
    world = 8
    res = _launch("covis_full", {"seed": g["seed"], "sessions": g["sessions"]}, tmp_path, world=world, timeout=800)
    files = np.concatenate([r["files"] for r in res])
    assert sorted(files.tolist()) == list(range(g["files"]))
    assert sum(int(r["events"][0]) for r in res) == g["events"]
    M = (1 << 64) - 1
    for n in NAMES:
        ref = g["rules"][n]
        dig = [sum(int(r[f"digest/{n}"][i]) for r in res) & M for i in range(5)]
        assert (dig[0], dig[1], dig[2], dig[3]) == (ref["d_count"], ref["d_count_ge2"], ref["pairs"], ref["pairs_ge2"]), n
        for r in res:  # the global per-file statistics on every rank
            st = r[f"stats/{n}"]
            assert (int(st[0]), int(st[1])) == (ref["file_rows"], ref["file_rows_ge2"]), n
        assert sum(int(r[f"stats/{n}"][3]) for r in res) == ref["pairs"], n
        got = oracle.canonical_digest({n: tuple(res[0][f"final/{n}"][:, i] for i in range(3))})[n]
        a6 = g["a6"][n]
        assert (got["rows"], got["sum"], got["sha256"]) == (a6["rows"], a6["sum"], a6["sha256"]), n
        assert len({bytes(r[f"final_sha/{n}"]) for r in res}) == 1, n  # identical on every rank
    x = np.stack([r["exchange"] for r in res])
    assert int(x[:, 1].max()) < 2 ** 31 and int(x[:, 3].max()) < 2 ** 31
    # every word sent is received; the symmetric rules' pairs travel once per unordered pair
    assert int(x[:, 0].sum()) == int(x[:, 2].sum()) < sum(g["rules"][n]["pairs"] for n in NAMES)
    print("config4 full: count_s", [round(float(r["count_s"][0]), 2) for r in res],
          "a6_s", {n: round(max(float(r[f"a6_s/{n}"][0]) for r in res), 2) for n in NAMES},
          "words recv per rank", x[:, 2].tolist())


def test_covis_sharded_part_boundary_on_file_end(gpu, tmp_path):
    """Branch (2) with a part boundary exactly on a file end next to one that cuts a file: files of
    400, 400, 600, 600, 400 click_to_click rows (tests/dist_rank.structured_events) in 3 parts of 800 rows, so
    part 0 is files 0-1 whole (no key cut) and parts 1-2 meet inside file 3. Every part must use one storage
    mode (dist.concat_files_w_stats_sharded counts all parts with sym=False): a symmetric part 0 would keep the
    mirror (j + 5000, j) at owner(j) while parts 1-2 hold it at owner(j + 5000), and the owner-local merge of
    the parts would leave the key split over two ranks (count 18 on one, 27 on the other, instead of 45)."""
    from otto_recommender_amd.covis import part_plan
    cfg = {"structured": [100, 100, 150, 150, 100], "rules": ["click_to_click"],
           "merges": {"boundary": {"click_filter_rows": 10**9, "max_rows_groupby": 2_000, "optim_rows": 800,
                                   "max_pairs": 10**6}}}
    plan = part_plan([400, 400, 600, 600, 400], 3)
    assert plan[:2] == [(0, 0, 1, 400), (2, 0, 3, 200)], plan  # part 0: whole files; part 1 ends inside file 3
    res, per_file = _check_covis_sharded(cfg, tmp_path, world=2)
    assert [len(p["click_to_click"][0]) for p in per_file] == [400, 400, 600, 600, 400]
    f = res[0]["final/boundary/click_to_click"]
    m = (f[:, 0] >= 5000) & (f[:, 1] < 100)
    assert m.sum() == 100 and set(f[m, 2].tolist()) == {45}  # (j + 5000, j) summed over all three parts


def _check_covis_sharded(cfg, tmp_path, world, timeout=240):
    import otto_recommender_amd.synth as synth
    res = _launch("covis", cfg, tmp_path, world=world, timeout=timeout)
    if "structured" in cfg:
        from dist_rank import structured_events
        ev, fb = structured_events(cfg)
    else:
        ev = synth.generate(cfg["sessions"], first_session=cfg["first_session"])
        fb = synth.file_session_bounds(ev.n_sessions, per_file=cfg["per_file"])
    per_file = oracle.count_co_events_files(ev.session_offsets, ev.aid, ev.ts, ev.type, fb)
    files = np.concatenate([r["files"] for r in res])
    assert sorted(files.tolist()) == list(range(len(fb) - 1)) and all(len(r["files"]) for r in res)
    for n in NAMES:
        a = np.concatenate([p[n][0] for p in per_file]); b = np.concatenate([p[n][1] for p in per_file])
        c = np.concatenate([p[n][2] for p in per_file]).astype(np.int64)
        ra, rb, rc = oracle._groupby_sum(a, b, c)
        _, _, rg = oracle._groupby_sum(a, b, np.where(c >= 2, c, 0))
        # a symmetric rule is exchanged once per unordered pair: owner(min(aid, aid_next)) holds both orders
        own = _owner(np.minimum(ra, rb) if n in SYM_RULES else ra, world)
        for r, got in enumerate(res):
            m = own == r
            np.testing.assert_array_equal(got[f"shard/{n}"], np.stack([ra[m], rb[m], rc[m], rg[m]], 1).astype(np.int64),
                                          err_msg=f"shard {r} {n}")
            np.testing.assert_array_equal(got[f"stats/{n}"], [len(a), int((c >= 2).sum())])
        for tag, kw in cfg["merges"].items():
            if n not in cfg.get("rules", NAMES):
                continue
            ref = np.stack([np.asarray(x, np.int64) for x in
                            oracle.concat_files_w_stats(n, [p[n] for p in per_file], **kw)], 1)
            for r, got in enumerate(res):
                np.testing.assert_array_equal(got[f"final/{tag}/{n}"], ref, err_msg=f"final {tag} rank {r} {n}")
            sl = np.concatenate([got[f"slice/{tag}/{n}"] for got in res])
            o = np.lexsort((sl[:, 1], sl[:, 0], -sl[:, 2]))
            np.testing.assert_array_equal(sl[o], ref, err_msg=f"slices {tag} {n}")
            if tag == "scaled" and n in ("click_to_click", "click_to_cart_or_buy"):
                assert len(ref) == kw["max_pairs"], (n, len(ref))  # the global cut is active
    return res, per_file


def test_pipeline_two_ranks_equals_one_gpu(gpu, tmp_path):
    """BASELINE configs[4] split over 2 ranks (pipeline.run(group=...)): train/test files dealt per
    folder, sharded A6 per folder, kNN queries split, KMeans rows sharded with all-reduced exact
    sums, C3 counters all-reduced, candidates per rank. Every shard-level output must equal the
    1-GPU run on the same input: A7 tables, kNN lists, cluster labels, pop lists, the union of
    the per-rank candidates, and recall."""
    cfg = {"sessions": 30_000, "first_session": 808, "clusters": 6, "iters": 15, "queries": 20_000, "n_init": 2,
           "per_file": 2_500}
    _check_pipeline_ranks(cfg, tmp_path, world=2)


def test_pipeline_eight_ranks_equals_one_gpu(gpu, tmp_path):
    """BASELINE configs[4] at world 8 (8 fresh rank processes on cuda:0): the same checks as the
    2-rank test, with files small enough that every rank holds train files and some rank holds no
    test file (no candidate sessions of its own)."""
    cfg = {"sessions": 24_000, "first_session": 9090, "clusters": 6, "iters": 12, "queries": 16_000, "n_init": 2,
           "per_file": 1_000}
    res = _check_pipeline_ranks(cfg, tmp_path, world=8)
    assert min(int(r["n_test_files"][0]) for r in res) == 0  # a rank without test files (no candidates of its own)


def _check_pipeline_ranks(cfg, tmp_path, world):
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import pipeline as pl
    res = _launch("pipeline", cfg, tmp_path, world=world, timeout=400)
    ev = synth.generate(cfg["sessions"], first_session=cfg["first_session"])
    train, test, labels = synth.split_test_labels(ev)
    words = synth.item_words()
    emb = synth.embeddings(len(words), seed=1)
    emb2 = synth.embeddings(len(words), seed=3)
    one = pl.run(train, test, labels, words, emb, words, emb2, n_clusters=cfg["clusters"], kmeans_iter=cfg["iters"],
                 knn_queries=cfg["queries"], keep_tables=True, n_init=cfg["n_init"], per_file=cfg["per_file"])
    im = one["intermediates"]
    for r in res:
        for n, v in im["tables"].items():
            np.testing.assert_array_equal(r[f"table/{n}"], np.stack([np.asarray(x, np.int64) for x in v], 1), err_msg=n)
        for i, v in enumerate(im["knn"]):
            np.testing.assert_array_equal(r[f"knn/{i}"], np.stack([np.asarray(x, np.int64) for x in v], 1))
        np.testing.assert_array_equal(r["pop"], im["pop"].to_numpy().astype(np.int64))
        assert r["candidates_total"][0] == one["candidates"]
        ref_rec = [one["recall"][t][k] for t in ("clicks", "carts", "orders", "total")
                   for k in ("top20", "top100", "top200", "topall")]
        np.testing.assert_allclose(r["recall"], ref_rec, rtol=0, atol=1e-12)
    rows = np.concatenate([r["cluster_rows"] for r in res])
    lab = np.concatenate([r["cluster_labels"] for r in res])
    assert sorted(rows.tolist()) == list(range(len(im["cluster_labels"])))
    np.testing.assert_array_equal(lab[np.argsort(rows)], im["cluster_labels"])
    cols = list(res[0]["cand_cols"])
    got = np.concatenate([r["cand"] for r in res])
    got = got[np.lexsort((got[:, 1], got[:, cols.index("ts_order_aid")], got[:, 0]))]
    ref = im["candidates"][cols].to_numpy().astype(np.int64)
    ref = ref[np.lexsort((ref[:, 1], ref[:, cols.index("ts_order_aid")], ref[:, 0]))]
    np.testing.assert_array_equal(got, ref)
    assert sum(int(r["candidates_total"][1]) for r in res) == one["candidates"]
    return res
