"""Regenerates the committed golden fixtures (run from the repo root):

    python tests/golden/make_golden.py

kat_appendix_a.json  SURVEY.md Appendix A known-answer test (hand-derived, checked by both
                     restatements: oracle/covis_oracle.c and oracle/covis_pandas.py)
covis_1k.npz         five per-rule tables of the first 1,000 otto-synth sessions (seed 0),
                     produced by the op-for-op pandas restatement of count_co_events.py:17-94
digest_220m.json     (--full) BASELINE configs[1] at full size: per rule the order-independent
                     checksums of the merged table, from per-file oracle tables (linear sums);
                     (--full-a6) under "a6" the canonical digests of every rule's A6 output
                     (concat_files_w_stats incl. branch (2) for click_to_click), streamed
digest_config5.json  (--config5) BASELINE configs[4] at full size (12.9 M sessions): canonical digests of
                     the A7 train+test tables of the rules without the part-wise branch
digests.json         sha256 of canonical (aid, aid_next, count) streams:
                     config-1 slice (first 10,000 sessions, click_to_click) and a 3-file slice
                     (300,000 sessions, all five rules, per-file tables merged with c / c_ge2)
The reference itself cannot run here (polars absent): parity is unpinned
against it; these fixtures pin the build's restatement.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import covis  # noqa: E402
import covis_pandas  # noqa: E402
import otto_recommender_amd.synth as synth  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

KAT_EVENTS = [(1, 10, 0, 0), (1, 20, 100, 0), (1, 10, 200, 1), (1, 30, 50000, 0), (1, 20, 90000, 2),
              (2, 10, 1000, 0), (2, 10, 1000, 0), (2, 10, 1060, 0), (2, 20, 1100, 1), (2, 20, 1100, 2),
              (3, 40, 0, 0), (3, 50, 43200, 0), (3, 60, 86401, 0)]
KAT_EXPECTED = {
    "click_to_click": [[10, 10, 2], [10, 20, 1], [20, 10, 1], [40, 50, 1], [50, 40, 1]],
    "click_to_cart_or_buy": [[10, 10, 1], [10, 20, 4], [20, 10, 1], [30, 10, 1], [30, 20, 1]],
    "cart_to_cart": [],
    "cart_to_buy": [[20, 20, 1]],
    "buy_to_buy": [],
}


def merged_tables(per_file):
    """sum over files of count and of per-file counts >= 2 (the build's c / c_ge2)."""
    out = {}
    for name in per_file[0]:
        a = np.concatenate([p[name][0] for p in per_file]); b = np.concatenate([p[name][1] for p in per_file])
        c = np.concatenate([p[name][2] for p in per_file]).astype(np.int64)
        ga, gb, gc = covis._groupby_sum(a, b, c)
        _, _, g2 = covis._groupby_sum(a, b, np.where(c >= 2, c, 0))
        out[name] = (ga, gb, gc, g2)
    return out


def main():
    a = np.array(KAT_EVENTS)
    ev = synth.events_from_columns(a[:, 0], a[:, 1], a[:, 2], a[:, 3])
    got = covis.count_co_events_file(ev.session_offsets, ev.aid, ev.ts, ev.type)
    got = {k: [[int(x), int(y), int(c)] for x, y, c in zip(*v)] for k, v in got.items()}
    assert got == KAT_EXPECTED, got
    with open(os.path.join(HERE, "kat_appendix_a.json"), "w") as f:
        json.dump({"events": KAT_EVENTS, "expected": KAT_EXPECTED}, f, indent=1)

    ev = synth.generate(1000)
    tp = covis_pandas.as_arrays(covis_pandas.count_file(ev.to_pandas()))
    arrs = {}
    for k, (x, y, c) in tp.items():
        arrs[f"{k}.aid"], arrs[f"{k}.aid_next"], arrs[f"{k}.count"] = x, y, c
    np.savez_compressed(os.path.join(HERE, "covis_1k.npz"), **arrs)

    dig = {}
    ev = synth.generate(10_000)
    t = covis.count_co_events_file(ev.session_offsets, ev.aid, ev.ts, ev.type,
                                   rules={"click_to_click": covis.REFERENCE_RULES["click_to_click"]})
    dig["config1_10k_click_to_click"] = covis.canonical_digest(t)
    ev = synth.generate(300_000)
    fb = synth.file_session_bounds(ev.n_sessions)
    per_file = covis.count_co_events_files(ev.session_offsets, ev.aid, ev.ts, ev.type, fb)
    m = merged_tables(per_file)
    dig["slice_300k_3files_count"] = covis.canonical_digest({k: v[:3] for k, v in m.items()})
    dig["slice_300k_3files_count_ge2"] = covis.canonical_digest(
        {k: (v[0][v[3] > 0], v[1][v[3] > 0], v[3][v[3] > 0]) for k, v in m.items()})
    dig["slice_300k_3files_file_rows"] = {k: int(sum(len(p[k][0]) for p in per_file)) for k in m}
    dig["slice_300k_3files_file_rows_ge2"] = {k: int(sum(int((p[k][2] >= 2).sum()) for p in per_file)) for k in m}
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(dig, f, indent=1, sort_keys=True)
    # the streamed A6 of config5_c2c equals the in-memory restatement (branches (1), (2), (3))
    for n in ("click_to_click", "click_to_cart_or_buy"):
        full = [p[n] for p in per_file]
        ge2 = [tuple(x[t[2] >= 2] for x in t) for t in full]
        kw = dict(max_rows_groupby=1_500_000, optim_rows=700_000, max_pairs=50_000, click_filter_rows=2_000_000)
        want = covis.concat_files_w_stats(n, full, **kw)
        got = concat_files_w_stats_streamed(n, full, ge2, sum(len(t[0]) for t in full), **kw)
        for x, y in zip(want, got):
            assert np.array_equal(x, y), n




def full_digest(target_events: int = 220_000_000, seed: int = 0, threads: int = 0) -> dict:
    """BASELINE configs[1] (220M events, 100k-session files, all five rules): per rule the linear
    checksums of every file's table (oracle/covis.py files_digest, OpenMP over files), which equal
    ottohip_table_digest of the build's merged table. Written to digest_220m.json."""
    n_sess, n_ev = synth.sessions_for_events(target_events, 0, seed)
    ev = synth.generate(n_sess, 0, seed)
    fb = synth.file_session_bounds(n_sess)
    d = covis.files_digest(ev.session_offsets, ev.aid, ev.ts, ev.type, fb, threads)
    return {"events": int(ev.n_events), "sessions": int(n_sess), "files": int(len(fb) - 1), "seed": seed,
            "rules": d, "note": "d_* are wrapping u64 sums of splitmix64(rule<<48|aid<<24|aid_next ^ seed) x count "
                                 "(seed 1) / x count_ge2 (seed 2); pairs = sum count; file_rows = per-file rows"}


def _count_file_worker(args):
    """one 100k-session file of a folder, the non-click_to_click rules (C oracle, per-file table)"""
    path, f, names = args
    d = np.load(path)
    off, aid, ts, ty, fb = d["off"], d["aid"], d["ts"], d["type"], d["fb"]
    s0, s1 = int(fb[f]), int(fb[f + 1])
    e0, e1 = int(off[s0]), int(off[s1])
    rules = {n: covis.REFERENCE_RULES[n] for n in names}
    return covis.count_co_events_file(off[s0:s1 + 1] - off[s0], aid[e0:e1], ts[e0:e1], ty[e0:e1], rules)


def _count_file_a6_worker(args):
    """one 100k-session file, all five rules (C oracle): per rule (rows, rows with count >= 2, the
    table or None, its count >= 2 part or None). click_to_* rules keep only the count >= 2 part
    (branch (1) of A6 applies to them at 220 M events; the caller asserts it), the others keep
    the whole table."""
    t = _count_file_worker(args)
    out = {}
    for n, (a, b, c) in t.items():
        keep = c >= 2
        if n.startswith("click_to"):
            out[n] = (len(a), int(keep.sum()), None, (a[keep], b[keep], c[keep]))
        else:
            out[n] = (len(a), int(keep.sum()), (a, b, c), None)
    return out


def full_a6(target_events: int = 220_000_000, seed: int = 0, workers: int = 8) -> dict:
    """BASELINE configs[1] A6 (concat_files_w_stats, model/count_co_events.py:103-181) of every rule at
    full size: per-file tables of the 135 files (C oracle, a process pool), then the streamed restatement
    (concat_files_w_stats_streamed: branch (1) for click_to_* rules, branch (2) by row slices for
    click_to_click, MIN_COUNT_TO_SAVE, count desc, head). Per rule the canonical digest (rows, sum,
    sha256 of the (aid, aid_next, count) rows) of the final table, written under "a6" in
    digest_220m.json."""
    import multiprocessing as mp
    import tempfile
    n_sess, _ = synth.sessions_for_events(target_events, 0, seed)
    ev = synth.generate(n_sess, 0, seed)
    fb = synth.file_session_bounds(n_sess)
    names = list(covis.REFERENCE_RULES)
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "events.npz")
        np.savez(path, off=ev.session_offsets - ev.session_offsets[0], aid=ev.aid, ts=ev.ts, type=ev.type, fb=fb)
        del ev
        with mp.get_context("spawn").Pool(workers) as pool:
            res = pool.map(_count_file_a6_worker, [(path, f, names) for f in range(len(fb) - 1)], chunksize=1)
    out = {}
    for n in names:
        rows = sum(r[n][0] for r in res)
        if n.startswith("click_to"):
            assert rows > 100_000_000, (n, rows)  # branch (1): the per-file count >= 2 parts suffice
        tabs_full = [r[n][2] for r in res]
        tabs_ge2 = [r[n][3] for r in res]
        a, b, c = concat_files_w_stats_streamed(n, tabs_full, tabs_ge2, rows)
        d = covis.canonical_digest({n: (a, b, c)})[n]
        d["file_rows"], d["file_rows_ge2"] = rows, sum(r[n][1] for r in res)
        out[n] = d
        for r in res:
            r[n] = None
    return out


def config5_a7(n_sessions: int = 12_900_000, workers: int = 8, names=None) -> dict:
    """BASELINE configs[4] co-visitation stage at full size (the bench's 12.9 M sessions, seed 0):
    train / truncated-test split (synth.split_test_labels), per-file tables of each folder's
    100k-session files (C oracle), A6 per folder and the A7 train+test merge (oracle/covis.py
    merge_train_test) for the rules whose A6 does not take the part-wise branch (2). Per rule the
    canonical digest (rows, sum, sha256) of the final table, written to digest_config5.json."""
    import multiprocessing as mp
    import tempfile
    names = names or ["click_to_cart_or_buy", "cart_to_cart", "cart_to_buy", "buy_to_buy"]
    ev = synth.generate(n_sessions)
    train, test, _ = synth.split_test_labels(ev)
    del ev
    per = {}
    with tempfile.TemporaryDirectory() as tmp:
        for tag, e in (("train", train), ("test", test)):
            fb = synth.file_session_bounds(e.n_sessions)
            path = os.path.join(tmp, f"{tag}.npz")
            np.savez(path, off=e.session_offsets - e.session_offsets[0], aid=e.aid, ts=e.ts, type=e.type, fb=fb)
            with mp.get_context("spawn").Pool(workers) as pool:
                per[tag] = pool.map(_count_file_worker, [(path, f, names) for f in range(len(fb) - 1)], chunksize=1)
    out = {"sessions": n_sessions, "train_sessions": int(train.n_sessions), "test_sessions": int(test.n_sessions),
           "train_files": len(per["train"]), "test_files": len(per["test"]), "rules": {}}
    for n in names:
        tr, te = [p[n] for p in per["train"]], [p[n] for p in per["test"]]
        n_tr = sum(len(t[0]) for t in tr)
        assert n_tr <= covis.MAX_ROWS_POLARS_GROUPBY, (n, n_tr)  # (2) not taken: the digest is exact
        out["rules"][n] = covis.canonical_digest({n: covis.merge_train_test(n, tr, te)})[n]
        out["rules"][n]["folder_rows"] = [n_tr, sum(len(t[0]) for t in te)]
    return out


def _count_file_c2c_worker(args):
    """one file's click_to_click table: (rows, rows with count >= 2, the table, its count >= 2 part)"""
    t = _count_file_worker(args)["click_to_click"]
    keep = t[2] >= 2
    return len(t[0]), int(keep.sum()), None, tuple(x[keep] for x in t)  # (1) applies at this size: no full table


def concat_files_w_stats_streamed(name, tables_full, tables_ge2, n_rows, max_rows_groupby=covis.MAX_ROWS_POLARS_GROUPBY,
                                  optim_rows=covis.OPTIM_ROWS_POLARS_GROUPBY,
                                  max_pairs=covis.MAX_CO_EVENT_PAIRS_TO_SAVE_DISK, click_filter_rows=100_000_000):
    """oracle/covis.py concat_files_w_stats (model/count_co_events.py:103-181) without materialising
    the concatenation: the per-file tables (each in (aid, aid_next) order) are consumed file by file
    into the row slices of branch (2). Checked equal to the in-memory restatement in main()."""
    import math
    use_ge2 = "click_to" in name and n_rows > click_filter_rows
    tabs = tables_ge2 if use_ge2 else tables_full
    if tabs is None or any(t is None for t in tabs):
        raise ValueError("the per-file tables this branch needs were not kept")
    N = sum(len(t[0]) for t in tabs)
    thr_part = covis.MIN_COUNT_IN_PART.get(name, 1)
    if N > max_rows_groupby:
        n_parts = math.ceil(N / optim_rows)
        max_rows_part = int(max_rows_groupby / N * optim_rows)
        rows_part = math.ceil(N / n_parts)
        parts, cur, filled = [], [], 0

        def close(chunks):
            a, b, c = (np.concatenate([x[i] for x in chunks]) for i in range(3))
            sa, sb, sc = covis._groupby_sum(a, b, c.astype(np.int64))
            k = sc >= thr_part
            sa, sb, sc = covis._sort_count_desc(sa[k], sb[k], sc[k])
            parts.append((sa[:max_rows_part], sb[:max_rows_part], sc[:max_rows_part]))

        for t in tabs:
            pos = 0
            while pos < len(t[0]):
                take = min(rows_part - filled, len(t[0]) - pos)
                cur.append(tuple(x[pos:pos + take] for x in t))
                pos += take
                filled += take
                if filled == rows_part:
                    close(cur)
                    cur, filled = [], 0
        if cur:
            close(cur)
        tabs = parts
    a, b, c = (np.concatenate([x[i] for x in tabs]) for i in range(3))
    a, b, c = covis._groupby_sum(a, b, c.astype(np.int64))
    k = c >= covis.MIN_COUNT_TO_SAVE.get(name, 1)
    a, b, c = covis._sort_count_desc(a[k], b[k], c[k])
    return a[:max_pairs], b[:max_pairs], c[:max_pairs].astype(np.int32)


def config5_c2c(n_sessions: int = 12_900_000, workers: int = 8) -> dict:
    """click_to_click of config5_a7: the train folder takes A6 branches (1) and (2) (row slices of the
    per-file tables in (aid, aid_next) order), so the folder merge is streamed
    (concat_files_w_stats_streamed); the test folder and the A7 merge as in config5_a7."""
    import multiprocessing as mp
    import tempfile
    ev = synth.generate(n_sessions)
    train, test, _ = synth.split_test_labels(ev)
    del ev
    folders = []
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for tag, e in (("train", train), ("test", test)):
            fb = synth.file_session_bounds(e.n_sessions)
            path = os.path.join(tmp, f"{tag}.npz")
            np.savez(path, off=e.session_offsets - e.session_offsets[0], aid=e.aid, ts=e.ts, type=e.type, fb=fb)
            with mp.get_context("spawn").Pool(workers) as pool:
                res = pool.map(_count_file_c2c_worker, [(path, f, ["click_to_click"]) for f in range(len(fb) - 1)],
                               chunksize=1)
            n_rows = sum(r[0] for r in res)
            n_ge2 = sum(r[1] for r in res)
            out[f"{tag}_rows"], out[f"{tag}_rows_ge2"] = n_rows, n_ge2
            folders.append(concat_files_w_stats_streamed("click_to_click", [r[2] for r in res], [r[3] for r in res],
                                                         n_rows))
            del res
    out.update(covis.canonical_digest({"click_to_click": covis.concat_files_w_stats("click_to_click", folders)})[
        "click_to_click"])
    return out


if __name__ == "__main__":
    if "--full" in sys.argv:  # ~1 min on 8 cores: the 220M-event digest only
        g = full_digest()
        old = os.path.join(HERE, "digest_220m.json")
        if os.path.exists(old) and "a6" in json.load(open(old)):
            g["a6"] = json.load(open(old))["a6"]
        json.dump(g, open(old, "w"), indent=1)
    elif "--full-a6" in sys.argv:  # a few minutes on 8 cores (~30 GB): the 220M-event A6 digests
        path = os.path.join(HERE, "digest_220m.json")
        g = json.load(open(path))
        g["a6"] = full_a6(seed=g["seed"])
        json.dump(g, open(path, "w"), indent=1)
    elif "--config5" in sys.argv:  # a few minutes on 8 cores (~40 GB): the config-5 A7 digests
        d = config5_a7()
        d["rules"]["click_to_click"] = config5_c2c()
        json.dump(d, open(os.path.join(HERE, "digest_config5.json"), "w"), indent=1)
    else:
        main()
