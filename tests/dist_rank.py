"""One rank of a multi-process GPU test (launched as a fresh child process by tests/test_dist_gpu.py;
never imported by pytest). Runs the PRODUCT multi-GPU path -- otto-recommender_amd/dist.py over
torch.distributed -- and saves what this rank holds to an .npz for the parent to check against
the oracle. It does not import oracle/.

  python tests/dist_rank.py covis <out.npz> <json config>
Environment: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (gloo: all ranks may share cuda:0).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _my_events(ev, fb, files):
    import otto_recommender_amd.synth as synth
    parts = [ev.slice_sessions(int(fb[f]), int(fb[f + 1])) for f in files]
    bounds = np.concatenate([[0], np.cumsum([p.n_sessions for p in parts])]).astype(np.int64)
    off = np.zeros(int(bounds[-1]) + 1, np.int64)
    pos = 0
    for i, p in enumerate(parts):
        off[bounds[i]:bounds[i + 1] + 1] = p.session_offsets - p.session_offsets[0] + pos
        pos += p.n_events
    cat = lambda k, dt: (np.concatenate([getattr(p, k) for p in parts]) if parts else np.zeros(0, dt))
    return synth.Events(off, cat("session", np.int32), cat("aid", np.int32), cat("ts", np.int32),
                        cat("type", np.int8)), bounds


def structured_events(cfg):
    """Events whose per-file click_to_click tables have exactly 2 * m_f rows (cfg["structured"] = [m_f per file]):
    session j of every file clicks aids j and j + 5000 three times each, alternating, a minute apart, so its
    table holds (j, j + 5000) and (j + 5000, j) with count 9, and the same keys recur in every file. The row
    counts are chosen by the caller to put a branch-(2) part boundary exactly on a file end."""
    import otto_recommender_amd.synth as synth
    rows, fb, s = [], [0], 0
    for m in cfg["structured"]:
        for j in range(m):
            for e in range(6):
                rows.append((s, j if e % 2 == 0 else j + 5000, 1_000_000 + 60 * e, 0))
            s += 1
        fb.append(s)
    a = np.array(rows, np.int64)
    ev = synth.events_from_columns(a[:, 0], a[:, 1], a[:, 2], a[:, 3])
    return ev, np.array(fb, np.int64)


def covis(out, cfg):
    import torch
    import torch.distributed as dist
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import covis as gc, dist as gd, config
    rank, world = dist.get_rank(), dist.get_world_size()
    if "structured" in cfg:
        ev, fb = structured_events(cfg)
    else:
        ev = synth.generate(cfg["sessions"], first_session=cfg.get("first_session", 0))
        fb = synth.file_session_bounds(ev.n_sessions, per_file=cfg["per_file"])
    n_files = len(fb) - 1
    lens = np.diff(ev.session_offsets).astype(np.float64)
    w = [float((lens[fb[f]:fb[f + 1]] ** 2).sum()) for f in range(n_files)]
    mine = gd.deal_files(n_files, rank, world, weights=w)
    my_ev, my_fb = _my_events(ev, fb, mine)
    dev = gc.DeviceEvents.from_host(my_ev, my_fb)
    res = {"files": np.asarray(mine, np.int64)}
    tab = gd.count_co_events_sharded(dev, mine, n_files)
    # the exchange in 1 and 3 file chunks (overlapped all-to-alls), and global file batches of 2
    # (more files than a pair word holds: per-batch shards merge-summed per owner), give the same shard
    for ch, mf in ((1, None), (3, None), (2, 2)):
        t2 = gd.count_co_events_sharded(dev, mine, n_files, chunks=ch, max_files=mf)
        for n in tab.names:
            for x, y in zip(tab.to_numpy(n), t2.to_numpy(n)):
                assert np.array_equal(x, y), (ch, mf, n)
            assert tab.stats(n) == t2.stats(n), (ch, mf, n)
        t2.free()
    for n in tab.names:
        a, b, c, c2 = tab.to_numpy(n)
        st = tab.stats(n)
        res[f"shard/{n}"] = np.stack([a.astype(np.int64), b, c.astype(np.int64), c2.astype(np.int64)], 1)
        res[f"stats/{n}"] = np.array([st["file_rows"], st["file_rows_ge2"]], np.int64)
    for tag, kw in cfg["merges"].items():
        for n in cfg.get("rules", config.CO_EVENTS_TO_COUNT):
            a, b, c = gd.concat_files_w_stats_sharded(dev, mine, n_files, n, table=tab, **kw)
            res[f"final/{tag}/{n}"] = np.stack([x.cpu().numpy().astype(np.int64) for x in (a, b, c)], 1)
            a, b, c = gd.concat_files_w_stats_sharded(dev, mine, n_files, n, table=tab, gather=False, **kw)
            res[f"slice/{tag}/{n}"] = np.stack([x.cpu().numpy().astype(np.int64) for x in (a, b, c)], 1)
    tab.free()
    torch.cuda.synchronize()
    np.savez(out, **res)


def covis_full(out, cfg):
    """BASELINE configs[3] at its real size: the 220 M-event stream's 100k-session files dealt to the ranks by
    Σ n_s² (as bench.py), each rank generating only its own files; the sharded count of all five rules, then the
    sharded A6 of every rule (branch (2) of click_to_click at N = 694 M included). Saves per rule the shard's
    order-independent digests (they add over ranks to the single-table digests), the global statistics, the
    exchange sizes, a sha256 of this rank's final table, and rank 0's final tables."""
    import hashlib
    import time
    import torch
    import torch.distributed as dist
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import covis as gc, dist as gd
    rank, world = dist.get_rank(), dist.get_world_size()
    seed, n_sess = int(cfg["seed"]), int(cfg["sessions"])
    fb_all = synth.file_session_bounds(n_sess)
    n_files = len(fb_all) - 1
    lens = synth.session_lengths(n_sess, 0, seed).astype(np.float64)
    weights = [float((lens[fb_all[f]:fb_all[f + 1]] ** 2).sum()) for f in range(n_files)]
    mine = gd.deal_files(n_files, rank, world, weights)
    parts = [synth.generate(int(fb_all[f + 1] - fb_all[f]), int(fb_all[f]), seed) for f in mine]
    fb = np.concatenate([[0], np.cumsum([p.n_sessions for p in parts])]).astype(np.int64)
    off = np.zeros(int(fb[-1]) + 1, np.int64)
    base = 0
    for i, p in enumerate(parts):
        off[fb[i]:fb[i + 1] + 1] = p.session_offsets + base
        base += p.n_events
    ev = synth.Events(off, np.concatenate([p.session for p in parts]), np.concatenate([p.aid for p in parts]),
                      np.concatenate([p.ts for p in parts]), np.concatenate([p.type for p in parts]))
    del parts
    dev = gc.DeviceEvents.from_host(ev, fb)
    res = {"files": np.asarray(mine, np.int64), "events": np.array([ev.n_events], np.int64)}
    del ev
    t0 = time.perf_counter()
    tab = gd.count_co_events_sharded(dev, mine, n_files)
    torch.cuda.synchronize()
    res["count_s"] = np.array([time.perf_counter() - t0])
    xs = tab.exchange_stats
    res["exchange"] = np.array([xs["words_sent"], xs["max_words_to_peer"], xs["words_recv"], xs["max_words_from_peer"],
                                xs["pieces_sent"], xs["pieces_recv"]], np.int64)
    for n in tab.names:
        d, st = tab.digest(n), tab.stats(n)
        res[f"digest/{n}"] = np.array([d["d_count"], d["d_count_ge2"], d["pairs"], d["pairs_ge2"], d["rows"]], np.uint64)
        res[f"stats/{n}"] = np.array([st["file_rows"], st["file_rows_ge2"], st["n_rows"], st["n_pairs"]], np.int64)
    for n in tab.names:
        t0 = time.perf_counter()
        a, b, c = gd.concat_files_w_stats_sharded(dev, mine, n_files, n, table=tab)
        torch.cuda.synchronize()
        res[f"a6_s/{n}"] = np.array([time.perf_counter() - t0])
        x = torch.stack([a, b, c], 1).cpu().numpy().astype(np.int32)
        res[f"final_sha/{n}"] = np.frombuffer(hashlib.sha256(x.tobytes()).digest(), np.uint8)
        if rank == 0:
            res[f"final/{n}"] = x
        del a, b, c, x
    tab.free()
    torch.cuda.synchronize()
    np.savez(out, **res)


def pipeline(out, cfg):
    import torch.distributed as dist
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import pipeline as pl
    ev = synth.generate(cfg["sessions"], first_session=cfg.get("first_session", 0))
    train, test, labels = synth.split_test_labels(ev)
    words = synth.item_words()
    emb = synth.embeddings(len(words), seed=1)
    emb2 = synth.embeddings(len(words), seed=3)
    res = pl.run(train, test, labels, words, emb, words, emb2, n_clusters=cfg["clusters"], kmeans_iter=cfg["iters"],
                 knn_queries=cfg["queries"], keep_tables=True, group=dist.group.WORLD, n_init=cfg["n_init"],
                 per_file=cfg["per_file"])
    im = res["intermediates"]
    o = {"candidates_total": np.array([res["candidates"], res["local_candidates"]], np.int64),
         "n_test_files": np.array([res.get("local_test_files", -1)], np.int64),
         "recall": np.array([res["recall"][t][k] for t in ("clicks", "carts", "orders", "total")
                             for k in ("top20", "top100", "top200", "topall")]),
         "cluster_labels": im["cluster_labels"], "cluster_rows": im["cluster_rows"],
         "pop": im["pop"].to_numpy().astype(np.int64)}
    for n, v in im["tables"].items():
        o[f"table/{n}"] = np.stack([np.asarray(x, np.int64) for x in v], 1)
    for i, v in enumerate(im["knn"]):
        o[f"knn/{i}"] = np.stack([np.asarray(x, np.int64) for x in v], 1)
    c = im["candidates"]
    o["cand_cols"] = np.array(list(c.columns))
    o["cand"] = c.to_numpy().astype(np.int64)
    np.savez(out, **o)


def main():
    import torch
    import torch.distributed as dist
    mode, out, cfg = sys.argv[1], sys.argv[2], json.loads(sys.argv[3])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    try:
        {"covis": covis, "covis_full": covis_full, "pipeline": pipeline}[mode](out, cfg)
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
