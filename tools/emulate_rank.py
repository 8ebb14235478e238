"""Single-GPU emulation of one rank of the N-GPU co-visitation build (bench.py --gpus N).

Rank `--rank` of `--world` gets its balanced whole files of the 220M-event stream, counts
them, packs rows by owner and merge-sums ALL of its packed records as if they were the
records it receives (same volume in expectation: owner(aid) is a uniform hash). Prints per
phase device times (HIP events): the per-rank compute of the N-GPU step, without the
all-to-all itself."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--events", type=int, default=220_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import covis as gc, dist as gd, _lib
    torch.cuda.set_device(0)
    n_sess, _ = synth.sessions_for_events(args.events, 0, 0)
    fb_all = synth.file_session_bounds(n_sess)
    n_files = len(fb_all) - 1
    lens = synth.session_lengths(n_sess, 0, 0).astype(np.float64)
    w = [float((lens[fb_all[f]:fb_all[f + 1]] ** 2).sum()) for f in range(n_files)]
    mine = gd.deal_files(n_files, args.rank, args.world, w)
    parts = [synth.generate(int(fb_all[f + 1] - fb_all[f]), int(fb_all[f]), 0) for f in mine]
    fb = np.concatenate([[0], np.cumsum([p.n_sessions for p in parts])]).astype(np.int64)
    off = np.zeros(int(fb[-1]) + 1, np.int64)
    base = 0
    for i, p in enumerate(parts):
        off[fb[i]:fb[i + 1] + 1] = p.session_offsets + base
        base += p.n_events
    cat = lambda k: np.concatenate([getattr(p, k) for p in parts])
    ev = synth.Events(off, cat("session"), cat("aid"), cat("ts"), cat("type"))
    dev = gc.DeviceEvents.from_host(ev, fb)
    ctx = _lib.context()
    res = []
    for rep in range(args.reps):
        ctx.set_timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        local = gc.count_co_events_fused(dev, ctx=ctx)
        ph = ctx.timings()
        recs, counts = gd.pack_by_owner(local, args.world)
        ph += ctx.timings()
        names = local.names
        st = [local.stats(n) for n in names]
        local.free()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        shard = gd.table_from_records(recs, names, 1855603, [(s["file_rows"], s["file_rows_ge2"]) for s in st], ctx=ctx)
        ph += ctx.timings()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ctx.set_timing(False)
        res = {"world": args.world, "rank": args.rank, "files": len(mine), "events": int(ev.n_events),
               "local_pairs": int(sum(s["n_pairs"] for s in st)), "local_rows": int(sum(s["n_rows"] for s in st)),
               "records": int(recs.shape[0]), "per_owner": counts,
               "count_pack_s": t1 - t0, "merge_s": t2 - t1,
               "phases_ms": {n: round(ms, 3) for n, ms, _ in ph}}
        shard.free()
        del recs
    print(json.dumps(res))


if __name__ == "__main__":
    main()
