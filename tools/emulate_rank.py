"""Single-GPU emulation of one rank of the N-GPU co-visitation build (bench.py --gpus N).

Rank `--rank` of `--world` gets its balanced whole files of the 220M-event stream, counts
them, packs rows by owner and merge-sums ALL of its packed records as if they were the
records it receives (same volume in expectation: owner(aid) is a uniform hash). Prints per
phase device times (HIP events): the per-rank compute of the N-GPU step, without the
all-to-all itself. --sym 1 (default): the symmetric rules travel once per unordered pair, as
dist.count_co_events_sharded sends them; the exchange is modelled as max(sent, received remote bytes)
over 7 xGMI links at 153 GB/s each (and at half that rate)."""
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
    ap.add_argument("--sym", type=int, default=1)
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
    G = args.world
    # (1) this rank's emit: S1-S4 of its own files, words laid out by owner
    for rep in range(args.reps):
        ctx.set_timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w, wpp, pc, ppp, names = gd.emit_for_owners(dev, G, mine, n_files, ctx=ctx, sym=bool(args.sym))
        torch.cuda.synchronize()
        t_emit = time.perf_counter() - t0
        own_wpp, own_ppp = list(wpp), list(ppp)  # this rank's send segments (words, pieces) per owner
        ph_emit = ctx.timings()
        ctx.set_timing(False)
        del w, pc
    del dev
    # (2) what owner `rank` receives: its segment of every file's words (emit of ALL files, untimed)
    full = [synth.generate(int(fb_all[f + 1] - fb_all[f]), int(fb_all[f]), 0) for f in range(n_files)]
    off = np.zeros(n_sess + 1, np.int64)
    base = 0
    for f, p in enumerate(full):
        off[fb_all[f]:fb_all[f + 1] + 1] = p.session_offsets + base
        base += p.n_events
    catf = lambda k: np.concatenate([getattr(p, k) for p in full])
    evf = synth.Events(off, catf("session"), catf("aid"), catf("ts"), catf("type"))
    del full
    devf = gc.DeviceEvents.from_host(evf, fb_all)
    del evf
    w, wpp, pc, ppp, names = gd.emit_for_owners(devf, G, None, n_files, ctx=ctx, sym=bool(args.sym))
    del devf
    o = args.rank
    ws = w[sum(wpp[:o]):sum(wpp[:o + 1])].clone()
    ps = pc[sum(ppp[:o]):sum(ppp[:o + 1])].clone()
    del w, pc
    torch.cuda.empty_cache()
    for rep in range(args.reps):
        ctx.set_timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        shard = gd.reduce_received(ws, ps, names, n_files, ctx=ctx, sym=bool(args.sym))
        torch.cuda.synchronize()
        t_red = time.perf_counter() - t0
        ph_red = ctx.timings()
        ctx.set_timing(False)
        rows = sum(shard.stats(n)["n_rows"] for n in names)
        shard.free()
    # received from the other ranks: owner o's segment of every file minus its own files' (uniform hash: the
    # own files' share of the segment is their share of the sent words)
    send_remote = 4 * int(sum(own_wpp) - own_wpp[args.rank]) + 8 * int(sum(own_ppp) - own_ppp[args.rank])
    recv_remote = 4 * int(ws.numel() - own_wpp[args.rank]) + 8 * int(ps.numel() - own_ppp[args.rank])
    link = 7 * 153e9
    res = {"world": G, "rank": args.rank, "sym": args.sym, "files": len(mine), "events": int(ev.n_events),
           "send_words": int(sum(own_wpp)), "recv_words": int(ws.numel()), "recv_pieces": int(ps.numel()),
           "shard_rows": int(rows), "emit_s": t_emit, "reduce_received_s": t_red,
           "send_bytes_remote": send_remote, "recv_bytes_remote": recv_remote,
           "xgmi_ms_peak": round(max(send_remote, recv_remote) / link * 1e3, 3),
           "xgmi_ms_half": round(2 * max(send_remote, recv_remote) / link * 1e3, 3),
           "phases_ms": {n: round(ms, 3) for n, ms, _ in ph_emit + ph_red}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
