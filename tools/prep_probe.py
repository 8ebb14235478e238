"""Time S1-S3 (prep_count, rows) of the 220 M-event one-GPU build alone, several reps (ottohip_covis_emit with one
part: the front only, no emit or reduce), so a compile-time ablation of S2 that breaks the counts (tools/build_ab.sh
-DOH_PREP_ABL=..., OTTOHIP_LIB) can still be timed.  python tools/prep_probe.py [--reps 5]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=220_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import covis as gc, dist as gd, _lib
    torch.cuda.set_device(0)
    n_sess, _ = synth.sessions_for_events(args.events, 0, 0)
    ev = synth.generate(n_sess, 0, 0)
    fb = synth.file_session_bounds(n_sess)
    dev = gc.DeviceEvents.from_host(ev, fb)
    del ev
    ctx = _lib.context()
    ctx.set_timing(True)
    out = {}
    for rep in range(args.reps + 1):
        e = gd.OwnerEmit(dev, 1, ctx=ctx, sym=True)
        torch.cuda.synchronize()
        t = {n: ms for n, ms, _ in ctx.timings()}
        if rep:
            for k, v in t.items():
                out.setdefault(k, []).append(round(v, 3))
        del e
    print(json.dumps({"lib": os.environ.get("OTTOHIP_LIB", "in-tree"), "ms": out,
                      "median": {k: float(np.median(v)) for k, v in out.items()}}))


if __name__ == "__main__":
    main()
