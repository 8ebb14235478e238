"""A6 click_to_click on the 220 M-event workload with the library's phase timings of its part-tagged count
(prep_count / rows / emit / reduce ...): python tools/a6_probe.py [events]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import covis as gc, _lib
    n_ev = int(sys.argv[1]) if len(sys.argv) > 1 else 220_000_000
    n_sess, _ = synth.sessions_for_events(n_ev, 0, 0)
    fb = synth.file_session_bounds(n_sess)
    parts = [synth.generate(int(fb[f + 1] - fb[f]), int(fb[f]), 0) for f in range(len(fb) - 1)]
    off = np.zeros(n_sess + 1, np.int64)
    base = 0
    for f, p in enumerate(parts):
        off[fb[f]:fb[f + 1] + 1] = p.session_offsets + base
        base += p.n_events
    cat = lambda k: np.concatenate([getattr(p, k) for p in parts])
    ev = synth.Events(off, cat("session"), cat("aid"), cat("ts"), cat("type"))
    del parts
    dev = gc.DeviceEvents.from_host(ev, np.asarray(fb, np.int64))
    del ev
    ctx = _lib.context()
    tab = gc.count_co_events_fused(dev, ctx=ctx, per_file_rule="click_to_click")
    for rep in range(2):
        ctx.set_timing(True)
        st = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gc.concat_files_w_stats_fused(dev, "click_to_click", table=tab, ctx=ctx, timings=st)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        ph = {}
        for n, t, _ in ctx.timings():
            ph[n] = round(ph.get(n, 0.0) + t, 2)
        ctx.set_timing(False)
        print(json.dumps({"rep": rep, "ms": round(ms, 2), "stages_ms": {k: round(v * 1e3, 2) for k, v in st.items()},
                          "phases_ms": ph}))


if __name__ == "__main__":
    main()
