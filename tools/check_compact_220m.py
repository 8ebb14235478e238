"""Full-size check of the per-rule compaction (table slots > 2^32): for every rule of the 220 M-event
table, the compacted rows (ottohip_table_copy) must match the reduce's own statistics (row count,
sum of counts), and finalize's kept rows must match a torch count of count >= MIN_COUNT_TO_SAVE."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import otto_recommender_amd.synth as synth
from otto_recommender_amd import covis as gc, config as cfg

n_sess, _ = synth.sessions_for_events(220_000_000, 0, 0)
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
dev = gc.DeviceEvents.from_host(ev, fb)
del ev
tab = gc.count_co_events_fused(dev)
print("slots > 2^32:", sum(tab.stats(n)["n_pairs"] for n in tab.names) > 2**32, flush=True)
for n in tab.names:
    st = tab.stats(n)
    a, b, c, c2 = tab.to_torch(n)
    ok_rows = a.numel() == st["n_rows"]
    ok_pairs = int(c.to(torch.int64).sum().item()) == st["n_pairs"]
    thr = max(cfg.MIN_COUNT_TO_SAVE.get(n, 1), 1)
    use_ge2 = "click_to" in n and st["file_rows"] > cfg.CLICK_FILTER_ROWS
    col = c2 if use_ge2 else c
    expect = int((col >= thr).sum().item())
    del a, b, c, c2, col
    t0 = time.perf_counter()
    try:
        fa, fb_, fc = tab.finalize(n, max_rows=1 << 40)
        got = fa.numel()
    except Exception as e:  # part-wise branch rules raise ELIMIT here
        got = repr(e)[:60]
    print(n, "rows", ok_rows, "pairs", ok_pairs, "finalize kept", got, "expected", expect,
          f"{(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
