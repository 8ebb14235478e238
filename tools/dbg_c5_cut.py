"""Debug: config-5 train folder, click_to_click, A6 branch (2) part counts with key cuts (conservation)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import otto_recommender_amd.synth as synth
from otto_recommender_amd import covis as gc, pipeline, _lib

ev = synth.generate(12_900_000)
train, test, labels = synth.split_test_labels(ev)
del ev
fb = synth.file_session_bounds(train.n_sessions)
dev = gc.DeviceEvents.from_host(train, fb)
n = "click_to_click"
t = gc.count_co_events_fused(dev, [n], cuts=gc.FileCuts(n, per_file=True))
R = t.file_rows_ge2_per_file
print("N", int(R.sum()), t.stats(n), flush=True)
t.free()
plan = gc.part_plan(R, -(-int(R.sum()) // 100_000_000))
print(plan, flush=True)
keys = gc.boundary_keys(dev, n, plan, R, True, gc.config.N_ITEMS_OTTO)
print(keys, flush=True)
for fa, lo, fb_, hi in plan:
    for cuts in (gc.FileCuts(n, lo=(0, keys[(fa, lo)]) if lo > 0 else None, hi=(fb_ - fa, keys[(fb_, hi)]) if hi < int(R[fb_]) else None, per_file=True),
                 gc.FileCuts(n, lo=(0, keys[(fa, lo)]) if lo > 0 else None, per_file=True),
                 gc.FileCuts(n, hi=(fb_ - fa, keys[(fb_, hi)]) if hi < int(R[fb_]) else None, per_file=True),
                 gc.FileCuts(n, per_file=True)):
        try:
            tt = gc.count_co_events_fused(dev.subset_files(fa, fb_ + 1), [n], cuts=cuts)
            pf = tt.file_rows_ge2_per_file
            print("part", fa, lo, fb_, hi, "lo" if cuts.lo else "-", "hi" if cuts.hi else "-", "ok rows_ge2", int(pf.sum()),
                  "first", int(pf[0]), "last", int(pf[-1]), "R", int(R[fa]), int(R[fb_]), flush=True)
            tt.free()
        except Exception as e:
            print("part", fa, lo, fb_, hi, "lo" if cuts.lo else "-", "hi" if cuts.hi else "-", "FAIL", e, flush=True)
