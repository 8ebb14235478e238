"""Debug: conservation of key cuts on a hot-row dataset (expected cut words from the oracle)."""
import os, re, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import covis as oracle
import otto_recommender_amd.synth as synth
from otto_recommender_amd import covis as gc, _lib

rng = np.random.default_rng(11)
n_s, n = 4000, 40
rows = []
for s in range(n_s):
    ts = np.sort(rng.integers(0, 3600, n))
    aid = np.where(rng.random(n) < 0.5, 7, rng.integers(0, 200_000, n))
    rows.append(np.stack([np.full(n, s), aid, ts, np.zeros(n, np.int64)], 1))
a = np.concatenate(rows)
ev = synth.events_from_columns(a[:, 0], a[:, 1], a[:, 2], a[:, 3])
fb = synth.file_session_bounds(ev.n_sessions, per_file=n_s // 4)
nm = "click_to_click"
per_file = oracle.count_co_events_files(ev.session_offsets, ev.aid, ev.ts, ev.type, fb, rules={nm: oracle.REFERENCE_RULES[nm]})
dev = gc.DeviceEvents.from_host(ev, fb)
key = lambda t: (t[0].astype(np.uint64) << np.uint64(32)) | t[1].astype(np.uint64)
k1, k2 = key(per_file[1][nm]), key(per_file[2][nm])
hot1 = np.flatnonzero(per_file[1][nm][0] == 7)
hot2 = np.flatnonzero(per_file[2][nm][0] == 7)
lo, hi = int(k1[hot1[len(hot1) // 3]]), int(k2[hot2[len(hot2) // 2]])
exp_lo = int(per_file[1][nm][2][k1 < lo].sum()); exp_hi = int(per_file[2][nm][2][k2 >= hi].sum())
print("expected cut lo", exp_lo, "hi", exp_hi, "total pairs", sum(int(p[nm][2].sum()) for p in per_file), flush=True)
if "diff" in sys.argv:
    os.environ["OTTOHIP_CONSERVATION_WARN"] = "1"
for env in (() if ("diff" in sys.argv or "levels" in sys.argv) else ("1",)):
    os.environ["OTTOHIP_REDUCE_OVERLAP"] = env
    for tag, cuts in (("none+pf", gc.FileCuts(nm, per_file=True)), ("lo", gc.FileCuts(nm, lo=(1, lo))),
                      ("hi", gc.FileCuts(nm, hi=(2, hi))), ("lo+hi", gc.FileCuts(nm, lo=(1, lo), hi=(2, hi))),
                      ("lo=file0 all", gc.FileCuts(nm, lo=(0, 1 << 62)))):
        try:
            t = gc.count_co_events_fused(dev, [nm], cuts=cuts)
            print(env, tag, "ok", t.stats(nm), flush=True)
            t.free()
        except Exception as e:
            print(env, tag, "FAIL", e, flush=True)
    break
if "levels" in sys.argv:
    os.environ["OTTOHIP_DEBUG"] = "1"
    os.environ["OTTOHIP_CONSERVATION_WARN"] = "1"
    for tag, cuts in (("hi", gc.FileCuts(nm, hi=(2, hi))), ("lo", gc.FileCuts(nm, lo=(1, lo)))):
        print("=== levels", tag, flush=True)
        t = gc.count_co_events_fused(dev, [nm], cuts=cuts)
        t.free()
if "diff" not in sys.argv:
    sys.exit(0)

# the hi-cut table against the oracle: which keys differ
os.environ.pop("OTTOHIP_DEBUG", None)
os.environ["OTTOHIP_CONSERVATION_WARN"] = "1"
t = gc.count_co_events_fused(dev, [nm], cuts=gc.FileCuts(nm, hi=(2, hi)))
parts = [per_file[0][nm], per_file[1][nm], tuple(x[k2 < hi] for x in per_file[2][nm]), per_file[3][nm]]
ga, gb, gcnt = oracle._groupby_sum(*(np.concatenate([p[i] for p in parts]) for i in range(3)))
a_, b_, c_, _ = t.to_numpy(nm)
print("rows dev", len(a_), "oracle", len(ga), flush=True)
kd = (a_.astype(np.int64) << 32) | b_.astype(np.int64)
ko = (ga.astype(np.int64) << 32) | gb.astype(np.int64)
extra = np.setdiff1d(kd, ko); missing = np.setdiff1d(ko, kd)
print("extra keys", len(extra), [(int(k >> 32), int(k & 0xFFFFFFFF)) for k in extra[:20]], flush=True)
print("missing keys", len(missing), [(int(k >> 32), int(k & 0xFFFFFFFF)) for k in missing[:20]], flush=True)
common, i1, i2 = np.intersect1d(kd, ko, return_indices=True)
diff = np.flatnonzero(c_[i1].astype(np.int64) != gcnt[i2])
print("count diffs", len(diff), [(int(common[j] >> 32), int(common[j] & 0xFFFFFFFF), int(c_[i1][j]), int(gcnt[i2][j])) for j in diff[:20]], flush=True)
print("hi key", hi >> 32, hi & 0xFFFFFFFF, flush=True)
# expected split of the hi cut between the level-1 hash task (level-0 digit of (7, 7)) and the rest
def _mix(x, level):
    x = (x ^ ((level * 0x9E3779B9) & 0xFFFFFFFF)) & 0xFFFFFFFF
    x ^= x >> 16; x = (x * 0x7feb352d) & 0xFFFFFFFF; x ^= x >> 15; x = (x * 0x846ca68b) & 0xFFFFFFFF; x ^= x >> 16
    return x
if "levels" in sys.argv:
    dig = lambda k: (_mix(int(k), 0) * 512) >> 32
    d7 = dig(7)
    tot_h = drop_h = 0
    for f, p in enumerate(per_file):
        a_, b_, c_ = p[nm]
        m = (a_ == 7) & np.array([dig(x) == d7 for x in b_])
        tot_h += int(c_[m].sum())
        if f == 2:
            kk = (a_.astype(np.uint64) << np.uint64(32)) | b_.astype(np.uint64)
            drop_h += int(c_[m & (kk >= hi)].sum())
    print("expected hash task words", tot_h, "dropped there", drop_h, "kept", tot_h - drop_h, flush=True)
