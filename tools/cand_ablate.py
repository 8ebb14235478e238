"""Times k_cand_build ablations (OTTOHIP_CAND_DBG bits: 1 no sort, 2 no pop, 4 no list expansion)
on a synthetic config-5 candidate workload; each variant in its own process."""
import json, os, subprocess, sys
code = r'''
import sys, time, json, numpy as np, torch
sys.path.insert(0, ".")
import otto_recommender_amd.synth as synth
from otto_recommender_amd import candidates as gc, _lib
ev = synth.generate(int(sys.argv[1]))
tr, te, lab = synth.split_test_labels(ev)
uni = np.arange(1855603, dtype=np.int32)
rng = np.random.default_rng(0)
def lists(k, nq):
    q = uni[:nq]; nb = rng.integers(0, 1855603, (nq, k - 1)).astype(np.int32)
    return (np.repeat(q, k), np.concatenate([q[:, None], nb], 1).ravel(), np.tile(np.arange(1, k + 1, dtype=np.int16), nq))
r1 = {n: lists(10 if n.startswith("click") else 20, 900_000) for n in ["click_to_click","click_to_cart_or_buy","cart_to_cart","cart_to_buy","buy_to_buy"]}
src = gc.CandidateSources(r1, lists(20, 600_000), lists(20, 600_000), (rng.integers(0, 50, 5000).astype(np.int32), rng.integers(0, 1855603, 5000).astype(np.int32)), 50)
cl = rng.integers(0, 50, te.n_sessions).astype(np.int32)
ctx = _lib.context(); ctx.set_timing(True)
for i in range(2):
    c = gc.generate(te.session_offsets, te.aid, te.ts, te.type, src, cl)
    ph = {n: round(ms, 2) for n, ms, _ in ctx.timings()}
    n = c.n_cand; c.free()
print(json.dumps({"cand": n, "phases": ph}))
'''
for dbg in (0, 1, 2, 4, 7):
    env = dict(os.environ, OTTOHIP_CAND_DBG=str(dbg))
    out = subprocess.run([sys.executable, "-c", code, sys.argv[1] if len(sys.argv) > 1 else "4000000"], env=env,
                         capture_output=True, text=True)
    print(dbg, out.stdout.strip()[-300:], out.stderr.strip()[-300:] if out.returncode else "")
