"""Reduce task statistics of one 220 M-event build (OTTOHIP_DEBUG=1 level lines on stderr)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import otto_recommender_amd.synth as synth
from otto_recommender_amd import covis as gc
n_sess, n_ev = synth.sessions_for_events(int(sys.argv[1]) if len(sys.argv) > 1 else 220_000_000, 0, 0)
ev = synth.generate(n_sess, 0, 0)
dev = gc.DeviceEvents.from_host(ev, synth.file_session_bounds(n_sess))
del ev
t = gc.count_co_events_fused(dev)
t.free()
os.environ["OTTOHIP_DEBUG"] = "1"
t0 = time.time()
t = gc.count_co_events_fused(dev)
print("build s", time.time() - t0, flush=True)
