"""Sum rocprofv3 --pmc counters per kernel: python tools/pmc_sum.py run_counter_collection.csv [substr...]"""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
ns = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    ns[k].add(r["Dispatch_Id"])
subs = sys.argv[2:]
for k in sorted(agg, key=lambda k: -agg[k].get("SQ_WAVE_CYCLES", 0)):
    if subs and not any(s in k for s in subs):
        continue
    c = agg[k]
    print(f"{k[:60]:60s} n={len(ns[k]):3d} " + " ".join(f"{n.replace('SQ_', '')}={v:.3g}" for n, v in sorted(c.items())))
