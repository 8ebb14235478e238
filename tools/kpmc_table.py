"""Per-kernel table from tools/gpu_pmc_r2.sh output: time (kernel trace), HBM fetch (x2, gfx950
FETCH_SIZE correction) and write, VALU / LDS / SALU instructions. usage: python tools/kpmc_table.py gpurun_out/<tag> [n]"""
import csv
import sys
from collections import defaultdict

O = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30


def short(n):
    return n.replace('ottohip::', '').split('(')[0].replace('void ', '')


t, cnt = defaultdict(float), defaultdict(int)
for r in csv.DictReader(open(f'{O}/k/run_kernel_trace.csv')):
    k = short(r['Kernel_Name'])
    t[k] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    cnt[k] += 1
agg = defaultdict(lambda: defaultdict(float))
for f in ('f', 'w', 'a'):
    for r in csv.DictReader(open(f'{O}/{f}/run_counter_collection.csv')):
        agg[short(r['Kernel_Name'])][r['Counter_Name']] += float(r['Counter_Value'])
print(f"{'kernel':40s} {'n':>4s} {'ms':>8s} {'fetchGB':>8s} {'writeGB':>8s} {'VALU(G)':>8s} {'LDS(G)':>8s} {'SALU(G)':>8s}")
for k in sorted(t, key=lambda k: -t[k])[:top]:
    c = agg[k]
    print(f"{k[:40]:40s} {cnt[k]:4d} {t[k]:8.2f} {2 * c['FETCH_SIZE'] * 1024 / 1e9:8.2f} {c['WRITE_SIZE'] * 1024 / 1e9:8.2f} "
          f"{c['SQ_INSTS_VALU'] / 1e9:8.3f} {c['SQ_INSTS_LDS'] / 1e9:8.3f} {c['SQ_INSTS_SALU'] / 1e9:8.3f}")
