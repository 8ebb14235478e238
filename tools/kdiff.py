"""Per-kernel difference of two rocprofv3 kernel_stats.csv files (a - b), divided by a pass count:
python tools/kdiff.py a.csv b.csv [passes]"""
import csv
import sys


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        name = r["Name"].replace("void ", "").replace("ottohip::", "").split("(")[0]
        t, c = out.get(name, (0.0, 0))
        out[name] = (t + float(r["TotalDurationNs"]), c + int(r["Calls"]))
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
k = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
rows = []
for n in set(a) | set(b):
    ta, ca = a.get(n, (0.0, 0))
    tb, cb = b.get(n, (0.0, 0))
    rows.append(((ta - tb) / 1e6 / k, (ca - cb) / k, n))
rows.sort(reverse=True)
print(f"{'kernel':60s} {'ms/pass':>8s} {'calls/pass':>10s}")
tot = 0.0
for t, c, n in rows:
    tot += t
    print(f"{n[:60]:60s} {t:8.2f} {c:10.1f}")
print(f"{'total':60s} {tot:8.2f}")
