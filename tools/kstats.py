"""Print a rocprofv3 kernel_stats.csv as a table (name, calls, total ms, avg ms, share)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':70s} {'calls':>6s} {'total ms':>9s} {'avg ms':>8s} {'share':>6s}")
for r in rows:
    name = r["Name"].replace("void ", "").replace("ottohip::", "").split("(")[0]
    t = float(r["TotalDurationNs"])
    print(f"{name[:70]:70s} {r['Calls']:>6s} {t / 1e6:9.2f} {float(r['AverageNs']) / 1e6:8.3f} {100 * t / tot:5.1f}%")
