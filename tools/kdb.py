"""Per-kernel totals from rocprofv3 sqlite results (run_results.db): python tools/kdb.py a.db [b.db [passes]]
prints a's per-kernel time and calls, or (a - b) / passes."""
import collections
import re
import sqlite3
import sys


def load(path):
    c = sqlite3.connect(path)
    d = collections.defaultdict(lambda: [0.0, 0])
    for name, st, en in c.execute("select name, start, end from kernels"):
        n = re.sub(r"\(.*", "", name).replace("void ", "").replace("ottohip::", "")
        d[n][0] += (en - st) / 1e6
        d[n][1] += 1
    return d


a = load(sys.argv[1])
b = load(sys.argv[2]) if len(sys.argv) > 2 else {}
k = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
out = []
for n in set(a) | set(b):
    ta, ca = a.get(n, [0.0, 0])
    tb, cb = b.get(n, [0.0, 0])
    out.append(((ta - tb) / k, (ca - cb) / k, n))
out.sort(reverse=True)
print(f"{'kernel':70s} {'ms':>8s} {'calls':>8s}")
for t, c, n in out:
    if abs(t) >= 0.01:
        print(f"{n[:70]:70s} {t:8.2f} {c:8.1f}")
print(f"{'total':70s} {sum(x[0] for x in out):8.2f}")
