"""Timeline of the last co-visitation build in a rocprofv3 kernel trace (csv): every kernel from the
last k_block_first on, with its start offset, duration and queue, plus per-queue busy time.
Usage: python tools/timeline.py run_kernel_trace.csv"""
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("ottohip::", "")
    return name[:48]


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q, short(r["Kernel_Name"])))
    ev.sort()
    starts = [i for i, e in enumerate(ev) if e[3] == "k_block_first"]
    if not starts:
        print("no k_block_first in the trace")
        return
    sel = ev[starts[-1]:]
    # stop at the first kernel that is not part of a covis build (the next sub-benchmark)
    t0 = sel[0][0]
    busy = {}
    last_end = t0
    for s, e, q, n in sel:
        busy[q] = busy.get(q, 0) + (e - s)
        last_end = max(last_end, e)
        print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} q{q:>3} {n}")
    print(f"span {(last_end - t0) / 1e6:.3f} ms; busy per queue:",
          {q: round(b / 1e6, 3) for q, b in busy.items()})


if __name__ == "__main__":
    main(sys.argv[1])
