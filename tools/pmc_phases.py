"""Per-phase HBM traffic of the co-visitation build (and per-launch traffic of k_knn_main) from two
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of `bench.py --steps 1 --warmup 0 --knn-steps 1`.

FETCH_SIZE / WRITE_SIZE are reported in KiB per dispatch; FETCH_SIZE is doubled
(MI355X_MICROARCH.md §HBM: gfx950 tallies 128-B read requests at 64 B). Dispatches are cut into
builds at k_block_first and into phases by their first kernels:
  prep_count: k_block_first ..   rows: first kernel after k_prep_count / k_count_long
  emit: k_emit ..                reduce: first kernel after the last k_emit of the build
usage: python tools/pmc_phases.py FETCH.csv WRITE.csv > profiles/<round>_pmc_traffic.json"""
import csv
import json
import sys


def load(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0) for r in rows]


def phases(disp):
    builds, cur = [], None
    for name, v in disp:
        short = name.replace("ottohip::", "").split("(")[0].replace("void ", "")
        if short.startswith("k_block_first"):
            cur = {"prep_count": 0.0, "rows": 0.0, "emit": 0.0, "reduce": 0.0, "_ph": "prep_count"}
            builds.append(cur)
        if cur is None:
            continue
        if short.startswith("k_knn") or short.startswith("k_pack"):
            cur = None
            continue
        ph = cur["_ph"]
        if short.startswith("k_emit"):
            ph = "emit"
        elif ph == "emit":
            ph = "reduce"
        elif ph == "prep_count" and not (short.startswith(("k_block_first", "k_prep", "k_count")) or "rocclr" in short):
            ph = "rows"
        cur["_ph"] = ph
        cur[ph] += v
    return [{k: v for k, v in b.items() if not k.startswith("_")} for b in builds]


fetch, write = load(sys.argv[1]), load(sys.argv[2])
bf, bw = phases(fetch), phases(write)
n = min(len(bf), len(bw))
out = {"note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes of bench.py --steps 1 --warmup 0 "
               "--knn-steps 1 --cand-steps 0 --no-cpu --no-a6 --no-ingest; FETCH_SIZE (KiB) doubled per MI355X_MICROARCH.md; bytes per "
               f"build phase averaged over {n} full builds (run with --no-a6 --no-ingest, so no A6 part recounts or other kernels follow a build); k_knn_main per launch; produced by tools/pmc_phases.py"}
for ph in ("prep_count", "rows", "emit", "reduce"):
    f = sum(b[ph] for b in bf[:n]) / n
    w = sum(b[ph] for b in bw[:n]) / n
    out[f"covis_{ph}_phase"] = {"fetch_raw": f, "write": w, "traffic_bytes": 2 * f + w}
f = sum(sum(b[p] for p in ("prep_count", "rows", "emit", "reduce")) for b in bf[:n]) / n
w = sum(sum(b[p] for p in ("prep_count", "rows", "emit", "reduce")) for b in bw[:n]) / n
out["covis_step"] = {"fetch_raw": f, "write": w, "traffic_bytes": 2 * f + w}
# the main pass only: k_knn_main<0, ...> (the pre-pass k_knn_main<2, ...> shares the name; averaging both halved
# the round-4 figure, 44.4 GB against the per-kernel table's 85.7 GB per main launch)
is_main = lambda k: "k_knn_main<0" in k.replace("void ", "").replace("ottohip::", "")
kf = [v for k, v in fetch if is_main(k)]
kw = [v for k, v in write if is_main(k)]
if kf and kw:
    f, w = sum(kf) / len(kf), sum(kw) / len(kw)
    out["k_knn_main"] = {"fetch_raw": f, "write": w, "traffic_bytes": 2 * f + w}
print(json.dumps(out, indent=1))
