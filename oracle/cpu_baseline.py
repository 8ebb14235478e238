"""CPU baseline of the co-visitation count (TEST INFRASTRUCTURE: bench.py's cpu_baseline leg).

Run as a child process of bench.py (it never touches the GPU):
    python oracle/cpu_baseline.py <json config>   ->  one JSON line
Times, on the host cores available to this process, the per-file stage of
count_co_events_all_files (model/count_co_events.py:80-100) over whole 100k-session files of
the same synthetic stream as the GPU line:
  "port"      oracle/covis_oracle.c (dedup -> per-session pairs -> window filter -> per-rule
              groupby, no materialised join), files in parallel over OpenMP threads;
  "pandas"    oracle/covis_pandas.py, the op-for-op pandas restatement of the reference's
              dataframe pipeline (:17-94: unique, 10k-session parts, join on session, filters,
              groupby count), a process pool over files -- the reference's own algorithm.
Both report qualifying pairs / s over the sample.
  "merge"     count + merge (the reference's deliverable, :202 + :210): the C per-file tables, then the
              numpy restatement of concat_files_w_stats (:103-181) over them.
"""
from __future__ import annotations

import ctypes
import json
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE]


def host_cores() -> dict:
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2 CPU quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(p)))
    except Exception:
        pass
    usable = min(aff, quota) if quota else aff
    return {"usable": usable, "affinity": aff, "cgroup_quota": quota, "os_cpu_count": os.cpu_count()}


def _files(n_files: int, seed: int):
    import otto_recommender_amd.synth as synth
    n = n_files * synth.SESSIONS_PER_FILE
    ev = synth.generate(n, 0, seed)
    return ev, synth.file_session_bounds(n)


def port(n_files: int, threads: int, seed: int) -> dict:
    import covis as oracle
    ev, fb = _files(n_files, seed)
    lib = oracle._lib()
    names, this, mask, wmax = oracle._rule_arrays(oracle.REFERENCE_RULES)
    tot = np.zeros(2 * len(names), np.int64)
    f = lib.oracle_count_files_omp
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 5 + [ctypes.c_int] + [ctypes.c_void_p] * 3 + [
        ctypes.c_int32, ctypes.c_int32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    off = np.ascontiguousarray(ev.session_offsets, np.int64)
    fb = np.ascontiguousarray(fb, np.int64)
    t0 = time.perf_counter()
    rc = f(len(fb) - 1, fb.ctypes.data, off.ctypes.data, ev.aid.ctypes.data, ev.ts.ctypes.data, ev.type.ctypes.data,
           len(names), this.ctypes.data, mask.ctypes.data, wmax.ctypes.data, oracle.MIN_TIME_TO_NEXT,
           oracle.MAX_TIME_TO_NEXT, threads, tot.ctypes.data, None)
    dt = time.perf_counter() - t0
    if rc:
        raise RuntimeError(f"oracle_count_files_omp failed ({rc})")
    pairs = int(tot[1::2].sum())
    return {"value": pairs / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"per-file counting only, no cross-file merge: first {len(fb) - 1} files ({ev.n_sessions} "
                      f"sessions, {ev.n_events} events, {pairs} pairs) of the same stream; oracle/covis_oracle.c "
                      f"per-file count, files over {threads} OpenMP threads, {dt:.1f} s", "seconds": dt, "pairs": pairs, "files": len(fb) - 1}


def _pandas_file(args):
    f, seed = args
    import covis_pandas
    import otto_recommender_amd.synth as synth
    ev = synth.generate(synth.SESSIONS_PER_FILE, f * synth.SESSIONS_PER_FILE, seed)
    df = ev.to_pandas()
    t0 = time.perf_counter()
    tabs = covis_pandas.count_file(df)
    dt = time.perf_counter() - t0
    return dt, int(sum(int(g["count"].sum()) for g in tabs.values()))


def pandas_pool(n_files: int, workers: int, seed: int) -> dict:
    import multiprocessing as mp
    ctx = mp.get_context("spawn")  # fresh interpreters: libgomp (the port leg, synth) is not fork-safe
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_pandas_file, [(f, seed) for f in range(n_files)], chunksize=1)
    wall = time.perf_counter() - t0
    pairs = sum(p for _, p in res)
    busy = sum(d for d, _ in res)
    return {"value": pairs / wall, "unit": "pairs/s", "cores": workers, "kind": "port",
            "sample": f"per-file counting only, no cross-file merge: first {n_files} files ({n_files * 100000} "
                      f"sessions, {pairs} pairs); oracle/covis_pandas.py "
                      f"op-for-op restatement of model/count_co_events.py:17-94 (unique, 10k-session parts, join, "
                      f"filters, groupby), process pool of {workers}; {wall:.1f} s wall (includes generating each "
                      f"file in its worker), {busy:.1f} s summed counting time",
            "seconds": wall, "pairs": pairs, "per_core_pairs_per_s": pairs / busy if busy else None}


def count_plus_merge(n_files: int, threads: int, seed: int) -> dict:
    """The reference's deliverable is count (ETA 20 min, model/count_co_events.py:202) PLUS merge (ETA 30 min,
    :210): the per-file tables of the first n_files files (oracle/covis_oracle.c, files over a pool of
    `threads` threads, the tables materialised as the reference writes them, :94-100), then
    concat_files_w_stats (:103-181, the numpy restatement oracle/covis.py with the reference's thresholds:
    per-file count >= 2 filter of click_to tables when N > 1e8, MIN_COUNT_TO_SAVE, count desc, head) of
    every rule over those tables. value = qualifying pairs / (count + merge seconds)."""
    from concurrent.futures import ThreadPoolExecutor
    import covis as oracle
    ev, fb = _files(n_files, seed)
    off = np.asarray(ev.session_offsets, np.int64)

    def one(f):
        s0, s1 = int(fb[f]), int(fb[f + 1])
        e0, e1 = int(off[s0]), int(off[s1])
        return oracle.count_co_events_file(off[s0:s1 + 1], ev.aid[e0:e1], ev.ts[e0:e1], ev.type[e0:e1])

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as pool:  # ctypes releases the GIL inside the C count
        tabs = list(pool.map(one, range(len(fb) - 1)))
    count_s = time.perf_counter() - t0
    pairs = sum(int(t[n][2].sum(dtype=np.int64)) for t in tabs for n in oracle.REFERENCE_RULES)
    rows_in = sum(len(t[n][0]) for t in tabs for n in oracle.REFERENCE_RULES)
    t0 = time.perf_counter()
    rows_out = {}
    for n in oracle.REFERENCE_RULES:
        a, _, _ = oracle.concat_files_w_stats(n, [t[n] for t in tabs])
        rows_out[n] = int(len(a))
    merge_s = time.perf_counter() - t0
    return {"value": pairs / (count_s + merge_s), "unit": "pairs/s", "cores": threads, "kind": "port",
            "count_s": round(count_s, 2), "merge_s": round(merge_s, 2), "pairs": pairs, "file_rows": rows_in,
            "merge_rows_per_s": rows_in / merge_s, "rows_out": rows_out, "files": len(fb) - 1,
            "sample": f"count + merge of the first {len(fb) - 1} files ({ev.n_sessions} sessions, {pairs} pairs, "
                      f"{rows_in} per-file rows): oracle/covis_oracle.c per-file tables over {threads} threads "
                      f"({count_s:.1f} s), then oracle/covis.py concat_files_w_stats of the 5 rules with the "
                      f"reference's thresholds (numpy, one core, {merge_s:.1f} s)"}


def main():
    cfg = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
    cores = host_cores()
    n = int(cfg.get("threads") or cores["usable"])
    seed = int(cfg.get("seed", 0))
    out = {"host": cores}
    pf = int(cfg.get("port_files", max(10, 2 * n)))
    out["port"] = port(min(pf, int(cfg.get("max_files", 135))), n, seed)
    pdf = int(cfg.get("pandas_files", 10))
    if pdf > 0:
        out["pandas"] = pandas_pool(pdf, min(n, pdf), seed)
    mf = int(cfg.get("merge_files", 16))
    if mf > 0:
        out["merge"] = count_plus_merge(mf, n, seed)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
