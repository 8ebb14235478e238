"""Benchmark: co-visitation build over synthetic OTTO-shaped sessions on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--events E]

One step = one full co-visitation build of BASELINE.json configs[1]: all five rules over
~220M events (100k-session files) -> per-(rule, aid, aid_next) count and count_ge2 tables
resident in HBM (model/count_co_events.py:80-100 + the cross-file groupby of :168).
Inputs are resident in HBM before the timed region. Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
# latest committed PMC traffic summary (tools/evidence_r2.sh -> profiles/r<NN>_pmc_traffic.json)
def _latest_pmc_file():
    import re
    best = (-1, os.path.join(ROOT, "profiles", "none"))
    for f in os.listdir(os.path.join(ROOT, "profiles")):
        m = re.fullmatch(r"r(\d+)_pmc_traffic\.json", f)
        if m and int(m.group(1)) > best[0]:
            best = (int(m.group(1)), os.path.join(ROOT, "profiles", f))
    return best[1]


PMC_FILE = _latest_pmc_file()
# kernels of each co-visitation phase (HIP-event timed on the launch stream; rocprof sums agree)
PHASE_KERNELS = {"prep_count": "k_block_first + k_prep_count", "rows": "radix sort (k_rs_*), k_gather_counts, scans, k_rows",
                 "emit": "k_emit", "reduce": "k_classify_rows, k_agg_sort<M>, k_agg_hash, k_split_*, scans"}


def pmc_traffic(key: str):
    """Measured HBM bytes per launch/step (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate --pmc
    passes of this same command; see PMC_FILE), or None if not collected."""
    try:
        return float(json.load(open(PMC_FILE))[key]["traffic_bytes"])
    except Exception:
        return None


def cpu_baseline(seed: int = 0, pandas_files: int = 10) -> dict:
    """The CPU path timed on this host's cores in a child process (oracle/cpu_baseline.py, which
    never touches the GPU): the C restatement over whole files of the same stream on every usable
    core (OpenMP, the strong CPU baseline: `value`), and the pandas op-for-op restatement of the
    reference's dataframe pipeline as a process pool over `pandas_files` files
    (`reference_algorithm`). BASELINE.md §2."""
    import subprocess
    cfg = json.dumps({"seed": seed, "pandas_files": pandas_files})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), cfg], capture_output=True,
                       text=True, timeout=900)
    if r.returncode != 0:
        return {"error": r.stderr[-2000:]}
    res = json.loads(r.stdout.strip().splitlines()[-1])
    out = dict(res["port"])
    out["host_cpus"] = res["host"]
    if "pandas" in res:
        out["reference_algorithm"] = res["pandas"]
    if "merge" in res:  # count + merge on the CPU (beside a6.count_plus_merge_pairs_per_s)
        out["count_plus_merge"] = res["merge"]
    return out


MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16, /opt/skills/guides/MI355X_MICROARCH.md


def bench_a6(dev, ctx, reps: int = 3) -> dict:
    """Count + merge, the reference's deliverable (ETAs :202, :210): the count that A6 (model/count_co_events.py:
    103-181) needs -- all five rules with click_to_click's rows histogrammed per file (branch (2)'s row-slice plan;
    OTTOHIP_A6_REFOLD=1 also keeps the pair words, covis.a6_refold) -- timed `reps` times (min: count_ms), then per
    rule A6 on that table: the per-file count >= 2 filter, branch (2) where
    N > MAX_ROWS_POLARS_GROUPBY, MIN_COUNT_TO_SAVE, count-desc order and head. Reported beside the line, not
    part of `value`. A6: one untimed warmup pass, then `reps` timed passes (min reported, every run listed);
    the last run records per-stage times of the part-wise rule."""
    import torch
    from otto_recommender_amd import covis as gc, config as cfg
    cts = []
    tab = None
    for _ in range(reps + 1):  # the first: untimed warmup (allocations)
        if tab is not None:
            tab.free()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tab = gc.count_co_events_fused(dev, ctx=ctx, per_file_rule="click_to_click", keep_words=gc.a6_refold())
        torch.cuda.synchronize()
        cts.append((time.perf_counter() - t0) * 1e3)
    count_ms = min(cts[1:])
    per = {}
    totals = []
    # one untimed warmup pass first (its first-use allocations: the part-wise count's word buffers and
    # table at > 100 GB resident), reported as warmup_ms
    torch.cuda.synchronize()
    tw = time.perf_counter()
    for n in tab.names:
        gc.concat_files_w_stats_fused(dev, n, table=tab, ctx=ctx)
    torch.cuda.synchronize()
    warm_ms = (time.perf_counter() - tw) * 1e3
    for rep in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for n in tab.names:
            t1 = time.perf_counter()
            stages = {} if rep == reps - 1 else None
            a, _, _ = gc.concat_files_w_stats_fused(dev, n, table=tab, ctx=ctx, timings=stages)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t1) * 1e3
            st = tab.stats(n)
            use_ge2 = "click_to" in n and st["file_rows"] > cfg.CLICK_FILTER_ROWS
            N = st["file_rows_ge2"] if use_ge2 else st["file_rows"]
            d = per.setdefault(n, {"ms_runs": [], "rows_out": int(a.numel()), "file_rows_N": int(N),
                                   "part_wise": bool(N > cfg.MAX_ROWS_POLARS_GROUPBY)})
            d["ms_runs"].append(round(ms, 2))
            if stages:
                d["stages_ms"] = {k: round(v * 1e3, 2) for k, v in stages.items()}
            del a
        totals.append((time.perf_counter() - t0) * 1e3)
    for d in per.values():
        d["ms"] = min(d["ms_runs"])
    tab.free()
    return {"per_rule": per, "total_ms": round(min(totals), 2), "total_ms_runs": [round(x, 2) for x in totals],
            "max_over_min": round(max(totals) / min(totals), 3), "reps": reps, "warmup_ms": round(warm_ms, 2),
            "count_ms": round(count_ms, 2), "count_ms_runs": [round(x, 2) for x in cts[1:]],
            "count_note": "the count A6 uses: the line's build plus click_to_click's per-file row histogram"}


def bench_ingest(ev, fb, dev, ctx, reps: int = 3) -> dict:
    """Event ingest: the raw rows of the 220 M-event workload, resident in HBM as
    the reference's parquet columns (session, aid, ts, type) in file order, grouped into the session CSR
    by ottohip_events_csr file by file (`DeviceEvents.from_columns`, the path of `from_parquet`).
    Algorithmic bytes: read session 4E, write offsets 8S, copy aid/ts/type 9E + 9E. Checked against
    the host-built CSR the co-visitation line counts on."""
    import torch
    from otto_recommender_amd import covis as gc
    cols = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (ev.session, ev.aid, ev.ts, ev.type)]
    off = ev.session_offsets
    file_rows = (off[fb[1:]] - off[fb[:-1]]).tolist()
    gc.DeviceEvents.from_columns(*cols, file_rows=file_rows, ctx=ctx)  # warmup (workspace)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        d = gc.DeviceEvents.from_columns(*cols, file_rows=file_rows, ctx=ctx)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ok = bool(torch.equal(d.offsets, dev.offsets) and torch.equal(d.aid, dev.aid) and torch.equal(d.ts, dev.ts)
              and torch.equal(d.type, dev.type) and np.array_equal(d.file_bounds, dev.file_bounds))
    E, S = ev.n_events, ev.n_sessions
    alg = 4.0 * E + 8.0 * (S + 1) + 18.0 * E
    return {"ms": round(dt * 1e3, 3), "events_per_s": E / dt, "files": len(file_rows), "matches_host_csr": ok,
            "roofline": {"bound": "hbm", "achieved": alg / dt / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / dt / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": alg,
                         "note": "host-clock time of one ottohip_events_csr_files call over all files (three small device->host reads)"}}


def bench_knn(steps: int, warmup: int, n_items: int, n_q: int, with_cpu: bool, group=None) -> dict:
    """BASELINE configs[2]: exact top-20 kNN of the first n_q vocabulary rows. group: the queries
    are split in equal ranges over the ranks (the item matrix replicated on every GPU, SURVEY.md
    §8(e)); value = all ranks' queries / the slowest rank's time."""
    import torch
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import _lib
    from otto_recommender_amd.w2vec import KnnIndex
    ctx = _lib.context()
    emb = synth.embeddings(n_items)
    n_q = min(n_q, n_items)
    index = KnnIndex(emb, ctx)
    world, rank, rows, n_mine = 1, 0, None, n_q
    if group is not None:
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        q0, q1 = n_q * rank // world, n_q * (rank + 1) // world
        rows = torch.arange(q0, q1, dtype=torch.int32, device=torch.device("cuda", ctx.device))
        n_mine = q1 - q0

    def search():
        return index.search(rows, k=20) if rows is not None else index.search(None, n_q=n_q, k=20)

    def barrier():
        if group is not None:
            import torch.distributed as dist
            dist.barrier(group)

    for _ in range(warmup):
        search()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        idx, d2 = search()
    torch.cuda.synchronize()
    barrier()
    dt = (time.perf_counter() - t0) / steps
    if group is not None:  # slowest rank
        import torch.distributed as dist
        cdev = torch.device("cuda", ctx.device) if dist.get_backend(group) == "nccl" else "cpu"
        m = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
        dt = float(m.item())
    ctx.set_timing(True)
    search()
    ph = {n: ms for n, ms, _ in ctx.timings()}
    ctx.set_timing(False)
    flops = 2.0 * n_mine * n_items * emb.shape[1]  # this rank's launch
    main_ms = ph.get("knn_main", dt * 1e3)
    out = {"metric": "W2V top-20 kNN queries/s (exact, bf16 MFMA + fp32 rerank)", "value": n_q / dt,
           "unit": "queries/s", "ms_per_step": dt * 1e3, "steps": steps, "n_gpus": world,
           "config": {"workload": "configs[2]: 1.86M items x 100-d, 600k queries, k=20", "items": n_items,
                      "queries": n_q, "k": 20},
           "dtype": "bf16 (fp32 accumulate, fp32 rerank)",
           "roofline": {"bound": "mfma", "kernel": "k_knn_main", "achieved": flops / (main_ms / 1e3) / 1e12,
                        "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": flops / (main_ms / 1e3) / 1e12 / MFMA_BF16_PEAK_TFLOPS,
                        "traffic": pmc_traffic("k_knn_main") if n_items == 1_855_603 and n_mine == 600_000 else None,
                        "traffic_note": "HBM/fabric bytes per launch (every 512-query workgroup streams the item matrix)",
                        "flops_model": "2*Q*V*100 (the padded K (104 for dim 100: the +-norm columns and zeros) and the top-k epilogue not counted)",
                        # the whole search (pre-pass, main pass, candidate selection, rerank) on the same flops
                        "search_ms": sum(ph.values()),
                        "search_frac": flops / (sum(ph.values()) / 1e3) / 1e12 / MFMA_BF16_PEAK_TFLOPS if ph else None},
           "phases_ms": {k: round(v, 3) for k, v in ph.items()},
           "reference_faiss_ivf_queries_per_s": 705}
    if world > 1:
        out["config"]["parallelism"] = f"queries split over {world} GPU(s), item matrix replicated"
    if with_cpu and world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import knn as oracle_knn  # checker / baseline only
        from cpu_baseline import host_cores
        hc = host_cores()
        torch.set_num_threads(hc["usable"])
        nq_cpu = 2000
        t0 = time.perf_counter()
        ri, _ = oracle_knn.topk_exact(emb, np.arange(nq_cpu), 20)
        tc = time.perf_counter() - t0
        gi = idx[:nq_cpu].cpu().numpy()
        out["sample_exact_match"] = float(np.mean([set(a) == set(b) for a, b in zip(gi, ri)]))
        out["cpu_baseline"] = {"value": nq_cpu / tc, "unit": "queries/s", "cores": torch.get_num_threads(), "host_cpus": hc,
                               "kind": "port",
                               "sample": f"{nq_cpu} queries, exact brute force (oracle/knn.py: torch-CPU fp32 "
                                         f"preselect + fp64 rerank), {tc:.1f} s"}
    index.free()
    return out


def bench_candidates(n_sessions: int, steps: int, kmeans_iter: int, group=None, warmup: int = 1) -> dict:
    """BASELINE configs[4]: end-to-end candidate generation (co-visit + W2V kNN + pop-cluster) for
    the test split of n_sessions synthetic sessions; value = candidate rows / s of the whole job.
    group: the sharded pipeline over every rank (files, kNN queries, KMeans rows, C3 counters and
    test sessions split; pipeline.run(group=...)), timed as the max over ranks."""
    import torch
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import pipeline, config as cfg
    ev = synth.generate(n_sessions)
    train, test, labels = synth.split_test_labels(ev)
    del ev
    words = synth.item_words()
    emb_all = synth.embeddings(len(words), seed=1)
    emb_12 = synth.embeddings(len(words), seed=3)
    res, dts = None, []
    for _ in range(warmup):  # untimed: first-use device allocations, code object loads
        pipeline.run(train, test, labels, words, emb_all, words, emb_12, kmeans_iter=kmeans_iter, group=group)
    for _ in range(max(steps, 1)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        T = {}
        res = pipeline.run(train, test, labels, words, emb_all, words, emb_12, kmeans_iter=kmeans_iter, timings=T,
                           group=group)
        torch.cuda.synchronize()
        dts.append(time.perf_counter() - t0)
    world = 1
    if group is not None:  # slowest rank
        import torch.distributed as dist
        world = dist.get_world_size(group)
        cdev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
        m = torch.tensor(dts, dtype=torch.float64, device=cdev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
        dts = m.tolist()
    # inputs resident in HBM: the host->device upload of the event table and the label rows is input
    # preparation, reported but not in the timed step (the label CSR is built on the device, timed)
    prep = res["timings_s"].get("upload", 0.0)
    dt = min(dts) - prep
    return {"metric": "candidates/sec, end-to-end candidate generation (co-visit + W2V kNN + pop-cluster)",
            "value": res["candidates"] / dt, "unit": "candidates/s", "ms_per_step": dt * 1e3,
            "input_prep_s": round(prep, 4), "steps": max(steps, 1), "warmup": warmup,
            "n_gpus": world,
            "config": {"workload": f"configs[4] on {world} GPU(s): train + truncated test split of synthetic sessions",
                       "sessions": n_sessions, "test_sessions": res["test_sessions"], "candidates": res["candidates"],
                       "co_visit_pairs": res["pairs"], "kmeans_iter": res["kmeans_iter"]},
            "recall@20": {k: round(v["top20"], 6) for k, v in res["recall"].items()},
            "recall_topall": {k: round(v["topall"], 6) for k, v in res["recall"].items()},
            "stages_s": {k: round(v, 4) for k, v in res["timings_s"].items()},
            "outside_stages_s": round(min(dts) - sum(res["timings_s"].values()), 4),
            "data": "synthetic (otto-synth seed 0, embeddings seeds 1/3, labels by the OTTO protocol)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--events", type=int, default=220_000_000)
    ap.add_argument("--pandas-files", type=int, default=10, help="files of the pandas reference-algorithm baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-a6", action="store_true", help="skip the A6 (concat_files_w_stats) timing beside the line")
    ap.add_argument("--no-ingest", action="store_true", help="skip the event-ingest (device CSR build) timing")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--knn-steps", type=int, default=2, help="0 disables the configs[2] kNN measurement")
    ap.add_argument("--workload", choices=["covis", "knn", "candidates"], default="covis",
                    help="covis: configs[1] line (+ the kNN sub-object); knn: only configs[2]; "
                         "candidates: configs[4] end-to-end on 1 GPU")
    ap.add_argument("--cand-sessions", type=int, default=12_900_000)
    ap.add_argument("--cand-steps", type=int, default=1, help="0 disables the configs[4] candidates sub-object")
    ap.add_argument("--kmeans-iter", type=int, default=100)
    ap.add_argument("--knn-items", type=int, default=1_855_603)
    ap.add_argument("--knn-queries", type=int, default=600_000)
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI (the product); gloo = host-staged rehearsal on fewer GPUs")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import covis as gc
    from otto_recommender_amd import _lib

    if args.workload == "candidates":
        torch.cuda.set_device(0)
        print(json.dumps(bench_candidates(args.cand_sessions, args.steps, args.kmeans_iter)))
        return
    if args.workload == "knn":
        torch.cuda.set_device(0)
        print(json.dumps(bench_knn(max(args.knn_steps, 1), 1, args.knn_items, args.knn_queries, not args.no_cpu)))
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        local = local % max(torch.cuda.device_count(), 1)  # gloo rehearsals may share a GPU
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    from otto_recommender_amd import dist as gd

    # ---- workload: sessions until E events, 100k-session files, files dealt to ranks
    n_sess, n_ev = synth.sessions_for_events(args.events, 0, args.seed)
    fb_all = synth.file_session_bounds(n_sess)
    n_files = len(fb_all) - 1
    if world > 1:  # whole files per rank, balanced by sum of n_s^2 (work ∝ pairs)
        lens = synth.session_lengths(n_sess, 0, args.seed).astype(np.float64)
        weights = [float((lens[fb_all[f]:fb_all[f + 1]] ** 2).sum()) for f in range(n_files)]
        my_files = gd.deal_files(n_files, rank, world, weights)
    else:
        my_files = list(range(n_files))
    t0 = time.perf_counter()
    parts = [synth.generate(int(fb_all[f + 1] - fb_all[f]), int(fb_all[f]), args.seed) for f in my_files]
    sizes = [p.n_sessions for p in parts]
    fb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    off = np.zeros(int(fb[-1]) + 1, np.int64)
    base = 0
    for i, p in enumerate(parts):
        off[fb[i]:fb[i + 1] + 1] = p.session_offsets + base
        base += p.n_events
    ev = synth.Events(off, np.concatenate([p.session for p in parts]), np.concatenate([p.aid for p in parts]),
                      np.concatenate([p.ts for p in parts]), np.concatenate([p.type for p in parts]))
    del parts
    gen_s = time.perf_counter() - t0
    dev = gc.DeviceEvents.from_host(ev, fb)
    ctx = _lib.context()
    torch.cuda.synchronize()

    # the line's build: the five count tables (configs[1]); A/B switches: OTTOHIP_BENCH_PER_FILE=<rule> adds a
    # rule's per-file row histogram, OTTOHIP_BENCH_KEEP=1 keeps the pair words (what A6's count adds, bench_a6)
    pfr = os.environ.get("OTTOHIP_BENCH_PER_FILE", "none")
    pfr = None if pfr in ("", "none", "0") else pfr
    keep = os.environ.get("OTTOHIP_BENCH_KEEP", "0") == "1"

    def step():
        if world > 1:  # local count -> pack by owner -> all-to-all-v (RCCL) -> merge-sum
            return gd.count_co_events_sharded(dev, my_files, n_files, ctx=ctx, per_file_rule=pfr)
        return gc.count_co_events_fused(dev, ctx=ctx, per_file_rule=pfr, keep_words=keep)

    for _ in range(args.warmup):
        step().free()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tab = None
    for _ in range(args.steps):
        if tab is not None:
            tab.free()  # returns its buffers to the context for the next build
        tab = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    stats = {n: tab.stats(n) for n in tab.names}
    pairs = sum(s["n_pairs"] for s in stats.values())
    rows = sum(s["n_rows"] for s in stats.values())

    # phase timing of one extra (untimed) step with HIP events on the launch stream
    ctx.set_timing(True)
    tab.free()
    tab = step()
    phases = ctx.timings()
    ctx.set_timing(False)
    a6 = None
    tab.free()
    if world == 1 and not args.no_a6:
        ctx.trim()  # the build's word buffers
        try:  # reported beside the line; it must not cost the main line
            a6 = bench_a6(dev, ctx)
        except Exception as exc:  # noqa: BLE001
            a6 = {"error": repr(exc)}
    ingest = None
    if world == 1 and not args.no_ingest:
        ctx.trim()
        try:  # reported beside the line
            ingest = bench_ingest(ev, fb, dev, ctx)
        except Exception as exc:  # noqa: BLE001
            ingest = {"error": repr(exc)}
        ctx.trim()
        torch.cuda.empty_cache()

    t_step = dt / args.steps
    if world > 1:
        cdev = "cuda" if args.dist_backend == "nccl" else "cpu"
        tt = torch.tensor([t_step, float(pairs), float(rows), float(ev.n_events)], dtype=torch.float64, device=cdev)
        t_max = tt[:1].clone(); dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        tot = tt[1:].clone(); dist.all_reduce(tot)
        t_step = float(t_max.item()); pairs, rows, n_events = (float(x) for x in tot.tolist())
    else:
        n_events = ev.n_events
    if rank != 0:  # the other ranks join the sharded kNN and config-5 runs, then leave
        del dev, tab
        ctx.trim()
        torch.cuda.empty_cache()
        if args.knn_steps > 0:
            bench_knn(args.knn_steps, 1, args.knn_items, args.knn_queries, False, dist.group.WORLD)
            ctx.trim()
            torch.cuda.empty_cache()
        if args.cand_steps > 0:
            try:
                bench_candidates(args.cand_sessions, args.cand_steps, args.kmeans_iter, dist.group.WORLD)
            except Exception:  # noqa: BLE001  (rank 0 reports the error)
                pass
        dist.destroy_process_group()
        return
    # byte model of SURVEY.md §8(d): B = 9E + 8(S+1) + 16P + 12U
    b_model = 9.0 * n_events + 8.0 * (n_sess + 1) + 16.0 * pairs + 12.0 * rows
    # algorithmic bytes per phase (one launch group per build; DESIGN.md §5 derives each):
    #   prep_count  read aid/ts/type + offsets (9E + 8S), write ev, cnt, row key, position (20E)
    #   rows        read row keys + counts (8E), write word offsets (8E) + row keys / starts (12U_r)
    #   emit        read ev, cnt, word offsets + offsets (20E + 8S), write one 4-B word per pair (4P)
    #   reduce      read every pair word once (4P), write every output row once (17U)
    E_, S_ = n_events / world, n_sess / world
    alg = {"prep_count": 29.0 * E_ + 8.0 * S_, "rows": 16.0 * E_, "emit": 20.0 * E_ + 8.0 * S_ + 4.0 * pairs / world,
           "reduce": 4.0 * pairs / world + 17.0 * rows / world}
    ph_ms = {p[0]: p[1] for p in phases}
    dom = max(phases, key=lambda p: p[1]) if phases else ("step", t_step * 1e3, b_model)

    def roof(ph):
        a = alg.get(ph, b_model) / (ph_ms[ph] / 1e3) / 1e9
        tr = pmc_traffic(f"covis_{ph}_phase") if world == 1 else None
        return {"bound": "hbm", "kernel": ph, "kernels": PHASE_KERNELS.get(ph, ph), "achieved": a,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": a / HBM_PEAK_GBS, "traffic": tr,
                "algorithmic_bytes": alg.get(ph, b_model), "ms": ph_ms[ph],
                "traffic_source": f"{os.path.relpath(PMC_FILE, ROOT)} (rocprofv3 --pmc FETCH_SIZE x2, WRITE_SIZE)"}
    out = {
        "metric": "co-visit pairs/sec + candidates/sec at 220M events, 1/2/4/8 MI355X",
        "value": pairs / t_step,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_step * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (otto-synth seed 0, SURVEY.md §8(d)); inputs resident in HBM",
        "config": {"workload": "configs[1]: all 5 co-visitation rules, 220M events, 100k-session files",
                   "events": int(n_events), "sessions": int(n_sess), "files": n_files,
                   "parallelism": f"files dealt over {world} GPU(s)" + (
                       f", owner(aid) all-to-all-v merge over {args.dist_backend}" if world > 1 else "")},
        "pairs": int(pairs), "rows": int(rows),
        "events_per_s": n_events / t_step,
        "step_roofline": {"bound": "hbm", "model_bytes": b_model, "achieved": b_model / t_step / 1e9,
                          "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": b_model / t_step / 1e9 / HBM_PEAK_GBS},
        "roofline": roof(dom[0]),
        "phase_rooflines": {ph: roof(ph) for ph in ph_ms if ph in alg},
        "phases_ms": {p[0]: round(p[1], 3) for p in phases},
        "gen_s": round(gen_s, 1),
    }
    if a6 is not None:
        if "total_ms" in a6:
            cpm = (a6["count_ms"] + a6["total_ms"]) / 1e3
            a6["count_plus_merge_ms"] = round(cpm * 1e3, 2)
            # the reference's deliverable is count + merge (ETAs :202, :210): pairs counted per second of both
            a6["count_plus_merge_pairs_per_s"] = pairs / cpm
        out["a6"] = a6
    if ingest is not None:
        out["ingest"] = ingest
    if not args.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(args.seed, args.pandas_files)
    if args.knn_steps > 0:
        del dev
        ctx.trim()  # each sub-benchmark starts from an empty workspace (its own buffers only)
        torch.cuda.empty_cache()
        out["knn"] = bench_knn(args.knn_steps, 1, args.knn_items, args.knn_queries, not args.no_cpu and world == 1,
                               dist.group.WORLD if world > 1 else None)
    if args.cand_steps > 0:
        if world > 1 and args.knn_steps == 0:
            del dev
        ctx.trim()
        torch.cuda.empty_cache()
        try:  # the sub-object must not cost the main line
            cand = bench_candidates(args.cand_sessions, args.cand_steps, args.kmeans_iter,
                                    dist.group.WORLD if world > 1 else None)
        except Exception as e:  # noqa: BLE001
            cand = {"error": f"{type(e).__name__}: {e}"[:2000]}
        if rank == 0:
            out["candidates"] = cand
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
