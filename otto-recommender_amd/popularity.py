"""Pop-cluster source of config 5 and session-item similarity.

  compute_sessions_embeddings   model/kmeans_sessions.py:40-86
  KMeans (fit / labels_)        model/kmeans_sessions.py:140-171, the scikit-learn==1.2 branch
                                (init='random', n_init='auto' = 10 runs, empty-cluster relocation,
                                strict convergence); the reference's dask-ml k-means|| default is
                                not reproducible
  count_popularity              model/count_popularity.py:53-85 (ranks_for_clusters)
  session_item_similarity       model/retrieve.py:604-625
All compute runs in libottohip.so (csrc/popularity.hip).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from . import config

RANK_COLS = ["rank_clicks", "rank_carts", "rank_orders", "rank_clicks_7d", "rank_carts_7d", "rank_orders_7d"]


def _t(x, dev, dtype):
    import torch
    return (x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))).to(dev, dtype).contiguous()


def row_of_aid_map(words, n_items: int, dev):
    """aid -> embedding row (vocabulary order), -1 for aids without an embedding."""
    import torch
    words = np.asarray(words, np.int64)
    n = max(int(n_items), int(words.max()) + 1 if len(words) else 1)
    m = np.full(n, -1, np.int32)
    m[words] = np.arange(len(words), dtype=np.int32)
    return torch.from_numpy(m).to(dev)


def compute_sessions_embeddings(offsets, aid, ts, type_, words, embeddings, n_items: int = config.N_ITEMS_OTTO,
                                ctx=None, stream=None, rmap=None):
    """C1 for a session-sorted event table: torch f32 [n_sessions, dim] on the device.
    rmap: row_of_aid_map(words, n_items, device), if the caller holds it already."""
    import torch
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    off = _t(offsets, dev, torch.int64)
    off = off - off[0]
    a, s_, y = _t(aid, dev, torch.int32), _t(ts, dev, torch.int32), _t(type_, dev, torch.int8)
    emb = _t(embeddings, dev, torch.float32)
    rmap = row_of_aid_map(words, n_items, dev) if rmap is None else rmap
    S = int(off.numel()) - 1
    dim = int(emb.shape[1])
    out = torch.empty((max(S, 1), dim), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().ottohip_session_embeddings(ctx.h, _lib.ptr(off), S, _lib.ptr(a), _lib.ptr(s_), _lib.ptr(y),
                                                      _lib.ptr(rmap), int(rmap.numel()), _lib.ptr(emb), dim,
                                                      _lib.ptr(out), _lib.stream_handle(stream)))
    return out[:S]


FX = float(1 << 24)  # fixed-point scale of the device sums (csrc/popularity.hip KM_FX)
LLOYD_BATCH = 10  # Lloyd steps per ottohip_kmeans_lloyd_steps call (the stop checks run on the device)
KM_GROUP = 1  # n_init runs in lockstep per read of X (ottohip_kmeans_lloyd_steps_multi); 1: one bounded run at a time
KM_LANES = 1  # runs on this many host threads, each with its own context and stream (OTTOHIP_KM_LANES); 2 lanes measured slower


def _allreduce(t, group):
    if group is None:
        return t
    from .dist import _allreduce_sum
    return _allreduce_sum(t, group)


class SeedHeads:
    """numpy RandomState(seed).permutation(n)[:k] for `runs` successive calls (sklearn 1.2's
    KMeans(init='random') seeds of its n_init runs), by the library's MT19937 replica
    (ottohip_rs_permutation_head). All `runs` heads are drawn in order by a background thread from
    construction on (ctypes releases the GIL): built before the stages that precede C2 (pipeline.run),
    the ~0.1-0.3 s of draws for n ~ 13 M no longer sit in front of the first Lloyd step. Iterating
    yields the heads in run order (blocking until each is drawn)."""

    def __init__(self, seed: int, n: int, k: int, runs: int):
        import queue
        import threading
        self.key = (int(seed), int(n), int(k), int(runs))
        self._q = queue.Queue()
        self._t = threading.Thread(target=self._work, daemon=True)
        self._t.start()

    def _work(self):
        seed, n, k, runs = self.key
        lib = _lib.load()
        h = ctypes.c_void_p()
        try:
            _lib.check(lib.ottohip_rs_create(seed & 0xFFFFFFFF, ctypes.byref(h)))
            for _ in range(runs):
                out = np.empty(k, np.int64)
                _lib.check(lib.ottohip_rs_permutation_head(h, n, k, out.ctypes.data))
                self._q.put(out)
        except BaseException as e:  # re-raised in the consumer
            self._q.put(e)
        finally:
            if h:
                lib.ottohip_rs_destroy(h)

    def __iter__(self):
        return self

    def __next__(self):
        item = self._q.get()
        if isinstance(item, BaseException):
            raise item
        return item

    def close(self):
        self._t.join()


def _permutation_heads(seed: int, n: int, k: int, runs: int) -> SeedHeads:
    return SeedHeads(seed, n, k, runs)


class KMeans:
    """KMeans(n_clusters, init='random', n_init='auto', max_iter=100, tol=1e-3, random_state=42):
    the reference's scikit-learn branch (model/kmeans_sessions.py:152-159, scikit-learn==1.2) on a
    device matrix, run as sklearn 1.2's KMeans.fit + _kmeans_single_lloyd:
      - X is centred on its column means; tol is scaled by the mean column variance;
      - n_init ('auto' = 10 for init='random') runs, each seeded by the rows
        RandomState(random_state).permutation(n)[:k] of the same RandomState (sklearn 1.2
        _init_centroids); the run with the lowest inertia is kept;
      - Lloyd iterations: E-step, per-cluster sums, empty clusters relocated to the rows farthest
        from their centroid (_relocate_empty_clusters_dense), M-step; stop when no label changed
        (strict convergence) or the squared centre shift <= tol; without strict convergence the
        labels are recomputed with the final centres; inertia = sum |x - c[label]|^2.
    The reference's default dask-ml k-means|| path draws from dask's chunked random streams and is
    not reproducible. group: rows sharded over ranks: the sums,
    counts and statistics are all-reduced (exact 2^-24 fixed point), so every rank ends with the
    single-GPU result. Ties between equal inertias keep the earlier run (sklearn also skips a run
    that is the same clustering)."""

    def __init__(self, n_clusters: int = 50, max_iter: int = 100, tol: float = 1e-3, random_state: int = 42,
                 init: str = "random", n_init="auto"):
        if init != "random":
            raise ValueError("init='random' (the reference's sklearn branch) is the supported initialisation")
        self.n_clusters, self.max_iter, self.tol, self.random_state = n_clusters, max_iter, tol, random_state
        self.init = init
        self.n_init = 10 if n_init == "auto" else int(n_init)

    def fit(self, X, ctx=None, stream=None, group=None, global_rows=None, seed_heads=None):
        """seed_heads: a SeedHeads(random_state, n_samples, n_clusters, n_init) started earlier (the same draws,
        computed ahead); one with another key is not used."""
        import torch
        ctx = ctx or _lib.context()
        dev = torch.device("cuda", ctx.device)
        lib = _lib.load()
        sh = _lib.stream_handle(stream)
        X = _t(X, dev, torch.float32)
        n, dim = (int(v) for v in X.shape)
        k = self.n_clusters
        if group is not None:  # this rank's rows are the global rows `global_rows` (increasing)
            from .dist import all_gather_sizes
            n_all = sum(all_gather_sizes(n, group))
            grows = np.arange(n, dtype=np.int64) if global_rows is None else np.asarray(global_rows, np.int64)
            if len(grows) != n or np.any(np.diff(grows) <= 0):
                raise ValueError("global_rows: one increasing global row id per local row")
        else:
            n_all, grows = n, None  # one GPU: local row = global row (no 8 B per row of host ids)
        if n_all < k:
            raise ValueError(f"n_samples={n_all} should be >= n_clusters={k}")
        # column means (exact fixed-point sums), centring, tol = mean variance * tol
        s1 = torch.empty(dim, dtype=torch.int64, device=dev)
        s2 = torch.empty(dim, dtype=torch.int64, device=dev)
        _lib.check(lib.ottohip_col_sums(ctx.h, _lib.ptr(X), n, dim, None, _lib.ptr(s1), _lib.ptr(s2), sh))
        s1 = _allreduce(s1, group)
        mean = (s1.cpu().numpy().astype(np.float64) / FX / n_all).astype(np.float32)
        mean_d = torch.from_numpy(mean).to(dev)
        Xc = torch.empty_like(X)
        _lib.check(lib.ottohip_center_rows(ctx.h, _lib.ptr(X), n, dim, _lib.ptr(mean_d), _lib.ptr(Xc), sh))
        _lib.check(lib.ottohip_col_sums(ctx.h, _lib.ptr(Xc), n, dim, None, _lib.ptr(s1), _lib.ptr(s2), sh))
        s1, s2 = _allreduce(s1, group), _allreduce(s2, group)
        m1 = s1.cpu().numpy().astype(np.float64) / FX / n_all
        var = s2.cpu().numpy().astype(np.float64) / FX / n_all - m1 * m1
        tol_abs = float(np.mean(var)) * self.tol
        key = (int(self.random_state), int(n_all), int(k), int(self.n_init))
        seed_stream = seed_heads if seed_heads is not None and seed_heads.key == key else \
            _permutation_heads(self.random_state, n_all, k, self.n_init)
        # one GPU: the E-steps read f16 copies of the centred rows (exact f32 scoring of the near ties keeps the
        # f32 labels); every fit attaches its own Xc, so a reused allocation never meets a stale copy
        half = group is None and dim % 4 == 0 and os.environ.get("OTTOHIP_KM_H16", "1") != "0"
        if half:
            # refused (ELIMIT) when some |x| is outside the f16 range bound: the E-steps then score the f32 rows
            rc = lib.ottohip_kmeans_attach_half(ctx.h, _lib.ptr(Xc), n, dim, sh)
            half = rc == 0
            if rc not in (0, _lib.OTTOHIP_ELIMIT):
                _lib.check(rc)
        try:
            return self._fit_runs(X, Xc, n, dim, k, group, grows, tol_abs, seed_stream, mean_d, ctx, sh, dev, half)
        finally:
            seed_stream.close()
            if half:  # always paired with the attach: a later fit never meets this fit's f16 copy
                lib.ottohip_kmeans_detach_half(ctx.h)

    def _fit_runs(self, X, Xc, n, dim, k, group, grows, tol_abs, seed_stream, mean_d, ctx, sh, dev, half=False):
        """fit's n_init runs (the Lloyd loops) over the centred rows Xc; keeps the best by inertia."""
        import torch
        lib = _lib.load()
        sums = torch.empty(k * dim, dtype=torch.int64, device=dev)
        counts = torch.empty(k, dtype=torch.int64, device=dev)
        labels = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        best = None
        inr, chg, shift = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        st6 = (ctypes.c_double * 6)()
        # one GPU: up to KM_GROUP runs in lockstep over one read of X per Lloyd step
        # (ottohip_kmeans_lloyd_steps_multi); OTTOHIP_KM_GROUP=1 runs them one at a time with distance bounds
        grp = int(os.environ.get("OTTOHIP_KM_GROUP", str(KM_GROUP)))
        multi_ok = group is None and 32 < k <= 64 and dim <= 112 and dim % 4 == 0 and grp >= 2
        pending = []  # later runs of a lockstep group, in run order
        lanes = int(os.environ.get("OTTOHIP_KM_LANES", str(KM_LANES)))
        if group is None and not multi_ok and lanes >= 2 and self.n_init >= 2:
            best = self._fit_lanes(Xc, n, dim, k, seed_stream, tol_abs, ctx, min(lanes, self.n_init), half)
            self.inertia_, C, self.labels_, self.n_iter_ = best[:4]
            self.best_run_ = best[4]
            self.cluster_centers_ = C + mean_d
            return self
        self.run_stats_ = []  # (inertia, n_iter) of every run, in run order
        for run in range(self.n_init):
            if pending:
                res = pending.pop(0)
                self.run_stats_.append((res[0], res[3]))
                if best is None or res[0] < best[0]:
                    best = res + (run,)
                continue
            if multi_ok and run + 1 < self.n_init:
                g = min(grp, self.n_init - run, 4)
                res = self._fit_multi(Xc, [next(seed_stream) for _ in range(g)], grows, tol_abs, ctx, sh)
                pending = res[1:]
                self.run_stats_.append((res[0][0], res[0][3]))
                if best is None or res[0][0] < best[0]:
                    best = res[0] + (run,)
                continue
            seeds = next(seed_stream)
            C = self._gather_rows(Xc, seeds, grows, group)
            labels.fill_(-1)
            sums.zero_()  # the one-GPU iteration keeps sums / counts of the current labels incrementally
            counts.zero_()
            strict, it = False, 0
            if group is None:  # batches of Lloyd steps, the stop checks on the device, one copy per batch
                while it < self.max_iter:
                    _lib.check(lib.ottohip_kmeans_lloyd_steps(ctx.h, _lib.ptr(Xc), n, dim, _lib.ptr(C), k,
                                                              _lib.ptr(labels), _lib.ptr(sums), _lib.ptr(counts),
                                                              min(LLOYD_BATCH, self.max_iter - it), tol_abs, st6, sh))
                    it += int(st6[4])
                    n_changed, reason = int(st6[1]), int(st6[5])
                    shift.value = st6[2]
                    if reason == 3:  # empty clusters: relocate on a copy (sums / counts follow the labels), M-step
                        rs_, rc_ = sums.clone(), counts.clone()
                        empty = np.flatnonzero(rc_.cpu().numpy() == 0)
                        self._relocate(Xc, C, labels, rs_, rc_, empty, grows, group, ctx, sh)
                        _lib.check(lib.ottohip_kmeans_update(ctx.h, _lib.ptr(C), _lib.ptr(rs_), _lib.ptr(rc_), k,
                                                             dim, ctypes.byref(shift), sh))
                        reason = 1 if n_changed == 0 else (2 if shift.value <= tol_abs else 0)
                    if reason == 1:
                        strict = True
                    if reason in (1, 2):
                        break
            else:
                for it in range(1, self.max_iter + 1):
                    _lib.check(lib.ottohip_kmeans_partial(ctx.h, _lib.ptr(Xc), n, dim, _lib.ptr(C), k,
                                                          _lib.ptr(labels), _lib.ptr(sums), _lib.ptr(counts),
                                                          ctypes.byref(inr), ctypes.byref(chg), sh))
                    sums, counts = _allreduce(sums, group), _allreduce(counts, group)
                    n_changed = int(_allreduce(torch.tensor([chg.value], dtype=torch.int64), group).item())
                    cnt = counts.cpu().numpy()
                    empty = np.flatnonzero(cnt == 0)
                    if len(empty):
                        self._relocate(Xc, C, labels, sums, counts, empty, grows, group, ctx, sh)
                    _lib.check(lib.ottohip_kmeans_update(ctx.h, _lib.ptr(C), _lib.ptr(sums), _lib.ptr(counts), k,
                                                         dim, ctypes.byref(shift), sh))
                    if n_changed == 0:
                        strict = True
                        break
                    if shift.value <= tol_abs:
                        break
            if not strict:  # E-step with the final centres (labels match cluster_centers_)
                _lib.check(lib.ottohip_kmeans_partial(ctx.h, _lib.ptr(Xc), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                                      _lib.ptr(sums), _lib.ptr(counts), ctypes.byref(inr),
                                                      ctypes.byref(chg), sh))
            _lib.check(lib.ottohip_kmeans_inertia(ctx.h, _lib.ptr(Xc), n, dim, _lib.ptr(C), _lib.ptr(labels),
                                                  ctypes.byref(inr), sh))
            inertia = float(_allreduce(torch.tensor([inr.value], dtype=torch.float64), group).item())
            self.run_stats_.append((inertia, it))
            if best is None or inertia < best[0]:
                best = (inertia, C.clone(), labels[:n].clone(), it, run)
        self.inertia_, C, self.labels_, self.n_iter_, self.best_run_ = best
        self.cluster_centers_ = C + mean_d
        return self

    def _run_one(self, Xc, n, dim, k, seeds, tol_abs, ctx, sh, labels, sums, counts):
        """One single-GPU run (batched device Lloyd steps, empty-cluster relocation, final E-step and inertia)
        on ctx / stream sh and torch's current stream: (inertia, C, labels, n_iter)."""
        import torch
        lib = _lib.load()
        st6 = (ctypes.c_double * 6)()
        inr, chg, shift = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        C = self._gather_rows(Xc, seeds, None, None)
        labels.fill_(-1)
        sums.zero_()
        counts.zero_()
        strict, it = False, 0
        while it < self.max_iter:
            _lib.check(lib.ottohip_kmeans_lloyd_steps(ctx.h, _lib.ptr(Xc), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                                      _lib.ptr(sums), _lib.ptr(counts),
                                                      min(LLOYD_BATCH, self.max_iter - it), tol_abs, st6, sh))
            it += int(st6[4])
            n_changed, reason = int(st6[1]), int(st6[5])
            shift.value = st6[2]
            if reason == 3:  # empty clusters: relocate on a copy (sums / counts follow the labels), M-step
                rs_, rc_ = sums.clone(), counts.clone()
                empty = np.flatnonzero(rc_.cpu().numpy() == 0)
                self._relocate(Xc, C, labels, rs_, rc_, empty, None, None, ctx, sh)
                _lib.check(lib.ottohip_kmeans_update(ctx.h, _lib.ptr(C), _lib.ptr(rs_), _lib.ptr(rc_), k, dim,
                                                     ctypes.byref(shift), sh))
                reason = 1 if n_changed == 0 else (2 if shift.value <= tol_abs else 0)
            if reason == 1:
                strict = True
            if reason in (1, 2):
                break
        if not strict:  # E-step with the final centres (labels match cluster_centers_)
            _lib.check(lib.ottohip_kmeans_partial(ctx.h, _lib.ptr(Xc), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                                  _lib.ptr(sums), _lib.ptr(counts), ctypes.byref(inr),
                                                  ctypes.byref(chg), sh))
        _lib.check(lib.ottohip_kmeans_inertia(ctx.h, _lib.ptr(Xc), n, dim, _lib.ptr(C), _lib.ptr(labels),
                                              ctypes.byref(inr), sh))
        return float(inr.value), C, labels[:n].clone(), it

    def _fit_lanes(self, Xc, n, dim, k, seed_stream, tol_abs, ctx, lanes, half):
        """One GPU, n_init runs on `lanes` host threads, each with its own library context (workspace, distance
        bounds, f16 rows) and HIP stream: run r on lane r % lanes, so one run's small per-step kernels (filter,
        near ties, centre update) overlap another run's E-step. Every run is computed as alone (bit-identical
        to the sequential loop); the best is the lowest inertia, the earlier run on ties."""
        import threading
        import torch
        lib = _lib.load()
        dev = Xc.device
        seeds = [next(seed_stream) for _ in range(self.n_init)]
        caller = torch.cuda.current_stream(dev)
        ctxs = [ctx] + [_lib.lane_context(ctx.device, i) for i in range(1, lanes)]
        streams = [torch.cuda.Stream(dev) for _ in range(lanes)]
        for st in streams:
            st.wait_stream(caller)  # Xc, its f16 copy on ctx and the seeds' inputs are ready
        attached = []
        results = [None] * self.n_init
        errors = []

        def lane(li):
            try:
                with torch.cuda.stream(streams[li]):
                    lsh = _lib.stream_handle(streams[li])
                    if li > 0 and half:
                        rc = lib.ottohip_kmeans_attach_half(ctxs[li].h, _lib.ptr(Xc), n, dim, lsh)
                        if rc == 0:
                            attached.append(li)
                        elif rc != _lib.OTTOHIP_ELIMIT:
                            _lib.check(rc)
                    sums = torch.empty(k * dim, dtype=torch.int64, device=dev)
                    counts = torch.empty(k, dtype=torch.int64, device=dev)
                    labels = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
                    for run in range(li, self.n_init, lanes):
                        results[run] = self._run_one(Xc, n, dim, k, seeds[run], tol_abs, ctxs[li],
                                                     _lib.stream_handle(streams[li]), labels, sums, counts)
            except BaseException as e:  # noqa: BLE001 -- re-raised on the caller's thread
                errors.append(e)

        threads = [threading.Thread(target=lane, args=(li,), daemon=True) for li in range(lanes)]
        try:
            for t in threads:
                t.start()
        finally:
            for t in threads:
                t.join()
            for li in attached:
                lib.ottohip_kmeans_detach_half(ctxs[li].h)
            for st in streams:
                caller.wait_stream(st)
        if errors:
            raise errors[0]
        best = None
        self.run_stats_ = [(r[0], r[3]) for r in results]
        for run, res in enumerate(results):  # run order: an equal inertia keeps the earlier run
            if best is None or res[0] < best[0]:
                best = res + (run,)
        # the kept run's tensors were allocated on its lane's stream and are used (and later freed) on the
        # caller's: tell the caching allocator, so a reused pool stream cannot take their blocks early
        best[1].record_stream(caller)
        best[2].record_stream(caller)
        return best

    def _fit_multi(self, Xc, seeds, grows, tol_abs, ctx, sh):
        """G <= 4 runs of fit's single-GPU loop in lockstep: the same batches of device Lloyd steps, stop
        checks and empty-cluster relocations per run, every run's E-step sharing one read of X with the
        others'. Returns [(inertia, C, labels, n_iter)] for the runs, in run order."""
        import torch
        lib = _lib.load()
        n, dim = (int(v) for v in Xc.shape)
        k = self.n_clusters
        dev = Xc.device
        G = len(seeds)
        C = [self._gather_rows(Xc, sd, grows, None) for sd in seeds]
        lab = [torch.full((max(n, 1),), -1, dtype=torch.int32, device=dev) for _ in range(G)]
        sums = [torch.zeros(k * dim, dtype=torch.int64, device=dev) for _ in range(G)]
        counts = [torch.zeros(k, dtype=torch.int64, device=dev) for _ in range(G)]
        P = ctypes.c_void_p * G
        pc, pl = P(*[_lib.ptr(x) for x in C]), P(*[_lib.ptr(x) for x in lab])
        ps, pn = P(*[_lib.ptr(x) for x in sums]), P(*[_lib.ptr(x) for x in counts])
        it, done, strict = [0] * G, [False] * G, [False] * G
        st = (ctypes.c_double * (6 * G))()
        shift = ctypes.c_double()
        while not all(done):
            steps = (ctypes.c_int * G)(*[0 if done[g] else min(LLOYD_BATCH, self.max_iter - it[g]) for g in range(G)])
            _lib.check(lib.ottohip_kmeans_lloyd_steps_multi(ctx.h, _lib.ptr(Xc), n, dim, pc, k, pl, ps, pn, steps, G,
                                                            tol_abs, st, sh))
            st12 = st
            for g in range(G):
                if done[g]:
                    continue
                it[g] += int(st12[6 * g + 4])
                n_changed, reason = int(st12[6 * g + 1]), int(st12[6 * g + 5])
                shift.value = st12[6 * g + 2]
                if reason == 3:  # empty clusters: relocate on a copy (sums / counts follow the labels), M-step
                    rs_, rc_ = sums[g].clone(), counts[g].clone()
                    empty = np.flatnonzero(rc_.cpu().numpy() == 0)
                    self._relocate(Xc, C[g], lab[g], rs_, rc_, empty, grows, None, ctx, sh)
                    _lib.check(lib.ottohip_kmeans_update(ctx.h, _lib.ptr(C[g]), _lib.ptr(rs_), _lib.ptr(rc_), k, dim,
                                                         ctypes.byref(shift), sh))
                    reason = 1 if n_changed == 0 else (2 if shift.value <= tol_abs else 0)
                if reason == 1:
                    strict[g] = True
                if reason in (1, 2) or it[g] >= self.max_iter:
                    done[g] = True
        out = []
        inr, chg = ctypes.c_double(), ctypes.c_int64()
        for g in range(G):
            if not strict[g]:  # E-step with the final centres (labels match cluster_centers_)
                _lib.check(lib.ottohip_kmeans_partial(ctx.h, _lib.ptr(Xc), n, dim, _lib.ptr(C[g]), k, _lib.ptr(lab[g]),
                                                      _lib.ptr(sums[g]), _lib.ptr(counts[g]), ctypes.byref(inr),
                                                      ctypes.byref(chg), sh))
            _lib.check(lib.ottohip_kmeans_inertia(ctx.h, _lib.ptr(Xc), n, dim, _lib.ptr(C[g]), _lib.ptr(lab[g]),
                                                  ctypes.byref(inr), sh))
            out.append((float(inr.value), C[g], lab[g][:n], it[g]))
        return out

    @staticmethod
    def _gather_rows(Xc, rows, grows, group):
        """global rows of the (row-sharded) matrix, replicated: each rank fills the ones it owns
        (grows None: the rows are the global rows 0..n-1)."""
        import torch
        rows = np.asarray(rows, np.int64)
        C = torch.zeros((len(rows), Xc.shape[1]), dtype=torch.float32, device=Xc.device)
        if grows is None:
            loc = rows
            mine = np.flatnonzero((rows >= 0) & (rows < Xc.shape[0]))
        else:
            loc = np.searchsorted(grows, rows)
            mine = np.flatnonzero((loc < len(grows)) & (grows[np.minimum(loc, len(grows) - 1)] == rows)) if len(grows) else []
        if len(mine):
            C[torch.from_numpy(mine).to(Xc.device)] = Xc[torch.from_numpy(loc[mine]).to(Xc.device)]
        return _allreduce(C, group).contiguous()

    def _relocate(self, Xc, C, labels, sums, counts, empty, grows, group, ctx, sh):
        """_relocate_empty_clusters_dense: the len(empty) rows farthest from their centroid (all
        ranks: distance desc, global row asc) leave their cluster for the empty ones."""
        import torch
        m = len(empty)
        n = int(Xc.shape[0])
        rows = (ctypes.c_int64 * m)()
        d2 = (ctypes.c_float * m)()
        _lib.check(_lib.load().ottohip_kmeans_farthest(ctx.h, _lib.ptr(Xc), n, Xc.shape[1], _lib.ptr(C),
                                                       _lib.ptr(labels), m, rows, d2, sh))
        gid = (lambda r: int(r)) if grows is None else (lambda r: int(grows[r]))
        cand = [(float(d2[j]), gid(rows[j]), int(labels[rows[j]].item())) for j in range(m) if rows[j] >= 0]
        if group is not None:
            import torch.distributed as dist
            allc = [None] * dist.get_world_size(group)
            dist.all_gather_object(allc, cand, group=group)
            cand = [c for part in allc for c in part]
        cand.sort(key=lambda c: (-c[0], c[1]))
        cand = cand[:m]
        vecs = self._gather_rows(Xc, [c[1] for c in cand], grows, group)
        moves = np.stack([np.array([c[2] for c in cand], np.int32), np.asarray(empty[:len(cand)], np.int32)], 1).ravel()
        mv = (ctypes.c_int32 * len(moves))(*moves.tolist())
        _lib.check(_lib.load().ottohip_kmeans_relocate(ctx.h, _lib.ptr(sums), _lib.ptr(counts), self.n_clusters,
                                                       Xc.shape[1], _lib.ptr(vecs), mv, len(cand), sh))


def count_popularity(offsets, aid, ts, type_, session_cl, n_clusters: int, n_items: int = config.N_ITEMS_OTTO,
                     keep_top_k: int = config.KEEP_TOP_K, ts_max: int | None = None, suffix: str = "cl50",
                     ctx=None, stream=None, group=None):
    """C3 for one clustering (dense cluster index per session). Returns pandas
    DataFrame[aid, {suffix}, rank_*_{suffix} (6 columns)], rows sorted by (cluster, aid).
    group: sessions sharded over ranks; every rank returns the same (global) ranks."""
    import pandas as pd
    import torch
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    off = _t(offsets, dev, torch.int64)
    off = off - off[0]
    a, s_, y = _t(aid, dev, torch.int32), _t(ts, dev, torch.int32), _t(type_, dev, torch.int8)
    cl = _t(session_cl, dev, torch.int32)
    S = int(off.numel()) - 1
    if ts_max is None:
        ts_max = int(s_.max().item()) if s_.numel() else -(1 << 31)
        if group is not None:  # the latest event over every rank's sessions
            import torch.distributed as dist
            from .dist import _comm_device
            t = torch.tensor([ts_max], dtype=torch.int64, device=_comm_device(group))
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            ts_max = int(t.item())
    ts_7d = int(ts_max) - 7 * 24 * 60 * 60                     # count_popularity.py:54-55
    h = ctypes.c_void_p()
    nout = ctypes.c_int64()
    lib = _lib.load()
    sh = _lib.stream_handle(stream)
    if group is None:
        _lib.check(lib.ottohip_popularity_ranks(ctx.h, _lib.ptr(off), S, _lib.ptr(a), _lib.ptr(s_), _lib.ptr(y),
                                                _lib.ptr(cl), int(n_items), int(n_clusters), ts_7d, int(keep_top_k),
                                                ctypes.byref(h), ctypes.byref(nout), sh))
    else:  # sessions sharded: per-rank counters, all-reduced, ranked identically on every rank
        cnt = torch.zeros(6 * int(n_clusters) * int(n_items), dtype=torch.int32, device=dev)
        _lib.check(lib.ottohip_pop_counts(ctx.h, _lib.ptr(off), S, _lib.ptr(a), _lib.ptr(s_), _lib.ptr(y), _lib.ptr(cl),
                                          int(n_items), int(n_clusters), ts_7d, _lib.ptr(cnt), sh))
        cnt = _allreduce(cnt, group)
        _lib.check(lib.ottohip_popularity_from_counts(ctx.h, _lib.ptr(cnt), int(n_items), int(n_clusters),
                                                      int(keep_top_k), ctypes.byref(h), ctypes.byref(nout), sh))
    n = int(nout.value)
    try:
        oa = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        oc = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        orr = torch.empty((max(n, 1), 6), dtype=torch.int16, device=dev)
        _lib.check(lib.ottohip_pop_copy(h, _lib.ptr(oa), _lib.ptr(oc), _lib.ptr(orr), _lib.stream_handle(stream)))
    finally:
        lib.ottohip_pop_free(h)
    r = orr[:n].cpu().numpy()
    out = {"aid": oa[:n].cpu().numpy(), suffix: oc[:n].cpu().numpy()}
    for i, c in enumerate(RANK_COLS):
        out[f"{c}_{suffix}"] = r[:, i]
    return pd.DataFrame(out)


def session_item_similarity(cand_off, aid_next, sess_emb, words, embeddings, sess_has=None,
                            n_items: int = config.N_ITEMS_OTTO, ctx=None, stream=None, rmap=None):
    """R7 for candidates in CSR (cand_off [S+1]): torch (cos_sim_ses_aid, eucl_dist_ses_aid) f32.
    cand_off may be a candidates.Candidates (aid_next None): its device arrays are read in place."""
    import torch
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", ctx.device)
    if hasattr(cand_off, "view") and hasattr(cand_off, "n_cand"):
        v = cand_off.view()
        S, n, p_off, p_nxt = cand_off.n_sessions, cand_off.n_cand, v["off"], v["aid_next"]
    else:
        off = _t(cand_off, dev, torch.int64)
        nxt = _t(aid_next, dev, torch.int32)
        S, n, p_off, p_nxt = int(off.numel()) - 1, int(nxt.numel()), _lib.ptr(off), _lib.ptr(nxt)
    se = _t(sess_emb, dev, torch.float32)
    emb = _t(embeddings, dev, torch.float32)
    has = None if sess_has is None else _t(sess_has, dev, torch.uint8)
    rmap = row_of_aid_map(words, n_items, dev) if rmap is None else rmap
    cos = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    eu = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    _lib.check(_lib.load().ottohip_session_item_similarity(
        ctx.h, p_off, S, p_nxt if n else None, _lib.ptr(se), _lib.ptr(has) if has is not None else None,
        _lib.ptr(rmap), int(rmap.numel()), _lib.ptr(emb), int(emb.shape[1]), _lib.ptr(cos), _lib.ptr(eu),
        _lib.stream_handle(stream)))
    return cos[:n], eu[:n]
