"""Multi-GPU co-visitation build: one process per GPU, files dealt to ranks.

The reference is single-process (model/count_co_events.py:80-100 loops over files, then
concat_files_w_stats :103-181 groups over all per-file tables). Here each rank counts its own
WHOLE files on its GPU (so the per-file count>=2 rule of :131-132 stays exact), and one
all-to-all-v exchange routes every (rule, aid, aid_next) row to owner(aid); the owner
merge-sums what it receives. Rank g then holds exactly the single-GPU table restricted to
{aid : owner(aid) == g}. Communication is torch.distributed (RCCL over xGMI for the "nccl"
backend, gloo on CPU for tests); compute is libottohip.so (csrc/shard.hip).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from . import config

REC_WORDS = 4  # table-row record = u32 {rule << 29 | aid, aid_next, count, count_ge2}


def owner_of(aid, n_parts: int) -> np.ndarray:
    """Owner rank of each aid: multiplicative hash range-reduced to [0, n_parts)
    (the same function as ottohip_owner_of / owner_dev in csrc/shard.hip)."""
    a = np.asarray(aid).astype(np.uint32).astype(np.uint64)
    h = (a * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)
    return ((h * np.uint64(n_parts)) >> np.uint64(32)).astype(np.int64)


def deal_files(n_files: int, rank: int, world: int, weights=None) -> list:
    """Whole files per rank. Without weights: round-robin (file f -> rank f mod world).
    With weights (e.g. per-file sum of n_s^2, work ∝ pairs): greedy longest-processing-time
    assignment, deterministic (ties by file index, then by rank)."""
    if weights is None:
        return list(range(rank, n_files, world))
    w = np.asarray(weights, np.float64)
    order = sorted(range(n_files), key=lambda f: (-w[f], f))
    load = [0.0] * world
    mine = []
    for f in order:
        r = min(range(world), key=lambda i: (load[i], i))
        load[r] += w[f]
        if r == rank:
            mine.append(f)
    return sorted(mine)


def _comm_device(group=None):
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def exchange(send, send_counts, group=None, return_counts=False):
    """All-to-all-v along dim 0: send holds send_counts[p] leading-dim entries for rank p, in
    rank order. Returns what every rank sent to this one, concatenated in source-rank order
    (and, with return_counts, the per-source entry counts)."""
    import torch
    import torch.distributed as dist
    dev = _comm_device(group)
    sc = torch.tensor([int(c) for c in send_counts], dtype=torch.int64, device=dev)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(x) for x in rc.tolist()]
    # gloo (CPU tests, single-GPU rehearsals) exchanges host copies; RCCL moves device memory
    src = send if send.device == dev else send.to(dev)
    recv = torch.empty((sum(recv_counts),) + tuple(send.shape[1:]), dtype=send.dtype, device=dev)
    dist.all_to_all_single(recv, src.contiguous(), recv_counts, [int(c) for c in send_counts], group=group)
    recv = recv if recv.device == send.device else recv.to(send.device)
    return (recv, recv_counts) if return_counts else recv


def start_count_exchange(counts_per_peer, group=None):
    """Non-blocking all-to-all of k entry counts per peer (counts_per_peer: [world][k] ints): returns
    a handle for finish_count_exchange, so the small exchange runs while the caller launches more
    device work (the payload sizes are needed only when the payload exchange is posted)."""
    import torch
    import torch.distributed as dist
    dev = _comm_device(group)
    sc = torch.tensor([[int(x) for x in row] for row in counts_per_peer], dtype=torch.int64, device=dev)
    rc = torch.empty_like(sc)
    work = dist.all_to_all_single(rc, sc, group=group, async_op=True)
    return work, rc, sc


def finish_count_exchange(handle):
    """[world][k] counts received from every peer (host ints)."""
    work, rc, _sc = handle
    work.wait()
    return [[int(x) for x in row] for row in rc.cpu().tolist()]


def exchange_async(send, send_counts, group=None, recv_counts=None):
    """exchange() with the payload all-to-all left in flight: without recv_counts the entry counts
    are exchanged first (the receive size); the payload returns a handle. finish_exchange(handle)
    waits and returns the received tensor; meanwhile the current stream keeps computing (RCCL runs
    on its own stream, ordered after torch's current stream)."""
    import torch
    import torch.distributed as dist
    dev = _comm_device(group)
    if recv_counts is None:
        sc = torch.tensor([int(c) for c in send_counts], dtype=torch.int64, device=dev)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=group)
        recv_counts = [int(x) for x in rc.tolist()]
    src = send if send.device == dev else send.to(dev)
    recv = torch.empty((sum(recv_counts),) + tuple(send.shape[1:]), dtype=send.dtype, device=dev)
    work = dist.all_to_all_single(recv, src.contiguous(), recv_counts, [int(c) for c in send_counts], group=group,
                                  async_op=True)
    return work, recv, send.device, src


def finish_exchange(handle):
    work, recv, home, _src = handle  # _src: the send buffer stays referenced until the wait
    work.wait()
    return recv if recv.device == home else recv.to(home)


def exchange_records(send, send_counts, group=None):
    """All-to-all-v of table-row records [n, 4] int32 grouped by destination rank."""
    return exchange(send, send_counts, group)


def allreduce_file_stats(per_rule, group=None) -> list:
    """Sum the per-file row statistics (file_rows, file_rows_ge2: the N of
    count_co_events.py:117,131) over ranks; per_rule = [(file_rows, file_rows_ge2), ...]."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(per_rule, dtype=torch.int64, device=_comm_device(group)).reshape(-1, 2)
    dist.all_reduce(t, group=group)
    return [tuple(int(x) for x in row) for row in t.cpu().tolist()]


def pack_by_owner(table, n_parts: int, stream=None):
    """Device records [n_rows, 4] int32 grouped by owner, plus rows per owner (host list)."""
    import torch
    n = sum(table.stats(r)["n_rows"] for r in range(len(table.names)))
    dev = torch.device("cuda", table.ctx.device)
    recs = torch.empty((max(n, 1), REC_WORDS), dtype=torch.int32, device=dev)
    counts = (ctypes.c_int64 * n_parts)()
    _lib.check(_lib.load().ottohip_table_pack_by_owner(table.ctx.h, table.h, n_parts, _lib.ptr(recs), counts,
                                                       _lib.stream_handle(stream)))
    return recs[:n], [int(c) for c in counts]


def table_from_records(recs, names, n_items: int, file_stats=None, ctx=None, stream=None):
    """Merge-sum received records into a CovisTable (see ottohip_table_from_records).
    file_stats: global [(file_rows, file_rows_ge2)] per rule, needed by CovisTable.finalize."""
    from .covis import CovisTable
    ctx = ctx or _lib.context()
    st = None
    if file_stats is not None:
        st = (_lib.RuleStats * len(names))()
        for i, (fr, fr2) in enumerate(file_stats):
            st[i].file_rows, st[i].file_rows_ge2 = int(fr), int(fr2)
    h = ctypes.c_void_p()
    n = int(recs.shape[0])
    _lib.check(_lib.load().ottohip_table_from_records(ctx.h, _lib.ptr(recs) if n else None, n, len(names),
                                                      int(n_items), st, ctypes.byref(h), _lib.stream_handle(stream)))
    return CovisTable(h, names, ctx)


class OwnerEmit:
    """S1-S3 of this rank's files with owner-major rows (ottohip_covis_emit): words_per_owner and
    pieces_per_owner are known when the constructor returns; write() runs S4 into fresh device
    buffers (ottohip_emit_write) and returns (words int32 [P], pieces int64 [rows])."""

    def __init__(self, events, n_parts: int, file_ids=None, n_files_total: int | None = None, names=None,
                 n_items: int = config.N_ITEMS_OTTO, dedup: bool = True, stream=None, ctx=None, sym: bool = False):
        from .covis import reference_rules
        self.ctx = ctx or _lib.context()
        self.names, rules = reference_rules(names)
        p = _lib.CovisParams()
        p.min_dt, p.max_dt, p.n_items, p.dedup = (config.MIN_TIME_TO_NEXT, config.MAX_TIME_TO_NEXT, int(n_items),
                                                  int(dedup))
        p.sym = 1 if sym else 0  # symmetric rules sent once per unordered pair (the owners must reduce with sym)
        ev = events.abi()
        nf = ev.n_files
        fids = (ctypes.c_int32 * nf)(*(range(nf) if file_ids is None else [int(f) for f in file_ids]))
        n_tot = nf if n_files_total is None else int(n_files_total)
        self.h = ctypes.c_void_p()
        wpp = (ctypes.c_int64 * n_parts)()
        rpp = (ctypes.c_int64 * n_parts)()
        self.sh = _lib.stream_handle(stream)
        _lib.check(_lib.load().ottohip_covis_emit(self.ctx.h, ctypes.byref(ev), rules, len(self.names), ctypes.byref(p),
                                                  fids, n_tot, n_parts, ctypes.byref(self.h), wpp, rpp, self.sh))
        self._events = events  # the event buffers stay referenced until write()
        self.words_per_owner, self.pieces_per_owner = list(wpp), list(rpp)

    def write(self):
        import torch
        lib = _lib.load()
        try:
            dev = torch.device("cuda", self.ctx.device)
            words = torch.empty(sum(self.words_per_owner), dtype=torch.int32, device=dev)
            pieces = torch.empty(sum(self.pieces_per_owner), dtype=torch.int64, device=dev)
            _lib.check(lib.ottohip_emit_write(self.h, _lib.ptr(words) if words.numel() else None,
                                              _lib.ptr(pieces) if pieces.numel() else None, self.sh))
        finally:
            lib.ottohip_emit_free(self.h)
            self.h = None
            self._events = None
        return words, pieces


def emit_for_owners(events, n_parts: int, file_ids=None, n_files_total: int | None = None, names=None,
                    n_items: int = config.N_ITEMS_OTTO, dedup: bool = True, stream=None, ctx=None, sym: bool = False):
    """Pair words of this rank's files, laid out owner-major (ottohip_covis_emit + emit_write).
    Returns (words int32 [P], words_per_owner, pieces int64 [rows], pieces_per_owner, names)."""
    em = OwnerEmit(events, n_parts, file_ids, n_files_total, names, n_items, dedup, stream, ctx, sym)
    words, pieces = em.write()
    return words, em.words_per_owner, pieces, em.pieces_per_owner, em.names


def reduce_received(words, pieces, names, n_files_total: int, n_items: int = config.N_ITEMS_OTTO, dedup: bool = True,
                    stream=None, ctx=None, cuts=None, sym: bool = False):
    """Assemble the received segments (one word range per row) and reduce them to a table.
    cuts: covis.FileCuts in global file ids (per_file: this owner's rows per file, which the caller
    all-reduces). sym: the senders' storage (OwnerEmit sym): symmetric rules once per unordered pair."""
    from .covis import CovisTable, reference_rules
    ctx = ctx or _lib.context()
    names, rules = reference_rules(names)
    p = _lib.CovisParams()
    p.min_dt, p.max_dt, p.n_items, p.dedup = config.MIN_TIME_TO_NEXT, config.MAX_TIME_TO_NEXT, int(n_items), int(dedup)
    p.sym = 1 if sym else 0
    h = ctypes.c_void_p()
    nw, npc = int(words.numel()), int(pieces.numel())
    args = (ctx.h, rules, len(names), ctypes.byref(p), int(n_files_total), _lib.ptr(words) if nw else None, nw,
            _lib.ptr(pieces) if npc else None, npc)
    if cuts is None:
        _lib.check(_lib.load().ottohip_covis_reduce_received(*args, ctypes.byref(h), _lib.stream_handle(stream)))
        return CovisTable(h, names, ctx)
    o, rows, rows2 = cuts.abi(names, int(n_files_total))
    _lib.check(_lib.load().ottohip_covis_reduce_received_opts(*args, ctypes.byref(o), ctypes.byref(h),
                                                              _lib.stream_handle(stream)))
    tab = CovisTable(h, names, ctx)
    if cuts.per_file:
        tab.file_rows_per_file, tab.file_rows_ge2_per_file = rows[:int(n_files_total)], rows2[:int(n_files_total)]
    return tab


def set_file_stats(table, file_stats):
    """Install global per-file row statistics [(file_rows, file_rows_ge2)] per rule on a shard."""
    for r, (fr, fr2) in enumerate(file_stats):
        _lib.check(_lib.load().ottohip_table_set_file_stats(table.h, r, int(fr), int(fr2)))


def _chunk_files(events, n_chunks: int) -> list:
    """File bounds of n_chunks contiguous groups of the rank's files, balanced by events (the
    per-file event counts are read once per DeviceEvents)."""
    nf = len(events.file_bounds) - 1
    if nf <= 0:
        return [0] * (n_chunks + 1)
    key = ("_chunk_bounds", n_chunks)
    memo = events.__dict__.setdefault("_memo", {})
    if key not in memo:
        import torch
        fbt = torch.as_tensor(events.file_bounds, dtype=torch.int64, device=events.offsets.device)
        e = events.offsets[fbt].cpu().numpy().astype(np.int64)  # events before each file bound
        tot = max(int(e[-1]), 1)
        b = [0]
        for c in range(1, n_chunks):
            b.append(max(b[-1], int(np.searchsorted(e, tot * c / n_chunks, side="left"))))
        b.append(nf)
        memo[key] = [min(x, nf) for x in b]
    return memo[key]


def _count_sharded_batches(events, file_ids, n_files_total: int, cap: int, group, names, n_items, dedup, stream, ctx,
                           chunks, cuts=None, sym=None):
    """More global files than a pair word can tell apart: batches of cap global file ids, each
    counted sharded (batch-local file ids), and every rank merge-sums its own shard tables (the
    owner partition is the same in every batch, so no exchange)."""
    import torch
    fids = np.asarray(file_ids if file_ids is not None else range(len(events.file_bounds) - 1), np.int64)
    recs, fs, out_names, pf, pf2, xs = [], None, None, [], [], {}
    for g0 in range(0, int(n_files_total), cap):
        g1 = min(int(n_files_total), g0 + cap)
        sel = np.nonzero((fids >= g0) & (fids < g1))[0]  # the rank's files are in ascending global order
        lo, hi = (int(sel[0]), int(sel[-1]) + 1) if len(sel) else (0, 0)
        sub = events.subset_files(lo, hi)
        t = count_co_events_sharded(sub, (fids[lo:hi] - g0).tolist(), g1 - g0, group, names, n_items, dedup, stream,
                                    ctx, chunks, max_files=cap,
                                    cuts=cuts.shifted(g0, g1) if cuts is not None else None, sym=sym)
        st = [(t.stats(r)["file_rows"], t.stats(r)["file_rows_ge2"]) for r in range(len(t.names))]
        fs = st if fs is None else [(a + c, b + d) for (a, b), (c, d) in zip(fs, st)]
        if cuts is not None and cuts.per_file:
            pf.append(t.file_rows_per_file); pf2.append(t.file_rows_ge2_per_file)
        for k, v in t.exchange_stats.items():
            xs[k] = max(xs.get(k, 0), v) if k.startswith("max") else xs.get(k, 0) + v
        r, _ = pack_by_owner(t, 1, stream)
        recs.append(r.clone())
        out_names = t.names
        t.free()
    tab = table_from_records(torch.cat(recs).contiguous(), out_names, n_items, fs, ctx=ctx, stream=stream)
    if pf:
        tab.file_rows_per_file, tab.file_rows_ge2_per_file = np.concatenate(pf), np.concatenate(pf2)
    tab.exchange_stats = xs
    return tab


def allreduce_per_file(rows, rows2, group=None):
    """Sum the owners' per-file row counts (each owner holds its aids' rows of every file)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(np.stack([rows, rows2]), dtype=torch.int64, device=_comm_device(group))
    dist.all_reduce(t, group=group)
    t = t.cpu().numpy()
    return t[0].copy(), t[1].copy()


def count_co_events_sharded(events, file_ids, n_files_total: int, group=None, names=None,
                            n_items: int = config.N_ITEMS_OTTO, dedup: bool = True, stream=None, ctx=None,
                            chunks: int | None = None, max_files: int | None = None, cuts=None,
                            per_file_rule: str | None = None, sym: bool | None = None):
    """The N-GPU build: this rank's whole files (global ids file_ids) -> pair words laid out by
    owner -> all-to-all-v of words and row pieces (RCCL) -> assemble + reduce of the owner's
    rows. Returns this rank's shard (rows with owner(aid) == rank) of the single-GPU table;
    its file_rows / file_rows_ge2 are the GLOBAL per-file row counts (all-reduced), which is
    what concat_files_w_stats compares against its thresholds (:131, :135). cuts: covis.FileCuts
    in global file ids, applied by the owners; per_file statistics are all-reduced (global).
    per_file_rule: every global file's rows of that rule from this count (covis.count_co_events_fused's
    option), so that concat_files_w_stats_sharded plans branch (2) without a count of its own.
    sym: None = symmetric rules stored once per unordered pair unless key cuts are given; False = every ordered
    pair at owner(aid) (the storage every part of one branch-(2) plan must share, so that a key lives on one
    rank in all parts). The mode is decided once here and holds for every file batch of the call."""
    import torch.distributed as dist
    import torch
    from .covis import reference_rules, FileCuts
    from .covis import max_files_per_call
    if per_file_rule is not None and cuts is None and per_file_rule in (names or config.CO_EVENTS_TO_COUNT):
        tab = count_co_events_sharded(events, file_ids, n_files_total, group, names, n_items, dedup, stream, ctx,
                                      chunks, max_files, FileCuts(per_file_rule, per_file=True), sym=sym)
        tab.per_file_rule = per_file_rule
        return tab
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    # symmetric rules (click_to_click, cart_to_cart, buy_to_buy; model/count_co_events.py:64-71) go to the owners
    # once per unordered pair: the row (a, b), a <= b, at owner(a), which also stands for its mirror (b, a) (the
    # shard's readers produce it). Key cuts (branch (2)'s parts) need both orders stored; OTTOHIP_DIST_SYM=0 = off
    key_cut = cuts is not None and (cuts.lo is not None or cuts.hi is not None)
    if sym and key_cut:
        raise ValueError("symmetric storage cannot take key cuts (both orders of a pair are needed)")
    if sym is None:
        sym = not key_cut and os.environ.get("OTTOHIP_DIST_SYM", "1") != "0"
    cap = max_files or max_files_per_call(names, n_items)
    if cuts is not None and cuts.per_file:
        cap = min(cap, 1024)  # the per-file histogram's file range (ottohip_file_opts)
    if int(n_files_total) > cap:
        tab = _count_sharded_batches(events, file_ids, n_files_total, cap, group, names, n_items, dedup, stream,
                                     ctx or _lib.context(), chunks, cuts, sym)
        tab.rank, tab.world = rank, world
        return tab
    # the rank's files in n_chunks contiguous groups (balanced by events): chunk c's all-to-all
    # runs on RCCL's stream while chunk c + 1 is counted and emitted. Every rank joins n_chunks
    # exchanges (empty chunks included); the receiver concatenates the chunks' words and pieces in
    # arrival order, which keeps each piece's words where reduce_received expects them.
    n_chunks = chunks if chunks is not None else int(os.environ.get("OTTOHIP_DIST_CHUNKS", "2"))
    nf = len(events.file_bounds) - 1
    bounds = _chunk_files(events, max(1, n_chunks))
    names = reference_rules(names)[0]
    dev = torch.device("cuda", (ctx or _lib.context()).device)
    fids = list(range(nf)) if file_ids is None else [int(f) for f in file_ids]
    pending = []
    # exchange sizes (entries; all_to_all_single takes them as int64 split sizes, RCCL as size_t counts)
    xs = {"words_sent": 0, "max_words_to_peer": 0, "words_recv": 0, "max_words_from_peer": 0, "pieces_sent": 0,
          "pieces_recv": 0}
    for c in range(len(bounds) - 1):
        f0, f1 = bounds[c], bounds[c + 1]
        em = None
        if f1 > f0:
            sub = events if (f0, f1) == (0, nf) else events.subset_files(f0, f1)
            em = OwnerEmit(sub, world, fids[f0:f1], n_files_total, names, n_items, dedup, stream, ctx, sym)
            wpp, ppp = em.words_per_owner, em.pieces_per_owner
        else:  # no files in this chunk (e.g. a rank without files of one part): it still joins the exchange
            wpp, ppp = [0] * world, [0] * world
        # the receive sizes travel while S4 writes the words (no host wait on the exchange path
        # beyond the library's own end-of-emit check)
        cnt = start_count_exchange([[w, p] for w, p in zip(wpp, ppp)], group)
        if em is not None:
            words, pieces = em.write()
        else:
            words, pieces = torch.empty(0, dtype=torch.int32, device=dev), torch.empty(0, dtype=torch.int64, device=dev)
        rc = finish_count_exchange(cnt)
        xs["words_sent"] += sum(wpp); xs["pieces_sent"] += sum(ppp)
        xs["max_words_to_peer"] = max([xs["max_words_to_peer"]] + list(wpp))
        xs["words_recv"] += sum(r[0] for r in rc); xs["pieces_recv"] += sum(r[1] for r in rc)
        xs["max_words_from_peer"] = max([xs["max_words_from_peer"]] + [r[0] for r in rc])
        if stream is not None and words.is_cuda:
            # RCCL orders its work after torch's current stream: make that stream wait for the
            # caller's stream (an event wait on the device, not a host synchronize)
            torch.cuda.current_stream().wait_stream(stream)
        pending.append((exchange_async(words, wpp, group, recv_counts=[r[0] for r in rc]),
                        exchange_async(pieces, ppp, group, recv_counts=[r[1] for r in rc])))
        del words, pieces
    got = [(finish_exchange(hw), finish_exchange(hp)) for hw, hp in pending]
    del pending
    rw = got[0][0] if len(got) == 1 else torch.cat([g[0] for g in got])
    rp = got[0][1] if len(got) == 1 else torch.cat([g[1] for g in got])
    del got
    if stream is not None and rw.is_cuda:
        # work.wait() (RCCL) orders only torch's current stream after the transfer (and the cat ran
        # there): the caller's stream, on which the reduce runs, waits for it
        stream.wait_stream(torch.cuda.current_stream())
    tab = reduce_received(rw, rp, names, n_files_total, n_items, dedup, stream, ctx, cuts, sym)
    del rw, rp
    fs = allreduce_file_stats([(tab.stats(r)["file_rows"], tab.stats(r)["file_rows_ge2"]) for r in range(len(names))],
                              group)
    set_file_stats(tab, fs)
    if cuts is not None and cuts.per_file:
        tab.file_rows_per_file, tab.file_rows_ge2_per_file = allreduce_per_file(tab.file_rows_per_file,
                                                                                tab.file_rows_ge2_per_file, group)
    tab.rank, tab.world = rank, world
    tab.exchange_stats = xs
    return tab


def merge_tables_by_owner(events, group=None, names=None, n_items: int = config.N_ITEMS_OTTO, dedup: bool = True,
                          stream=None, ctx=None):
    """Row-level alternative (also the A7 train+test table merge): count this rank's files to
    a table, then exchange table rows by owner and merge-sum them."""
    import torch.distributed as dist
    from .covis import count_co_events_fused
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    local = count_co_events_fused(events, names, n_items=n_items, dedup=dedup, stream=stream, ctx=ctx)
    names = local.names
    fs = allreduce_file_stats([(local.stats(r)["file_rows"], local.stats(r)["file_rows_ge2"])
                               for r in range(len(names))], group)
    recs, counts = pack_by_owner(local, world, stream)
    local.free()
    if stream is not None and recs.is_cuda:
        import torch
        torch.cuda.current_stream().wait_stream(stream)  # RCCL orders after torch's current stream
    recv = exchange_records(recs, counts, group)
    del recs
    if stream is not None and recv.is_cuda:  # the exchange is ordered on torch's current stream only
        import torch
        stream.wait_stream(torch.cuda.current_stream())
    tab = table_from_records(recv, names, n_items, fs, ctx=local.ctx, stream=stream)
    tab.rank, tab.world = rank, world
    return tab


# ---------------------------------------------------------------- sharded A6
_HUGE = 1 << 62


def _allreduce_sum(t, group=None):
    import torch.distributed as dist
    dev = _comm_device(group)
    x = t.to(dev) if t.device != dev else t.clone()
    dist.all_reduce(x, group=group)
    return x.to(t.device) if x.device != t.device else x


def run_hist(x, lo: int, hi: int, shift: int, mask: int, n_bins: int, ctx=None, stream=None):
    """Device u64 histogram of (x >> shift) & mask over x[lo:hi] (runs of equal keys contiguous)."""
    import torch
    ctx = ctx or _lib.context()
    h = torch.empty(int(n_bins), dtype=torch.int64, device=x.device)
    _lib.check(_lib.load().ottohip_run_hist(ctx.h, _lib.ptr(x) if x.numel() else None, int(lo), int(hi), int(shift),
                                            int(mask) & 0xFFFFFFFF, int(n_bins), _lib.ptr(h), _lib.stream_handle(stream)))
    return h


def head_cut(aid, aid_next, count, max_rows: int, n_items: int, group=None, ctx=None, stream=None) -> int:
    """Length of this shard's share of the GLOBAL head(max_rows) of the (count desc, aid asc,
    aid_next asc) order, given the shard's rows already in that order (a finalize output).
    Exact and collective (every rank calls it): the cut count c* is found by a two-level 16-bit
    radix select over all-reduced count histograms, ties at c* by an all-reduced histogram over
    aid (a*), then ties at (c*, a*) by an all-reduced histogram over aid_next (n*): the rows of one
    aid may sit on several ranks (a symmetric rule's shard holds the mirrors (b, a) of its rows
    (a, b) at owner(a)), but every key (aid, aid_next) is on exactly one rank. A shard's kept rows
    are always a prefix of its order."""
    import torch
    import torch.distributed as dist
    m = int(count.numel())
    tot = _allreduce_sum(torch.tensor([m], dtype=torch.int64), group)
    if int(tot.item()) <= max_rows:
        return m
    K = int(max_rows)
    if K <= 0:
        return 0
    # level 1: count >> 16
    h1 = run_hist(count, 0, m, 16, 0xFFFF, 1 << 16, ctx, stream)
    g1 = _allreduce_sum(h1, group).cpu().numpy()
    h1 = h1.cpu().numpy()
    above = np.concatenate([np.cumsum(g1[::-1])[::-1][1:], [0]])  # global rows with a larger high part
    hi = int(np.flatnonzero(above + g1 >= K).max())
    lo1 = int(h1[hi + 1:].sum())
    # level 2: count & 0xFFFF among rows of that high part
    h2 = run_hist(count, lo1, lo1 + int(h1[hi]), 0, 0xFFFF, 1 << 16, ctx, stream)
    g2 = _allreduce_sum(h2, group).cpu().numpy()
    h2 = h2.cpu().numpy()
    above2 = int(above[hi]) + np.concatenate([np.cumsum(g2[::-1])[::-1][1:], [0]])
    lo = int(np.flatnonzero(above2 + g2 >= K).max())
    need = K - int(above2[lo])  # rows of count c* = hi << 16 | lo still to keep, 1 <= need <= g2[lo]
    lo_c = lo1 + int(h2[lo + 1:].sum())
    # ties at c*: aid histogram of the count == c* rows (a contiguous aid-ascending range)
    h3 = run_hist(aid, lo_c, lo_c + int(h2[lo]), 0, 0xFFFFFFFF, n_items, ctx, stream)
    g3 = _allreduce_sum(h3, group)
    cg = torch.cumsum(g3, 0)
    a_star = int(torch.searchsorted(cg, torch.tensor([need], dtype=cg.dtype, device=cg.device)).item())
    before = int(cg[a_star].item()) - int(g3[a_star].item())
    mine = int(h3[:a_star].sum().item())
    own = int(h3[a_star].item())
    need2 = need - before  # (c*, a*) rows still to keep, 1 <= need2 <= g3[a_star]
    # ties at (c*, a*): aid_next histogram of those rows (a contiguous aid_next-ascending range on each rank)
    lo_a = lo_c + mine
    h4 = run_hist(aid_next, lo_a, lo_a + own, 0, 0xFFFFFFFF, n_items, ctx, stream)
    g4 = _allreduce_sum(h4, group)
    cg4 = torch.cumsum(g4, 0)
    n_star = int(torch.searchsorted(cg4, torch.tensor([need2], dtype=cg4.dtype, device=cg4.device)).item())
    return lo_a + int(h4[:n_star + 1].sum().item())


def _records(a, b, c):
    import torch
    c = c.to(torch.int32)
    return torch.stack([a.to(torch.int32), b.to(torch.int32), c, c], 1).contiguous()


def all_gather_sizes(n: int, group=None) -> list:
    """Every rank's n, in rank order."""
    import torch
    import torch.distributed as dist
    dev = _comm_device(group)
    t = torch.tensor([int(n)], dtype=torch.int64, device=dev)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return [int(x.item()) for x in out]


def all_gather_rows(cols, group=None):
    """All-gather of variable-length (aid, aid_next, count) device columns, in rank order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = _comm_device(group)
    n = torch.tensor([int(cols[0].numel())], dtype=torch.int64, device=dev)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    mx = max(max(ns), 1)
    x = torch.zeros((mx, 3), dtype=torch.int32, device=dev)
    if ns[dist.get_rank(group)]:
        x[:ns[dist.get_rank(group)]] = torch.stack(list(cols), 1).to(dev)
    out = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(out, x, group=group)
    rows = torch.cat([o[:k] for o, k in zip(out, ns)]).to(cols[0].device)
    return rows[:, 0].contiguous(), rows[:, 1].contiguous(), rows[:, 2].contiguous()


def finalize_sharded(table, name, max_rows=None, params: dict | None = None, gather: bool = True,
                     n_items: int = config.N_ITEMS_OTTO, group=None, stream=None):
    """A6 step (3) of concat_files_w_stats (model/count_co_events.py:168-175) on an owner-sharded
    table whose file statistics are the GLOBAL ones (count_co_events_sharded installs them): each
    rank thresholds and orders its rows, head_cut finds the exact global head(max_rows) share of
    every rank, and with gather=True the shares are all-gathered and ordered into the global
    final table, identical on every rank and identical to the single-GPU finalize (the
    consumers -- R1 per aid, candidate generation per session -- need it whole on every rank).
    gather=False returns this rank's share only (still in global order)."""
    ctx = table.ctx
    mr = config.MAX_CO_EVENT_PAIRS_TO_SAVE_DISK if max_rows is None else int(max_rows)
    p = dict(params or {})
    p["max_rows_groupby"] = _HUGE
    a, b, c = table.finalize(name, max_rows=_HUGE, params=p, stream=stream)
    k = head_cut(a, b, c, mr, n_items, group, ctx, stream)
    a, b, c = a[:k], b[:k], c[:k]
    if not gather:
        return a, b, c
    return _order_rows(all_gather_rows((a, b, c), group), name, n_items, ctx, stream)


def _order_rows(cols, name, n_items, ctx, stream=None):
    """(count desc, aid, aid_next) order of disjoint rows (one device finalize, no threshold)."""
    t = table_from_records(_records(*cols), [name], n_items, ctx=ctx, stream=stream)
    out = t.finalize(name, max_rows=_HUGE, params={"click_rule": 0, "min_count": 1, "filter_rows": _HUGE,
                                                    "max_rows_groupby": _HUGE}, stream=stream)
    t.free()
    return out


def concat_files_w_stats_sharded(events, file_ids, n_files_total: int, name: str, table=None, group=None,
                                 n_items: int = config.N_ITEMS_OTTO,
                                 max_rows_groupby: int = config.MAX_ROWS_POLARS_GROUPBY,
                                 optim_rows: int = config.OPTIM_ROWS_POLARS_GROUPBY,
                                 max_pairs: int = config.MAX_CO_EVENT_PAIRS_TO_SAVE_DISK,
                                 click_filter_rows: int = config.CLICK_FILTER_ROWS, gather: bool = True,
                                 stream=None, ctx=None):
    """concat_files_w_stats (model/count_co_events.py:103-181) for one rule over files dealt to
    ranks: the N-GPU form of covis.concat_files_w_stats_fused, same results on every rank.
    (1) per-file count >= 2 when the GLOBAL N > click_filter_rows; (2) when still > max_rows_groupby,
    ceil(N / optim_rows) row slices of the concatenated per-file tables (each in (aid, aid_next)
    order, as on one GPU): one sharded pass gives every global file's rows (the owners' per-file
    counts, all-reduced), the holder of a file cut by a part boundary reads the boundary key from
    its own count of that file, and each part is counted sharded (every rank counts its files of
    the part, the owners cut the boundary files to the part's key range), thresholded at
    MIN_COUNT_IN_PART and cut to its GLOBAL head(int(max_rows_groupby / N * optim_rows)); the
    owner-local part outputs are merge-summed locally (ownership is by aid, so no exchange); (3)
    MIN_COUNT_TO_SAVE and the global head(max_pairs) (finalize_sharded)."""
    import math
    import torch
    from .covis import FileCuts, part_plan, count_co_events_fused, table_keys_at
    ctx = ctx or _lib.context()
    file_ids = [int(f) for f in file_ids]
    own = table is None
    tab = table if table is not None else count_co_events_sharded(events, file_ids, n_files_total, group, [name],
                                                                  n_items, stream=stream, ctx=ctx, per_file_rule=name)
    st = tab.stats(name)
    use_ge2 = "click_to" in name and st["file_rows"] > click_filter_rows
    N = st["file_rows_ge2"] if use_ge2 else st["file_rows"]
    base = {"filter_rows": click_filter_rows}
    if N <= max_rows_groupby:
        out = finalize_sharded(tab, name, max_pairs, base, gather, n_items, group, stream)
        if own:
            tab.free()
        return out
    if own:
        tab.free()
    n_parts = math.ceil(N / optim_rows)
    max_rows_part = int(max_rows_groupby / N * optim_rows)
    fid = np.asarray(file_ids, np.int64)
    if np.any(np.diff(fid) <= 0):
        raise ValueError("file_ids must be increasing (the rank's files in events order)")
    if getattr(tab, "per_file_rule", None) == name:  # from the table's own count
        R = tab.file_rows_ge2_per_file if use_ge2 else tab.file_rows_per_file
    else:
        t = count_co_events_sharded(events, file_ids, n_files_total, group, [name], n_items, stream=stream, ctx=ctx,
                                    cuts=FileCuts(name, per_file=True))
        R = t.file_rows_ge2_per_file if use_ge2 else t.file_rows_per_file
        t.free()
    if int(R.sum()) != N:
        raise RuntimeError(f"{name}: per-file rows sum to {int(R.sum())}, the global N is {N}")
    plan = part_plan(R, n_parts)
    # boundary keys: every rank walks the same list; the holder of the file fills its entries
    need = sorted({(fa, lo) for fa, lo, _, _ in plan if lo > 0} |
                  {(fb, hi) for _, _, fb, hi in plan if hi < int(R[fb])})
    kv = np.zeros(max(len(need), 1), np.int64)
    for f in sorted({f for f, _ in need}):
        pos = np.flatnonzero(fid == f)
        if len(pos) == 0:
            continue
        rows = [r for g, r in need if g == f]
        t = count_co_events_fused(events.subset_files(int(pos[0]), int(pos[0]) + 1), [name], n_items=n_items, ctx=ctx,
                                  stream=stream)
        for r, k in zip(rows, table_keys_at(t, name, use_ge2, rows, stream)):
            kv[need.index((f, r))] = int(k)
        t.free()
    kv = _allreduce_sum(torch.from_numpy(kv), group).numpy()
    keys = {fr: int(kv[i]) for i, fr in enumerate(need)}
    part = {"click_rule": 1 if use_ge2 else 0, "filter_rows": -1,
            "min_count": config.MIN_COUNT_IN_PART.get(name, 1)}
    pieces = []
    for fa, lo, fb, hi in plan:
        l0, l1 = int(np.searchsorted(fid, fa)), int(np.searchsorted(fid, fb + 1))
        cuts = FileCuts(name, lo=(fa, keys[(fa, lo)]) if lo > 0 else None,
                        hi=(fb, keys[(fb, hi)]) if hi < int(R[fb]) else None)
        # one storage mode for every part (sym=False): a part whose boundaries both fall on file ends would
        # otherwise store its mirrors at owner(min(a, b)) while the key-cut parts hold (b, a) at owner(b), and the
        # owner-local merge below could not sum them
        t = count_co_events_sharded(events.subset_files(l0, l1), file_ids[l0:l1], n_files_total, group, [name],
                                    n_items, stream=stream, ctx=ctx, cuts=cuts, sym=False)
        pieces.append(finalize_sharded(t, name, max_rows_part, part, False, n_items, group, stream))
        t.free()
    dev = torch.device("cuda", ctx.device)
    cat = [torch.cat([p[i] for p in pieces]) if pieces else torch.zeros(0, dtype=torch.int32, device=dev)
           for i in range(3)]
    merged = table_from_records(_records(*cat), [name], n_items, ctx=ctx, stream=stream)
    out = finalize_sharded(merged, name, max_pairs, {"click_rule": 0, "filter_rows": _HUGE,
                                                     "min_count": config.MIN_COUNT_TO_SAVE.get(name, 1)},
                           gather, n_items, group, stream)
    merged.free()
    return out
