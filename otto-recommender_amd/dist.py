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


def emit_for_owners(events, n_parts: int, file_ids=None, n_files_total: int | None = None, names=None,
                    n_items: int = config.N_ITEMS_OTTO, dedup: bool = True, stream=None, ctx=None):
    """Pair words of this rank's files, laid out owner-major (ottohip_covis_emit + emit_write).
    Returns (words int32 [P], words_per_owner, pieces int64 [rows], pieces_per_owner, names)."""
    import torch
    from .covis import reference_rules
    ctx = ctx or _lib.context()
    names, rules = reference_rules(names)
    p = _lib.CovisParams()
    p.min_dt, p.max_dt, p.n_items, p.dedup = config.MIN_TIME_TO_NEXT, config.MAX_TIME_TO_NEXT, int(n_items), int(dedup)
    ev = events.abi()
    nf = ev.n_files
    fids = (ctypes.c_int32 * nf)(*(range(nf) if file_ids is None else [int(f) for f in file_ids]))
    n_tot = nf if n_files_total is None else int(n_files_total)
    em = ctypes.c_void_p()
    wpp = (ctypes.c_int64 * n_parts)()
    rpp = (ctypes.c_int64 * n_parts)()
    lib = _lib.load()
    sh = _lib.stream_handle(stream)
    _lib.check(lib.ottohip_covis_emit(ctx.h, ctypes.byref(ev), rules, len(names), ctypes.byref(p), fids, n_tot, n_parts,
                                      ctypes.byref(em), wpp, rpp, sh))
    try:
        dev = torch.device("cuda", ctx.device)
        words = torch.empty(sum(wpp), dtype=torch.int32, device=dev)
        pieces = torch.empty(sum(rpp), dtype=torch.int64, device=dev)
        _lib.check(lib.ottohip_emit_write(em, _lib.ptr(words) if words.numel() else None,
                                          _lib.ptr(pieces) if pieces.numel() else None, sh))
    finally:
        lib.ottohip_emit_free(em)
    return words, list(wpp), pieces, list(rpp), names


def reduce_received(words, pieces, names, n_files_total: int, n_items: int = config.N_ITEMS_OTTO, dedup: bool = True,
                    stream=None, ctx=None):
    """Assemble the received segments (one word range per row) and reduce them to a table."""
    from .covis import CovisTable, reference_rules
    ctx = ctx or _lib.context()
    names, rules = reference_rules(names)
    p = _lib.CovisParams()
    p.min_dt, p.max_dt, p.n_items, p.dedup = config.MIN_TIME_TO_NEXT, config.MAX_TIME_TO_NEXT, int(n_items), int(dedup)
    h = ctypes.c_void_p()
    nw, npc = int(words.numel()), int(pieces.numel())
    _lib.check(_lib.load().ottohip_covis_reduce_received(ctx.h, rules, len(names), ctypes.byref(p), int(n_files_total),
                                                         _lib.ptr(words) if nw else None, nw,
                                                         _lib.ptr(pieces) if npc else None, npc, ctypes.byref(h),
                                                         _lib.stream_handle(stream)))
    return CovisTable(h, names, ctx)


def set_file_stats(table, file_stats):
    """Install global per-file row statistics [(file_rows, file_rows_ge2)] per rule on a shard."""
    for r, (fr, fr2) in enumerate(file_stats):
        _lib.check(_lib.load().ottohip_table_set_file_stats(table.h, r, int(fr), int(fr2)))


def count_co_events_sharded(events, file_ids, n_files_total: int, group=None, names=None,
                            n_items: int = config.N_ITEMS_OTTO, dedup: bool = True, stream=None, ctx=None):
    """The N-GPU build: this rank's whole files (global ids file_ids) -> pair words laid out by
    owner -> all-to-all-v of words and row pieces (RCCL) -> assemble + reduce of the owner's
    rows. Returns this rank's shard (rows with owner(aid) == rank) of the single-GPU table;
    its file_rows / file_rows_ge2 are the GLOBAL per-file row counts (all-reduced), which is
    what concat_files_w_stats compares against its thresholds (:131, :135)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    words, wpp, pieces, ppp, names = emit_for_owners(events, world, file_ids, n_files_total, names, n_items, dedup,
                                                      stream, ctx)
    rw = exchange(words, wpp, group)
    del words
    rp = exchange(pieces, ppp, group)
    del pieces
    tab = reduce_received(rw, rp, names, n_files_total, n_items, dedup, stream, ctx)
    del rw, rp
    fs = allreduce_file_stats([(tab.stats(r)["file_rows"], tab.stats(r)["file_rows_ge2"]) for r in range(len(names))],
                              group)
    set_file_stats(tab, fs)
    tab.rank, tab.world = rank, world
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
    if stream is not None:
        stream.synchronize()
    recv = exchange_records(recs, counts, group)
    del recs
    tab = table_from_records(recv, names, n_items, fs, ctx=local.ctx, stream=stream)
    tab.rank, tab.world = rank, world
    return tab
