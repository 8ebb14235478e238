"""Multi-process (gloo, world_size 2, CPU) tests of the multi-GPU host layer (dist.py).

The device kernels (pack / merge, csrc/shard.hip) are covered by tests/test_shard_gpu.py;
here the exchange plumbing runs for real across two processes: each rank deals itself whole
files (deal_files), counts them with the CPU oracle, packs rows by owner_of, exchanges them
with exchange_records and merge-sums what it receives. The union of the shards must equal the
oracle's global cross-file merge (model/count_co_events.py:168), split by owner."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _merge(a, b, c, g):
    import covis as oracle
    ra, rb, rc = oracle._groupby_sum(a, b, c)
    _, _, rg = oracle._groupby_sum(a, b, g)
    return ra, rb, rc, rg


def _worker(rank, world, port, n_sessions, per_file, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    import torch
    import torch.distributed as dist
    import covis as oracle
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import dist as gd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    names = list(oracle.REFERENCE_RULES)
    ev = synth.generate(n_sessions, first_session=999)
    fb = synth.file_session_bounds(ev.n_sessions, per_file=per_file)
    lens = np.diff(ev.session_offsets).astype(np.float64)
    w = [float((lens[fb[f]:fb[f + 1]] ** 2).sum()) for f in range(len(fb) - 1)]
    mine = gd.deal_files(len(fb) - 1, rank, world, weights=w)
    per_file = oracle.count_co_events_files(ev.session_offsets, ev.aid, ev.ts, ev.type,
                                            np.asarray(fb)) if mine else []
    per_file = [per_file[f] for f in mine]
    # local table over my files: (rule, aid, aid_next, count, count_ge2)
    recs, stats = [], []
    for i, n in enumerate(names):
        if per_file:
            a = np.concatenate([p[n][0] for p in per_file]); b = np.concatenate([p[n][1] for p in per_file])
            c = np.concatenate([p[n][2] for p in per_file]).astype(np.int64)
        else:
            a = b = np.zeros(0, np.int32); c = np.zeros(0, np.int64)
        ra, rb, rc, rg = _merge(a, b, c, np.where(c >= 2, c, 0))
        stats.append((len(a), int((c >= 2).sum())))
        recs.append(np.stack([(i << 29) | ra.astype(np.int64), rb, rc, rg], 1))
    recs = np.concatenate(recs) if recs else np.zeros((0, 4), np.int64)
    own = gd.owner_of(recs[:, 0] & ((1 << 29) - 1), world)
    order = np.argsort(own, kind="stable")
    send = torch.from_numpy(recs[order].astype(np.uint32).view(np.int32).copy())
    counts = np.bincount(own, minlength=world).tolist()
    recv = gd.exchange_records(send, counts).numpy().view(np.uint32).astype(np.int64)
    fs = gd.allreduce_file_stats(stats)
    shard = {}
    for i, n in enumerate(names):
        m = (recv[:, 0] >> 29) == i
        r = recv[m]
        shard[n] = [x.tolist() for x in _merge(r[:, 0] & ((1 << 29) - 1), r[:, 1], r[:, 2], r[:, 3])]
    import json
    json.dump({"files": mine, "file_stats": fs, "shard": shard}, open(os.path.join(out_dir, f"r{rank}.json"), "w"))
    dist.destroy_process_group()


def test_deal_files_round_robin_and_balanced():
    from otto_recommender_amd import dist as gd
    assert gd.deal_files(5, 0, 2) == [0, 2, 4] and gd.deal_files(5, 1, 2) == [1, 3]
    w = [10, 1, 1, 1, 9, 2]
    parts = [gd.deal_files(6, r, 3, weights=w) for r in range(3)]
    assert sorted(sum(parts, [])) == list(range(6))
    loads = [sum(w[f] for f in p) for p in parts]
    assert max(loads) <= 10 + 1e-9


def test_owner_of_is_balanced_and_stable():
    from otto_recommender_amd import dist as gd
    aids = np.arange(1_855_603)
    for g in (2, 8):
        cnt = np.bincount(gd.owner_of(aids, g), minlength=g)
        assert cnt.min() > 0.99 * len(aids) / g
    assert gd.owner_of(np.array([12345]), 8).tolist() == gd.owner_of(np.array([12345]), 8).tolist()


def test_gloo_two_rank_exchange_equals_global_merge(tmp_path):
    import json
    import torch.multiprocessing as mp
    import covis as oracle
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import dist as gd
    n_sessions, per_file = 9_000, 2_000
    mp.spawn(_worker, args=(2, _free_port(), n_sessions, per_file, str(tmp_path)), nprocs=2, join=True)
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    assert sorted(res[0]["files"] + res[1]["files"]) == list(range(5))
    ev = synth.generate(n_sessions, first_session=999)
    fb = synth.file_session_bounds(ev.n_sessions, per_file=per_file)
    per_file_all = oracle.count_co_events_files(ev.session_offsets, ev.aid, ev.ts, ev.type, np.asarray(fb))
    for i, n in enumerate(oracle.REFERENCE_RULES):
        a = np.concatenate([p[n][0] for p in per_file_all]); b = np.concatenate([p[n][1] for p in per_file_all])
        c = np.concatenate([p[n][2] for p in per_file_all]).astype(np.int64)
        ra, rb, rc, rg = _merge(a, b, c, np.where(c >= 2, c, 0))
        for r in range(2):
            k = gd.owner_of(ra, 2) == r
            got = res[r]["shard"][n]
            assert got[0] == ra[k].tolist() and got[1] == rb[k].tolist(), n
            assert got[2] == rc[k].tolist() and got[3] == rg[k].tolist(), n
            assert res[r]["file_stats"][i] == [len(a), int((c >= 2).sum())]
