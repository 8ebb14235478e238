"""GPU parity of the event ingest: reference-schema parquet rows
(etl/jsonl_to_parquet.py:23-29, 100k-session files :59-84, read at model/count_co_events.py:81,91)
grouped into the session CSR by ottohip_events_csr. Checked against a numpy restatement of the
grouping: rows of contiguous, distinct sessions keep their order; otherwise a stable sort by session."""
import ctypes

import numpy as np
import pytest

import otto_recommender_amd.synth as synth

pytestmark = pytest.mark.gpu


def _csr_ref(sess, aid, ts, ty):
    """numpy restatement: keep the order if every run of equal ids is a whole session, else stable-sort"""
    sess = np.asarray(sess, np.int32)
    n = len(sess)
    starts = np.flatnonzero(np.r_[True, sess[1:] != sess[:-1]]) if n else np.zeros(0, np.int64)
    reordered = len(np.unique(sess[starts])) != len(starts)
    if reordered:
        o = np.argsort(sess, kind="stable")
        sess, aid, ts, ty = sess[o], np.asarray(aid)[o], np.asarray(ts)[o], np.asarray(ty)[o]
        starts = np.flatnonzero(np.r_[True, sess[1:] != sess[:-1]])
    off = np.r_[starts, n].astype(np.int64)
    return off, sess[starts], np.asarray(aid, np.int32), np.asarray(ts, np.int32), np.asarray(ty, np.int8), reordered


def _csr_dev(ctx, sess, aid, ts, ty, base=0):
    import torch
    from otto_recommender_amd import _lib
    d = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).cuda()
    s, a, t, y = d(sess, np.int32), d(aid, np.int32), d(ts, np.int32), d(ty, np.int8)
    n = len(sess)
    off = torch.full((n + 1,), -7, dtype=torch.int64, device="cuda")
    ids = torch.full((max(n, 1),), -7, dtype=torch.int32, device="cuda")
    ao, to, yo = torch.empty_like(a), torch.empty_like(t), torch.empty_like(y)
    ns, re = ctypes.c_int64(), ctypes.c_int()
    _lib.check(_lib.load().ottohip_events_csr(ctx.h, _lib.ptr(s), _lib.ptr(a), _lib.ptr(t), _lib.ptr(y), n, base,
                                              _lib.ptr(off), _lib.ptr(ids), _lib.ptr(ao), _lib.ptr(to), _lib.ptr(yo),
                                              ctypes.byref(ns), ctypes.byref(re), None))
    torch.cuda.synchronize()
    S = ns.value
    return (off[:S + 1].cpu().numpy() - base, ids[:S].cpu().numpy(), ao.cpu().numpy(), to.cpu().numpy(),
            yo.cpu().numpy(), bool(re.value))


def _check(ctx, sess, aid, ts, ty, expect_reordered=None, base=0):
    got = _csr_dev(ctx, sess, aid, ts, ty, base)
    ref = _csr_ref(sess, aid, ts, ty)
    for g, r, what in zip(got[:5], ref[:5], ("offsets", "ids", "aid", "ts", "type")):
        np.testing.assert_array_equal(g, r, err_msg=what)
    assert got[5] == ref[5]
    if expect_reordered is not None:
        assert got[5] == expect_reordered


def _rows(ev):
    return ev.session, ev.aid, ev.ts, ev.type


def test_csr_reference_files_keep_order(gpu):
    ev = synth.generate(20_000, first_session=1234)
    off, ids, aid, ts, ty, re = _csr_dev(gpu, *_rows(ev))
    assert not re
    np.testing.assert_array_equal(off, ev.session_offsets - ev.session_offsets[0])
    np.testing.assert_array_equal(ids, np.arange(1234, 1234 + 20_000, dtype=np.int32))
    np.testing.assert_array_equal(aid, ev.aid)
    np.testing.assert_array_equal(ts, ev.ts)
    np.testing.assert_array_equal(ty, ev.type)
    _check(gpu, *_rows(ev), expect_reordered=False, base=777)


def test_csr_distinct_runs_in_any_order_keep_order(gpu):
    """contiguous sessions with distinct ids in a shuffled order: nothing to regroup"""
    ev = synth.generate(5_000, first_session=0)
    rng = np.random.default_rng(3)
    order = rng.permutation(ev.n_sessions)
    parts = [ev.slice_sessions(int(i), int(i) + 1) for i in order]
    cols = [np.concatenate([getattr(p, k) for p in parts]) for k in ("session", "aid", "ts", "type")]
    _check(gpu, *cols, expect_reordered=False)
    # the session ids come back in file order, not ascending (documented in ottohip.h)
    _, ids, _, _, _, re = _csr_dev(gpu, *cols)
    assert not re
    np.testing.assert_array_equal(ids, order.astype(np.int32))


@pytest.mark.parametrize("n,seed", [(37, 0), (5_000, 1), (2_000_003, 2)])
def test_csr_split_sessions_stable_sort(gpu, n, seed):
    """rows of a session spread over the table (negative and extreme ids included): stable regroup"""
    rng = np.random.default_rng(seed)
    sess = rng.integers(-50, max(60, n // 7), n).astype(np.int32)
    sess[: min(n, 3)] = [np.iinfo(np.int32).min, np.iinfo(np.int32).max, -1][: min(n, 3)]
    aid = rng.integers(0, 1_855_603, n).astype(np.int32)
    ts = rng.integers(1_659_304_800, 1_662_328_791, n).astype(np.int32)
    ty = rng.integers(0, 3, n).astype(np.int8)
    _check(gpu, sess, aid, ts, ty, expect_reordered=True)


def test_csr_edges(gpu):
    e = np.zeros(0, np.int32)
    off, ids, *_ , re = _csr_dev(gpu, e, e, e, np.zeros(0, np.int8), base=5)
    assert off.tolist() == [0] and len(ids) == 0 and not re
    _check(gpu, [9], [1], [2], [0], expect_reordered=False)
    _check(gpu, [4, 4, 4], [1, 2, 3], [5, 5, 5], [0, 1, 2], expect_reordered=False)
    _check(gpu, [2, 1, 2], [1, 2, 3], [5, 5, 5], [0, 1, 2], expect_reordered=True)
    _check(gpu, [3, 1, 2, 0], [1, 2, 3, 4], [5, 5, 5, 5], [0, 1, 2, 0], expect_reordered=False)
    with pytest.raises(Exception):
        from otto_recommender_amd import _lib
        _lib.check(_lib.load().ottohip_events_csr(gpu.h, None, None, None, None, 4, 0, None, None, None, None, None,
                                                  ctypes.byref(ctypes.c_int64()), None, None))


def test_from_parquet_counts_like_host_csr(gpu, tmp_path):
    """parquet files -> device CSR (file bounds = files) -> counts: the same table as the host-built CSR"""
    from otto_recommender_amd import covis as gc
    ev = synth.generate(7_000, first_session=500)
    paths = synth.write_parquet_files(ev, str(tmp_path), per_file=2_000)
    dev = gc.DeviceEvents.from_parquet(sorted(paths))
    np.testing.assert_array_equal(dev.file_bounds, [0, 2_000, 4_000, 6_000, 7_000])
    host = gc.DeviceEvents.from_host(ev, np.array([0, 2_000, 4_000, 6_000, 7_000], np.int64))
    np.testing.assert_array_equal(dev.offsets.cpu().numpy(), host.offsets.cpu().numpy())
    for k in ("aid", "ts", "type"):
        np.testing.assert_array_equal(getattr(dev, k).cpu().numpy(), getattr(host, k).cpu().numpy())
    a = gc.count_co_events_fused(dev)
    b = gc.count_co_events_fused(host)
    for n in a.names:
        for x, y in zip(a.to_numpy(n), b.to_numpy(n)):
            np.testing.assert_array_equal(x, y, err_msg=n)
        assert a.stats(n) == b.stats(n)


def _files_ref(sess, aid, ts, ty, file_rows):
    """per-file restatement: each file grouped on its own, appended at its row offset"""
    offs, cols, bounds, r0 = [np.zeros(1, np.int64)], [[], [], []], [0], 0
    for rows in file_rows:
        sl = slice(r0, r0 + rows)
        off, _, a, t, y, _ = _csr_ref(sess[sl], aid[sl], ts[sl], ty[sl])
        offs.append(off[1:] + r0)
        for c, x in zip(cols, (a, t, y)):
            c.append(x)
        bounds.append(bounds[-1] + len(off) - 1)
        r0 += rows
    return np.concatenate(offs), [np.concatenate(c) if c else c for c in cols], np.array(bounds, np.int64)


@pytest.mark.parametrize("case", ["reference", "id_continues", "split_in_file", "empty_files"])
def test_csr_files(gpu, case):
    """ottohip_events_csr_files (DeviceEvents.from_columns): one pass over the reference's files, file by
    file when a session id continues into the next file or a file's sessions are split"""
    from otto_recommender_amd import covis as gc
    ev = synth.generate(9_000, first_session=10)
    sess, aid, ts, ty = (np.array(x) for x in _rows(ev))
    cut = [int(ev.session_offsets[i]) for i in (0, 3_000, 6_000, 9_000)]
    file_rows = list(np.diff(cut))
    if case == "id_continues":  # file 1 starts with file 0's last session id
        sess[cut[1]:cut[1] + 5] = sess[cut[1] - 1]
    elif case == "split_in_file":
        rng = np.random.default_rng(4)
        o = cut[2] + rng.permutation(cut[3] - cut[2])
        sess[cut[2]:], aid[cut[2]:], ts[cut[2]:], ty[cut[2]:] = sess[o], aid[o], ts[o], ty[o]
    elif case == "empty_files":
        file_rows = [0, file_rows[0], 0, file_rows[1] + file_rows[2], 0]
    d = gc.DeviceEvents.from_columns(sess, aid, ts, ty, file_rows=file_rows, ctx=gpu)
    off, cols, bounds = _files_ref(sess, aid, ts, ty, file_rows)
    np.testing.assert_array_equal(d.file_bounds, bounds)
    np.testing.assert_array_equal(d.offsets.cpu().numpy(), off)
    for g, r in zip((d.aid, d.ts, d.type), cols):
        np.testing.assert_array_equal(g.cpu().numpy(), r)
    assert d.n_sessions == bounds[-1] and d.n_events == len(sess)
    if case == "reference":
        np.testing.assert_array_equal(off, ev.session_offsets - ev.session_offsets[0])
