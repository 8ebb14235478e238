"""GPU parity of R1 (ottohip_topk_per_aid) against the numpy restatement of
get_df_count_for_co_event_type (model/retrieve.py:18-63). Integer outputs: bit-exact."""
import json
import os

import numpy as np
import pytest

import retrieve as oracle_retrieve

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
COLS = ["aid", "aid_next", "count", "count_pop", "perc_pop", "rank", "count_rel"]


def _check(aid, nxt, cnt, first_n, n_items=1855603):
    from otto_recommender_amd import retrieve as gr
    got = gr.topk_per_aid(aid, nxt, cnt, first_n, n_items=n_items)
    ref = oracle_retrieve.get_df_count_for_co_event_type(aid, nxt, cnt, first_n)
    for c in COLS:
        np.testing.assert_array_equal(got[c].cpu().numpy(), ref[c], err_msg=c)
        assert got[c].cpu().numpy().dtype == ref[c].dtype, c


def test_r1_known_answer(gpu):
    g = json.load(open(os.path.join(GOLD, "kat_r1.json")))
    t = np.array(g["table"], np.int32)
    from otto_recommender_amd import retrieve as gr
    got = gr.topk_per_aid(t[:, 0], t[:, 1], t[:, 2], g["first_n"], n_items=100)
    rows = np.stack([got[c].cpu().numpy().astype(np.int64) for c in g["expected_columns"]], 1).tolist()
    assert rows == g["expected"]


@pytest.mark.parametrize("n,sorted_file,first_n", [(1, True, 10), (1000, True, 10), (1_000_003, True, 20),
                                                   (300_000, False, 10), (50_000, True, 100000)])
def test_r1_random_tables(gpu, n, sorted_file, first_n):
    rng = np.random.default_rng(n)
    aid = rng.integers(0, max(1, n // 20), n).astype(np.int32)
    nxt = rng.integers(0, 1855603, n).astype(np.int32)
    cnt = (rng.pareto(1.2, n) * 3 + 2).astype(np.int64).clip(2, 2**31 - 1).astype(np.int32)
    if sorted_file:
        o = np.lexsort((nxt, aid, -cnt.astype(np.int64)))
        aid, nxt, cnt = aid[o], nxt[o], cnt[o]
    _check(aid, nxt, cnt, first_n)


def test_r1_on_finalized_covis_table(gpu):
    """The chain the reference runs: count -> concat_files_w_stats -> get_df_count_for_co_event_type."""
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import covis as gc, config
    ev = synth.generate(200_000, first_session=31)
    tab = gc.count_co_events_fused(gc.DeviceEvents.from_host(ev, synth.file_session_bounds(ev.n_sessions)))
    for name in ("click_to_click", "cart_to_buy"):
        a, b, c = (x.cpu().numpy() for x in tab.finalize(name))
        _check(a, b, c, config.RETRIEVAL_FIRST_N_CO_COUNTS[name])
    tab.free()


def test_r1_edges(gpu):
    import otto_recommender_amd._lib as L
    from otto_recommender_amd import retrieve as gr
    z = np.zeros(0, np.int32)
    assert gr.topk_per_aid(z, z, z, 10)["aid"].numel() == 0
    one = np.array([5], np.int32)
    r = gr.topk_per_aid(one, one, one, 0)
    assert r["aid"].numel() == 0
    with pytest.raises(L.OttoHipError):
        gr.topk_per_aid(one, one, np.array([-1], np.int32), 10)
    with pytest.raises(L.OttoHipError):
        gr.topk_per_aid(np.array([200], np.int32), one, one, 10, n_items=100)
    # all counts equal: q == min -> count_pop 0 (documented)
    same = np.full(10, 7, np.int32)
    _check(np.arange(10, dtype=np.int32) % 3, np.arange(10, dtype=np.int32), same, 2)
