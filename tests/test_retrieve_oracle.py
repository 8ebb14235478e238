"""CPU checks of the retrieval oracle (oracle/retrieve.py) against hand-derived known answers.

The reference has no tests; R1 (model/retrieve.py:18-63) is pinned by the hand-worked table in
tests/golden/kat_r1.json (polars 'nearest' quantile, ordinal ranks with file-order ties)."""
import json
import os

import numpy as np

import retrieve as oracle_retrieve

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_r1_oracle_known_answer():
    g = json.load(open(os.path.join(GOLD, "kat_r1.json")))
    t = np.array(g["table"])
    res = oracle_retrieve.get_df_count_for_co_event_type(t[:, 0], t[:, 1], t[:, 2], g["first_n"])
    rows = np.stack([res[c].astype(np.int64) for c in g["expected_columns"]], 1).tolist()
    assert rows == g["expected"]


def test_r1_oracle_properties():
    rng = np.random.default_rng(5)
    n = 20000
    aid = rng.integers(0, 500, n).astype(np.int32)
    nxt = rng.integers(0, 10**6, n).astype(np.int32)
    cnt = (rng.pareto(1.5, n) * 3 + 2).astype(np.int32)
    order = np.lexsort((nxt, aid, -cnt))  # the finalize order (count desc, aid, aid_next)
    aid, nxt, cnt = aid[order], nxt[order], cnt[order]
    res = oracle_retrieve.get_df_count_for_co_event_type(aid, nxt, cnt, 10)
    # at most 10 per aid, ranks 1..k consecutive, counts non-increasing within aid
    for a in np.unique(res["aid"])[:50]:
        m = res["aid"] == a
        assert res["rank"][m].tolist() == list(range(1, m.sum() + 1))
        assert np.all(np.diff(res["count"][m]) <= 0)
        assert res["count_rel"][m][0] == 100
    assert res["count_pop"].max() <= 10000 and res["count_pop"].min() >= 0
