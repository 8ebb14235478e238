"""Host-side logic of the device paths (no GPU): part planning of A6 branch (2) by rows."""
import numpy as np


def test_part_plan_rows():
    """part_plan: row slices of concat_files_w_stats' branch (2) over per-file row counts
    (empty files, a part inside one file, a part ending exactly at a file end)."""
    from otto_recommender_amd.covis import part_plan
    R = [5, 0, 7, 3, 0, 10]
    for n_parts in range(1, 26):
        plan = part_plan(R, n_parts)
        C = np.concatenate([[0], np.cumsum(R)])
        got = []
        for fa, lo, fb, hi in plan:
            assert 0 <= lo < R[fa] and 0 < hi <= R[fb] and fa <= fb
            got.append((int(C[fa] + lo), int(C[fb] + hi)))
        rp = -(-sum(R) // n_parts)
        want = [(i * rp, min((i + 1) * rp, sum(R))) for i in range(n_parts) if i * rp < sum(R)]
        assert got == want, n_parts


def test_word_rows_lookup():
    """w2vec.word_rows (get_top_k_similar_faiss' vocabulary lookup, w2vec_aids.py:156-163): rows of
    the query words in vocabulary order, -1 for unknown words; large vocabularies (> 5 M) and an
    empty one work without a per-word host loop."""
    from otto_recommender_amd.w2vec import word_rows
    rng = np.random.default_rng(5)
    words = rng.permutation(np.arange(0, 60_000_000, 7, dtype=np.int64))[:6_000_000]
    q = np.concatenate([words[[0, 17, 5_999_999]], [1, 3, -5], words[rng.integers(0, len(words), 1000)]])
    got = word_rows(words, q)
    want = {int(w): i for i, w in enumerate(words[:10])}
    assert got[0] == 0 and got[1] == 17 and got[2] == 5_999_999
    assert (got[3:6] == -1).all()
    np.testing.assert_array_equal(words[got[6:]], q[6:])
    assert want[int(words[3])] == 3
    assert (word_rows(np.zeros(0, np.int64), q[:4]) == -1).all()


def test_duplicate_keys_take_the_last_row():
    """Duplicated vocabulary words / session rows resolve to their LAST row, as the reference's
    dict lookups do (w2vec.word_rows, candidates.session_cluster_index)."""
    import pandas as pd
    from otto_recommender_amd.w2vec import word_rows
    from otto_recommender_amd.candidates import session_cluster_index
    words = np.array([40, 10, 40, 30, 10, 10], np.int64)
    np.testing.assert_array_equal(word_rows(words, [10, 40, 30, 20]), [5, 2, 3, -1])
    df = pd.DataFrame({"session": [7, 3, 7, 9, 5], "cl50": [1.0, 4.0, 2.0, np.nan, 1.0]})
    clusters = np.array([1.0, 2.0, 4.0])
    np.testing.assert_array_equal(session_cluster_index(df, clusters, np.array([7, 3, 9, 5, 8])), [1, 2, -1, 0, -1])
    empty = df.iloc[:0]
    np.testing.assert_array_equal(session_cluster_index(empty, clusters, np.array([7])), [-1])
