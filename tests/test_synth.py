"""otto-synth generator: determinism, slicing and the distribution targets of SURVEY.md §8(d)."""
import numpy as np

import otto_recommender_amd.synth as synth


def test_deterministic_and_sliceable():
    a = synth.generate(2000)
    b = synth.generate(1000, first_session=1000)
    s = a.slice_sessions(1000, 2000)
    np.testing.assert_array_equal(s.aid, b.aid)
    np.testing.assert_array_equal(s.ts, b.ts)
    np.testing.assert_array_equal(s.type, b.type)
    np.testing.assert_array_equal(s.session, b.session)


def test_distribution_targets():
    ev = synth.generate(50_000)
    L = np.diff(ev.session_offsets)
    assert L.min() >= 2 and L.max() <= 500
    assert 15.0 < L.mean() < 18.0 and np.median(L) == 6
    frac = np.bincount(ev.type, minlength=3) / ev.n_events
    np.testing.assert_allclose(frac, [0.8985, 0.0780, 0.0235], atol=0.004)
    same = np.diff(ev.session) == 0
    assert np.all(np.diff(ev.ts.astype(np.int64))[same] >= 0)
    assert 0 <= ev.aid.min() and ev.aid.max() < 1855603


def test_parquet_roundtrip(tmp_path):
    ev = synth.generate(250, first_session=0)
    paths = synth.write_parquet_files(ev, str(tmp_path), per_file=100)
    assert [p.split("/")[-1] for p in paths] == ["000_100.parquet", "100_200.parquet", "200_300.parquet"]
    back = [synth.read_parquet_events(p) for p in paths]
    assert sum(b.n_events for b in back) == ev.n_events
    np.testing.assert_array_equal(np.concatenate([b.aid for b in back]), ev.aid)
