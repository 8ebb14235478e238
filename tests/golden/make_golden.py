"""Regenerates the committed golden fixtures (run from the repo root):

    python tests/golden/make_golden.py

kat_appendix_a.json  SURVEY.md Appendix A known-answer test (hand-derived, checked by both
                     restatements: oracle/covis_oracle.c and oracle/covis_pandas.py)
covis_1k.npz         five per-rule tables of the first 1,000 otto-synth sessions (seed 0),
                     produced by the op-for-op pandas restatement of count_co_events.py:17-94
digest_220m.json     (--full) BASELINE configs[1] at full size: per rule the order-independent
                     checksums of the merged table, from per-file oracle tables (linear sums)
digests.json         sha256 of canonical (aid, aid_next, count) streams:
                     config-1 slice (first 10,000 sessions, click_to_click) and a 3-file slice
                     (300,000 sessions, all five rules, per-file tables merged with c / c_ge2)
The reference itself cannot run here (polars absent): parity is unpinned
against it; these fixtures pin the build's restatement.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import covis  # noqa: E402
import covis_pandas  # noqa: E402
import otto_recommender_amd.synth as synth  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

KAT_EVENTS = [(1, 10, 0, 0), (1, 20, 100, 0), (1, 10, 200, 1), (1, 30, 50000, 0), (1, 20, 90000, 2),
              (2, 10, 1000, 0), (2, 10, 1000, 0), (2, 10, 1060, 0), (2, 20, 1100, 1), (2, 20, 1100, 2),
              (3, 40, 0, 0), (3, 50, 43200, 0), (3, 60, 86401, 0)]
KAT_EXPECTED = {
    "click_to_click": [[10, 10, 2], [10, 20, 1], [20, 10, 1], [40, 50, 1], [50, 40, 1]],
    "click_to_cart_or_buy": [[10, 10, 1], [10, 20, 4], [20, 10, 1], [30, 10, 1], [30, 20, 1]],
    "cart_to_cart": [],
    "cart_to_buy": [[20, 20, 1]],
    "buy_to_buy": [],
}


def merged_tables(per_file):
    """sum over files of count and of per-file counts >= 2 (the build's c / c_ge2)."""
    out = {}
    for name in per_file[0]:
        a = np.concatenate([p[name][0] for p in per_file]); b = np.concatenate([p[name][1] for p in per_file])
        c = np.concatenate([p[name][2] for p in per_file]).astype(np.int64)
        ga, gb, gc = covis._groupby_sum(a, b, c)
        _, _, g2 = covis._groupby_sum(a, b, np.where(c >= 2, c, 0))
        out[name] = (ga, gb, gc, g2)
    return out


def main():
    a = np.array(KAT_EVENTS)
    ev = synth.events_from_columns(a[:, 0], a[:, 1], a[:, 2], a[:, 3])
    got = covis.count_co_events_file(ev.session_offsets, ev.aid, ev.ts, ev.type)
    got = {k: [[int(x), int(y), int(c)] for x, y, c in zip(*v)] for k, v in got.items()}
    assert got == KAT_EXPECTED, got
    with open(os.path.join(HERE, "kat_appendix_a.json"), "w") as f:
        json.dump({"events": KAT_EVENTS, "expected": KAT_EXPECTED}, f, indent=1)

    ev = synth.generate(1000)
    tp = covis_pandas.as_arrays(covis_pandas.count_file(ev.to_pandas()))
    arrs = {}
    for k, (x, y, c) in tp.items():
        arrs[f"{k}.aid"], arrs[f"{k}.aid_next"], arrs[f"{k}.count"] = x, y, c
    np.savez_compressed(os.path.join(HERE, "covis_1k.npz"), **arrs)

    dig = {}
    ev = synth.generate(10_000)
    t = covis.count_co_events_file(ev.session_offsets, ev.aid, ev.ts, ev.type,
                                   rules={"click_to_click": covis.REFERENCE_RULES["click_to_click"]})
    dig["config1_10k_click_to_click"] = covis.canonical_digest(t)
    ev = synth.generate(300_000)
    fb = synth.file_session_bounds(ev.n_sessions)
    per_file = covis.count_co_events_files(ev.session_offsets, ev.aid, ev.ts, ev.type, fb)
    m = merged_tables(per_file)
    dig["slice_300k_3files_count"] = covis.canonical_digest({k: v[:3] for k, v in m.items()})
    dig["slice_300k_3files_count_ge2"] = covis.canonical_digest(
        {k: (v[0][v[3] > 0], v[1][v[3] > 0], v[3][v[3] > 0]) for k, v in m.items()})
    dig["slice_300k_3files_file_rows"] = {k: int(sum(len(p[k][0]) for p in per_file)) for k in m}
    dig["slice_300k_3files_file_rows_ge2"] = {k: int(sum(int((p[k][2] >= 2).sum()) for p in per_file)) for k in m}
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(dig, f, indent=1, sort_keys=True)




def full_digest(target_events: int = 220_000_000, seed: int = 0, threads: int = 0) -> dict:
    """BASELINE configs[1] (220M events, 100k-session files, all five rules): per rule the linear
    checksums of every file's table (oracle/covis.py files_digest, OpenMP over files), which equal
    ottohip_table_digest of the build's merged table. Written to digest_220m.json."""
    n_sess, n_ev = synth.sessions_for_events(target_events, 0, seed)
    ev = synth.generate(n_sess, 0, seed)
    fb = synth.file_session_bounds(n_sess)
    d = covis.files_digest(ev.session_offsets, ev.aid, ev.ts, ev.type, fb, threads)
    return {"events": int(ev.n_events), "sessions": int(n_sess), "files": int(len(fb) - 1), "seed": seed,
            "rules": d, "note": "d_* are wrapping u64 sums of splitmix64(rule<<48|aid<<24|aid_next ^ seed) x count "
                                 "(seed 1) / x count_ge2 (seed 2); pairs = sum count; file_rows = per-file rows"}


if __name__ == "__main__":
    if "--full" in sys.argv:  # ~1 min on 8 cores: the 220M-event digest only
        json.dump(full_digest(), open(os.path.join(HERE, "digest_220m.json"), "w"), indent=1)
    else:
        main()
