"""How many co-visitation pair words a within-session pre-aggregation saves (measure first).

Over synthetic sessions (the bench's generator) and the reference's self-join (oracle/covis_pandas.py, an op-for-op
restatement of model/count_co_events.py:17-38, 64-71), per rule:
  P      qualifying ordered pairs (session, event i, event j) -- one word each today (k_emit);
  W1     distinct (session, event i, aid_next): combining equal partners inside ONE event's window;
  D      distinct (session, aid, aid_next): combining across the session's events of the same aid (revisits) too;
  EV     distinct (session, type, aid, partner event): one word per partner event of a grouped row entry (the union of
         the group's windows), the combination computable from interval unions without an aid-level dedupe;
  EVs    EV for groups of <= 4 events only (their multiplicity fits the 2 spare word bits), larger groups uncombined;
  RUN    distinct (run, partner run): runs = consecutive events of one aid in a session's per-type ts-ordered list;
  words4 words with a 2-bit in-word multiplicity (1-4, larger counts as repeated words) for each of W1 and D.
Symmetric rules (click_to_click, cart_to_cart, buy_to_buy) store only partners with aid_next >= aid
(DESIGN.md §5): their 'stored' lines count that half. Counts are additive over any grouping of pairs, so either
combination is exact for count and for the per-file count_ge2 (one file holds whole sessions).

  python tools/pair_multiplicity.py [--sessions 6000] [--first 200000]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

SYM = {"click_to_click", "cart_to_cart", "buy_to_buy"}


def _words4(mult):
    return int(np.sum((mult + 3) // 4))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=6000)
    ap.add_argument("--first", type=int, default=200_000)
    args = ap.parse_args()
    import covis_pandas as cp
    from covis import REFERENCE_RULES
    import otto_recommender_amd.synth as synth
    df = synth.generate(args.sessions, first_session=args.first).to_pandas().drop_duplicates()
    df = df.sort_values(["session", "type", "ts", "aid"]).reset_index(drop=True)
    newrun = (df["session"].ne(df["session"].shift()) | df["type"].ne(df["type"].shift())
              | df["aid"].ne(df["aid"].shift()))
    df["run"] = np.cumsum(newrun.to_numpy())
    df["gsize"] = df.groupby(["session", "type", "aid"])["aid"].transform("size")
    df["ev"] = np.arange(len(df))
    m = cp.self_merge_big_df(df, 2000)
    out = {"sessions": args.sessions, "first_session": args.first, "events": len(df), "rules": {}}
    tot = {"P": 0, "W1": 0, "D": 0, "W1_words4": 0, "D_words4": 0, "EV": 0, "EVs": 0, "RUN": 0}
    tot_s = dict(tot)
    for name, (this, nxt, w) in REFERENCE_RULES.items():
        d = m[(m["type"] == this) & (m["type_next"].isin(list(nxt))) & (m["time_to_next"].abs() <= w)]
        res = {}
        for tag, dd in (("all", d), ("stored", d[d["aid_next"] >= d["aid"]] if name in SYM else None)):
            if dd is None:
                continue
            P = len(dd)
            g1 = dd.groupby(["session", "ev", "aid_next"]).size().to_numpy()
            gd = dd.groupby(["session", "aid", "aid_next"]).size().to_numpy()
            ev = dd.groupby(["session", "type", "aid", "ev_next"]).size().to_numpy()
            sm = dd[dd["gsize"] <= 4]
            evs = len(sm.groupby(["session", "type", "aid", "ev_next"]).size()) + int((dd["gsize"] > 4).sum())
            rr = dd.groupby(["run", "run_next"]).size().to_numpy()
            hist = np.bincount(np.minimum(gd, 5), minlength=6)[1:]
            res[tag] = {"P": P, "W1": len(g1), "D": len(gd), "W1_over_P": len(g1) / max(P, 1),
                        "D_over_P": len(gd) / max(P, 1), "W1_words4_over_P": _words4(g1) / max(P, 1),
                        "D_words4_over_P": _words4(gd) / max(P, 1), "EV_over_P": len(ev) / max(P, 1),
                        "EVs_over_P": evs / max(P, 1), "RUN_over_P": len(rr) / max(P, 1),
                        "D_mult_hist_1_2_3_4_ge5": (hist / max(len(gd), 1)).round(4).tolist()}
            acc = tot if tag == "all" else None
            for t, a in (("all", tot), ("stored", tot_s)):
                if (tag == t) or (t == "stored" and tag == "all" and name not in SYM):
                    a["P"] += P; a["W1"] += len(g1); a["D"] += len(gd)
                    a["W1_words4"] += _words4(g1); a["D_words4"] += _words4(gd)
                    a["EV"] += len(ev); a["EVs"] += evs; a["RUN"] += len(rr)
            del acc
        out["rules"][name] = res
    for tag, a in (("all", tot), ("stored", tot_s)):
        out[f"total_{tag}"] = {k: v for k, v in a.items()} | {
            "W1_over_P": a["W1"] / a["P"], "D_over_P": a["D"] / a["P"], "EV_over_P": a["EV"] / a["P"],
            "EVs_over_P": a["EVs"] / a["P"], "RUN_over_P": a["RUN"] / a["P"],
            "W1_words4_over_P": a["W1_words4"] / a["P"], "D_words4_over_P": a["D_words4"] / a["P"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
