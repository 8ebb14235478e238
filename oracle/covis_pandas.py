"""Op-for-op pandas restatement of model/count_co_events.py:17-94 (TEST INFRASTRUCTURE ONLY).

Used to cross-check the C oracle and to produce the committed goldens. It follows the
reference's dataframe pipeline step by step (polars -> pandas, same column names):
  df.unique()                                   :92
  join(on='session', suffix='_next')            :19
  filter ~(aid==aid_next & ts==ts_next & type==type_next)   :23-27
  time_to_next = ts_next - ts                   :30
  filter MIN_TIME_TO_NEXT <= dt <= MAX_TIME_TO_NEXT          :33-36
  per rule: filter(type==this & type_next.isin(next) & |dt|<=W).groupby([aid, aid_next]).count  :64-71
Small inputs only (the join materialises Σ n_s² rows, exactly like the reference).
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from covis import MAX_TIME_TO_NEXT, MIN_TIME_TO_NEXT, REFERENCE_RULES


def self_merge(df_part: pd.DataFrame) -> pd.DataFrame:
    m = df_part.merge(df_part, on="session", suffixes=("", "_next"))
    m = m[~((m["aid"] == m["aid_next"]) & (m["ts"] == m["ts_next"]) & (m["type"] == m["type_next"]))]
    m = m.assign(time_to_next=m["ts_next"].astype(np.int32) - m["ts"].astype(np.int32))
    m = m[(m["time_to_next"] >= MIN_TIME_TO_NEXT) & (m["time_to_next"] <= MAX_TIME_TO_NEXT)]
    return m


def self_merge_big_df(df: pd.DataFrame, n_sessions_in_part: int = 10_000) -> pd.DataFrame:
    sessions = df["session"].unique()
    parts = []
    for i in range(0, len(sessions), n_sessions_in_part):
        part = df[df["session"].isin(sessions[i:i + n_sessions_in_part])]
        parts.append(self_merge(part))
    return pd.concat(parts) if parts else self_merge(df)


def count_co_events(df_merged: pd.DataFrame, rules=REFERENCE_RULES) -> dict:
    out = {}
    for name, (this, nxt, w) in rules.items():
        d = df_merged[(df_merged["type"] == this) & (df_merged["type_next"].isin(list(nxt)))
                      & (df_merged["time_to_next"].abs() <= w)]
        g = d.groupby(["aid", "aid_next"]).size().reset_index(name="count")
        out[name] = g
    return out


def count_file(df: pd.DataFrame, rules=REFERENCE_RULES) -> dict:
    df = df.drop_duplicates()
    return count_co_events(self_merge_big_df(df), rules)


def as_arrays(tables: dict) -> dict:
    res = {}
    for name, g in tables.items():
        g = g.sort_values(["aid", "aid_next"])
        res[name] = (g["aid"].to_numpy(np.int32), g["aid_next"].to_numpy(np.int32),
                     g["count"].to_numpy(np.uint32))
    return res
