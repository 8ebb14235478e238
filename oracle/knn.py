"""Exact brute-force kNN oracle for the Word2Vec similarity lookup (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
Restates model/w2vec_aids.py:125-173 without the IVF approximation: for each query row the k
rows of smallest squared L2 distance (ties by row index). The reference's own search is
faiss IVFFlat (nlist 100, nprobe 3); faiss is not installed here, so parity
is pinned to this exact search: parity unpinned against faiss itself.
Distances are computed in float64 on the candidates of an fp32 preselection.
"""
from __future__ import annotations

import numpy as np


def topk_exact(emb: np.ndarray, query_rows: np.ndarray, k: int = 20, pre: int = 128, chunk: int = 512):
    import torch
    E = torch.from_numpy(np.ascontiguousarray(emb, np.float32))
    E64 = E.double()
    vn = (E * E).sum(1)
    qr = torch.from_numpy(np.asarray(query_rows, np.int64))
    out_i = np.empty((len(qr), k), np.int64)
    out_d = np.empty((len(qr), k), np.float64)
    pre = min(pre, E.shape[0])
    for a in range(0, len(qr), chunk):
        rows = qr[a:a + chunk]
        Q = E[rows]
        d = (Q * Q).sum(1, keepdim=True) + vn[None, :] - 2.0 * (Q @ E.T)
        cand = torch.topk(d, pre, dim=1, largest=False).indices          # fp32 preselection
        diff = E64[rows][:, None, :] - E64[cand]                        # exact float64
        d2 = (diff * diff).sum(-1)
        d2n, cn = d2.numpy(), cand.numpy()
        for i in range(len(rows)):
            o = np.lexsort((cn[i], d2n[i]))[:k]
            out_i[a + i] = cn[i][o]
            out_d[a + i] = d2n[i][o]
    return out_i, out_d
