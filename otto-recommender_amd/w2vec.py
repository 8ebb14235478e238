"""Word2Vec top-K similarity lookup on MI355X behind the reference's signatures.

Mirrors model/w2vec_aids.py:
  load_index_faiss_ivff(embeddings, model_name)                           :98-110
  get_top_k_similar_faiss(words_q, words, map_word_embedding, index, k)   :125-173
  retrieve_w2vec_knns_via_faiss_index(model_name, k, first_n_aids)        :176-206
The index is exact (bf16 MFMA scores + fp32 rerank, see csrc/knn.hip); the reference's
faiss IVFFlat (nlist 100, nprobe 3) is approximate. Word2Vec training (gensim) is out of
scope: embeddings are an input (a vocabulary `words` in index_to_key order + vectors).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from . import config


class KnnIndex:
    """Device index over item embeddings (fp32 [V, dim] kept resident + packed bf16 operand)."""

    def __init__(self, embeddings, ctx=None, stream=None):
        import torch
        _lib.require_gpu()
        self.ctx = ctx or _lib.context()
        dev = torch.device("cuda", self.ctx.device)
        emb = embeddings if isinstance(embeddings, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(embeddings))
        self.emb = emb.to(dev, torch.float32).contiguous()
        self.n_items, self.dim = (int(x) for x in self.emb.shape)
        self.h = ctypes.c_void_p()
        _lib.check(_lib.load().ottohip_knn_index_create(self.ctx.h, _lib.ptr(self.emb), self.n_items, self.dim,
                                                        ctypes.byref(self.h), _lib.stream_handle(stream)))

    def free(self):
        if self.h:
            _lib.load().ottohip_knn_index_free(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def search(self, query_rows=None, n_q=None, k: int = 20, stream=None):
        """k nearest rows per query row in ascending squared L2 (ties by row index):
        returns torch (idx:int32 [n_q, k], d2:float32 [n_q, k]) on the device."""
        import torch
        dev = self.emb.device
        if query_rows is None:
            n = self.n_items if n_q is None else int(n_q)
            qr = None
        else:
            qr = torch.as_tensor(query_rows, dtype=torch.int32).to(dev).contiguous()
            n = int(qr.numel())
        idx = torch.empty((n, k), dtype=torch.int32, device=dev)
        d2 = torch.empty((n, k), dtype=torch.float32, device=dev)
        _lib.check(_lib.load().ottohip_knn_topk(self.ctx.h, self.h, _lib.ptr(qr), n, k, _lib.ptr(idx), _lib.ptr(d2),
                                                _lib.stream_handle(stream)))
        return idx, d2


def load_index_faiss_ivff(embeddings, model_name: str | None = None) -> KnnIndex:
    """w2vec_aids.py:98-110 (the nlist/nprobe of config.W2VEC_MODELS do not apply: exact search)."""
    return KnnIndex(embeddings)


def word_rows(words, words_q) -> np.ndarray:
    """Row of each query word in the vocabulary `words` (-1 = not in it): the index lookup of
    w2vec_aids.py:156-163 as one sorted search (any vocabulary size, no per-word host loop).
    A word listed more than once maps to its LAST row, as the reference's dict(zip(words, ...))
    keeps the last value of a duplicated key."""
    words = np.asarray(words, np.int64)
    wq = np.asarray(words_q, np.int64)
    if len(words) == 0:
        return np.full(len(wq), -1, np.int64)
    order = np.argsort(words, kind="stable")
    sw = words[order]
    pos = np.searchsorted(sw, wq, side="right") - 1  # the last of equal words (stable order)
    hit = pos >= 0
    hit[hit] = sw[pos[hit]] == wq[hit]
    return np.where(hit, order[np.maximum(pos, 0)], -1).astype(np.int64)


def get_top_k_similar_faiss(words_q, words, map_word_embedding=None, index_faiss_ivff=None, k: int = 20,
                            return_itself: bool = True):
    """w2vec_aids.py:125-173. words_q: query aids; words: the vocabulary (row order of the
    index); index_faiss_ivff: a KnnIndex over embeddings in `words` order (map_word_embedding
    is accepted for signature compatibility; rows come from `words`). Words without an
    embedding are dropped as in :156-163. Returns pandas DataFrame
    [aid:int32, aid_next:int32, dist_w2vec:int32, rank_w2vec:int8] (dist_w2vec = trunc of the
    squared L2 distance, :169; rank_w2vec = ordinal position 1..k clipped at 127, :170-171)."""
    import pandas as pd
    import torch
    index = index_faiss_ivff
    if index is None:
        raise ValueError("index_faiss_ivff (a KnnIndex) is required")
    words = np.asarray(words, np.int64)
    wq = np.asarray(words_q, np.int64)
    rows = word_rows(words, wq)
    found = rows >= 0
    rows, wq = rows[found], wq[found]
    if len(rows) == 0:
        return pd.DataFrame({"aid": np.zeros(0, np.int32), "aid_next": np.zeros(0, np.int32),
                             "dist_w2vec": np.zeros(0, np.int32), "rank_w2vec": np.zeros(0, np.int8)})
    res = knn_table(index, torch.from_numpy(words.astype(np.int32)), torch.from_numpy(rows.astype(np.int32)), k)
    return pd.DataFrame({c: t.cpu().numpy() for c, t in res.items()})


def knn_table(index: KnnIndex, words, query_rows, k: int = 20, stream=None) -> dict:
    """Device form of the output of :167-171 for query rows: dict of torch columns
    aid, aid_next (int32), dist_w2vec (int32, truncated squared L2), rank_w2vec (int8)."""
    import torch
    dev = index.emb.device
    words = torch.as_tensor(words).to(dev, torch.int32)
    qr = torch.as_tensor(query_rows).to(dev, torch.int32)
    idx, d2 = index.search(qr, k=k, stream=stream)
    n = qr.numel()
    valid = idx >= 0
    aid = words[qr.long()].view(n, 1).expand(n, k)
    nxt = torch.where(valid, words[idx.clamp(min=0).long()], torch.full_like(idx, -1))
    dist = torch.trunc(d2).to(torch.int32)
    rank = torch.arange(1, k + 1, device=dev, dtype=torch.int32).clamp(max=127).to(torch.int8).view(1, k).expand(n, k)
    m = valid.reshape(-1)
    return {"aid": aid.reshape(-1)[m].contiguous(), "aid_next": nxt.reshape(-1)[m].contiguous(),
            "dist_w2vec": dist.reshape(-1)[m].contiguous(), "rank_w2vec": rank.reshape(-1)[m].contiguous()}


def retrieve_w2vec_knns_via_faiss_index(embeddings, words, k: int | None = None, first_n_aids: int | None = None,
                                        cache_file: str | None = None):
    """w2vec_aids.py:176-206 with the trained model replaced by its outputs (vocabulary `words`
    in index_to_key order and `embeddings`): neighbours of the first `first_n_aids` words,
    cached to parquet like :191-204."""
    import pandas as pd
    k = config.W2VEC_K if k is None else k
    first_n_aids = config.W2VEC_SEARCH_SIMILAR_FOR_FIRST_N_AIDS if first_n_aids is None else first_n_aids
    if cache_file and os.path.exists(cache_file):
        return pd.read_parquet(cache_file)
    index = KnnIndex(embeddings)
    n_q = min(first_n_aids, index.n_items)
    import torch
    res = knn_table(index, torch.as_tensor(np.asarray(words, np.int32)), torch.arange(n_q, dtype=torch.int32), k)
    df = pd.DataFrame({c: t.cpu().numpy() for c, t in res.items()})
    index.free()
    if cache_file:
        os.makedirs(os.path.dirname(cache_file) or ".", exist_ok=True)
        df.to_parquet(cache_file)
    return df
