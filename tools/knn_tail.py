"""kNN grid-tail probe: k_knn_main time per query at query counts filling 4, 4.58 and 5 rounds of
one workgroup per CU (512 queries per workgroup, 256 CUs)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import otto_recommender_amd.synth as synth
from otto_recommender_amd.w2vec import KnnIndex

emb = synth.embeddings(1_855_603)
ix = KnnIndex(emb)
ix.ctx.set_timing(True)
for nq in [int(a) for a in sys.argv[1:]] or [524_288, 600_000, 655_360]:
    ix.search(None, n_q=nq, k=20)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(2):
        ix.search(None, n_q=nq, k=20)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 2 * 1e3
    print(f"n_q={nq} wg={-(-nq // 512)} ms={ms:.1f} us_per_1k_q={ms / nq * 1e6:.2f} phases={[(n, round(m, 2)) for n, m, _ in ix.ctx.timings()]}", flush=True)
