"""Timing of one KMeans E-step + partial M-step (ottohip_kmeans_partial) at config-5 size:
python tools/km_bench.py [n_rows] [k] [iters]   (set OTTOHIP_KM_MFMA=1 for the MFMA variant)"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from otto_recommender_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_900_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 50
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dim = 100
ctx = _lib.context(0)
g = torch.Generator(device="cuda").manual_seed(0)
C0 = torch.randn(k, dim, device="cuda", generator=g) * 2
X = (C0[torch.randint(0, k, (n,), device="cuda", generator=g)] + torch.randn(n, dim, device="cuda", generator=g)).contiguous()
C = X[:k].clone().contiguous()
labels = torch.full((n,), -1, dtype=torch.int32, device="cuda")
sums = torch.empty(k * dim, dtype=torch.int64, device="cuda")
counts = torch.empty(k, dtype=torch.int64, device="cuda")
inr, chg = ctypes.c_double(), ctypes.c_int64()
lib = _lib.load()
sh = _lib.stream_handle()


MODE = os.environ.get("KM_MODE", "partial")  # partial (sklearn loop) | step (ottohip_kmeans_step) | lloyd (fused)
sh2 = ctypes.c_double()


st4 = (ctypes.c_double * 4)()


def step():
    if MODE == "assign":  # E-step without the per-cluster sums
        _lib.check(lib.ottohip_kmeans_assign(ctx.h, _lib.ptr(X), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                             ctypes.byref(inr), sh))
        return
    if MODE == "lloyd":
        _lib.check(lib.ottohip_kmeans_lloyd_iter(ctx.h, _lib.ptr(X), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                                 _lib.ptr(sums), _lib.ptr(counts), st4, sh))
        return
    if MODE == "step":
        _lib.check(lib.ottohip_kmeans_step(ctx.h, _lib.ptr(X), n, dim, _lib.ptr(C), k, _lib.ptr(labels),
                                           ctypes.byref(sh2), ctypes.byref(inr), sh))
        return
    _lib.check(lib.ottohip_kmeans_partial(ctx.h, _lib.ptr(X), n, dim, _lib.ptr(C), k, _lib.ptr(labels), _lib.ptr(sums),
                                          _lib.ptr(counts), ctypes.byref(inr), ctypes.byref(chg), sh))


for _ in range(3):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / iters
print(f"[{MODE} mfma={os.environ.get('OTTOHIP_KM_MFMA', '0')}] n={n} k={k} dim={dim}: {dt * 1e3:.3f} ms per call (incl. 2 D2H syncs); "
      f"X read {n * dim * 4 / dt / 1e9:.0f} GB/s, {2 * n * dim * k / dt / 1e12:.1f} TFLOP/s")
