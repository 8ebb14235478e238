"""KMeans fit at config-5 shape (12.9 M x 100, k = 50) with n_init runs in lockstep groups (OTTOHIP_KM_GROUP):
python tools/km_group_prof.py [n_rows] [n_init] [max_iter] -- prints the fit's wall time."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from otto_recommender_amd import popularity as gp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_900_000
n_init = int(sys.argv[2]) if len(sys.argv) > 2 else 4
it = int(sys.argv[3]) if len(sys.argv) > 3 else 20
g = torch.Generator(device="cuda").manual_seed(0)
C0 = torch.randn(50, 100, device="cuda", generator=g) * 0.3
X = (C0[torch.randint(0, 50, (n,), device="cuda", generator=g)] + torch.randn(n, 100, device="cuda", generator=g)).contiguous()
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    km = gp.KMeans(n_clusters=50, max_iter=it, n_init=n_init).fit(X)
    torch.cuda.synchronize()
    print(f"group {os.environ.get('OTTOHIP_KM_GROUP', gp.KM_GROUP)} rep {rep}: {time.perf_counter() - t0:.3f} s, iter {km.n_iter_}")
