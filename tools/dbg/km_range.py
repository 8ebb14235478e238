# KMeans determinism with a large-magnitude feature: fit twice with OTTOHIP_KM_H16 = 0 and twice with 1
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from otto_recommender_amd import popularity as gp
rng = np.random.default_rng(23)
centers = rng.normal(scale=3, size=(12, 100))
X = (centers[rng.integers(0, 12, 12000)] + rng.normal(size=(12000, 100))).astype(np.float32)
for scale in (1.0, 1e3, 4e4):
    Y = X.copy(); Y[:, 7] *= scale
    os.environ["OTTOHIP_KM_GROUP"] = "1"
    res = []
    for h in ("0", "0", "1", "1"):
        os.environ["OTTOHIP_KM_H16"] = h
        km = gp.KMeans(n_clusters=10, random_state=42, n_init=2).fit(Y)
        res.append((km.labels_.cpu().numpy(), km.inertia_, km.n_iter_))
    print(scale, [(r[1], r[2]) for r in res], [bool(np.array_equal(res[0][0], r[0])) for r in res], flush=True)
