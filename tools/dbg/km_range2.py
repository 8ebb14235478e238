# Which part of the KMeans E-step makes two identical fits differ on a large-magnitude feature
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from otto_recommender_amd import popularity as gp
rng = np.random.default_rng(23)
centers = rng.normal(scale=3, size=(12, 100))
X = (centers[rng.integers(0, 12, 12000)] + rng.normal(size=(12000, 100))).astype(np.float32)
os.environ["OTTOHIP_KM_GROUP"] = "1"
os.environ["OTTOHIP_KM_H16"] = "0"
for scale in (1e4, 4e4):
    Y = X.copy(); Y[:, 7] *= scale
    for var in ({}, {"OTTOHIP_KM_BOUNDS": "0"}, {"OTTOHIP_KM_SPLIT": "0"}, {"OTTOHIP_KM_BOUNDS": "0", "OTTOHIP_KM_SPLIT": "0"}):
        for k in ("OTTOHIP_KM_BOUNDS", "OTTOHIP_KM_SPLIT"):
            os.environ.pop(k, None)
        os.environ.update(var)
        res = []
        for _ in range(3):
            km = gp.KMeans(n_clusters=10, random_state=42, n_init=2).fit(Y)
            res.append((km.labels_.cpu().numpy(), km.inertia_, km.n_iter_))
        print(scale, var, [r[2] for r in res], [bool(np.array_equal(res[0][0], r[0])) for r in res], flush=True)
