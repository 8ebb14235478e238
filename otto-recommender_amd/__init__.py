"""otto-recommender_amd: MI355X-native co-visitation + embedding-retrieval engine.

Drop-in for the hot path of nicolaivicol/otto-recommender (model/count_co_events.py,
model/retrieve.py, model/w2vec_aids.py): Python host code mirrors the reference's
function names and file contracts; compute runs in hand-written gfx950 HIP kernels
behind the C-ABI in include/ottohip.h (libottohip.so).
"""
__version__ = "0.1.0"
