"""Config-5 pipeline (otto-recommender_amd/pipeline.py) end to end on a small synthetic split:
every stage runs on the device and the candidates / recall of the pipeline equal the
candidates built from the same intermediate tables (no stage is skipped or cached)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_pipeline_small(gpu):
    import otto_recommender_amd.synth as synth
    from otto_recommender_amd import pipeline
    ev = synth.generate(60_000)
    train, test, labels = synth.split_test_labels(ev)
    words = synth.item_words()
    emb = synth.embeddings(len(words), seed=1)
    emb2 = synth.embeddings(len(words), seed=3)
    T = {}
    res = pipeline.run(train, test, labels, words, emb, words, emb2, n_clusters=8, kmeans_iter=20,
                       knn_queries=20_000, timings=T)
    assert res["test_sessions"] == test.n_sessions > 0
    assert res["candidates"] > 10 * res["test_sessions"]
    for t in ("clicks", "carts", "orders", "total"):
        for k in ("top20", "top100", "top200", "topall"):
            assert 0.0 <= res["recall"][t][k] <= 1.0
        assert res["recall"][t]["top20"] <= res["recall"][t]["top100"] <= res["recall"][t]["topall"]
    assert res["recall"]["total"]["topall"] > 0.1  # self + co-visit candidates recover revisits
    for stage in ("covis_count", "R1", "knn", "C1_embeddings", "C2_kmeans", "C3_popularity", "candidates", "recall"):
        assert stage in T, stage
