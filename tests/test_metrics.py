"""The Python host mirror's clustering metrics (noparama_amd.metrics; reference
src/clustering_performance.cpp:38-82) against sklearn goldens (tests/golden/metrics.json)."""
import json
import math
import os

import numpy as np

from noparama_amd import metrics

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "metrics.json")


def test_python_metrics_match_sklearn_goldens():
    for c in json.load(open(GOLD)):
        m = metrics.similarity(c["truth"], c["result"])
        assert abs(m["purity"] - c["purity"]) <= 1e-12
        assert abs(m["rand_index"] - c["rand_index"]) <= 1e-12
        if math.isnan(m["adjusted_rand_index"]):  # the reference's 0/0; sklearn calls it 1.0
            assert c["ari"] == 1.0
        else:
            assert abs(m["adjusted_rand_index"] - c["ari"]) <= 1e-12


def test_python_metrics_label_values_and_overflow():
    truth = np.repeat([7, -3], 150_000)  # any label values (the contingency uses their ranks)
    m = metrics.similarity(truth, truth * 2 + 1)
    assert m["purity"] == 1.0 and m["rand_index"] == 1.0 and abs(m["adjusted_rand_index"] - 1.0) < 1e-12
