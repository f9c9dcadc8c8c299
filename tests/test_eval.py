"""Test-set evaluation (Engine::computeTestScores Engine.cpp:73-96 + Metrics.cpp:27-164).

CPU side: the oracle's metric restatement is pinned to the reference's known answers
(MetricsTest.cpp:35-88), and the ranked-statistics metrics (qmf_amd.metrics, the Python twin
of the C++ RankedUser path the engines use on the device output) equal the dense metrics on
the oracle's brute-force statistics, ties and non-positive labels included.
"""
import numpy as np
import pytest

import pyoracle as po
from qmf_amd import metrics as qm


def test_oracle_metrics_known_answers():
    # MetricsTest.cpp:35-88
    assert po.metric_mse([1.0, 0.0], [0.5, 0.5]) == 0.25
    assert po.metric_mse([1.0, 0.0, 1.0], [0.0, 1.0, 2.0]) == 1.0
    auc = [([1, 0], [3, 2], 1.0), ([0, 1], [3, 2], 0.0), ([1, 1, 0], [3, 2, 0], 1.0),
           ([1, 0, 1], [3, 2, 0], 0.5), ([0, 1, 1], [3, 2, 0], 0.0)]
    for l, s, v in auc:
        assert po.metric_auc(np.array(l, float), np.array(s, float)) == v
    p = [(1, [1, 0], [3, 2], 1.0), (1, [1, 1], [3, 2], 1.0), (1, [0, 1], [3, 2], 0.0),
         (2, [1, 0], [3, 2], 0.5), (2, [1, 1], [3, 2], 1.0), (2, [0, 1], [3, 2], 0.5),
         (2, [0, 1, 0], [3, 2, 1], 0.5), (2, [0, 1, 0], [3, 1, 2], 0.0)]
    for k, l, s, v in p:
        assert po.metric_precision(np.array(l, float), np.array(s, float), k) == v
    r = [(1, [1, 0], [3, 2], 1.0), (1, [1, 1], [3, 2], 0.5), (1, [0, 1], [3, 2], 0.0),
         (2, [1, 0], [3, 2], 1.0), (2, [1, 1], [3, 2], 1.0), (2, [0, 1], [3, 2], 1.0),
         (2, [0, 1, 0], [3, 2, 1], 1.0), (2, [0, 1, 0], [3, 1, 2], 0.0)]
    for k, l, s, v in r:
        assert po.metric_recall(np.array(l, float), np.array(s, float), k) == v
    ap = [([1, 0], [3, 2], 1.0), ([1, 1], [3, 2], 1.0), ([0, 1], [3, 2], 0.5),
          ([0, 1, 0], [3, 2, 1], 0.5), ([0, 1, 0], [3, 1, 2], 1.0 / 3)]
    for l, s, v in ap:
        assert po.metric_ap(np.array(l, float), np.array(s, float)) == pytest.approx(v, rel=1e-15)


def _check_user(labels, scores):
    sq, ps, above = po.rank_stats(labels, scores)
    lab = np.nonzero(labels != 0)[0]
    lv, sv = labels[lab], scores[lab]
    u = qm.RankedUser(len(labels), sq + float(np.sum((lv - sv) ** 2 - sv * sv)), ps, above)
    tol = dict(rel=1e-12, abs=1e-15)
    assert qm.mse(u) == pytest.approx(po.metric_mse(labels, scores), **tol)
    npos = int(np.count_nonzero(labels > 0))
    if 0 < npos < len(labels):
        assert qm.auc(u) == pytest.approx(po.metric_auc(labels, scores), **tol)
    if npos:
        assert qm.average_precision(u) == pytest.approx(po.metric_ap(labels, scores), **tol)
    for k in (1, 2, 5, 10):
        if len(labels) >= k:
            assert qm.precision(u, k) == po.metric_precision(labels, scores, k)
            if npos:
                assert qm.recall(u, k) == po.metric_recall(labels, scores, k)


def test_ranked_metrics_equal_dense_with_ties():
    rng = np.random.default_rng(5)
    for trial in range(300):
        n = int(rng.integers(1, 80))
        labels = rng.choice([-1.0, 0.0, 0.0, 0.0, 1.0, 3.0], n)
        scores = (rng.integers(0, 4, n).astype(float) if trial % 2
                  else rng.normal(size=n))
        _check_user(labels, scores)


def test_ranked_metric_errors():
    u = qm.RankedUser(3, 0.0, [], [])
    assert qm.auc(u) == 1.0
    with pytest.raises(qm.QmfxError):
        qm.average_precision(u)
    with pytest.raises(qm.QmfxError):
        qm.precision(u, 4)
