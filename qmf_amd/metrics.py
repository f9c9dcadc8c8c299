"""Per-user test metrics from the device-reduced ranking (qmfx_eval_ranks).

Python twin of the C++ ``qmf::RankedUser`` path (host/qmf/metrics/Metrics.cpp): the
reference's metrics (Metrics.cpp:27-164) evaluated from, per test user, Σ (label − score)²
and the places of the positives in the (score, label > 0)-descending order — no dense score
vector.  Same names and error behaviour as the reference metrics.
"""
from __future__ import annotations

import numpy as np

from ._abi import QmfxError


class RankedUser:
    def __init__(self, nitems, sse, pos_scores, above):
        self.nitems = int(nitems)
        self.sse = float(sse)
        s = np.asarray(pos_scores, np.float64)
        a = np.asarray(above, np.int64)
        order = np.argsort(-s, kind="stable")
        s, a = s[order], a[order]
        # equal-scored positives are equal (score, true) pairs: places above, above + 1, ...
        pos = np.empty(len(s), np.int64)
        for r in range(len(s)):
            pos[r] = pos[r - 1] + 1 if r > 0 and s[r] == s[r - 1] else a[r]
        self.positions = pos


def ranked_users(ctx_result, rowptr, values, nitems):
    """RankedUser per test slot from (label_scores, above, sq_sum) of Context.eval_ranks and
    the label CSR that was uploaded (rowptr over test slots, label values)."""
    ls, above, sq = ctx_result
    out, p = [], 0
    for t in range(len(rowptr) - 1):
        b, e = rowptr[t], rowptr[t + 1]
        lv, sv = np.asarray(values[b:e], np.float64), ls[b:e]
        sse = sq[t] + float(np.sum((lv - sv) * (lv - sv) - sv * sv))
        m = lv > 0
        npos = int(m.sum())
        out.append(RankedUser(nitems, sse, sv[m], above[p:p + npos]))
        p += npos
    return out


def mse(u):
    if u.nitems <= 0:
        raise QmfxError("MSE needs at least 1 element")
    return u.sse / u.nitems


def auc(u):
    pos = len(u.positions)
    neg = u.nitems - pos
    if pos == 0 or neg == 0:
        return 1.0  # the reference logs an error and returns 1
    nxt = np.append(u.positions[1:], u.nitems)
    negs = nxt - u.positions - 1
    m = np.arange(1, pos + 1, dtype=np.float64)
    return float(np.sum(negs * (m / pos / neg)))


def precision(u, k):
    if u.nitems < k:
        raise QmfxError("P@k needs at least k ranked elements")
    return int(np.count_nonzero(u.positions < k)) / k


def recall(u, k):
    if u.nitems < k:
        raise QmfxError("R@k needs at least k ranked elements")
    if len(u.positions) == 0:
        raise QmfxError("R@k needs at least 1 positive")
    return int(np.count_nonzero(u.positions < k)) / len(u.positions)


def average_precision(u):
    if len(u.positions) == 0:
        raise QmfxError("AP needs at least 1 positive")
    m = np.arange(1, len(u.positions) + 1, dtype=np.float64)
    return float(np.sum(m / (u.positions + 1))) / len(u.positions)
