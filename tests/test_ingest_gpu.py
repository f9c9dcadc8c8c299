"""Device ingest (qmfx_group_signals) on the MI355X: ids, idx and both CSR orientations built
on the GPU from raw (user id, item id, value) records must equal the reference's grouping
(WALSEngine::groupSignals / sortDataset, WALSEngine.cpp:130-163; IdIndex.cpp:21-31)
bit-exactly: against the oracle's restatement on the committed fixtures, and against the
independent numpy restatement (tests/helpers.csr_from_triples: stable, so duplicate (u, i)
pairs keep input order, as the device's stable radix sort does) on signed, scattered ids
with duplicates, and at a few million interactions."""
import numpy as np
import pytest

import pyoracle as po
import qmf_amd
from helpers import csr_from_triples, load_ml100k, load_tiny

pytestmark = pytest.mark.gpu


def device_group(users, items, values, precision=64):
    c = qmf_amd.Context(8, precision)
    uids, iids = c.group_signals(users, items, values)
    csr = [c.download_csr(side) for side in (0, 1)]
    c.close()
    return uids, iids, csr


def check_exact(users, items, values, precision=64):
    uids, iids, csr = device_group(users, items, values, precision)
    ruids, riids, ru, ri = csr_from_triples(users, items, values)
    assert np.array_equal(uids, ruids) and np.array_equal(iids, riids)
    for (rp, col, val), (xrp, xcol, xval) in zip(csr, (ru, ri)):
        assert np.array_equal(rp, xrp)
        assert np.array_equal(col, xcol)
        # download_csr returns the device's values in double (an fp32 context's widened)
        assert val.dtype == np.float64
        assert np.array_equal(val, xval if precision == 64 else xval.astype(np.float32).astype(np.float64))
    return uids, iids, csr


def test_ingest_tiny_fixture_vs_oracle():
    u, i, v = load_tiny()
    uids, iids, csr = check_exact(u, i, v)
    o = po.OracleWALS(u, i, v, 4)
    assert np.array_equal(uids, o.ids(0)) and np.array_equal(iids, o.ids(1))
    for side in (0, 1):
        rp, col, _ = o.csr(side)
        assert np.array_equal(csr[side][0], rp) and np.array_equal(csr[side][1], col)


@pytest.mark.parametrize("precision", [32, 64])
def test_ingest_ml100k_shape_vs_oracle(precision):
    d = load_ml100k()
    uids, iids, csr = check_exact(d["users"], d["items"], d["values"], precision)
    o = po.OracleWALS(d["users"], d["items"], d["values"], 4)
    assert np.array_equal(uids, o.ids(0)) and np.array_equal(iids, o.ids(1))
    for side in (0, 1):
        rp, col, val = o.csr(side)
        assert np.array_equal(csr[side][0], rp) and np.array_equal(csr[side][1], col)
        assert np.array_equal(csr[side][2], val.astype(np.float32))


def test_ingest_signed_ids_duplicates_and_extremes():
    rng = np.random.default_rng(7)
    n = 20000
    pool_u = np.unique(rng.integers(-2**62, 2**62, 900))
    pool_u = np.concatenate([pool_u, [np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1]])
    pool_i = np.concatenate([rng.integers(-10**12, 10**12, 300), [-2**63, 2**63 - 1]])
    users = rng.choice(pool_u, n)
    items = rng.choice(pool_i, n)
    # many duplicates of (u, i) pairs with distinct values: their order must be input order
    dup = rng.integers(0, n, 3000)
    users = np.concatenate([users, users[dup]])
    items = np.concatenate([items, items[dup]])
    values = rng.integers(0, 6, len(users)).astype(np.float64) + \
        np.arange(len(users)) * 2.0 ** -10
    check_exact(users, items, values)


def test_ingest_single_record_and_single_row():
    check_exact(np.array([5]), np.array([-3]), np.array([2.0]))
    check_exact(np.full(70, 9), np.arange(70)[::-1] * 3, np.arange(70, dtype=np.float64))


def test_ingest_millions():
    rng = np.random.default_rng(11)
    n = 3_000_000
    users = rng.integers(0, 200_000, n) * 7919 - 10**9
    items = rng.zipf(1.3, n) % 50_000
    values = rng.integers(1, 6, n).astype(np.float64)
    check_exact(users, items, values, precision=32)


@pytest.mark.parametrize("precision", [32, 64])
def test_download_csr_returns_device_values_in_double(precision):
    # real-valued weights (not fp32-exact): an fp64 context hands back exactly its doubles,
    # an fp32 context its floats widened -- what bench.py's parity check and CPU baseline
    # feed the oracle, so they solve the device's own problem
    rng = np.random.default_rng(23)
    n = 20_000
    users = rng.integers(0, 3000, n)
    items = rng.integers(0, 700, n)
    values = rng.uniform(0.1, 5.0, n)
    check_exact(users, items, values, precision)
    assert not np.array_equal(values, values.astype(np.float32).astype(np.float64))
