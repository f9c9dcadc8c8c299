"""The multi-GPU partition on one GPU: `world` contexts, each set up as one rank by
qmfx_dist_init without a communicator (its nnz-balanced row range of both sides, the
solve pieces of the all-gather schedule, and only its own signals kept on the device).
Each half, every context solves only its rows; the test assembles the ranks' ranges (the
all-gather the RCCL path does) and checks the result and the summed loss against the
oracle's single-process half (WALSEngine::iterate, WALSEngine.cpp:165-218)."""
import numpy as np
import pytest

import pyoracle as po
import qmf_amd
from helpers import csr_from_triples, rel_err, synth

pytestmark = pytest.mark.gpu
LAM, ALPHA = 0.05, 40.0


@pytest.mark.parametrize("k,precision,world,ingest", [
    (16, 64, 2, "upload"), (16, 64, 3, "upload"), (128, 32, 2, "upload"), (128, 64, 2, "upload"),
    (256, 32, 3, "upload"),
    # ranks ≥ 1 copy rank 0's CSR device to device (qmfx_import_signals: the drop-in engine's
    # --ngpus ingest) before sharding
    (16, 64, 3, "import"), (128, 64, 2, "import")])
def test_partitioned_ranks_assemble_the_full_half(k, precision, world, ingest):
    u, i, v = synth(3000, 600, 60000, seed=k + world)
    v = v.copy()
    v[::97] = -3.0  # a few indefinite rows: the pivoted re-solve runs on sharded signals
    o = po.OracleWALS(u, i, v, k, LAM, ALPHA)
    uids, iids, ucsr, icsr = csr_from_triples(u, i, v)
    init = np.random.default_rng(2).uniform(-0.01, 0.01, (len(iids), k))
    o.set_factors(1, init)
    ranks = []
    for r in range(world):
        c = qmf_amd.Context(k, precision)
        if ingest == "import" and r > 0:
            c.import_signals(ranks[0])
        else:
            c.set_shape(len(uids), len(iids))
            c.upload_csr(0, *ucsr)
            c.upload_csr(1, *icsr)
        c.set_factors(1, init)
        ranks.append(c)
    for r, c in enumerate(ranks):  # rank 0 shards last: the others imported its full CSR
        if r > 0:
            c.dist_init(r, world, None)
    ranks[0].dist_init(0, world, None)
    with pytest.raises(qmf_amd.QmfxError, match="sharded"):
        ranks[0].download_csr(0)
    # fp64: 1e-7, not 1e-9 — the indefinite rows' pivoted solves amplify rounding by cond(A)
    tol = 1e-7 if precision == 64 else 1e-4
    for side, csr in ((0, ucsr), (1, icsr)):
        lo = o.iterate(side)
        ld = sum(c.wals_half(side, ALPHA, LAM) for c in ranks) / (o.nusers * o.nitems)
        plan = qmf_amd.dist_plan(csr[0], world, 4)
        full = np.zeros_like(o.factors(side))
        for r, c in enumerate(ranks):
            b, e = plan[r, 0], plan[r, -1]
            full[b:e] = c.factors(side)[b:e]
        assert rel_err(full, o.factors(side)) < tol, side
        assert abs(ld - lo) < tol * abs(lo), side
        for c in ranks:  # the all-gather
            c.set_factors(side, full)
    for c in ranks:
        c.close()


@pytest.mark.parametrize("k,precision,pieces", [(16, 64, "1"), (128, 32, "1"), (128, 32, "4")])
def test_rccl_loopback_matches_plain(k, precision, pieces, monkeypatch):
    """One rank with a real RCCL communicator (qmfx_dist_init(0, 1, id)): every half runs
    the grouped per-piece ncclBroadcasts on the collective stream and the loss
    ncclAllReduce, and must give bit-for-bit the factors and loss of a context without a
    communicator — the RCCL path's init, stream and event ordering on real hardware."""
    monkeypatch.setenv("QMFX_PIECES", pieces)  # 4: the broadcasts overlap the next piece
    u, i, v = synth(3000, 600, 60000, seed=5)
    uids, iids, ucsr, icsr = csr_from_triples(u, i, v)
    init = np.random.default_rng(4).uniform(-0.01, 0.01, (len(iids), k))
    ctxs = []
    for uid in (None, qmf_amd.rccl_unique_id()):
        c = qmf_amd.Context(k, precision)
        c.set_shape(len(uids), len(iids))
        c.upload_csr(0, *ucsr)
        c.upload_csr(1, *icsr)
        c.set_factors(1, init)
        if uid is not None:
            c.dist_init(0, 1, uid)
        ctxs.append(c)
    ctxs[1].reset_stats()
    for _ in range(2):
        for side in (0, 1):
            l0, l1 = (c.wals_half(side, ALPHA, LAM) for c in ctxs)
            assert l0 == l1, side
            assert np.array_equal(ctxs[0].factors(side), ctxs[1].factors(side)), side
    # the exchange is timed on the collective stream (bench.py --gpus N reports it per half)
    for side in (0, 1):
        x = ctxs[1].exchange_stats(side)
        assert x["halves"] == 2 and x["solve_ms"] > 0, x
        assert 0 <= x["exposed_ms"] and 0 <= x["exchange_ms"] < 1e4, x
        assert ctxs[0].exchange_stats(side)["halves"] == 0
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("k,precision", [(16, 64), (128, 64), (128, 32)])
def test_multi_context_driver_matches_plain(k, precision, monkeypatch):
    """The one-process multi-GPU driver (qmfx_dist_init_all + qmfx_wals_half_multi, the C++
    engine's --ngpus path) on the one GPU here: a one-rank clique runs the phased half with
    the grouped per-piece broadcasts and the status all-reduce, and must reproduce a plain
    context bit for bit."""
    monkeypatch.setenv("QMFX_PIECES", "3")
    u, i, v = synth(3000, 600, 60000, seed=6)
    uids, iids, ucsr, icsr = csr_from_triples(u, i, v)
    init = np.random.default_rng(5).uniform(-0.01, 0.01, (len(iids), k))
    ctxs = []
    for r in range(2):
        c = qmf_amd.Context(k, precision)
        if r == 0:
            c.set_shape(len(uids), len(iids))
            c.upload_csr(0, *ucsr)
            c.upload_csr(1, *icsr)
        else:
            c.import_signals(ctxs[0])  # the --ngpus ingest: one build, device-to-device copies
        c.set_factors(1, init)
        ctxs.append(c)
    qmf_amd.dist_init_all([ctxs[1]])
    for _ in range(2):
        for side in (0, 1):
            l0 = ctxs[0].wals_half(side, ALPHA, LAM)
            l1 = qmf_amd.wals_half_multi([ctxs[1]], side, ALPHA, LAM)
            assert l0 == l1, side
            assert np.array_equal(ctxs[0].factors(side), ctxs[1].factors(side)), side
    for c in ctxs:
        c.close()


def test_multi_context_driver_failed_collective_aborts_the_clique(monkeypatch):
    """A context that fails after the clique's group has started (the broadcasts
    already posted would wait for peers that never join, and the next sync would hang) must
    make qmfx_wals_half_multi RETURN the error, with every communicator aborted, and later
    halves on those contexts must fail loudly instead of running or hanging."""
    monkeypatch.setenv("QMFX_PIECES", "2")
    # read once by the context: rank 0's piece broadcasts fail after the first half's two
    monkeypatch.setenv("QMFX_FAULT_COMM_RANK", "0:2")
    u, i, v = synth(2000, 400, 30000, seed=8)
    uids, iids, ucsr, icsr = csr_from_triples(u, i, v)
    c = qmf_amd.Context(16, 64)
    c.set_shape(len(uids), len(iids))
    c.upload_csr(0, *ucsr)
    c.upload_csr(1, *icsr)
    c.set_factors(1, np.random.default_rng(3).uniform(-0.01, 0.01, (len(iids), 16)))
    qmf_amd.dist_init_all([c])
    qmf_amd.wals_half_multi([c], 0, ALPHA, LAM)  # healthy first
    with pytest.raises(qmf_amd.QmfxError, match="injected collective failure"):
        qmf_amd.wals_half_multi([c], 1, ALPHA, LAM)
    with pytest.raises(qmf_amd.QmfxError, match="clique was aborted"):
        qmf_amd.wals_half_multi([c], 1, ALPHA, LAM)
    c.close()


def test_multi_context_driver_rejects_a_shared_device():
    """Two ranks on one GPU are refused (RCCL needs one device per rank): the drop-in CLI's
    --ngpus 2 on a one-GPU box fails instead of silently running one rank."""
    a, b = qmf_amd.Context(16, 64), qmf_amd.Context(16, 64)
    for c in (a, b):
        c.set_shape(10, 10)
    with pytest.raises(qmf_amd.QmfxError, match="two contexts on device"):
        qmf_amd.dist_init_all([a, b])
    a.close()
    b.close()


@pytest.mark.parametrize("comm", ["none", "loopback", "clique"])
def test_singular_rows_fail_every_rank(comm):
    """An exactly singular row system (λ = 0 and an all-zero fixed side: dsysv_'s info > 0,
    CHECK(info == 0) at Matrix.cpp:94) fails the half with -6.  With a communicator the
    half's status block (loss, re-solved and singular counts) is all-reduced, so every rank
    sees the count and fails in the same half."""
    u, i, v = synth(200, 50, 1500, seed=1)
    uids, iids, ucsr, icsr = csr_from_triples(u, i, v)
    c = qmf_amd.Context(8, 64)
    c.set_shape(len(uids), len(iids))
    c.upload_csr(0, *ucsr)
    c.upload_csr(1, *icsr)
    c.set_factors(1, np.zeros((len(iids), 8)))
    if comm == "loopback":
        c.dist_init(0, 1, qmf_amd.rccl_unique_id())
    elif comm == "clique":
        qmf_amd.dist_init_all([c])
    with pytest.raises(qmf_amd.QmfxError, match="singular"):
        if comm == "clique":
            qmf_amd.wals_half_multi([c], 0, ALPHA, 0.0)
        else:
            c.wals_half(0, ALPHA, 0.0)
    c.close()
