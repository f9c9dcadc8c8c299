"""WALS parity on the MI355X: the HIP path (through the C ABI) against the CPU oracle on
identical inputs and initial factors, at the reference's λ = 0.05, α = 40.

Tolerances (BASELINE.json north_star: factors within 1e-4 relative; index/ID bookkeeping
bit-exact): fp64 path (the CLI default) 1e-9 normwise-relative per half step (only rounding
differs: MFMA accumulation order and Cholesky vs Bunch-Kaufman); fp32 path 1e-4 on
well-posed inputs, and its k·cond·u bound on an ill-conditioned one.
"""
import os

import numpy as np
import pytest

import pyoracle as po
import qmf_amd
from helpers import csr_from_triples, load_ml100k, load_tiny, rel_err, synth

pytestmark = pytest.mark.gpu

LAM, ALPHA = 0.05, 40.0
NTHR = min(16, len(os.sched_getaffinity(0)))  # oracle threads (the box's CPU share)


def make_pair(users, items, values, k, precision, init=None, seed=0, lam=LAM, alpha=ALPHA):
    """(oracle, device context) on the same dataset with identical item-factor init."""
    o = po.OracleWALS(users, items, values, k, lam, alpha)
    uids, iids, (urp, ucol, uval), (irp, icol, ival) = csr_from_triples(users, items, values)
    # bookkeeping: the independent numpy CSR must equal the oracle's (bit-exact)
    assert np.array_equal(uids, o.ids(0)) and np.array_equal(iids, o.ids(1))
    for side, (rp, col, val) in ((0, (urp, ucol, uval)), (1, (irp, icol, ival))):
        orp, ocol, oval = o.csr(side)
        assert np.array_equal(orp, rp) and np.array_equal(ocol, col)
        # std::sort leaves the order of duplicate (u, i) pairs unspecified: compare the
        # values of duplicates as multisets
        row = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
        a = np.lexsort((oval, ocol, row))
        b = np.lexsort((val, col, row))
        assert np.array_equal(oval[a], val[b])
    c = qmf_amd.Context(k, precision)
    c.set_shape(len(uids), len(iids))
    c.upload_csr(0, urp, ucol, uval)
    c.upload_csr(1, irp, icol, ival)
    if init is None:
        init = np.random.default_rng(seed).uniform(-0.01, 0.01, (len(iids), k))
    o.set_factors(1, init)
    c.set_factors(1, init)
    return o, c


def test_mfma_layout_f32_f64():
    rng = np.random.default_rng(0)
    A = rng.integers(-8, 8, (16, 4)).astype(np.float64)
    B = rng.integers(-8, 8, (4, 16)).astype(np.float64)
    for prec in (32, 64):
        np.testing.assert_array_equal(qmf_amd.selftest_mfma(prec, A, B), A @ B)


@pytest.mark.parametrize("k", [8, 16, 30])
def test_tiny_half_steps(k):
    """The edge-case fixture (duplicates, zero values, signed ids) through the default fp64
    path at the reference's λ/α, per half in lock-step."""
    u, i, v = load_tiny()
    o, c = make_pair(u, i, v, k, 64, seed=k)
    for epoch in range(2):
        for side in (0, 1):
            lo = o.iterate(side)
            ld = c.wals_half(side, ALPHA, LAM) / (o.nusers * o.nitems)
            assert rel_err(c.factors(side), o.factors(side)) < 1e-9
            assert abs(ld - lo) <= 1e-8 * max(1.0, abs(lo))
            # keep the two in lock-step for the next half
            c.set_factors(side, o.factors(side))


def row_conditions(o, side):
    """cond₂ of every row system A = YᵀY + Σ αv y yᵀ + λI of `side` (numpy, from the
    oracle's CSR and fixed-side factors)."""
    rp, col, val = o.csr(side)
    Y = o.factors(1 - side)
    M = Y.T @ Y + LAM * np.eye(Y.shape[1])
    out = []
    for r in range(len(rp) - 1):
        y = Y[col[rp[r]:rp[r + 1]]]
        out.append(np.linalg.cond(M + (y.T * (ALPHA * val[rp[r]:rp[r + 1]])) @ y))
    return np.array(out)


@pytest.mark.parametrize("k", [8, 16])
def test_fp32_error_is_bounded_by_conditioning(k):
    """The opt-in fp32 path on an ILL-conditioned fixture at the reference's λ/α: the tiny
    fixture has 9 users, so its item systems reach cond ≈ 1e4–1e5 and no fp32 solve (nor
    fp32 storage of the fixed side alone) can be within 1e-4 of the fp64 reference there.
    What fp32 does guarantee is the normwise bound k·cond·u (u = 2⁻²⁴); that is checked
    here.  Well-posed inputs meet 1e-4 (the tests below and
    tests/test_configs_gpu.py)."""
    u, i, v = load_tiny()
    o, c = make_pair(u, i, v, k, 32, seed=k)
    for side in (0, 1):
        kappa = row_conditions(o, side).max()
        o.iterate(side)
        c.wals_half(side, ALPHA, LAM)
        err = rel_err(c.factors(side), o.factors(side))
        assert err < k * kappa * 2.0 ** -24, (side, err, kappa)
        c.set_factors(side, o.factors(side))


@pytest.mark.parametrize("precision,tol", [(64, 1e-9), (32, 1e-4)])
def test_ml100k_shape_ten_epochs(precision, tol):
    """The survey's reference-pinned dataset: 10 epochs run
    independently on both sides at the reference's λ/α; factors and the per-epoch loss must
    track the oracle (fp32 measured at ≈1e-5 after 10 epochs)."""
    d = load_ml100k()
    k = 30
    init = d["init"][: 1682 * k].reshape(1682, k)
    o, c = make_pair(d["users"], d["items"], d["values"], k, precision, init=init)
    ol = o.optimize(10, 4)
    dl = []
    for _ in range(10):
        c.wals_half(0, ALPHA, LAM)
        dl.append(c.wals_half(1, ALPHA, LAM) / (o.nusers * o.nitems))
    # the reference's printed losses carry 6 significant digits
    assert abs(dl[0] - float(d["ref_loss_epoch1"])) < 5e-6
    assert abs(dl[9] - float(d["ref_loss_epoch10"])) < 5e-7
    np.testing.assert_allclose(dl, ol, rtol=tol)
    assert rel_err(c.factors(0), o.factors(0)) < tol
    assert rel_err(c.factors(1), o.factors(1)) < tol


@pytest.mark.parametrize("k", [32, 64, 96, 128])
def test_synthetic_fp32_one_epoch(k):
    u, i, v = synth(3000, 700, 40000, seed=k)
    o, c = make_pair(u, i, v, k, 32, seed=1)
    for side in (0, 1):
        lo = o.iterate(side)
        ld = c.wals_half(side, ALPHA, LAM) / (o.nusers * o.nitems)
        assert rel_err(c.factors(side), o.factors(side)) < 1e-4
        assert abs(ld - lo) < 1e-4 * abs(lo)


def test_single_signal_rows_and_tails():
    # rows with 1..9 signals exercise every k-step tail of the 4-wide MFMA loop
    users, items = [], []
    for r in range(1, 10):
        for j in range(r):
            users.append(r)
            items.append((r * 7 + j * 3) % 23)
    v = np.arange(len(users)) % 5 + 1.0
    o, c = make_pair(users, items, v, 8, 64, seed=3)
    o.iterate(0)
    c.wals_half(0, ALPHA, LAM)
    assert rel_err(c.factors(0), o.factors(0)) < 1e-10


def test_update_factors_for_one_known_answer():
    # WALSEngineTest.cpp:145-205 through the device path: Y ≡ 0.1, α = λ = 1 → x = 0.4/1.12
    c = qmf_amd.Context(3, 64)
    c.set_shape(1, 2)
    c.upload_csr(0, [0, 2], [0, 1], [1.0, 1.0])
    c.upload_csr(1, [0, 1, 2], [0, 0], [1.0, 1.0])
    c.set_factors(1, np.full((2, 3), 0.1))
    c.wals_half(0, 1.0, 1.0)
    np.testing.assert_allclose(c.factors(0), np.full((1, 3), 0.4 / 1.12), rtol=1e-12)


def test_zero_and_negative_values_spd_path():
    # value 0 contributes only to b (c = 1), never to A; still SPD
    u, i, v = load_tiny()
    assert (v == 0).any()
    o, c = make_pair(u, i, v, 8, 64, seed=5)
    o.iterate(0)
    c.wals_half(0, ALPHA, LAM)
    assert len(c.failed_rows()) == 0
    assert rel_err(c.factors(0), o.factors(0)) < 1e-9


@pytest.mark.parametrize("precision", [64, 32])
def test_indefinite_rows_are_resolved_on_device(precision):
    """1 + α·v < 0 makes some systems indefinite: the Cholesky kernels flag them and the
    device re-solves them in fp64 with a pivoted factorization (dsysv_'s role,
    Matrix.cpp:81-96) before the half ends — factors and loss match the oracle."""
    u = np.array([0, 0, 0, 1, 1, 2])
    i = np.array([0, 1, 2, 0, 2, 1])
    v = np.array([-5.0, -5.0, -5.0, 1.0, 2.0, 1.0])
    o, c = make_pair(u, i, v, 8, precision, init=np.full((3, 8), 0.3), lam=0.01, alpha=40.0)
    lo = o.iterate(0)
    ld = c.wals_half(0, 40.0, 0.01) / (o.nusers * o.nitems)
    assert 0 in set(c.failed_rows().tolist())
    tol = 1e-9 if precision == 64 else 1e-4  # fp32: the fixed side and YᵀY are fp32
    assert rel_err(c.factors(0), o.factors(0)) < tol
    assert abs(ld - lo) < tol * abs(lo)


@pytest.mark.parametrize("k", [16, 128, 256])
def test_heavy_indefinite_rows_fallback(k):
    """Negative values on long rows at every row-kernel route (direct, multi-wave): many
    flagged rows, several per workgroup share, rows longer than the 16-signal staging."""
    u, i, v = synth(2000, 300, 30000, seed=k)
    v = v.copy()
    v[::7] = -3.0
    o, c = make_pair(u, i, v, k, 64, seed=2)
    for side in (0, 1):
        lo = o.iterate(side, NTHR)
        ld = c.wals_half(side, ALPHA, LAM) / (o.nusers * o.nitems)
        assert len(c.failed_rows()) > 0
        # indefinite systems, different pivot orders (GEPP vs Bunch-Kaufman): rounding is
        # amplified by cond(A), hence 1e-7 rather than the SPD path's 1e-9
        assert rel_err(c.factors(side), o.factors(side)) < 1e-7, side
        assert abs(ld - lo) < 1e-7 * abs(lo), side
        c.set_factors(side, o.factors(side))


def test_row_system_matches_oracle():
    """qmfx_wals_row_system builds one row's k×k system on the device (A with λ, b, Σc)."""
    u, i, v = synth(500, 120, 8000, seed=3)
    o, c = make_pair(u, i, v, 24, 64, seed=1)
    rp, col, val = o.csr(1)
    Y = o.factors(0)
    c.set_factors(0, Y)
    r = int(np.argmax(np.diff(rp)))
    A, b, cs = c.row_system(1, r, ALPHA, LAM)
    ys = Y[col[rp[r]:rp[r + 1]]]
    w = ALPHA * val[rp[r]:rp[r + 1]]
    A_ref = Y.T @ Y + (ys.T * w) @ ys + LAM * np.eye(24)
    np.testing.assert_allclose(A, A_ref, rtol=1e-12, atol=1e-12 * np.abs(A_ref).max())
    np.testing.assert_allclose(b, ys.T @ (1 + w), rtol=1e-12)
    assert abs(cs - np.sum(1 + w)) < 1e-9


@pytest.mark.parametrize("k,precision,nnz", [
    (256, 32, 30000), (128, 32, 30000), (64, 32, 30000), (64, 64, 30000), (32, 64, 30000),
    # fp64 k = 80..128 run the streamed fp64 kernel; the 160K-signal sets put users at ~40
    # signals (every n×n bucket up to n = 64)
    (128, 64, 30000), (128, 64, 160000), (80, 64, 160000), (112, 64, 160000), (80, 64, 30000),
    (256, 32, 160000),
    # k = 64, ~40 signals per user: fp32 whitens n ≤ 64 (the NTN = 3 / 4 buckets), fp64
    # n ≤ 48 on the streamed fp64 kernel (round 5)
    (64, 32, 160000), (64, 64, 160000),
    # fp32 k = 256 / 128, ~100 signals per user: the n = 65..128 buckets (two signals per
    # lane)
    (256, 32, 400000), (128, 32, 400000),
    # fp64 k = 128, ~100 signals per user: the streamed fp64 kernel's n = 65..80 bucket (two
    # signals per lane, second ballot words, 5-tile fp64 Cholesky)
    (128, 64, 400000),
    # fp64 k = 256 (C5 at the reference's precision): the streamed fp64 kernel beside the
    # big k×k kernel, every bucket up to n = 80
    (256, 64, 30000), (256, 64, 160000), (256, 64, 400000)])
def test_whitened_rows_match_direct_and_oracle(k, precision, nnz, monkeypatch):
    """Short rows (n ≤ KP/2) take the whitened n×n path; the same half step with
    QMFX_NO_WHITEN=1 (direct k×k path for every row) and the oracle must agree."""
    u, i, v = synth(4000, 900, nnz, seed=11)  # ~7.5 (or ~40) signals per user
    v[::7] = 0.0  # zero-valued signals (Q set: c = 1, w = 0)
    o, c = make_pair(u, i, v, k, precision, seed=2)
    if nnz == 400000:
        # the two-signals-per-lane buckets (n > 64 → 5 or more 16-row tiles) hold rows
        wb = c.row_classes(0)["whitened"]
        assert wb[4] > 0, wb
    if k == 64 and nnz == 160000:
        wb = c.row_classes(0)["whitened"]
        assert wb[2] > 0 and (wb[3] > 0) == (precision == 32), wb
    monkeypatch.setenv("QMFX_NO_WHITEN", "1")
    _, cd = make_pair(u, i, v, k, precision, seed=2)
    assert sum(cd.row_classes(0)["whitened"]) == 0
    monkeypatch.delenv("QMFX_NO_WHITEN")
    tol = 1e-4 if precision == 32 else 1e-9
    for side in (0, 1):
        lo = o.iterate(side)
        lw = c.wals_half(side, ALPHA, LAM) / (o.nusers * o.nitems)
        ld = cd.wals_half(side, ALPHA, LAM) / (o.nusers * o.nitems)
        # SPD rows: the pivoted re-solve must not have run (it would mask a kernel bug)
        assert len(c.failed_rows()) == 0 and len(cd.failed_rows()) == 0, side
        assert rel_err(c.factors(side), o.factors(side)) < tol, side
        assert rel_err(cd.factors(side), o.factors(side)) < tol, side
        assert abs(lw - lo) < tol * abs(lo) * 10 and abs(ld - lo) < tol * abs(lo) * 10
        c.set_factors(side, o.factors(side))
        cd.set_factors(side, o.factors(side))


@pytest.mark.parametrize("k,precision", [(144, 32), (192, 32), (256, 32), (80, 64), (112, 64),
                                         (128, 64), (200, 64), (256, 64)])
def test_large_k_multiwave_rows(k, precision):
    """k beyond one wave's registers (fp32 > 128, fp64 > 64): the multi-wave row kernel
    (LDS-staged Gram, distributed Cholesky) and the strip YᵀY, against the oracle at the
    reference's λ/α; rows from 1 to ~150 signals cover partial LDS stages and every
    panel-slot count.  800 items ≫ k keeps the item systems well-posed for fp32.  fp64
    k = 80..128 rows run the one-wave direct kernel (accumulators across VGPR + AGPR)."""
    u, i, v = synth(4000, 800, 100000, seed=k)
    o, c = make_pair(u, i, v, k, precision, seed=3)
    tol = 1e-9 if precision == 64 else 1e-4
    for side in (0, 1):
        lo = o.iterate(side, NTHR)
        ld = c.wals_half(side, ALPHA, LAM) / (o.nusers * o.nitems)
        # SPD systems: no row may need the pivoted re-solve (it would mask a kernel bug)
        assert len(c.failed_rows()) == 0, side
        assert rel_err(c.factors(side), o.factors(side)) < tol, side
        assert abs(ld - lo) < tol * abs(lo), side
        c.set_factors(side, o.factors(side))  # lock-step: each half checked on its own


@pytest.mark.parametrize("k", [96, 128])
def test_long_rows_fp32_direct(k):
    """Rows with hundreds of signals on the fp32 direct kernel at the reference's λ/α: the
    LDS-staged (column, value) chunks of the split-bf16 Gram (prologue, chunk hand-over,
    ragged last step, zero-row padding) against the oracle, on both halves.  ~500 signals
    per item, ~5 per user, 400 items ≫ k."""
    u, i, v = synth(40000, 400, 200000, seed=k)
    o, c = make_pair(u, i, v, k, 32, seed=4)
    for side in (0, 1):
        lo = o.iterate(side, NTHR)
        ld = c.wals_half(side, ALPHA, LAM) / (o.nusers * o.nitems)
        assert len(c.failed_rows()) == 0, side
        assert rel_err(c.factors(side), o.factors(side)) < 1e-4, side
        assert abs(ld - lo) < 1e-4 * abs(lo), side
        c.set_factors(side, o.factors(side))


@pytest.mark.parametrize("k,precision,lam", [(64, 32, LAM), (128, 32, LAM), (32, 64, LAM),
                                             (64, 32, 0.0)])
def test_solve_pieces_bit_identical(k, precision, lam, monkeypatch):
    """A half solved in several pieces (QMFX_PIECES: the multi-GPU schedule, where piece j
    is all-gathered while piece j+1 is solved) must give bit-identical factors to the
    one-piece solve (rows are independent).  The loss sum agrees to 1e-9 relative: a few
    whitened rows' fp32 loss terms differ in the last bit with the launch layout.  Mixed row
    lengths put whitened and direct rows in every piece; λ = 0 forces every row direct."""
    u, i, v = synth(3000, 700, 60000, seed=5)
    u = np.concatenate([u, np.full(300, 3001)])  # one heavy user
    i = np.concatenate([i, np.arange(300)])
    v = np.concatenate([v, np.ones(300)])
    _, c1 = make_pair(u, i, v, k, precision, seed=4, lam=max(lam, LAM))
    for pieces in (3, 7):
        monkeypatch.setenv("QMFX_PIECES", str(pieces))
        _, cp = make_pair(u, i, v, k, precision, seed=4, lam=max(lam, LAM))
        monkeypatch.delenv("QMFX_PIECES")
        c1.set_factors(1, cp.factors(1))
        for side in (0, 1):
            l1 = c1.wals_half(side, ALPHA, lam)
            lp = cp.wals_half(side, ALPHA, lam)
            assert np.array_equal(c1.factors(side), cp.factors(side)), (pieces, side)
            assert abs(l1 - lp) <= 1e-9 * abs(l1), (pieces, side)


@pytest.mark.parametrize("k", [256, 128])
def test_row_chunked_launches_bit_identical(k, monkeypatch):
    """Per-row kernels are launched in chunks below 2^31 threads (10M rows × 512 threads of
    the k = 256 kernel overflowed a single launch and silently skipped rows).  Forcing tiny
    chunks (QMFX_ROW_CHUNK) must not change a single bit."""
    u, i, v = synth(1200, 300, 30000, seed=9)
    _, c1 = make_pair(u, i, v, k, 32, seed=6)
    _, c2 = make_pair(u, i, v, k, 32, seed=6)
    for side in (0, 1):
        l1 = c1.wals_half(side, ALPHA, LAM)
        # the chunk is read per launch: set only around the chunked context's half
        monkeypatch.setenv("QMFX_ROW_CHUNK", "37")
        l2 = c2.wals_half(side, ALPHA, LAM)
        monkeypatch.delenv("QMFX_ROW_CHUNK")
        assert np.array_equal(c1.factors(side), c2.factors(side)), side
        assert l1 == l2, side


@pytest.mark.parametrize("k", [64, 128])
def test_whitening_grid_strides_bit_identical(k, monkeypatch):
    """fp64 k ≤ 128 whitening GEMMs (x = L⁻ᵀx' over the whitened rows, Z = YL⁻ᵀ over the
    fixed side) run on a persistent grid with L⁻¹ in LDS (whiten_lds_kernel).  Cut to one
    workgroup (QMFX_WHITEN_GRID=1, read per launch) every wave strides over ~80 32-row
    blocks; the half must not change a bit, and it must match the oracle."""
    u, i, v = synth(20000, 900, 300000, seed=13)  # ~15 signals per user: users whitened
    o, c1 = make_pair(u, i, v, k, 64, seed=2)
    _, c2 = make_pair(u, i, v, k, 64, seed=2)
    assert sum(c1.row_classes(0)["whitened"]) > 15000
    for side in (0, 1):
        lo = o.iterate(side, NTHR)
        l1 = c1.wals_half(side, ALPHA, LAM)
        monkeypatch.setenv("QMFX_WHITEN_GRID", "1")
        l2 = c2.wals_half(side, ALPHA, LAM)
        monkeypatch.delenv("QMFX_WHITEN_GRID")
        assert np.array_equal(c1.factors(side), c2.factors(side)), side
        assert l1 == l2, side
        assert rel_err(c1.factors(side), o.factors(side)) < 1e-9, side
        assert abs(l1 / (o.nusers * o.nitems) - lo) < 1e-9 * abs(lo), side
        c1.set_factors(side, o.factors(side))
        c2.set_factors(side, o.factors(side))
