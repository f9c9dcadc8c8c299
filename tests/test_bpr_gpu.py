"""BPR Hogwild epoch kernel (qmfx_bpr_epoch) on the MI355X, exact single-wave semantics.

With min(nusers, nitems) < 32 the epoch runs on one wave, i.e. serially, as the reference's
1-thread Hogwild (BPREngine::optimize/iterateBlock, BPREngine.cpp:146-176, -inl.h:31-46).
The visiting order (identity, or the seeded affine permutation when shuffling) and every
negative (counter-based draw: one splitmix64 key per positive, a murmur3 finaliser per
attempt, rejected against the user's positives; -inl.h:48-60 draws from mt19937 instead, so
the stream itself is this build's) are restated here; the
resulting (u, p, n) sequence run through the oracle's BPREngine::update
(BPREngine.cpp:178-220) must reproduce the device's factors and biases.  Tolerance: fp64
1e-12, fp32 1e-5 relative."""
import numpy as np
import pytest

import pyoracle as po
import qmf_amd

pytestmark = pytest.mark.gpu
M64 = (1 << 64) - 1
M32 = (1 << 32) - 1


def mix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def fmix32(x):
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & M32
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & M32
    return x ^ (x >> 16)


def permutation(seed, npos, shuffle):
    if not shuffle:
        return 1, 0
    pa = (mix64(seed ^ 0xA5A5A5A5) % npos) | 1
    while np.gcd(pa, npos) != 1:
        pa += 2
    pa %= npos
    pa = pa or 1
    return pa, mix64(seed ^ 0x5A5A5A5A) % npos


def triplets(users, items, nitems, seed, num_neg, shuffle):
    npos = len(users)
    pos = {}
    for u, i in zip(users, items):
        pos.setdefault(int(u), set()).add(int(i))
    pa, pb = permutation(seed, npos, shuffle)
    seed_key = mix64(seed ^ 0xB5AD4ECEDA1CE2A9)
    out = []
    for i in range(npos):
        slot = (pa * i + pb) % npos
        u, p = int(users[slot]), int(items[slot])
        pkey = mix64(seed_key ^ slot)
        fk = (pkey & M32) ^ (pkey >> 32)
        for j in range(num_neg):
            attempt = 0
            while True:
                h = fmix32((fk + ((4099 * j + attempt) * 0x9E3779B9)) & M32)
                cand = (h * nitems) >> 32
                if cand not in pos[u] or attempt >= 4096:
                    break
                attempt += 1
            out.append((u, p, cand))
    return np.array(out, np.int64)


@pytest.mark.parametrize("precision,tol", [(64, 1e-12), (32, 1e-5)])
@pytest.mark.parametrize("use_biases", [False, True])
@pytest.mark.parametrize("num_neg", [3, 6])
@pytest.mark.parametrize("atomic_user", ["0", "1"])
def test_bpr_epoch_single_wave_exact(precision, tol, use_biases, num_neg, atomic_user,
                                     monkeypatch):
    """One wave (the reference's serial order): both ways of writing the user row back (plain
    store, C4's default; atomic add of the net change, skewed users) are exact."""
    monkeypatch.setenv("QMFX_BPR_ATOMIC_USER", atomic_user)
    rng = np.random.default_rng(num_neg + 10 * use_biases)
    nu, ni, k = 20, 300, 16
    # user 0 has > 64 positives (rejection scans memory), others a few; few items per
    # user leaves repeated negatives within a positive likely for num_neg = 6
    users = np.concatenate([np.zeros(90, np.int64), rng.integers(1, nu, 400)])
    items = np.concatenate([rng.permutation(ni)[:90], rng.integers(0, ni, 400)])
    keys = np.unique(users * ni + items, return_index=True)[1]
    users, items = users[np.sort(keys)], items[np.sort(keys)]
    U0 = rng.normal(0, 0.1, (nu, k))
    I0 = rng.normal(0, 0.1, (ni, k))
    b0 = rng.normal(0, 0.1, ni) if use_biases else np.zeros(ni)
    lr, lam = 0.05, (1.0, 0.025, 0.0025)
    with qmf_amd.Context(k, precision) as c:
        c.set_shape(nu, ni)
        c.set_factors(0, U0)
        c.set_factors(1, I0)
        c.bpr_set_biases(b0)
        c.bpr_set_positives(users, items)
        U, I, b = U0.copy(), I0.copy(), b0.copy()
        for epoch, (seed, shuffle) in enumerate(((7, False), (8, True))):
            c.bpr_epoch(seed, num_neg, lr, *lam, use_biases, shuffle=shuffle)
            trip = triplets(users, items, ni, seed, num_neg, shuffle)
            po.bpr_update_seq(U, I, b, trip, lr, *lam, use_biases)
            scale = max(np.abs(U).max(), np.abs(I).max())
            assert np.max(np.abs(c.factors(0) - U)) <= tol * scale, epoch
            assert np.max(np.abs(c.factors(1) - I)) <= tol * scale, epoch
            if use_biases:
                assert np.max(np.abs(c.bpr_biases() - b)) <= tol * max(np.abs(b).max(), 1), epoch
            assert c.bpr_plan() == (1, int(atomic_user))


@pytest.mark.parametrize("skewed", [False, True])
def test_bpr_atomic_user_follows_user_skew(skewed):
    """The user row is stored plainly while concurrent waves rarely hold the same user; a
    dataset with one dominant user (≥ 1% of the positives per concurrent wave) switches it to
    the atomic add (qmfx.cpp bpr_args)."""
    rng = np.random.default_rng(5)
    # 800 items → 50 concurrent waves; ~50 positives per user (the largest ≈ 80): 50 × 80 <
    # 1% of ~1M positives.  Skewed: user 0 holds all 800 items
    nu, ni, k, npos = 20000, 800, 16, 1000000
    users = rng.integers(0, nu, npos)
    if skewed:
        users[: npos // 10] = 0  # one user holds 10% of the positives
    items = rng.integers(0, ni, npos)
    keys = np.unique(users * ni + items, return_index=True)[1]
    users, items = users[np.sort(keys)], items[np.sort(keys)]
    with qmf_amd.Context(k, 32) as c:
        c.set_shape(nu, ni)
        c.fill_uniform(0, 0.01, 1)
        c.fill_uniform(1, 0.01, 2)
        c.bpr_set_positives(users, items)
        c.bpr_epoch(3, 3, 0.05, 1.0, 0.025, 0.0025, False, shuffle=False)
        waves, atomic = c.bpr_plan()
    assert waves > 1
    assert atomic == (1 if skewed else 0)
