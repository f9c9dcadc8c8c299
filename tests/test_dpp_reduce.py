"""The butterfly row sums of csrc/rowsolve.h (row16_sum4_split, row16_sum8_split) on a lane
model of the DPP patterns they use (no GPU): after the exchanges, lane i of every 16-lane row
must hold the row's full sum of the column the header names (v[i >> 2], resp. column
4·b3 + 2·b2 + b0 of i).  The GPU whitened-row tests check the same code on hardware through
x' = Zₛᵀu; this pins the lane algebra the kernels' stores rely on."""
import numpy as np


def dpp(src, ctl):
    """64-lane DPP move: src[lane] -> value lane receives, for the controls rowsolve.h uses."""
    out = np.empty_like(src)
    for lane in range(64):
        row, i = divmod(lane, 16)
        if 0x121 <= ctl <= 0x12F:          # row_ror:r — rotate right within the 16-lane row
            j = (i - (ctl - 0x120)) % 16
        elif ctl == 0x141:                 # row_half_mirror — reverse each half row of 8
            j = (i & 8) | (7 - (i & 7))
        elif ctl <= 0xFF:                  # quad_perm — lane 4q + x reads 4q + sel[x]
            j = (i & ~3) | ((ctl >> (2 * (i & 3))) & 3)
        else:
            raise ValueError(hex(ctl))
        out[lane] = src[16 * row + j]
    return out


def sel(c, a, b):
    return np.where(c, a, b)


def sum4_split(v):  # v: [4][64]
    cl = np.arange(64) % 16
    b3, b2 = (cl & 8) != 0, (cl & 4) != 0
    k0, k1 = sel(b3, v[2], v[0]), sel(b3, v[3], v[1])
    s0, s1 = sel(b3, v[0], v[2]), sel(b3, v[1], v[3])
    k0 = k0 + dpp(s0, 0x128)
    k1 = k1 + dpp(s1, 0x128)
    k = sel(b2, k1, k0)
    k = k + dpp(sel(b2, k0, k1), 0x141)
    k = k + dpp(k, 0xB1)
    k = k + dpp(k, 0x4E)
    return k


def sum8_split(v):  # v: [2][4][64]
    cl = np.arange(64) % 16
    b3, b2, b0 = (cl & 8) != 0, (cl & 4) != 0, (cl & 1) != 0
    k = []
    for c in range(4):
        kc = sel(b3, v[1][c], v[0][c])
        k.append(kc + dpp(sel(b3, v[0][c], v[1][c]), 0x128))
    m0, m1 = sel(b2, k[2], k[0]), sel(b2, k[3], k[1])
    m0 = m0 + dpp(sel(b2, k[0], k[2]), 0x141)
    m1 = m1 + dpp(sel(b2, k[1], k[3]), 0x141)
    r = sel(b0, m1, m0)
    r = r + dpp(sel(b0, m0, m1), 0xB1)
    r = r + dpp(r, 0x4E)
    return r


def test_quad_perm_controls_are_the_xor_pairs():
    x = np.arange(64)
    assert (dpp(x, 0xB1) == (x ^ 1)).all()
    assert (dpp(x, 0x4E) == (x ^ 2)).all()
    assert (dpp(x, 0x141) == (x ^ 7)).all()
    assert (dpp(x, 0x128) == (x ^ 8)).all()


def test_row16_sum4_split_gives_each_lane_its_columns_row_sum():
    rng = np.random.default_rng(1)
    # integers: the sums are exact in any order
    v = rng.integers(-1000, 1000, size=(4, 64)).astype(np.int64)
    got = sum4_split(v)
    for lane in range(64):
        row, i = divmod(lane, 16)
        c = i >> 2
        assert got[lane] == v[c, 16 * row:16 * row + 16].sum()


def test_row16_sum8_split_gives_each_lane_its_columns_row_sum():
    rng = np.random.default_rng(2)
    v = rng.integers(-1000, 1000, size=(2, 4, 64)).astype(np.int64)
    got = sum8_split(v)
    for lane in range(64):
        row, i = divmod(lane, 16)
        col = 4 * ((i >> 3) & 1) + 2 * ((i >> 2) & 1) + (i & 1)  # row16_sum8_column
        h, c = divmod(col, 4)
        assert got[lane] == v[h, c, 16 * row:16 * row + 16].sum()
    # the storing lanes (cl & 2 == 0) cover the eight columns once per row
    cols = sorted(4 * ((i >> 3) & 1) + 2 * ((i >> 2) & 1) + (i & 1) for i in range(16) if not i & 2)
    assert cols == list(range(8))
