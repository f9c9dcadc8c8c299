"""Run C3-shaped halves with QMFX_TRACE and summarise the row kernels' phases: per-phase
cycle medians by row length, and how the waves of each SIMD overlap.
Whitened rows: load, K+setup, chol, x'+store.  Direct rows: G image, Gram, chol, store."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
path = os.path.join(ROOT, "gpurun_out", "trace")
os.environ["QMFX_TRACE"] = path
import qmf_amd  # noqa: E402

cfg = [int(x) for x in sys.argv[1:5]] if len(sys.argv) > 4 else [10_000_000, 1_000_000, 500_000_000, 128]
c = qmf_amd.Context(cfg[3], int(os.environ.get("PREC", "32")))
c.gen_synthetic(cfg[0], cfg[1], cfg[2], 3)
c.fill_uniform(1, 0.01, 103)
side = int(os.environ.get("SIDE", "0"))
c.fill_uniform(0, 0.01, 104)
c.wals_half(side, 40.0, 0.05)
c.wals_half(side, 40.0, 0.05)
t = np.fromfile(path + "_side%d.bin" % side, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
os.remove(path + "_side%d.bin" % side)
# rows without a record (all-zero: the split-K heavy rows' segment/solve launches and the fp32
# streamed whitened kernel, which has no traced instance, do not stamp) are left out, and
# counted so their absence is visible
untraced = int((t[:, 0] == 0).sum())
t = t[t[:, 0] > 0]
if untraced:
    print("rows without a trace record (split-K heavy rows; fp32 whitened rows), left out:", untraced)
ph = np.diff(t[:, 0:5], axis=1)  # load, K+setup, chol, x'+store
n = t[:, 6]
print("rows traced", len(t))
names = ["load", "K+setup", "chol", "x'+store"]
bins = ((1, 16), (17, 32), (33, 48), (49, 64), (65, 128), (129, 400), (401, 600), (601, 10**9))
for lo, hi in bins:
    m = (n >= lo) & (n <= hi)
    if m.sum() == 0:
        continue
    med = np.median(ph[m], axis=0)
    print(f"n {lo:2d}-{hi:2d}: rows {m.sum():8d}  " +
          "  ".join(f"{nm} {v:7.0f}" for nm, v in zip(names, med)) + f"  total {med.sum():7.0f} cyc")
# per-SIMD concurrency: key = (xcc, cu bits, simd)
hw = t[:, 5]
hw1 = (hw >> 40) & 0xffff  # two-wave kernels: wave 1's HW_ID
if (hw1 != 0).any():
    same_cu = ((hw >> 8) & 0xff) == ((hw1 >> 8) & 0xff)
    same_simd = same_cu & (((hw >> 4) & 3) == ((hw1 >> 4) & 3))
    print(f"two-wave rows: waves on the same CU {same_cu.mean():.3f}, on the same SIMD {same_simd.mean():.3f}")
hw = hw & 0xffffffffff
key = (hw >> 32) * 4096 + ((hw >> 8) & 0xff) * 4 + ((hw >> 4) & 3)
order = np.lexsort((t[:, 0], key))
t, key = t[order], key[order]
uk, starts = np.unique(key, return_index=True)
ends = np.r_[starts[1:], len(key)]
busy2 = load2 = tot = gap = 0
sample = np.linspace(0, len(uk) - 1, min(len(uk), 400)).astype(int)
for s_i in sample:
    a, b = starts[s_i], ends[s_i]
    seg = t[a:b]
    lo_, hi_ = seg[:, 0].min(), seg[:, 4].max()
    T = hi_ - lo_
    if T <= 0:
        continue
    grid = np.zeros(int(T // 64) + 1, dtype=np.int8)   # waves in compute per 64-cycle bin
    lgrid = np.zeros_like(grid)                          # waves in load phase
    for r in seg:
        grid[(r[1] - lo_) // 64:(r[4] - lo_) // 64] += 1
        lgrid[(r[0] - lo_) // 64:(r[1] - lo_) // 64] += 1
    tot += len(grid)
    busy2 += (grid >= 2).sum()
    load2 += ((grid == 0) & (lgrid >= 1)).sum()
    gap += ((grid == 0) & (lgrid == 0)).sum()
print(f"SIMD time with >=2 waves computing {busy2 / tot:.3f}, only loading {load2 / tot:.3f}, "
      f"idle {gap / tot:.3f}, exactly one computing {1 - (busy2 + load2 + gap) / tot:.3f}")
print("waves per SIMD (median rows per SIMD):", int(np.median(ends - starts)))
