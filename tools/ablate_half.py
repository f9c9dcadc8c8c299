"""Per-kernel timing of one WALS half under QMFX_ABLATE modes (timing experiments only:
results are garbage when a phase is skipped).  Prints the rocprof-free per-class event
times of the user half (whitened-dominated) and the item half (direct) at C3.
Bits: 1 skip direct Gram, 2 skip panel factorisation, 4 skip SYRK, 8 skip backward solve,
16 skip whitened K = ZZᵀ, 32 skip x' = Zᵀu.  PREC=64 for fp64 (default 32)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, json
sys.path.insert(0, %r)
import qmf_amd
nu, ni, nnz, k = %d, %d, %d, %d
c = qmf_amd.Context(k, %d)
c.gen_synthetic(nu, ni, nnz, 3)
c.fill_uniform(1, 0.01, 103)
c.fill_uniform(0, 0.01, 104)
res = {}
for side in (0, 1):
    c.wals_half(side, 40.0, 0.05)
    c.reset_stats()
    c.wals_half(side, 40.0, 0.05)
    res[side] = {n: round(c.kernel_stats(cl)["ms"], 2) for cl, n in ((0, "direct"), (1, "whitened"), (2, "half"))}
print(json.dumps(res))
"""
cfg = [int(x) for x in sys.argv[1:5]] if len(sys.argv) > 4 else [10_000_000, 1_000_000, 500_000_000, 128]
modes = [int(x) for x in os.environ.get("MODES", "0 16 32 2 4 8 14 62").split()]
for mode in modes:
    env = dict(os.environ, QMFX_ABLATE=str(mode))
    out = subprocess.run([sys.executable, "-c", CODE % (ROOT, *cfg, int(os.environ.get("PREC", "32")))], env=env, capture_output=True,
                         text=True, timeout=600)
    print("mode", mode, out.stdout.strip() or out.stderr[-500:], flush=True)
