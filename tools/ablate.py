"""Timing ablation of the fused WALS kernel phases (QMFX_ABLATE bit mask; outputs garbage
when a phase is skipped).  Runs each mode in a subprocess and prints kernel ms per half."""
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
c = qmf_amd.Context(k, 32)
c.gen_synthetic(nu, ni, nnz, 3)
c.fill_uniform(1, 0.01, 103)
c.fill_uniform(0, 0.01, 104)
res = {}
for side in (0, 1):
    c.wals_half(side, 40.0, 0.05)
    c.reset_stats()
    c.wals_half(side, 40.0, 0.05)
    res[side] = c.solve_stats()["ms"]
print(json.dumps(res))
"""
cfg = [int(x) for x in sys.argv[1:5]] if len(sys.argv) > 4 else [10_000_000, 1_000_000, 500_000_000, 128]
for mode in [0, 1, 2, 4, 8, 6, 15]:
    env = dict(os.environ, QMFX_ABLATE=str(mode))
    out = subprocess.run([sys.executable, "-c", CODE % (ROOT, *cfg)], env=env, capture_output=True,
                         text=True, timeout=600)
    print("mode", mode, out.stdout.strip() or out.stderr[-500:], flush=True)
