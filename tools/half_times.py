"""Per-half timing of a bench workload: python tools/half_times.py CONFIG PRECISION [epochs]
Prints the wall time of each user half and item half and the per-class kernel time
(direct/big, whitened) of each, from the context's HIP-event accounting."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import qmf_amd  # noqa: E402

cfg, prec = sys.argv[1], int(sys.argv[2])
epochs = int(sys.argv[3]) if len(sys.argv) > 3 else 2
nu, ni, nnz, k, seed = bench.CONFIGS[cfg]
c = qmf_amd.Context(k, prec)
c.gen_synthetic(nu, ni, nnz, seed)
c.fill_uniform(1, 0.01, seed + 100)
c.sync()
for ep in range(epochs):
    for side in (0, 1):
        before = [c.kernel_stats(cl)["ms"] for cl in (0, 1)]
        t0 = time.perf_counter()
        c.wals_half(side, bench.ALPHA, bench.LAM)
        c.sync()
        dt = (time.perf_counter() - t0) * 1e3
        after = [c.kernel_stats(cl)["ms"] for cl in (0, 1)]
        print("%s f%d epoch %d %s half: %.1f ms (direct/big %.1f, whitened %.1f)" % (
            cfg, prec, ep, "user" if side == 0 else "item", dt, after[0] - before[0],
            after[1] - before[1]), flush=True)
