"""Is the direct-row Gram memory-latency bound?  Item-side half over 100K rows x 500 signals
(C3's item shape, k=128) with the signals' user rows drawn from all 10M users vs from a
small, cache-resident set.  Prints ms per half for each."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import qmf_amd  # noqa: E402

nu, ni, per, k = 10_000_000, 100_000, 500, 128
rng = np.random.default_rng(0)
rp = np.arange(ni + 1, dtype=np.int64) * per
val = rng.integers(1, 6, ni * per).astype(np.float32)
for span in (nu, 1 << 20, 1 << 14, 1 << 10):
    col = np.sort(rng.integers(0, span, (ni, per)).astype(np.int32), axis=1).reshape(-1)
    with qmf_amd.Context(k, 32) as c:
        c.set_shape(nu, ni)
        c.upload_csr(1, rp, col, val)
        urp = np.zeros(nu + 1, dtype=np.int64)  # users: empty rows (only the item half runs)
        c.upload_csr(0, urp, np.zeros(0, np.int32), np.zeros(0, np.float32))
        c.fill_uniform(0, 0.01, 1)
        c.fill_uniform(1, 0.01, 2)
        c.wals_half(1, 40.0, 0.05)
        c.sync()
        c.reset_stats()
        t = time.time()
        for _ in range(3):
            c.wals_half(1, 40.0, 0.05)
        c.sync()
        ks = c.kernel_stats(0)
        print(f"user-row span {span:9d}: direct kernel {ks['ms'] / max(ks['launches'], 1):7.2f} ms/launch"
              f"  half {(time.time() - t) / 3 * 1e3:7.2f} ms", flush=True)
