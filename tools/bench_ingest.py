"""Device ingest throughput (qmfx_group_signals): N raw (user id, item id, value) records in
file order -> id tables + both CSR orientations on the GPU, host->device copy included.
usage: python tools/bench_ingest.py N_RECORDS [NUSERS NITEMS]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import qmf_amd  # noqa: E402

n = int(float(sys.argv[1]))
nu = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10_000_000
ni = int(float(sys.argv[3])) if len(sys.argv) > 3 else 1_000_000
rng = np.random.default_rng(5)
rec = np.empty(n, dtype=np.dtype([("u", "<i8"), ("i", "<i8"), ("v", "<f8")]))
rec["u"] = rng.integers(0, nu, n) * 2654435761 - 10**12  # scattered signed ids
rec["i"] = rng.integers(0, ni, n) * 40503 + 17
rec["v"] = rng.integers(1, 6, n)
c = qmf_amd.Context(128, 32)
# warm-up on a small slice (hipcub kernels, allocator)
c.group_signals(rec["u"][:100000], rec["i"][:100000], rec["v"][:100000])
t = time.perf_counter()
nu_out, ni_out = c.group_signals(rec["u"], rec["i"], rec["v"])
el = time.perf_counter() - t
out = {"records": n, "users": len(nu_out), "items": len(ni_out), "seconds": round(el, 3),
                  "records_per_s": round(n / el, 1), "note": "qmfx_group_signals incl. H2D copy of "
                  "24-byte records and the id-table download"}
cpu_n = int(float(os.environ.get("CPU_SAMPLE", "0")))
if cpu_n:
    # the oracle's WALSEngine::init restatement (dataset copy, std::sort by (user, item),
    # group, swap, std::sort, group; WALSEngine.cpp:37-69, 130-163), one thread
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle as po
    t = time.perf_counter()
    o = po.OracleWALS(rec["u"][:cpu_n], rec["i"][:cpu_n], rec["v"][:cpu_n], 4)
    el = time.perf_counter() - t
    out["cpu_baseline"] = {"records": cpu_n, "seconds": round(el, 3), "records_per_s": round(cpu_n / el, 1),
                           "cores": 1, "kind": "port"}
print(json.dumps(out), flush=True)
