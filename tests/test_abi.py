"""CPU-side checks of the C ABI library: it loads, exports every symbol include/qmfx.h
declares, and its host-only helpers work without a GPU."""
import os
import re

import numpy as np
import pytest

import qmf_amd
from helpers import ROOT


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "qmfx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int)\s+(qmfx_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_entry_points():
    syms = _declared_symbols()
    assert "qmfx_wals_half" in syms and "qmfx_bpr_epoch" in syms and len(syms) >= 25


def test_library_exports_every_declared_symbol():
    L = qmf_amd.lib()
    missing = [s for s in _declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    # and the Python binding covers the whole header
    assert set(_declared_symbols()) == set(qmf_amd._abi.SIGNATURES)


def test_version():
    assert qmf_amd.version() == 1


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partition_rows_nnz_balanced(world):
    rng = np.random.default_rng(world)
    deg = rng.integers(0, 200, size=1000)
    rp = np.concatenate([[0], np.cumsum(deg)])
    bounds = [qmf_amd.partition_rows(rp, world, r) for r in range(world)]
    assert bounds[0][0] == 0 and bounds[-1][1] == 1000
    for (b0, e0), (b1, e1) in zip(bounds, bounds[1:]):
        assert e0 == b1  # contiguous, disjoint cover
    loads = [rp[e] - rp[b] for b, e in bounds]
    assert max(loads) - min(loads) <= 2 * deg.max()


def test_create_without_gpu_fails_loudly():
    # In the CPU container there is no device: creating a context must raise, never
    # silently run on the CPU.
    import ctypes
    cnt = ctypes.c_int(0)
    rc = qmf_amd.lib().qmfx_device_count(ctypes.byref(cnt))
    if rc == 0 and cnt.value > 0:
        pytest.skip("GPU present")
    with pytest.raises(qmf_amd.QmfxError):
        qmf_amd.Context(8, 32)


def test_download_csr_is_double_across_the_abi():
    # qmfx_download_csr hands values back in double (an fp32 context's widened exactly), so
    # host-side checkers never see an fp32-narrowed problem
    src = open(os.path.join(ROOT, "include", "qmfx.h")).read()
    decl = re.search(r"int qmfx_download_csr\(([^)]*)\)", src).group(1)
    assert "double* values" in decl and "float" not in decl
    import ctypes
    assert qmf_amd._abi.SIGNATURES["qmfx_download_csr"][-1] is ctypes.POINTER(ctypes.c_double)
