"""qmf_amd — MI355X-native implicit-feedback matrix factorisation (WALS + BPR).

The product is the C ABI in ``include/qmfx.h`` implemented by ``qmf_amd/_build/libqmfx.so``
(hand-written HIP kernels for gfx950) and the drop-in C++ ``qmf`` engine / CLIs built on it
(``qmf_amd/host``).  This Python module is a thin ctypes front-end used by the tests and
``bench.py``; it never falls back to a CPU implementation: if the library is missing or no
GPU is present the calls fail loudly.
"""
from ._abi import (  # noqa: F401
    LIB_PATH, QmfxError, Context, build, device_count, dist_init_all, dist_plan, lib, partition_rows, rccl_unique_id, selftest_mfma,
    version, wals_half_multi,
)

USERS = 0
ITEMS = 1
