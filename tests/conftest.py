import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def host_math():
    """Test-only gcc build of heatmap_amd/csrc/hm_project.h (see tests/host_math)."""
    import ctypes

    src = os.path.join(REPO, "tests", "host_math", "hm_host_math.c")
    out_dir = os.path.join(REPO, "tests", "host_math", "_build")
    out = os.path.join(out_dir, "libhm_host_math.so")
    deps = [src] + [os.path.join(REPO, "heatmap_amd", "csrc", f) for f in
                    ("hm_project.h", "hm_glibc_emul.h", "hm_branred.h", "hm_common.h", "hm_ytab.h")]
    if not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps):
        os.makedirs(out_dir, exist_ok=True)
        subprocess.check_call(["gcc", "-O2", "-mfma", "-ffp-contract=off", "-fPIC", "-shared", "-w",
                               "-I" + os.path.join(REPO, "heatmap_amd", "csrc"), src, "-o", out, "-lm"])
    L = ctypes.CDLL(out)
    P = ctypes.POINTER
    L.hmh_project.argtypes = [P(ctypes.c_double), P(ctypes.c_double), ctypes.c_int64, ctypes.c_int,
                              P(ctypes.c_int64), P(ctypes.c_int64), P(ctypes.c_uint8), P(ctypes.c_uint8)]
    L.hmh_fast_Y_maxerr.argtypes = [P(ctypes.c_double), ctypes.c_int64, P(ctypes.c_double)]
    L.hmh_fast_Y_maxerr.restype = ctypes.c_double
    L.hmh_glibc_check.argtypes = [ctypes.c_int, P(ctypes.c_double), ctypes.c_int64, P(ctypes.c_int64)]
    L.hmh_glibc_check.restype = ctypes.c_int64
    L.hmh_project_fast.argtypes = [P(ctypes.c_double), P(ctypes.c_double), ctypes.c_int64, ctypes.c_int,
                                   P(ctypes.c_int32), P(ctypes.c_int32), P(ctypes.c_uint8)]
    L.hmh_project_fast.restype = ctypes.c_int64
    return L


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from heatmap_amd import _lib

    _lib.load()
    return torch


def cells_digest(zoom, row, col, count):
    """Order-free digest of a cell multiset: (cells, total count, sum and xor of
    a 64-bit mix of each (zoom, row, col, count)).  Large comparisons use it
    instead of sorting hundreds of millions of cells."""
    import numpy as np

    with np.errstate(over="ignore"):
        x = (np.asarray(zoom, np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ np.asarray(row).astype(np.uint64)
        x = (x * np.uint64(0xBF58476D1CE4E5B9)) ^ np.asarray(col).astype(np.uint64)
        x = (x * np.uint64(0x94D049BB133111EB)) ^ np.asarray(count).astype(np.uint64)
        x ^= x >> np.uint64(31)
        x *= np.uint64(0xD6E8FEB86659FD93)
        x ^= x >> np.uint64(32)
        return (int(x.size), int(np.asarray(count).sum()), int(x.sum(dtype=np.uint64)),
                int(np.bitwise_xor.reduce(x)) if x.size else 0)
