"""CPU: the C-ABI library loads and exports every entry point include/heatmap_amd.h
declares; without a GPU every device entry point fails loudly (no CPU fallback).
No compute call is made here."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "heatmap_amd.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(hm_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared()
    for n in ("hm_project", "hm_count", "hm_count_tiles", "hm_count_grouped", "hm_last_error", "hm_ctx_create"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from heatmap_amd import _lib

    L = _lib.load()
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.lib_path()], text=True)
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    assert set(_lib.EXPORTS) == set(declared())
    assert L.hm_abi_version() == _lib.HM_ABI_VERSION == 7
    assert _lib.status_string(_lib.HM_E_DOMAIN) == "math domain error"
    assert _lib.status_string(_lib.HM_E_NAN) == "cannot convert float NaN to integer"


def test_error_mapping_matches_reference_exceptions():
    from heatmap_amd import _lib

    with pytest.raises(ValueError, match="^math domain error$"):
        _lib.raise_for(_lib.HM_E_DOMAIN)
    with pytest.raises(ValueError, match="^cannot convert float NaN to integer$"):
        _lib.raise_for(_lib.HM_E_NAN)
    with pytest.raises(OverflowError, match="^cannot convert float infinity to integer$"):
        _lib.raise_for(_lib.HM_E_INF)
    with pytest.raises(_lib.DevicePathUnsupported):
        _lib.raise_for(_lib.HM_E_EXOTIC)
    _lib.raise_for(_lib.HM_OK)


def test_no_gpu_fails_loudly():
    """Without a GPU the product raises instead of computing on the CPU."""
    code = r"""
import sys, ctypes
import torch
if torch.cuda.is_available():
    print("SKIP"); sys.exit(0)
from heatmap_amd import _lib, device
try:
    device.project([1.0], [2.0], 3)
except _lib.DeviceUnavailable as e:
    print("RAISED", e)
from heatmap_amd.stream import StreamingHeatmap
try:
    StreamingHeatmap(0, 18)
except _lib.DeviceUnavailable as e:
    print("STREAM RAISED", e)
L = _lib.load()
p = ctypes.c_void_p()
st = L.hm_ctx_create(ctypes.byref(p), 0, None)
print("CTX", st)
print("STREAM ARG", L.hm_stream_create(None, 0, 18, 0, 0, 0, ctypes.byref(p)))
"""
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, timeout=300)
    if "SKIP" in r.stdout:
        pytest.skip("a GPU is present")
    assert "RAISED" in r.stdout, r.stdout + r.stderr
    assert "CTX 18" in r.stdout, r.stdout + r.stderr     # HM_E_HIP
    assert "STREAM RAISED" in r.stdout, r.stdout + r.stderr
    assert "STREAM ARG 16" in r.stdout, r.stdout + r.stderr  # HM_E_ARG: no context


def test_product_does_not_import_the_oracle():
    pkg = os.path.join(REPO, "heatmap_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(root, f)).read()
                assert "from oracle" not in txt and "import oracle" not in txt and "hm_oracle" not in txt, f
