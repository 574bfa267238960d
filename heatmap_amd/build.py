"""Build the gfx950 shared library in-tree: heatmap_amd/_lib/libheatmap_amd.so.

    python -m heatmap_amd.build            # incremental
    python -m heatmap_amd.build --force

hipcc cross-compiles for gfx950 without a GPU.  -ffp-contract=off is part of
the numerical contract: the projection arithmetic must not fuse a*b+c except
where the source writes fma() (see csrc/hm_common.h).
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIBDIR, "libheatmap_amd.so")
SOURCES = ["hm_kernels.hip", "hm_general.hip", "hm_stream.hip", "hm_merge.hip", "hm_api.cpp", "hm_host.c"]
HEADERS = ["hm_common.h", "hm_device.h", "hm_glibc_emul.h", "hm_branred.h", "hm_project.h", "hm_pipeline.h",
           "hm_ytab.h", "hm_table.h"]
ARCH = os.environ.get("HM_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=" + ARCH,
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unknown-pragmas",
         "-Wno-unused-label"]

HOST_FLAGS = ["-O2", "-fPIC", "-ffp-contract=off", "-std=c11", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
              "-Wno-unknown-pragmas"]


def _stale() -> bool:
    if not os.path.exists(LIB) or not os.path.exists(scalar_module_path()):
        return True
    if os.path.getmtime(os.path.join(CSRC, SCALAR_SRC)) > os.path.getmtime(scalar_module_path()):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "heatmap_amd.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True, out: str = None, defines=(), csrc: str = None) -> str:
    """Compile the library (out/defines/csrc: tools/variants.py builds tuning
    variants, from a patched copy of the sources for timing experiments)."""
    lib = out or LIB
    src_dir = csrc or CSRC
    if not force and out is None and not _stale():
        return LIB
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs, procs = [], []
    for src in SOURCES:   # the translation units compile in parallel
        obj = os.path.join(os.path.dirname(lib), os.path.basename(lib) + "." + src.rsplit(".", 1)[0] + ".o")
        if src.endswith(".c"):   # host C (hm_project_scalar): gcc, contraction off as everywhere
            cmd = [os.environ.get("CC", "gcc"), *HOST_FLAGS, "-c", os.path.join(src_dir, src), "-o", obj]
        else:
            cmd = [hipcc, *FLAGS, *["-D" + d for d in defines], "-c", os.path.join(src_dir, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    cmd = [hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", *objs, "-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(lib + ".tmp", lib)
    if out is None:
        build_scalar(verbose)
    return lib


SCALAR_SRC = "hm_pyscalar.c"


def scalar_module_path() -> str:
    import sysconfig

    return os.path.join(HERE, "_hm_scalar" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_scalar(verbose: bool = True) -> str:
    """The CPython binding of hm_project_scalar (per-record Tile calls), linked
    against the library next to it (rpath $ORIGIN/_lib)."""
    import sysconfig

    out = scalar_module_path()
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-shared", "-Wall", "-I" + sysconfig.get_paths()["include"],
           os.path.join(CSRC, SCALAR_SRC), "-L" + LIBDIR, "-lheatmap_amd", "-Wl,-rpath,$ORIGIN/_lib",
           "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force))
    sys.exit(0)
