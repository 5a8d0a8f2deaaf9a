"""Build libcanu_ovl.so (overlapInCore) and libcanu_mhap.so (MHAP stage) for gfx950 in-tree
(canu_amd/lib/) with hipcc."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "lib")
OUT = os.path.join(OUT_DIR, "libcanu_ovl.so")
SOURCES = ["ovl_api.hip", "ovl_index.hip", "ovl_seed.hip", "ovl_extend.hip", "ovl_common.h",
           "ovl_ovb.h"]

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               # doubles in the extension (branch score, slope, quality) must round exactly
               # as the reference's: no fused multiply-add contraction
               "-ffp-contract=off"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES]
    deps.append(os.path.join(HERE, "..", "include", "canu_ovl.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


PROF_OUT = os.path.join(OUT_DIR, "libcanu_ovl_prof.so")
MHAP_OUT = os.path.join(OUT_DIR, "libcanu_mhap.so")
MHAP_DEPS = [os.path.join(CSRC, "mhap.hip"), os.path.join(HERE, "..", "include", "canu_mhap.h")]


def build_mhap(force: bool = False, verbose: bool = True) -> str:
    if not force and os.path.exists(MHAP_OUT) and \
            all(os.path.getmtime(d) <= os.path.getmtime(MHAP_OUT) for d in MHAP_DEPS):
        return MHAP_OUT
    os.makedirs(OUT_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *HIPCC_FLAGS, "-o", MHAP_OUT + ".tmp", os.path.join(CSRC, "mhap.hip")]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(MHAP_OUT + ".tmp", MHAP_OUT)
    return MHAP_OUT


BIN_DIR = os.path.join(HERE, "bin")
CLI_OUT = os.path.join(BIN_DIR, "overlapInCore")
CLI_DEPS = [os.path.join(CSRC, "oic_main.cpp"), os.path.join(CSRC, "gkp_store.h"),
            os.path.join(HERE, "..", "include", "canu_ovl.h")]


def build_cli(force: bool = False, verbose: bool = True) -> str:
    """canu_amd/bin/overlapInCore: the overlapInCore-compatible executable (host C++ over
    libcanu_ovl.so, found next to it through the rpath)."""
    lib = build(verbose=verbose)
    if not force and os.path.exists(CLI_OUT) and \
            all(os.path.getmtime(d) <= os.path.getmtime(CLI_OUT) for d in CLI_DEPS + [lib]):
        return CLI_OUT
    os.makedirs(BIN_DIR, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O2", "-std=c++17", "-Wall", "-o", CLI_OUT + ".tmp",
           os.path.join(CSRC, "oic_main.cpp"), "-L" + OUT_DIR, "-lcanu_ovl",
           "-Wl,-rpath,$ORIGIN/../lib", "-Wl,--allow-shlib-undefined"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(CLI_OUT + ".tmp", CLI_OUT)
    return CLI_OUT


MHAP_CLI_OUT = os.path.join(BIN_DIR, "mhap")


def build_mhap_cli(force: bool = False, verbose: bool = True) -> str:
    """canu_amd/bin/mhap: the MHAP command line canu's mhap.sh / precompute.sh run (host
    C++ over libcanu_mhap.so, found next to it through the rpath; zlib for -f .gz)."""
    lib = build_mhap(verbose=verbose)
    src = os.path.join(CSRC, "mhap_main.cpp")
    deps = [src, lib, os.path.join(HERE, "..", "include", "canu_mhap.h")]
    if not force and os.path.exists(MHAP_CLI_OUT) and \
            all(os.path.getmtime(d) <= os.path.getmtime(MHAP_CLI_OUT) for d in deps):
        return MHAP_CLI_OUT
    os.makedirs(BIN_DIR, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(HERE, "..", "include"),
           "-o", MHAP_CLI_OUT + ".tmp", src, "-L" + OUT_DIR, "-lcanu_mhap", "-lz",
           "-Wl,-rpath,$ORIGIN/../lib", "-Wl,--allow-shlib-undefined"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(MHAP_CLI_OUT + ".tmp", MHAP_CLI_OUT)
    return MHAP_CLI_OUT


def build(force: bool = False, verbose: bool = True, profile: bool = False) -> str:
    """profile=True builds the instrumented variant (in-kernel cycle stamps, OVL_DEBUG=1
    prints them) as libcanu_ovl_prof.so; load it with CANU_OVL_LIB."""
    out = PROF_OUT if profile else OUT
    if not force and not profile and not needs_build():
        return out
    os.makedirs(OUT_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    extra = ["-DOVL_PROFILE"] if profile else []
    cmd = [hipcc, *HIPCC_FLAGS, *extra, "-o", out + ".tmp", os.path.join(CSRC, "ovl_api.hip")]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, profile="--profile" in sys.argv)
    if "--profile" not in sys.argv:
        build_mhap(force="--force" in sys.argv)
        build_cli(force="--force" in sys.argv)
