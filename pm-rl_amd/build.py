"""Build the in-tree native libraries.

    python pm-rl_amd/build.py            # libpmenv.so (HIP, gfx950), tools/libpmenv_ab.so, oracle/liboracle.so

libpmenv.so is the product (the C ABI of include/pmenv.h). oracle/liboracle.so is
the CPU parity checker (test infrastructure). Both are built in place so they
travel with the repository snapshot to the GPU box.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "pmenv", "libpmenv.so")
AB_LIB = os.path.join(ROOT, "tools", "libpmenv_ab.so")
SRC = os.path.join(HERE, "csrc", "pmenv.hip")
AB_DIR = os.path.join(ROOT, "tools", "ab")
AB_SRC = os.path.join(AB_DIR, "pmenv_ab.hip")     # the tools build's hooks (linked with SRC)
ORACLE_SRC = os.path.join(ROOT, "oracle", "pmenv_oracle.c")
ORACLE_LIB = os.path.join(ROOT, "oracle", "liboracle.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PMENV_ARCH", "gfx950")


def _stale(out, *srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def _run(cmd):
    print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build_pmenv(force=False, ab=False):
    """The product library; ab=True: the tools build (tools/libpmenv_ab.so: the product's
    translation unit linked with tools/ab/pmenv_ab.hip, whose pmenv_tools hooks alone read
    the PMENV_* A/B knobs and launch the measured alternatives and the timing-only
    ablations)."""
    out = AB_LIB if ab else LIB
    deps = [os.path.join(ROOT, "include", "pmenv.h")] + [
        os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc")) if f.endswith(".h")]
    srcs = [SRC] + ([AB_SRC] if ab else [])
    if ab:
        deps += [os.path.join(AB_DIR, f) for f in os.listdir(AB_DIR) if f.endswith(".h")]
    if not force and not _stale(out, *srcs, *deps, __file__):
        return out
    _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
          "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include"), "-o", out] + srcs)
    return out


def build_oracle(force=False):
    hdrs = [os.path.join(ROOT, "oracle", "pmenv_oracle.h"), os.path.join(ROOT, "include", "pmenv.h")]
    if not force and not _stale(ORACLE_LIB, ORACLE_SRC, *hdrs):
        return ORACLE_LIB
    _run(["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-fopenmp", "-Wall", "-Wextra",
          "-Wno-unused-parameter", "-o", ORACLE_LIB, ORACLE_SRC, "-lm"])
    return ORACLE_LIB


C_ABI_SRC = os.path.join(ROOT, "tests", "c_abi", "c_abi_step.c")
C_ABI_BIN = os.path.join(ROOT, "tests", "c_abi", "c_abi_step")


def build_c_abi_test(force=False):
    """A plain C caller of the C ABI linked against libpmenv.so and the parity checker
    (test infrastructure: tests/test_gpu_c_abi.py runs it on the GPU box)."""
    hdrs = [os.path.join(ROOT, "include", "pmenv.h"), os.path.join(ROOT, "oracle", "pmenv_oracle.h")]
    if not force and not _stale(C_ABI_BIN, C_ABI_SRC, LIB, ORACLE_LIB, *hdrs):
        return C_ABI_BIN
    rocm = os.path.dirname(os.path.dirname(os.path.realpath(HIPCC)))
    _run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-D__HIP_PLATFORM_AMD__",
          "-I", os.path.join(rocm, "include"), "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
          "-o", C_ABI_BIN, C_ABI_SRC, "-L", os.path.dirname(LIB), "-lpmenv", "-L", os.path.dirname(ORACLE_LIB),
          "-loracle", "-L", os.path.join(rocm, "lib"), "-lamdhip64", "-lm",
          "-Wl,-rpath,$ORIGIN/../../pm-rl_amd/pmenv:$ORIGIN/../../oracle:" + os.path.join(rocm, "lib")])
    return C_ABI_BIN


def build_all(force=False):
    build_pmenv(force)
    build_pmenv(force, ab=True)
    build_oracle(force)
    build_c_abi_test(force)


if __name__ == "__main__":
    if "--ab-only" in sys.argv:      # the tools library alone (an A/B run on the GPU box builds it there)
        build_pmenv("--force" in sys.argv, ab=True)
    else:
        build_all(force="--force" in sys.argv)
