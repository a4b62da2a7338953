"""In-tree build of the engine for gfx950 (no pip install; the .so files travel with the repo).

    python gym-eldorado_amd/build_ext.py          # library + bindings (+ oracle checkers)

Outputs (git-ignored, shipped to the GPU box by the snapshot):
    gym-eldorado_amd/city_of_gold/libcog_hip.so          HIP kernels + C ABI (hipcc, gfx950)
    gym-eldorado_amd/city_of_gold/libcog_hip_fence.so    the same with -DCOG_TRIO_FENCE (tests only)
    gym-eldorado_amd/city_of_gold/_city_of_gold*.so      pybind11 host module (links the above)
    oracle/liboracle.so                                  C oracle (test infrastructure only)
    oracle/_ref/libref.so                                reference core (only where /root/reference exists)
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "city_of_gold")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("COG_OFFLOAD_ARCH", "gfx950")

LIB = os.path.join(OUT, "libcog_hip.so")
# the same engine with the trio's progress counters published by workgroup-scope release stores
# (-DCOG_TRIO_FENCE) instead of relaxed in-order LDS stores: a test-only build that the GPU tests
# compare with the oracle beside the product's (tests/test_gpu_trio_fence.py), so that a compiler
# or scheduler change breaking the relaxed form's ordering shows up as a parity difference
LIB_FENCE = os.path.join(OUT, "libcog_hip_fence.so")
EXT = os.path.join(OUT, "_city_of_gold" + sysconfig.get_config_var("EXT_SUFFIX"))

ENGINE_SRCS = [os.path.join(CSRC, f) for f in ("cog_engine.hip", "cog_abi.cpp")]
ENGINE_DEPS = ENGINE_SRCS + [os.path.join(CSRC, f) for f in ("cog_engine.h", "cog_tables.h", "cog_rng.h")] + [
    os.path.join(INCLUDE, f) for f in ("cog.h", "cog_types.h")]
EXT_SRCS = [os.path.join(CSRC, "pybind_module.cpp")]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, cwd=None):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=cwd)


OBJ = os.path.join(PKG, "build")
HEADERS = [os.path.join(CSRC, f) for f in ("cog_engine.h", "cog_tables.h", "cog_rng.h")] + [
    os.path.join(INCLUDE, f) for f in ("cog.h", "cog_types.h")]


def _compile_cmd(src, obj, defs=()):
    # max-ilp scheduling: the rollout runs one wave per SIMD, so only instruction-level
    # parallelism hides latency (1 % faster than the default, tools/flags_exp.sh); loop heads on
    # 64-B instruction-cache lines: the trio's step time otherwise moves by 1-2 % with unrelated
    # code size changes (profiles/r06_compact_decks_ab.txt)
    return [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c",
            "-ffp-contract=off", "-mllvm", "-amdgpu-sched-strategy=max-ilp", "-falign-loops=64", "-Wall",
            *defs, f"-I{INCLUDE}", f"-I{CSRC}", src, "-o", obj]


def build_engine(force=False, fence=True):
    """One object per source (the kernels' TU takes about two minutes, the ABI's seconds), then
    the shared library; the kernels' TU of the COG_TRIO_FENCE test build compiles beside it."""
    os.makedirs(OBJ, exist_ok=True)
    jobs, objs = [], []
    for src in ENGINE_SRCS:
        obj = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + HEADERS):
            jobs.append(_compile_cmd(src, obj))
    eng_fence = os.path.join(OBJ, "cog_engine_fence.hip.o")
    if fence and (force or _stale(eng_fence, [ENGINE_SRCS[0]] + HEADERS)):
        jobs.append(_compile_cmd(ENGINE_SRCS[0], eng_fence, ["-DCOG_TRIO_FENCE"]))
    procs = []
    for cmd in jobs:                                       # (concurrently: the two kernel TUs)
        print("+", " ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc")
    if force or _stale(LIB, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB])
    if fence and (force or _stale(LIB_FENCE, [eng_fence, objs[1]])):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", eng_fence, objs[1], "-o", LIB_FENCE])
    return LIB


def build_bindings(force=False):
    import pybind11

    if force or _stale(EXT, EXT_SRCS + [LIB, os.path.join(INCLUDE, "cog.h"), os.path.join(INCLUDE, "cog_types.h")]):
        cxx = os.environ.get("CXX", "g++")
        _run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-fvisibility=hidden",
              f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{INCLUDE}",
              *EXT_SRCS, "-o", EXT, f"-L{OUT}", "-lcog_hip", "-Wl,-rpath,$ORIGIN"])
    return EXT


def build_oracle():
    """Checkers only (tests / smoke / bench cpu_baseline); never linked by the product."""
    _run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"])
    if os.path.isdir("/root/reference/src"):
        _run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "oracle"), "ref"])


def build_all(force=False, oracle=True):
    build_engine(force)
    build_bindings(force)
    if oracle:
        build_oracle()


def add_to_path():
    if PKG not in sys.path:
        sys.path.insert(0, PKG)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
