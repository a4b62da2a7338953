"""CPU: the kernels' uniform_int_distribution variants (gym-eldorado_amd/csrc/cog_rng.h: uid_fast
with one division, uid_small with none) against the libstdc++ formula they replace (uid), on the
boundary cases of every k the engine uses -- each quotient boundary j*s-1, j*s, the rejection
boundary past-1, past and the range end -- and on random states.  The header is plain integer
code; g++ builds it here after defining COG_HD."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gym-eldorado_amd", "csrc")
P = 2 ** 31 - 1
RANGE = 2147483645

HARNESS = r"""
#define COG_HD static inline
#include "cog_rng.h"
extern "C" void run(const uint32_t *x0, const uint32_t *k, uint32_t n, int which, uint32_t *out, uint32_t *xout) {
  for (uint32_t i = 0; i < n; i++) {
    uint32_t x = x0[i];
    out[i] = which == 0 ? cog::uid(x, k[i]) : which == 1 ? cog::uid_fast(x, k[i]) : cog::uid_small(x, k[i]);
    xout[i] = x;
  }
}
// the table form: one accepted draw, r < k s (uid_small_accepted's precondition as well)
extern "C" uint32_t run_tab(const uint32_t *r, const uint32_t *k, uint32_t n, uint32_t *out) {
  uint32_t bad = 0;
  for (uint32_t i = 0; i < n; i++) {
    const cog::UidEntry e = cog::uid_entry(k[i]);
    out[i] = cog::uid_tab_accepted(r[i], e.s, e.m);
    bad += out[i] != cog::uid_small_accepted(r[i], k[i]);
  }
  return bad;
}
// mr_jump(x, 16807^j) for j = 1..4 against j sequential mr_next steps
extern "C" uint32_t run_jump(const uint32_t *x0, uint32_t n) {
  uint32_t bad = 0;
  const uint32_t c[4] = {cog::mr_pow(1), cog::mr_pow(2), cog::mr_pow(3), cog::mr_pow(4)};
  for (uint32_t i = 0; i < n; i++) {
    uint32_t x = x0[i];
    for (int j = 0; j < 4; j++) {
      cog::mr_next(x);
      bad += cog::mr_jump(x0[i], c[j]) != x;
    }
  }
  return bad;
}
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("rng")
    src, so = d / "harness.cpp", d / "librng.so"
    src.write_text(HARNESS)
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", f"-I{CSRC}", str(src), "-o", str(so)], check=True)
    lib = ctypes.CDLL(str(so))
    lib.run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.run_jump.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    lib.run_jump.restype = ctypes.c_uint32
    lib.run_tab.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    lib.run_tab.restype = ctypes.c_uint32
    return lib


def call(lib, which, x0, k):
    x0 = np.ascontiguousarray(x0, dtype=np.uint32)
    k = np.ascontiguousarray(k, dtype=np.uint32)
    out, xo = np.empty_like(x0), np.empty_like(x0)
    lib.run(x0.ctypes.data, k.ctypes.data, len(x0), which, out.ctypes.data, xo.ctypes.data)
    return out, xo


def state_before(r):
    """minstd_rand0 state whose next draw gives urng() - 1 == r."""
    inv = pow(16807, -1, P)
    return (r + 1) * inv % P


def boundary_cases(kmax):
    xs, ks = [], []
    for k in range(1, kmax + 1):
        s = RANGE // k
        past = k * s
        rs = {0, 1, past - 1, past, min(past + 1, RANGE), RANGE - 1, RANGE}
        for j in range(1, k + 1):
            rs |= {j * s - 1, j * s, j * s + 1}
        for r in sorted(r for r in rs if 0 <= r <= RANGE):
            xs.append(state_before(r))
            ks.append(k)
    return np.array(xs), np.array(ks)


@pytest.mark.parametrize("which,kmax", [(1, 300), (2, 31)])
def test_boundaries(lib, which, kmax):
    x0, k = boundary_cases(kmax)
    ref, xref = call(lib, 0, x0, k)
    got, xgot = call(lib, which, x0, k)
    bad = np.nonzero((ref != got) | (xref != xgot))[0]
    assert bad.size == 0, f"k={k[bad[:5]]} x0={x0[bad[:5]]}: {ref[bad[:5]]} vs {got[bad[:5]]}"


@pytest.mark.parametrize("which,kmax", [(1, 255), (2, 31)])
def test_random_states(lib, which, kmax):
    rng = np.random.default_rng(7 + which)
    x0 = rng.integers(1, P, size=2_000_000, dtype=np.uint64).astype(np.uint32)
    k = rng.integers(1, kmax + 1, size=x0.size, dtype=np.uint64).astype(np.uint32)
    ref, xref = call(lib, 0, x0, k)
    got, xgot = call(lib, which, x0, k)
    assert np.array_equal(ref, got) and np.array_equal(xref, xgot)


def test_jump_ahead(lib):
    """The draw's jump-ahead states (x * 16807^j mod 2^31-1) equal j sequential steps: random
    states plus the extremes of the state space."""
    rng = np.random.default_rng(11)
    x0 = np.concatenate([np.array([1, 2, 16807, P - 2, P - 1, 2 ** 30, 2 ** 31 - 2], dtype=np.uint64),
                         rng.integers(1, P, size=1_000_000, dtype=np.uint64)]).astype(np.uint32)
    assert lib.run_jump(x0.ctypes.data, len(x0)) == 0


def test_table_uniform(lib):
    """uid_tab_accepted (the LDS-table form the kernels use for k <= 31) equals r / (range / k) on
    every quotient boundary of every k and on random accepted draws."""
    rs, ks = [], []
    for k in range(1, 32):
        s = RANGE // k
        for j in range(1, k + 1):
            rs += [j * s - 2, j * s - 1, j * s, j * s + 1]
        rs += [0, 1, k * s - 1]
        ks += [k] * (4 * k + 3)
    rng = np.random.default_rng(5)
    kr = rng.integers(1, 32, size=1_000_000)
    rr = (rng.random(kr.size) * (RANGE // kr * kr)).astype(np.int64)
    r = np.concatenate([np.array(rs, dtype=np.int64), rr])
    k = np.concatenate([np.array(ks, dtype=np.int64), kr])
    keep = (r >= 0) & (r < (RANGE // k) * k)
    r, k = r[keep].astype(np.uint32), k[keep].astype(np.uint32)
    out = np.empty_like(r)
    assert lib.run_tab(r.ctypes.data, k.ctypes.data, len(r), out.ctypes.data) == 0
    assert np.array_equal(out, (r.astype(np.int64) // (RANGE // k.astype(np.int64))).astype(np.uint32))
