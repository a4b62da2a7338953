"""Calibrate the CPU baseline: reference core (oracle/_ref, -O2) vs the C oracle (port, -O2) on
the same host, same workload shape (4 players, HARD, n_pieces=3, selected-mask loop, 1 thread).
Dev container only (needs the reference build).  Prints env-steps/s of both."""
import ctypes as C
import sys
import os
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
import pyoracle as po

n, steps = 256, 2000
seeds = []
s = 12345
while len(seeds) < n:
    if po.OracleVec(1) and True:
        o = po.OracleVec(1)
        o.reset(s, 4, 3, 2, 100000)
        if not (o.flags(0) & po.REF_UNSAFE):
            seeds.append(s)
    s += 1
lib = po._Lib.ref()
lib.ref_bench_seq.restype = C.c_double
lib.ref_bench_seq.argtypes = [C.POINTER(C.c_uint32), C.c_int, C.c_int, C.c_uint8, C.c_uint8, C.c_int]
arr = (C.c_uint32 * n)(*seeds)
t_ref = min(lib.ref_bench_seq(arr, n, steps, 4, 3, 2) for _ in range(3))
vec, smp = po.OracleVec(n), po.OracleSampler(n, 12345)
vec.reset(12345, 4, 3, 2, 100000)
t_orc = min(po.run_threaded(vec, smp, steps, 1) for _ in range(3))
print(f"reference core (1 thread, C++ loop): {n * steps / t_ref / 1e6:.2f} M env-steps/s")
print(f"C oracle port  (1 thread, runner loop): {n * steps / t_orc / 1e6:.2f} M env-steps/s")
print(f"port / reference = {t_ref / t_orc:.2f}")
