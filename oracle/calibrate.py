"""Calibrate the CPU baseline: reference core (oracle/_ref, -O2) vs the C oracle (port, -O2) on
the same host, same workload shape (4 players, HARD, n_pieces=3, selected-mask loop, 1 thread).
Dev container only (needs the reference build).  Prints env-steps/s of both; --json PATH also
writes them (profiles/calibration.json: bench.py's cpu_baseline.port_over_reference).

    python oracle/calibrate.py [--json profiles/calibration.json] [--reps 3]"""
import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
import pyoracle as po

ap = argparse.ArgumentParser()
ap.add_argument("--json")
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
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
ratios = []
for rep in range(args.reps):                     # (interleaved: the host's drift hits both alike)
    t_ref = min(lib.ref_bench_seq(arr, n, steps, 4, 3, 2) for _ in range(3))
    vec, smp = po.OracleVec(n), po.OracleSampler(n, 12345)
    vec.reset(12345, 4, 3, 2, 100000)
    t_orc = min(po.run_threaded(vec, smp, steps, 1) for _ in range(3))
    ratios.append((n * steps / t_ref, n * steps / t_orc))
    print(f"reference core (1 thread, C++ loop): {n * steps / t_ref / 1e6:.2f} M env-steps/s")
    print(f"C oracle port  (1 thread, runner loop): {n * steps / t_orc / 1e6:.2f} M env-steps/s")
    print(f"port / reference = {t_ref / t_orc:.2f}")
if args.json:
    r = sorted(o / f for f, o in ratios)
    json.dump({"port_over_reference": r[len(r) // 2], "ratios": r,
               "reference_env_steps_per_s": [f for f, _ in ratios], "port_env_steps_per_s": [o for _, o in ratios],
               "workload": f"{n} hazard-free envs from seed 12345, 4p HARD n_pieces 3, max_steps 100000, "
                           f"{steps} steps of sample(selected masks)+step, 1 thread, best of 3 per rep",
               "host": f"{platform.machine()} {os.cpu_count()} CPUs (the dev container)",
               "date": time.strftime("%Y-%m-%d")}, open(args.json, "w"), indent=1)
