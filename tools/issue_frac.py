"""The stepping wave's per-step instruction count from the trio kernel's ISA (diagnostic; no GPU).

    python tools/issue_frac.py [--obj OBJ] [--lat 0|1] [--chain profiles/r06_chainprobe.txt]
                                   [--json profiles/issue_profile.json]

Compiles the engine with -DCOG_ISSUE_COUNT (the product source with the stepping wave's rare
sampling fallback -- step_action behind the wave-uniform `ballot(!fast)` skip, never taken on a
canonical step -- replaced by a park, so that its code is out of the listing; build/ is left
alone, the object goes to /tmp unless --obj names one), disassembles k_env_rollout_trio
(tools/isa.sh), takes the stepping wave's region (from its s_setprio 3 to the kernel's end)
and in it the step loop: the largest loop whose body holds the ring record's ds_write_b128
stores and no s_barrier (the per-block prologue's).  The count leaves out the progress waits'
spin loops (s_sleep); what remains is an upper bound of what a wave issues on a canonical step:
every lane-divergent `if` of the lean step is issued whenever any of the 64 lanes takes it, which
in a 64-env wave is nearly every step, and the park paths (skipped when no lane parks) are
counted too.  bench.py's roofline.limiter.issue_frac =
this count x the lone-wave dependent-chain cost per instruction (tools/chainprobe.hip,
profiles/*_chainprobe.txt) / the stepping wave's measured busy ticks per step
(profiles/stamps_profile.json).
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def disasm(obj, lat):
    sym = "k_env_rollout_trioILi0ELb%d" % lat
    env = dict(os.environ, OBJ=obj)
    return subprocess.run(["bash", os.path.join(ROOT, "tools/isa.sh"), sym], capture_output=True, text=True,
                          env=env, check=True).stdout


def parse(text):
    ins = []
    for line in text.split("\n"):
        m = re.match(r"\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return ins


def loops(ins, lo):
    idx = {a: k for k, (a, _, _) in enumerate(ins)}
    out = []
    for k, (a, op, args) in enumerate(ins):
        if k < lo or not op.startswith(("s_branch", "s_cbranch")):
            continue
        m = re.search(r"(-?\d+)$", args.strip())
        if not m:
            continue
        off = int(m.group(1))
        off = off - 65536 if off > 32767 else off
        dst = a + 4 + off * 4
        if dst < a and dst in idx and idx[dst] >= lo:
            out.append((idx[dst], k))
    return out


def count(ins, lat):
    sp = [k for k, x in enumerate(ins) if x[1] == "s_setprio"]
    if not sp:
        raise SystemExit("no s_setprio: not the trio kernel")
    lo = sp[0]
    lps = loops(ins, lo)
    spins = [(s, e) for s, e in lps if e - s < 60 and any(op == "s_sleep" for _, op, _ in ins[s:e + 1])]
    cand = [(e - s, s, e) for s, e in lps if (s, e) not in spins
            and any(op == "ds_write_b128" for _, op, _ in ins[s:e + 1])
            and not any(op == "s_barrier" for _, op, _ in ins[s:e + 1])]
    if not cand:
        raise SystemExit("no step loop found")
    _, s, e = max(cand)
    body = list(range(s, e + 1))
    spin_set = {j for ss, ee in spins if s <= ss and ee <= e for j in range(ss, ee + 1)}
    hot = [j for j in body if j not in spin_set]
    mix = collections.Counter("valu" if ins[j][1].startswith("v_") else "salu" if ins[j][1].startswith("s_")
                              else "lds" if ins[j][1].startswith("ds_") else "vmem" for j in hot)
    return {"kernel": "k_env_rollout_trio<selected, %s>" % ("LAT" if lat else "two per CU"),
            "step_loop_static": len(body), "spin_loop_instructions": len(spin_set),
            "per_step_instructions": len(hot), "mix": dict(mix),
            "loop_addresses": "%x..%x" % (ins[s][0], ins[e][0])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--obj")
    ap.add_argument("--lat", type=int, default=None)
    ap.add_argument("--json")
    ap.add_argument("--chain")
    a = ap.parse_args()
    if not a.obj:                                          # the COG_ISSUE_COUNT build of this source
        sys.path.insert(0, os.path.join(ROOT, "gym-eldorado_amd"))
        import build_ext
        a.obj = "/tmp/cog_engine_issue_count.o"
        subprocess.run(build_ext._compile_cmd(os.path.join(ROOT, "gym-eldorado_amd/csrc/cog_engine.hip"), a.obj,
                                              ["-DCOG_ISSUE_COUNT"]), check=True, capture_output=True)
    res = {}
    for lat in ([a.lat] if a.lat is not None else [0, 1]):
        res["lat" if lat else "two_per_cu"] = count(parse(disasm(a.obj, lat)), lat)
    if a.chain:                                            # the lone-wave costs (tools/chainprobe.hip)
        cost = {}
        for line in open(a.chain):
            m = re.match(r"CHAIN (.+?)\s+([\d.]+) ticks per link,\s+([\d.]+) per instruction \(lone wave, (\w+)\)", line)
            if m:
                cost[m.group(1).strip()] = float(m.group(3))
        res["costs"] = {
            "issue": {"valu": cost["ISSUE 4 x v_add_u32"], "salu": cost["ISSUE 4 x s_add_u32"],
                      "lds": cost["ISSUE 4 x ds_read_b32 + wait"], "vmem": cost["ISSUE 4 x ds_read_b32 + wait"]},
            "dependent": {"valu": cost["v_add_u32"], "salu": cost["s_add_u32"],
                          "lds": cost["ds_read_b32+wait+v_and"], "vmem": cost["ds_read_b32+wait+v_and"]},
            "source": os.path.relpath(a.chain, ROOT), "unit": "s_memtime ticks per instruction (the stamps' unit)"}
        for key in ("lat", "two_per_cu"):
            if key in res:
                mix = res[key]["mix"]
                for form in ("issue", "dependent"):
                    res[key]["ticks_per_step_" + form] = sum(mix.get(t, 0) * res["costs"][form][t] for t in mix)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        from pmc_profile import engine_hash
        res["engine_sha"] = engine_hash()
    except Exception:
        pass
    print(json.dumps(res, indent=1))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
