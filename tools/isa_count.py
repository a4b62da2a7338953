"""Diagnostic: static instruction counts of the rollout kernel's first (lean) loop, by mnemonic.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp \
          --cuda-device-only -S -Iinclude -Igym-eldorado_amd/csrc gym-eldorado_amd/csrc/cog_engine.hip -o /tmp/eng.s
    python3 tools/isa_count.py /tmp/eng.s [SRC]

Static counts over the loop's blocks (every path once): a proxy for the step's issue cost, which
the PMC passes measure (tools/pmc_profile.py)."""
import collections
import re
import sys


def loop_blocks(txt, sym):
    start = txt.index(sym + ":")
    end = txt.index("s_endpgm", start)
    lines = txt[start:end].split("\n")
    header = None
    cur, keep, out = None, False, []
    for ln in lines:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):.*?(?:;\s*(.*))?$", ln)
        if m:
            note = ln.split(";", 2)[-1] if ln.count(";") >= 1 else ""
            if header is None and "=>This Loop Header: Depth=1" in ln:
                header = re.match(r"^\.LBB(\d+_\d+)", ln).group(1)
            keep = header is not None and (f"BB{header}" in ln or "=>This Loop Header" in ln and f"BB{header}" in ln
                                           or ln.startswith(f".LBB{header}:"))
            if keep and header is not None and "Depth=1" not in ln and f"Parent Loop BB{header}" not in ln \
                    and not ln.startswith(f".LBB{header}:"):
                keep = False
            continue
        if keep:
            out.append(ln.strip())
    return out


def main():
    path = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else "0"
    txt = open(path).read()
    sym = f"_ZN3cog13k_env_rolloutILi{src}ELi64EEEvNS_8DevStateEiPjPh"
    body = loop_blocks(txt, sym)
    c = collections.Counter()
    for ln in body:
        if not ln or ln.startswith((".", ";")):
            continue
        c[ln.split()[0]] += 1
    cls = collections.Counter()
    for k, v in c.items():
        key = ("valu" if k.startswith("v_") else "salu" if k.startswith("s_") and not k.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_load", "s_buffer")) else
               "branch" if k.startswith(("s_cbranch", "s_branch")) else "wait" if k.startswith("s_waitcnt") else
               "lds" if k.startswith("ds_") else "vmem" if k.startswith(("global_", "buffer_", "flat_")) else
               "smem" if k.startswith(("s_load", "s_buffer")) else "other")
        cls[key] += v
    print("loop instructions", sum(c.values()), dict(cls))
    for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 60):
        print(f"  {k:28s}{v}")


if __name__ == "__main__":
    main()
