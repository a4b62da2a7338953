"""Static instruction count of the outermost loop of a wave's region in an llvm-objdump listing
(diagnostic: tools/isa.sh output).  Spin loops (those containing s_sleep) are excluded.
    python tools/loopcount.py listing.s FIRST_LINE LAST_LINE"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
lo, hi = int(sys.argv[2]), int(sys.argv[3])
ins = []
for n in range(lo - 1, min(hi, len(lines))):
    m = re.match(r"\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", lines[n])
    if m:
        ins.append((int(m.group(3), 16), m.group(1), m.group(2)))
addr_idx = {a: k for k, (a, _, _) in enumerate(ins)}
loops = []
for k, (a, op, args) in enumerate(ins):
    if op.startswith("s_branch") or op.startswith("s_cbranch"):
        m = re.search(r"(0x[0-9a-f]+|[0-9a-f]{6,})", args)
        t = re.search(r"<[^>]*\+0x([0-9a-f]+)>", args)
        if t is None:
            continue
tgt = []
for k, (a, op, args) in enumerate(ins):
    if op.startswith(("s_branch", "s_cbranch")):
        m = re.search(r"(-?\d+)$", args.strip())
        if m:
            off = int(m.group(1))
            off = off - 65536 if off > 32767 else off
            dst = a + 4 + off * 4
            if dst < a and dst in addr_idx:
                tgt.append((addr_idx[dst], k))
spins = [(s, e) for s, e in tgt if e - s < 60 and any(op == "s_sleep" for _, op, _ in ins[s:e + 1])]
outer = max((e - s, s, e) for s, e in tgt if (s, e) not in spins) if tgt else None
print("backward branches:", len(tgt), "spin loops:", len(spins))
if outer:
    _, s, e = outer
    body = [x for j, x in enumerate(ins[s:e + 1], s) if not any(ss <= j <= ee for ss, ee in spins)]
    c = collections.Counter("v" if op.startswith("v_") else "s" if op.startswith("s_") else
                            "ds" if op.startswith("ds_") else "mem" for _, op, _ in body)
    print("outer loop: %d instructions (spin loops excluded)" % len(body), dict(c))
    print(collections.Counter(op for _, op, _ in body).most_common(25))
    print("outer loop addresses: %x .. %x" % (ins[s][0], ins[e][0]))
