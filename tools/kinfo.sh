#!/bin/bash
# Register / LDS / spill figures of the engine's kernels from the built object (no GPU needed).
#     tools/kinfo.sh [pattern]
set -e
B=/opt/rocm/lib/llvm/bin
O=${OBJ:-gym-eldorado_amd/build/cog_engine.hip.o}
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$O" /dev/null
$B/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/eng.co
$B/llvm-readelf --notes $T/eng.co | python3 -c '
import sys, re
pat = sys.argv[1] if len(sys.argv) > 1 else ""
cur = {}
rows = []
for line in sys.stdin:
    m = re.match(r"\s+\.(\w+):\s+(.*)", line)
    if not m: continue
    k, v = m.groups()
    if k == "name" and not v.endswith(".kd"):
        cur = {"name": v}; rows.append(cur)
    elif cur is not None and k in ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size",
                                   "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
        cur[k] = v
for r in rows:
    if pat in r["name"]:
        print("%-70s vgpr %4s agpr %4s sgpr %4s lds %6s scratch %5s spill v%s s%s" % (
            r["name"][:70], r.get("vgpr_count"), r.get("agpr_count"), r.get("sgpr_count"),
            r.get("group_segment_fixed_size"), r.get("private_segment_fixed_size"),
            r.get("vgpr_spill_count"), r.get("sgpr_spill_count")))
' "${1:-}"
rm -rf $T
