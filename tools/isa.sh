#!/bin/bash
# Disassembly of one kernel of the built engine object (no GPU needed).
#     tools/isa.sh [kernel symbol substring] > out.s
set -e
B=/opt/rocm/lib/llvm/bin
O=${OBJ:-gym-eldorado_amd/build/cog_engine.hip.o}
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$O" /dev/null
$B/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/eng.co
SYM=$($B/llvm-readelf -s $T/eng.co | awk '$4=="FUNC"{print $8}' | grep "${1:-k_env_rollout_trio}" | head -1)
$B/llvm-objdump -d --no-show-raw-insn --disassemble-symbols="$SYM" $T/eng.co
rm -rf $T
