#!/bin/bash
# Build libcog_hip.so of another revision's engine sources into tools/abA/ (for A/B timing on one
# box: LD_LIBRARY_PATH=tools/abA runs a tool linked against the library with the A build).
#     tools/build_abA.sh [REV]          (default HEAD)
set -e
REV=${1:-HEAD}
D=tools/abA
C="$D/gym-eldorado_amd/csrc"                           # (the ABI includes ../../include/cog.h)
rm -rf "$D" && mkdir -p "$C" "$D/include"
for f in cog_engine.hip cog_abi.cpp cog_engine.h cog_tables.h cog_rng.h; do
  git show "$REV:gym-eldorado_amd/csrc/$f" > "$C/$f"
done
for f in cog.h cog_types.h; do git show "$REV:include/$f" > "$D/include/$f"; done
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp"
/opt/rocm/bin/hipcc $FLAGS -c -I"$D/include" -I"$C" "$C/cog_engine.hip" -o "$D/engine.o"
/opt/rocm/bin/hipcc $FLAGS -c -I"$D/include" -I"$C" "$C/cog_abi.cpp" -o "$D/abi.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$D/engine.o" "$D/abi.o" -o "$D/libcog_hip.so"
rm -rf "$D"/*.o "$D/gym-eldorado_amd" "$D/include"
git rev-parse "$REV" > "$D/REV"
echo "built $D/libcog_hip.so from $(cat $D/REV)"
