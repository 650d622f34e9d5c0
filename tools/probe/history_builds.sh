#!/bin/bash
# Probe builds (not product): light16 variants that no longer ship, rebuilt from the commits that had
# them into tools/ab/<name>.so for tools/determinism.py / tools/protocol_eu.py (ALBEDO_ALS_LIB=...).
#   tools/probe/history_builds.sh asm        r05's asm-form light16 (fused v_fmac_f32_dpp row_newbcast
#                                            FMAs; the pair determinism failure), commit 1823ba7^
#   tools/probe/history_builds.sh asm_nop4   the same with s_nop 4 before every asm DPP instruction
#                                            (r06 probe: still fails, so not a wait-state hazard)
#   tools/probe/history_builds.sh dm         r04's degree-specialised light16 units (-DALBEDO_L16_DM at
#                                            0b6ddfc, reverted: run-to-run non-deterministic)
#   tools/probe/history_builds.sh nanfill    the NaN-fill debug build (-DALBEDO_DEBUG_NANFILL at 0b6ddfc)
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
name=${1:?variant}
case $name in
  asm|asm_nop4) rev=1823ba7^; flags= ;;
  dm) rev=0b6ddfc; flags=-DALBEDO_L16_DM ;;
  nanfill) rev=0b6ddfc; flags=-DALBEDO_DEBUG_NANFILL ;;
  *) echo "unknown variant $name"; exit 2 ;;
esac
W=$(mktemp -d /tmp/albedo_hist_XXXX)
git -C "$ROOT" worktree add --detach "$W" "$rev" > /dev/null
trap 'git -C "$ROOT" worktree remove --force "$W"' EXIT
cd "$W/albedo_amd/csrc"
if [ "$name" = asm_nop4 ]; then
  python3 - <<'EOF'
s = open("device_common.h").read()
a = s.index("template <int M, bool NOP>\n__device__ __forceinline__ void fnmac_bc16")
b = s.index("// bc16 for a source written by asm")
s = s[:a] + '''template <int M, bool NOP>
__device__ __forceinline__ void fnmac_bc16(float& acc, float v, float w) {
  asm volatile("s_nop 4\\n\\tv_fmac_f32_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
               : "+v"(acc) : "v"(v), "v"(w), "n"(M));
}
''' + s[b:]
s = s.replace('asm volatile("s_nop 1\\n\\tv_mov_b32_dpp %0, %1 row_newbcast:%2', 'asm volatile("s_nop 4\\n\\tv_mov_b32_dpp %0, %1 row_newbcast:%2')
open("device_common.h", "w").write(s)
EOF
fi
mkdir -p "$ROOT/tools/ab"
make -j8 OUT="$ROOT/tools/ab/l16_$name.so" CXXFLAGS="-O3 -std=c++17 -fPIC -I../../include -I. --offload-arch=gfx950 -Wall -Wno-unused-function $flags"
echo "built tools/ab/l16_$name.so from $rev"
