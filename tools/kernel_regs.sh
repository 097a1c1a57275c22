#!/bin/bash
# VGPR / SGPR / spill counts of the kernels in one object file's gfx950 code object:
# tools/kernel_regs.sh genomics-gpu_amd/build/dispatch.o [name-filter]
set -eu
obj=$1; filt=${2:-}
d=$(mktemp -d)
L=/opt/rocm/lib/llvm/bin
$L/llvm-objcopy --dump-section=.hip_fatbin=$d/fat.bin "$obj"
$L/clang-offload-bundler --unbundle --type=o --input=$d/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$d/d.co
$L/llvm-readelf --notes $d/d.co | awk -v f="$filt" '
  /\.name:/ {name=$2} /\.vgpr_count:/ {v=$2} /\.sgpr_count:/ {s=$2}
  /\.vgpr_spill_count:/ {vs=$2; if (f == "" || index(name, f)) printf "%-90s vgpr=%s sgpr=%s vspill=%s\n", substr(name,1,90), v, s, vs}'
rm -rf $d
