#!/bin/bash
# Per-kernel register / spill / occupancy summary of a HIP source (gfx950),
# from the compiler's kernel-resource-usage remarks (development aid):
#   tools/regs.sh metadamage_amd/csrc/mdfit.hip [-DFLAG ...]
src=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result --cuda-device-only \
  -c "$src" -o /dev/null -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/^Function Name:/ {if (n) print line; n=$3; line=n; next}
       /^(VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes\/lane\]|Occupancy \[waves\/SIMD\]|SGPRs Spill|VGPRs Spill):/ {
         k=$0; sub(/:.*/, "", k); v=$NF; line=line "  " k "=" v}
       END {if (n) print line}' |
  sed -e 's/ScratchSize \[bytes\/lane\]/scratch/' -e 's/Occupancy \[waves\/SIMD\]/occ/' | c++filt -_ 2>/dev/null | sed 's/(.*)//'
