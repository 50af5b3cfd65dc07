#!/bin/bash
# Per-kernel register use and spills of one HIP source (gfx950): tools/regs.sh <file.hip> [filter]
src=$1; filt=${2:-.}
cd "$(dirname "$src")" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$(git rev-parse --show-toplevel)/include" \
  -c "$(basename "$src")" -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name/{n=$NF} /remark:     VGPRs:/{v=$NF} /AGPRs:/{a=$NF} /SGPRs Spill/{s=$NF} /VGPRs Spill/{print n, "v="v, "a="a, "sspill="s, "vspill="$NF}' |
  grep -E "$filt"
rm -f /tmp/regs_$$.o
