#!/bin/bash
# Per-kernel resource usage (VGPRs, SGPR spills, LDS, occupancy) of renderer.hip for gfx950.
# usage: scripts/kres.sh [extra -D flags]
cd "$(dirname "$0")/../pathtracerap_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-slp-vectorize --cuda-device-only -c \
  -Rpass-analysis=kernel-resource-usage "$@" csrc/renderer.hip -o /tmp/kres.o 2>&1 | grep "remark:" |
  sed -e 's/ \[-Rpass-analysis=kernel-resource-usage\]//' -e 's/.*remark: *//' |
  awk '/^Function Name/{n=$NF} /^VGPRs:/{v=$NF} /^SGPRs Spill/{ss=$NF} /^VGPRs Spill/{vs=$NF} /^Occupancy/{o=$NF} /^LDS Size/{l=$NF; if (n ~ /k_bounce|k_trace|k_primary/) printf "%-45s vgpr=%s vgpr_spill=%s sgpr_spill=%s lds=%s occ=%s\n", n, v, vs, ss, l, o}'
