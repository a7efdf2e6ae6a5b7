#!/bin/bash
# VGPRs / spills / occupancy of the trace kernels for each compile-time A/B of round 5
# (CPU only: hipcc -Rpass-analysis=kernel-resource-usage).  usage: kres_variants.sh > profiles/r05/kres_variants.txt
cd "$(dirname "$0")/../.."
V=(
 "default|"
 "binary BLAS (ab_bvh4)|-DPT_GF_BVH4=0 -DPT_BVH_BVH4=0"
 "near/far off (ab_nearfar; switch removed with the count-free node step)|-DPT_NEARFAR=0"
 "node step 4 (ab_nodestep4_bvh)|-DPT_NODE_STEP=4"
 "node step 6|-DPT_NODE_STEP=6"
 "node step 12|-DPT_NODE_STEP=12"
 "lane minimum 4|-DPT_NODE_MINLANES=4"
 "lane minimum 16|-DPT_NODE_MINLANES=16"
 "one-pipeline node step 8|-DPT_NODE_STEP_1P=8"
 "k_trace_bvh 5 waves/SIMD|-DPT_BVH_MINWAVES=5"
 "k_trace_gf 5 waves/SIMD|-DPT_GF_MINWAVES=5"
 "fast certificate alone (ab_walk)|-DPT_CERT_MODE=2"
 "walk weight 16 (ab_walk)|-DPT_WALK_W=16"
 "leaf weight 2 (ab_weights4)|-DPT_LEAF_W=2"
 "select weight 6 (ab_weights4)|-DPT_SEL_W=6"
)
i=0
for v in "${V[@]}"; do
  name=${v%%|*}; flags=${v#*|}
  ( bash scripts/kres.sh $flags | grep k_trace > /tmp/kres/$i.txt; echo "$name|$flags" > /tmp/kres/$i.name ) &
  i=$((i+1)); if (( i % 6 == 0 )); then wait; fi
done
wait
echo "# trace-kernel resources per compile-time variant (gfx950, hipcc -Rpass-analysis=kernel-resource-usage)"
for ((j=0; j<i; j++)); do
  echo "== $(cat /tmp/kres/$j.name)"
  sed -e 's/^_Z[0-9]*//' /tmp/kres/$j.txt
done
