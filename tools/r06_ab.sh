#!/bin/bash
# A/B of two tuning builds (r6exp/libcimq_base.so, r6exp/libcimq_cur.so) on four layers, GW5_SP8 off / on
set -o pipefail
mkdir -p gpurun_out/r06_ab
for v in 0 1; do
  CIMQ_TUNE_GW5_SP8=$v CIMQ_EXP_DIR=r6exp CIMQ_EXP_VARIANTS=base,cur timeout -k 10 300 python -u tools/kernel_experiment.py \
    --layer layer1.0.conv1 --layer layer2.1.conv1 --layer layer2.0.conv1 --layer layer3.1.conv1 --iters 30 2>&1 \
    | grep -v amdgpu | sed "s/^/sp8=$v /" >> gpurun_out/r06_ab/t.log || exit 1
done
