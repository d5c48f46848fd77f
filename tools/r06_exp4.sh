#!/bin/bash
# round 6 (second session): the fused grad_x loop unrolled by two, c1's fences every second slice, against cur
set -o pipefail
mkdir -p gpurun_out/r06_exp4
CIMQ_EXP_DIR=r6exp CIMQ_EXP_VARIANTS=cur,f_cbu2,c1_sb2 timeout -k 10 300 python -u tools/kernel_experiment.py \
  --layer conv1 --layer layer3.1.conv1 --iters 30 > gpurun_out/r06_exp4/t.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r06_exp4/t.log
