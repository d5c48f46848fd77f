#!/bin/bash
# round 6 (second session): fused-kernel attribution / prefetch and c1 variants, per-launch times
set -o pipefail
mkdir -p gpurun_out/r06_exp2
CIMQ_EXP_DIR=r6exp CIMQ_EXP_VARIANTS=base,fold_xb4,f_pf2,f_nogx,f_nogw,f_nostage,f_nogxgw timeout -k 10 300 python -u tools/kernel_experiment.py \
  --layer layer3.1.conv1 --layer layer2.0.conv1 --iters 30 > gpurun_out/r06_exp2/fused.log 2>&1 || exit 1
CIMQ_EXP_DIR=r6exp CIMQ_EXP_VARIANTS=base,c1_ldsadd,c1_xpf,c1_both,c1_nopairs timeout -k 10 300 python -u tools/kernel_experiment.py \
  --layer conv1 --iters 30 > gpurun_out/r06_exp2/c1.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r06_exp2/fused.log gpurun_out/r06_exp2/c1.log
