#!/bin/bash
# round 6 (second session): where gx5's time goes (run as its own launch: CIMQ_TUNE_GXW5=0), per-launch times
set -o pipefail
mkdir -p gpurun_out/r06_exp6
CIMQ_TUNE_GXW5=0 CIMQ_EXP_DIR=r6exp CIMQ_EXP_VARIANTS=cur,gx5_noploop,gx5_nosync,gx5_noepi,gx5_skel,gx5_bare timeout -k 10 400 \
  python -u tools/kernel_experiment.py --layer layer1.0.conv2 --layer layer2.1.conv1 --iters 30 > gpurun_out/r06_exp6/t.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r06_exp6/t.log
