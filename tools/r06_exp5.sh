#!/bin/bash
# round 6 (second session): the merged grad_x + grad_w launch's workgroup order (cur: grad_x first; il: interleaved;
# wf: grad_w first), per-launch times on a 16- and a 32-channel layer
set -o pipefail
mkdir -p gpurun_out/r06_exp5
CIMQ_EXP_DIR=r6exp CIMQ_EXP_VARIANTS=cur,gxw5_il,gxw5_wf timeout -k 10 300 python -u tools/kernel_experiment.py \
  --layer layer1.0.conv1 --layer layer2.1.conv1 --iters 30 > gpurun_out/r06_exp5/t.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r06_exp5/t.log
