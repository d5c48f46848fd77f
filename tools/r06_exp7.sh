#!/bin/bash
# round 6 (second session): gx5's second K-step as a 16-deep MFMA (cur; k16all: also at two input blocks) against
# base, then the whole GPU suite on the product library
set -o pipefail
mkdir -p gpurun_out/r06_exp7
CIMQ_EXP_DIR=r6exp CIMQ_EXP_VARIANTS=base,cur,gx5_k16all timeout -k 10 300 python -u tools/kernel_experiment.py \
  --layer layer1.0.conv2 --layer layer2.1.conv1 --iters 30 > gpurun_out/r06_exp7/t.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r06_exp7/t.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_exp7/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_exp7/tests.log; exit $rc
