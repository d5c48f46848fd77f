#!/bin/bash
# round 6 (second session): c1 with its slices unrolled on the standard-mask path (cur) against base
set -o pipefail
mkdir -p gpurun_out/r06_exp3
CIMQ_EXP_DIR=r6exp CIMQ_EXP_VARIANTS=base,cur timeout -k 10 300 python -u tools/kernel_experiment.py \
  --layer conv1 --layer layer3.1.conv1 --iters 30 > gpurun_out/r06_exp3/c1.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r06_exp3/c1.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_bench_composition.py \
  tests/test_gpu_chain.py tests/test_gpu_parity.py > gpurun_out/r06_exp3/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_exp3/tests.log; exit $rc
