#!/bin/bash
# cfg5 dense forward A/B on the GPU box: the 64-row (DENSE_FWD8=0) and 128-row (=1) threshold kernels, tuning build
set -e
mkdir -p gpurun_out/r06_d5
for v in 0 1 0 1; do
  CIMQ_EXP_DIR=r6exp CIMQ_TUNE_DENSE_FWD8=$v timeout -k 10 120 python -u tools/cfg5_probe.py base | sed "s/^/fwd8=$v /" >> gpurun_out/r06_d5/ab.log
done
