#!/bin/bash
# usage: tools/sweep.sh <layer> "<CIMQ_TUNE_x=.. ...>" ...   -- kernel-trace one layer per env setting
# (launch-shape knobs exist only in a -DCIMQ_TUNING build: tools/kernel_experiment.py --build
#  makes exp/libcimq_base.so, which this script loads)
export CIMQ_LIB_PATH=${CIMQ_LIB_PATH:-exp/libcimq_base.so}
L=$1; shift
mkdir -p gpurun_out/sweep
n=0
for cfg in "$@"; do
  n=$((n+1))
  env $cfg timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sweep/r$n -o p -- python tools/layer_probe.py --layer $L --iters 3 > /dev/null 2>&1 || echo "fail $cfg"
  echo "== $cfg" >> gpurun_out/sweep/index.txt
  python tools/trace_cimq.py gpurun_out/sweep/r$n/p_kernel_trace.csv >> gpurun_out/sweep/index.txt
done
