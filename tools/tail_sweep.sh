#!/bin/bash
# usage: tools/tail_sweep.sh "<CIMQ_TUNE_x=.. ...>" ...  -- the whole bench step under a kernel trace per
# env setting, with the tuning build (CIMQ_EXP_VARIANTS=base CIMQ_EXP_DIR=r4exp
# tools/kernel_experiment.py --build); prints the epilogue kernels' and the step's times
set -o pipefail
export CIMQ_LIB_PATH=${CIMQ_LIB_PATH:-r4exp/libcimq_base.so}
O=gpurun_out/tail_sweep
mkdir -p $O
n=0
for cfg in "$@"; do
  n=$((n+1))
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/r$n -o p -- python bench.py --steps 10 --no-cpu-baseline --no-cfg5 --no-peaks > $O/b$n.json 2> $O/e$n.log || { echo "fail $cfg"; exit 1; }
  echo "== $cfg" >> $O/index.txt
  python tools/tail_trace.py $O/r$n/p_kernel_trace.csv >> $O/index.txt
  python tools/step_breakdown.py $O/r$n/p_kernel_trace.csv | head -1 >> $O/index.txt
  rm -f $O/r$n/p_kernel_trace.csv
done
