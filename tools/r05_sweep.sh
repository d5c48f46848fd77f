#!/bin/bash
# usage: tools/r05_sweep.sh <outdir> "<CIMQ_TUNE_x=.. ...>" ...  -- round 5 A/B of the new kernels: the whole
# bench step under a kernel trace per env setting, with the tuning build (r5tune/libcimq_tune.so:
# build.build(..., defines=["CIMQ_TUNING"])); per setting the step breakdown (tools/step_breakdown.py)
set -o pipefail
export CIMQ_LIB_PATH=${CIMQ_LIB_PATH:-r5tune/libcimq_tune.so}
O=$1
shift
mkdir -p $O
n=0
for cfg in "$@"; do
  n=$((n+1))
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/r$n -o p -- python bench.py --steps 10 --no-cpu-baseline --no-cfg5 --no-peaks > $O/b$n.json 2> $O/e$n.log || { echo "fail $cfg"; tail -20 $O/e$n.log; exit 1; }
  echo "== $cfg" >> $O/index.txt
  python tools/step_breakdown.py $O/r$n/p_kernel_trace.csv >> $O/index.txt
  rm -f $O/r$n/p_kernel_trace.csv
done
cat $O/index.txt
