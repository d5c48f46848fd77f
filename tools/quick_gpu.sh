#!/bin/bash
# usage: tools/quick_gpu.sh <outdir> [pytest -k expr] -- one kernel-change iteration on the GPU box:
# the GPU parity tests (optionally a subset), the bench line, and a rocprofv3 kernel trace of the
# bench with its per-step kernel breakdown (tools/step_breakdown.py)
set -o pipefail
O=$1
K=${2:-}
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1 || exit 1
else
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o p -- python bench.py --steps 10 --no-cpu-baseline --no-cfg5 --no-peaks > $O/bench_under_rocprof.json 2> $O/rocprof.err || exit 1
python tools/step_breakdown.py $O/kt/p_kernel_trace.csv > $O/step_breakdown.txt
rm -f $O/kt/p_kernel_trace.csv
echo done
