#!/bin/bash
# one build -> GPU iteration (round 5): a subset (or all) of the GPU parity suite, the smoke, the bench
# line (no extras) and a kernel trace of the bench with its per-step breakdown
# usage: tools/r05_iter.sh <outdir> [pytest -k expression]
set -o pipefail
O=${1:-gpurun_out/r05}
K=${2:-}
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
fi
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-cfg5 --no-peaks > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o p -- python bench.py --steps 10 --no-cpu-baseline --no-cfg5 --no-peaks > $O/bench_under_rocprof.json 2> $O/rocprof.err || exit 1
python tools/step_breakdown.py $O/kt/p_kernel_trace.csv > $O/step_breakdown.txt
rm -f $O/kt/p_kernel_trace.csv
cat $O/step_breakdown.txt | head -25
echo done
