#!/bin/bash
# one build -> GPU iteration: the GPU parity suite, the bench line (no extras) and a kernel trace
set -o pipefail
O=${1:-gpurun_out/r04}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-cfg5 --no-peaks > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o p -- python bench.py --steps 10 --no-cpu-baseline --no-cfg5 --no-peaks > $O/bench_under_rocprof.json 2> $O/rocprof.err || exit 1
python tools/step_breakdown.py $O/kt/p_kernel_trace.csv > $O/step_breakdown.txt
rm -f $O/kt/p_kernel_trace.csv
echo done
