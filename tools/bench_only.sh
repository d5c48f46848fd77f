set -o pipefail
O=$1
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o p -- python bench.py --steps 10 --no-cpu-baseline --no-cfg5 --no-peaks > $O/bench_under_rocprof.json 2> $O/rocprof.err || exit 1
python tools/step_breakdown.py $O/kt/p_kernel_trace.csv > $O/step_breakdown.txt
rm -f $O/kt/p_kernel_trace.csv
