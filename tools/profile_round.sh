#!/bin/bash
# usage: tools/profile_round.sh <outdir>  -- the judged evidence of one round on one GPU:
# GPU tests, smoke, bench line, rocprofv3 kernel stats of the bench, two PMC passes (HBM
# traffic per kernel, MI355X_MICROARCH.md: traffic = 2 * FETCH_SIZE + WRITE_SIZE KiB) and a VALU pass
# (SQ_INSTS_VALU, SQ_WAVES: the bench line's VALU-issue roof).
set -o pipefail
O=$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o p -- python bench.py --steps 10 --no-cpu-baseline --no-cfg5 --no-peaks > $O/bench_under_rocprof.json 2> $O/rocprof.err || exit 1
cp $O/kt/p_kernel_stats.csv $O/kernel_stats.csv
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cfg5 --no-peaks --no-graph > $O/pmc_f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cfg5 --no-peaks --no-graph > $O/pmc_w.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/pmc_v -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cfg5 --no-peaks --no-graph > $O/pmc_v.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/pmc_f/p_counter_collection.csv $O/pmc_w/p_counter_collection.csv $O/pmc_v/p_counter_collection.csv > $O/pmc_traffic.json
rm -rf $O/pmc_f $O/pmc_w $O/pmc_v
# the bench line again, its roofline.traffic read from the passes just taken (same sources)
CIMQ_TRAFFIC_JSON=$O/pmc_traffic.json timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_with_traffic.json 2> $O/bench_with_traffic.err || exit 1
python tools/step_breakdown.py $O/kt/p_kernel_trace.csv > $O/step_breakdown.txt
rm -f $O/kt/p_kernel_trace.csv
echo done
