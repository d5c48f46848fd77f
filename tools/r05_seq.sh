set -o pipefail
O=gpurun_out/r05_seq
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o p -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-cfg5 --no-peaks > $O/b.json 2> $O/err.log || exit 1
python tools/step_sequence.py $O/kt/p_kernel_trace.csv > $O/seq.txt
rm -f $O/kt/p_kernel_trace.csv
cat $O/seq.txt
