#!/bin/bash
# A/B of the merged grad_x + grad_w launch (cimq_part_gxw5.hip): the whole bench step with the tuning build
# exp/libcimq_cur.so, GXW5 off / on, alternated; then the parity tests on the product library (GXW5 on)
set -o pipefail
mkdir -p gpurun_out/gxw5
for r in 1 2; do
  for v in 0 1; do
    CIMQ_TUNE_GXW5=$v CIMQ_LIB_PATH=r6exp/libcimq_gxw5.so timeout -k 10 240 python -u bench.py --steps 60 --warmup 10 \
      > gpurun_out/gxw5/bench_${v}_$r.json 2> gpurun_out/gxw5/bench_${v}_$r.err || exit 1
    echo "gxw5=$v run $r: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'])" gpurun_out/gxw5/bench_${v}_$r.json)"
  done
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_function_lsq.py \
  tests/test_gpu_bench_composition.py tests/test_gpu_parity.py tests/test_gpu_ctx_format.py > gpurun_out/gxw5/tests.log 2>&1
rc=$?; tail -3 gpurun_out/gxw5/tests.log; exit $rc
