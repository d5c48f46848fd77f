#!/bin/bash
# round 6 (second session): grid knobs of the merged grad_x + grad_w launch (GX5_GRID: grad_x workgroups, GW5_BLOCKS:
# grad_w workgroups) on the whole bench step, tuning build of the committed sources, alternated
set -o pipefail
mkdir -p gpurun_out/r06_grid
run() {  # name, env...
  local n=$1; shift
  env "$@" CIMQ_LIB_PATH=r6exp/libcimq_base.so timeout -k 10 240 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline \
    --no-cfg5 --no-peaks > gpurun_out/r06_grid/$n.json 2> gpurun_out/r06_grid/$n.err || exit 1
  echo "$n $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4))" gpurun_out/r06_grid/$n.json)"
}
if [ "$1" = "3" ]; then  # the forward's grid (FWD5_GRID: workgroups per output-block group; NOB2: two output blocks per
  # 1024-thread workgroup), with grad_x's 256 workgroups as the sources now default to
run f_d1 CIMQ_TUNE_GX5_GRID=256
run f_g384 CIMQ_TUNE_GX5_GRID=256 CIMQ_TUNE_FWD5_GRID=384
run f_g512 CIMQ_TUNE_GX5_GRID=256 CIMQ_TUNE_FWD5_GRID=512
run f_nob1 CIMQ_TUNE_GX5_GRID=256 CIMQ_TUNE_FWD5_NOB2=0
run f_d2 CIMQ_TUNE_GX5_GRID=256
run f_g192 CIMQ_TUNE_GX5_GRID=256 CIMQ_TUNE_FWD5_GRID=192
run f_g768 CIMQ_TUNE_GX5_GRID=256 CIMQ_TUNE_FWD5_GRID=768
run f_d3 CIMQ_TUNE_GX5_GRID=256
exit 0
fi
if [ "$1" = "2" ]; then
run d1 X=0
run gx256a CIMQ_TUNE_GX5_GRID=256
run gx192 CIMQ_TUNE_GX5_GRID=192
run gx128 CIMQ_TUNE_GX5_GRID=128
run d2 X=0
run gx256b CIMQ_TUNE_GX5_GRID=256
run gx320 CIMQ_TUNE_GX5_GRID=320
run gx384 CIMQ_TUNE_GX5_GRID=384
run d3 X=0
exit 0
fi
run def1 X=0
run gx1024 CIMQ_TUNE_GX5_GRID=1024
run gx256 CIMQ_TUNE_GX5_GRID=256
run gw1024 CIMQ_TUNE_GW5_BLOCKS=1024
run gw256 CIMQ_TUNE_GW5_BLOCKS=256
run def2 X=0
run gx768 CIMQ_TUNE_GX5_GRID=768
run gw768 CIMQ_TUNE_GW5_BLOCKS=768
run def3 X=0
