#!/bin/bash
# usage: tools/r05_combo.sh <outdir> [pytest -k expression] -- one GPU visit of round 5: the smoke (one
# production-shaped module layer on the new kernels), the GPU parity tests (a subset with -k), then the A/B
# sweep of the new kernels (tools/r05_sweep.sh).  Test failures (pytest exit 1) are recorded and the visit
# goes on; a fault, abort or time limit ends it.
set -o pipefail
O=${1:-gpurun_out/r05_combo}
K=${2:-}
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as e; e.smoke()" > $O/smoke.log 2>&1
rc=$?
tail -3 $O/smoke.log
if [ $rc -ne 0 ]; then echo "smoke rc $rc: stopping"; exit $rc; fi
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1
else
  timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
rc=$?
tail -5 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
if grep -q "illegal memory\|Memory access fault" $O/gpu_tests.log; then echo "memory fault in the tests: stopping"; exit 1; fi
tools/r05_sweep.sh $O/sweep "CIMQ_TUNE_NONE=0" "CIMQ_TUNE_FWD5=0" "CIMQ_TUNE_GW5=0" "CIMQ_TUNE_GX5=0" "CIMQ_TUNE_FUSED=0" "CIMQ_TUNE_FWD5=0 CIMQ_TUNE_GW5=0 CIMQ_TUNE_GX5=0"
