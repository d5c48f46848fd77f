#!/bin/bash
# usage: tools/r05_visit.sh <outdir> [sweep settings ...] -- smoke, the full GPU parity suite, then the step
# breakdown per setting (tools/r05_sweep.sh, tuning build).  Test failures (pytest exit 1) are recorded and
# the visit goes on; a fault, abort or time limit ends it.
set -o pipefail
O=${1:-gpurun_out/r05_visit}; shift
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as e; e.smoke()" > $O/smoke.log 2>&1
rc=$?
tail -3 $O/smoke.log
if [ $rc -ne 0 ]; then echo "smoke rc $rc: stopping"; exit $rc; fi
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -5 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
if grep -q "illegal memory\|Memory access fault" $O/gpu_tests.log; then echo "memory fault in the tests: stopping"; exit 1; fi
tools/r05_sweep.sh $O/sweep "$@"
