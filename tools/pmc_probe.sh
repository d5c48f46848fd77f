#!/bin/bash
# usage: tools/pmc_probe.sh <outdir> <layer> ...  -- three SQ counter passes over one layer's
# fwd+bwd (tools/layer_probe.py); summarise with tools/pmc_summary.py <outdir>/*/*/p_counter_collection.csv
OUT=$1; shift
mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAVE_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
P3="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FLOPS_FP32 SQ_VALU_MFMA_COEXEC_CYCLES"
for L in "$@"; do
  n=0
  for P in "$P1" "$P2" "$P3"; do
    n=$((n+1))
    timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d $OUT/$L/p$n -o p -- python tools/layer_probe.py --layer $L --iters 2 > $OUT/$L.p$n.log 2>&1 || { echo "pass $n of $L failed"; exit 1; }
  done
done
