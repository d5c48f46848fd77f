#!/bin/bash
# usage: tools/pmc_cfg5.sh <outdir> -- the three SQ counter passes of tools/pmc_probe.sh over the
# BASELINE cfg5 layer (tools/cfg5_probe.py, one timed step); summarise with
# tools/pmc_summary.py <outdir>/p*/p_counter_collection.csv
OUT=$1
mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAVE_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
P3="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FLOPS_FP32 SQ_VALU_MFMA_COEXEC_CYCLES"
n=0
for P in "$P1" "$P2" "$P3"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$n -o p -- python tools/cfg5_probe.py 1 > $OUT/p$n.log 2>&1 || { echo "pass $n failed"; exit 1; }
done
