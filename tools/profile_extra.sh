#!/bin/bash
# usage: tools/profile_extra.sh <outdir> -- the round's secondary evidence on one GPU: SQ counters of
# three ResNet-20 layers (tools/pmc_probe.sh), and rocprofv3 kernel tables of BASELINE cfg4 (alpha
# only and with the scale/shift ADC, tools/cfg4_probe.py) and cfg5 (tools/cfg5_probe.py)
set -o pipefail
O=$1
mkdir -p $O
bash tools/pmc_probe.sh $O/sq layer1.0.conv1 layer3.1.conv1 conv1 || exit 1
python tools/pmc_summary.py $O/sq/*/*/p_counter_collection.csv > $O/pmc_sq_counters.txt || exit 1
rm -rf $O/sq
for v in "" "--shift"; do
  n=cfg4${v:+_shift}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o p -- python tools/cfg4_probe.py $v 3 > $O/$n.log 2>&1 || exit 1
  rm -f $O/$n/p_kernel_trace.csv
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg5 -o p -- python tools/cfg5_probe.py 5 > $O/cfg5.log 2>&1 || exit 1
rm -f $O/cfg5/p_kernel_trace.csv
echo done
