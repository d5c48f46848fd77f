#!/bin/bash
# usage: tools/r05_pmc.sh <outdir> [layer ...] -- counter passes over single ResNet-20 layers (tools/layer_probe.py):
# the three SQ passes of tools/pmc_probe.sh plus FETCH_SIZE / WRITE_SIZE, each pass its own rocprofv3 run;
# summaries in <outdir>/<layer>.sq.txt and <outdir>/<layer>.traffic.json
O=${1:-gpurun_out/r05_pmc}; shift
LAYERS=${@:-layer1.0.conv1 layer2.1.conv1}
mkdir -p $O
for L in $LAYERS; do
  tools/pmc_probe.sh $O $L || exit 1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$L/f -o p -- python tools/layer_probe.py --layer $L --iters 2 > $O/$L.f.log 2>&1 || { echo "fetch pass of $L failed"; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$L/w -o p -- python tools/layer_probe.py --layer $L --iters 2 > $O/$L.w.log 2>&1 || { echo "write pass of $L failed"; exit 1; }
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$L/t -o p -- python tools/layer_probe.py --layer $L --iters 4 > $O/$L.t.log 2>&1 || { echo "trace of $L failed"; exit 1; }
  python tools/pmc_summary.py $O/$L/p*/p_counter_collection.csv > $O/$L.sq.txt
  python tools/pmc_traffic.py $O/$L/f/p_counter_collection.csv $O/$L/w/p_counter_collection.csv > $O/$L.traffic.json
  cp $O/$L/t/p_kernel_stats.csv $O/$L.kstats.csv
  rm -rf $O/$L
done
