#!/bin/bash
# usage: tools/r06_sq.sh <outdir> [layer ...] -- the three SQ counter passes of tools/pmc_probe.sh over single
# ResNet-20 layers (tools/layer_probe.py, eager fwd+bwd), summarised per kernel by tools/pmc_summary.py into
# <outdir>/<layer>.sq.txt (the raw csv directories are removed)
O=${1:-gpurun_out/r06_sq}; shift
LAYERS=${@:-layer1.0.conv1 layer2.1.conv1 layer3.1.conv1 conv1 layer2.0.conv1}
mkdir -p $O
for L in $LAYERS; do
  tools/pmc_probe.sh $O $L || exit 1
  python tools/pmc_summary.py $O/$L/p*/p_counter_collection.csv > $O/$L.sq.txt || exit 1
  rm -rf $O/$L
  echo "sq $L done"
done
