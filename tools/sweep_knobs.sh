set -o pipefail
for L in layer1.0.conv1 layer2.1.conv1 layer3.1.conv1; do
  bash tools/sweep.sh $L "CIMQ_TUNE_GW_BLOCKS=512" "CIMQ_TUNE_GW_BLOCKS=256" "CIMQ_TUNE_GW_BLOCKS=384" "CIMQ_TUNE_GW_BLOCKS=768" "CIMQ_TUNE_GW_BLOCKS=1024" "CIMQ_TUNE_GX_RB=4" "CIMQ_TUNE_GX_RB=16" || exit 1
  mv gpurun_out/sweep gpurun_out/sweep_$L
done
echo done
