#!/bin/bash
# Interleaved A/B of ResNet-50 launch knobs (run from the repo root via gpurun): bash tools/knob_ab_r50.sh -> gpurun_out/kn50/
mkdir -p gpurun_out/kn50
for i in 1 2; do
  for cfg in base LBT_CHAIN_BLOCKS=4096 LBT_BWD_WGS=2048 LBT_STEM_WIDE_WGS=768; do
    if [ $cfg = base ]; then E=""; else E="$cfg"; fi
    env $E timeout -k 10 200 python bench.py --workload resnet50 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline \
      > gpurun_out/kn50/${cfg}_$i.json 2>/dev/null || exit 1
    echo "$cfg $i done"
  done
done
