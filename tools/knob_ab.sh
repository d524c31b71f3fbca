#!/bin/bash
# Interleaved A/B of ResNet-20 tuning knobs (run from the repo root via gpurun): bash tools/knob_ab.sh -> gpurun_out/kn/
mkdir -p gpurun_out/kn
for i in 1 2 3; do
  for cfg in base LBT_TILE_ROWS1=4 LBT_WGRAD_CPW=4 LBT_WGRAD_CPW=16 LBT_WGRAD_MIN_UNITS=64; do
    if [ $cfg = base ]; then E=""; else E="$cfg"; fi
    env $E timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-roofline > gpurun_out/kn/${cfg}_$i.json 2>/dev/null || exit 1
  done
done
