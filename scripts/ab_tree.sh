#!/bin/bash
# A/B of the current tree against ab_old/ (a previous build), interleaved, driver bench command
# without the CPU baseline.  Output: gpurun_out/ab_{new,old}_<round>.json
for r in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=ab_old
    (cd $d && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline) \
      > gpurun_out/ab_${t}_$r.json 2> gpurun_out/ab_${t}_$r.err || exit 1
  done
done
