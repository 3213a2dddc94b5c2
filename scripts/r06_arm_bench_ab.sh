#!/bin/bash
# The driver's bench command with the armed lone dispatch on and off (DORA_GPU_ARMED, A/B only),
# interleaved, two rounds; details under gpurun_out/$1/.
out=gpurun_out/${1:-r6armb}
mkdir -p $out
for r in 1 2; do
  for m in ${MODES:-1 0}; do
    DORA_GPU_ARMED=$m timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 \
      --detail $out/detail_${m}_$r.json > $out/bench_${m}_$r.json 2> $out/bench_${m}_$r.err || exit 1
    echo "armed=$m round $r"; tail -c 400 $out/bench_${m}_$r.json
  done
done
