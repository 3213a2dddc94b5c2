#!/bin/bash
# Read-signalled pack grid for mid sizes: at least 1 or 4 (shipped since) / 8 units of 16 B per
# lane (DORA_GPU_READ_LANE_MIN, an A/B switch of that measurement only, removed since), interleaved: the bench's synchronous 40.96 MB and 4 MiB legs.
out=gpurun_out/${1:-r6rg}
mkdir -p $out
for r in 1 2; do
  for m in 1 4 8; do
    DORA_GPU_READ_LANE_MIN=$m timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-ladder \
      --no-c3 --detail $out/detail_${m}_$r.json > $out/bench_${m}_$r.json 2> $out/bench_${m}_$r.err || exit 1
    python3 -c "
import json
j = json.loads(open('$out/bench_${m}_$r.json').read().strip().splitlines()[-1])
print('lane_min=$m r$r', j['value'], j.get('sync_send'), j.get('sync_send_4mb'))
"
  done
done
