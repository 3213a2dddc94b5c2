#!/bin/bash
# AQL queues per sending process, 4 (shipped) against 3 (DORA_GPU_AQL_QUEUES, an A/B switch of
# this measurement only, removed since), interleaved: the driver's bench command twice each.
out=gpurun_out/${1:-r6q}
mkdir -p $out
for r in 1 2; do
  for m in 4 3; do
    DORA_GPU_AQL_QUEUES=$m timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 \
      --detail $out/detail_${m}_$r.json > $out/bench_${m}_$r.json 2> $out/bench_${m}_$r.err || exit 1
    python3 -c "
import json
j = json.loads(open('$out/bench_${m}_$r.json').read().strip().splitlines()[-1])
print('queues=$m r$r', j['value'], j['roofline']['frac'], j.get('c3'), j.get('mid_us_frac'), j['latency_summary'].get('4194304'), j.get('sync_send',{}).get('us_per_msg'))
"
  done
done
