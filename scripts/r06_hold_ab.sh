#!/bin/bash
# Keeping the command processor awake: the keep-awake thread (default), nothing, or one pending
# barrier-AND packet on a queue of its own (scripts/small_lat_probe.py --cp-hold), interleaved.
out=gpurun_out/${1:-r6hold}
mkdir -p $out
for r in 1 2; do
  timeout -k 10 120 python -u scripts/small_lat_probe.py --n 300 >> $out/default.jsonl 2>>$out/err.log || exit 1
  timeout -k 10 120 python -u scripts/small_lat_probe.py --n 300 --keep-awake-us 0 >> $out/off.jsonl 2>>$out/err.log || exit 1
  timeout -k 10 120 python -u scripts/small_lat_probe.py --n 300 --keep-awake-us 0 --cp-hold >> $out/hold.jsonl 2>>$out/err.log || exit 1
done
for f in default off hold; do echo "== $f"; python -c "
import json,sys
for l in open('$out/$f.jsonl'):
    r=json.loads(l); print(r['case'], r['latency_p50_us'], r['latency_p99_us'], (r.get('stages_p50_us') or {}).get('gpu_dispatch'))
"; done
# a dispatch written ahead behind a barrier-AND vs one rung after the gap (scripts/arm_probe.py)
timeout -k 10 120 python -u scripts/arm_probe.py --n 400 --gaps-us 20,200,1000 --keep-awake-us 0 > $out/arm.jsonl 2>>$out/err.log || exit 1
cat $out/arm.jsonl
