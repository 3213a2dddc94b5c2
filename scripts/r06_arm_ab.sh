#!/bin/bash
# Armed lone dispatch against the keep-awake thread, interleaved: the armed GPU
# test first, then small_lat_probe default / armed / armed without keep-awake, two rounds.
out=gpurun_out/${1:-r6arm}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_armed.py > $out/test.log 2>&1 || { tail -30 $out/test.log; exit 1; }
tail -3 $out/test.log
for r in 1 2; do
  timeout -k 10 120 python -u scripts/small_lat_probe.py --n 300 >> $out/default.jsonl 2>>$out/err.log || exit 1
  timeout -k 10 120 python -u scripts/small_lat_probe.py --n 300 --armed >> $out/armed.jsonl 2>>$out/err.log || exit 1
  timeout -k 10 120 python -u scripts/small_lat_probe.py --n 300 --armed --keep-awake-us 0 >> $out/armed_nowarm.jsonl 2>>$out/err.log || exit 1
done
for f in default armed armed_nowarm; do echo "== $f"; python -c "
import json
for l in open('$out/$f.jsonl'):
    r=json.loads(l)
    if 'case' in r: print(r['case'], r['latency_p50_us'], r['latency_p99_us'], r.get('incl_send_p50_us'), (r.get('stages_p50_us') or {}).get('gpu_dispatch'), r.get('armed'))
"; done
