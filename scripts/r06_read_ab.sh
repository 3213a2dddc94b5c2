#!/bin/bash
# Read-signalled synchronous packs (aql_kernels.hip dora_aql_pack1r_u4): the source-rewrite GPU
# test, then the driver's bench command twice (its `sync_send` block).  The on/off A/B of
# profiles/r06_read_signal_ab.jsonl ran this with a temporary DORA_GPU_READ_SIGNAL switch.
out=gpurun_out/${1:-r6read}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dataflow.py -k "rewritten_on_unrelated" > $out/test.log 2>&1 || { tail -40 $out/test.log; exit 1; }
grep -E "PASS|FAIL|corrupted" $out/test.log | tail -8
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --detail $out/detail_$r.json \
    > $out/bench_$r.json 2> $out/bench_$r.err || exit 1
  python -c "
import json
j = json.loads(open('$out/bench_$r.json').read().strip().splitlines()[-1])
print('round $r', j['value'], j['roofline']['frac'], j.get('sync_send'), j.get('c3'))
"
done
