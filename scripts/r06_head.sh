#!/bin/bash
# The final tree on one box: every GPU test, the smoke, then the driver's bench command three
# times (the HEAD distribution), details under gpurun_out/$1/.
out=gpurun_out/${1:-r6head}
bash scripts/r06_check.sh "${1:-r6head}" || exit 1
for r in 2 3 4; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --detail $out/bench_detail_$r.json \
    > $out/bench_$r.json 2> $out/bench_$r.err || exit 1
  tail -c 300 $out/bench_$r.json; echo
done
