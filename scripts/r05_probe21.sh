#!/bin/bash
# Round-5 probes, twenty-first set: the headline region's first send (timed_region.first_send_us,
# ~6 us against ~1.3 for the next ones) split into its phases (DORA_BENCH_FIRST_PHASES=1, which
# costs one call inside the region), three runs of the headline alone.
# usage: bash scripts/r05_probe21.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2 3; do
  DORA_BENCH_FIRST_PHASES=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-ladder \
    --no-c3 --no-cpu-baseline --detail "$out/d_$r.json" > "$out/b_$r.json" 2> "$out/e_$r.log"
done
echo done
