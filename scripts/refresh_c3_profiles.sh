#!/bin/bash
# C3 evidence of the current build: rocprofv3 kernel trace + stats, PMC FETCH_SIZE / WRITE_SIZE
# passes.  Under gpurun_out/r02c3/; post-process with scripts/rocprof_region.py and
# scripts/pmc_traffic.py into profiles/r02_c3_*.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/r02c3
mkdir -p $o
bash scripts/run_steps.sh \
 "c3_fetch:120:timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/c3pmc_fetch -o run -- python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 40 --warmup 5 > $o/c3pmc_fetch.json" \
 "c3_write:120:timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/c3pmc_write -o run -- python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 40 --warmup 5 > $o/c3pmc_write.json" \
 "c3_prof:300:rocprofv3 --kernel-trace --stats --output-format csv -d $o/c3prof -o run -- python bench.py --workload c3 --no-ladder --no-cpu-baseline --steps 1000 > $o/c3prof_run.json"
