#!/bin/bash
# r02 final evidence from the current build: bench lines (driver command, 1000 steps, C3), rocprofv3
# kernel trace + stats of the headline workload, PMC FETCH_SIZE / WRITE_SIZE passes, C3 kernel
# stats.  Everything under gpurun_out/r02final/; post-process with scripts/rocprof_region.py and
# scripts/pmc_traffic.py into profiles/r02_*.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
o=gpurun_out/r02final
mkdir -p $o
bash scripts/box_diag.sh r02final && mv gpurun_out/box_diag_r02final.txt $o/ || true
bash scripts/run_steps.sh \
 "f_bench:300:python bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json" \
 "f_bench1000:300:python bench.py --steps 1000 --no-cpu-baseline > $o/bench1000.json" \
 "f_c3:300:python bench.py --workload c3 --no-cpu-baseline > $o/c3.json" \
 "f_prof:300:rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python bench.py --no-ladder --no-cpu-baseline --steps 200 --warmup 20 > $o/prof_run.json" \
 "f_fetch:120:timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/pmc_fetch -o run -- python bench.py --no-cpu-baseline --no-ladder --steps 40 --warmup 5 > $o/pmc_fetch.json" \
 "f_write:120:timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/pmc_write -o run -- python bench.py --no-cpu-baseline --no-ladder --steps 40 --warmup 5 > $o/pmc_write.json" \
 "f_c3fetch:120:timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/c3pmc_fetch -o run -- python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 40 --warmup 5 > $o/c3pmc_fetch.json" \
 "f_c3write:120:timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/c3pmc_write -o run -- python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 40 --warmup 5 > $o/c3pmc_write.json" \
 "f_c3prof:300:rocprofv3 --kernel-trace --stats --output-format csv -d $o/c3prof -o run -- python bench.py --workload c3 --no-ladder --no-cpu-baseline --steps 1000 > $o/c3prof_run.json"
