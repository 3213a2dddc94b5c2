export TMPDIR=/tmp
bash scripts/run_steps.sh \
 "bench:400:python bench.py > gpurun_out/bench.json" \
 "c3:300:python bench.py --workload c3 > gpurun_out/c3.json" \
 "prof:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --no-ladder --no-cpu-baseline > gpurun_out/prof_run.json" \
 "fetch:120:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --no-cpu-baseline --no-ladder --steps 40 --warmup 5" \
 "write:120:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --no-cpu-baseline --no-ladder --steps 40 --warmup 5"
