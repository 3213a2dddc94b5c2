mkdir -p gpurun_out/r6b
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_host_edges.py tests/test_gpu_host_paths.py -s > gpurun_out/r6b/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 gpurun_out/r6b/tests.log
if [ $rc -eq 0 ]; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --detail gpurun_out/r6b/bench_detail.json > gpurun_out/r6b/bench.json 2> gpurun_out/r6b/bench.err
  echo "bench rc=$?"
  tail -c 2500 gpurun_out/r6b/bench.json
fi
