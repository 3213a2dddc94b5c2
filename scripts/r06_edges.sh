#!/bin/bash
# The host-edge GPU tests alone (tests/test_gpu_host_edges.py, test_gpu_host_paths.py).
out=gpurun_out/${1:-r6edges}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_host_edges.py tests/test_gpu_host_paths.py tests/test_gpu_aql_slots.py > $out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "p50|passed|failed|Error" $out/tests.log | tail -12
exit $rc
