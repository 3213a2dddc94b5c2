#!/bin/bash
# One GPU check of the tree: every -m gpu test, the driver's smoke, the driver's bench command.
# Output under gpurun_out/$1/ (default r6check).
out=gpurun_out/${1:-r6check}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  > $out/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -3 $out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --detail $out/bench_detail.json \
  > $out/bench.json 2> $out/bench.err
rc=$?
echo "bench rc=$rc"; tail -c 2200 $out/bench.json
exit $rc
