#!/bin/bash
# Persistent pack-engine probe sweep (scripts/engine_probe.hip).  Output: gpurun_out/engine_ab.jsonl
mkdir -p gpurun_out
for spec in "4194304 24 4 256 16384" "4194304 24 8 128 16384" "4194304 24 2 512 8192" "4194304 32 4 256 16384" \
            "4194304 24 4 128 32768" "1048576 24 4 256 4096" "13107200 8 2 512 16384" "40960000 8 2 512 32768"; do
  set -- $spec
  timeout -k 5 30 build/engine_probe $1 5000 $2 $3 $4 $5 >> gpurun_out/engine_ab.jsonl || { rc=$?; echo "rc=$rc at $spec"; exit $rc; }
done
