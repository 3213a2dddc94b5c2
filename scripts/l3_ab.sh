#!/bin/bash
# A/B of L3-domain placement (DORA_GPU_PIN_L3) on the native node ladder, interleaved runs on
# one box; CPU topology recorded alongside.  Output: gpurun_out/l3_ab.jsonl, gpurun_out/cpu.txt
mkdir -p gpurun_out
{ lscpu; grep Cpus_allowed_list /proc/self/status;
  for c in 0 1 8 16 64; do echo "cpu$c L3: $(cat /sys/devices/system/cpu/cpu$c/cache/index3/shared_cpu_list 2>/dev/null)"; done;
  ls /sys/devices/system/node | grep node; } > gpurun_out/cpu.txt 2>&1
for v in 1 0 1 0; do
  DORA_GPU_PIN_L3=$v timeout -k 10 120 python scripts/native_tp.py --sizes "${SIZES:-4096,4096000}" --n 5000 \
    | sed "s/^{/{\"pin_l3\": $v, /" >> gpurun_out/l3_ab.jsonl || exit $?
done
