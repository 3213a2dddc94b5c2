#!/bin/bash
# Interrupts of the GPU's IRQ lines (amdgpu) across a Python 4 MiB throughput run, with the
# command processor's completion signals (default) and without (DORA_GPU_AQL_CP_SIGNAL=0): does a
# CP-signalled pack cost the host an interrupt?   usage: bash scripts/irq_probe.sh <out dir>
set -o pipefail
out=${1:-gpurun_out/irq}
mkdir -p "$out"
irqs() { grep -i amdgpu /proc/interrupts | awk '{s=0; for(i=2;i<=NF;i++) if ($i ~ /^[0-9]+$/) s+=$i; t+=s} END {print t+0}'; }
for cfg in on off; do
  if [ $cfg = off ]; then export DORA_GPU_AQL_CP_SIGNAL=0; else unset DORA_GPU_AQL_CP_SIGNAL; fi
  a=$(irqs)
  timeout -k 10 120 python -u scripts/py_tp.py --sizes 4194304 --n 20000 > "$out/tp_$cfg.json" 2> "$out/tp_$cfg.err" || exit 1
  b=$(irqs)
  echo "{\"cfg\": \"$cfg\", \"amdgpu_irqs\": $((b - a)), \"msgs\": 20000}" >> "$out/irq.jsonl"
done
grep -i amdgpu /proc/interrupts | head -3 > "$out/lines.txt" || true
echo ok
