#!/bin/bash
# The inline / BAR small-message tail, traced (scripts/inline_tail_probe.py), twice on one box.
out=gpurun_out/${1:-r6tail}
mkdir -p $out
timeout -k 10 300 python -u scripts/inline_tail_probe.py --sizes 8,4096 --n 2000 --out $out/a > $out/a.log 2>&1 && \
timeout -k 10 300 python -u scripts/inline_tail_probe.py --sizes 8,4096 --n 2000 --out $out/b > $out/b.log 2>&1
echo rc=$?
cat /proc/loadavg
