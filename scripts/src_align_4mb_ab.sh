#!/bin/bash
# Python node at 4 MB: 16 rotating sources allocated at their exact size vs rounded up to 2 MiB
# (every source then starts on a 2 MiB boundary, like the slots), and one source.
# Output: gpurun_out/src_align_4mb_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/src_align_4mb_ab.jsonl
: > "$out"
for r in 1 2; do
  for spec in "16 0" "16 2097152" "1 0" "16 65536"; do
    set -- $spec
    timeout -k 10 120 python scripts/py_tp.py --sizes 4096000 --n 20000 --sources $1 --align $2 \
      | sed "s/^{/{\"sources\": $1, \"align\": $2, /" >> "$out" || exit 1
  done
done
