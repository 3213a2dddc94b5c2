#!/bin/bash
# HBM traffic of the CP-signalled 4 MiB packs (Python ladder shape): FETCH_SIZE and WRITE_SIZE in
# separate passes (they cannot share one on gfx950).   usage: bash scripts/pmc_4mb.sh <out dir>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python scripts/py_tp.py --sizes 4194304 --n 2000 > "$out/fetch_tp.json" 2> "$out/fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python scripts/py_tp.py --sizes 4194304 --n 2000 > "$out/write_tp.json" 2> "$out/write.err"
echo done
