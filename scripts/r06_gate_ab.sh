#!/bin/bash
# A/B of read-first packs whose stores wait for every workgroup's loads (this tree) against the
# tree in ./ab_base (a git worktree of the commit before, built; stores right after the
# workgroup's own loads): the read-signal tests on this
# tree, then the bench interleaved, three runs each.  Output under gpurun_out/gate_ab/.
out=gpurun_out/gate_ab
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_read_signal.py tests/test_gpu_dataflow.py -k "read_signal or rewritten" \
  > $out/tests.log 2>&1 || { tail -5 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2 3; do
  for t in base gate; do
    if [ $t = base ]; then d=ab_base; else d=.; fi
    (cd $d && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > /tmp/b_$t.json 2>/dev/null) || exit 1
    python - "$t" "$r" /tmp/b_$t.json >> $out/ab.jsonl <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[3]) if l.startswith("{")][-1]
print(json.dumps({"tree": sys.argv[1], "round": int(sys.argv[2]), "value": d["value"],
                  "frac": d["roofline"]["frac"], "sync": d["sync_send"],
                  "sync_4mb": d.get("sync_send_4mb"), "c3": d["c3"]["frac"]}))
PY
    tail -1 $out/ab.jsonl
  done
done
