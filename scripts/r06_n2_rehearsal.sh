#!/bin/bash
# The driver's N=2 bench command rehearsed on one GPU (DORA_BENCH_GPUS=1: both ranks' dataflows
# on GPU 0 and, pinned by L3 domain, on one 16-CPU share), then the N=1 command on the same box.
# Two dataflows' processes need more than the GPU's 24 compute queues unless HIP keeps to one
# queue per process, hence the default N2_ENV.
out=gpurun_out/${1:-r6n2}
N2_ENV=${N2_ENV-GPU_MAX_HW_QUEUES=1}
mkdir -p $out
env DORA_BENCH_GPUS=1 ${N2_ENV} timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 \
  --detail $out/detail_n2.json > $out/bench_n2.json 2> $out/bench_n2.err || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --detail $out/detail_n1.json \
  > $out/bench_n1.json 2> $out/bench_n1.err || exit 1
for n in n2 n1; do python3 -c "
import json
j = json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1])
d = json.load(open('$out/detail_$n.json'))
print('$n', j['value'], j['roofline']['frac'], j['sink_dropped'], j['latency_summary'], j.get('sync_send'))
print('   cpu', d.get('cpu_share'), d.get('affinity_after_init'))
"; done
