#!/usr/bin/env bash
# A/B on the MI355X box's 16-CPU share: controller/synchronizer worker count at 4 and 8
# CPU ranks (gloo), to choose the harness default for multi-rank runs.
set -o pipefail
out=gpurun_out/workers_ab
mkdir -p $out
for n in 4 8; do
  for w in 16 64; do
    echo "[$(date +%T)] n=$n workers=$w"
    BGC_BENCH_CPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29700+n+w)) bench.py --gpus $n --steps 20 --warmup 3 \
      --no-tuned-phase --controller-workers $w --sync-workers $w \
      --json-out $out/n${n}_w${w}.json > $out/n${n}_w${w}.log 2>&1 || exit 1
  done
done
for f in $out/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['reconcile_p99_ms'], d['apply_to_ready_p99_ms'], d['cpu_ms_per_cr']['product_total'], d['cpu_ms_per_cr']['kube_lite'])"; done
