#!/usr/bin/env bash
# GPU-box rehearsal of the driver's bench runs: N=1 on the MI355X (twice), then 2/4/8
# ranks with BGC_BENCH_CPU=1 (gloo, ranks do not touch the card) to see how the whole-job
# value moves with rank count on this box's CPU share.  Results: gpurun_out/scale/.
set -o pipefail
out=gpurun_out/scale
mkdir -p $out
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 40 --warmup 3 --report-cpu --json-out $out/n1_$i.json > $out/n1_$i.log 2>&1 || exit 1
done
for n in 2 4 8; do
  BGC_BENCH_CPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 20 --warmup 3 \
    --json-out $out/cpu_n$n.json > $out/cpu_n$n.log 2>&1 || exit 1
done
