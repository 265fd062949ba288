#!/usr/bin/env bash
# N=2 and N=4 rank rehearsal of the final tree on a 1-GPU box: gloo CPU ranks
# (BGC_BENCH_CPU=1, no rank touches the card); results in gpurun_out/r6_scale24/.
set -o pipefail
out=gpurun_out/r6_scale24; mkdir -p $out
for n in 2 4; do
  BGC_BENCH_CPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --report-cpu \
    --json-out $out/cpu_n$n.json > $out/cpu_n$n.log 2>&1 || exit 1
  echo "n=$n done"
done
