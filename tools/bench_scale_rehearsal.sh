#!/usr/bin/env bash
# GPU-box rehearsal of the driver's bench runs: N=1 on the MI355X, then 2/4/8 ranks with
# BGC_BENCH_CPU=1 (gloo, ranks do not touch the card) on this box's 16-CPU share, each
# with --report-cpu so the CR/s change with N can be attributed per component
# (cpu_ms_per_cr: controller / admission / synchronizer / node_agent / kube_lite /
# load_driver).  Results: $OUT (default gpurun_out/scale/); $EXTRA is appended to every
# bench.py command line (e.g. EXTRA=--no-driver-server-filter).
set -o pipefail
out=${OUT:-gpurun_out/scale}
mkdir -p $out
timeout -k 10 240 python -u bench.py --steps 30 --warmup 3 --report-cpu --no-tuned-phase $EXTRA \
  --json-out $out/n1.json > $out/n1.log 2>&1 || exit 1
for n in 2 4 8; do
  BGC_BENCH_CPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 20 --warmup 3 \
    --report-cpu --no-tuned-phase $EXTRA --json-out $out/cpu_n$n.json > $out/cpu_n$n.log 2>&1 || exit 1
done
python3 - "$out" <<'PY'
import json, sys
out = sys.argv[1]
rows = []
for n, f in ((1, "n1"), (2, "cpu_n2"), (4, "cpu_n4"), (8, "cpu_n8")):
    d = json.load(open(f"{out}/{f}.json"))
    rows.append({"n": n, "cr_s": d["value"], "reconcile_p99_ms": d["reconcile_p99_ms"],
                 "admission_p50_ms": d["admission_p50_ms"], "apply_to_ready_p99_ms": d["apply_to_ready_p99_ms"],
                 "cpu_ms_per_cr": d["cpu_ms_per_cr"], "requests_per_cr": d["apiserver_requests_per_cr"],
                 "store_lock": d["apiserver_store_lock"]})
json.dump(rows, open(f"{out}/summary.json", "w"), indent=1)
for r in rows:
    print(r["n"], r["cr_s"], r["reconcile_p99_ms"], r["cpu_ms_per_cr"])
PY
