#!/usr/bin/env bash
# Interleaved A/B (or A/B/C...) of the headline bench on one box, run through gpurun from
# the repo root.  Every rep runs every arm once, in order, so slow drift (clock, page
# cache, a neighbour) hits all arms alike; the summary reports the median per arm.
#
#   tools/gpu_ab.sh [-n NPROC] [-r REPS] [-o OUT] [-t SECONDS] -- NAME 'ARGS' [NAME 'ARGS' ...]
#
# ARGS are bench.py arguments; leading VAR=value words become the arm's environment.
# NPROC > 1 runs torch.distributed.run with that many ranks (the control plane on CPU
# ranks: BGC_BENCH_CPU=1, never more than the box's GPUs).  Examples (the rounds' studies):
#
#   # webhook h2 vs HTTP/1.1 at 8 ranks (profiles/archive/http2_r2)
#   tools/gpu_ab.sh -n 8 -r 2 -- h2 '--no-tuned-phase' h1 '--no-tuned-phase --apiserver-arg=--webhook-http1'
#   # metadata-only watches vs full objects (profiles/archive/metadata_watches_r2)
#   tools/gpu_ab.sh -r 3 -- meta '' full '--controller-env=CONF_METADATA_WATCHES=false'
#   # kube-lite store lock (profiles/archive/kl_store_lock_r2)
#   tools/gpu_ab.sh -n 8 -r 2 -- rw 'BGC_KL_RWLOCK=writer --no-tuned-phase' mx 'BGC_KL_RWLOCK=mutex --no-tuned-phase'
#   # glibc tcache depth (profiles/archive/tcache_ab_r1)
#   tools/gpu_ab.sh -r 2 -- t64 'GLIBC_TUNABLES=glibc.malloc.tcache_count=64 --steps 300' t7 'GLIBC_TUNABLES=glibc.malloc.tcache_count=7 --steps 300'
#   # an older build's binaries against this one (profiles/cpuprof_r3)
#   tools/gpu_ab.sh -r 3 -- base "BGC_BIN_DIR=$PWD/ab/base" cur ''
#   # worker counts
#   tools/gpu_ab.sh -n 8 -- w16 '--controller-workers 16 --sync-workers 16' w64 '--controller-workers 64 --sync-workers 64'
#
# Each run has its own time limit and the first failure ends the call.  Results:
# OUT/<name>_<rep>.json and .log, OUT/summary.json.
set -o pipefail
nproc=1; reps=3; out=gpurun_out/ab; limit=300
while getopts "n:r:o:t:" opt; do
  case $opt in
    n) nproc=$OPTARG ;; r) reps=$OPTARG ;; o) out=$OPTARG ;; t) limit=$OPTARG ;;
    *) echo "usage: $0 [-n NPROC] [-r REPS] [-o OUT] [-t SECONDS] -- NAME 'ARGS' ..." >&2; exit 2 ;;
  esac
done
shift $((OPTIND - 1))
[ "${1:-}" = "--" ] && shift
if [ $# -lt 2 ] || [ $(($# % 2)) -ne 0 ]; then echo "need NAME 'ARGS' pairs" >&2; exit 2; fi
names=(); specs=()
while [ $# -gt 0 ]; do names+=("$1"); specs+=("$2"); shift 2; done
mkdir -p "$out"
export TMPDIR=/tmp

run_arm() {  # name, rep, spec
  local name=$1 rep=$2 envs=() args=() w
  # shellcheck disable=SC2086
  for w in $3; do
    if [ ${#args[@]} -eq 0 ] && [[ $w =~ ^[A-Z_][A-Z0-9_]*= ]]; then envs+=("$w"); else args+=("$w"); fi
  done
  echo "[$(date +%T)] $name rep $rep: ${envs[*]} bench.py ${args[*]}"
  if [ "$nproc" -gt 1 ]; then
    env "${envs[@]}" BGC_BENCH_CPU=1 timeout -k 10 "$limit" python -u -m torch.distributed.run --nnodes=1 \
      --nproc-per-node "$nproc" --master-addr 127.0.0.1 --master-port $((29600 + nproc)) bench.py --gpus "$nproc" \
      --steps 20 --warmup 3 --report-cpu "${args[@]}" --json-out "$out/${name}_$rep.json" > "$out/${name}_$rep.log" 2>&1
  else
    env "${envs[@]}" timeout -k 10 "$limit" python -u bench.py --report-cpu "${args[@]}" \
      --json-out "$out/${name}_$rep.json" > "$out/${name}_$rep.log" 2>&1
  fi
}

for rep in $(seq 1 "$reps"); do
  for i in "${!names[@]}"; do
    run_arm "${names[$i]}" "$rep" "${specs[$i]}" || { rc=$?; echo "${names[$i]} rep $rep failed rc=$rc"; tail -20 "$out/${names[$i]}_$rep.log"; exit $rc; }
  done
done

python3 - "$out" "$reps" "${names[@]}" <<'PY'
import json, statistics, sys
out, reps, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
keys = ["value", "admission_p50_ms", "reconcile_p99_ms", "apply_to_ready_p99_ms"]
cpu_keys = ["admission", "controller", "kube_lite", "product_total"]
summary = {}
for name in names:
    rows = [json.load(open(f"{out}/{name}_{r}.json")) for r in range(1, reps + 1)]
    arm = {k: [d.get(k) for d in rows] for k in keys}
    for k in cpu_keys:
        arm[f"cpu_ms_per_cr.{k}"] = [(d.get("cpu_ms_per_cr") or {}).get(k) for d in rows]
    for k in ("contended_pct", "wait_s_per_s"):
        arm[f"store_lock.{k}"] = [(d.get("apiserver_store_lock") or {}).get(k) for d in rows]
    arm["admission_p99_ms"] = [d.get("admission_p99_ms") for d in rows]
    arm["apply_to_ready_p50_ms"] = [d.get("apply_to_ready_p50_ms") for d in rows]
    arm["cgroup_throttled_periods"] = [(d.get("cgroup_throttled") or {}).get("throttled_periods", 0) for d in rows]
    summary[name] = {k: {"median": statistics.median(v) if all(x is not None for x in v) else None, "all": v}
                     for k, v in arm.items()}
json.dump(summary, open(f"{out}/summary.json", "w"), indent=1)
cols = list(summary[names[0]])
print("metric".ljust(26) + "".join(n.rjust(14) for n in names))
for c in cols:
    print(c.ljust(26) + "".join(("%14.4f" % summary[n][c]["median"]) if summary[n][c]["median"] is not None else "%14s" % "-"
                                 for n in names))
PY
