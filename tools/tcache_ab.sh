#!/usr/bin/env bash
# glibc tcache A/B on the MI355X box: bench.py --report-cpu at several GLIBC_TUNABLES settings,
# interleaved, twice each.  Results: gpurun_out/tcache_ab/<tag>_r<rep>.json
#   tools/tcache_ab.sh STEPS TAG=TUNABLES [TAG=TUNABLES ...]
set -e
steps=${1:?steps}; shift
mkdir -p gpurun_out/tcache_ab
for rep in 1 2; do
  for spec in "$@"; do
    tag=${spec%%=*}; tun=${spec#*=}
    GLIBC_TUNABLES="$tun" timeout -k 10 300 python -u bench.py --steps "$steps" --warmup 5 --report-cpu \
      --json-out gpurun_out/tcache_ab/${tag}_r${rep}.json > gpurun_out/tcache_ab/${tag}_r${rep}.log 2>&1
    echo "$tag rep=$rep done"
  done
done
