#!/usr/bin/env bash
# Interleaved A/B of the load driver's open-loop threads (128 default against 24) on a GPU box:
# four pairs of default bench runs; results in gpurun_out/r6_drvthreads/ (profiles/r6_drvthreads/).
set -o pipefail
OUT=gpurun_out/r6_drvthreads; mkdir -p $OUT
for i in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py > $OUT/def_$i.json 2> $OUT/def_$i.err || exit $?
  timeout -k 10 300 python -u bench.py --latency-workers 24 > $OUT/w24_$i.json 2> $OUT/w24_$i.err || exit $?
  echo "pair $i done"
done
