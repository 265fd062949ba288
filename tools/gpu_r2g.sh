set -o pipefail
OUT=gpurun_out/r2g; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --json-out $OUT/c4.json --apiserver-arg=--webhook-h2-connections --apiserver-arg=4 > $OUT/c4.log 2>&1 &&
timeout -k 10 300 python -u bench.py --json-out $OUT/c16.json --apiserver-arg=--webhook-h2-connections --apiserver-arg=16 > $OUT/c16.log 2>&1 &&
timeout -k 10 300 python -u bench.py --json-out $OUT/c1.json > $OUT/c1.log 2>&1
