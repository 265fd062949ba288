set -o pipefail
OUT=gpurun_out/${OUT_NAME:-r5_trim}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python -u bench.py --report-cpu > "$OUT/bench_1.json" 2> "$OUT/bench_1.err" &&
timeout -k 10 420 python -u bench.py --report-cpu > "$OUT/bench_2.json" 2> "$OUT/bench_2.err"
