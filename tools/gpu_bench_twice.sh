set -o pipefail
OUT=gpurun_out/r5_bench1
mkdir -p "$OUT"
export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 300 python -u bench.py > "$OUT/bench_1.json" 2> "$OUT/bench_1.err"
rc=$?
echo "run_s=$(( $(date +%s) - start )) rc=$rc" > "$OUT/timing.txt"
[ $rc -eq 0 ] && start=$(date +%s) && timeout -k 10 300 python -u bench.py > "$OUT/bench_2.json" 2> "$OUT/bench_2.err"
rc=$?
echo "run2_s=$(( $(date +%s) - start )) rc=$rc" >> "$OUT/timing.txt"
cat "$OUT/timing.txt"
exit $rc
