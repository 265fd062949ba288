#!/usr/bin/env bash
# Run bench.py with the native sampling profiler on every control-plane binary and write a
# symbolized report per binary:  tools/profile_bench.sh OUT_DIR [bench args...]
set -euo pipefail
cd "$(dirname "$0")/.."
out=${1:?out dir}; shift
mkdir -p "$out/raw"
out=$(cd "$out" && pwd)
rm -f "$out"/raw/*.prof
BGC_CPU_PROFILE="$out/raw/%p.prof" python3 bench.py --report-cpu --json-out "$out/bench.json" "$@" > "$out/bench.log" 2>&1
for f in "$out"/raw/*.prof; do
  bin=$(grep -m1 -o "/bin/[a-z-]*$" "$f" | head -1 | sed 's#/bin/##')
  [ -n "$bin" ] || bin=unknown
  python3 tools/cpuprof_report.py "$f" --top 30 --collapsed "$out/$bin.collapsed" > "$out/$bin.txt"
done
cat "$out/bench.json"
