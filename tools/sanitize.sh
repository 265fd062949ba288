#!/usr/bin/env bash
# Build the service binaries with sanitizers and run the process-level integration
# tests against them (host code only; GPU sanitizers are not available on this pool).
#   tools/sanitize.sh asan|ubsan|tsan [pytest args]
# Component logs are kept under build-<preset>/logs; any sanitizer report fails the run.
set -uo pipefail
cd "$(dirname "$0")/.."
preset=${1:-asan}
cmake --preset "$preset" >/dev/null || exit 1
ninja -C "build-$preset" -j "${JOBS:-8}" controller admission synchronizer node-agent kube-lite || exit 1
logs="$PWD/build-$preset/logs"
rm -rf "$logs"
export BGC_BIN_DIR="$PWD/build-$preset/bin" BGC_CLUSTER_LOGDIR="$logs"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1 suppressions=$PWD/tools/tsan.supp"
python3 -m pytest tests/integration -q -p no:cacheprovider "${@:2}"
rc=$?
if grep -l "Sanitizer\|runtime error:" "$logs"/*/*.log 2>/dev/null; then
  echo "sanitizer reports found (files above)"
  exit 1
fi
exit $rc
