#!/usr/bin/env bash
# Sanitizer runs (host code only; GPU sanitizers are not available on this pool).
#   tools/sanitize.sh asan|ubsan|tsan [pytest args]
#       builds the service binaries with the sanitizer and runs the process-level
#       integration tests against them; component logs are kept under
#       build-<preset>/logs and any sanitizer report fails the run.  ASan runs with
#       LeakSanitizer on (detect_leaks=1): the services exit gracefully on SIGTERM, so
#       every allocation still live at exit is reported.
#   tools/sanitize.sh asan-py [pytest args]
#       the pybind11 module built with ASan+UBSan, preloaded into CPython, under the
#       unit tests (every C++ unit the bindings expose); leak records that involve this
#       repository's code fail the run (tools/lsan_filter.py: CPython's own end-of-life
#       allocations are not ours).  test_parallel.py is skipped: it forks torch/gloo
#       workers, no native code of ours.
set -uo pipefail
cd "$(dirname "$0")/.."
mode=${1:-asan}
preset=$mode
[ "$mode" = asan-py ] && preset=asan
cmake --preset "$preset" >/dev/null || exit 1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export LSAN_OPTIONS="suppressions=$PWD/tools/lsan.supp:print_suppressions=0"
if [ "$mode" = asan-py ]; then
  ninja -C "build-$preset" -j "${JOBS:-8}" _native || exit 1
  logs="$PWD/build-$preset/pylogs"
  rm -rf "$logs" && mkdir -p "$logs"
  mod=$(ls "$PWD"/build-$preset/py/_native*.so)
  # libstdc++ must be preloaded too, or ASan cannot find the real __cxa_throw
  LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libstdc++.so)" \
  ASAN_OPTIONS="detect_leaks=1:log_path=$logs/asan" LSAN_OPTIONS="$LSAN_OPTIONS:exitcode=0" BGC_NATIVE_MODULE="$mod" \
    python3 -m pytest tests/unit -q -p no:cacheprovider --ignore=tests/unit/test_parallel.py "${@:2}"
  rc=$?
  if grep -l "ERROR: AddressSanitizer\|runtime error:" "$logs"/asan* 2>/dev/null; then
    echo "sanitizer errors found (files above)"
    exit 1
  fi
  python3 tools/lsan_filter.py "$logs"/asan* || exit 1
  exit $rc
fi
ninja -C "build-$preset" -j "${JOBS:-8}" controller admission synchronizer node-agent kube-lite crdgen || exit 1
logs="$PWD/build-$preset/logs"
rm -rf "$logs"
export BGC_BIN_DIR="$PWD/build-$preset/bin" BGC_CLUSTER_LOGDIR="$logs"
export ASAN_OPTIONS=${ASAN_OPTIONS:-detect_leaks=1:abort_on_error=1}
export TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1 suppressions=$PWD/tools/tsan.supp"
python3 -m pytest tests/integration -q -p no:cacheprovider "${@:2}"
rc=$?
if grep -l "Sanitizer\|runtime error:" "$logs"/*/*.log 2>/dev/null; then
  echo "sanitizer reports found (files above)"
  exit 1
fi
exit $rc
