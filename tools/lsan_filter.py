"""Report only the LeakSanitizer records that involve this repository's native code.

The pybind11 unit tests run under ASan inside CPython (tools/sanitize.sh asan-py), whose
interpreter, numpy and protobuf intentionally keep memory until exit; LSan reports those
too.  A record counts when any frame of its allocation stack is in native/ sources or the
_native module.  Usage: lsan_filter.py <log files...>; exit status 1 when any remain."""
import re
import sys

OURS = re.compile(r"/native/(core|kube|crd|admission|controller|sync|gpu|apiserver|bench|python)/|_native\.cpython")


def records(text):
    cur = []
    for line in text.splitlines():
        if line.startswith(("Direct leak", "Indirect leak")):
            if cur:
                yield cur
            cur = [line]
        elif cur and line.strip().startswith("#"):
            cur.append(line)
        elif cur and not line.strip():
            yield cur
            cur = []
    if cur:
        yield cur


def main(paths):
    found = 0
    for p in paths:
        for rec in records(open(p, errors="replace").read()):
            if any(OURS.search(l) for l in rec[1:]):
                found += 1
                print(f"== {p}")
                print("\n".join(rec[:25]))
    print(f"{found} leak record(s) in native code", file=sys.stderr)
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
