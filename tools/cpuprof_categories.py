#!/usr/bin/env python3
"""Group a controller CPU profile (the .collapsed output of tools/cpuprof_report.py) into
the stages of its work: applies (TLS write/read, request building, JSON), reconcile
planning and checks, watch streams (read, parse, cache, queue) and the worker queue.

    tools/cpuprof_categories.py profiles/controller_cpu_r4/cpuprof_final/controller.collapsed [--top N]
"""
import argparse
import collections


def category(frames):
    s = ";".join(frames)
    if "Reconciler::apply_child" in s:
        if "TlsStream::write_all" in s:
            return "apply: tls write"
        if "TlsStream::read_some" in s or "Reader::fill" in s:
            return "apply: tls read"
        if "build_request" in s:
            return "apply: build_request"
        if "json::" in s:
            return "apply: json"
        return "apply: other"
    if "Reconciler::reconcile" in s:
        for key, name in (("desired_children", "plan"), ("up_to_date", "up_to_date"), ("fresh", "fresh"),
                          ("log::", "log")):
            if key in s:
                return "reconcile: " + name
        return "reconcile: other"
    if "Watcher::run" in s:
        if "next_line" in s or "StreamingResponse::pull" in s:
            return "watch: stream read"
        if "json::" in s and "Store::apply" not in s:
            return "watch: parse"
        for key, name in (("Store::apply", "cache"), ("is_own_write", "own-write check"), ("WorkQueue", "queue"),
                          ("forget", "forget")):
            if key in s:
                return "watch: " + name
        return "watch: other"
    if "WorkQueue" in s:
        return "queue (workers)"
    if "log::" in s:
        return "log"
    return "other: " + (frames[-1] if frames else "")


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("collapsed")
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    cats = collections.Counter()
    total = 0
    with open(args.collapsed) as f:
        for line in f:
            stack, n = line.rstrip("\n").rsplit(" ", 1)
            cats[category(stack.split(";"))] += int(n)
            total += int(n)
    print(f"samples {total}")
    for k, v in cats.most_common(args.top):
        print(f"{100 * v / total:5.1f}% {k}")


if __name__ == "__main__":
    main()
