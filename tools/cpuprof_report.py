#!/usr/bin/env python3
"""Symbolize a native/core/cpuprof.cc profile and print self/inclusive hot spots.

    BGC_CPU_PROFILE=/tmp/kl.%p.prof bin/kube-lite ...      # run, then stop the process
    python3 tools/cpuprof_report.py /tmp/kl.1234.prof [--top 25] [--collapsed out.txt]

addr2line (binutils) resolves each PC against the mapped ELF file; --collapsed writes
"frame;frame;leaf count" lines for flame-graph tools.
"""
import argparse
import bisect
import collections
import subprocess
import sys


def parse(path):
    maps, stacks, header = [], [], ""
    with open(path) as f:
        header = f.readline().strip()
        assert f.readline().strip() == "maps", "not a bgc cpuprof file"
        for line in f:
            line = line.rstrip("\n")
            if line == "end maps":
                break
            parts = line.split(None, 5)
            if len(parts) < 6 or "x" not in parts[1]:
                continue
            lo, hi = (int(x, 16) for x in parts[0].split("-"))
            maps.append((lo, hi, int(parts[2], 16), parts[5]))
        for line in f:
            parts = line.split()
            if parts:
                stacks.append((int(parts[0]), [int(x, 16) for x in parts[1:]]))
    maps.sort()
    return header, maps, stacks


def symbolize(maps, pcs):
    starts = [m[0] for m in maps]
    by_file = collections.defaultdict(list)
    where = {}
    for pc in pcs:
        i = bisect.bisect_right(starts, pc) - 1
        if i < 0 or pc >= maps[i][1]:
            where[pc] = None
            continue
        lo, _, off, path = maps[i]
        rel = pc - lo + off
        where[pc] = (path, rel)
        by_file[path].append(rel)
    names = {}
    for path, rels in by_file.items():
        rels = sorted(set(rels))
        short = path.rsplit("/", 1)[-1]
        try:
            out = subprocess.run(["addr2line", "-f", "-C", "-e", path] + [hex(r) for r in rels],
                                 capture_output=True, text=True, timeout=300).stdout.split("\n")
        except (OSError, subprocess.TimeoutExpired):
            out = []
        for k, r in enumerate(rels):
            fn = out[2 * k] if 2 * k < len(out) else "??"
            names[(path, r)] = fn if fn and fn != "??" else f"{short}+{r:#x}"
    return {pc: ("[unknown]" if w is None else names.get(w, "??")) for pc, w in where.items()}


def simplify(fn):
    # drop argument lists and template noise for readable tables
    depth, out = 0, []
    for ch in fn:
        if ch in "(<":
            if depth == 0:
                out.append("(…)" if ch == "(" else "<…>")
            depth += 1
        elif ch in ")>":
            depth = max(0, depth - 1)
        elif depth == 0:
            out.append(ch)
    return "".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("profile")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--collapsed", default="")
    ap.add_argument("--full-names", action="store_true")
    a = ap.parse_args()
    header, maps, stacks = parse(a.profile)
    pcs = {pc for _, st in stacks for pc in st}
    sym = symbolize(maps, pcs)
    name = (lambda pc: sym[pc]) if a.full_names else (lambda pc: simplify(sym[pc]))
    total = sum(c for c, _ in stacks)
    self_c, incl_c = collections.Counter(), collections.Counter()
    for c, st in stacks:
        frames = [name(pc) for pc in st]
        self_c[frames[0]] += c
        for fn in set(frames):
            incl_c[fn] += c
    print(f"{header}  total={total}")
    print(f"\n{'self%':>7} {'samples':>8}  function")
    for fn, c in self_c.most_common(a.top):
        print(f"{100.0 * c / total:7.2f} {c:8d}  {fn}")
    print(f"\n{'incl%':>7} {'samples':>8}  function")
    for fn, c in incl_c.most_common(a.top):
        print(f"{100.0 * c / total:7.2f} {c:8d}  {fn}")
    if a.collapsed:
        agg = collections.Counter()
        for c, st in stacks:
            agg[";".join(name(pc) for pc in reversed(st))] += c
        with open(a.collapsed, "w") as f:
            for k, c in agg.most_common():
                f.write(f"{k} {c}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
