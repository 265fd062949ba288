"""Per-CR latency attribution for the open-loop windows.

Every process of the stack marks the moments a traced tenant passes through it
(native/core/trace.h): the load driver (scheduled arrival, create sent, create answered,
each child seen), kube-lite (each write received, webhook called/answered, committed,
response sent; each watch event written to each watcher), the admission server (review
received/answered), the controller (UserBootstrap and child events, reconcile start/end,
each apply sent/answered) and the synchronizer (UserBootstrap event, dequeue, quota PATCH
and status PUT sent/answered).  All timestamps are CLOCK_MONOTONIC, shared by every
process on the host, so the marks of one tenant join into one timeline.

For each tenant the critical path to Ready is the chain of the child seen last (usually the
RoleBinding: it waits for the status write):

    arrival -> create sent -> kube-lite received -> webhook -> committed
      -> synchronizer event -> quota PATCH committed -> status PUT committed
      -> controller event -> reconcile -> RoleBinding apply committed -> driver saw it

Each milestone is the first mark of its stage at or after the previous milestone (a stage
with no mark is skipped and its time falls into the next segment), so the segments of a
tenant add up exactly to its apply->Ready latency.  A window reports each segment's p50
and p99, and for its tail tenants (apply->Ready above max(p99, --tail-ms)) which segment
took the longest, which process's stall sampler (native/core/stall.h) reported a
stall overlapping it, and which thread's slow section (a watch event's handling, a watch
write or reconnect: stall::note_slow) overlapped it.

Reference: /root/reference/src/controller.rs:81-154 (the reconcile round trips being
compared), src/synchronizer.rs:289-330 (the status and quota writes).
"""
import re

# Critical-path chains: one regular expression per milestone, in causal order.
_CREATE = [
    ("arrival", r"drv\.sched"),
    ("sent", r"drv\.sent"),
    ("kl_recv", r"kl\.userbootstraps\.POST\.[^.]+\.recv"),
    ("hook_call", r"kl\.userbootstraps\.POST\.[^.]+\.hook0"),
    ("adm_recv", r"adm\.review0\.CREATE"),
    ("adm_done", r"adm\.review1\.CREATE"),
    ("hook_done", r"kl\.userbootstraps\.POST\.[^.]+\.hook1"),
    ("ub_commit", r"kl\.userbootstraps\.POST\.[^.]+\.commit"),
]
_SYNC = [
    ("sync_watch_sent", r"kl\.watch\.userbootstraps\.synchronizer\.sent"),
    ("sync_event", r"sync\.ub_event"),
    ("sync_dequeue", r"sync\.dequeue"),
    ("quota_send", r"sync\.quota\.send"),
    ("quota_kl_recv", r"kl\.userbootstraps\.PATCH\.[^.]+\.recv"),
    ("quota_adm", r"adm\.review1\.UPDATE"),
    ("quota_commit", r"kl\.userbootstraps\.PATCH\.[^.]+\.commit"),
]
_STATUS = [
    ("status_send", r"sync\.status\.send"),
    ("status_kl_recv", r"kl\.userbootstraps/status\.PUT\.[^.]+\.recv"),
    ("status_commit", r"kl\.userbootstraps/status\.PUT\.[^.]+\.commit"),
]


def _ctl(child):
    return [
        ("ctl_watch_sent", r"kl\.watch\.userbootstraps\.controller\.sent"),
        ("ctl_read", r"ctl\.primary_read"),
        ("ctl_event", r"ctl\.primary_event"),
        ("reconcile", r"ctl\.reconcile0"),
        (f"{child}_apply_send", rf"ctl\.apply\.{child}\.send"),
        (f"{child}_kl_recv", rf"kl\.{child}\.PATCH\.[^.]+\.recv"),
        (f"{child}_commit", rf"kl\.{child}\.PATCH\.[^.]+\.commit"),
        (f"{child}_watch_sent", rf"kl\.watch\.{child}\.(?!controller\.|synchronizer\.)[^.]+\.sent"),
    ]


CHAINS = {
    "namespaces": _CREATE + _ctl("namespaces") + [("seen", r"drv\.ns_seen")],
    "resourcequotas": _CREATE + _SYNC + _ctl("resourcequotas") + [("seen", r"drv\.rq_seen")],
    "rolebindings": _CREATE + _SYNC + _STATUS + _ctl("rolebindings") + [("seen", r"drv\.rb_seen")],
}
# kube-lite's ".written" mark (after its write returned) is not on the chain: the reader can
# read the bytes before the writer's clock is read.  Its distance from ".sent" is kept as a
# side statistic per watch, the write's own time.
_WATCH_MARK = re.compile(r"kl\.watch\.([^.]+\.[^.]+)\.(sent|written)$")
_SEEN = {"namespaces": "drv.ns_seen", "resourcequotas": "drv.rq_seen", "rolebindings": "drv.rb_seen"}
_COMPILED = {k: [(n, re.compile(p + r"$")) for n, p in v] for k, v in CHAINS.items()}


def group_marks(dumps):
    """{tenant: [(t_ns, stage), ...] sorted} from /debug/trace documents (any process)."""
    out = {}
    for d in dumps:
        for name, stage, t in (d or {}).get("marks", []):
            out.setdefault(name, []).append((int(t), stage))
    for v in out.values():
        v.sort()
    return out


def critical_path(marks, why=None):
    """(child, [(milestone, t_ns), ...]) for one tenant's marks, or None when it never got
    Ready (`why`, a dict, then counts the reason).  The child is the one the driver saw last."""
    seen = {}
    for t, st in marks:
        for child, s in _SEEN.items():
            if st == s and child not in seen:
                seen[child] = t
    if len(seen) < 3:
        if why is not None:
            why["not_seen_ready"] = why.get("not_seen_ready", 0) + 1
        return None
    child = max(seen, key=seen.get)
    t_seen = seen[child]
    path = []
    i = 0
    for name, rx in _COMPILED[child]:
        j = i
        while j < len(marks) and marks[j][0] <= t_seen and not rx.match(marks[j][1]):
            j += 1
        if j == len(marks) or marks[j][0] > t_seen:
            # no such mark between the previous milestone and Ready: skipped (e.g. the
            # RoleBinding was applied by a reconcile a child event queued, which read the
            # status before the controller's own status event arrived)
            continue
        path.append((name, marks[j][0]))
        i = j
    if not path or path[0][0] != "arrival" or path[-1][0] != "seen":
        if why is not None:
            k = "no_arrival" if not path or path[0][0] != "arrival" else "seen_out_of_order"
            why[k] = why.get(k, 0) + 1
        return None
    return child, path


def _pct(v, q):
    if not v:
        return None
    v = sorted(v)
    k = max(0, min(len(v) - 1, int(round(q * len(v) + 0.5)) - 1))
    return v[k]


def _stall_owner(stalls, t0, t1):
    """The processes whose stall sampler reported a stall overlapping [t0, t1] (a stall
    record ends at its timestamp and lasted its oversleep + malloc time)."""
    owners = {}
    for proc, recs in stalls.items():
        for t_end, over_us, _runq_us, malloc_us in recs:
            start = t_end - int((over_us + malloc_us) * 1e3) - 1_000_000
            if start <= t1 and t_end >= t0:
                owners[proc] = max(owners.get(proc, 0.0), over_us + malloc_us)
    return owners


def _slow_overlap(slow, t0, t1):
    """{"<process> <section>": longest ms} of the slow sections (stall.h note_slow: a watch
    event's handling, a watch write or reconnect) overlapping [t0, t1]."""
    out = {}
    for proc, recs in slow.items():
        for t_end, dur_us, what in recs:
            if t_end - int(dur_us * 1e3) <= t1 and t_end >= t0:
                k = f"{proc} {what}"
                out[k] = max(out.get(k, 0.0), round(dur_us / 1e3, 3))
    return out


def analyze(dumps, stall_dumps=(), tail_ms=5.0, detail=None):
    """Segment table of one window.

    Returns {"tenants": n, "attributed": n, "critical_child": {child: n},
             "segments": {"a->b": {"p50_ms", "p99_ms", "max_ms", "n"}},   (critical-path order)
             "tail": {"threshold_ms", "n", "blame": {"a->b": n}, "blame_ms": {"a->b": total},
                      "stall_overlap": {process: n}, "examples": [...]},
             "stalls": {process: {"n", "max_ms", "sum_ms"}}}"""
    marks = group_marks(dumps)
    writes = {}  # every traced object's watch writes, tenant or not
    for m in marks.values():
        pending = {}
        for t, st in m:
            hit = _WATCH_MARK.match(st)
            if not hit:
                continue
            watch, kind = hit.groups()
            if kind == "sent":
                pending.setdefault(watch, t)
            elif watch in pending:
                writes.setdefault(watch, []).append((t - pending.pop(watch)) / 1e6)
    # tenants are the names the load driver scheduled; other objects sharing the prefix (the
    # controller's Events, named "<tenant>.<suffix>") are not
    others = [n for n, m in marks.items() if not any(st == "drv.sched" for _, st in m)]
    for n in others:
        del marks[n]
    stalls, slow = {}, {}
    for d in stall_dumps:
        if d and d.get("stalls") is not None:
            stalls.setdefault(d.get("process") or "?", []).extend(d["stalls"])
        if d and d.get("slow"):
            slow.setdefault(d.get("process") or "?", []).extend(d["slow"])
    seg_vals, order = {}, []
    per_tenant = []
    children, why, why_examples = {}, {}, []
    for name, m in marks.items():
        cp = critical_path(m, why)
        if cp is None:
            if len(why_examples) < 3:
                t0 = m[0][0]
                why_examples.append({"tenant": name, "timeline_us": [[round((t - t0) / 1e3, 1), st] for t, st in m]})
            continue
        child, path = cp
        children[child] = children.get(child, 0) + 1
        segs = []
        for (a, ta), (b, tb) in zip(path, path[1:]):
            key = f"{a}->{b}"
            if key not in seg_vals:
                seg_vals[key] = []
                order.append(key)
            seg_vals[key].append((tb - ta) / 1e6)
            segs.append((key, ta, tb))
        per_tenant.append((name, (path[-1][1] - path[0][1]) / 1e6, segs))
    total = [t for _, t, _ in per_tenant]
    out = {"tenants": len(marks), "other_objects": len(others), "attributed": len(per_tenant), "unattributed": why,
           "unattributed_examples": why_examples, "critical_child": children,
           "apply_to_ready_p50_ms": _round(_pct(total, 0.5)), "apply_to_ready_p99_ms": _round(_pct(total, 0.99)),
           "segments": {k: {"p50_ms": _round(_pct(seg_vals[k], 0.5)), "p99_ms": _round(_pct(seg_vals[k], 0.99)),
                            "max_ms": _round(max(seg_vals[k])), "n": len(seg_vals[k])} for k in order},
           # kube-lite's write of each watch event (".sent" -> ".written"), per watch
           "watch_writes": {k: {"p50_ms": _round(_pct(v, 0.5)), "p99_ms": _round(_pct(v, 0.99)),
                                "max_ms": _round(max(v)), "n": len(v)} for k, v in sorted(writes.items())}}
    thr = max(_pct(total, 0.99) or 0.0, tail_ms)
    tail = [t for t in per_tenant if t[1] > thr]
    blame, blame_ms, overlap, slow_hits, examples = {}, {}, {}, {}, []
    for name, tot, segs in sorted(tail, key=lambda x: -x[1]):
        key, ta, tb = max(segs, key=lambda s: s[2] - s[1])
        blame[key] = blame.get(key, 0) + 1
        blame_ms[key] = round(blame_ms.get(key, 0.0) + (tb - ta) / 1e6, 3)
        owners = _stall_owner(stalls, ta, tb)
        for p in owners:
            overlap[p] = overlap.get(p, 0) + 1
        sections = _slow_overlap(slow, ta, tb)
        for k in sections:
            slow_hits[k] = slow_hits.get(k, 0) + 1
        if len(examples) < 5:
            examples.append({"tenant": name, "total_ms": round(tot, 3), "longest": key,
                             "longest_ms": round((tb - ta) / 1e6, 3),
                             "stalls_ms": {p: round(v / 1e3, 2) for p, v in owners.items()},
                             "slow_ms": sections})
    out["tail"] = {"threshold_ms": round(thr, 3), "n": len(tail), "blame": blame, "blame_ms": blame_ms,
                   "stall_overlap": overlap, "slow_overlap": slow_hits, "examples": examples}
    if detail is not None and tail:
        # for offline study (--trace-dump): the worst tail tenants' full timelines, and every
        # mark of every tenant within 10 ms around the worst one's longest segment
        worst = sorted(tail, key=lambda x: -x[1])[:20]
        detail["tail_timelines"] = {}
        for name, tot, segs in worst:
            m = marks[name]
            detail["tail_timelines"][name] = {"total_ms": round(tot, 3), "t0_ns": m[0][0],
                                              "marks_us": [[round((t - m[0][0]) / 1e3, 1), st] for t, st in m]}
        key, ta, tb = max(worst[0][2], key=lambda s: s[2] - s[1])
        lo, hi = ta - 10_000_000, tb + 10_000_000
        detail["context"] = {"segment": key, "from_ns": ta, "to_ns": tb,
                             "marks": sorted([t, n, st] for n, m in marks.items() for t, st in m if lo <= t <= hi)}
    out["stalls"] = {p: {"n": len(r), "max_ms": round(max((x[1] + x[3] for x in r), default=0.0) / 1e3, 3),
                         "sum_ms": round(sum(x[1] + x[3] for x in r) / 1e3, 3)} for p, r in stalls.items()}
    sections = {}
    for p, recs in slow.items():
        for _, dur_us, what in recs:
            n, worst = sections.get(f"{p} {what}", (0, 0.0))
            sections[f"{p} {what}"] = (n + 1, max(worst, dur_us / 1e3))
    out["slow_sections"] = {k: {"n": n, "max_ms": round(w, 3)} for k, (n, w) in sorted(sections.items())}
    return out


def _round(v):
    return None if v is None else round(v, 4)
