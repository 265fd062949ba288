"""Headline benchmark: UserBootstrap onboarding churn on an MI355X node.

Metric (BASELINE.json): "reconcile p99 (ms) + admission p50 (ms); CR apply→Ready/sec on
8×MI355X node", reported at 1/2/4/8 advertised GPUs.

One rank per GPU (torchrun).  Rank 0 brings up the control plane: kube-lite (API
server), the TLS admission webhook, the controller, the synchronizer (watch mode, fed by
a fake Google Drive sheet that approves every benchmark tenant) and the node agent,
which advertises the N GPUs of this job as `amd.com/gpu` (amdsmi discovery + telemetry
side thread).  Every rank then acts as a tenant population on its GPU: each step it
applies B UserBootstraps as OIDC users in group `gpu` and waits until each is Ready
(Namespace + ResourceQuota with requests.amd.com/gpu + RoleBinding — BASELINE.md's
definition), deleting the previous step's tenants (GC churn) in the same step.

Weak scaling: per-rank work (B CRs/step) is fixed; the whole-job value is
total Ready CRs / wall time of the K timed steps (max over ranks).
"""
import argparse
import glob
import json
import os
import resource
import statistics
import sys
import time

METRIC = "reconcile p99 (ms) + admission p50 (ms); CR apply→Ready/sec on 8×MI355X node"


def _pct(v, q):
    if not v:
        return None
    v = sorted(v)
    k = max(0, min(len(v) - 1, int(round(q * len(v) + 0.5)) - 1))
    return v[k]


class Dist:
    """torch.distributed wrapper (RCCL on GPUs, gloo on CPU); trivial for one rank."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.torch = None
        self.cuda = False
        try:
            import torch

            self.torch = torch
            torch.set_num_threads(1)  # ranks do no tensor math on the CPU: keep thread count low
            # BGC_BENCH_CPU=1: gloo and no device work, to rehearse several ranks on a box
            # with fewer GPUs than ranks
            self.cuda = os.environ.get("BGC_BENCH_CPU") != "1" and torch.cuda.is_available()
        except Exception:  # noqa: BLE001
            self.torch = None
        if self.cuda:
            self.torch.cuda.set_device(self.local_rank % max(1, self.torch.cuda.device_count()))
        if self.world > 1:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group(backend="nccl" if self.cuda else "gloo")
            self.dist = dist
        else:
            self.dist = None

    def barrier(self):
        if self.dist:
            if self.cuda:
                self.dist.barrier(device_ids=[self.torch.cuda.current_device()])
            else:
                self.dist.barrier()

    def sync(self):
        if self.cuda:
            self.torch.cuda.synchronize()

    def broadcast_obj(self, obj):
        if not self.dist:
            return obj
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=0)
        return lst[0]

    def gather_obj(self, obj):
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def max_scalar(self, x):
        if not self.dist:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device="cuda" if self.cuda else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def _cpu_seconds(pid):
    """utime+stime of a process (for per-component CPU cost reporting)."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        tck = os.sysconf("SC_CLK_TCK")
        return round((int(fields[11]) + int(fields[12])) / tck, 3)
    except (OSError, IndexError, ValueError):
        return None


def effective_cpus():
    """CPUs this job may use: the affinity mask capped by a cgroup v2 cpu.max quota (the
    MI355X boxes expose every host CPU but grant a 16-CPU quota per GPU)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max" and int(period) > 0:
            n = min(n, -(-int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def _cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def _cpulist_text(cpus):
    out, run = [], []
    for c in sorted(cpus):
        if run and c == run[-1] + 1:
            run.append(c)
        else:
            if run:
                out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
            run = [c]
    if run:
        out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
    return ",".join(out)


def _gpu_local_cpus():
    """CPUs of the NUMA node of this job's GPU: the container's own /dev/dri render node
    names its sysfs device (every GPU of the host shows in /sys); else the first AMD GPU."""
    devs = [f"/sys/class/drm/{os.path.basename(n)}/device" for n in sorted(glob.glob("/dev/dri/renderD*"))]
    devs += sorted(glob.glob("/sys/class/drm/renderD*/device"))
    for dev in devs:
        try:
            with open(os.path.join(dev, "vendor")) as f:
                if f.read().strip() != "0x1002":
                    continue
            with open(os.path.join(dev, "local_cpulist")) as f:
                return _cpulist(f.read())
        except (OSError, ValueError):
            continue
    return set()


def _cpu_busy(cpus, interval=0.3):
    """Share of the last `interval` seconds each CPU spent busy (other tenants' work too)."""
    def snap():
        out = {}
        try:
            with open("/proc/stat") as f:
                for line in f:
                    if line.startswith("cpu") and line[3:4].isdigit():
                        p = line.split()
                        v = [int(x) for x in p[1:]]
                        out[int(p[0][3:])] = (sum(v), v[3] + (v[4] if len(v) > 4 else 0))
        except (OSError, ValueError):
            pass
        return out
    a = snap()
    time.sleep(interval)
    b = snap()
    busy = {}
    for c in cpus:
        if c in a and c in b and b[c][0] > a[c][0]:
            busy[c] = 1.0 - (b[c][1] - a[c][1]) / (b[c][0] - a[c][0])
        else:
            busy[c] = 0.0
    return busy


def _core_of(c):
    """The physical core a CPU belongs to (its SMT siblings share it)."""
    try:
        with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
            return min(_cpulist(f.read()))
    except (OSError, ValueError):
        return c


def quota_cpuset(measure=True):
    """The CPUs to run the control plane on when the cgroup's CPU quota is smaller than the
    affinity mask (the MI355X boxes: a 16-CPU quota per GPU over 256 visible CPUs), or None.

    Unpinned, the job's threads spread over every visible CPU, spend the quota in a fraction
    of each 100 ms CFS period and are then frozen for the rest of it: tail latencies of the
    whole stack jump to 40-50 ms whenever the load outruns the quota (measured on the box:
    33 of 97 periods throttled in a headline run, profiles/kl_shard_r4/).  Pinned to as many
    CPUs as the quota grants, the same CPU time is shared instead (what a Kubernetes pod gets
    from the static CPU manager, or a Go service from a quota-sized GOMAXPROCS).

    Which CPUs: those of the GPU's NUMA node, CPU 0 (interrupts) left out, the idlest first
    (the host runs other tenants: one of them held a CPU at 100 % in a sample on the box),
    one per physical core before any SMT sibling."""
    if not hasattr(os, "sched_getaffinity"):
        return None
    aff = sorted(os.sched_getaffinity(0))
    n = effective_cpus()
    if n >= len(aff):
        return None
    local = _gpu_local_cpus() & set(aff)
    pool = [c for c in aff if c in local and c != 0] or [c for c in aff if c != 0] or aff
    if len(pool) < n:
        pool += [c for c in aff if c not in pool]
    if measure:
        busy = _cpu_busy(pool)
        # 5 % steps: CPUs equally idle keep their index order
        order = {c: i for i, c in enumerate(pool)}
        pool.sort(key=lambda c: (round(busy.get(c, 0.0) * 20), order[c]))
    chosen, cores = [], set()
    for c in pool:  # one CPU per physical core first
        core = _core_of(c)
        if core not in cores:
            chosen.append(c)
            cores.add(core)
        if len(chosen) == n:
            break
    for c in pool:  # then SMT siblings, if the node has fewer idle cores than the quota
        if len(chosen) == n:
            break
        if c not in chosen:
            chosen.append(c)
    return sorted(chosen)


def cgroup_throttling():
    """cgroup v2 cpu.stat: CFS bandwidth periods and throttled time so far (None if absent)."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            st = dict(line.split() for line in f if line.strip())
        return {"periods": int(st["nr_periods"]), "throttled": int(st["nr_throttled"]),
                "throttled_ms": int(st["throttled_usec"]) / 1e3}
    except (OSError, KeyError, ValueError):
        return None


def runqueue_wait_ms(pids):
    """Time the threads of `pids` spent runnable but waiting for a CPU (/proc/<pid>/task/*/
    schedstat, second field), summed: a window whose latencies jump while this jumps lost
    its CPUs (to the job's own processes or to anything else on them)."""
    total = 0
    for pid in pids:
        try:
            tids = os.listdir(f"/proc/{pid}/task")
        except OSError:
            continue
        for tid in tids:
            try:
                with open(f"/proc/{pid}/task/{tid}/schedstat") as f:
                    total += int(f.read().split()[1])
            except (OSError, IndexError, ValueError):
                pass
    return total / 1e6


def cpu_ticks(cpus):
    """(busy, total, steal) jiffies summed over `cpus` (/proc/stat), for the job's CPU share.
    steal: time the hypervisor ran something else while these (virtual) CPUs had work."""
    busy = total = steal = 0
    try:
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3:4].isdigit():
                    p = line.split()
                    if int(p[0][3:]) in cpus:
                        v = [int(x) for x in p[1:]]
                        total += sum(v[:8])
                        busy += sum(v[:8]) - v[3] - (v[4] if len(v) > 4 else 0)
                        steal += v[7] if len(v) > 7 else 0
    except (OSError, ValueError):
        pass
    return busy, total, steal


def thread_cpu(procs):
    """{(process, thread name, tid): (cpu seconds, run-queue wait seconds)} over every thread
    of `procs` ({process name: pid}): the name from /proc/<pid>/task/<tid>/comm, both times
    from its schedstat (on-CPU ns, runnable-but-waiting ns)."""
    out = {}
    for pname, pid in procs.items():
        try:
            tids = os.listdir(f"/proc/{pid}/task")
        except OSError:
            continue
        for tid in tids:
            try:
                with open(f"/proc/{pid}/task/{tid}/comm") as f:
                    comm = f.read().strip()
                with open(f"/proc/{pid}/task/{tid}/schedstat") as f:
                    run, wait = f.read().split()[:2]
                out[(pname, comm, tid)] = (int(run) / 1e9, int(wait) / 1e9)
            except (OSError, ValueError):
                pass  # the thread exited meanwhile
    return out


def llc_groups(cpus):
    """The CPUs of `cpus` grouped by the last-level cache they share (sysfs cache index3),
    as cpulist strings; [] when the topology is not readable."""
    groups = {}
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                key = f.read().strip()
        except OSError:
            return []
        groups.setdefault(key, []).append(c)
    return [_cpulist_text(set(v)) for v in sorted(groups.values())]


def busiest_threads(t0, t1, dt, top=6):
    """The threads that used the most CPU between two thread_cpu() readings, as share of
    one CPU: a single-threaded stage near 1.0 is a pipeline bottleneck (its queue grows)."""
    used = []
    for k, v in t1.items():
        d = v[0] - t0.get(k, (0.0, 0.0))[0]
        if d > 0:
            used.append((d / dt, k))
    used.sort(reverse=True)
    return [{"process": k[0], "thread": k[1], "cpu": round(u, 2)} for u, k in used[:top]]


def waiting_threads(t0, t1, top=6):
    """The threads that waited longest for a CPU between two thread_cpu() readings (ms over
    the window; summed over the threads sharing a name).  A stage whose thread is here while
    the job's CPUs are not all busy lost its CPU to the scheduler's placement, not to load."""
    waited = {}
    for k, v in t1.items():
        d = v[1] - t0.get(k, (0.0, 0.0))[1]
        if d > 0:
            name = (k[0], k[1])
            n, tot, worst = waited.get(name, (0, 0.0, 0.0))
            waited[name] = (n + 1, tot + d, max(worst, d))
    ranked = sorted(waited.items(), key=lambda x: -x[1][1])
    # plus every watch reader (w:<resource>): one thread each, on every tenant's critical path
    rows = ranked[:top] + [r for r in ranked[top:] if r[0][1].startswith("w:")]
    return [{"process": p, "thread": t, "threads": n, "runq_ms": round(tot * 1e3, 2),
             "worst_thread_runq_ms": round(worst * 1e3, 2)} for (p, t), (n, tot, worst) in rows]


def job_cpu_seconds(pids):
    """utime+stime of every process in `pids` (all threads), seconds."""
    return sum(_cpu_seconds(p) or 0.0 for p in pids)


def auto_concurrency(world, cpus):
    """In-flight creates per rank.  The control plane is CPU-bound, so the total in flight
    is sized to its CPU share rather than fixed per rank: measured on the MI355X box
    (16 CPUs, profiles/archive/concurrency_sweep_r1/), 32 per rank costs 20-45 % throughput and
    2x apply->Ready latency at every N against ~cpus/(2*sqrt(N)) per rank."""
    return int(min(32, max(4, round(cpus / (2.0 * world ** 0.5)))))


def _rss_mb(pid):
    """Resident set size of a component (leak check over long runs)."""
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("VmRSS:"):
                    return round(int(line.split()[1]) / 1024.0, 1)
    except (OSError, ValueError, IndexError):
        pass
    return None


def _names(rank, phase, step, batch):
    return [f"r{rank}-{phase}{step}-u{i}" for i in range(batch)]


class TruncatedWindow(RuntimeError):
    """A latency window lost samples: no percentile may be reported over it."""


def _get_json(url, method="GET", verify=None):
    """GET/DELETE a /debug/samples/<name> document; None when the process has no such log."""
    import requests

    r = requests.request(method, url, timeout=10, verify=verify)
    if r.status_code == 404:
        return None
    r.raise_for_status()
    return r.json()


def _samples(url, verify=None):
    return _get_json(url, verify=verify)


def _clear(url, verify=None):
    """Starts a window: clears the log and returns its counts at that instant."""
    return _get_json(url, method="DELETE", verify=verify)


def linked_delta(doc, start):
    """Increments of the log's linked counters (e.g. bgc_reconcile_total) over the window.
    They are counted inside the log's lock together with each sample (SampleLog::add), so
    for a complete window this equals the number of samples exactly."""
    if not doc or not doc.get("linked"):
        return None
    base = (start or {}).get("linked", {})
    return int(round(sum(v - base.get(k, 0.0) for k, v in doc["linked"].items())))


def window_samples(doc, start=None, required=True):
    """The samples of one measurement window, checked complete.

    `doc` is GET /debug/samples/<name> at the end of the window, `start` the DELETE response
    at its start.  Raises TruncatedWindow when the log dropped samples (capacity reached or
    recording off) or when its linked counters moved by other than the number of samples,
    so a truncated window can never turn into a reported percentile."""
    if doc is None:
        if required:
            raise TruncatedWindow("sample log missing (is CONF_DEBUG_ENDPOINTS on?)")
        return []
    name, samples = doc.get("name"), doc["samples"]
    if doc.get("dropped", 0) or len(samples) != doc["total"]:
        raise TruncatedWindow(f"{name}: {len(samples)} of {doc['total']} samples kept (capacity "
                              f"{doc.get('capacity')}, dropped {doc.get('dropped')}): refusing a percentile "
                              "over a truncated window")
    delta = linked_delta(doc, start)
    if delta is not None and start is not None and delta != len(samples):
        raise TruncatedWindow(f"{name}: {len(samples)} samples but linked counters moved by {delta}")
    return samples


def _lock_report(l0, l1, elapsed):
    """kube-lite's store locks over the window: every acquisition of a per-object shard lock
    and of a type's commit-order lock (seq), how many had to wait and for how long; the
    busiest type is the one whose seq section (the serialized part of its commits) was held
    the largest share of the window."""
    t0, t1 = l0["total"], l1["total"]
    busiest, util = None, 0.0
    for k, v in l1["by_type"].items():
        h = v["hold_ms"] - l0["by_type"].get(k, {}).get("hold_ms", 0.0)
        if h / (elapsed * 1e3) > util:
            busiest, util = k, h / (elapsed * 1e3)
    acq = t1["acquisitions"] - t0["acquisitions"]
    contended = t1["contended"] - t0["contended"]
    wait_ms = t1["wait_ms"] - t0["wait_ms"]
    return {"store_shards": l1.get("store_shards"),
            "acquisitions": acq,
            "contended": contended,
            "contended_pct": round(100.0 * contended / acq, 2) if acq else 0.0,
            "hold_ms": round(t1["hold_ms"] - t0["hold_ms"], 3),
            "wait_ms": round(wait_ms, 3),
            "wait_s_per_s": round(wait_ms / 1e3 / elapsed, 3) if elapsed > 0 else None,
            "busiest_type": busiest, "busiest_utilisation": round(util, 4)}


def _gpu_telemetry(url):
    import requests

    d = requests.get(url + "/gpus", timeout=10).json()
    keep = ("index", "power_w", "temp_hotspot_c", "temp_mem_c", "gfx_activity_pct", "umc_activity_pct",
            "vram_used_mb", "gfxclk_mhz", "uclk_mhz", "xgmi_links_up", "ecc_uncorrectable")
    return {"backend": d.get("backend"), "advertised": len(d.get("gpus", [])), "healthy": d.get("healthy"),
            "product": (d.get("gpus") or [{}])[0].get("market_name"),
            "devices": [{k: t[k] for k in keep if k in t} for t in d.get("telemetry", [])]}


def _kl_lock(info):
    import requests

    st = requests.get(info["server"] + "/_kl/stats", timeout=10, verify=info["apiserver_verify"]).json()
    return {"total": st["store_lock"], "by_type": st.get("by_type_lock", {}), "requests": st["requests"],
            "by_kind": st.get("requests_by_kind", {}), "store_shards": st.get("store_shards")}


PRODUCT = ("controller", "admission", "synchronizer", "node-agent")


def _cpu_snapshot(cluster):
    return {name: _cpu_seconds(p.p.pid) for name, p in cluster.procs.items()}


def _sample_logs(info):
    """The latency logs a phase reads: key -> (URL, TLS verify)."""
    return {"reconcile": (info["controller"] + "/debug/samples/reconcile", None),
            "webhook": (info["server"] + "/debug/samples/webhook", info["apiserver_verify"]),
            "admission": (info["admission"] + "/debug/samples/admission", info["ca"]),
            "h2_server": (info["admission"] + "/debug/samples/h2_server", info["ca"]),
            "telemetry_poll": (info["node_agent"] + "/debug/samples/telemetry_poll", None),
            "telemetry_poll_cpu": (info["node_agent"] + "/debug/samples/telemetry_poll_cpu", None),
            "telemetry_poll_runq": (info["node_agent"] + "/debug/samples/telemetry_poll_runq", None),
            "sync_ub": (info["synchronizer"] + "/debug/samples/sync_ub", None)}


def _phase(d, nat, info, args, phase, concurrency, warmup, steps, cluster):
    """One measured phase: `warmup` untimed + `steps` timed steps at `concurrency` creates in
    flight per rank.  Returns the per-phase record on rank 0 (None elsewhere)."""
    total_steps = warmup + steps
    from bacchus_gpu_controller_amd.testing.cluster import ADMIN_TOKEN

    driver = nat.ChurnDriver(info["server"], ADMIN_TOKEN, f"r{d.rank}-", concurrency,
                             ca_pem=info["apiserver_ca"], approve_url=info.get("approve_url", ""),
                             http2=args.driver_http2, server_filter=args.driver_server_filter)
    driver.start()
    time.sleep(0.2)
    prev = None
    lat, clat, ap_lat, ap_ready = [], [], [], []
    stage = {"ns": [], "rq": [], "rb": []}
    ready = failed = timeouts = 0
    lock0 = cpu0 = thr0 = thr1 = None
    starts = {}
    t_start = None
    errors = []
    last_note = time.perf_counter()
    try:
        for s in range(total_steps):
            if d.rank == 0 and time.perf_counter() - last_note > 15:
                # slow modes (the reference's 60 s sheet tick) must still show progress
                print(f"[bench] phase {phase} step {s}/{total_steps}", file=sys.stderr, flush=True)
                last_note = time.perf_counter()
            if s == warmup:
                d.barrier()
                d.sync()
                if d.rank == 0:
                    starts = {key: _clear(url, verify) for key, (url, verify) in _sample_logs(info).items()}
                    lock0 = _kl_lock(info)
                    cpu0 = _cpu_snapshot(cluster)
                    thr0 = cgroup_throttling()
                d.barrier()
                t_start = time.perf_counter()
                ru0 = resource.getrusage(resource.RUSAGE_SELF)
            for r in range(args.rounds):
                # one round: `batch` tenants applied `concurrency` at a time and waited to
                # Ready, deleting the previous round's tenants (GC churn) meanwhile
                names = _names(d.rank, phase, s * args.rounds + r, args.batch)
                res = json.loads(driver.step_with_delete(names, prev or [], args.timeout))
                prev = names
                if cluster is not None and res.get("timeouts"):
                    # a component that died stalls every later tenant: fail now, not after
                    # a timeout per round
                    dead = [n for n, pr in cluster.procs.items() if not pr.alive()]
                    if dead:
                        raise RuntimeError(f"control-plane process(es) exited during the run: {', '.join(dead)}")
                if s >= warmup:
                    lat += res["ready_latency_s"]
                    clat += res["create_latency_s"]
                    ap_lat += res.get("approve_latency_s", [])
                    ap_ready += res.get("approve_to_ready_latency_s", [])
                    for k in stage:
                        stage[k] += res[f"{k}_latency_s"]
                    ready += res["ready"]
                    failed += res["failed"]
                    timeouts += res["timeouts"]
                    errors += res["errors"]
        d.sync()
        d.barrier()
        elapsed = time.perf_counter() - t_start
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu1 = _cpu_snapshot(cluster) if d.rank == 0 else None
        thr1 = cgroup_throttling() if d.rank == 0 else None
        driver_cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
        elapsed = d.max_scalar(elapsed)
        driver.remove(prev)
    finally:
        driver.stop()
    per_rank = d.gather_obj({"ready": ready, "failed": failed, "timeouts": timeouts, "lat": lat, "clat": clat,
                             "ap_lat": ap_lat, "ap_ready": ap_ready, "stage": stage, "errors": errors[:3],
                             "driver_cpu_s": driver_cpu})
    if d.rank != 0:
        return None
    lock1 = _kl_lock(info)
    docs = {key: _samples(url, verify) for key, (url, verify) in _sample_logs(info).items()}
    # every log is checked complete over the window; the headline two must exist
    win = {key: window_samples(docs[key], starts.get(key), required=key in ("reconcile", "webhook"))
           for key in docs}
    rec, hook, adm = win["reconcile"], win["webhook"], win["admission"]
    # HTTP/2 webhook requests: request complete on the server's reader -> response written
    h2s, tel, syn = win["h2_server"], win["telemetry_poll"], win["sync_ub"]
    total_ready = sum(p["ready"] for p in per_rank)
    total_failed = sum(p["failed"] + p["timeouts"] for p in per_rank)
    flat = lambda key: [x for p in per_rank for x in p[key]]  # noqa: E731
    all_lat, all_clat = flat("lat"), flat("clat")
    ms = lambda v: None if v is None else round(v * 1e3, 4)  # noqa: E731
    per_cr = max(1, total_ready)
    cpu_ms = {}
    for name in cpu0:
        if cpu0[name] is not None and cpu1.get(name) is not None:
            cpu_ms["kube_lite" if name == "apiserver" else name.replace("-", "_")] = round(
                (cpu1[name] - cpu0[name]) * 1e3 / per_cr, 4)
    cpu_ms["load_driver"] = round(sum(p["driver_cpu_s"] for p in per_rank) * 1e3 / per_cr, 4)
    cpu_ms["product_total"] = round(sum(cpu_ms.get(c.replace("-", "_"), 0.0) for c in PRODUCT), 4)
    out = {
        "value": round(total_ready / elapsed if elapsed > 0 else 0.0, 3),
        "elapsed_s": elapsed,
        "steps": steps,
        "warmup": warmup,
        "concurrency_per_rank": concurrency,
        "reconcile_p99_ms": ms(_pct(rec, 0.99)),
        "reconcile_p50_ms": ms(_pct(rec, 0.50)),
        # every reconcile of the window: len(samples) == the increase of the controller's
        # bgc_reconcile_total (counted with each sample, under the log's lock)
        "reconciles": len(rec),
        "reconcile_total_delta": linked_delta(docs["reconcile"], starts.get("reconcile")),
        "webhook_calls": len(hook),
        "webhook_calls_total_delta": linked_delta(docs["webhook"], starts.get("webhook")),
        "samples_complete": True,
        # webhook round trip as the API server measures it (TLS + handler + response)
        "admission_p50_ms": ms(_pct(hook, 0.50)),
        "admission_p99_ms": ms(_pct(hook, 0.99)),
        "admission_handler_p50_ms": ms(_pct(adm, 0.50)),
        "admission_h2_server_p50_ms": ms(_pct(h2s, 0.50)),
        "admission_h2_server_p99_ms": ms(_pct(h2s, 0.99)),
        "apply_to_ready_p50_ms": ms(_pct(all_lat, 0.50)),
        "apply_to_ready_p99_ms": ms(_pct(all_lat, 0.99)),
        "create_p50_ms": ms(_pct(all_clat, 0.50)),
        # apply -> first observation of each child (Namespace; ResourceQuota with the sheet's
        # quota; RoleBinding after the status write)
        "stage_p50_ms": {k: ms(_pct([x for p in per_rank for x in p["stage"][k]], 0.50)) for k in ("ns", "rq", "rb")},
        "telemetry_poll_p50_ms": ms(_pct(tel, 0.50)),
        # the poll's wall time split (core/schedstat.h): on a CPU, waiting for one, and the
        # rest blocked in amdsmi's ioctls
        "telemetry_poll_split_p50_ms": {"cpu": ms(_pct(win["telemetry_poll_cpu"], 0.50)),
                                        "runq": ms(_pct(win["telemetry_poll_runq"], 0.50)),
                                        "runq_p99": ms(_pct(win["telemetry_poll_runq"], 0.99))},
        "sync_one_p50_ms": ms(_pct(syn, 0.50)),
        # CPU time each process spent in the timed region, per Ready CR.  kube_lite is the
        # test API server and load_driver the tenant simulator: neither ships.
        "cpu_ms_per_cr": cpu_ms,
        "apiserver_store_lock": _lock_report(lock0, lock1, elapsed),
        "apiserver_requests_per_cr": round((lock1["requests"] - lock0["requests"]) / per_cr, 2),
        "apiserver_requests_per_cr_by_kind": {
            k: round((v - lock0["by_kind"].get(k, 0)) / per_cr, 3)
            for k, v in sorted(lock1["by_kind"].items()) if v - lock0["by_kind"].get(k, 0) > 0},
        "ready_crs": total_ready,
        "failed_crs": total_failed,
    }
    if thr0 and thr1:
        # CFS bandwidth control over the window: periods in which the job's cgroup ran out
        # of its CPU quota and was frozen until the next period (see quota_cpuset)
        periods = thr1["periods"] - thr0["periods"]
        out["cgroup_throttled"] = {"periods": periods, "throttled_periods": thr1["throttled"] - thr0["throttled"],
                                   "throttled_ms": round(thr1["throttled_ms"] - thr0["throttled_ms"], 1)}
    if info.get("approve_url"):
        out["approve_to_ready_p50_ms"] = ms(_pct(flat("ap_ready"), 0.50))
        out["approve_to_ready_p99_ms"] = ms(_pct(flat("ap_ready"), 0.99))
        out["create_to_approve_p50_ms"] = ms(_pct(flat("ap_lat"), 0.50))
    if total_failed:
        out["errors"] = [e for p in per_rank for e in p["errors"]][:5]
    return out


def _warm(d, nat, info, args, key, concurrency, steps):
    """Untimed closed-loop steps (`steps` x --rounds rounds of --batch tenants per rank),
    every tenant deleted afterwards."""
    from bacchus_gpu_controller_amd.testing.cluster import ADMIN_TOKEN

    driver = nat.ChurnDriver(info["server"], ADMIN_TOKEN, f"r{d.rank}-", concurrency, ca_pem=info["apiserver_ca"],
                             http2=args.driver_http2, server_filter=args.driver_server_filter)
    driver.start()
    prev = None
    try:
        for s in range(steps * args.rounds):
            names = _names(d.rank, key, s, args.batch)
            driver.step_with_delete(names, prev or [], args.timeout)
            prev = names
        driver.remove(prev or [])
    finally:
        driver.stop()
    d.barrier()


def _settle(info, timeout=10.0):
    """Waits until kube-lite's garbage collector has caught up (the cascades of the previous
    phase's deletions), so a phase does not start on the tail of another one's work."""
    import requests

    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        try:
            st = requests.get(info["server"] + "/_kl/stats", timeout=5, verify=info["apiserver_verify"]).json()
            if not st.get("gc_pending"):
                break
        except Exception:  # noqa: BLE001
            break
        time.sleep(0.05)
    time.sleep(0.2)


def _rate_names(rank, key, rate, part, n):
    return [f"r{rank}-{key}{int(rate)}{part}-u{i}" for i in range(n)]


def _debug_processes(info):
    """(process, base URL, TLS verify) of every process serving /debug/trace and /debug/stalls."""
    return [("kube-lite", info["server"], info["apiserver_verify"]), ("controller", info["controller"], None),
            ("admission", info["admission"], info["ca"]), ("synchronizer", info["synchronizer"], None),
            ("node-agent", info["node_agent"], None)]


def _debug_call(method, url, verify, data=None):
    import requests

    try:
        r = requests.request(method, url, data=data, timeout=30, verify=verify)
        return r.json() if r.status_code == 200 and method != "POST" else None
    except Exception:  # noqa: BLE001
        return None


def _rate_phase(d, nat, info, args, key, rate, cluster):
    """Open-loop latency at a fixed offered rate: tenants arrive as a Poisson
    process of `rate` CR/s over the whole job (each rank offers rate/world), whatever the
    system's progress, and each leaves once Ready.  Unlike the closed-loop phases, whose
    latencies grow with the CR/s they reach (a faster controller queues more work on the
    same CPUs), every arm here carries the same load, so reconcile p99 and admission p50
    compare like for like.  `--latency-window-s` timed after `--latency-warmup-s` untimed.

    The timed window is traced: every process marks each tenant's stages
    (native/core/trace.h) and keeps its stalls (native/core/stall.h); bench/attribution.py
    joins them into the per-stage table of the window ("attribution")."""
    import requests

    from bacchus_gpu_controller_amd.bench import attribution
    from bacchus_gpu_controller_amd.testing.cluster import ADMIN_TOKEN

    per_rank = rate / d.world
    n_warm = max(1, int(round(per_rank * args.latency_warmup_s)))
    n_timed = max(1, int(round(per_rank * args.latency_window_s)))
    driver = nat.ChurnDriver(info["server"], ADMIN_TOKEN, f"r{d.rank}-", args.latency_workers,
                             ca_pem=info["apiserver_ca"], http2=args.driver_http2,
                             server_filter=args.driver_server_filter)
    driver.start()
    coalesce_prev = None
    if d.rank == 0:
        _settle(info)
        if args.latency_watch_coalesce_us >= 0:
            # kube-lite's watch writers hold an event up to --watch-coalesce-us for a burst to
            # grow (a throughput setting of the test apiserver); under load that timed wait
            # overshoots to ms, so the windows time latency without it
            r = requests.post(info["server"] + "/_kl/watch-coalesce-us", data=str(args.latency_watch_coalesce_us),
                              timeout=10, verify=info["apiserver_verify"])
            r.raise_for_status()
            coalesce_prev = r.text.strip()
    d.barrier()
    traced = args.trace_windows
    prefixes = ",".join(f"r{r}-{key}{int(rate)}t" for r in range(d.world))
    try:
        driver.open_loop(_rate_names(d.rank, key, rate, "w", n_warm), args.latency_warmup_s, args.timeout, 7 + d.rank)
        d.barrier()
        starts = thr0 = rq0 = None
        pids = [os.getpid()] + [p.p.pid for p in cluster.procs.values()] if d.rank == 0 and cluster else []
        if traced:
            nat.trace_arm(prefixes)
            nat.stall_take()
        if d.rank == 0:
            starts = {k: _clear(url, verify) for k, (url, verify) in _sample_logs(info).items()}
            thr0 = cgroup_throttling()
            rq0 = runqueue_wait_ms(pids)
            # CPU time on the job's CPUs that the job itself did not use: another tenant of
            # the host (the box shares its CPUs) competing for the share
            job_cpus = set(os.sched_getaffinity(0))
            tick0, own0, wall0 = cpu_ticks(job_cpus), job_cpu_seconds(pids), time.monotonic()
            named = {"load-driver": os.getpid(), **{n: p.p.pid for n, p in cluster.procs.items()}}
            thr_cpu0 = thread_cpu(named)
            if traced:
                for _, base, verify in _debug_processes(info):
                    _debug_call("POST", base + "/debug/trace", verify, data=prefixes)
                    _debug_call("DELETE", base + "/debug/stalls", verify)
        d.barrier()
        res = json.loads(driver.open_loop(_rate_names(d.rank, key, rate, "t", n_timed), args.latency_window_s,
                                          args.timeout, 1000 + d.rank))
        d.barrier()
        thr1 = cgroup_throttling() if d.rank == 0 else None
        rq1 = runqueue_wait_ms(pids) if d.rank == 0 else None
        if d.rank == 0:
            tick1, own1, wall1 = cpu_ticks(job_cpus), job_cpu_seconds(pids), time.monotonic()
            thr_cpu1 = thread_cpu(named)
        mine = {"trace": json.loads(nat.trace_take()), "stalls": json.loads(nat.stall_take())} if traced else None
    finally:
        driver.stop()
        if coalesce_prev is not None:
            requests.post(info["server"] + "/_kl/watch-coalesce-us", data=coalesce_prev, timeout=10,
                          verify=info["apiserver_verify"]).raise_for_status()
    per = d.gather_obj({k: res[k] for k in ("ready", "failed", "timeouts", "offered_rate", "achieved_rate",
                                            "issue_lag_p99_s", "ready_latency_s", "errors")})
    drv = d.gather_obj(mine)
    if d.rank != 0:
        return None
    traces, stalls = [], []
    if traced:
        for proc, base, verify in _debug_processes(info):
            traces.append(_debug_call("DELETE", base + "/debug/trace", verify))
            st = _debug_call("DELETE", base + "/debug/stalls", verify)
            if st is not None:
                st["process"] = proc
            stalls.append(st)
        for r, m in enumerate(drv):
            traces.append(m["trace"])
            m["stalls"]["process"] = f"load-driver-r{r}"
            stalls.append(m["stalls"])
    docs = {k: _samples(url, verify) for k, (url, verify) in _sample_logs(info).items()}
    rec = window_samples(docs["reconcile"], starts.get("reconcile"))
    hook = window_samples(docs["webhook"], starts.get("webhook"))
    adm = window_samples(docs["admission"], starts.get("admission"), required=False)
    lat = [x for p in per for x in p["ready_latency_s"]]
    ms = lambda v: None if v is None else round(v * 1e3, 4)  # noqa: E731
    offered = sum(p["offered_rate"] for p in per)
    achieved = sum(p["achieved_rate"] for p in per)
    out = {"offered_rate": round(offered, 1), "achieved_rate": round(achieved, 1),
           "achieved_within_2pct": bool(offered and abs(achieved - offered) <= 0.02 * offered),
           "reconcile_p99_ms": ms(_pct(rec, 0.99)), "reconcile_p50_ms": ms(_pct(rec, 0.50)),
           "reconciles": len(rec),
           "admission_p50_ms": ms(_pct(hook, 0.50)), "admission_p99_ms": ms(_pct(hook, 0.99)),
           "admission_handler_p50_ms": ms(_pct(adm, 0.50)),
           "apply_to_ready_p50_ms": ms(_pct(lat, 0.50)), "apply_to_ready_p99_ms": ms(_pct(lat, 0.99)),
           "issue_lag_p99_ms": ms(max(p["issue_lag_p99_s"] for p in per)),
           "ready_crs": sum(p["ready"] for p in per),
           "failed_crs": sum(p["failed"] + p["timeouts"] for p in per),
           # raw samples for pooling a rate's windows (removed before the output is printed)
           "_raw": {"rec": rec, "hook": hook, "lat": lat}}
    if thr0 and thr1:
        out["cgroup_throttled_periods"] = thr1["throttled"] - thr0["throttled"]
    if rq0 is not None and rq1 is not None:
        # CPU-ms the job's threads waited in run queues per second of window
        out["runqueue_wait_ms_per_s"] = round((rq1 - rq0) / max(args.latency_window_s, 1e-9), 1)
        hz = os.sysconf("SC_CLK_TCK")
        busy_s = (tick1[0] - tick0[0]) / hz
        dt = max(wall1 - wall0, 1e-9)
        out["cpus_busy"] = round(busy_s / dt, 2)           # CPUs' worth busy on the job's CPU set
        out["job_cpus_used"] = round((own1 - own0) / dt, 2)  # of which the job's own processes
        out["foreign_cpus"] = round(max(0.0, busy_s - (own1 - own0)) / dt, 2)
        out["steal_cpus"] = round((tick1[2] - tick0[2]) / hz / dt, 3)  # of which the hypervisor's
        out["busiest_threads"] = busiest_threads(thr_cpu0, thr_cpu1, dt)
        out["waiting_threads"] = waiting_threads(thr_cpu0, thr_cpu1)
    if traced:
        detail = {} if args.trace_dump else None
        out["attribution"] = attribution.analyze(traces, stalls, tail_ms=args.tail_ms, detail=detail)
        if detail:
            os.makedirs(args.trace_dump, exist_ok=True)
            detail["stalls"] = stalls
            with open(os.path.join(args.trace_dump, f"{key}.json"), "w") as f:
                json.dump(detail, f)
        out["attribution"]["trace_marks"] = sum(len((t or {}).get("marks", [])) for t in traces)
        out["attribution"]["trace_dropped"] = sum((t or {}).get("dropped", 0) for t in traces)
    errs = [e for p in per for e in p["errors"]]
    if errs:
        out["errors"] = errs[:3]
    return out


_WINDOW_KEYS = ("offered_rate", "achieved_rate", "achieved_within_2pct", "reconcile_p99_ms", "reconcile_p50_ms",
                "reconciles", "admission_p50_ms", "admission_p99_ms", "admission_handler_p50_ms",
                "apply_to_ready_p50_ms", "apply_to_ready_p99_ms", "issue_lag_p99_ms", "ready_crs", "failed_crs",
                "cgroup_throttled_periods", "runqueue_wait_ms_per_s", "cpus_busy", "job_cpus_used", "foreign_cpus", "steal_cpus",
                "busiest_threads", "waiting_threads", "errors")


def _pool_arm(results, prefix, rates, windows):
    """Per rate: the arm's windows pooled (percentiles over every sample of its windows) plus
    each window's own row, in run order."""
    ms = lambda v: None if v is None else round(v * 1e3, 4)  # noqa: E731
    out = {}
    for i, r in enumerate(rates):
        ws = [results[f"{prefix}{i}w{k}"] for k in range(windows) if results.get(f"{prefix}{i}w{k}")]
        if not ws:
            continue
        rec = [x for w in ws for x in w["_raw"]["rec"]]
        hook = [x for w in ws for x in w["_raw"]["hook"]]
        lat = [x for w in ws for x in w["_raw"]["lat"]]
        out[f"{r:g}"] = {"offered_rate": round(sum(w["offered_rate"] for w in ws) / len(ws), 1),
                         "achieved_rate": round(sum(w["achieved_rate"] for w in ws) / len(ws), 1),
                         "reconcile_p99_ms": ms(_pct(rec, 0.99)), "reconcile_p50_ms": ms(_pct(rec, 0.50)),
                         "admission_p50_ms": ms(_pct(hook, 0.50)), "apply_to_ready_p50_ms": ms(_pct(lat, 0.50)),
                         "apply_to_ready_p99_ms": ms(_pct(lat, 0.99)),
                         "ready_crs": sum(w["ready_crs"] for w in ws), "failed_crs": sum(w["failed_crs"] for w in ws),
                         "windows": [{k: w[k] for k in _WINDOW_KEYS if k in w} for w in ws]}
    return out


def _stage_summary(results, prefix, rates, windows, top=3):
    """Compact per-stage table of an arm (the bench line's last field, so the driver's
    2,000-character tail of the output keeps it): per rate, the apply->Ready p99 of each
    window, the critical-path segments with the largest p99 (worst window), and which
    segment the tail tenants spent the most in, summed over the windows."""
    out = {}
    for i, r in enumerate(rates):
        atts = [results[f"{prefix}{i}w{k}"].get("attribution") for k in range(windows)
                if results.get(f"{prefix}{i}w{k}")]
        atts = [a for a in atts if a]
        if not atts:
            continue
        seg = {}
        for a in atts:
            for k, v in a["segments"].items():
                if v["p99_ms"] is not None:
                    seg[k] = max(seg.get(k, 0.0), v["p99_ms"])
        blame, stall = {}, {}
        for a in atts:
            for k, n in a["tail"]["blame"].items():
                blame[k] = blame.get(k, 0) + n
            for k, n in a["tail"]["stall_overlap"].items():
                stall[k] = stall.get(k, 0) + n
        r2 = lambda v: None if v is None else round(v, 2)  # noqa: E731
        out[f"{r:g}"] = {"a2r_p99": [r2(a["apply_to_ready_p99_ms"]) for a in atts],
                         "seg_p99": {k: r2(v) for k, v in sorted(seg.items(), key=lambda kv: -kv[1])[:top]},
                         "tail_n": sum(a["tail"]["n"] for a in atts),
                         "tail_blame": dict(sorted(blame.items(), key=lambda kv: -kv[1])[:2]),
                         "tail_stalls": stall}
    return out


def _latency_at_rate(results, rates, windows, args):
    this_q = _pool_arm(results, "qa", rates, windows)
    ref_q = _pool_arm(results, "qb", rates, windows)
    out = {"rates_cr_per_s": [float(f"{r:g}") for r in rates], "window_s": args.latency_window_s,
           "windows_per_arm": windows, "order": "A B B A (this, reference, reference, this)",
           "arrivals": "poisson (open loop)",
           # kube-lite's watch write coalescing during the windows (null: kube-lite's own setting)
           "kube_lite_watch_coalesce_us": args.latency_watch_coalesce_us if args.latency_watch_coalesce_us >= 0 else None,
           "this": this_q}
    if ref_q:
        out["reference_controller"] = ref_q
        out["this_over_reference"] = _compare_at_rate(this_q, ref_q)
    att = {}
    for arm, prefix in (("this", "qa"), ("reference_controller", "qb")):
        per = {}
        for i, r in enumerate(rates):
            ws = [results[f"{prefix}{i}w{k}"].get("attribution") for k in range(windows)
                  if results.get(f"{prefix}{i}w{k}")]
            if any(ws):
                per[f"{r:g}"] = ws
        if per:
            att[arm] = per
    if att:
        out["attribution"] = att
    return out


def _compare_at_rate(this, ref):
    """Per rate: this build's latency over the reference arm's (< 1 = this build lower)."""
    out = {}
    for rate, t in this.items():
        r = ref.get(rate)
        if not r:
            continue
        row = {}
        for k in ("reconcile_p99_ms", "admission_p50_ms", "apply_to_ready_p99_ms"):
            if t.get(k) and r.get(k):
                row[k.replace("_ms", "_ratio")] = round(t[k] / r[k], 3)
        row["this_lower_reconcile_p99"] = bool(t.get("reconcile_p99_ms") is not None and r.get("reconcile_p99_ms")
                                               and t["reconcile_p99_ms"] < r["reconcile_p99_ms"])
        row["this_lower_admission_p50"] = bool(t.get("admission_p50_ms") is not None and r.get("admission_p50_ms")
                                               and t["admission_p50_ms"] < r["admission_p50_ms"])
        # window by window (this build's k-th window against the reference arm's k-th)
        tw, rw = t.get("windows") or [], r.get("windows") or []
        pairs = list(zip(tw, rw))
        if pairs:
            row["reconcile_p99_lower_by_window"] = [bool(a.get("reconcile_p99_ms") is not None and b.get("reconcile_p99_ms")
                                                         and a["reconcile_p99_ms"] < b["reconcile_p99_ms"])
                                                    for a, b in pairs]
            row["apply_to_ready_p99_ms_by_window"] = [[a.get("apply_to_ready_p99_ms"), b.get("apply_to_ready_p99_ms")]
                                                      for a, b in pairs]
        out[rate] = row
    return out


def _xgmi_probe(d, args):
    """RCCL all-reduce over the ranks' GPUs (N5, parallel/rccl_probe.py), after the timed
    region: busbw per size, exact results, hive placement and the bytes amdsmi saw on each
    GPU's xGMI links. Only with N>1 ranks on GPUs; a failure is reported, not raised."""
    sizes = [float(x) for x in args.xgmi_probe_mb.split(",") if x]
    if d.world < 2 or not d.cuda or not sizes:
        return None
    try:
        from ..parallel.rccl_probe import sweep

        r = sweep(sizes, iters=5, warmup=2)
        return {k: r[k] for k in ("world_size", "single_hive", "traffic_on_xgmi", "all_correct",
                                  "max_busbw_gbps", "results", "hives", "xgmi_traffic")}
    except Exception as e:  # noqa: BLE001
        return {"error": f"{type(e).__name__}: {e}"}


class _Phase:
    """One timed phase: key (tenant-name prefix), in-flight creates per rank, API server ->
    webhook protocol, controller semantics, kube-lite write latency, warmup and timed steps.
    With `rate`, an open-loop phase at that offered rate instead (_rate_phase)."""

    def __init__(self, key, concurrency, protocol, semantics, write_latency_ms, warmup, steps, rate=None,
                 isolated=False):
        self.key, self.concurrency, self.protocol, self.semantics = key, concurrency, protocol, semantics
        self.write_latency_ms, self.warmup, self.steps = write_latency_ms, warmup, steps
        self.rate, self.isolated = rate, isolated


def _dump_components(cluster):
    """On a failed run: every component's state and the errors in its log, on stderr (a
    synchronizer that exits on a write error, as the reference's does, shows up here)."""
    for name, proc in cluster.procs.items():
        try:
            rc = proc.p.poll()
            text = proc.output()
            lines = text.splitlines()
            errors = [l for l in lines if " ERROR " in l or " WARN " in l][-15:]
            tail = lines[-5:] if rc is not None else []
            print(f"[bench] component {name}: pid {proc.p.pid}, {'running' if rc is None else f'exited {rc}'}",
                  file=sys.stderr)
            for l in errors + [t for t in tail if t not in errors]:
                print(f"[bench]   {name}: {l[:400]}", file=sys.stderr)
        except Exception as e:  # noqa: BLE001
            print(f"[bench] component {name}: state unavailable ({e})", file=sys.stderr)


FIXTURES = ("apiserver",)  # kube-lite; the load driver and the fake Google run in the bench process


def _pin_process(pid, cpus):
    """Every thread of `pid` onto `cpus` (threads it starts later inherit their creator's)."""
    for tid in os.listdir(f"/proc/{pid}/task"):
        try:
            os.sched_setaffinity(int(tid), cpus)
        except OSError:
            pass


def isolation_split(cpus, cpu_ms):
    """(fixture CPUs, product CPUs): `cpus` split in proportion to the CPU time per CR the
    fixtures (kube-lite + load driver) and the shipped binaries spent in the headline phase."""
    cpus = sorted(cpus)
    fixture = (cpu_ms.get("kube_lite") or 0.0) + (cpu_ms.get("load_driver") or 0.0)
    product = cpu_ms.get("product_total") or 0.0
    share = fixture / (fixture + product) if fixture + product > 0 else 0.5
    n_fix = min(len(cpus) - 1, max(1, int(round(len(cpus) * share))))
    return cpus[:n_fix], cpus[n_fix:]


class _Isolated:
    """Context: kube-lite and this process (load driver, fake Google) on the fixture CPUs,
    the four shipped binaries on the rest; every process back on `cpus` afterwards."""

    def __init__(self, cluster, cpus, cpu_ms):
        self.cluster, self.cpus = cluster, sorted(cpus)
        self.fixture, self.product = isolation_split(self.cpus, cpu_ms)

    def __enter__(self):
        for name, proc in self.cluster.procs.items():
            _pin_process(proc.p.pid, self.fixture if name in FIXTURES else self.product)
        _pin_process(os.getpid(), self.fixture)
        return self

    def __exit__(self, *exc):
        for proc in self.cluster.procs.values():
            _pin_process(proc.p.pid, self.cpus)
        _pin_process(os.getpid(), self.cpus)


def pin_to_quota(d=None):
    """Pins every thread of this process (and so the control plane it starts) to
    quota_cpuset(), chosen on rank 0 and shared with every rank (the quota covers the whole
    job); the CPU list, or None when no pinning is needed."""
    cs = quota_cpuset() if d is None or d.rank == 0 else None
    if d is not None:
        cs = d.broadcast_obj(cs)
    if cs:
        for tid in os.listdir("/proc/self/task"):
            try:
                os.sched_setaffinity(int(tid), cs)
            except OSError:
                pass
    return cs


def run(args):
    t_run = time.monotonic()
    d = Dist()
    n = args.gpus if args.gpus else d.world
    # every rank pins itself to the same CPUs: the quota covers the whole job
    cpuset = pin_to_quota(d) if args.pin_to_quota else None
    from bacchus_gpu_controller_amd import native
    from bacchus_gpu_controller_amd.testing.cluster import Cluster
    from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle

    nat = native()
    if args.trace_windows:
        nat.stall_start("load-driver")  # the load generator's own stalls, next to the services'
    cluster = google = None
    info = None
    cpus = effective_cpus()
    tuned = args.tuned_concurrency if args.tuned_concurrency > 0 else auto_concurrency(d.world, cpus)
    # BASELINE config #3 is 100 concurrent CRs on the node: by default that total is split
    # over the ranks (ceil), so N load generators offer the same in-flight load as one
    conc = args.concurrency if args.concurrency_scope == "rank" else max(1, -(-args.concurrency // d.world))
    semantics0 = "reference" if args.reference_semantics else args.semantics
    phases = [_Phase("m", conc, args.webhook_protocol, semantics0, args.write_latency_ms, args.warmup, args.steps)]
    # The secondary closed-loop phases (tuned concurrency, HTTP/1.1 webhook, the 2 ms
    # write-latency arms) run at N=1 only: at N ranks each does N times the work (weak
    # scaling) and the scaling runs report the headline alone.  They run last, and only
    # while the run's wall time stays inside --time-budget-s.
    secondary = d.world == 1
    if args.isolated_phase and d.world == 1:
        # the headline again, with the fixtures (kube-lite, load driver) and the product on
        # disjoint CPUs: how much of the headline latencies is queueing behind the fixtures
        phases.append(_Phase("pi", conc, args.webhook_protocol, semantics0, args.write_latency_ms,
                             args.warmup, args.steps, isolated=True))
    semantics = "reference" if args.reference_semantics else args.semantics
    rates = [float(x) for x in args.latency_rates.split(",") if x.strip()]
    windows = max(1, args.latency_windows)
    # Open loop at equal offered load, the arms interleaved A B B A: this
    # build's first window per rate, the reference-controller arm's windows, then this
    # build's remaining windows, so drift of the box over the run hits both arms alike.
    qa = lambda k: [_Phase(f"qa{i}w{k}", 0, args.webhook_protocol, semantics0, args.write_latency_ms, 0, 0,  # noqa: E731
                           rate=r) for i, r in enumerate(rates)]
    if rates:
        phases += qa(0)
    if args.reference_arms and semantics == "this":
        # same-stack comparison, timed like the headline: the reference's controller
        # behaviour (controller.rs:81-154: sequential, unconditional applies) on this stack,
        # at the headline's storage latency and with a write-latency (etcd commit) model
        phases.append(_Phase("rc", conc, args.webhook_protocol, "reference-controller", args.write_latency_ms,
                             args.warmup, args.steps))
        # ... then the reference controller's windows at the same rates, while it runs
        phases += [_Phase(f"qb{i}w{k}", 0, args.webhook_protocol, "reference-controller", args.write_latency_ms, 0, 0,
                          rate=r) for k in range(windows) for i, r in enumerate(rates)]
        if args.arm_write_latency_ms > 0 and secondary:
            phases.append(_Phase("rl", conc, args.webhook_protocol, "reference-controller",
                                 args.arm_write_latency_ms, args.arm_warmup, args.arm_steps))
        for k in range(1, windows):
            phases += qa(k)
        if args.arm_write_latency_ms > 0 and secondary:
            phases.append(_Phase("ml", conc, args.webhook_protocol, "this", args.arm_write_latency_ms,
                                 args.arm_warmup, args.arm_steps))
    else:
        for k in range(1, windows):
            phases += qa(k)
    if args.tuned_phase and tuned != conc and secondary:
        phases.append(_Phase("t", tuned, args.webhook_protocol, semantics0, args.write_latency_ms,
                             args.warmup, args.steps))
    if args.http1_phase and args.webhook_protocol == "h2" and secondary:
        # secondary: the same load with the webhook called over HTTP/1.1 (keep-alive pool)
        phases.append(_Phase("w", conc, "http/1.1", semantics0, args.write_latency_ms, args.warmup, args.steps))
    optional = {"rl", "ml", "t", "w"}
    # Reconcile/sync workers spend most of their time waiting on API round trips, so they
    # are not sized to the CPU share like the offered load is: the services' defaults
    # (CONF_WORKERS: controller 8, synchronizer 8; profiles/r6_workers_ab/)
    controller_workers = args.controller_workers or 8
    sync_workers = args.sync_workers or 8

    def controller_env(sem):
        env = {"CONF_WORKERS": str(controller_workers)}
        env.update(dict(kv.split("=", 1) for kv in args.controller_env))
        if sem in ("reference", "reference-controller"):
            # the reference's controller on this same stack: children applied one after
            # another and re-applied on every reconcile (controller.rs:81-149)
            env.update({"CONF_SKIP_UNCHANGED": "false", "CONF_PARALLEL_CHILDREN": "false",
                        "CONF_LABEL_CHILDREN": "false",  # .owns() on every object of each kind
                        "CONF_DEBOUNCE_MS": "0"})  # every event reconciles at once
        return env

    if d.rank == 0:
        google = FakeGoogle().start()
        rows = []
        if not args.approve_after_create:
            # pre-approved sheet: every tenant's row is marked O before it applies
            rows = [{"id_username": name} for r in range(d.world) for p in phases if p.rate is None
                    for s in range((p.warmup + p.steps) * args.rounds)
                    for name in _names(r, p.key, s, args.batch)]
        # ... and the warm-up tenants of a rate window that follows a controller restart
        sem = semantics
        for p in phases:
            if controller_env(p.semantics) != controller_env(sem):
                sem = p.semantics
                if p.rate is not None and args.restart_warmup_steps > 0:
                    rows += [{"id_username": name} for r in range(d.world)
                             for s in range(args.restart_warmup_steps * args.rounds)
                             for name in _names(r, f"x{p.key}", s, args.batch)]
        # the open-loop phases' tenants are pre-approved in either flow
        for p in phases:
            if p.rate is not None:
                per_rank = p.rate / d.world
                for r in range(d.world):
                    for part, secs in (("w", args.latency_warmup_s), ("t", args.latency_window_s)):
                        rows += [{"id_username": name} for name in
                                 _rate_names(r, p.key, p.rate, part, max(1, int(round(per_rank * secs))))]
        if rows:
            google.set_rows(rows)
        ctrl_env = controller_env(semantics)
        sync_env = {"CONF_WATCH": "true", "CONF_WORKERS": str(sync_workers), "RUST_LOG": args.log_level,
                    "CONF_SHEET_POLL_MS": str(args.sheet_poll_ms)}
        if semantics == "reference":
            # ... and its synchronizer: sheet read only on the periodic tick
            # (synchronizer.rs:192), every tick rewrites every matched tenant
            sync_env.update({"CONF_WATCH": "false", "CONF_SKIP_UNCHANGED": "false"})
        apiserver_args = list(args.apiserver_arg)
        if args.write_latency_ms > 0:
            apiserver_args += ["--write-latency-ms", str(args.write_latency_ms)]
        if args.webhook_protocol == "h2" and "--webhook-http2" not in apiserver_args:
            # what a real apiserver negotiates with the admission server (ALPN h2, one
            # multiplexed connection): the production webhook transport
            apiserver_args.append("--webhook-http2")
        cluster = Cluster(controller_env=ctrl_env, log_level=args.log_level, tls_apiserver=args.tls_apiserver,
                          apiserver_args=apiserver_args,
                          admission_env=dict(kv.split("=", 1) for kv in args.admission_env))
        cluster.start()
        cluster.start_synchronizer(google, interval=args.sync_interval, extra_env=sync_env)
        cluster.start_node_agent(max_gpus=n, n_mock_gpus=n, poll_interval_ms=args.poll_ms,
                                 extra_env={"RUST_LOG": args.log_level})
        info = {"server": cluster.server, "controller": f"http://127.0.0.1:{cluster.controller_port}",
                "admission": f"https://127.0.0.1:{cluster.admission_port}",
                "ca": os.path.join(cluster.cert_dir, "ca.crt"),
                "node_agent": f"http://127.0.0.1:{cluster.node_agent_port}",
                "synchronizer": f"http://127.0.0.1:{cluster.sync_port}",
                "apiserver_ca": open(cluster.apiserver_ca).read() if args.tls_apiserver else "",
                "apiserver_verify": cluster.verify,
                "approve_url": google.base + "/_fake/rows" if args.approve_after_create else ""}
    info = d.broadcast_obj(info)
    try:
        results = {}
        running = semantics  # controller semantics of the running controller
        latency = args.write_latency_ms  # kube-lite's current storage latency
        phase_wall = {"setup": round(time.monotonic() - t_run, 2)}  # wall seconds per phase (rank 0's view)
        skipped = []
        restarted = False
        for p in phases:
            t_phase = time.monotonic()
            if p.key in optional and args.time_budget_s > 0:
                # an estimate from the headline's pace: a closed-loop step at the 2 ms write
                # latency takes about 6x a headline step
                per_step = phase_wall["m"] / max(1, args.warmup + args.steps)
                est = per_step * (p.warmup + p.steps) * (6 if p.write_latency_ms > 0 else 1)
                if p.key == "rl":
                    # the write-latency pair goes together: rl only if ml still fits after it
                    # and after the open-loop windows that always run in between
                    later = phases[phases.index(p) + 1:]
                    ml = next((q for q in later if q.key == "ml"), None)
                    if ml is not None:
                        between = [q for q in later[:later.index(ml)] if q.key not in optional]
                        rate_walls = [phase_wall[q.key] for q in phases if q.rate is not None and q.key in phase_wall]
                        per_window = sum(rate_walls) / len(rate_walls) if rate_walls else 3.0
                        est += len(between) * per_window + per_step * (ml.warmup + ml.steps) * 6
                over = d.max_scalar(time.monotonic() - t_run + est) > args.time_budget_s
                if p.key == "ml":  # the write-latency pair goes together (decided at rl)
                    over = "rl" in skipped
                if over:
                    skipped.append(p.key)
                    continue
            if d.rank == 0:
                import requests

                requests.post(info["server"] + "/_kl/webhook-protocol", data=p.protocol, timeout=10,
                              verify=info["apiserver_verify"]).raise_for_status()
                if p.write_latency_ms != latency:
                    requests.post(info["server"] + "/_kl/write-latency-us", data=str(int(p.write_latency_ms * 1000)),
                                  timeout=10, verify=info["apiserver_verify"]).raise_for_status()
                    latency = p.write_latency_ms
                if controller_env(p.semantics) != controller_env(running):
                    # the other controller behaviour: a fresh controller process, which
                    # re-lists every object like any controller start
                    cluster.procs["controller"].stop()
                    cluster.controller_env = controller_env(p.semantics)
                    cluster.start_controller()
                    info["controller"] = f"http://127.0.0.1:{cluster.controller_port}"
                    running = p.semantics
                    restarted = True
            restarted = d.broadcast_obj(restarted)
            d.barrier()
            if p.rate is not None and restarted and args.restart_warmup_steps > 0:
                # A freshly started controller has no pooled API connections (each worker
                # dials and handshakes TLS on its first requests, kube-lite spawns a thread
                # per connection) and verifies every owner's children on its first reconcile:
                # its first second is not its steady state (10-20 ms apply->Ready tails in
                # the first window after a restart, profiles/r6_tails/).  Untimed closed-loop
                # steps warm it, as the reference arm's closed-loop phase warms it before its
                # windows.
                _warm(d, nat, info, args, f"x{p.key}", conc, args.restart_warmup_steps)
            restarted = False
            if p.rate is not None:
                results[p.key] = _rate_phase(d, nat, info, args, p.key, p.rate, cluster)
                if results[p.key] is not None:
                    results[p.key]["semantics"] = p.semantics
                phase_wall[p.key] = round(time.monotonic() - t_phase, 2)
                continue
            if p.isolated:
                _settle(info)
                cpus = cpuset or sorted(os.sched_getaffinity(0))
                with _Isolated(cluster, cpus, results["m"]["cpu_ms_per_cr"]) as iso:
                    results[p.key] = _phase(d, nat, info, args, p.key, p.concurrency, p.warmup, p.steps, cluster)
                results[p.key]["cpus"] = {"fixtures": _cpulist_text(iso.fixture), "product": _cpulist_text(iso.product)}
            else:
                results[p.key] = _phase(d, nat, info, args, p.key, p.concurrency, p.warmup, p.steps, cluster)
            if results[p.key] is not None:
                results[p.key]["semantics"] = p.semantics
                results[p.key]["apiserver_write_latency_ms"] = p.write_latency_ms
            phase_wall[p.key] = round(time.monotonic() - t_phase, 2)
        xgmi = _xgmi_probe(d, args)
        if d.rank != 0:
            return None
        main_r = results["m"]
        gpu_tel = _gpu_telemetry(info["node_agent"])
        elapsed = main_r.pop("elapsed_s")
        for k in ("steps", "warmup", "semantics", "apiserver_write_latency_ms"):
            main_r.pop(k, None)  # in the top-level fields and config already
        model = ("UserBootstrap onboarding churn (kube-lite" + (" over HTTPS" if args.tls_apiserver else "")
                 + " + TLS admission + controller + synchronizer + MI355X node-agent)")
        flow = "create->approve->Ready" if args.approve_after_create else "pre-approved sheet"
        out = {
            "metric": METRIC,
            "value": main_r.pop("value"),
            "unit": "CR/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # a control plane: no tensor math, so no compute dtype (BASELINE names none)
            "dtype": "none",
            "data": "synthetic tenants (UserBootstrap CRs), fake Google sheet",
            "config": {"model": model, "global_batch": args.batch * args.rounds * d.world, "seq_len": None,
                       "rounds_per_step": args.rounds, "tenants_per_round": args.batch,
                       "parallelism": f"dp{d.world}", "semantics": semantics, "flow": flow,
                       "concurrency_per_rank": conc, "concurrency_total": conc * d.world,
                       "concurrency_scope": args.concurrency_scope, "log_level": args.log_level,
                       "apiserver_write_latency_ms": args.write_latency_ms, "control_plane_cpus": cpus,
                       "controller_workers": controller_workers, "sync_workers": sync_workers,
                       "sheet_poll_ms": args.sheet_poll_ms, "sync_interval_s": args.sync_interval,
                       # API server -> webhook protocol of the headline phase: h2 (what the
                       # admission server's ALPN gives a real apiserver) unless --webhook-protocol
                       "webhook_protocol": args.webhook_protocol,
                       "driver_protocol": "h2" if args.driver_http2 and args.tls_apiserver else "http/1.1",
                       # each rank's load driver watches only its own tenants' children
                       # (kube-lite name-prefix field selector); the product is unaffected
                       "driver_server_filter": args.driver_server_filter,
                       # CPUs the job was pinned to (quota_cpuset), or null when not pinned
                       "cpuset": _cpulist_text(cpuset) if cpuset else None,
                       # the job's CPUs grouped by shared L3: the scheduler places a woken
                       # thread within its waker's group first
                       "cpu_llc_groups": llc_groups(sorted(os.sched_getaffinity(0)))},
        }
        out.update(main_r)
        if "t" in results:
            # secondary: same stack, offered load sized to the CPU share (auto_concurrency)
            t = results["t"]
            out["tuned"] = {k: t.get(k) for k in ("value", "concurrency_per_rank", "reconcile_p99_ms",
                                                  "admission_p50_ms", "apply_to_ready_p50_ms",
                                                  "apply_to_ready_p99_ms", "cpu_ms_per_cr", "failed_crs")}
        if "pi" in results:
            pi = results["pi"]
            out["product_isolated"] = {k: pi.get(k) for k in (
                "value", "cpus", "reconcile_p99_ms", "reconcile_p50_ms", "admission_p50_ms", "admission_p99_ms",
                "admission_handler_p50_ms", "admission_h2_server_p50_ms", "apply_to_ready_p50_ms",
                "apply_to_ready_p99_ms", "cpu_ms_per_cr", "cgroup_throttled", "failed_crs")}
        if "w" in results:
            w = results["w"]
            out["webhook_http1"] = {k: w.get(k) for k in ("value", "admission_p50_ms", "admission_p99_ms",
                                                          "admission_handler_p50_ms", "reconcile_p99_ms",
                                                          "apply_to_ready_p50_ms", "failed_crs")}
        arm_keys = ("value", "steps", "warmup", "semantics", "apiserver_write_latency_ms", "reconcile_p99_ms",
                    "reconcile_p50_ms", "reconciles", "reconcile_total_delta", "admission_p50_ms",
                    "apply_to_ready_p50_ms", "apply_to_ready_p99_ms", "apiserver_requests_per_cr", "cpu_ms_per_cr",
                    "ready_crs", "failed_crs")
        arm = lambda r: {k: r.get(k) for k in arm_keys}  # noqa: E731
        ratio = lambda a, b: round(a / b, 3) if a and b else None  # noqa: E731
        if "rc" in results:
            # same stack, the reference's controller behaviour (an emulation, not a published
            # number: vs_baseline stays null)
            rc = arm(results["rc"])
            rc["this_over_reference_cr_per_s"] = ratio(out["value"], rc["value"])
            out["reference_controller"] = rc
        if "rl" in results and "ml" in results:
            this_l, ref_l = arm(results["ml"]), arm(results["rl"])
            out[f"write_latency_{args.arm_write_latency_ms:g}ms"] = {
                "this": this_l, "reference_controller": ref_l,
                "this_over_reference_cr_per_s": ratio(this_l["value"], ref_l["value"])}
        if rates:
            out["latency_at_rate"] = _latency_at_rate(results, rates, windows, args)
        # amdsmi counters of the advertised GPUs at the end of the timed region (node agent)
        out["gpu_telemetry"] = gpu_tel
        phase_wall["total"] = round(time.monotonic() - t_run, 2)
        out["phase_wall_s"] = phase_wall
        if skipped:  # secondary phases left out to keep the run inside --time-budget-s
            out["skipped_phases"] = skipped
        if xgmi is not None:
            out["rccl_xgmi"] = xgmi
        out["reference_structural"] = {"apply_to_ready_p50_s": 30.0, "apply_to_ready_p99_s": 59.4,
                                       "note": "reference gates readiness on a 60 s sheet poll (synchronizer.rs:192)"}
        if args.report_cpu and cluster is not None:
            out["component_rss_mb"] = {name: _rss_mb(p.p.pid) for name, p in cluster.procs.items()}
            try:
                st = cluster.stats()
                out["apiserver_objects"] = {"live": st.get("objects"), "gc_collected": st.get("gc_collected"),
                                            "gc_pending": st.get("gc_pending")}
            except Exception:  # noqa: BLE001
                pass
            try:  # the periodic malloc_trim pass of each process (core/process.cc), kube-lite included
                import requests

                trims, heap = {}, {}
                for comp, url, verify in (("controller", info["controller"], None),
                                          ("admission", info["admission"], info["ca"]),
                                          ("synchronizer", info["synchronizer"], None),
                                          ("node_agent", info["node_agent"], None),
                                          ("kube_lite", info["server"], info["apiserver_verify"])):
                    txt = requests.get(url + "/metrics", timeout=10, verify=verify).text
                    vals = {l.split()[0]: float(l.split()[1]) for l in txt.splitlines()
                            if l.startswith(("bgc_malloc_trim_seconds_sum", "bgc_malloc_trim_seconds_count",
                                             "bgc_malloc_trim_last_seconds", "bgc_heap_"))}
                    trims[comp] = {"passes": int(vals.get("bgc_malloc_trim_seconds_count", 0)),
                                   "total_ms": round(vals.get("bgc_malloc_trim_seconds_sum", 0.0) * 1e3, 3),
                                   "last_ms": round(vals.get("bgc_malloc_trim_last_seconds", 0.0) * 1e3, 3)}
                    # live malloc data vs free space the arenas hold (RSS alone cannot tell them apart)
                    heap[comp] = {"allocated_mb": round(vals.get("bgc_heap_allocated_bytes", 0.0) / 1e6, 1),
                                  "free_mb": round(vals.get("bgc_heap_free_bytes", 0.0) / 1e6, 1)}
                out["malloc_trim"] = trims
                out["component_heap_mb"] = heap
            except Exception:  # noqa: BLE001
                pass
            try:  # controller cache sizes (bounded-memory check under churn)
                import requests

                txt = requests.get(info["controller"] + "/metrics", timeout=10).text
                out["controller_gauges"] = {l.split()[0]: float(l.split()[1]) for l in txt.splitlines()
                                            if l.startswith(("bgc_controller_apply_cache_entries",
                                                             "bgc_controller_queue_depth", "bgc_heap_",
                                                             "bgc_controller_owner_state_entries",
                                                             "bgc_controller_store_objects",
                                                             "bgc_reconcile_total", "bgc_reconcile_fast_total",
                                                             "bgc_apply_total", "bgc_apply_skipped_total",
                                                             "bgc_controller_own_write_events_total"))}
            except Exception:  # noqa: BLE001
                pass
        if rates and args.trace_windows:
            # last, so the driver's 2,000-character tail of the output keeps it: the per-stage
            # table of each arm (full tables in latency_at_rate.attribution)
            out["stage_table"] = {"this": _stage_summary(results, "qa", rates, windows),
                                  "reference_controller": _stage_summary(results, "qb", rates, windows)}
        return out
    except BaseException:
        if cluster is not None:
            _dump_components(cluster)
        raise
    finally:
        if cluster is not None:
            cluster.stop()
        if google is not None:
            google.stop()
        d.close()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    # a step is 10 rounds of 100 tenants per rank, ~120 ms at N=1: the driver's 20 timed
    # steps span ~2.5 s, long enough for a stable rate and p99, while no more than 100
    # tenants per rank are ever on their way to Ready at once (BASELINE config #3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=100, help="UserBootstraps applied per rank per round")
    ap.add_argument("--rounds", type=int, default=12,
                    help="rounds of --batch tenants per step (12: the 20 timed steps span >= 2.4 s even at 10k CR/s)")
    ap.add_argument("--concurrency", type=int, default=100,
                    help="in-flight creates (BASELINE config #3: 100 concurrent CRs on the node)")
    ap.add_argument("--concurrency-scope", choices=("total", "rank"), default="total",
                    help="total: --concurrency is split over the ranks; rank: every rank keeps that many in flight")
    ap.add_argument("--tuned-phase", action=argparse.BooleanOptionalAction, default=True,
                    help="also measure a secondary phase with the offered load sized to the CPU share")
    ap.add_argument("--tuned-concurrency", type=int, default=0, help="0 = auto_concurrency()")
    ap.add_argument("--webhook-protocol", choices=("h2", "http/1.1"), default="h2",
                    help="API server -> admission webhook transport of the headline phase")
    ap.add_argument("--isolated-phase", action=argparse.BooleanOptionalAction, default=True,
                    help="N=1: also time the headline with kube-lite and the load driver on CPUs of their own, "
                         "apart from the shipped binaries (product_isolated; split by the headline's CPU per CR)")
    ap.add_argument("--http1-phase", action=argparse.BooleanOptionalAction, default=True,
                    help="with --webhook-protocol h2: also time the webhook over HTTP/1.1 (secondary field)")
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--controller-workers", type=int, default=0, help="0 = 8 (the controller's default)")
    ap.add_argument("--sync-workers", type=int, default=0, help="0 = 8 (the synchronizer's default)")
    ap.add_argument("--poll-ms", type=int, default=250)
    ap.add_argument("--log-level", default="info", help="RUST_LOG of every service (chart default: info)")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--driver-server-filter", action=argparse.BooleanOptionalAction, default=True,
                    help="per-rank load drivers ask kube-lite to filter their child watches by tenant-name "
                         "prefix (no N-fold watch fan-out from the load generators themselves)")
    ap.add_argument("--xgmi-probe-mb", default="16,256",
                    help="N>1 GPUs: all-reduce sizes (MiB) for the RCCL/xGMI probe after the timed region ('' = off)")
    ap.add_argument("--semantics", choices=("this", "reference", "reference-controller"), default="this",
                    help="reference: the reference's controller and synchronizer behaviour on this stack "
                         "(periodic sheet sync only, sequential unconditional child applies); "
                         "reference-controller: only the controller side")
    ap.add_argument("--reference-semantics", action="store_true", help="alias for --semantics reference")
    ap.add_argument("--pin-to-quota", action=argparse.BooleanOptionalAction, default=True,
                    help="when the cgroup CPU quota grants fewer CPUs than are visible, run the job on that "
                         "many CPUs (quota_cpuset) instead of bursting over all of them and being throttled")
    ap.add_argument("--reference-arms", action=argparse.BooleanOptionalAction, default=True,
                    help="also time the reference's controller behaviour on this stack (reference_controller) "
                         "and both controllers at --arm-write-latency-ms (secondary fields)")
    ap.add_argument("--arm-write-latency-ms", type=float, default=2.0,
                    help="kube-lite storage commit latency of the write-latency arms (0 = no such arms)")
    ap.add_argument("--arm-steps", type=int, default=5, help="timed steps of each write-latency arm")
    ap.add_argument("--arm-warmup", type=int, default=1, help="warmup steps of each write-latency arm")
    ap.add_argument("--time-budget-s", type=float, default=54.0,
                    help="wall seconds of the run after which the secondary phases (write-latency arms, tuned, "
                         "HTTP/1.1 webhook) are skipped (listed in skipped_phases); 0 = no budget")
    ap.add_argument("--latency-rates", default="2000,6000",
                    help="open-loop offered rates (CR/s, whole job) at which this build and the reference-controller "
                         "arm are both timed (latency_at_rate; '' = none)")
    ap.add_argument("--latency-window-s", type=float, default=1.0, help="timed window of each open-loop phase")
    ap.add_argument("--latency-warmup-s", type=float, default=0.5, help="untimed lead-in of each open-loop phase")
    ap.add_argument("--latency-windows", type=int, default=2,
                    help="timed windows per rate and arm, interleaved A B B A with the reference-controller arm")
    ap.add_argument("--trace-windows", action=argparse.BooleanOptionalAction, default=True,
                    help="trace every tenant of each open-loop window through every process and attribute its "
                         "apply->Ready time to stages (latency_at_rate.attribution; bench/attribution.py)")
    ap.add_argument("--restart-warmup-steps", type=int, default=3,
                    help="untimed closed-loop steps that warm a restarted controller before an open-loop window")
    ap.add_argument("--trace-dump", default="",
                    help="directory: per open-loop window, the worst tail tenants' full timelines and every mark "
                         "around the worst one (bench/attribution.py analyze(detail=...))")
    ap.add_argument("--tail-ms", type=float, default=5.0,
                    help="attribution: tenants above max(p99, this) apply->Ready are the window's tail")
    ap.add_argument("--latency-watch-coalesce-us", type=int, default=0,
                    help="kube-lite's watch write coalescing during the open-loop windows (-1 = leave it at "
                         "kube-lite's setting, 50 us; the closed-loop phases keep that): a timed hold per event "
                         "that overshoots to ms under load (profiles/r6_coalesce_ab/)")
    ap.add_argument("--latency-workers", type=int, default=128,
                    help="open loop: threads issuing creates per rank (arrivals never wait for one below ~that "
                         "many in flight)")
    ap.add_argument("--approve-after-create", action="store_true",
                    help="tenants apply first; each step's batch is approved by one sheet edit once its "
                         "Namespaces exist (the reference's onboarding order); times create->approve->Ready")
    ap.add_argument("--sheet-poll-ms", type=int, default=5000,
                    help="synchronizer Drive version poll (CONF_SHEET_POLL_MS; product default 5000)")
    ap.add_argument("--write-latency-ms", type=float, default=0.0,
                    help="kube-lite storage commit latency per write (etcd model)")
    ap.add_argument("--sync-interval", type=int, default=60, help="synchronizer tick (s); the reference default is 60")
    ap.add_argument("--apiserver-arg", action="append", default=[], help="extra kube-lite flag (repeatable)")
    ap.add_argument("--controller-env", action="append", default=[], metavar="CONF_X=V",
                    help="extra controller environment (repeatable), e.g. CONF_METADATA_WATCHES=false")
    ap.add_argument("--admission-env", action="append", default=[], metavar="CONF_X=V",
                    help="extra admission environment (repeatable), e.g. CONF_HTTP2_INLINE=false")
    ap.add_argument("--report-cpu", action="store_true", help="add RSS, object counts and controller gauges")
    ap.add_argument("--driver-http2", action=argparse.BooleanOptionalAction, default=False,
                    help="tenant load over HTTP/2 multiplexed connections (profiles/archive/http2_r2/: no gain at N=1, "
                         "worse at N=8 on kube-lite)")
    ap.add_argument("--tls-apiserver", action=argparse.BooleanOptionalAction, default=True,
                    help="components reach kube-lite over HTTPS via kubeconfigs, as in a real cluster")
    args = ap.parse_args(argv)
    out = run(args)
    if out is not None:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
