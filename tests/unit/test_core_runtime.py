"""Core runtime pieces: work queue semantics, RUST_LOG targets, envy config, kubeconfig,
crypto helpers (checked against Python stdlib / the openssl CLI)."""
import base64
import hashlib
import os
import re
import subprocess
import tempfile
import threading
import time

import pytest


def test_workqueue_dedup_and_delay(nat):
    q = nat.WorkQueue()
    q.add("a")
    q.add("a")
    q.add_after("b", 50)
    assert q.pending() == 2
    assert q.get() == "a"
    t0 = time.time()
    assert q.get() == "b"
    assert time.time() - t0 >= 0.04
    q.done("a")
    q.done("b")


def test_workqueue_earliest_due_wins(nat):
    q = nat.WorkQueue()
    q.add_after("k", 5000)   # requeue(30s)-style entry
    q.add("k")               # event arrives: run now
    t0 = time.time()
    assert q.get() == "k"
    assert time.time() - t0 < 1.0
    q.done("k")
    assert q.pending() == 0  # the later entry was superseded, not duplicated


def test_workqueue_per_key_exclusivity(nat):
    q = nat.WorkQueue()
    q.add("x")
    assert q.get() == "x"
    q.add("x")                       # re-added while in flight: deferred
    got = []
    th = threading.Thread(target=lambda: got.append(q.get()))
    th.start()
    time.sleep(0.1)
    assert not got                   # not handed to a second worker
    q.done("x")
    th.join(2)
    assert got == ["x"]
    q.done("x")
    q.shutdown()
    assert q.get() is None


def test_workqueue_shards_keep_per_key_semantics(nat):
    """A sharded queue (round 6: one lock per shard, worker i serves shard i % shards): every
    key is served by its shard's workers, once, with dedup, delay and exclusivity intact."""
    assert [nat.WorkQueue.shards_for(w) for w in (1, 4, 16, 64)] == [1, 1, 1, 1]  # BGC_QUEUE_SHARDS unset
    q = nat.WorkQueue(4)
    assert q.shards() == 4
    keys = [f"k{i}" for i in range(64)]
    for k in keys:
        q.add(k)
        q.add(k)  # dedup within the key's shard
    assert q.pending() == 64
    got, lock = {}, threading.Lock()

    def worker(i):
        while True:
            k = q.get(i)
            if k is None:
                return
            with lock:
                got.setdefault(i % 4, []).append(k)
                first_k0 = k == "k0" and sum(v.count("k0") for v in got.values()) == 1
            if first_k0:
                q.add(k)  # re-added while in flight: deferred until done
            q.done(k)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ths:
        t.start()
    deadline = time.time() + 5
    while q.pending() or q.in_flight():
        assert time.time() < deadline, (q.pending(), q.in_flight())
        time.sleep(0.01)
    q.shutdown()
    for t in ths:
        t.join(2)
    served = [k for v in got.values() for k in v]
    # every key once, k0 once more (its re-add while in flight ran after done), each within one shard
    assert sorted(served) == sorted(keys + ["k0"])
    for shard, ks in got.items():  # a key is served by one shard only
        assert all(sum(k in got[s] for s in got) == 1 for k in ks), shard
    assert set(got) == {0, 1, 2, 3}  # the keys spread over all four shards


def test_workqueue_no_lost_wakeup_behind_a_far_timer(nat):
    """Bursts of adds while a timer waiter is parked on a 30 s requeue: every key is dequeued
    promptly.  A woken worker stays counted as idle until it re-takes the lock, so the queue
    counts its unconsumed signals; once every idle worker is signalled, a further due key
    wakes the timer waiter instead of signalling nobody (round 6)."""
    q = nat.WorkQueue(1)
    q.add_after("far", 30000)
    added, lat, lock = {}, [], threading.Lock()

    def worker(i):
        while True:
            k = q.get(i)
            if k is None:
                return
            with lock:
                if k in added:
                    lat.append(time.monotonic() - added.pop(k))
            time.sleep(0.0005)
            q.done(k)

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for t in ths:
        t.start()
    for burst in range(40):
        for j in range(8):
            k = f"b{burst}-{j}"
            with lock:
                added[k] = time.monotonic()
            q.add(k)
        time.sleep(0.003)
    deadline = time.monotonic() + 5
    while True:
        with lock:
            if not added:
                break
        assert time.monotonic() < deadline, f"{len(added)} keys never dequeued"
        time.sleep(0.01)
    q.shutdown()
    for t in ths:
        t.join(2)
    assert len(lat) == 320 and max(lat) < 1.0, max(lat)


def test_workqueue_shard_timer_and_shutdown(nat):
    q = nat.WorkQueue(2)
    q.add_after("late", 100)
    out = []
    ths = [threading.Thread(target=lambda i=i: out.append(q.get(i))) for i in range(2)]
    t0 = time.time()
    for t in ths:
        t.start()
    time.sleep(0.3)
    assert out == ["late"] and time.time() - t0 >= 0.1  # its shard's worker timed it
    q.done("late")
    q.shutdown()  # the other shard's idle worker wakes and returns None
    for t in ths:
        t.join(2)
    assert out == ["late", None]


@pytest.mark.parametrize("spec,level,target,on", [
    ("info", "info", "controller", True),
    ("info", "debug", "controller", False),
    ("warn,controller=debug", "debug", "controller", True),
    ("warn,controller=debug", "info", "admission", False),
    ("controller=trace", "info", "admission", False),     # no default => off for others
    ("kube=debug,info", "debug", "kube::watcher", True),  # module-path prefix
    ("", "info", "x", True),                              # empty => INFO default
])
def test_rust_log_targets(nat, spec, level, target, on):
    assert nat.log_enabled(spec, level, target) is on


def test_env_config_envy_semantics(nat):
    base = {"CONF_LISTEN_ADDR": "0.0.0.0", "CONF_LISTEN_PORT": "12321", "CONF_CERT_PATH": "c",
            "CONF_KEY_PATH": "k", "CONF_OIDC_USERNAME_PREFIX": "oidc:", "CONF_DEFAULT_ROLE_NAME": "edit",
            "CONF_AUTHORIZED_GROUP_NAMES": "gpu,admin"}
    d = nat.env_config(base, "admission")
    assert d["authorized_group_names"] == ["gpu", "admin"] and d["listen_port"] == 12321
    assert nat.env_config(dict(base, CONF_AUTHORIZED_GROUP_NAMES=""), "admission")["authorized_group_names"] == [""]
    assert nat.env_config(dict(base, CONF_AUTHORIZED_GROUP_NAMES=" gpu , x"), "admission")["authorized_group_names"] == [" gpu ", " x"]
    with pytest.raises(ValueError, match="missing value for field cert_path"):
        nat.env_config({k: v for k, v in base.items() if k != "CONF_CERT_PATH"}, "admission")
    with pytest.raises(ValueError, match="listen_port"):
        nat.env_config(dict(base, CONF_LISTEN_PORT="70000"), "admission")
    s = nat.env_config({"CONF_LISTEN_ADDR": "a", "CONF_LISTEN_PORT": "1", "CONF_GOOGLE_SERVICE_ACCOUNT_JSON_PATH": "p",
                        "CONF_GOOGLE_FILE_ID": "f", "CONF_GPU_SERVER_NAME": ""}, "synchronizer")
    assert s["sync_interval_secs"] == 60


def test_kubeconfig(nat, tmp_path):
    ca = base64.b64encode(b"-----BEGIN CERTIFICATE-----\nx\n-----END CERTIFICATE-----\n").decode()
    (tmp_path / "tok").write_text("file-token\n")
    (tmp_path / "config").write_text(f"""
apiVersion: v1
kind: Config
current-context: dev
clusters:
- name: c1
  cluster:
    server: https://10.0.0.1:6443
    certificate-authority-data: {ca}
- name: c2
  cluster: {{server: "http://127.0.0.1:8080", insecure-skip-tls-verify: true}}
contexts:
- name: dev
  context: {{cluster: c1, user: u1}}
- name: local
  context: {{cluster: c2, user: u2}}
users:
- name: u1
  user:
    token: abc
    as: oidc:alice
    as-groups: [gpu]
- name: u2
  user:
    tokenFile: tok
""")
    d = nat.kubeconfig_parse(str(tmp_path / "config"))
    assert d["server"] == "https://10.0.0.1:6443" and d["token"] == "abc"
    assert d["ca_pem"].startswith("-----BEGIN CERTIFICATE-----")
    assert d["impersonate_user"] == "oidc:alice" and d["impersonate_groups"] == ["gpu"]
    d2 = nat.kubeconfig_parse(str(tmp_path / "config"), "local")
    assert d2["server"] == "http://127.0.0.1:8080" and d2["insecure"] and d2["token"] == "file-token"


def test_crypto_against_stdlib(nat):
    data = os.urandom(1000)
    assert nat.sha256_hex(data) == hashlib.sha256(data).hexdigest()
    for n in range(0, 7):
        assert nat.base64_encode(data[:n]) == base64.b64encode(data[:n]).decode()
        assert nat.base64_encode(data[:n], True, False) == base64.urlsafe_b64encode(data[:n]).decode().rstrip("=")
        assert nat.base64_decode(base64.b64encode(data[:n]).decode()) == data[:n]
    assert re.fullmatch(r"[0-9a-f]{8}-[0-9a-f]{4}-4[0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}", nat.uuid_v4())


def test_uuids_unique_across_threads_and_forks(nat):
    """uuid_v4 draws from a per-thread CSPRNG pool: unique across pool refills and
    threads, and a forked child never repeats the parent's pending pool."""
    import os
    import threading
    pat = re.compile(r"[0-9a-f]{8}-[0-9a-f]{4}-4[0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}")
    seen = [nat.uuid_v4() for _ in range(1000)]  # several 4 KiB pool refills
    out = []
    ts = [threading.Thread(target=lambda: out.extend(nat.uuid_v4() for _ in range(600))) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    seen += out
    assert all(pat.fullmatch(u) for u in seen) and len(set(seen)) == len(seen) == 3400
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:  # child: the next UUIDs of the inherited pool must not be the parent's
        os.close(r)
        os.write(w, "".join(nat.uuid_v4() for _ in range(4)).encode())
        os._exit(0)
    os.close(w)
    child = os.read(r, 4096).decode()
    os.close(r)
    os.waitpid(pid, 0)
    parent = "".join(nat.uuid_v4() for _ in range(4))
    assert len(child) == len(parent) == 144 and child != parent


def test_certificates_verify_with_openssl(nat, tmp_path):
    b = nat.make_ca_and_leaf("bgc-admission", ["bgc-admission.bgc.svc", "127.0.0.1"], 90)
    (tmp_path / "ca.crt").write_text(b["ca_cert"])
    (tmp_path / "tls.crt").write_text(b["cert"])
    r = subprocess.run(["openssl", "verify", "-CAfile", str(tmp_path / "ca.crt"), str(tmp_path / "tls.crt")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    txt = subprocess.run(["openssl", "x509", "-in", str(tmp_path / "tls.crt"), "-noout", "-text"],
                         capture_output=True, text=True).stdout
    assert "DNS:bgc-admission.bgc.svc" in txt and "IP Address:127.0.0.1" in txt


def test_workqueue_many_workers_no_lost_wakeups(nat):
    """8 workers, 600 keys with mixed immediate/delayed due times, re-adds while in flight:
    every key is processed, never by two workers at once, and nothing waits past its due
    time by more than a scheduling slack (one timer waiter, no thundering herd)."""
    import random

    q = nat.WorkQueue()
    rnd = random.Random(7)
    due = {}
    t0 = time.time()
    for i in range(600):
        d = rnd.choice([0, 0, 5, 20, 60])
        due[f"k{i}"] = t0 + d / 1000.0
        q.add_after(f"k{i}", d)
    seen, late, active, lock = {}, [], set(), threading.Lock()
    readded = set()

    def worker():
        while True:
            k = q.get()
            if k is None:
                return
            now = time.time()
            with lock:
                assert k not in active
                active.add(k)
                seen[k] = seen.get(k, 0) + 1
                late.append(now - due[k])
                again = k not in readded and int(k[1:]) % 10 == 0
                if again:
                    readded.add(k)
                    due[k] = now  # deferred re-add while in flight runs right after done()
            if again:
                q.add(k)
            time.sleep(0.0005)
            with lock:
                active.discard(k)
            q.done(k)

    threads = [threading.Thread(target=worker) for _ in range(8)]
    for th in threads:
        th.start()
    deadline = time.time() + 10
    while time.time() < deadline and (len(seen) < 600 or sum(seen.values()) < 660 or q.pending()):
        time.sleep(0.01)
    q.shutdown()
    for th in threads:
        th.join(5)
    assert len(seen) == 600 and sum(seen.values()) == 660
    late.sort()
    assert late[len(late) // 2] < 0.05 and late[-1] < 1.0


def test_workqueue_forget_drops_pending_requeue(nat):
    import threading
    import time

    q = nat.WorkQueue()
    q.add_after("gone", 50)   # e.g. the 30 s requeue of an object deleted since
    q.add_after("kept", 80)
    assert q.pending() == 2
    q.forget("gone")
    q.forget("never-added")   # no-op
    assert q.pending() == 1
    t0 = time.time()
    assert q.get() == "kept"  # the forgotten key is never handed out
    assert time.time() - t0 >= 0.06
    q.done("kept")
    # an in-flight key is not affected: forget only drops pending entries
    q.add("busy")
    assert q.get() == "busy"
    q.forget("busy")
    q.add("busy")             # deferred re-add while processing
    q.done("busy")
    got = []
    th = threading.Thread(target=lambda: got.append(q.get()))
    th.start()
    th.join(2)
    assert got == ["busy"]
    q.shutdown()


def test_workqueue_forget_while_in_flight_drops_the_workers_requeue(nat):
    """The object is deleted while its reconcile runs: the reconcile's 30 s requeue is not kept
    (native/kube/runtime.cc WorkQueue::requeue), unless a new event re-adds the key."""
    q = nat.WorkQueue()
    q.add("gone")
    assert q.get() == "gone"
    q.forget("gone")          # DELETED event arrives mid-reconcile
    q.requeue("gone", 30000)  # the reconcile finishes and asks for its periodic requeue
    q.done("gone")
    assert q.pending() == 0
    # re-created while in flight: the ADDED event's add() wins over the forget
    q.add("back")
    assert q.get() == "back"
    q.forget("back")
    q.add_after("back", 30000)
    q.requeue("back", 30000)
    q.done("back")
    assert q.pending() == 1
    # the forgotten mark ends with the reconcile: a later requeue of the key is kept
    q.add("again")
    assert q.get() == "again"
    q.forget("again")
    q.done("again")
    q.requeue("again", 30000)
    assert q.pending() == 2
    q.shutdown()


def test_lsan_filter_keeps_only_native_leaks(tmp_path):
    """tools/lsan_filter.py (tools/sanitize.sh asan-py): CPython's end-of-life allocations
    are dropped, a leak with a frame in native/ or the _native module is reported."""
    import subprocess
    import sys

    from bacchus_gpu_controller_amd import REPO_ROOT

    log = tmp_path / "asan.1"
    log.write_text(
        "==1==ERROR: LeakSanitizer: detected memory leaks\n\n"
        "Direct leak of 64 byte(s) in 1 object(s) allocated from:\n"
        "    #0 0x7f in __interceptor_malloc asan_malloc_linux.cpp:145\n"
        "    #1 0x55 in _PyObject_Malloc (/usr/bin/python3.10+0x1)\n\n"
        "Direct leak of 32 byte(s) in 1 object(s) allocated from:\n"
        "    #0 0x7f in operator new(unsigned long) asan_new_delete.cpp:95\n"
        "    #1 0x7f in bgc::json::parse(std::string_view) /root/repo/native/core/json.cc:400\n"
        "    #2 0x7f in pybind11::cpp_function::dispatcher (_native.cpython-310-x86_64-linux-gnu.so+0x1)\n\n")
    tool = os.path.join(REPO_ROOT, "tools", "lsan_filter.py")
    r = subprocess.run([sys.executable, tool, str(log)], capture_output=True, text=True)
    assert r.returncode == 1 and "1 leak record(s)" in r.stderr and "json.cc:400" in r.stdout
    log.write_text(log.read_text().split("Direct leak of 32")[0])
    r = subprocess.run([sys.executable, tool, str(log)], capture_output=True, text=True)
    assert r.returncode == 0 and "0 leak record(s)" in r.stderr


def test_cert_bundle_key_types(nat, tmp_path):
    import subprocess

    for kt, want in (("ec", "id-ecPublicKey"), ("rsa", "rsaEncryption")):
        b = nat.make_ca_and_leaf("svc", ["svc.ns.svc", "127.0.0.1"], 30, kt)
        (tmp_path / "ca.crt").write_text(b["ca_cert"])
        (tmp_path / "leaf.crt").write_text(b["cert"])
        txt = subprocess.run(["openssl", "x509", "-in", str(tmp_path / "leaf.crt"), "-noout", "-text"],
                             capture_output=True, text=True, check=True).stdout
        assert want in txt and "DNS:svc.ns.svc" in txt and "IP Address:127.0.0.1" in txt
        assert ("Key Encipherment" in txt) == (kt == "rsa")
        v = subprocess.run(["openssl", "verify", "-CAfile", str(tmp_path / "ca.crt"), str(tmp_path / "leaf.crt")],
                           capture_output=True, text=True)
        assert v.returncode == 0, v.stdout + v.stderr


def test_retry_limiter_exponential_cap_and_bucket(nat):
    """client-go's controller rate limiter: base * 2^(n-1) per key, capped, max'd with an
    overall token bucket; forget() restarts a key's backoff."""
    r = nat.RetryLimiter(5, 60000, 1e6, 1000)
    assert [r.when("a") for _ in range(6)] == [5, 10, 20, 40, 80, 160]
    assert r.failures("a") == 6 and r.when("b") == 5  # keys are independent
    for _ in range(20):
        r.when("a")
    assert r.when("a") == 60000  # capped
    r.forget("a")
    assert r.failures("a") == 0 and r.when("a") == 5
    # the bucket: 10 qps with burst 2 -> the third immediate retry waits ~100 ms
    b = nat.RetryLimiter(1, 1, 10.0, 2)
    d = [b.when(f"k{i}") for i in range(4)]
    assert d[:2] == [1, 1] and 90 <= d[2] <= 101 and 190 <= d[3] <= 201


def test_event_rate_limiter_keeps_a_flooding_objects_bucket(nat):
    """The recorder's per-object bucket (client-go EventSourceObjectSpamFilter): `burst`
    events, then refill_per_minute.  Past max_keys objects, buckets that refilled to the
    burst are dropped first (identical to a fresh one), else the longest-idle one, and never
    the object just charged, so an object flooding events stays limited however many other
    objects come and go (eviction used to drop the lexicographically first key)."""
    lim = nat.EventRateLimiter(burst=3, refill_per_minute=6, max_keys=4)
    t = 0.0
    # "a-flood" sorts first: the old eviction (buckets_.begin()) would have reset it
    assert [lim.allow("a-flood", t) for _ in range(5)] == [True, True, True, False, False]
    for i in range(50):  # many one-off objects over 5 s, each charged once
        t += 0.1
        assert lim.allow(f"obj-{i:03d}", t)
        assert lim.size() <= 5
        assert not lim.allow("a-flood", t)  # 5 s at 6/min refills half a token: still drained
    # 5.5 s more completes one token (denied events cost nothing) -> exactly one more event
    t += 5.5
    assert lim.allow("a-flood", t)
    assert not lim.allow("a-flood", t)
    # a bucket that refilled to the burst is evicted before a draining one
    lim2 = nat.EventRateLimiter(burst=2, refill_per_minute=60, max_keys=2)
    assert lim2.allow("idle", 0.0)
    assert lim2.allow("busy", 10.0) and lim2.allow("busy", 10.0)  # drained at t=10
    assert lim2.allow("new", 10.5)  # 3 keys > 2: "idle" refilled (60/min) -> evicted
    assert lim2.size() == 2
    assert not lim2.allow("busy", 10.5)  # "busy" kept its drained bucket
