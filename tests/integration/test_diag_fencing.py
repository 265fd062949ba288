"""Node-agent diagnostics on a whole node (native/gpu/diag_runner.cc, node_agent.cc):

* a periodic pass fences its GPUs in the device plugin — the kubelet sees them Unhealthy,
  Allocate refuses them, GetPreferredAllocation leaves them out — and releases them once
  the verdicts are in;
* a GPU that a pod takes while the fence settles is released untouched, not burned;
* every GPU is diagnosed on its own thread: 8 GPUs take about one GPU's wall time;
* the burn-in is one node-level phase, judged on the summed power and on the slowest GPU
  against the fastest under the shared load.

The mock backend's fixture scripts the diagnostics engine ("diag_script": per-GPU durations
and outcomes), so this runs on CPU; tests/gpu/test_gpu_health_r3.py runs the HIP engine.
The fake kubelet is python grpcio (an independent gRPC stack, as grpc-go in a real kubelet).
"""
import json
import os
import subprocess
import time

import grpc
import pytest
import requests

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for
from bacchus_gpu_controller_amd.testing.kubelet import FakeKubelet, FakePodResources, PluginClient, pb

pytestmark = pytest.mark.slow


def _fixture(nat, n, script, power_w=None):
    fx = json.loads(nat.default_mi355x_fixture(n))
    fx["diag_script"] = script
    if power_w is not None:
        for g in fx["gpus"]:
            g["telemetry"]["power_w"] = power_w
    return fx


def _describe(c, node):
    return requests.get(f"http://127.0.0.1:{c.node_agent_ports[node]}/gpus", timeout=5).json()


def test_periodic_pass_fences_gpus_from_the_kubelet(nat, tmp_path):
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    pr = FakePodResources(str(tmp_path / "pod-resources" / "kubelet.sock")).start()
    script = {"checks_ms": 2500, "burn_tflops": 2400}
    try:
        with Cluster(admission=False, controller=False) as c:
            c.start_node_agent(node_name="mi355x-fence", backend="mock", poll_interval_ms=100,
                               fixture_obj=_fixture(nat, 4, {"checks_ms": 50}),
                               extra_env={"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d,
                                          "CONF_RUN_DIAG": "true", "CONF_DIAG_INTERVAL_SECS": "1",
                                          "CONF_DIAG_FENCE_SETTLE_MS": "300", "CONF_DIAG_BURN_MS": "200",
                                          "CONF_POD_RESOURCES_SOCKET": pr.path, "CONF_HEARTBEAT_SECS": "1"})
            assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists, timeout=15)
            ids = [x[0] for x in kubelet.device_lists[-1][1]]
            assert all(x[1] == "Healthy" for x in kubelet.device_lists[-1][1])  # start-up pass passed
            c.set_gpu_fixture("mi355x-fence", _fixture(nat, 4, script))  # periodic passes now take 2.5 s
            pr.assign("train-0", "amd.com/gpu", [ids[0]])  # GPU 0 busy: never fenced
            fenced = lambda: [x[1] for x in kubelet.device_lists[-1][1]] == ["Healthy"] + ["Unhealthy"] * 3
            assert kubelet.wait(fenced, timeout=15), kubelet.device_lists[-3:]
            client = PluginClient(os.path.join(d, "bgc-amd-gpu.sock"))
            try:
                # Allocate of a fenced GPU is refused with a gRPC error, a free one is served
                req = pb["AllocateRequest"]()
                req.container_requests.add().devices_ids.extend([ids[2]])
                with pytest.raises(grpc.RpcError) as ei:
                    client.allocate(req, timeout=5)
                assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
                assert "under node diagnostics" in ei.value.details()
                ok = pb["AllocateRequest"]()
                ok.container_requests.add().devices_ids.extend([ids[0]])
                assert client.allocate(ok, timeout=5).container_responses[0].envs["BGC_AMD_GPU_IDS"] == ids[0]
                # preferred allocation leaves fenced GPUs out when it can
                pref = pb["PreferredAllocationRequest"]()
                cr = pref.container_requests.add()
                cr.available_deviceIDs.extend(ids)
                cr.allocation_size = 1
                assert list(client.preferred(pref, timeout=5).container_responses[0].deviceIDs) == [ids[0]]
            finally:
                client.close()
            desc = _describe(c, "mi355x-fence")
            assert sorted(desc["device_plugin"]["fenced"]) == sorted(ids[1:])
            assert desc["device_plugin"]["refused_fenced"] >= 1
            # the pass ends: every GPU back to Healthy, the fence lifted, busy GPU 0 skipped
            assert kubelet.wait(lambda: all(x[1] == "Healthy" for x in kubelet.device_lists[-1][1]), timeout=15)
            desc = wait_for(lambda: (lambda g: g if g["diag_runs"] >= 2 and not g["device_plugin"]["fenced"] else None)(
                _describe(c, "mi355x-fence")), timeout=15, desc="pass finished")
            assert desc["diag_last_diagnosed"] == 3 and desc["diag_skipped_in_use"] >= 1
            assert all(r["passed"] for r in desc["diag"][1:])
            assert desc["diag_node_burn"]["gpus"] == 3
    finally:
        pr.stop()
        kubelet.stop()


def test_gpu_allocated_while_fence_settles_is_released_untouched(nat, tmp_path):
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    pr = FakePodResources(str(tmp_path / "pod-resources" / "kubelet.sock")).start()
    try:
        with Cluster(admission=False, controller=False) as c:
            c.start_node_agent(node_name="mi355x-race", backend="mock", poll_interval_ms=100,
                               fixture_obj=_fixture(nat, 2, {"checks_ms": 50}),
                               extra_env={"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d,
                                          "CONF_RUN_DIAG": "true", "CONF_DIAG_INTERVAL_SECS": "1",
                                          "CONF_DIAG_FENCE_SETTLE_MS": "3000",
                                          "CONF_POD_RESOURCES_SOCKET": pr.path, "CONF_HEARTBEAT_SECS": "1"})
            assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists, timeout=15)
            ids = [x[0] for x in kubelet.device_lists[-1][1]]
            assert kubelet.wait(lambda: all(x[1] == "Unhealthy" for x in kubelet.device_lists[-1][1]), timeout=15)
            # the kubelet admitted a pod onto GPU 1 just before the fence reached it
            pr.assign("late-pod", "amd.com/gpu", [ids[1]])
            desc = wait_for(lambda: (lambda g: g if g["diag_fence_races"] >= 1 and g["diag_runs"] >= 2 else None)(
                _describe(c, "mi355x-race")), timeout=20, desc="raced GPU released")
            assert desc["diag_last_diagnosed"] == 1  # only GPU 0 ran
            # GPU 1 is released at once (not held for the pass) and never fenced again while held
            assert kubelet.wait(lambda: [x[1] for x in kubelet.device_lists[-1][1]][1] == "Healthy", timeout=10)
    finally:
        pr.stop()
        kubelet.stop()


def test_eight_gpus_diagnosed_in_one_gpus_wall_time(nat):
    """Start-up pass on 8 GPUs: checks 800 ms + node burn 400 ms each.  Serial would be
    8 x 1.2 s = 9.6 s; concurrent is ~1.2 s."""
    with Cluster(admission=False, controller=False) as c:
        c.start_node_agent(node_name="mi355x-8", backend="mock", poll_interval_ms=200,
                           fixture_obj=_fixture(nat, 8, {"checks_ms": 800}, power_w=1100),
                           extra_env={"CONF_RUN_DIAG": "true", "CONF_DIAG_BURN_MS": "400"})
        desc = _describe(c, "mi355x-8")
        assert desc["diag_engine"] == "scripted" and desc["diag_last_diagnosed"] == 8
        assert all(r["passed"] for r in desc["diag"]), [r["failures"] for r in desc["diag"]]
        assert 1200 <= desc["diag_last_pass_ms"] < 2400, desc["diag_last_pass_ms"]
        assert max(r["checks_started_ms"] for r in desc["diag"]) < 300
        nb = desc["diag_node_burn"]
        assert nb["gpus"] == 8 and nb["passed"] and nb["balance"] == 1.0
        assert nb["power_sum_max_w"] == pytest.approx(8 * 1100)
        st = desc["startup_ms"]
        assert st["diagnostics"] < 2400 and st["first_advertise"] >= st["diagnostics"]


def test_node_burn_gates_on_summed_power_and_balance(nat):
    script = {"checks_ms": 50, "gpus": {"3": {"burn_tflops": 1900}}}
    with Cluster(admission=False, controller=False) as c:
        c.start_node_agent(node_name="mi355x-pw", backend="mock", poll_interval_ms=200,
                           fixture_obj=_fixture(nat, 8, script, power_w=1200),
                           extra_env={"CONF_RUN_DIAG": "true", "CONF_DIAG_BURN_MS": "400",
                                      "CONF_DIAG_MAX_NODE_POWER_W": "8000"})
        desc = _describe(c, "mi355x-pw")
        nb = desc["diag_node_burn"]
        assert not nb["passed"] and "node drew 9600 W" in nb["failures"][0]
        assert nb["balance"] == pytest.approx(1900 / 2400)
        for i, r in enumerate(desc["diag"]):
            assert not r["passed"]
            assert any("node drew" in f for f in r["failures"])
            assert any("of the node's fastest GPU" in f for f in r["failures"]) == (i == 3)
        node = wait_for(lambda: (lambda n: n if n and n["metadata"]["labels"].get("amd.com/gpu.diag") == "failed" else None)(
            c.admin.get_or_none("nodes", "mi355x-pw")), timeout=15, desc="diag label")
        assert node["metadata"]["labels"]["amd.com/gpu.healthy-count"] == "0"


def test_mx_burn_dtype_scales_the_burn_floor(nat):
    """DIAG_BURN_DTYPE=fp4 runs the node burn on the MX fp4 path: its rate is held to the
    bf16 floor scaled 3.5x, so a GPU at fp4 speed passes and one at only twice the bf16
    rate fails with a message naming the dtype."""
    script = {"checks_ms": 50, "gpus": {"1": {"burn_tflops": 1000}}}  # scripted rates are bf16 rates
    with Cluster(admission=False, controller=False) as c:
        c.start_node_agent(node_name="mi355x-mx", backend="mock", poll_interval_ms=200,
                           fixture_obj=_fixture(nat, 2, script),
                           extra_env={"CONF_RUN_DIAG": "true", "CONF_DIAG_BURN_MS": "300",
                                      "CONF_DIAG_BURN_DTYPE": "fp4", "CONF_DIAG_MIN_NODE_BURN_BALANCE": "0"})
        desc = _describe(c, "mi355x-mx")
        assert desc["diag_node_burn"]["dtype"] == "fp4"
        ok, slow = desc["diag"]
        assert ok["burn"]["dtype"] == "fp4" and ok["burn"]["tflops_mean"] == pytest.approx(2400 * 3.5)
        assert ok["passed"], ok["failures"]
        assert not slow["passed"] and slow["failures"] == ["burn-in MFMA MX fp4 TFLOP/s 3500 below floor 6300"]


def test_unknown_burn_dtype_stops_the_agent(tmp_path):
    from bacchus_gpu_controller_amd import REPO_ROOT

    env = dict(os.environ, CONF_GPU_BACKEND="mock", CONF_NODE_NAME="n", CONF_DIAG_BURN_DTYPE="int8",
               CONF_LISTEN_ADDR="127.0.0.1", CONF_LISTEN_PORT="0", KUBE_API_URL="http://127.0.0.1:9")
    p = subprocess.run([os.path.join(REPO_ROOT, "bin", "node-agent")], env=env, capture_output=True, text=True,
                       timeout=30)
    assert p.returncode != 0 and "burn dtype must be bf16, fp8 or fp4, not 'int8'" in p.stderr


def test_restart_leaves_busy_gpus_alone(nat, tmp_path):
    """An agent (re)started on a node whose GPUs already run jobs must not burn or walk
    them: the start-up pass diagnoses only free GPUs, a busy one stays advertised without
    a verdict, and a later periodic pass diagnoses it once its job is gone."""
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    fx = _fixture(nat, 4, {"checks_ms": 50})
    fx["gpus"][2]["telemetry"]["busy_processes"] = 1  # a tenant process holds GPU 2 (amdsmi)
    try:
        with Cluster(admission=False, controller=False) as c:
            c.start_node_agent(node_name="mi355x-restart", backend="mock", poll_interval_ms=100, fixture_obj=fx,
                               extra_env={"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d,
                                          "CONF_RUN_DIAG": "true", "CONF_DIAG_INTERVAL_SECS": "1",
                                          "CONF_DIAG_FENCE_SETTLE_MS": "100", "CONF_DIAG_BURN_MS": "100",
                                          "CONF_HEARTBEAT_SECS": "1"})
            assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists, timeout=15)
            assert all(x[1] == "Healthy" for x in kubelet.device_lists[-1][1])  # the busy GPU is still offered
            desc = _describe(c, "mi355x-restart")
            assert desc["diag"][2] is None and desc["diag_skipped_in_use"] >= 1
            assert all(desc["diag"][i]["passed"] for i in (0, 1, 3))
            fx["gpus"][2]["telemetry"]["busy_processes"] = 0  # the job ends
            c.set_gpu_fixture("mi355x-restart", fx)
            wait_for(lambda: (_describe(c, "mi355x-restart")["diag"][2] or {}).get("passed"), timeout=20,
                     desc="GPU 2 diagnosed once free")
    finally:
        kubelet.stop()


def _children(pid):
    """Child processes of any thread of `pid` (workers are spawned from the diag threads)."""
    out = []
    try:
        tasks = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for t in tasks:
        try:
            with open(f"/proc/{pid}/task/{t}/children") as f:
                out += [int(x) for x in f.read().split()]
        except OSError:
            pass
    return out


def test_worker_processes_run_the_pass_and_stop_with_the_agent(nat, tmp_path):
    """The production engine runs every check and burn in `node-agent --diag-worker`
    processes (BGC_DIAG_WORKERS=1 puts the mock's diagnostics script inside them on a CPU
    host).  A pass's results come back through the workers, the burn starts after the
    common lead, and an agent stopped mid-pass kills its worker instead of waiting for it."""
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    try:
        with Cluster(admission=False, controller=False) as c:
            os.environ["BGC_DIAG_WORKERS"] = "1"
            try:
                c.start_node_agent(node_name="mi355x-workers", backend="mock", n_mock_gpus=2, poll_interval_ms=100,
                                   fixture_obj=_fixture(nat, 2, {"checks_ms": 100, "burn_tflops": 2400}),
                                   extra_env={"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d,
                                              "CONF_RUN_DIAG": "true", "CONF_DIAG_BURN_MS": "300",
                                              "CONF_DIAG_INTERVAL_SECS": "1", "CONF_DIAG_FENCE_SETTLE_MS": "100"})
            finally:
                del os.environ["BGC_DIAG_WORKERS"]
            assert kubelet.wait(lambda: kubelet.device_lists, timeout=30)
            desc = _describe(c, "mi355x-workers")
            assert desc["diag_isolation"] == "worker-process"
            assert all(r["passed"] and r["worker_ms"] > 100 for r in desc["diag"]), desc["diag"]
            assert desc["diag_node_burn"]["start_lead_ms"] >= 1900 and desc["diag_node_burn"]["gpus"] == 2
            agent = c.procs["node-agent"]
            # periodic passes now take 30 s each: stop the agent while a worker runs
            c.set_gpu_fixture("mi355x-workers", _fixture(nat, 2, {"checks_ms": 30000}))
            wait_for(lambda: _children(agent.p.pid), timeout=20, interval=0.05, desc="a worker running")
            workers = _children(agent.p.pid)
            t0 = time.time()
            agent.p.terminate()
            agent.p.wait(15)
            assert time.time() - t0 < 5, "the agent waited for its worker"
            time.sleep(0.3)
            assert not [w for w in workers if os.path.exists(f"/proc/{w}") and
                        open(f"/proc/{w}/stat").read().split()[2] != "Z"], "a worker outlived the agent"
            # a routine shutdown is not a GPU failure: the killed pass is dropped, with no
            # verdict, Event or health change published on the way out
            assert "diagnostics pass abandoned" in agent.output()
            evs = [e for e in c.admin.list("events", namespace="default")["items"]
                   if e["involvedObject"]["name"] == "mi355x-workers"]
            assert not [e for e in evs if e["reason"] in ("GPUDiagnosticsFailed", "GPUUnhealthy")], evs
            labels = c.admin.get("nodes", "mi355x-workers")["metadata"]["labels"]
            assert labels["amd.com/gpu.diag"] == "passed" and labels["amd.com/gpu.healthy-count"] == "2"
    finally:
        kubelet.stop()
