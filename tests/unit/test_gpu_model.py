"""GPU-side logic that runs without a GPU: mock discovery, telemetry poller, health
state machine (hysteresis), node label/status rendering (N1-N3)."""
import json
import time


def test_mock_discovery_fixture(nat):
    b = nat.gpu_backend("mock", nat.default_mi355x_fixture(8))
    gpus = json.loads(b.discover())
    assert len(gpus) == 8
    assert {g["gfx_target"] for g in gpus} == {"gfx950"}
    assert all(g["vram_total_mb"] == 294912 for g in gpus)
    assert len({g["xgmi_hive_id"] for g in gpus}) == 1


def test_poller_side_thread(nat):
    b = nat.gpu_backend("mock", nat.default_mi355x_fixture(4))
    p = nat.TelemetryPoller(b, [0, 1, 2, 3], 10)
    p.start()
    time.sleep(0.25)
    p.stop()
    assert p.polls() >= 5
    snap = json.loads(p.snapshot())
    assert len(snap["devices"]) == 4 and all(d["ok"] for d in snap["devices"])
    assert all(h["healthy"] for h in snap["health"])


def test_poller_stall_watchdog(nat):
    """A poll stuck in the backend past stall_ms publishes every device unhealthy; the poll
    that finally completes publishes the real readings again (native/gpu/telemetry.cc)."""
    fx = json.loads(nat.default_mi355x_fixture(2))
    fx["sample_hang_ms"] = 600  # the first poll's two readings block this long, later ones return
    fx["sample_hang_samples"] = 2
    b = nat.gpu_backend("mock", json.dumps(fx))
    p = nat.TelemetryPoller(b, [0, 1], 100, stall_ms=150)
    p.start()  # the first poll hangs for 600 ms
    time.sleep(0.4)
    snap = json.loads(p.snapshot())
    assert p.stalled() and snap["stalled"]
    assert [h["healthy"] for h in snap["health"]] == [False, False]
    assert all("telemetry stalled" in h["reason"] for h in snap["health"])
    # the hung poll completes after 600 ms, longer than the stall timeout: still stalled
    deadline = time.time() + 3
    while p.polls() < 1 and time.time() < deadline:
        time.sleep(0.005)
    assert p.stalled()
    # the next poll is fast: the real readings are back
    while p.polls() < 2 and time.time() < deadline:
        time.sleep(0.005)
    time.sleep(0.02)
    snap = json.loads(p.snapshot())
    p.stop()
    assert not snap["stalled"] and all(h["healthy"] for h in snap["health"])
    assert all(d["ok"] for d in snap["devices"])


def test_a_slow_backend_stays_withdrawn(nat):
    """Every poll answering only after the stall timeout keeps the devices unhealthy
    instead of flapping them back after each completed poll."""
    fx = json.loads(nat.default_mi355x_fixture(1))
    fx["sample_hang_ms"] = 250
    p = nat.TelemetryPoller(nat.gpu_backend("mock", json.dumps(fx)), [0], 20, stall_ms=100)
    p.start()
    deadline = time.time() + 5
    while p.polls() < 3 and time.time() < deadline:
        assert time.time() < deadline
        time.sleep(0.01)
        if p.polls() >= 1:
            assert p.stalled() and json.loads(p.snapshot())["stalled"]
    p.stop()
    assert p.polls() >= 3


def test_poller_without_stall_timeout_never_stalls(nat):
    fx = json.loads(nat.default_mi355x_fixture(1))
    fx["sample_hang_ms"] = 300
    p = nat.TelemetryPoller(nat.gpu_backend("mock", json.dumps(fx)), [0], 5000)
    p.start()
    time.sleep(0.2)
    assert not p.stalled() and not json.loads(p.snapshot())["stalled"]
    p.stop()


def test_health_hysteresis(nat):
    hot = {"temp_hotspot_c": 120}
    ok = {"temp_hotspot_c": 50}
    seq = [hot, hot, ok, hot, hot, hot, ok, ok, ok]
    out = nat.health_step(json.dumps(seq), 3, 3)
    healthy = [h for h, _ in out]
    # needs 3 consecutive bad samples to flip, 3 consecutive good ones to recover
    assert healthy == [True, True, True, True, True, False, False, False, True]
    assert "hotspot" in out[5][1]


def test_health_ecc_and_xgmi(nat):
    seq = [{"ecc_uncorrectable": 5}, {"ecc_uncorrectable": 6}]  # baseline 5, then +1
    out = nat.health_step(json.dumps(seq), 1, 1, json.dumps({"max_uncorrectable_at_start": 10}))
    assert out[0][0] is True and out[1][0] is False and "ECC" in out[1][1]
    out = nat.health_step(json.dumps([{"xgmi_links_up": 6, "xgmi_links_total": 7}]), 1, 1)
    assert out[0][0] is False and "xGMI" in out[0][1]
    out = nat.health_step(json.dumps([{"ok": False, "error": "gone"}]), 1, 1)
    assert out[0][0] is False


def test_node_patches(nat):
    gpus = json.loads(nat.gpu_backend("mock", nat.default_mi355x_fixture(8)).discover())
    labels, status = nat.node_patches(json.dumps(gpus), 7, "mi355x-0", True, True, "gpu3: hot")
    labels, status = json.loads(labels), json.loads(status)
    l = labels["metadata"]["labels"]
    assert l["amd.com/gpu.family"] == "gfx950"
    assert l["amd.com/gpu.product"] == "MI355X"
    assert l["amd.com/gpu.count"] == "8" and l["amd.com/gpu.healthy-count"] == "7"
    assert l["amd.com/gpu.vram-gb"] == "288"
    assert l["amd.com/gpu.xgmi-hive-id"] == "1a2b3c4d5e6f7788" and l["amd.com/gpu.xgmi-hives"] == "1"
    assert l["amd.com/gpu.diag"] == "passed"
    assert l["amd.com/gpu.driver-version"] == "6.16.6"
    assert l["amd.com/gpu.vbios-version"] == "022.040.003.043.000001"
    topo = json.loads(labels["metadata"]["annotations"]["amd.com/gpu.topology"])
    assert len(topo) == 8 and topo[3]["node"] == 3
    st = status["status"]
    assert st["capacity"] == {"amd.com/gpu": "8"} and st["allocatable"] == {"amd.com/gpu": "7"}
    assert st["conditions"][0]["type"] == "AMDGPUHealthy" and st["conditions"][0]["status"] == "False"


def test_mixed_hives_label(nat):
    f = json.loads(nat.default_mi355x_fixture(4))
    f["gpus"][2]["xgmi_hive_id"] = "00000000000000ff"
    gpus = json.loads(nat.gpu_backend("mock", json.dumps(f)).discover())
    labels = json.loads(nat.node_patches(json.dumps(gpus), 4)[0])["metadata"]["labels"]
    assert labels["amd.com/gpu.xgmi-hive-id"] == "mixed" and labels["amd.com/gpu.xgmi-hives"] == "2"


def test_driver_and_vbios_labels(nat):
    f = json.loads(nat.default_mi355x_fixture(4))
    f["gpus"][1]["vbios_version"] = "022.040.003.044.000001"  # one board mid-rollout
    for g in f["gpus"]:
        g["driver_version"] = ""
    gpus = json.loads(nat.gpu_backend("mock", json.dumps(f)).discover())
    assert gpus[0]["vbios_part_number"] == "113-M3550101-100" and gpus[0]["driver_name"] == "amdgpu"
    labels = json.loads(nat.node_patches(json.dumps(gpus), 4)[0])["metadata"]["labels"]
    assert labels["amd.com/gpu.vbios-version"] == "mixed"
    assert labels["amd.com/gpu.driver-version"] == "unknown"


def test_sanitize_label_value(nat):
    assert nat.sanitize_label_value("AMD Instinct MI355 OAM") == "AMD_Instinct_MI355_OAM"
    assert nat.sanitize_label_value("-x-") == "x"
    assert len(nat.sanitize_label_value("a" * 100)) == 63
