"""Round-2 N1/N2 depth without a GPU: RAS / violation health rules (each one flips the
state machine, and — through the node agent — ListAndWatch), violation percentages from
gpu_metrics accumulators, the throttle sentinel, the 8x8 xGMI link map in the mock
fixture and the topology annotation, link-aware preferred allocation, compute-partition
render nodes, the diagnostics floors (judge_diag) and the kubelet pod-resources codec
checked against an independent protobuf implementation."""
import json

import pytest


def _steps(nat, seq, policy=None, page_limit=0, fail=1, recover=1):
    return nat.health_step(json.dumps(seq), fail, recover, json.dumps(policy or {}), page_limit)


def test_preexisting_uncorrectable_at_start_is_unhealthy(nat):
    out = _steps(nat, [{"ecc_uncorrectable": 3}, {"ecc_uncorrectable": 3}])
    assert out[0][0] is False and "already present at agent start" in out[0][1]
    # tolerated when the operator allows a few (then only *new* errors count)
    out = _steps(nat, [{"ecc_uncorrectable": 3}, {"ecc_uncorrectable": 3}], {"max_uncorrectable_at_start": 3})
    assert [h for h, _ in out] == [True, True]
    out = _steps(nat, [{"ecc_uncorrectable": 0}, {"ecc_uncorrectable": 0}])
    assert [h for h, _ in out] == [True, True]


def test_retired_pages_over_threshold(nat):
    seq = [{"retired_pages": 10}, {"retired_pages": 64}, {"retired_pages": 65}]
    out = _steps(nat, seq)
    assert [h for h, _ in out] == [True, True, False]
    assert "retired HBM pages 65 > 64" in out[2][1]
    # the driver's own (lower) bad-page threshold caps the policy
    out = _steps(nat, [{"retired_pages": 11}], page_limit=10)
    assert out[0][0] is False and "> 10" in out[0][1]
    out = _steps(nat, [{"retired_pages": 0, "unreservable_pages": 1}])
    assert out[0][0] is False and "could not be retired" in out[0][1]


def test_sustained_thermal_violation(nat):
    # accumulators advance 1000 per sample; thermal residency 50 % of each interval
    seq = [{"acc_counter": 1000 * i, "acc_ppt": 0, "acc_thermal": 500 * i} for i in range(1, 8)]
    out = _steps(nat, seq, {"violation_sustain_polls": 4})
    healthy = [h for h, _ in out]
    # sample 1 has no previous sample (unknown %); samples 2..5 are 4 violating polls
    assert healthy == [True, True, True, True, False, False, False]
    assert "sustained thermal throttling: 50%" in out[4][1]
    # a short burst does not trip it
    burst = [{"acc_counter": 1000 * i, "acc_thermal": (500 * i if i < 4 else 1500)} for i in range(1, 9)]
    assert all(h for h, _ in _steps(nat, burst, {"violation_sustain_polls": 4}))


def test_power_cap_violation_off_by_default(nat):
    seq = [{"acc_counter": 1000 * i, "acc_ppt": 900 * i, "acc_thermal": 0} for i in range(1, 40)]
    assert all(h for h, _ in _steps(nat, seq))  # PPT capping is normal at full load
    out = _steps(nat, seq, {"max_ppt_violation_pct": 50, "violation_sustain_polls": 3})
    assert out[-1][0] is False and "power-cap" in out[-1][1]


def test_mock_violation_percent_and_throttle_sentinel(nat):
    f = json.loads(nat.default_mi355x_fixture(2))
    f["gpus"][1]["telemetry"]["violation_thermal_pct"] = 40
    f["gpus"][1]["telemetry"]["throttle_status"] = 4
    b = nat.gpu_backend("mock", json.dumps(f))
    p = nat.TelemetryPoller(b, [0, 1], 1000)
    p.poll_once()
    p.poll_once()
    devs = json.loads(p.snapshot())["devices"]
    assert devs[0]["violation_thermal_pct"] == 0 and devs[1]["violation_thermal_pct"] == pytest.approx(40, abs=0.2)
    # no throttle word in the fixture = not reported -> null, never a fake bit pattern
    assert devs[0]["throttle_status"] is None and devs[1]["throttle_status"] == 4


def test_sample_levels_and_ras_cache(nat):
    f = json.loads(nat.default_mi355x_fixture(1))
    t = f["gpus"][0]["telemetry"]
    t.update({"retired_pages": 7, "ecc_uncorrectable": 0, "ecc_correctable": 12,
              "ecc_blocks": [{"block": "umc", "ce": 12, "ue": 0, "de": 1}]})
    b = nat.gpu_backend("mock", json.dumps(f))
    fast = json.loads(b.sample(0, 0))
    assert "retired_pages" not in fast and fast["ecc_correctable"] == 0
    ras = json.loads(b.sample(0, 2))
    assert ras["retired_pages"] == 7 and ras["ecc_blocks"]["umc"] == {"ce": 12, "ue": 0, "de": 1}
    assert len(ras["links"]) == 0  # one GPU: no peers
    p = nat.TelemetryPoller(b, [0], 1000, "{}", 2, 4)
    for _ in range(3):
        p.poll_once()
    d = json.loads(p.snapshot())["devices"][0]  # poll 3 is Fast: RAS + slow fields cached
    assert d["retired_pages"] == 7 and d["ecc_correctable"] == 12


def test_fixture_has_full_xgmi_link_matrix(nat):
    gpus = json.loads(nat.gpu_backend("mock", nat.default_mi355x_fixture(8)).discover())
    for g in gpus:
        peers = sorted(l["peer"] for l in g["links"])
        assert peers == [j for j in range(8) if j != g["index"]]
        assert all(l["type"] == "xgmi" and l["hops"] == 1 and l["max_bw_mbps"] > 0 for l in g["links"])
        assert len(g["phys_links"]) == 7 and g["drm_render"] == 128 + g["index"]
    labels = json.loads(nat.node_patches(json.dumps(gpus), 8)[0])
    topo = json.loads(labels["metadata"]["annotations"]["amd.com/gpu.topology"])
    assert len(topo[0]["links"]) == 7 and topo[0]["xgmi_links_up"] == 7
    assert {l["peer"] for l in topo[5]["links"]} == {0, 1, 2, 3, 4, 6, 7}


def _two_quads(nat):
    """8 GPUs in one hive but wired as two 4-GPU xGMI quads joined only by PCIe (and the
    NUMA split deliberately *across* the quads, so NUMA alone would pick wrong)."""
    f = json.loads(nat.default_mi355x_fixture(8))
    quad = lambda i: i in (0, 2, 4, 6)  # noqa: E731
    for g in f["gpus"]:
        i = g["index"]
        for l in g["links"]:
            if quad(i) != quad(l["peer"]):
                l.update({"type": "pcie", "hops": 2, "weight": 40, "min_bw_mbps": 0, "max_bw_mbps": 0})
    return json.loads(nat.gpu_backend("mock", json.dumps(f)).discover())


def test_preferred_allocation_follows_link_map(nat):
    gpus = _two_quads(nat)
    ids = [g["bdf"] for g in gpus]
    pick = nat.preferred_allocation(json.dumps(gpus), ids, ids, [], 4)
    assert {ids.index(x) for x in pick} in ({0, 2, 4, 6}, {1, 3, 5, 7})
    pick = nat.preferred_allocation(json.dumps(gpus), ids, ids, [ids[3]], 3)
    assert pick[0] == ids[3] and {ids.index(x) for x in pick} <= {1, 3, 5, 7}
    # with a healthy full mesh the NUMA rules still decide (NUMA 1 quad for must=6)
    full = json.loads(nat.gpu_backend("mock", nat.default_mi355x_fixture(8)).discover())
    fids = [g["bdf"] for g in full]
    pick = nat.preferred_allocation(json.dumps(full), fids, fids, [fids[6]], 4)
    assert set(pick) == set(fids[4:8])


def test_partition_allocate_uses_own_render_node(nat, tmp_path):
    f = json.loads(nat.default_mi355x_fixture(4))
    for i, g in enumerate(f["gpus"]):
        g["compute_partition"] = "CPX"
        g["bdf"] = f["gpus"][0]["bdf"]
        g["drm_render"] = 200 + i
    gpus = json.loads(nat.gpu_backend("mock", json.dumps(f)).discover())
    # sysfs for the shared BDF names partition 0's node; partitions must not get it
    drm = tmp_path / "sys" / "bus" / "pci" / "devices" / gpus[0]["bdf"] / "drm"
    (drm / "renderD128").mkdir(parents=True)
    plugin = nat.DevicePlugin(json.dumps(gpus), {"plugin_dir": str(tmp_path / "dp"), "sysfs_root": str(tmp_path / "sys"),
                                                 "register": "false"})
    resp = json.loads(plugin.allocate_json([plugin.ids[2]]))
    hosts = {d["host_path"] for d in resp["devices"]}
    assert "/dev/dri/renderD202" in hosts and "/dev/dri/renderD128" not in hosts
    gpus[3]["drm_render"] = -1
    plugin2 = nat.DevicePlugin(json.dumps(gpus), {"plugin_dir": str(tmp_path / "dp2"), "register": "false"})
    with pytest.raises(ValueError, match="render node is unknown"):
        plugin2.allocate_json([plugin2.ids[3]])


MI355X_MEASURED = {
    "hbm": {"read_gbps": 5600.0, "copy_gbps": 5200.0, "write_gbps": 4800.0, "mismatches": 0},
    "mfma": {"tflops": 1900.0, "xcc_balance": 0.97, "xccs_seen": 8, "mismatches": 0, "bad_cus": 0,
             "throughput_ok": True},
    "gemm": {"passed": True},
}


def test_judge_diag_floors(nat):
    ok = json.loads(nat.judge_diag(json.dumps(MI355X_MEASURED)))
    assert ok["passed"] and ok["failures"] == []
    slow = json.loads(json.dumps(MI355X_MEASURED))
    slow["hbm"]["read_gbps"] = 2500.0
    slow["mfma"]["xcc_balance"] = 0.5
    r = json.loads(nat.judge_diag(json.dumps(slow)))
    assert not r["passed"] and len(r["failures"]) == 2
    assert any("HBM read" in x for x in r["failures"]) and any("XCC balance" in x for x in r["failures"])
    r = json.loads(nat.judge_diag(json.dumps(MI355X_MEASURED), json.dumps({"min_mfma_tflops": 1e9})))
    assert not r["passed"] and "MFMA bf16 TFLOP/s" in r["failures"][0]
    bad = json.loads(json.dumps(MI355X_MEASURED))
    bad["gemm"]["passed"] = False
    bad["hbm"]["mismatches"] = 3
    r = json.loads(nat.judge_diag(json.dumps(bad), json.dumps({"min_read_gbps": 0})))
    assert not r["passed"] and len(r["failures"]) == 2


def test_judge_diag_section_errors_are_failures(nat):
    """A section that could not run (a HIP fault, a worker timeout) reports {"error": ...};
    the cause must reach the failures list even when every floor is off."""
    floors_off = json.dumps({k: 0 for k in ("min_burn_tflops", "min_burn_sustain", "max_burn_hotspot_c",
                                            "max_burn_thermal_violation_pct")})
    crashed = dict(MI355X_MEASURED, burn={"error": "diagnostics worker timed out"})
    r = json.loads(nat.judge_diag(json.dumps(crashed), floors_off))
    assert not r["passed"] and r["failures"] == ["burn: diagnostics worker timed out"]
    r = json.loads(nat.judge_diag(json.dumps(dict(MI355X_MEASURED, pcie={"error": "hipMemcpy: fault"}))))
    assert "pcie: hipMemcpy: fault" in r["failures"]


def test_judge_diag_mx_lowp_section(nat):
    """The MX fp8/fp4 matrix-core check: any wrong tile, wrong accumulators or a rate under
    its floor fails the GPU, and the failure names the variant."""
    lowp = {"fp8_tflops": 4000.0, "fp4_tflops": 7000.0, "fp8_mismatches": 0, "fp8_scaled_mismatches": 0,
            "fp4_mismatches": 0, "fp4_scaled_mismatches": 0, "mismatches": 0, "bad_cus": 0, "throughput_ok": True}
    ok = json.loads(nat.judge_diag(json.dumps(dict(MI355X_MEASURED, lowp=lowp))))
    assert ok["passed"], ok["failures"]
    bad = dict(lowp, fp4_scaled_mismatches=12, mismatches=12, bad_cus=1)
    r = json.loads(nat.judge_diag(json.dumps(dict(MI355X_MEASURED, lowp=bad))))
    assert not r["passed"] and "fp4 scaled 12" in r["failures"][0] and "1 CU(s)" in r["failures"][0]
    r = json.loads(nat.judge_diag(json.dumps(dict(MI355X_MEASURED, lowp=dict(lowp, throughput_ok=False)))))
    assert r["failures"] == ["MX fp8/fp4 MFMA throughput accumulators wrong"]
    r = json.loads(nat.judge_diag(json.dumps(dict(MI355X_MEASURED, lowp=lowp)),
                                  json.dumps({"min_fp8_tflops": 5000, "min_fp4_tflops": 6000})))
    assert r["failures"] == ["MX fp8 MFMA TFLOP/s 4000 below floor 5000"]


def test_pod_resources_codec_matches_protobuf(nat):
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="podres_v1_test.proto", package="v1", syntax="proto3")

    def msg(name, *fields):
        m = fd.message_type.add(name=name)
        for num, fname, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname

    S, M, I64 = F.TYPE_STRING, F.TYPE_MESSAGE, F.TYPE_INT64
    opt, rep = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    msg("NUMANode", (1, "ID", I64, opt, None))
    msg("TopologyInfo", (1, "nodes", M, rep, ".v1.NUMANode"))
    msg("ContainerDevices", (1, "resource_name", S, opt, None), (2, "device_ids", S, rep, None),
        (3, "topology", M, opt, ".v1.TopologyInfo"))
    msg("ContainerResources", (1, "name", S, opt, None), (2, "devices", M, rep, ".v1.ContainerDevices"),
        (3, "cpu_ids", I64, rep, None))
    msg("PodResources", (1, "name", S, opt, None), (2, "namespace", S, opt, None),
        (3, "containers", M, rep, ".v1.ContainerResources"))
    msg("ListPodResourcesResponse", (1, "pod_resources", M, rep, ".v1.PodResources"))
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    Resp = message_factory.GetMessageClass(pool.FindMessageTypeByName("v1.ListPodResourcesResponse"))
    r = Resp()
    p = r.pod_resources.add(name="train-0", namespace="alice")
    c = p.containers.add(name="main")
    c.cpu_ids.extend([3, 4])
    d = c.devices.add(resource_name="amd.com/gpu")
    d.device_ids.extend(["0000:05:00.0", "0000:15:00.0"])
    d.topology.nodes.add(ID=0)
    c.devices.add(resource_name="example.com/nic", device_ids=["eth1"])
    decoded = json.loads(nat.pod_resources_decode(r.SerializeToString()))
    assert decoded == [
        {"pod": "train-0", "namespace": "alice", "container": "main", "resource": "amd.com/gpu",
         "ids": ["0000:05:00.0", "0000:15:00.0"]},
        {"pod": "train-0", "namespace": "alice", "container": "main", "resource": "example.com/nic", "ids": ["eth1"]},
    ]
    back = Resp.FromString(nat.pod_resources_encode(json.dumps(decoded[:1])))
    assert list(back.pod_resources[0].containers[0].devices[0].device_ids) == ["0000:05:00.0", "0000:15:00.0"]


def test_judge_diag_burn_in(nat):
    good = json.loads(json.dumps(MI355X_MEASURED))
    good["burn"] = {"tflops_mean": 1950.0, "sustain": 0.97, "max_hotspot_c": 78.0, "thermal_violation_pct": 0.0,
                    "mismatches": 0}
    assert json.loads(nat.judge_diag(json.dumps(good)))["passed"]
    bad = json.loads(json.dumps(good))
    bad["burn"].update({"sustain": 0.6, "max_hotspot_c": 104.0, "thermal_violation_pct": 35.0})
    r = json.loads(nat.judge_diag(json.dumps(bad)))
    assert not r["passed"] and len(r["failures"]) == 3
    assert any("sagged" in f for f in r["failures"]) and any("hotspot 104" in f for f in r["failures"])


MI355X_PCIE = {"device": 0, "bytes": 268435456, "iters": 5, "h2d_gbps": 57.14, "d2h_gbps": 56.69,
               "bidir_gbps": 97.02, "mismatches": 0, "passed": True, "link_width": 16, "link_speed_mts": 32000,
               "max_width": 16, "max_speed_mts": 32000, "max_gen": 5, "replays": 0, "recoveries": 0}


def test_judge_diag_pcie(nat):
    """Host<->device copy floors and the link state read while the copies ran
    (values measured on the MI355X box, profiles/archive/pcie_r2/probe.json)."""
    assert json.loads(nat.judge_diag(json.dumps({"pcie": MI355X_PCIE})))["passed"]
    x8 = dict(MI355X_PCIE, link_width=8, h2d_gbps=28.5, d2h_gbps=28.3)
    r = json.loads(nat.judge_diag(json.dumps({"pcie": x8})))
    assert not r["passed"] and "PCIe link x8 of x16" in r["failures"]
    assert any("host-to-device" in f for f in r["failures"]) and any("device-to-host" in f for f in r["failures"])
    gen3 = dict(MI355X_PCIE, link_speed_mts=8000)
    r = json.loads(nat.judge_diag(json.dumps({"pcie": gen3})))
    assert r["failures"] == ["PCIe link at 8000 of 32000 MT/s under load"]
    # a Gen4 link (half speed) passes the speed rule at the default fraction, and the
    # operator can relax the rates for Gen4 hosts
    gen4 = dict(MI355X_PCIE, link_speed_mts=16000, h2d_gbps=27.0, d2h_gbps=26.5)
    r = json.loads(nat.judge_diag(json.dumps({"pcie": gen4}), json.dumps({"min_pcie_h2d_gbps": 20,
                                                                          "min_pcie_d2h_gbps": 20})))
    assert r["passed"]
    bad = dict(MI355X_PCIE, mismatches=12)
    r = json.loads(nat.judge_diag(json.dumps({"pcie": bad})))
    assert r["failures"] == ["PCIe round-trip mismatches: 12"]


def test_pcie_width_and_replay_health_rules(nat):
    full = {"pcie_width": 16, "pcie_speed_mts": 32000, "pcie_replays": 0}
    out = _steps(nat, [full, dict(full, pcie_width=8), dict(full, pcie_width=8)], {"pcie_max_width": 16}, fail=2)
    assert [h for h, _ in out] == [True, True, False] and "PCIe link x8 of x16" in out[2][1]
    assert all(h for h, _ in _steps(nat, [dict(full, pcie_width=8)] * 3,
                                    {"pcie_max_width": 16, "require_full_pcie_width": False}))
    # width unknown at discovery: the rule is off
    assert all(h for h, _ in _steps(nat, [dict(full, pcie_width=8)] * 3))
    # replays: the delta between slow readings; fast polls (-1) keep the last verdict
    seq = [dict(full, pcie_replays=10), dict(full, pcie_replays=15), dict(full, pcie_replays=900),
           {"pcie_width": 16}, {"pcie_width": 16}, dict(full, pcie_replays=905)]
    out = _steps(nat, seq, {"max_pcie_replays_per_poll": 100})
    assert [h for h, _ in out] == [True, True, False, False, False, True]
    assert "PCIe link replays: 885" in out[2][1]


def test_mock_pcie_link_state(nat):
    f = json.loads(nat.default_mi355x_fixture(2))
    f["gpus"][1]["telemetry"]["pcie_width"] = 4
    b = nat.gpu_backend("mock", json.dumps(f))
    g = json.loads(b.discover())[0]
    assert (g["pcie_max_width"], g["pcie_max_speed_mts"], g["pcie_max_gen"]) == (16, 32000, 5)
    slow = json.loads(b.sample(0, 1))
    assert (slow["pcie_width"], slow["pcie_speed_mts"], slow["pcie_replays"]) == (16, 32000, 0)
    assert "pcie_width" not in json.loads(b.sample(0, 0))  # fast level: not read
    assert json.loads(b.sample(1, 1))["pcie_width"] == 4


def test_judge_diag_gemm_soak(nat):
    ok = {"m": 8192, "n": 8192, "k": 8192, "launches": 10, "tile": 256, "tflops_mean": 1253.0, "tflops_best": 1288.0,
          "row_mismatches": 0, "col_mismatches": 0, "passed": True}
    assert json.loads(nat.judge_diag(json.dumps({"soak": ok})))["passed"]
    r = json.loads(nat.judge_diag(json.dumps({"soak": dict(ok, row_mismatches=1, col_mismatches=1)})))
    assert r["failures"] == ["GEMM soak checksums wrong: 1 rows, 1 columns"]
    r = json.loads(nat.judge_diag(json.dumps({"soak": dict(ok, tflops_mean=600.0)})))
    assert r["failures"] == ["GEMM soak TFLOP/s 600 below floor 950"]


def test_mx_gemm_binding_checks_operand_sizes(nat):
    """diag_mx_gemm rejects mismatched code/scale buffers before it touches the library or
    a GPU (fp8: one byte per element, fp4: two per byte; scales one byte per 32 K)."""
    m, n, k = 16, 32, 128
    ok = dict(a=b"\0" * (m * k), a_scales=b"\x7f" * (m * k // 32), bt=b"\0" * (n * k), bt_scales=b"\x7f" * (n * k // 32))
    bad_cases = [
        dict(ok, a=b"\0" * (m * k - 1)),                      # fp8 A one byte short
        dict(ok, bt_scales=b"\x7f" * (n * k // 32 + 1)),      # scale rows too long
    ]
    for kw in bad_cases:
        with pytest.raises(ValueError):
            nat.diag_mx_gemm(0, 0, m, n, k, **kw)
    with pytest.raises(ValueError):  # fp4 wants packed nibbles: half the fp8 size
        nat.diag_mx_gemm(0, 4, m, n, k, **ok)
    with pytest.raises(ValueError):  # K must be a multiple of 128
        nat.diag_mx_gemm(0, 0, m, n, 96, a=b"\0" * (m * 96), a_scales=b"\x7f" * (m * 3), bt=b"\0" * (n * 96),
                         bt_scales=b"\x7f" * (n * 3))
    with pytest.raises(ValueError):  # only fp8 (0) and fp4 (4)
        nat.diag_mx_gemm(0, 2, m, n, k, **ok)
