"""Round-end smoke test on cuda:0 (driver contract `smoke()`).

One tiny end-to-end pass of the flagship path on a real MI355X:
  1. HIP/CDNA4 diagnostics on device 0 (1 GiB HBM pattern test, MFMA rate check, an MFMA
     GEMM compared with a host fp32 product, MX fp8 / fp4 block-scaled MFMA tiles, two
     launches of the 8-phase ping-pong soak GEMM at 1024^3 under its ABFT checksums) — the
     native kernels in libbgc_gpu_diag.so, no fallback;
  2. amdsmi discovery of device 0 (gfx950, HBM3E capacity);
  3. a one-tenant onboarding through kube-lite -> TLS webhook -> controller ->
     synchronizer, with the node agent advertising the GPU, until Ready.
Raises on any failure.
"""
import json
import time


def run_smoke(device=0):
    from . import native, ops
    from .testing.cluster import Cluster
    from .testing.fake_google import FakeGoogle
    from .testing.kubeapi import wait_for

    nat = native()
    arch = ops.device_arch(device)
    if not arch.startswith("gfx950"):
        raise RuntimeError(f"expected an MI355X (gfx950), found {arch}")
    # sized to reach the steady rates (a 64 MiB pass or 4 waves per CU mostly time the launch)
    hbm = ops.hbm(device, nbytes=1 << 30, iters=3)
    mfma = ops.mfma(device, waves_per_cu=32, iters=4096)
    gemm = json.loads(nat.diag_gemm_check(device, 64, 64, 256, 0x5eed))  # MFMA GEMM vs a host fp32 product
    soak = ops.gemm_soak(device, 1024, 1024, 1024, launches=2)
    lowp = ops.mfma_lowp(device, waves_per_cu=4, iters=256)
    if not (hbm["passed"] and mfma["passed"] and gemm["passed"] and soak["passed"] and lowp["passed"]):
        raise RuntimeError(f"GPU diagnostics failed: hbm={hbm} mfma={mfma} gemm={gemm} soak={soak} mx={lowp}")
    if soak.get("kernel") != "pingpong":
        raise RuntimeError(f"soak ran {soak.get('kernel')}, expected the ping-pong kernel")
    gpus = json.loads(nat.gpu_backend("amdsmi", "").discover())
    if not gpus:
        raise RuntimeError("amdsmi discovered no GPUs")

    google = FakeGoogle().start()
    google.set_rows([{"id_username": "smoke", "gpu": 1}])
    try:
        with Cluster() as c:
            c.start_synchronizer(google, interval=60)
            c.start_node_agent(max_gpus=1, backend="amdsmi", poll_interval_ms=200)
            t0 = time.time()
            c.as_user("oidc:smoke", ["gpu"]).create(
                "userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                   "metadata": {"name": "smoke"}, "spec": {}})
            wait_for(lambda: c.admin.get_or_none("rolebindings", "smoke", "smoke"), timeout=30, desc="smoke Ready")
            rq = c.admin.get("resourcequotas", "smoke", "smoke")
            node = c.admin.get("nodes", "mi355x-0")
            ready_ms = (time.time() - t0) * 1e3
    finally:
        google.stop()
    if rq["spec"]["hard"].get("requests.amd.com/gpu") != "1":
        raise RuntimeError(f"unexpected quota {rq['spec']}")
    if node["status"]["capacity"].get("amd.com/gpu") != "1":
        raise RuntimeError(f"node not advertised: {node['status']}")
    print(json.dumps({"smoke": "ok", "arch": arch, "hbm_read_gbps": round(hbm["read_gbps"], 1),
                      "mfma_tflops": round(mfma["tflops"], 1), "gemm_max_abs_err": gemm["max_abs_err"],
                      "soak_kernel": soak["kernel"], "mx_tiles_checked": lowp["tiles_checked"],
                      "apply_to_ready_ms": round(ready_ms, 2),
                      "node_labels": {k: v for k, v in node["metadata"]["labels"].items() if "product" in k or "vram" in k}}))


if __name__ == "__main__":
    run_smoke()
