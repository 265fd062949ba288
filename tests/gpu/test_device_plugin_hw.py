"""Device plugin on a real MI355X: amdsmi-discovered GPUs are served to a (grpcio) fake
kubelet, and Allocate hands out the host's actual DRM nodes, resolved through sysfs
from each GPU's PCI BDF."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu


def test_device_plugin_allocates_real_drm_nodes(tmp_path):
    from bacchus_gpu_controller_amd import native
    from bacchus_gpu_controller_amd.testing.kubelet import FakeKubelet, PluginClient, pb

    n = native()
    gpus = json.loads(n.gpu_backend("amdsmi", "").discover())
    assert gpus and gpus[0]["gfx_target"].startswith("gfx950")
    d = str(tmp_path / "dp")
    os.makedirs(d)
    kubelet = FakeKubelet(d).start()
    plugin = n.DevicePlugin(json.dumps(gpus), {"plugin_dir": d, "watch_interval_ms": "50"})
    plugin.start()
    try:
        assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists, timeout=15)
        devs = kubelet.device_lists[-1][1]
        assert [x[0] for x in devs] == [g["bdf"] for g in gpus]
        assert all(x[1] == "Healthy" for x in devs)
        c = PluginClient(plugin.socket_path)
        try:
            req = pb["AllocateRequest"]()
            req.container_requests.add().devices_ids.append(gpus[0]["bdf"])
            resp = c.allocate(req, timeout=10).container_responses[0]
        finally:
            c.close()
        paths = {x.container_path: x.host_path for x in resp.devices}
        assert paths["/dev/kfd"] == "/dev/kfd" and os.path.exists("/dev/kfd")
        drm = sorted(os.listdir(f"/sys/bus/pci/devices/{gpus[0]['bdf']}/drm"))
        render = next(x for x in drm if x.startswith("renderD"))
        assert paths[f"/dev/dri/{render}"] == f"/dev/dri/{render}"
        assert os.path.exists(f"/dev/dri/{render}")
        assert resp.envs["BGC_AMD_GPU_IDS"] == gpus[0]["bdf"]
    finally:
        plugin.stop()
        kubelet.stop()
