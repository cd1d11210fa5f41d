"""amd.com/gpu device plugin against an in-process fake kubelet (Registration
service on a temp unix socket) and a fake 8x MI355X sysfs tree."""
import os
import subprocess
import tempfile
import threading
import time
from concurrent import futures

import grpc
import pytest

from fake_node import make_node
from kubernetes_gpu_cluster_amd.k8s.deviceplugin import api
from kubernetes_gpu_cluster_amd.k8s.deviceplugin.plugin import AMDGPUPlugin, preferred

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def native():
    subprocess.run(["bash", os.path.join(ROOT, "native", "build.sh")], check=True)


class FakeKubelet:
    def __init__(self, sock):
        self.sock = sock
        self.requests = []
        self.event = threading.Event()
        self.server = None

    def Register(self, req, ctx):
        self.requests.append(req)
        self.event.set()
        return api.Empty()

    def start(self):
        h = grpc.method_handlers_generic_handler(f"{api.PACKAGE}.Registration", {
            "Register": grpc.unary_unary_rpc_method_handler(
                self.Register, request_deserializer=api.RegisterRequest.FromString,
                response_serializer=api.Empty.SerializeToString)})
        self.server = grpc.server(futures.ThreadPoolExecutor(2))
        self.server.add_generic_rpc_handlers((h,))
        self.server.add_insecure_port(f"unix://{self.sock}")
        self.server.start()

    def stop(self):
        self.server.stop(0).wait()
        if os.path.exists(self.sock):
            os.unlink(self.sock)


def _stub(sock):
    ch = grpc.insecure_channel(f"unix://{sock}")
    grpc.channel_ready_future(ch).result(timeout=5)
    def mk(name, req, resp, stream=False):
        f = ch.unary_stream if stream else ch.unary_unary
        return f(api.method_path("DevicePlugin", name), request_serializer=api.MSG[req].SerializeToString,
                 response_deserializer=api.MSG[resp].FromString)
    return ch, {n: mk(n, r, s, st) for n, r, s, st in api.SERVICES["DevicePlugin"]}


def test_plugin_lifecycle():
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        root = make_node(os.path.join(d, "node"))
        pdir = os.path.join(d, "dp")
        os.makedirs(pdir)
        kubelet = FakeKubelet(os.path.join(pdir, "kubelet.sock"))
        kubelet.start()
        plugin = AMDGPUPlugin(root=root, plugin_dir=pdir, health_interval=0.2)
        t = threading.Thread(target=plugin.run, daemon=True)
        t.start()
        try:
            assert kubelet.event.wait(10)
            reg = kubelet.requests[0]
            assert reg.resource_name == "amd.com/gpu" and reg.version == "v1beta1"
            assert reg.endpoint == "amd-gpu.sock" and reg.options.get_preferred_allocation_available
            ch, s = _stub(plugin.socket)
            opts = s["GetDevicePluginOptions"](api.Empty())
            assert opts.get_preferred_allocation_available
            stream = s["ListAndWatch"](api.Empty())
            first = next(stream)
            assert len(first.devices) == 8
            assert all(dv.health == api.HEALTHY for dv in first.devices)
            assert first.devices[5].topology.nodes[0].ID == 1
            ids = [dv.ID for dv in first.devices]
            # health change: RAS uncorrectable error on GPU 2 -> Unhealthy update
            with open(os.path.join(root, "sys/class/drm/card2/device/ras/umc_err_count"), "w") as f:
                f.write("ue: 1\nce: 0\n")
            upd = next(stream)
            assert [dv.health for dv in upd.devices].count(api.UNHEALTHY) == 1
            assert upd.devices[2].health == api.UNHEALTHY
            # Allocate -> device specs + env + annotation
            r = s["Allocate"](api.AllocateRequest(container_requests=[
                api.ContainerAllocateRequest(devices_ids=[ids[3], ids[1]])]))
            cr = r.container_responses[0]
            assert cr.envs["AMD_VISIBLE_DEVICES"] == "1,3"
            paths = [dv.container_path for dv in cr.devices]
            assert paths == ["/dev/kfd", "/dev/dri/renderD129", "/dev/dri/card1",
                             "/dev/dri/renderD131", "/dev/dri/card3"]
            assert all(dv.permissions == "rw" for dv in cr.devices)
            with pytest.raises(grpc.RpcError):
                s["Allocate"](api.AllocateRequest(container_requests=[
                    api.ContainerAllocateRequest(devices_ids=["bogus"])]))
            # preferred allocation: NUMA-local
            pr = s["GetPreferredAllocation"](api.PreferredAllocationRequest(container_requests=[
                api.ContainerPreferredAllocationRequest(available_deviceIDs=ids,
                                                        must_include_deviceIDs=[ids[5]],
                                                        allocation_size=3)]))
            got = list(pr.container_responses[0].deviceIDs)
            assert got[0] == ids[5] and all(ids.index(x) >= 4 for x in got)
            stream.cancel()
            ch.close()
            # kubelet restart -> re-registration
            kubelet.stop()
            kubelet.event.clear()
            kubelet2 = FakeKubelet(os.path.join(pdir, "kubelet.sock"))
            kubelet2.start()
            deadline = time.time() + 10
            while not kubelet2.requests and time.time() < deadline:
                time.sleep(0.1)
            assert kubelet2.requests and kubelet2.requests[0].resource_name == "amd.com/gpu"
            kubelet2.stop()
        finally:
            plugin.stop()


def test_preferred_packs_partitions():
    by_id = {f"d{i}": {"index": i, "unique_id": f"u{i // 4}", "numa_node": i // 8}
             for i in range(16)}
    got = preferred(list(by_id), ["d5"], 4, by_id)
    assert got[0] == "d5" and {by_id[d]["unique_id"] for d in got} == {"u1"}


def test_proto_wire_compat():
    """Field numbers/names survive a serialize round trip (wire contract)."""
    r = api.ContainerAllocateResponse()
    r.envs["A"] = "1"
    r.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
    r.cdi_devices.add(name="amd.com/gpu=0")
    r2 = api.ContainerAllocateResponse.FromString(r.SerializeToString())
    assert r2.envs["A"] == "1" and r2.devices[0].permissions == "rw"
    raw = api.RegisterRequest(version="v1beta1", endpoint="x.sock", resource_name="amd.com/gpu").SerializeToString()
    assert raw[:2] == b"\x0a\x07"     # field 1 (version), wire type 2, len 7
