"""``amd.com/gpu`` Kubernetes device plugin for MI355X nodes (replaces the NVIDIA
k8s-device-plugin DaemonSet of the reference, ``README.md:90``).

* Enumeration + health: libamdgpu-topo (KFD sysfs; a GPU whose render node is
  gone or whose RAS counters report uncorrectable errors goes ``Unhealthy``).
* ``ListAndWatch`` streams the device list with NUMA topology and re-sends it on
  any health change (poll interval ``--health-interval``).
* ``Allocate`` returns DeviceSpecs for ``/dev/kfd`` + the GPUs' render (and card)
  nodes -- the AMD analog of ``--pass-device-specs=true``, the setting that
  finally worked for the reference (``old_README.md:1164-1173``) -- so CRI-O adds
  the device-cgroup rules itself; plus ``AMD_VISIBLE_DEVICES`` for the OCI shim path
  and, with ``--device-list-strategy cdi``, CDI device names.
* ``GetPreferredAllocation`` packs requests xGMI/NUMA-locally: partitions of the
  same physical GPU first, then GPUs of one NUMA node, then lowest index.
* Re-registers when the kubelet restarts (its socket is re-created).

    python -m kubernetes_gpu_cluster_amd.k8s.deviceplugin.plugin [--root /] \\
        [--plugin-dir /var/lib/kubelet/device-plugins] [--device-list-strategy device-specs]
"""
from __future__ import annotations

import argparse
import logging
import os
import threading
import time
from concurrent import futures
from typing import Optional

import grpc

from .. import topo as topo_mod
from . import api

log = logging.getLogger("kgc.deviceplugin")

RESOURCE = "amd.com/gpu"
SOCKET_NAME = "amd-gpu.sock"


def device_id(g: dict) -> str:
    return g["pci_bdf"]


class AMDGPUPlugin:
    def __init__(self, root: str = "/", plugin_dir: str = api.DEVICE_PLUGIN_PATH,
                 health_interval: float = 5.0, strategy: str = "device-specs",
                 resource: str = RESOURCE, with_card: bool = True):
        self.root = root
        self.plugin_dir = plugin_dir
        self.health_interval = health_interval
        self.strategy = strategy
        self.resource = resource
        self.with_card = with_card
        self.socket = os.path.join(plugin_dir, SOCKET_NAME)
        self.kubelet_socket = os.path.join(plugin_dir, "kubelet.sock")
        self.server: Optional[grpc.Server] = None
        self._stop = threading.Event()
        self._changed = threading.Condition()
        self._gen = 0
        self.gpus: list[dict] = []
        self.refresh()

    # ------------------------------------------------------------------ inventory
    def refresh(self) -> bool:
        gpus = topo_mod.enumerate_gpus(self.root)
        key = [(device_id(g), g["healthy"]) for g in gpus]
        old = [(device_id(g), g["healthy"]) for g in self.gpus]
        if key != old:
            self.gpus = gpus
            with self._changed:
                self._gen += 1
                self._changed.notify_all()
            return True
        return False

    def devices(self) -> list:
        out = []
        for g in self.gpus:
            d = api.Device(ID=device_id(g), health=api.HEALTHY if g["healthy"] else api.UNHEALTHY)
            if g["numa_node"] >= 0:
                d.topology.nodes.add(ID=g["numa_node"])
            out.append(d)
        return out

    def _by_id(self) -> dict:
        return {device_id(g): g for g in self.gpus}

    # ------------------------------------------------------------------ RPCs
    def GetDevicePluginOptions(self, request, context):
        return api.DevicePluginOptions(pre_start_required=False,
                                       get_preferred_allocation_available=True)

    def ListAndWatch(self, request, context):
        gen = -1
        while not self._stop.is_set() and context.is_active():
            with self._changed:
                if gen == self._gen:
                    self._changed.wait(timeout=1.0)
                if gen == self._gen:
                    continue
                gen = self._gen
            yield api.ListAndWatchResponse(devices=self.devices())

    def GetPreferredAllocation(self, request, context):
        resp = api.PreferredAllocationResponse()
        by_id = self._by_id()
        for creq in request.container_requests:
            chosen = preferred(list(creq.available_deviceIDs), list(creq.must_include_deviceIDs),
                               creq.allocation_size, by_id)
            resp.container_responses.add(deviceIDs=chosen)
        return resp

    def Allocate(self, request, context):
        resp = api.AllocateResponse()
        by_id = self._by_id()
        for creq in request.container_requests:
            cr = resp.container_responses.add()
            gpus = []
            for did in creq.devices_ids:
                g = by_id.get(did)
                if g is None:
                    context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unknown device {did}")
                gpus.append(g)
            gpus.sort(key=lambda g: g["index"])
            idx = ",".join(str(g["index"]) for g in gpus)
            cr.envs["AMD_VISIBLE_DEVICES"] = idx
            if self.strategy in ("device-specs", "envvar+device-specs"):
                paths = ["/dev/kfd"]
                for g in gpus:
                    paths.append(f"/dev/dri/renderD{g['render_minor']}")
                    # the card node is optional for compute: only hand the kubelet device
                    # specs whose host node exists (a missing one fails container creation;
                    # seen on a real MI355X whose container exposes render nodes only)
                    card = f"/dev/dri/card{g['card']}"
                    if (self.with_card and g["card"] >= 0 and
                            os.path.exists(os.path.join(self.root, card.lstrip("/")))):
                        paths.append(card)
                for p in paths:
                    cr.devices.add(container_path=p, host_path=p, permissions="rw")
            if self.strategy == "cdi":
                for g in gpus:
                    cr.cdi_devices.add(name=f"{RESOURCE}={g['index']}")
            cr.annotations["amd.com/gpu.devices"] = idx
        return resp

    def PreStartContainer(self, request, context):
        return api.PreStartContainerResponse()

    # ------------------------------------------------------------------ server
    def _handlers(self):
        h = {}
        for name, req, resp, stream in api.SERVICES["DevicePlugin"]:
            fn = getattr(self, name)
            ctor = grpc.unary_stream_rpc_method_handler if stream else grpc.unary_unary_rpc_method_handler
            h[name] = ctor(fn, request_deserializer=api.MSG[req].FromString,
                           response_serializer=api.MSG[resp].SerializeToString)
        return grpc.method_handlers_generic_handler(f"{api.PACKAGE}.DevicePlugin", h)

    def serve(self) -> None:
        if os.path.exists(self.socket):
            os.unlink(self.socket)
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        self.server.add_generic_rpc_handlers((self._handlers(),))
        self.server.add_insecure_port(f"unix://{self.socket}")
        self.server.start()

    def register(self, timeout: float = 5.0) -> None:
        with grpc.insecure_channel(f"unix://{self.kubelet_socket}") as ch:
            grpc.channel_ready_future(ch).result(timeout=timeout)
            reg = ch.unary_unary(api.method_path("Registration", "Register"),
                                 request_serializer=api.RegisterRequest.SerializeToString,
                                 response_deserializer=api.Empty.FromString)
            reg(api.RegisterRequest(version=api.VERSION, endpoint=SOCKET_NAME,
                                    resource_name=self.resource,
                                    options=api.DevicePluginOptions(
                                        get_preferred_allocation_available=True)),
                timeout=timeout)
        log.info("registered %s with kubelet (%d devices)", self.resource, len(self.gpus))

    def stop(self) -> None:
        self._stop.set()
        with self._changed:
            self._changed.notify_all()
        if self.server:
            self.server.stop(grace=1).wait()

    def run(self) -> None:
        """Serve + register, then loop: health polling and kubelet-restart detection."""
        self.serve()
        self.register()
        ident = _sock_id(self.kubelet_socket)
        gone = False
        last = time.monotonic()
        while not self._stop.is_set():
            self._stop.wait(0.2)
            cur = _sock_id(self.kubelet_socket)
            if cur is None:
                gone = True          # kubelet went away; expect a new socket
            elif cur != ident or gone:
                log.info("kubelet restarted; re-registering")
                self.server.stop(grace=0)
                self.serve()
                try:
                    self.register()
                    ident, gone = cur, False
                except (grpc.RpcError, grpc.FutureTimeoutError) as e:
                    log.warning("re-register failed: %s", e)
            if time.monotonic() - last >= self.health_interval:
                last = time.monotonic()
                try:
                    if self.refresh():
                        log.info("device health changed: %s",
                                 [(device_id(g), g["healthy"]) for g in self.gpus])
                except Exception as e:  # noqa: BLE001
                    log.warning("health poll failed: %s", e)


def _sock_id(p: str) -> Optional[tuple]:
    """(inode, ctime) of the kubelet socket; a re-created socket may reuse the inode."""
    try:
        st = os.stat(p)
        return st.st_ino, st.st_ctime_ns
    except FileNotFoundError:
        return None


def preferred(available: list[str], must: list[str], size: int, by_id: dict) -> list[str]:
    """xGMI/NUMA-aware pick: keep must-include, then partitions of already-chosen
    physical GPUs, then GPUs on the chosen NUMA node, then lowest index."""
    chosen = [d for d in must if d in available or d in by_id][:size]
    rest = [d for d in available if d not in chosen and d in by_id]
    while len(chosen) < size and rest:
        uids = {by_id[d]["unique_id"] for d in chosen}
        numas = {by_id[d]["numa_node"] for d in chosen}

        def score(d):
            g = by_id[d]
            return (0 if g["unique_id"] in uids else 1,
                    0 if (not numas or g["numa_node"] in numas) else 1, g["index"])
        rest.sort(key=score)
        chosen.append(rest.pop(0))
    return chosen


def main(argv=None):
    p = argparse.ArgumentParser(description="amd.com/gpu device plugin")
    p.add_argument("--root", default="/")
    p.add_argument("--plugin-dir", default=api.DEVICE_PLUGIN_PATH)
    p.add_argument("--health-interval", type=float, default=5.0)
    p.add_argument("--device-list-strategy", default="device-specs",
                   choices=["device-specs", "envvar", "cdi", "envvar+device-specs"])
    p.add_argument("--resource-name", default=RESOURCE)
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(message)s")
    plugin = AMDGPUPlugin(a.root, a.plugin_dir, a.health_interval, a.device_list_strategy,
                          a.resource_name)
    while True:
        try:
            plugin.run()
            return
        except grpc.FutureTimeoutError:
            log.warning("kubelet socket not ready; retrying")
            time.sleep(2)


if __name__ == "__main__":
    main()
