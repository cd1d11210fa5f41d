"""Fake MI355X node trees for the native node-tool and device-plugin tests:
KFD topology sysfs, DRM render/card nodes, PCI NUMA, RAS counters, /etc/group and a
device-number manifest (``dev/.kgc_devices``) standing in for real char devices."""
from __future__ import annotations

import os

MI355X_DEVICE_ID = 0x75A3
GFX950 = 90500


def _w(path: str, text: str) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def make_node(root: str, n_gpus: int = 8, partitions: int = 1, cpu_nodes: int = 2,
              missing_render: tuple = (), ras_ue: dict | None = None) -> str:
    """Populate ``root`` with n_gpus physical GPUs (each split into `partitions`
    compute partitions).  Returns root."""
    ras_ue = ras_ue or {}
    topo = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    devlines = ["/dev/kfd 235 0"]
    node = 0
    for c in range(cpu_nodes):
        _w(f"{topo}/{node}/gpu_id", "0\n")
        _w(f"{topo}/{node}/properties", "cpu_cores_count 96\nsimd_count 0\n")
        node += 1
    gpu_nodes = []
    idx = 0
    for g in range(n_gpus):
        bus = 0x05 + 0x10 * g
        for p in range(partitions):
            minor = 128 + idx
            props = {
                "cpu_cores_count": 0, "simd_count": 1024 // partitions,
                "gfx_target_version": GFX950, "vendor_id": 0x1002, "device_id": MI355X_DEVICE_ID,
                "location_id": (bus << 8) | p, "domain": 0, "drm_render_minor": minor,
                "unique_id": 0xABC000 + g, "num_xcc": 8 // partitions, "hive_id": 0x77,
                "simd_per_cu": 4,
            }
            _w(f"{topo}/{node}/gpu_id", f"{1000 + idx}\n")
            _w(f"{topo}/{node}/properties", "".join(f"{k} {v}\n" for k, v in props.items()))
            _w(f"{topo}/{node}/mem_banks/0/properties",
               f"heap_type 1\nsize_in_bytes {288 * 10**9 // partitions}\n")
            bdf = f"0000:{bus:02x}:00.{p}"
            _w(os.path.join(root, f"sys/bus/pci/devices/{bdf}/numa_node"), f"{g // 4}\n")
            _w(os.path.join(root, f"sys/class/drm/renderD{minor}/device/drm/card{idx}/.keep"), "")
            ue = ras_ue.get(idx, 0)
            _w(os.path.join(root, f"sys/class/drm/card{idx}/device/ras/umc_err_count"),
               f"ue: {ue}\nce: 3\n")
            if idx not in missing_render:
                _w(os.path.join(root, f"dev/dri/renderD{minor}"), "")
                devlines.append(f"/dev/dri/renderD{minor} 226 {minor}")
            _w(os.path.join(root, f"dev/dri/card{idx}"), "")
            devlines.append(f"/dev/dri/card{idx} 226 {idx}")
            gpu_nodes.append((node, g))
            node += 1
            idx += 1
    # xGMI full mesh between physical GPUs (CRAT io-link type 11)
    for a, ga in gpu_nodes:
        k = 0
        for b, gb in gpu_nodes:
            if ga == gb:
                continue
            _w(f"{topo}/{a}/io_links/{k}/properties", f"type 11\nnode_from {a}\nnode_to {b}\nweight 15\n")
            k += 1
        _w(f"{topo}/{a}/io_links/{k}/properties", f"type 2\nnode_from {a}\nnode_to 0\nweight 20\n")
    _w(os.path.join(root, "dev/kfd"), "")
    _w(os.path.join(root, "dev/.kgc_devices"), "\n".join(devlines) + "\n")
    _w(os.path.join(root, "etc/group"), "root:x:0:\nvideo:x:44:\nrender:x:109:\n")
    return root


def make_bundle(path: str, env: list[str] | None = None, annotations: dict | None = None) -> str:
    import json
    os.makedirs(os.path.join(path, "rootfs/dev"), exist_ok=True)
    cfg = {"ociVersion": "1.0.2", "process": {"user": {"uid": 0, "gid": 0}, "args": ["sh"],
                                              "env": ["PATH=/usr/bin"] + (env or [])},
           "root": {"path": "rootfs"}, "linux": {"resources": {"devices": [
               {"allow": False, "access": "rwm"}]}}}
    if annotations:
        cfg["annotations"] = annotations
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(cfg, f)
    return path
