"""Python binding of libamdgpu-topo (native/topo) via ctypes, with a CLI fallback.

Used by the amd.com/gpu device plugin for enumeration and health."""
from __future__ import annotations

import ctypes
import json
import os
import shutil
import subprocess
from typing import Optional

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_SEARCH = [os.environ.get("KGC_TOPO_LIB", ""),
           os.path.join(_REPO, "build", "native", "libamdgpu_topo.so"),
           "/usr/local/lib/libamdgpu_topo.so", "/usr/lib/libamdgpu_topo.so"]
_lib: Optional[ctypes.CDLL] = None


def _load() -> Optional[ctypes.CDLL]:
    global _lib
    if _lib is None:
        for p in _SEARCH:
            if p and os.path.exists(p):
                lib = ctypes.CDLL(p)
                lib.kgc_topo_json.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
                lib.kgc_topo_json.restype = ctypes.c_int
                lib.kgc_topo_free.argtypes = [ctypes.c_void_p]
                _lib = lib
                break
    return _lib


def topology(root: str = "/") -> dict:
    lib = _load()
    if lib is not None:
        out = ctypes.c_void_p()
        if lib.kgc_topo_json(root.encode(), ctypes.byref(out)) == 0 and out.value:
            try:
                return json.loads(ctypes.string_at(out.value).decode())
            finally:
                lib.kgc_topo_free(out)
    cli = shutil.which("amdgpu-topo") or os.path.join(_REPO, "build", "native", "amdgpu-topo")
    if os.path.exists(cli):
        return json.loads(subprocess.run([cli, "--root", root], check=True, capture_output=True,
                                         text=True).stdout)
    raise RuntimeError("libamdgpu_topo not found (run native/build.sh)")


def enumerate_gpus(root: str = "/") -> list[dict]:
    return topology(root)["gpus"]
