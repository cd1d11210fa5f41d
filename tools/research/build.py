"""Build the research kernels (K9r ring GEMM, K9v VGPR-ring GEMM) into
``tools/research/_kgc_research.so`` -- a library of its own, separate from the engine's
``_kgc_ops.so``: both designs were measured slower than the shipped K9m
(profiles/README.md, "Round 3: K9r" / "Round 3: K9v") and the engine never loads them.

    python tools/research/build.py [--force]

Then ``torch.ops.load_library("tools/research/_kgc_research.so")`` exposes
``torch.ops.kgc_research.{ring_gemm, ring_pack, ring_cfg_info, ring_num_cfgs, dgemm_vreg}``
(tools/ring_bench.py, tools/dgemm_bench.py --research, tools/research/test_research_gpu.py).
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(HERE, "_kgc_research.so")
BUILD = os.path.join(ROOT, "build", "kgc_research")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def build(force: bool = False, arch: str = "gfx950") -> str:
    sys.path.insert(0, ROOT)
    from csrc.build import _torch_paths
    inc, api_inc, lib, abi = _torch_paths()
    os.makedirs(BUILD, exist_ok=True)
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={arch}", "-I", CSRC,
              "-I", os.path.join(CSRC, "kernels"), "-I", HERE, "-D__HIP_PLATFORM_AMD__=1",
              "-Wno-unused-result", "-ffp-contract=fast"]
    jobs = [(os.path.join(HERE, f), ["-x", "hip"] + common)
            for f in ("gemm_ring.hip", "gemm_vreg.hip", "gemm_wv.hip")]
    jobs.append((os.path.join(HERE, "bindings.cpp"),
                 ["-x", "hip", "-O2", "-fPIC", "-std=c++17", f"--offload-arch={arch}",
                  "-I", HERE, "-isystem", inc, "-isystem", api_inc,
                  "-isystem", sysconfig.get_paths()["include"],
                  f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
                  "-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-deprecated-declarations"]))
    objs, procs = [], []
    for src, flags in jobs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(src) > os.path.getmtime(obj):
            procs.append((src, subprocess.Popen([HIPCC] + flags + ["-c", src, "-o", obj],
                                                stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                                text=True)))
    for src, p in procs:
        out, err = p.communicate()
        if p.returncode:
            raise RuntimeError(f"build of {src} failed:\n{out}{err}")
    subprocess.run([HIPCC, "-shared", f"--offload-arch={arch}", "-fPIC", "-o", OUT] + objs +
                   ["-L", lib, "-Wl,-rpath," + lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
                    "-ltorch_hip", "-lamdhip64"], check=True)
    return OUT


def load():
    """Load the research library (building it first if needed); returns torch.ops.kgc_research."""
    import torch
    if not os.path.exists(OUT):
        build()
    torch.ops.load_library(OUT)
    return torch.ops.kgc_research


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(a.force))
