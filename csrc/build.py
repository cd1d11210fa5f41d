"""In-tree build of the gfx950 HIP kernels into ``kubernetes_gpu_cluster_amd/_kgc_ops.so``.

Drives ``hipcc`` directly (no hipify, no torch JIT cache) so the exact same
``.so`` travels with the repo snapshot to the GPU box:

    python csrc/build.py [--force] [-j N] [--arch gfx950]
    KGC_HIP_DEBUG=1 python csrc/build.py      # or --debug

The debug build (``_kgc_ops_debug.so``, its own object directory) defines
``KGC_DEBUG``: the attention / KV-write kernels (K1, K2, K3) range-check every block
table entry, slot and context length they read, clamp a bad one, and report it
through ``kgc.debug_errors()``.  ``KGC_HIP_DEBUG=1`` at run time makes
``ops.load_extension`` load that library and raise after every step that tripped a check.

Kernel translation units (``csrc/kernels/*.hip``) never include torch headers;
only ``csrc/bindings.cpp`` does.  Objects are rebuilt when their source or any
header under csrc/ is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
DEBUG = os.environ.get("KGC_HIP_DEBUG", "0") not in ("", "0")


def _paths(debug: bool) -> tuple[str, str]:
    name = "_kgc_ops_debug.so" if debug else "_kgc_ops.so"
    return (os.path.join(ROOT, "kubernetes_gpu_cluster_amd", name),
            os.path.join(ROOT, "build", "kgc_ops_debug" if debug else "kgc_ops"))


OUT, BUILD = _paths(DEBUG)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    base = os.path.dirname(torch.__file__)
    return (os.path.join(base, "include"), os.path.join(base, "include", "torch", "csrc", "api",
                                                        "include"),
            os.path.join(base, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI))


def _newest_header() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r.stderr


def build(force: bool = False, jobs: int = 8, arch: str = "gfx950", verbose: bool = False,
          debug: bool = DEBUG) -> str:
    inc, api_inc, lib, abi = _torch_paths()
    OUT, BUILD = _paths(debug)
    os.makedirs(BUILD, exist_ok=True)
    hdr_t = _newest_header()
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={arch}", "-I", CSRC,
              "-D__HIP_PLATFORM_AMD__=1", "-Wno-unused-result", "-ffp-contract=fast"]
    if debug:
        common.append("-DKGC_DEBUG=1")
    kern = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    jobs_list = []
    for src in kern:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        jobs_list.append((src, obj, ["-x", "hip"] + common))
    bind = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(BUILD, "bindings.o")
    bflags = ["-x", "hip", "-O2", "-fPIC", "-std=c++17", f"--offload-arch={arch}", "-I", CSRC,
              "-isystem", inc, "-isystem", api_inc,
              "-isystem", sysconfig.get_paths()["include"],
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
              "-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-deprecated-declarations",
              "-Wno-unused-parameter"] + (["-DKGC_DEBUG=1"] if debug else [])
    jobs_list.append((bind, bobj, bflags))

    def stale(src, obj):
        if force or not os.path.exists(obj):
            return True
        t = os.path.getmtime(obj)
        return os.path.getmtime(src) > t or hdr_t > t

    todo = [(s, o, f) for s, o, f in jobs_list if stale(s, o)]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {ex.submit(_run, [HIPCC] + f + ["-c", s, "-o", o]): s for s, o, f in todo}
        for fu in cf.as_completed(futs):
            msg = fu.result()
            if verbose and msg.strip():
                print(msg, file=sys.stderr)
    objs = [o for _, o, _ in jobs_list]
    if todo or not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT)
                                               for o in objs):
        tmp = OUT + ".tmp"
        _run([HIPCC, "-shared", f"--offload-arch={arch}", "-fPIC", "-o", tmp] + objs +
             ["-L", lib, "-Wl,-rpath," + lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
              "-ltorch_hip", "-lamdhip64"])
        os.replace(tmp, OUT)
    return OUT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 8))
    ap.add_argument("--arch", default="gfx950")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true", help="the KGC_DEBUG bounds-checking build")
    a = ap.parse_args()
    print(build(a.force, a.jobs, a.arch, a.verbose, debug=a.debug or DEBUG))


if __name__ == "__main__":
    main()
