"""The built HIP libraries register their op schemas on load, which needs no GPU: a
schema typo aborts the process at ``load_library`` -- catch it here on the CPU, not on
a GPU box.  (Skipped where the libraries were not built.)"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kubernetes_gpu_cluster_amd")

OPS = ["rms_norm", "rope_kv_write", "paged_decode", "paged_decode_rope", "prefill_attention", "sample", "sample_vp",
       "sample_vp_unpack", "dgemm", "dgemm_pack", "xgmi_allreduce", "xgmi_allreduce_rms",
       "moe_route", "debug_errors", "debug_build"]


@pytest.mark.parametrize("name,debug", [("_kgc_ops.so", False), ("_kgc_ops_debug.so", True)])
def test_library_registers_ops(name, debug):
    so = os.path.join(PKG, name)
    if not os.path.exists(so):
        pytest.skip(f"{name} not built")
    code = (f"import torch; torch.ops.load_library({so!r}); k = torch.ops.kgc; "
            f"missing = [o for o in {OPS!r} if not hasattr(k, o)]; "
            f"assert not missing, missing; assert bool(k.debug_build()) is {debug}; print('ok')")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
