"""The bounds-checking HIP build (``KGC_HIP_DEBUG=1 python csrc/build.py`` ->
``_kgc_ops_debug.so``): K1 paged decode, K2 prefill attention and K3 RoPE/KV-write
range-check the block-table entries, slots and lengths they read.  A bad value is
printed, clamped (no out-of-bounds access) and raised on the host by
``ops.debug_check()``.  Run in a child process: one process cannot load both builds."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import torch
from kubernetes_gpu_cluster_amd import ops
assert ops.DEBUG and ops.extension_path().endswith("_kgc_ops_debug.so")
ops.load_extension(strict=True)
assert torch.ops.kgc.debug_build()
dev = torch.device("cuda", 0)
nb, nkv, bs, d, nq = 8, 2, 16, 128, 4
kc = torch.zeros(nb, nkv, bs, d, dtype=torch.bfloat16, device=dev)
vc = torch.zeros(nb, nkv, bs // 8, d, 8, dtype=torch.bfloat16, device=dev)
q = torch.randn(2, nq, d, dtype=torch.bfloat16, device=dev)
cl = torch.tensor([20, 5], dtype=torch.int32, device=dev)
good = torch.tensor([[1, 2], [3, 0]], dtype=torch.int32, device=dev)
ops.paged_attention_decode(q, kc, vc, good, cl, d ** -0.5)
ops.debug_check()                                   # valid tables: no error
bad = torch.tensor([[1, 99], [3, 0]], dtype=torch.int32, device=dev)   # block 99 of 8
ops.paged_attention_decode(q, kc, vc, bad, cl, d ** -0.5)
try:
    ops.debug_check()
    raise SystemExit("decode: bad block id not reported")
except ops.KernelDebugCheckFailed as e:
    assert "K1" in str(e), e
# K3: slot beyond the cache
T = 3
qkv = torch.randn(T, (nq + 2 * nkv) * d, dtype=torch.bfloat16, device=dev)
pos = torch.arange(T, dtype=torch.int64, device=dev)
cs = torch.randn(64, d, device=dev)
slots = torch.tensor([0, 5, nb * bs + 3], dtype=torch.int64, device=dev)
ops.rope_kv_write(qkv, pos, cs, kc, vc, slots, nq, nkv, d)
try:
    ops.debug_check()
    raise SystemExit("rope: bad slot not reported")
except ops.KernelDebugCheckFailed as e:
    assert "K3" in str(e), e
ops.debug_check()                                   # cleared after the raise
# K1 with K3 folded in (decode-only steps): the new token's slot is range-checked too
qkv2 = torch.randn(2, (nq + 2 * nkv) * d, dtype=torch.bfloat16, device=dev)
pos2 = (cl - 1).long()
ok_slots = torch.tensor([2 * bs + 3, 3 * bs + 4], dtype=torch.int64, device=dev)
ops.paged_attention_decode_rope(qkv2, pos2, cs, kc, vc, ok_slots, nq, nkv, d, good, cl, d ** -0.5)
ops.debug_check()
bad_slots = torch.tensor([2 * bs + 3, nb * bs + 1], dtype=torch.int64, device=dev)
ops.paged_attention_decode_rope(qkv2, pos2, cs, kc, vc, bad_slots, nq, nkv, d, good, cl, d ** -0.5)
try:
    ops.debug_check()
    raise SystemExit("decode+rope: bad slot not reported")
except ops.KernelDebugCheckFailed as e:
    assert "K1" in str(e), e
print("DEBUG-BUILD-OK")
'''


def test_debug_build_reports_bad_indices(gpu):
    so = os.path.join(ROOT, "kubernetes_gpu_cluster_amd", "_kgc_ops_debug.so")
    if not os.path.exists(so):
        pytest.fail("debug build missing: run KGC_HIP_DEBUG=1 python csrc/build.py")
    # ROOT appended to (never replacing) the inherited PYTHONPATH: whatever the parent's
    # environment puts on the path (e.g. a harness's library-load observer) reaches the child
    pp = os.environ.get("PYTHONPATH", "")
    env = dict(os.environ, KGC_HIP_DEBUG="1",
               PYTHONPATH=os.pathsep.join([p for p in pp.split(os.pathsep) if p] + [ROOT]))
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0 and "DEBUG-BUILD-OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    assert "kgc debug check" in r.stdout + r.stderr     # the device printf names the value
