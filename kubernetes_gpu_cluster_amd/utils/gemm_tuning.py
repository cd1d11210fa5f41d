"""Load the offline-tuned hipBLASLt selections (tools/tune_gemms.py) for the
decode-graph GEMM shapes.  Read-only: untuned shapes (e.g. arbitrary prefill
token counts) keep hipBLASLt's default heuristic, nothing is tuned at run time.
Disable with KGC_GEMM_TUNING=0; point at another table with KGC_GEMM_TABLE."""
from __future__ import annotations

import logging
import os

log = logging.getLogger("kgc.gemm")
_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def default_table_path(model: str, tp: int = 1) -> str:
    return os.path.join(_REPO, "profiles", "tunableop", f"{model}_tp{tp}_gfx950.csv")


def enable_tuned_gemms(model: str, tp: int = 1) -> bool:
    if os.environ.get("KGC_GEMM_TUNING", "1") == "0":
        return False
    path = os.environ.get("KGC_GEMM_TABLE") or default_table_path(model, tp)
    if not os.path.exists(path):
        return False
    import torch
    try:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(False)
        torch.cuda.tunable.set_filename(path, insert_device_ordinal=False)
        ok = torch.cuda.tunable.read_file(path)
    except Exception as e:  # noqa: BLE001
        log.warning("tuned GEMM table %s not usable: %s", path, e)
        return False
    if not ok:
        log.warning("tuned GEMM table %s rejected (validator mismatch?)", path)
        torch.cuda.tunable.enable(False)
        return False
    log.info("using tuned GEMM table %s", path)
    return True
