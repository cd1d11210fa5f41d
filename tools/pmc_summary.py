"""Summarise a rocprofv3 PMC run (rocpd SQLite db) per kernel.

    python tools/pmc_summary.py gpurun_out/pmc_x/p_results.db [--match dgemm]

Prints, per kernel name: dispatches, mean duration, every collected counter averaged per
dispatch, plus derived values when their inputs were collected:
  clock_GHz   = GRBM_GUI_ACTIVE / 8 XCDs / duration   (MI355X_MICROARCH.md, DVFS give-back)
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES  (waves parked on s_waitcnt / barrier)
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select * from counters_collection limit 1").description
    cols = [d[0] for d in rows]
    name_col = "kernel_name" if "kernel_name" in cols else None
    q = ("select dispatch_id, {}, counter_name, value, start, end from counters_collection"
         .format(name_col or "kernel_id"))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for did, kname, cname, val, st, en in c.execute(q):
        kname = str(kname)
        if a.match and a.match not in kname:
            continue
        per[kname][cname].append(val)
        dur[kname][did] = en - st
    for k, cs in per.items():
        d = list(dur[k].values())
        ns = sum(d) / len(d)
        out = {"kernel": k[:110], "dispatches": len(d), "us": round(ns / 1e3, 2)}
        avg = {n: sum(v) / len(v) for n, v in cs.items()}
        for n, v in sorted(avg.items()):
            out[n] = round(v, 1)
        if "GRBM_GUI_ACTIVE" in avg:
            cyc = avg["GRBM_GUI_ACTIVE"] / 8
            out["clock_GHz"] = round(cyc / ns, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                out["mfma_busy"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 256 * 4), 3)
        if "SQ_WAIT_ANY" in avg and avg.get("SQ_WAVE_CYCLES"):
            out["wait_frac"] = round(avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"], 3)
            out["inst_wait_frac"] = round(avg.get("SQ_WAIT_INST_ANY", 0) / avg["SQ_WAVE_CYCLES"], 3)
        print(out)


if __name__ == "__main__":
    main()
