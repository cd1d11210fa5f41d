"""Summarise a rocprofv3 kernel trace of a bench run.

    python tools/trace_summary.py gpurun_out/prof2/runc/<pid>_kernel_trace.csv [--steps]
    python tools/trace_summary.py gpurun_out/prof4/run_results.db [--steps]   (rocpd)

Prints the per-kernel totals and, with --steps, the steady-state decode-step
anatomy: per step (delimited by the sampler kernel) the span, GPU-busy time,
host gap and the busy time per kernel family.
"""
import collections
import csv
import statistics
import sys


def family(name: str) -> str:
    n = name
    if "skinny_gemm" in n:
        return "skinny_gemm(K9)"
    if "moe_gemm" in n:
        return "moe_gemm(K14)"
    if "dgemm" in n:
        return "dgemm(K9m)"
    if "Cijk" in n or "gemm" in n.lower():
        return "gemm(hipblaslt)"
    for k in ("splitk_add_rms_norm", "splitk_reduce_silu", "splitk_reduce", "decode_gemm",
              "paged_decode_reduce", "paged_decode", "prefill_attn", "rms_norm",
              "silu_mul", "rope_kv", "sample_kernel", "layer_norm", "allreduce", "nccl", "rccl"):
        if k in n:
            return k
    return n[:60]


GRID = {}    # kernel dispatch (start, name) -> workgroups, where the trace records it


def _grid_cols(cols) -> list:
    """The grid-size columns of a rocpd kernels view / kernel-trace CSV, x / y / z order."""
    out = []
    for axis in ("x", "y", "z"):
        for c in cols:
            lc = c.lower()
            if "grid" in lc and lc.endswith(axis) and "workgroup" not in lc:
                out.append(c)
                break
    return out


def load(path: str):
    """(start_ns, end_ns, kernel name) of every dispatch, from a rocprofv3 kernel-trace
    CSV or a rocpd SQLite database (rocprofv3's default output format on ROCm 7).  Grid
    sizes, where present, go to GRID (the per-instantiation view splits shapes by them)."""
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
        g = _grid_cols(cols)
        wg = [c for c in cols if "workgroup_size" in c.lower() or c.lower().startswith("workgroup_")]
        if g:
            q = "select start, end, name, " + ", ".join(g + wg[:3]) + " from kernels"
            rows = list(con.execute(q))
            for r in rows:
                GRID[(r[0], r[2])] = tuple(r[3:])
            return sorted((r[0], r[1], r[2]) for r in rows)
        return sorted(con.execute("select start, end, name from kernels"))
    rows = list(csv.DictReader(open(path)))
    g = _grid_cols(rows[0].keys()) if rows else []
    for r in rows:
        if g:
            GRID[(int(r["Start_Timestamp"]), r["Kernel_Name"])] = tuple(r[c] for c in g)
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in rows)


def main():
    path = sys.argv[1]
    ev = load(path)
    tot = collections.Counter()
    cnt = collections.Counter()
    for s, e, n in ev:
        tot[family(n)] += e - s
        cnt[family(n)] += 1
    T = sum(tot.values())
    print(f"{'family':40} {'ms':>9} {'%':>6} {'calls':>7}")
    for k, v in tot.most_common(20):
        print(f"{k:40} {v / 1e6:9.2f} {100 * v / T:6.1f} {cnt[k]:7}")
    if "--steps" in sys.argv:
        samp = [i for i, (s, e, n) in enumerate(ev) if "sample_kernel" in n]
        steps = []
        for a, b in zip(samp, samp[1:]):
            seg = ev[a + 1:b + 1]
            span = seg[-1][1] - ev[a][1]
            busy = sum(e - s for s, e, n in seg)
            fam = collections.Counter()
            for s, e, n in seg:
                fam[family(n)] += e - s
            steps.append((span, busy, len(seg), fam))
        nk = statistics.median([s[2] for s in steps])
        dec = [s for s in steps if s[2] == nk]
        print(f"\ndecode steps (kernels/step={nk}): {len(dec)}")
        print(f"median span {statistics.median([s[0] for s in dec]) / 1e6:.3f} ms, "
              f"busy {statistics.median([s[1] for s in dec]) / 1e6:.3f} ms")
        agg = collections.Counter()
        for s in dec:
            agg.update(s[3])
        for k, v in agg.most_common(16):
            print(f"   {k:38} {v / len(dec) / 1e3:9.1f} us/step")
        # where the span - busy time goes: the lead gap (previous step's sampler -> this
        # step's first kernel: host-side scheduling / launch) and the gaps between the
        # step's own kernels, summed per (previous family -> next family) boundary
        lead, inner = [], []
        sites = collections.Counter()
        for a, b in zip(samp, samp[1:]):
            seg = ev[a + 1:b + 1]
            if len(seg) != nk:
                continue
            lead.append(max(0, seg[0][0] - ev[a][1]))
            g = 0
            for (s0, e0, n0), (s1, e1, n1) in zip(seg, seg[1:]):
                d = max(0, s1 - e0)
                g += d
                sites[(family(n0), family(n1))] += d
            inner.append(g)
        if lead:
            print(f"gaps: lead (host) median {statistics.median(lead) / 1e3:.1f} us, "
                  f"between the step's kernels median {statistics.median(inner) / 1e3:.1f} us")
            for (f0, f1), v in sites.most_common(8):
                print(f"   {f0[:30]:30} -> {f1[:30]:30} {v / len(lead) / 1e3:8.1f} us/step")
            # one steady-state step's first and last kernels: offset from the previous
            # sampler's end, duration and the gap before each
            mid = [(a, b) for a, b in zip(samp, samp[1:]) if b - a == nk]
            if mid:
                a, b = mid[len(mid) // 2]
                seg = ev[a + 1:b + 1]
                t0, prev = ev[a][1], ev[a][1]
                print("one decode step (offset us, dur us, gap before us, kernel):")
                for i, (s, e, n) in enumerate(seg):
                    if i < 10 or i >= len(seg) - 4:
                        print(f"   {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {(s - prev) / 1e3:7.1f}  {n[:70]}")
                    elif i == 10:
                        print("   ...")
                    prev = e
        if "--detail" in sys.argv:
            # per kernel instantiation (template arguments kept): calls per step, us per call
            # an instantiation called k times per layer (o and down share one) is split by
            # its occurrence index mod k: "#0", "#1" in call order
            # an instantiation launched with different grids (shapes) is split by grid
            # when the trace records it ("[g x,y,z]")
            def name_of(s, n):
                g = GRID.get((s, n))
                return f"{n} [g {','.join(str(v) for v in g)}]" if g else n
            per_step = collections.Counter(name_of(s, n) for s, e, n in ev[samp[0] + 1:samp[1] + 1])
            for a, b in zip(samp, samp[1:]):
                seg = ev[a + 1:b + 1]
                if len(seg) == nk:
                    per_step = collections.Counter(name_of(s, n) for s, e, n in seg)
                    break
            # layers per step: the attention launches (one per layer)
            layers = max(1, sum(v for n, v in per_step.items()
                                if "paged_decode" in n and "reduce" not in n)) or 32
            byname, ncall = collections.Counter(), collections.Counter()
            for a, b in zip(samp, samp[1:]):
                seg = ev[a + 1:b + 1]
                if len(seg) != nk:
                    continue
                seen = collections.Counter()
                for s, e, n0 in seg:
                    n = name_of(s, n0)
                    k = per_step[n] // layers if per_step[n] % layers == 0 else 1
                    key = f"#{seen[n] % k} {n}" if k > 1 else n
                    seen[n] += 1
                    byname[key] += e - s
                    ncall[key] += 1
            print("\ndecode-step kernels by instantiation (calls/step, us/call, us/step):")
            for n, v in byname.most_common(24):
                c = ncall[n] / len(dec)
                print(f"   {c:6.1f} {v / ncall[n] / 1e3:8.2f} {v / len(dec) / 1e3:9.1f}  {n[:150]}")
        # prefill (chunked) steps: the ones that run the prefill attention kernel and no
        # decode-sized GEMM (start-up tuning runs those between sampler calls too)
        pre = [s for s in steps if s[3].get("prefill_attn", 0) > 0
               and not s[3].get("skinny_gemm(K9)") and not s[3].get("dgemm(K9m)")]
        if pre:
            print(f"\nprefill steps: {len(pre)}")
            print(f"median span {statistics.median([s[0] for s in pre]) / 1e6:.3f} ms, "
                  f"busy {statistics.median([s[1] for s in pre]) / 1e6:.3f} ms, "
                  f"total span {sum(s[0] for s in pre) / 1e6:.1f} ms")
            agg = collections.Counter()
            for s in pre:
                agg.update(s[3])
            for k, v in agg.most_common(16):
                print(f"   {k:38} {v / len(pre) / 1e3:9.1f} us/step")


if __name__ == "__main__":
    main()
