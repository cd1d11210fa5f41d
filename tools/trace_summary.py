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


def load(path: str):
    """(start_ns, end_ns, kernel name) of every dispatch, from a rocprofv3 kernel-trace
    CSV or a rocpd SQLite database (rocprofv3's default output format on ROCm 7)."""
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        return sorted(con.execute("select start, end, name from kernels"))
    rows = list(csv.DictReader(open(path)))
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
        if "--detail" in sys.argv:
            # per kernel instantiation (template arguments kept): calls per step, us per call
            # an instantiation called k times per layer (o and down share one) is split by
            # its occurrence index mod k: "#0", "#1" in call order
            per_step = collections.Counter(n for s, e, n in ev[samp[0] + 1:samp[1] + 1])
            layers = 32
            for a, b in zip(samp, samp[1:]):
                seg = ev[a + 1:b + 1]
                if len(seg) == nk:
                    per_step = collections.Counter(n for s, e, n in seg)
                    break
            byname, ncall = collections.Counter(), collections.Counter()
            for a, b in zip(samp, samp[1:]):
                seg = ev[a + 1:b + 1]
                if len(seg) != nk:
                    continue
                seen = collections.Counter()
                for s, e, n in seg:
                    k = per_step[n] // layers if per_step[n] % layers == 0 else 1
                    key = f"#{seen[n] % k} {n}" if k > 1 else n
                    seen[n] += 1
                    byname[key] += e - s
                    ncall[key] += 1
            print("\ndecode-step kernels by instantiation (calls/step, us/call, us/step):")
            for n, v in byname.most_common(24):
                c = ncall[n] / len(dec)
                print(f"   {c:6.1f} {v / ncall[n] / 1e3:8.2f} {v / len(dec) / 1e3:9.1f}  {n[:110]}")
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
