"""Summarise a torch.profiler Chrome trace of engine steps (KGC_TORCH_PROFILE=dir:start:n):
the host-side runtime calls that take long (graph launches, copies, event / stream waits)
and the GPU idle gaps, on one time axis, so a GPU gap can be matched to what the host was
doing at that moment.

    python tools/host_trace_summary.py gpurun_out/tp/engine_steps_300_305.json [--min-us 20]
"""
import json
import sys


def main():
    path = sys.argv[1]
    min_us = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 20.0
    ev = json.load(open(path))
    ev = ev.get("traceEvents", ev)
    xs = [e for e in ev if e.get("ph") == "X" and "dur" in e]
    gpu = sorted((e for e in xs if e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset")),
                 key=lambda e: e["ts"])
    rt = sorted((e for e in xs if e.get("cat") in ("cuda_runtime", "cuda_driver")),
                key=lambda e: e["ts"])
    rows = []
    for e in rt:
        if e["dur"] >= min_us:
            rows.append((e["ts"], "host", e["name"], e["dur"]))
    for a, b in zip(gpu, gpu[1:]):
        gap = b["ts"] - (a["ts"] + a["dur"])
        if gap >= min_us:
            rows.append((a["ts"] + a["dur"], "GPU idle", f"{a['name'][:40]} -> {b['name'][:40]}", gap))
    for e in gpu:
        if e.get("cat") != "kernel":
            rows.append((e["ts"], "GPU " + e["cat"], e["name"][:60], e["dur"]))
    rows.sort()
    t0 = rows[0][0] if rows else 0
    for ts, kind, name, dur in rows:
        print(f"{(ts - t0) / 1e3:10.3f} ms  {kind:14} {dur:9.1f} us  {name}")
    tot = {}
    for e in rt:
        tot[e["name"]] = tot.get(e["name"], 0.0) + e["dur"]
    print("\nhost runtime totals (us):")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:12]:
        print(f"   {v:10.1f}  {k}")


if __name__ == "__main__":
    main()
