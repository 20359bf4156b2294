#!/usr/bin/env python3
"""tools/timed_stats.py — the rocprofv3 kernel trace of a bench.py run,
restricted to the bench's TIMED launches.

`rocprofv3 --kernel-trace --stats` summarises every dispatch of the process:
the first launch after set_scene (no launch-order feedback), the warm-up
launches, the counting build and the end-to-end launches after the timed
region.  bench.py reports which trace-kernel dispatches were timed
(`timed_launches`: [first, first + count) in dispatch order); this picks
those, the cull pass of each (the cull_groups_kernel dispatch just before it),
and writes a --stats-style CSV plus a JSON summary:

  * avg / min / max duration of the trace kernel and of the cull pass;
  * the frame span = first timed cull start -> last timed trace end, / count
    (kernels + gaps), which must agree with the bench line's ms_per_step.

  python tools/timed_stats.py TRACE_DIR BENCH_JSON OUT_PREFIX
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys


def main():
    trace_dir, bench_json, prefix = sys.argv[1:4]
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    assert files, f"no kernel_trace.csv under {trace_dir}"
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    line = [x for x in open(bench_json).read().splitlines() if x.startswith("{")][-1]
    bench = json.loads(line)
    tl = bench["timed_launches"]
    first, count = int(tl["first"]), int(tl["count"])

    def is_trace(name):
        return "trace_samples_kernel" in name or "trace_kernel<" in name

    # launches in dispatch order: each is [cull dispatch (compacted launches), trace dispatch]
    launches, pending_cull = [], None
    for r in rows:
        nm = r["Kernel_Name"]
        if "cull_groups_kernel" in nm:
            pending_cull = r
        elif is_trace(nm):
            launches.append((pending_cull, r))
            pending_cull = None
    timed = launches[first:first + count]
    assert len(timed) == count, (len(launches), first, count)
    name = timed[0][1]["Kernel_Name"]
    assert all(t[1]["Kernel_Name"] == name for t in timed), "timed launches changed kernel"

    def dur(r):
        return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])

    def stats(ds):
        ds = sorted(ds)
        return {"calls": len(ds), "avg_ns": sum(ds) / len(ds), "min_ns": ds[0], "max_ns": ds[-1],
                "total_ns": sum(ds)}

    tr = stats([dur(t[1]) for t in timed])
    culls = [t[0] for t in timed if t[0] is not None]
    cu = stats([dur(c) for c in culls]) if culls else None
    gaps = [int(t[1]["Start_Timestamp"]) - int(t[0]["End_Timestamp"]) for t in timed
            if t[0] is not None]
    start = int((timed[0][0] or timed[0][1])["Start_Timestamp"])
    end = int(timed[-1][1]["End_Timestamp"])
    span_ms = (end - start) / count / 1e6
    out = {"bench": os.path.basename(bench_json), "config": bench["config"]["workload"],
           "timed_launches": [first, count], "trace_kernel": name, "trace": tr, "cull": cu,
           "frame_span_ms": round(span_ms, 4),
           "cull_end_to_trace_start_us": round(sum(gaps) / len(gaps) / 1e3, 2) if gaps else None,
           "kernels_ms": round((tr["avg_ns"] + (cu["avg_ns"] if cu else 0)) / 1e6, 4),
           "bench_ms_per_step": bench["ms_per_step"], "bench_kernel_ms": bench["kernel_ms"],
           "first_launch_ms_bench": bench.get("first_launch_ms"),
           "all_dispatches_of_trace_kernel": sum(1 for l in launches if l[1]["Kernel_Name"] == name)}
    with open(prefix + ".json", "w") as f:
        json.dump(out, f, indent=1)
    with open(prefix + ".csv", "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
        w.writerow([name, tr["calls"], tr["total_ns"], tr["avg_ns"], tr["min_ns"], tr["max_ns"]])
        if cu:
            w.writerow([culls[0]["Kernel_Name"], cu["calls"], cu["total_ns"], cu["avg_ns"],
                        cu["min_ns"], cu["max_ns"]])
    print(json.dumps({k: v for k, v in out.items() if k not in ("trace", "cull")}))
    print(f"trace avg {tr['avg_ns'] / 1e6:.4f} ms, cull avg "
          f"{(cu['avg_ns'] / 1e6 if cu else 0):.4f} ms, span/launch {span_ms:.4f} ms, "
          f"bench ms_per_step {bench['ms_per_step']}")


if __name__ == "__main__":
    main()
