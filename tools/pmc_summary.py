#!/usr/bin/env python3
"""Summarise tools/gpu_pmc.sh output: per-counter average over the trace
kernel's dispatches, HBM traffic per launch (MI355X_MICROARCH.md: FETCH_SIZE
reads 1/2 of a wide coalesced stream on gfx950, so it is doubled; WRITE_SIZE
as is; both in KiB), and optionally a JSON record for bench.py.

  python tools/pmc_summary.py gpurun_out/pmc_TAG [--json profiles/pmc_c3.json]
"""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = ["raytracer-gamma_amd/csrc/rtg_trace.h", "raytracer-gamma_amd/csrc/rtg_trace_kernels.h"]


def source_md5():
    h = hashlib.md5()
    for f in SRC:
        h.update(open(os.path.join(ROOT, f), "rb").read())
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="rtg::trace_", help="kernel-name substring")
    ap.add_argument("--json", default=None)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--variant", type=int, default=0)
    a = ap.parse_args()
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(a.dir, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if a.kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in agg.items()}
    for k in sorted(avg):
        print(f"{k:28s} {avg[k]:.6g}  (n={len(agg[k])})")
    out = {"config": a.config, "variant": a.variant, "kernel": a.kernel,
           "source_md5": source_md5(), "counters": avg}
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        u = avg["SQ_THREAD_CYCLES_VALU"] / (avg["SQ_ACTIVE_INST_VALU"] * 64)
        out["valu_lane_utilisation"] = u
        print("VALU lane utilisation       %.3f" % u)
    if "SQ_INSTS_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
        # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles; 1024 SIMDs issue one
        # wave64 VALU instruction per 2 cycles (MI355X_MICROARCH.md)
        cyc = avg["GRBM_GUI_ACTIVE"] / 8
        out["valu_issue_utilisation"] = avg["SQ_INSTS_VALU"] / (1024 * cyc / 2)
        out["busy_ms_at_2p4GHz"] = cyc / 2.4e6
        print("VALU issue utilisation      %.3f  (%.3g wave instructions / %.3g slots)" % (
            out["valu_issue_utilisation"], avg["SQ_INSTS_VALU"], 1024 * cyc / 2))
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        rd = avg["FETCH_SIZE"] * 2 * 1024
        wr = avg["WRITE_SIZE"] * 1024
        out["hbm_read_bytes"] = rd
        out["hbm_write_bytes"] = wr
        out["traffic_bytes"] = rd + wr
        print("HBM read  (FETCH_SIZE x2, gfx950 correction) %.1f MB" % (rd / 1e6))
        print("HBM write (WRITE_SIZE)                       %.1f MB" % (wr / 1e6))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
        print("wrote", a.json)


if __name__ == "__main__":
    main()
