#!/usr/bin/env python3
"""Summarise a tools/prof/profile.sh run into profiles/ (committed evidence).

usage: summarize.py gpurun_out/prof_TAG_WL  profiles/  TAG  WL  [KERNEL-SUBSTRING]
Writes  profiles/TAG_WL_kernel_stats.csv   (rocprofv3 --stats, verbatim)
        profiles/TAG_WL_summary.json       (per-launch averages of every counter)
        profiles/traffic_WL.json           (HBM bytes per launch, calibrated; read by bench.py)
"""
import csv
import collections
import json
import os
import shutil
import sys

KERNEL = "crc32_rows_kernel"
CAL_BYTES = 2 << 30


def per_dispatch(path, match):
    rows = list(csv.DictReader(open(path)))
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        if match in r["Kernel_Name"]:
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    src, dst, tag, wl = sys.argv[1:5]
    global KERNEL
    if len(sys.argv) > 5:
        KERNEL = sys.argv[5]
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_{wl}_kernel_stats.csv"))
    kern = [r for r in csv.DictReader(open(stats)) if KERNEL in r["Name"]]
    summary = {"workload": wl, "kernel": kern[0]["Name"] if kern else None,
               "avg_ns": float(kern[0]["AverageNs"]) if kern else None,
               "calls": int(kern[0]["Calls"]) if kern else None, "counters": {}}
    # avg_ns covers every traced dispatch, the 0.5 s prewarm at ramping clocks
    # included; the bench's timed steps are the last `steps` dispatches
    tr = os.path.join(src, "trace", "trace_kernel_trace.csv")
    if os.path.exists(tr):
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(tr))
             if KERNEL in r["Kernel_Name"]]
        steps = 20
        try:
            for line in open(os.path.join(src, "bench_trace.log")):
                if line.startswith("{"):
                    js = json.loads(line)
                    steps = int(js.get("steps", steps))
                    summary["lnx_version"] = js.get("config", {}).get("kernel")
                    summary["build_id"] = js.get("config", {}).get("build_id")
        except (OSError, ValueError):
            pass
        if d:
            last = d[-steps:]
            summary["timed_steps_avg_ns"] = sum(last) / len(last)
            summary["timed_steps"] = len(last)
            summary["median_ns"] = sorted(d)[len(d) // 2]
    for i in range(1, 10):
        p = os.path.join(src, f"pmc{i}", "pmc_counter_collection.csv")
        if os.path.exists(p):
            avg, n = per_dispatch(p, KERNEL)
            summary["counters"].update(avg)
    cal, _ = per_dispatch(os.path.join(src, "calib", "calib_counter_collection.csv"), "rd<unsigned int>")
    cal4, _ = per_dispatch(os.path.join(src, "calib", "calib_counter_collection.csv"), "rd<HIP_vector_type")
    # FETCH_SIZE is in KiB; bytes actually fetched per KiB-unit for this access width:
    f_dw = CAL_BYTES / (cal["FETCH_SIZE"] * 1024) if cal else None
    f_x4 = CAL_BYTES / (cal4["FETCH_SIZE"] * 1024) if cal4 else None
    summary["calibration"] = {"bytes_per_fetch_size_byte_dword_loads": f_dw,
                              "bytes_per_fetch_size_byte_dwordx4_loads": f_x4,
                              "calib_bytes": CAL_BYTES}
    fs = summary["counters"].get("FETCH_SIZE")
    if fs and f_dw:
        hbm = fs * 1024 * f_dw
        summary["hbm_bytes_per_launch"] = hbm
        with open(os.path.join(dst, f"traffic_{wl}.json"), "w") as fh:
            json.dump({"hbm_bytes_per_launch": round(hbm), "fetch_size_kib": fs,
                       "calibration_factor": f_dw, "source": f"{tag}_{wl}_summary.json",
                       "method": "rocprofv3 --pmc FETCH_SIZE, own pass; x factor measured on tools/prof/calib "
                                 "(dword-per-lane reads of 2 GiB) in the same profiling run"}, fh, indent=1)
    c = summary["counters"]
    # the clock: GRBM_GUI_ACTIVE (cycles, summed over the 8 XCDs) over the SAME
    # dispatch's duration from the kernel trace of that pass (profile.sh traces
    # the GRBM pass); dividing by the other pass's durations mixed an un-warmed
    # PMC run with a warmed trace and read low (round 4's "1.9 GHz", profiles/r5l)
    clk = []
    for i in range(1, 10):
        cp = os.path.join(src, f"pmc{i}", "pmc_counter_collection.csv")
        kp = os.path.join(src, f"pmc{i}", "pmc_kernel_trace.csv")
        if not (os.path.exists(cp) and os.path.exists(kp)):
            continue
        dur = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
               for r in csv.DictReader(open(kp)) if KERNEL in r["Kernel_Name"]}
        grbm = collections.defaultdict(float)
        for r in csv.DictReader(open(cp)):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                grbm[r["Dispatch_Id"]] += float(r["Counter_Value"])
        ds = sorted((d for d in grbm if dur.get(d)), key=int)[-10:]  # the last, warmed dispatches
        clk += [grbm[d] / 8 / dur[d] for d in ds]
    if clk:
        summary["clock_ghz"] = sorted(clk)[len(clk) // 2]
        summary["clock_method"] = "median over dispatches of GRBM_GUI_ACTIVE / 8 XCDs / the dispatch's traced duration"
    summary["clock_ghz_est"] = summary.get("clock_ghz")
    keys = ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT")
    if all(k in c for k in keys):  # read by bench.py (roofline_compute): tied to the build that made them
        with open(os.path.join(dst, f"counters_{wl}.json"), "w") as fh:
            json.dump({**{k: c[k] for k in keys}, "build_id": summary.get("build_id"),
                       "clock_ghz_est": summary.get("clock_ghz_est"), "source": f"{tag}_{wl}_summary.json",
                       "method": "rocprofv3 --pmc, one counter group per pass (tools/prof/profile.sh), per-launch "
                                 "averages over the traced dispatches; SQ_* summed over all CUs"}, fh, indent=1)
    with open(os.path.join(dst, f"{tag}_{wl}_summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
