#!/usr/bin/env python3
"""Summarise a tools/b64_profile.sh run (gpurun_out/prof/<tag>/: a kernel trace
and the PMC passes over tools/b64_rate.py, 1,024 x 256 KiB per launch) into the
JSON of profiles/r05/b64/b64_r05*.json: per wire kernel the trace's dispatch
times, the mean of every counter per dispatch, instructions per wave, the split
of wave cycles, HBM bytes (FETCH_SIZE x 2, the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md; WRITE_SIZE as is; both in KiB), and the
fraction of the 8 TB/s peak the algorithmic bytes reach.

    python tools/b64_summary.py gpurun_out/prof/<tag> <out.json> [--what TEXT]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

CHUNKS, CHUNK = 1024, 262144
PEAK_TBS = 8.0
CUS = 256


def put_length(size):
    return 4 * (size // 3) + (4 if size % 3 else 0) + size // 3 // 18


# every wire kernel moves the chunk bytes one way and their text the other
ALGORITHMIC = CHUNKS * (CHUNK + put_length(CHUNK))


def short(name):
    m = re.search(r"b64_\w+", name)
    return m.group(0) if m else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--what", default="")
    a = ap.parse_args()
    out = {"what": a.what,
           "driver": "tools/b64_profile.sh over tools/b64_rate.py: 1,024 x 256 KiB chunks per launch, "
                     "FETCH_SIZE x2 (gfx950 correction)",
           "kernels": {}}
    for r in csv.DictReader(open(os.path.join(a.src, "trace", "trace_kernel_stats.csv"))):
        k = short(r["Name"])
        if k:
            out["kernels"].setdefault(k, {})["trace"] = {
                "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                "max_ns": float(r["MaxNs"])}
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(a.src, "pmc_*", "pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                key = (f, r["Dispatch_Id"])
                per[k][r["Counter_Name"]][key] = per[k][r["Counter_Name"]].get(key, 0.0) + float(r["Counter_Value"])
    for k, counters in per.items():
        c = {n: sum(v.values()) / len(v) for n, v in counters.items()}
        e = out["kernels"].setdefault(k, {})
        e["counters"] = c
        waves = c.get("SQ_WAVES")
        if waves:
            e["per_wave"] = {n: c[s] / waves for n, s in (("VALU", "SQ_INSTS_VALU"), ("SALU", "SQ_INSTS_SALU"),
                                                          ("LDS", "SQ_INSTS_LDS"), ("VMEM_RD", "SQ_INSTS_VMEM_RD"),
                                                          ("VMEM_WR", "SQ_INSTS_VMEM_WR")) if s in c}
        if c.get("SQ_WAVE_CYCLES"):
            e["wave_cycle_split"] = {n: c[s] / c["SQ_WAVE_CYCLES"] for n, s in (
                ("active_inst_any", "SQ_ACTIVE_INST_ANY"), ("wait_any", "SQ_WAIT_ANY"),
                ("wait_inst_any", "SQ_WAIT_INST_ANY")) if s in c}
        if "FETCH_SIZE" in c:
            e["hbm_read_bytes"] = 2 * 1024 * c["FETCH_SIZE"]
        if "WRITE_SIZE" in c:
            e["hbm_write_bytes"] = 1024 * c["WRITE_SIZE"]
        if c.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs, the _sum counters over the 256 CUs
            g = c["GRBM_GUI_ACTIVE"] / 8 * CUS
            e["busy_fraction_per_cu"] = {n: c[s] / g for n, s in (
                ("TA", "TA_TA_BUSY_sum"), ("TD", "TD_TD_BUSY_sum"),
                ("TCP_pending_stall", "TCP_PENDING_STALL_CYCLES_sum")) if s in c}
        if c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_over_active"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
    for k, e in out["kernels"].items():
        if "trace" in e and k != "b64_decode_kernel":
            e["algorithmic_bytes"] = ALGORITHMIC
            e["achieved_tbs"] = ALGORITHMIC / e["trace"]["avg_ns"] / 1e3
            e["hbm_frac"] = e["achieved_tbs"] / PEAK_TBS
            if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
                e["traffic_over_algorithmic"] = (e["hbm_read_bytes"] + e["hbm_write_bytes"]) / ALGORITHMIC
    json.dump(out, open(a.dst, "w"), indent=1)
    for k, e in out["kernels"].items():
        print(k, {x: round(e[x], 4) for x in ("hbm_frac", "traffic_over_algorithmic") if x in e},
              e.get("trace", {}).get("avg_ns"))


if __name__ == "__main__":
    main()
