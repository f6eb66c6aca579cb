#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/.

HBM traffic per launch of the chunk-hash kernel, corrected as
/opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes for gfx950:
  FETCH_SIZE (KiB) reports exactly half the bytes of a wide coalesced stream
  -> read bytes = 2 * FETCH_SIZE * 1024;  WRITE_SIZE (KiB) is exact for 16-B
  stores (uncalibrated for the 4-B digest stores, which are < 0.01 % here).
Also derives the effective clock from GRBM_GUI_ACTIVE (sum over 8 XCDs) and
the wave-cycle split (active / waiting on memory / issue-stalled).

Usage: tools/pmc_traffic.py gpurun_out/prof/<tag> profiles/<round>/<tag> [--file-bytes N]
Writes <dst>/summary.json, copies the kernel-stats CSV, and (with
--record) updates profiles/pmc_traffic.json read by bench.py.  Each record
carries the machine-code digest of the profiled kernel (code_sha256, from the
same lease's bench line); bench.py cites the traffic only while the library it
loads carries that same code.
"""
import argparse
import collections
import csv
import json
import os
import shutil


def per_kernel(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return agg, durs


def mean(x):
    return sum(x) / len(x) if x else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--file-bytes", type=int, default=4 << 30)
    ap.add_argument("--chunk-size", type=int, default=262144)
    ap.add_argument("--kernel", default=None,
                    help="kernel name substring; default: the kernel the traced bench line names (config.kernel)")
    ap.add_argument("--record", action="store_true")
    a = ap.parse_args()
    if a.kernel is None:
        a.kernel = "sha1_"
        try:  # the bench's own line in the traced run names its device-resident kernel
            for line in open(os.path.join(a.src, "trace.log")):
                if line.startswith("{"):
                    a.kernel = json.loads(line)["config"]["kernel"]
        except (OSError, ValueError, KeyError):
            pass
    os.makedirs(a.dst, exist_ok=True)
    out = {"file_bytes": a.file_bytes}

    # the plain bench line of the same session (tools/profile_round.sh step 0):
    # the evidence chain closes within one lease
    try:
        line = json.loads([x for x in open(os.path.join(a.src, "bench.json")) if x.startswith("{")][-1])
        out["bench_same_session"] = {"value": line["value"], "ms_per_step": line["ms_per_step"],
                                     "kernel_ms": line["roofline"]["kernel_ms"], "frac": line["roofline"]["frac"],
                                     "kernel": line["config"]["kernel"]}
        # the machine code of the kernel the lease ran (bench.py reads it out of the loaded library)
        if line["roofline"].get("kernel_code_sha256"):
            out["code_sha256"] = line["roofline"]["kernel_code_sha256"]
            out["code_symbol"] = line["roofline"].get("kernel_symbol")
    except (OSError, ValueError, KeyError, IndexError):
        pass
    # the bench line the traced run printed (its HIP events include the tracer's overhead)
    try:
        line = json.loads([x for x in open(os.path.join(a.src, "trace.log")) if x.startswith("{")][-1])
        out["bench_traced_run"] = {"value": line["value"], "ms_per_step": line["ms_per_step"],
                                   "kernel_ms": line["roofline"]["kernel_ms"], "steps": line["steps"],
                                   "warmup": line["warmup"]}
    except (OSError, ValueError, KeyError, IndexError):
        pass
    stats = os.path.join(a.src, "trace", "trace_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(a.dst, "kernel_stats.csv"))
        rows = [r for r in csv.DictReader(open(stats)) if a.kernel in r["Name"]]
        # the bench's device-resident launches are the uniform-mode kernels
        # (`<true, ...>`); the host legs' batches (`<false, ...>`) can total more
        # time since round 3's e2e passes, so prefer uniform mode, then total time
        rows.sort(key=lambda r: "<true" not in r["Name"])
        for r in rows:
            if "kernel" not in out:
                out["kernel"] = r["Name"]
                out["trace_avg_ns"] = float(r["AverageNs"])
                out["trace_calls"] = int(r["Calls"])

    # per-dispatch durations of the traced run: min / median beside the average
    # (the average carries the warm-up launches and the tracer's own overhead)
    trace = os.path.join(a.src, "trace", "trace_kernel_trace.csv")
    if os.path.exists(trace) and "kernel" in out:
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(trace))
             if r.get("Kernel_Name") == out["kernel"]]  # in dispatch order
        # the timed steps are the traced bench's last `steps` dispatches of this kernel
        steps = out.get("bench_traced_run", {}).get("steps", 0)
        timed = sorted(d[-steps:]) if steps and len(d) >= steps else []
        d = sorted(d)
        if timed:
            out["trace_timed_dispatches"] = len(timed)
            out["trace_timed_median_ns"] = (timed[len(timed) // 2] if len(timed) % 2 else
                                            (timed[len(timed) // 2 - 1] + timed[len(timed) // 2]) / 2)
            out["trace_timed_mean_ns"] = sum(timed) / len(timed)
        if d:
            out["trace_dispatches"] = len(d)
            out["trace_min_ns"] = d[0]
            out["trace_median_ns"] = d[len(d) // 2] if len(d) % 2 else (d[len(d) // 2 - 1] + d[len(d) // 2]) / 2
            out["trace_max_ns"] = d[-1]
    for key in ("bench_same_session", "bench_traced_run"):
        if key in out and "trace_median_ns" in out:
            out[f"trace_median_over_{key}_ms_per_step"] = out["trace_median_ns"] / 1e6 / out[key]["ms_per_step"]

    def pick(sub):
        p = os.path.join(a.src, sub, "pmc_counter_collection.csv")
        if not os.path.exists(p):
            return {}, {}
        agg, durs = per_kernel(p)
        for k in sorted(agg, key=lambda k: "<true" not in k):
            if a.kernel in k:
                return agg[k], durs[k]
        return {}, {}

    fetch, _ = pick("pmc_fetch")
    write, _ = pick("pmc_write")
    sq, sq_durs = pick("pmc_sq")
    if fetch:
        rd = 2 * mean(fetch["FETCH_SIZE"]) * 1024
        out["fetch_size_kib"] = mean(fetch["FETCH_SIZE"])
        out["read_bytes_per_launch"] = rd
    if write:
        out["write_size_kib"] = mean(write["WRITE_SIZE"])
        out["write_bytes_per_launch"] = mean(write["WRITE_SIZE"]) * 1024
    if fetch and write:
        out["hbm_bytes_per_launch"] = out["read_bytes_per_launch"] + out["write_bytes_per_launch"]
        out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / a.file_bytes
    if sq:
        wc = mean(sq["SQ_WAVE_CYCLES"])
        out["sq"] = {k: mean(v) for k, v in sq.items()}
        out["wave_cycle_split"] = {
            "active_inst_any": mean(sq["SQ_ACTIVE_INST_ANY"]) / wc,
            "wait_any(memory/barrier)": mean(sq["SQ_WAIT_ANY"]) / wc,
            "wait_inst_any(issue)": mean(sq["SQ_WAIT_INST_ANY"]) / wc,
        }
        if sq_durs:
            out["effective_clock_ghz"] = mean(sq["GRBM_GUI_ACTIVE"]) / 8 / mean(sq_durs)
    with open(os.path.join(a.dst, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
    if a.record and "hbm_bytes_per_launch" in out:
        # one entry per (file size, chunk size, kernel): bench.py looks its workload up here
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        path = os.path.join(root, "profiles", "pmc_traffic.json")
        rec = {"file_bytes": a.file_bytes, "chunk_size": a.chunk_size,
               "hbm_bytes_per_launch": out["hbm_bytes_per_launch"],
               "source": os.path.relpath(os.path.join(a.dst, "summary.json"), root),
               "kernel": out.get("kernel")}
        for k in ("code_sha256", "code_symbol", "trace_median_ns", "trace_timed_median_ns", "bench_same_session",
                  "bench_traced_run"):
            if k in out:
                rec[k] = out[k]
        try:
            old = json.load(open(path))
            entries = old.get("entries", [old])
        except (OSError, ValueError):
            entries = []
        entries = [e for e in entries if not (e.get("file_bytes") == a.file_bytes
                                              and e.get("chunk_size", 262144) == a.chunk_size
                                              and e.get("kernel") == rec["kernel"])]
        with open(path, "w") as f:
            json.dump({"entries": entries + [rec]}, f, indent=1)


if __name__ == "__main__":
    main()
