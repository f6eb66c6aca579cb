#!/usr/bin/env python3
"""One line per run of a tools/c5_ab.sh jsonl: variant, wall, payload GiB/s,
stage times, verdict and accept latencies (ms)."""
import json
import sys

for line in open(sys.argv[1]):
    d = json.loads(line)
    r = d["run"]
    v, a, le, se = r["verify_latency_us"], r["accept_latency_us"], r["leecher"], r["seeder"]
    print(f'{d["variant"]:5s} {d["round"]} {r["seconds"]:6.3f} s {r["payload_gibs"]:5.2f} GiB/s  '
          f'seeder v/e {se["verify_s"]:5.2f}/{se["encode_s"]:4.2f}  leecher v/w {le["verify_s"]:5.2f}/{le["write_s"]:4.2f} '
          f'batch {le["mean_batch"]:5.1f}  verdict p50/p90/p99/max {v["p50"]/1e3:5.1f}/{v["p90"]/1e3:5.1f}/'
          f'{v["p99"]/1e3:5.1f}/{v["max"]/1e3:5.1f}  accept p50/p99 {a["p50"]/1e3:5.1f}/{a["p99"]/1e3:5.1f}  '
          f'ok={r["files_identical"]} rej={le["rejected"]}')
