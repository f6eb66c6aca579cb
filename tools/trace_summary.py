"""Summarise a rocprofv3 --hip-trace --kernel-trace --memory-copy-trace
database (diagnostic, GPU box): host-side duration of the HIP calls the
staging pipeline makes, and a timeline of the last N events (API calls on the
staging thread, copies, kernels), so the database itself need not travel.

  python tools/trace_summary.py <results.db> [N]
"""
import sqlite3
import sys

db, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 80
c = sqlite3.connect(db)
calls = ("hipMemcpyAsync", "hipLaunchKernel", "hipStreamSynchronize", "hipEventSynchronize", "hipEventRecord",
         "hipModuleLaunchKernel", "hipExtModuleLaunchKernel")
print("# host-side duration of staging HIP calls (us): name count avg max")
for r in c.execute("select name, count(*), avg(duration)/1e3, max(duration)/1e3 from regions group by name"):
    if r[0] in calls:
        print("%-24s %7d %10.1f %10.1f" % r)
ev = []
for r in c.execute("select start, end, tid, name from regions"):
    if r[3] in calls:
        ev.append((r[0], r[1], "api t%d %s" % (r[2] % 100000, r[3])))
for r in c.execute("select start, end, stream_id, size, name from memory_copies"):
    ev.append((r[0], r[1], "copy s%s %s %.1f MiB" % (r[2], r[4][12:], r[3] / 2**20)))
for r in c.execute("select start, end, stream_id, name from kernels"):
    ev.append((r[0], r[1], "kernel s%s %s" % (r[2], r[3].split("(")[0][-40:])))
ev.sort()
t0 = ev[-n][0]
print("# last %d events: start_ms end_ms dur_ms what" % n)
for s, e, what in ev[-n:]:
    print("%9.3f %9.3f %8.3f %s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, what))
