#!/usr/bin/env python3
"""C3 end to end from files (diagnostic, GPU box): where does EncodeFile's time go?

Writes the 64 x 1 GiB files of tests/golden/c3.json (GPU-generated stream,
file f = seed f) to a directory (default /dev/shm), then times:
  * cli:      lbf_encoder --time over all 64 files in a fresh process (what
              test_c3_encode_file_cli_64_files measures), `--cli-runs` times;
  * inproc:   ChunkHasher.hash_files over the same files in this process, the
              first pass on a fresh context and then the best of 3;
  * pread:    the files read into one pageable buffer with `--threads` threads
              (no GPU), the host side alone.
Every digest set is checked against c3.json.  Prints one JSON line per phase.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime, loaded first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bitflood_amd import ChunkHasher, DeviceBuffer, chunk_table  # noqa: E402
from bitflood_amd import hashing as H  # noqa: E402

GIB = 1 << 30
ap = argparse.ArgumentParser()
ap.add_argument("--dir", default="/dev/shm")
ap.add_argument("--files", type=int, default=64, help="first N files of c3.json")
ap.add_argument("--cli-runs", type=int, default=2)
ap.add_argument("--threads", type=int, default=8)
ap.add_argument("--skip", default="", help="comma list of phases to skip: cli,inproc,pread")
ap.add_argument("--order", default="cli,inproc,pread", help="the phases in the order they run")
a = ap.parse_args()
skip = set(filter(None, a.skip.split(",")))

c3 = json.load(open(os.path.join(ROOT, "tests", "golden", "c3.json")))
fs, cs = c3["file_size"], c3["chunk_size"]
files = c3["files"][: a.files]


def emit(d):
    print(json.dumps(d), flush=True)


import shutil  # noqa: E402
if shutil.disk_usage(a.dir).free < len(files) * fs + 16 * GIB:
    raise SystemExit(f"{a.dir}: not enough free space for {len(files)} x {fs >> 30} GiB")
d = tempfile.mkdtemp(prefix="lbf_c3probe_", dir=a.dir)
try:
    t0 = time.perf_counter()
    buf = DeviceBuffer(fs)
    names = []
    try:
        for k, f in enumerate(files):
            buf.fill_synthetic(f["seed"], start=0)
            H.synchronize()
            name = os.path.join(d, f"f{f['seed']:02d}.bin")
            buf.download(fs).tofile(name)
            names.append(name)
            if k % 8 == 7:
                emit({"phase": "write", "files": k + 1, "s": round(time.perf_counter() - t0, 2)})
    finally:
        buf.free()
    total = len(names) * fs

    def check(dig, what):
        dig = dig.reshape(-1, 20)
        per = fs // cs
        ok = all(hashlib.sha1(dig[k * per:(k + 1) * per].tobytes()).hexdigest() == f["sha1_of_concat_raw_digests_hex"]
                 for k, f in enumerate(files))
        if not ok:
            raise SystemExit(f"{what}: digests differ from c3.json")
        return ok

    def phase_cli():
        lib = os.path.join(ROOT, "bitflood_amd", "lib")
        for r in range(a.cli_runs):
            out = subprocess.run([os.path.join(lib, "lbf_encoder"), *[os.path.basename(n) for n in names],
                                  "http://127.0.0.1:10101/", "c3.flood", "--time"], cwd=d, capture_output=True,
                                 text=True, timeout=600)
            if out.returncode:
                raise SystemExit(out.stderr)
            t = json.loads(out.stdout.strip().splitlines()[-1])
            emit({"phase": "cli", "run": r, **t, "gibs": round(t["bytes"] / GIB / t["encode_s"], 2)})

    o, s = chunk_table(fs, cs)
    file_of = np.repeat(np.arange(len(names), dtype=np.uint32), o.size)
    offs, sizes = np.tile(o, len(names)), np.tile(s, len(names))

    def phase_inproc():
        t = time.perf_counter()
        with ChunkHasher(device_mask=1) as h:
            t_ctx = time.perf_counter() - t
            t = time.perf_counter()
            first = h.hash_files(names, file_of, offs, sizes)
            t_first = time.perf_counter() - t
            check(first, "inproc first")
            best = 1e9
            for _ in range(3):
                t = time.perf_counter()
                dig = h.hash_files(names, file_of, offs, sizes)
                best = min(best, time.perf_counter() - t)
            check(dig, "inproc")
            st = h.staging_stats()
            place = h.worker_info(0)
        emit({"phase": "inproc", "ctx_create_s": round(t_ctx, 4), "first_s": round(t_first, 3),
              "first_gibs": round(total / GIB / t_first, 2), "best_s": round(best, 3),
              "best_gibs": round(total / GIB / best, 2), "staging": st, "placement": place})

    def phase_pread():
        dst = np.empty(fs * min(8, len(names)), dtype=np.uint8)  # 8 GiB window, reused

        def reader(k0, step):
            for k in range(k0, len(names), step):
                fd = os.open(names[k], os.O_RDONLY)
                try:
                    mv = memoryview(dst)[(k % 8) * fs:(k % 8 + 1) * fs]
                    got = 0
                    while got < fs:
                        n = os.preadv(fd, [mv[got:]], got)
                        if n <= 0:
                            break
                        got += n
                finally:
                    os.close(fd)

        dst[:] = 0  # first touch before timing
        for rep in range(2):
            t = time.perf_counter()
            th = [threading.Thread(target=reader, args=(k, a.threads)) for k in range(a.threads)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            dt = time.perf_counter() - t
            emit({"phase": "pread", "rep": rep, "threads": a.threads, "gibs": round(total / GIB / dt, 2)})

    phases = {"cli": phase_cli, "inproc": phase_inproc, "pread": phase_pread}
    for name in a.order.split(","):
        if name not in skip:
            phases[name]()
finally:
    subprocess.run(["rm", "-rf", d])
