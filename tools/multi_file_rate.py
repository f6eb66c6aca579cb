#!/usr/bin/env python3
"""Many files, one batch vs one call per file (diagnostic, GPU box).

Writes N files of S bytes (page-cache warm), then times their resume verify /
hash at 256 KiB chunks two ways: one lbf_file_ranges call per file (what a
per-file loop costs: each call pays at least one serial SHA-1 chain, ≈3 ms at
256 KiB) and one lbf_files_ranges batch over all of them.  Checks that both give
the same digests.  Usage: python tools/multi_file_rate.py [--files 512] [--mib 8]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime, loaded first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bitflood_amd import ChunkHasher, chunk_table  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--files", type=int, default=512)
ap.add_argument("--mib", type=float, default=8)
ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"), help="where the files go (/dev/shm: tmpfs)")
ap.add_argument("--batch-only", action="store_true", help="skip the per-file loop")
ap.add_argument("--warm-other", action="store_true", help="hash an unrelated 64 MiB file first (context warm-up)")
a = ap.parse_args()
CS = 262144
size = int(a.mib * (1 << 20))
rng = np.random.default_rng(9)
with tempfile.TemporaryDirectory(dir=a.dir) as d:
    paths = []
    for f in range(a.files):
        p = os.path.join(d, f"f{f:05d}.bin")
        rng.integers(0, 256, size, dtype=np.uint8).tofile(p)
        paths.append(p)
    o, s = chunk_table(size, CS)
    file_of = np.repeat(np.arange(a.files, dtype=np.uint32), o.size)
    offs, sizes = np.tile(o, a.files), np.tile(s, a.files)
    out = {"files": a.files, "bytes_per_file": size, "chunk_size": CS}
    with ChunkHasher(device_mask=1) as h:
        if a.warm_other:  # a pass over other files first: staging allocated, these files untouched by it
            other = os.path.join(d, "other.bin")
            rng.integers(0, 256, 64 << 20, dtype=np.uint8).tofile(other)
            oo, os_ = chunk_table(64 << 20, CS)
            h.hash_files([other], np.zeros(oo.size, np.uint32), oo, os_)
        t = time.perf_counter()
        first = h.hash_files(paths, file_of, offs, sizes)  # first pass over these files
        out["first_batch_gibs"] = round(a.files * size / 2**30 / (time.perf_counter() - t), 2)
        out["warm_other"] = a.warm_other
        best_loop = best_batch = 1e9
        for _ in range(3):
            if not a.batch_only:
                t = time.perf_counter()
                per = [h.hash_file(p, o, s) for p in paths]
                best_loop = min(best_loop, time.perf_counter() - t)
                assert np.array_equal(np.concatenate(per), first)
            t = time.perf_counter()
            batch = h.hash_files(paths, file_of, offs, sizes)
            best_batch = min(best_batch, time.perf_counter() - t)
        assert np.array_equal(first, batch)
    total = a.files * size / 2**30
    out["dir"] = a.dir
    out["one_batch_gibs"] = round(total / best_batch, 2)
    if not a.batch_only:
        out["per_file_calls_gibs"] = round(total / best_loop, 2)
        out["speedup"] = round(best_loop / best_batch, 2)
    print(json.dumps(out))
