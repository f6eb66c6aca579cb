#!/usr/bin/env python3
"""Single-call latency through the C ABI (diagnostic, GPU box): one 64 KiB and
one 256 KiB chunk (lbf_sha1_one, the Base64Encode path), and 100 x 256 KiB in
one batch (a wave with 36 idle lanes); ragged batches: 256 chunks of 64-256 KiB
(pc4) and 20,000 chunks of 16-64 KiB (pcx5).  Median of `reps` after warm-up.
Usage: [LBF_LIB=...] python tools/latency_ab.py [reps]"""
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bitflood_amd import ChunkHasher, chunk_table  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
data = np.random.default_rng(5).integers(0, 256, 256 * 262144, dtype=np.uint8)
offs, sizes = chunk_table(data.size, 262144)
rng = np.random.default_rng(9)
r_sizes = rng.integers(65536, 262145, 256).astype(np.uint32)
r_offs = (np.cumsum(r_sizes, dtype=np.uint64) - r_sizes).astype(np.uint64)
x_sizes = rng.integers(16384, 65537, 20000).astype(np.uint32)
x_offs = (rng.integers(0, data.size - 65536, 20000) & ~15).astype(np.uint64)
out = {"lib": os.path.basename(os.environ.get("LBF_LIB", "liblbfhash.so"))}
with ChunkHasher(device_mask=1) as h:
    cases = {"one_64KiB": lambda: h.sha1(data[:65536]),
             "one_256KiB": lambda: h.sha1(data[:262144]),
             "batch_100x256KiB": lambda: h.hash_chunks(data, offs, sizes),
             "ragged_256": lambda: h.hash_chunks(data, r_offs, r_sizes),
             "ragged_20000": lambda: h.hash_chunks(data, x_offs, x_sizes)}
    for name, f in cases.items():
        f()
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t)
        out[name + "_ms"] = round(float(np.median(ts)) * 1e3, 3)
print(json.dumps(out))
