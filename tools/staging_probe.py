#!/usr/bin/env python3
"""Per-call cost of the host staging path (diagnostic): hash_chunks over a
160 MiB pool with 3,000 random chunks and a uniform 256 KiB table, timed per
call, so a regression in the staging pipeline shows up as seconds, not ms.
Usage: [LBF_NUMA=0] python tools/staging_probe.py"""
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bitflood_amd import ChunkHasher, chunk_table  # noqa: E402

rng = np.random.default_rng(3)
pool = rng.integers(0, 256, 160 << 20, dtype=np.uint8)
sizes = rng.integers(0, 1 << 20, 3000).astype(np.uint32)
offs = np.array([rng.integers(0, pool.size - int(s) + 1) for s in sizes], dtype=np.uint64)
uo, us = chunk_table(pool.size, 262144)
out = {"numa": os.environ.get("LBF_NUMA", "1"), "random_ms": [], "uniform_ms": []}
with ChunkHasher(device_mask=1) as h:
    for _ in range(5):
        t = time.perf_counter()
        h.hash_chunks(pool, offs, sizes)
        out["random_ms"].append(round((time.perf_counter() - t) * 1e3, 1))
        t = time.perf_counter()
        h.hash_chunks(pool, uo, us)
        out["uniform_ms"].append(round((time.perf_counter() - t) * 1e3, 1))
    out["placement"] = h.worker_info(0)
print(json.dumps(out))
