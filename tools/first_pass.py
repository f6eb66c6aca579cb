#!/usr/bin/env python3
"""First job on a fresh context against the second (diagnostic, GPU box).

A one-shot encode pays for its staging inside its first job: the pinned host
ring (3 x LBF_PIN_MB) and the HBM batch slots are sized to the work and
allocated then (lbf_capi.cpp ensure_slot_bytes).  For each size this creates a
new context, times job 1 and job 2 (host memory in, digests out, 256 KiB
chunks) and reports both rates and the difference in ms.
Usage: [LBF_LIB=...] python tools/first_pass.py [reps]"""
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bitflood_amd import ChunkHasher, chunk_table  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
data = np.random.default_rng(1).integers(0, 256, 4 << 30, dtype=np.uint8)
with ChunkHasher(device_mask=1) as h:  # HIP initialised once, outside the timings
    h.sha1(data[:64])
res = {}
for mib in (256, 1024, 4096):
    offs, sizes = chunk_table(mib << 20, 262144)
    firsts, seconds = [], []
    for _ in range(reps):
        with ChunkHasher(device_mask=1) as h:
            t = time.perf_counter()
            h.hash_chunks(data, offs, sizes)
            firsts.append(time.perf_counter() - t)
            t = time.perf_counter()
            h.hash_chunks(data, offs, sizes)
            seconds.append(time.perf_counter() - t)
    f, s = min(firsts), min(seconds)
    res[mib] = {"first_gibs": round(mib / 1024 / f, 2), "second_gibs": round(mib / 1024 / s, 2),
                "extra_ms": round((f - s) * 1e3, 2)}
    print(mib, "MiB", res[mib], flush=True)
print(json.dumps({"lib": os.environ.get("LBF_LIB", "default"), "first_pass": res}))
