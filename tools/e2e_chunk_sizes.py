#!/usr/bin/env python3
"""PCIe-inclusive rate by chunk size (diagnostic, GPU box): host memory in ->
digests out for a 4 GiB buffer at 256 KiB .. 16 MiB chunks, best of 3 after a
warm pass.  Each staging group's kernel lasts one chunk's serial SHA-1 chain
(≈3.1 ms per 256 KiB), so large chunks need more bytes in flight to keep PCIe
busy.  Usage: [LBF_SLOTS=.. LBF_SLOT_MB=..] python tools/e2e_chunk_sizes.py"""
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bitflood_amd import ChunkHasher, chunk_table  # noqa: E402

data = np.random.default_rng(1).integers(0, 256, 4 << 30, dtype=np.uint8)
out = {"slots": os.environ.get("LBF_SLOTS", "3"), "slot_mb": os.environ.get("LBF_SLOT_MB", "512"), "gibs": {}}
with ChunkHasher(device_mask=1) as h:
    for cs in (262144, 1 << 20, 4 << 20, 16 << 20):
        offs, sizes = chunk_table(data.size, cs)
        h.hash_chunks(data, offs, sizes)
        best = 1e9
        for _ in range(3):
            t = time.perf_counter()
            h.hash_chunks(data, offs, sizes)
            best = min(best, time.perf_counter() - t)
        out["gibs"][cs >> 10] = round(data.size / best / 2**30, 2)
        print(cs >> 10, "KiB", out["gibs"][cs >> 10], flush=True)
print(json.dumps(out))
