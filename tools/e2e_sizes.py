"""PCIe-inclusive rate (host memory in -> digests out) by job size.

Diagnostic, GPU box: times ChunkHasher.hash_chunks on host buffers of
64 MiB .. 4 GiB at 256 KiB chunks (one warm pass, then the best of three), so
the staging pipeline's behaviour on mid-sized jobs is visible.
Env LBF_SLOTS / LBF_SLOT_MB select the staging shape, LBF_NUMA=0 turns the
NUMA placement of staging and copy threads off (A/B).  Spot-checks digests
against hashlib.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process, loaded first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bitflood_amd import ChunkHasher, chunk_table  # noqa: E402

CS = 262144
rng = np.random.default_rng(7)
big = rng.integers(0, 256, size=4 << 30, dtype=np.uint8)
out = {"slots": os.environ.get("LBF_SLOTS", "3"), "slot_mb": os.environ.get("LBF_SLOT_MB", "512"),
       "numa": os.environ.get("LBF_NUMA", "1"), "gibs": {}}
with ChunkHasher(device_mask=1) as h:
    for mib in (64, 256, 1024, 4096):
        data = big[: mib << 20]
        offs, sizes = chunk_table(data.size, CS)
        got = h.hash_chunks(data, offs, sizes)
        for i in (0, len(sizes) - 1):
            o = int(offs[i])
            assert bytes(got[i]) == hashlib.sha1(data[o:o + int(sizes[i])].tobytes()).digest(), (mib, i)
        best = 1e9
        for _ in range(3):
            t = time.perf_counter()
            h.hash_chunks(data, offs, sizes)
            best = min(best, time.perf_counter() - t)
        out["gibs"][mib] = round(data.size / best / 2**30, 2)
        print(mib, "MiB", out["gibs"][mib], "GiB/s", flush=True)
    out["placement"] = h.worker_info(0)
print(json.dumps(out))
