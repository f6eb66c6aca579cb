"""PCIe-inclusive rate (host memory in -> digests out) by job size.

Diagnostic, GPU box: times ChunkHasher.hash_chunks on host buffers of
64 MiB .. 4 GiB at 256 KiB chunks (one warm pass, then the best of three), so
the staging pipeline's behaviour on mid-sized jobs is visible.
Env LBF_SLOTS / LBF_SLOT_MB select the staging shape, LBF_NUMA=0 turns the
NUMA placement of staging and copy threads off (A/B).  --register pins each
buffer with lbf_host_register first (its cost printed separately), so the
batch goes straight from caller memory to HBM; --local first-touches the
source buffer on the GPU's NUMA node; --thp backs it with transparent huge
pages.  Spot-checks digests against
hashlib.
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
REGISTER = "--register" in sys.argv
LOCAL = "--local" in sys.argv
if LOCAL:
    # first-touch the source on the GPU's NUMA node (the node of its staging):
    # bind this thread there while the buffer is allocated and filled
    with ChunkHasher(device_mask=1) as h0:
        node = h0.worker_info(0)["numa_node"]
    if node >= 0:
        cpus = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
        allowed = set()
        for part in cpus.split(","):
            a, _, b = part.partition("-")
            allowed.update(range(int(a), int(b or a) + 1))
        old_aff = os.sched_getaffinity(0)
        os.sched_setaffinity(0, allowed & old_aff)
rng = np.random.default_rng(7)
if "--thp" in sys.argv:
    # back the source with transparent huge pages (madvise before first touch)
    import mmap
    _mm = mmap.mmap(-1, 4 << 30, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    _mm.madvise(mmap.MADV_HUGEPAGE)
    big = np.frombuffer(_mm, dtype=np.uint8)
    big[:] = rng.integers(0, 256, size=4 << 30, dtype=np.uint8)
else:
    big = rng.integers(0, 256, size=4 << 30, dtype=np.uint8)
if LOCAL and node >= 0:
    os.sched_setaffinity(0, old_aff)
out = {"slots": os.environ.get("LBF_SLOTS", "3"), "slot_mb": os.environ.get("LBF_SLOT_MB", "512"),
       "numa": os.environ.get("LBF_NUMA", "1"), "register": REGISTER, "local_source": LOCAL, "thp": "--thp" in sys.argv, "gibs": {}, "register_s": {}, "stats": {}}
with ChunkHasher(device_mask=1) as h:
    for mib in (64, 256, 1024, 4096):
        data = big[: mib << 20]
        offs, sizes = chunk_table(data.size, CS)
        if REGISTER:
            t = time.perf_counter()
            h.register_host(data)
            out["register_s"][mib] = round(time.perf_counter() - t, 4)
        s0 = h.staging_stats()
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
        s1 = h.staging_stats()
        out["stats"][mib] = {k: s1[k] - s0[k] for k in s1}  # bytes by route over the 4 passes
        if REGISTER:
            t = time.perf_counter()
            h.unregister_host(data)
            out["register_s"][mib] = [out["register_s"][mib], round(time.perf_counter() - t, 4)]
        print(mib, "MiB", out["gibs"][mib], "GiB/s", out["stats"][mib], flush=True)
    out["placement"] = h.worker_info(0)
print(json.dumps(out))
