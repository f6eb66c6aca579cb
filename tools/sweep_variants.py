#!/usr/bin/env python3
"""Kernel-variant sweep over chain counts (diagnostic, not the bench).

Times lbf_sha1_uniform_launch (HIP events on one stream) for each variant at
several chunk counts and chunk sizes over one device-resident synthetic region,
including the C3 shape (64 GiB at 256 KiB = 262,144 chunks) and the per-GPU C4
shape (32 GiB at 1 MiB = 32,768 chunks).  Prints one JSON line per point.
Usage: python tools/sweep_variants.py [--max-gib 64] [--reps 3]
Superseded and diagnostic variants (2-6, 8, 9, 13-23, 25-28) need the A/B library:
  make -C tools/experimental
  LBF_LIB=tools/build/experimental/liblbfhash.so python tools/sweep_variants.py --variants 4,7
"""
import argparse
import hashlib
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

from bitflood_amd import DeviceBuffer  # noqa: E402
from bitflood_amd import hashing as H  # noqa: E402
from bitflood_amd._capi import check, load  # noqa: E402

GIB = 1 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-gib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="1,7,10,11")
    ap.add_argument("--points", default="", help="chunk_size:count,... instead of the built-in list")
    a = ap.parse_args()
    size = a.max_gib * GIB
    points = [(262144, n) for n in (4096, 8192, 16384, 32768, 65536, 131072, 262144)]
    points += [(1 << 20, n) for n in (8192, 16384, 32768, 65536)]
    points += [(65536, n) for n in (16384, 65536, 262144, 1048576)]
    if a.points:
        points = [tuple(int(x) for x in pt.split(":")) for pt in a.points.split(",")]
    points = [(cs, n) for cs, n in points if n * cs <= size]
    if not points:
        return
    buf = DeviceBuffer(size)
    buf.fill_synthetic(0x5EED)
    # digests for the largest chunk count swept (the kernels write n x 20 bytes)
    dig = DeviceBuffer(max(n for _, n in points) * 20)
    H.synchronize()
    lib = load()
    for cs, n in points:
        assert n * 20 <= dig.nbytes and n * cs <= buf.nbytes
        ref = None
        for v in [int(x) for x in a.variants.split(",")]:
            H.set_kernel_variant(v)
            ms = ctypes.c_float()
            check(lib.lbf_time_uniform(buf.ptr, n * cs, cs, 0, n, dig.ptr, 1, None, ctypes.byref(ms)))  # warm
            check(lib.lbf_time_uniform(buf.ptr, n * cs, cs, 0, n, dig.ptr, a.reps, None, ctypes.byref(ms)))
            gbs = n * cs / (ms.value * 1e-3) / 1e9
            dd = hashlib.sha1(dig.download(n * 20).tobytes()).hexdigest()
            ref = ref or dd
            print(json.dumps({"chunk_size": cs, "chunks": n, "gib": n * cs / GIB, "variant": v,
                              "ms": round(ms.value, 4), "GB/s": round(gbs, 1),
                              "GiB/s": round(gbs * 1e9 / GIB, 1), "hbm_frac": round(gbs / 8000, 4),
                              "digests_agree": dd == ref}),
                  flush=True)
    H.set_kernel_variant(0)
    buf.free()
    dig.free()


if __name__ == "__main__":
    main()
