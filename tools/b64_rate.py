#!/usr/bin/env python3
"""Rate of lbf_b64_verify_batch and lbf_verify_encode_b64_batch (diagnostic,
GPU box): N chunks of C5 frames' base64 text decoded and verified on the
device, and N chunks verified and encoded, against the host decode the
leecher otherwise runs (PeerWire::Base64Get is C++; Python's binascii stands
in for its rate only as an order of magnitude).  Run it under
`rocprofv3 --kernel-trace --stats` for the decode kernel's own duration.

    python tools/b64_rate.py [--chunks 1024] [--chunk-kib 256] [--reps 5]
"""
import argparse
import base64
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (first: one HIP runtime per process)

from bitflood_amd import ChunkHasher  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402
from tests.test_gpu_b64 import xmlrpc_text  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1024)
    ap.add_argument("--chunk-kib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    cs, n = a.chunk_kib * 1024, a.chunks
    data = Oracle().synth(0x5EED, 0, cs * n, nthreads=16)
    one = xmlrpc_text(data[:cs].tobytes())
    slot = (len(one) + 16 + 15) // 16 * 16
    text = np.zeros(slot * n, dtype=np.uint8)
    tlen = np.zeros(n, dtype=np.uint32)
    for i in range(n):
        t = xmlrpc_text(data[i * cs:(i + 1) * cs].tobytes())
        text[i * slot:i * slot + len(t)] = np.frombuffer(t, np.uint8)
        tlen[i] = len(t)
    toff = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    exp = np.frombuffer(b"".join(hashlib.sha1(data[i * cs:(i + 1) * cs]).digest() for i in range(n)), np.uint8)
    out = np.zeros(cs * n, dtype=np.uint8)
    ooff = np.arange(n, dtype=np.uint64) * np.uint64(cs)
    esz = np.full(n, cs, dtype=np.uint32)
    res = {"chunks": n, "chunk_size": cs, "text_bytes": int(tlen.sum())}
    with ChunkHasher(device_mask=1) as h:
        for registered in (False, True):
            if registered:
                h.register_host(text)
                h.register_host(out)
            h.verify_b64(text, toff, tlen, esz, exp, out, ooff)  # warm: device scratch
            t0 = time.perf_counter()
            for _ in range(a.reps):
                ver, dec = h.verify_b64(text, toff, tlen, esz, exp, out, ooff)
            dt = (time.perf_counter() - t0) / a.reps
            ok = bool(ver.all() and (dec == cs).all() and np.array_equal(out, data))
            res["registered" if registered else "pageable"] = {"ms": round(dt * 1e3, 3),
                                                                "decoded_gibs": round(cs * n / dt / 2**30, 3),
                                                                "parity": ok}
        # the CPU-decode path's GPU half for comparison: verify of the decoded
        # bytes from registered memory (what the leecher's VerifyChunks does)
        h.verify_chunks(out, ooff, esz, exp)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            v2 = h.verify_chunks(out, ooff, esz, exp)
        dt = (time.perf_counter() - t0) / a.reps
        res["verify_decoded_registered"] = {"ms": round(dt * 1e3, 3), "parity": bool(v2.all())}
        # the sender's half: verify + encode of the same chunks into the same
        # text layout (both registered), whole call timed
        dptr = data.ctypes.data
        h.register_host(data)
        enc = np.zeros_like(text)
        h.register_host(enc)
        ver = np.zeros(n, dtype=np.uint8)
        dsz = np.full(n, cs, dtype=np.uint32)
        args = (h._h, dptr, data.size, ooff.ctypes.data, dsz.ctypes.data, n, exp.ctypes.data, ver.ctypes.data,
                enc.ctypes.data, enc.size, toff.ctypes.data)
        assert h._lib.lbf_verify_encode_b64_batch(*args) == 0
        t0 = time.perf_counter()
        for _ in range(a.reps):
            h._lib.lbf_verify_encode_b64_batch(*args)
        dt = (time.perf_counter() - t0) / a.reps
        same = all(bytes(enc[i * slot:i * slot + tlen[i]]) == bytes(text[i * slot:i * slot + tlen[i]])
                   for i in range(0, n, max(1, n // 16)))
        res["verify_encode_registered"] = {"ms": round(dt * 1e3, 3), "bytes_gibs": round(cs * n / dt / 2**30, 3),
                                           "parity": bool(ver.all()) and same}
        h.unregister_host(data)
        h.unregister_host(enc)
        h.unregister_host(text)
        h.unregister_host(out)
    # host decode of the same text, one thread, for scale (binascii, C)
    t0 = time.perf_counter()
    for i in range(min(n, 256)):
        base64.b64decode(bytes(text[i * slot:i * slot + tlen[i]]).replace(b" ", b""))
    dt = (time.perf_counter() - t0) / min(n, 256)
    res["host_binascii_one_thread_gibs"] = round(cs / dt / 2**30, 3)
    t0 = time.perf_counter()
    for i in range(min(n, 256)):
        base64.b64encode(data[i * cs:(i + 1) * cs])
    dt = (time.perf_counter() - t0) / min(n, 256)
    res["host_binascii_encode_one_thread_gibs"] = round(cs / dt / 2**30, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
