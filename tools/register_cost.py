#!/usr/bin/env python3
"""What does pinning cost, and where does the cost land? (VERDICT r05 next #5;
diagnostic, GPU box, one lease.)

For each size (64 MiB, 1 GiB, 4 GiB) and each of two sources, on FRESH memory
(never registered before, written once so its pages exist; --kind picks
4 KiB pages, transparent huge pages, or numpy's own allocation):

  raw HIP (hipHostRegister / hipMemcpy, no library):
    register_ms        hipHostRegister(portable) of the whole buffer
    copy1_ms, copy2_ms one synchronous H2D of the whole buffer into HBM, twice:
                       if the driver defers locking the pages, the first copy pays
    unregister_ms      hipHostUnregister
  the library (ChunkHasher, 256 KiB chunks, digests checked against hashlib):
    lbf_register_ms    lbf_host_register (hipHostRegister underneath)
    pass1_ms..pass3_ms hash_chunks over the registered buffer (direct route)
    lbf_unregister_ms  lbf_host_unregister
    autopin1/2_ms      hash_chunks on pageable fresh memory with on-the-fly pinning
                       (LBF_AUTOPIN=1: register + direct + unregister inside the call)
    staged1/2_ms       the same with LBF_AUTOPIN=0 (memcpy through pinned staging)

A register on memory that was never written is timed too (register_untouched_ms):
pages that do not exist yet must be faulted in by someone.  One JSON line.

    python tools/register_cost.py [--sizes 64,1024,4096] [--kind 4k|thp|numpy]
"""
import argparse
import ctypes
import hashlib
import json
import mmap
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process, loaded first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bitflood_amd import ChunkHasher, chunk_table  # noqa: E402

CS = 262144
MIB = 1 << 20


def hip_lib():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return hip


def ms(t0):
    return round((time.perf_counter() - t0) * 1e3, 3)


KIND = "4k"  # --kind: how fresh buffers are backed


class _NumpyOwner:
    def close(self):
        pass


def fresh(nbytes, seed):
    """A buffer never registered before, written once.  KIND: '4k' an anonymous
    mmap advised MADV_NOHUGEPAGE (what glibc malloc / new[] give a C++ caller
    when THP is 'madvise'), 'thp' one advised MADV_HUGEPAGE, 'numpy' np.empty
    (numpy advises huge pages itself for large arrays)."""
    if KIND == "numpy":
        a = np.empty(nbytes, dtype=np.uint8)
        mm = _NumpyOwner()
    else:
        mm = mmap.mmap(-1, nbytes)
        mm.madvise(mmap.MADV_HUGEPAGE if KIND == "thp" else mmap.MADV_NOHUGEPAGE)
        a = np.frombuffer(mm, dtype=np.uint8)
    a[:] = np.random.default_rng(seed).integers(0, 256, size=nbytes, dtype=np.uint8)
    return mm, a


def anon_huge_kib():
    try:
        for line in open("/proc/self/smaps_rollup"):
            if line.startswith("AnonHugePages:"):
                return int(line.split()[1])
    except OSError:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,1024,4096")
    ap.add_argument("--kind", choices=["4k", "thp", "numpy"], default="4k")
    a = ap.parse_args()
    global KIND
    KIND = a.kind
    hip = hip_lib()
    try:
        thp = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
    except OSError:
        thp = None
    out = {"chunk": CS, "kind": KIND, "thp_enabled": thp, "sizes_mib": {}}
    with ChunkHasher(device_mask=1) as h:
        for mib in [int(x) for x in a.sizes.split(",")]:
            n = mib * MIB
            r = {}
            dev = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(dev), n) == 0
            # raw HIP on fresh memory
            h0 = anon_huge_kib()
            mm, buf = fresh(n, mib)
            h1 = anon_huge_kib()
            if h0 is not None and h1 is not None:
                r["anon_huge_fraction"] = round((h1 - h0) * 1024 / n, 3)
            p = ctypes.c_void_p(buf.ctypes.data)
            t = time.perf_counter()
            assert hip.hipHostRegister(p, n, 1) == 0
            r["register_ms"] = ms(t)
            for k in (1, 2):
                t = time.perf_counter()
                assert hip.hipMemcpy(dev, p, n, 1) == 0  # hipMemcpyHostToDevice
                r[f"copy{k}_ms"] = ms(t)
            t = time.perf_counter()
            assert hip.hipHostUnregister(p) == 0
            r["unregister_ms"] = ms(t)
            t = time.perf_counter()
            assert hip.hipMemcpy(dev, p, n, 1) == 0  # the same bytes, pageable again
            r["copy_pageable_ms"] = ms(t)
            del buf
            mm.close()
            # register on memory whose pages were never written
            mm = mmap.mmap(-1, n)
            mm.madvise(mmap.MADV_HUGEPAGE if KIND == "thp" else mmap.MADV_NOHUGEPAGE)
            addr = ctypes.addressof(ctypes.c_char.from_buffer(mm))
            t = time.perf_counter()
            rc = hip.hipHostRegister(ctypes.c_void_p(addr), n, 1)
            r["register_untouched_ms"] = ms(t) if rc == 0 else f"rc={rc}"
            if rc == 0:
                t = time.perf_counter()
                assert hip.hipMemcpy(dev, ctypes.c_void_p(addr), n, 1) == 0
                r["untouched_copy1_ms"] = ms(t)
                assert hip.hipHostUnregister(ctypes.c_void_p(addr)) == 0
            mm.close()
            assert hip.hipFree(dev) == 0
            # the library on fresh memory: registered, then pinned on the fly, then staged
            mm, buf = fresh(n, mib + 1)
            offs, sizes = chunk_table(n, CS)
            last = hashlib.sha1(buf[int(offs[-1]):].tobytes()).digest()
            t = time.perf_counter()
            h.register_host(buf)
            r["lbf_register_ms"] = ms(t)
            for k in (1, 2, 3):
                s0 = h.staging_stats()["direct"]
                t = time.perf_counter()
                got = h.hash_chunks(buf, offs, sizes)
                r[f"pass{k}_ms"] = ms(t)
                assert bytes(got[-1]) == last and h.staging_stats()["direct"] - s0 == n
            t = time.perf_counter()
            h.unregister_host(buf)
            r["lbf_unregister_ms"] = ms(t)
            del buf
            mm.close()
            for mode, env in (("autopin", "1"), ("staged", "0")):
                mm, buf = fresh(n, mib + 2)
                last = hashlib.sha1(buf[int(offs[-1]):].tobytes()).digest()
                os.environ["LBF_AUTOPIN"] = env
                for k in (1, 2):
                    t = time.perf_counter()
                    got = h.hash_chunks(buf, offs, sizes)
                    r[f"{mode}{k}_ms"] = ms(t)
                    assert bytes(got[-1]) == last
                del buf
                mm.close()
            os.environ.pop("LBF_AUTOPIN", None)
            for k in [x for x in r if x.endswith("_ms") and isinstance(r[x], float) and r[x] > 0]:
                r[k.replace("_ms", "_gibs")] = round(n / (r[k] / 1e3) / 2**30, 2)
            out["sizes_mib"][mib] = r
            print(json.dumps({mib: r}), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
