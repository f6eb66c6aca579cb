#!/usr/bin/env python3
"""Where the encoder CLI's fixed ≈0.7 s goes (diagnostic).

Times, in a fresh process without torch (like lbf_encoder): loading
liblbfhash.so, the first HIP call, lbf_ctx_create (streams, device slots and
pinned staging), the first and second one-chunk hash, and lbf_ctx_destroy.
Usage: python tools/startup_probe.py [slot_mb]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    if len(sys.argv) > 1:
        os.environ["LBF_SLOT_MB"] = sys.argv[1]
    t = {}
    t0 = time.perf_counter()
    lib = ctypes.CDLL(os.path.join(ROOT, "bitflood_amd", "lib", "liblbfhash.so"))
    t["load_lib"] = time.perf_counter() - t0
    n = ctypes.c_int()
    t0 = time.perf_counter()
    lib.lbf_device_count(ctypes.byref(n))
    t["hip_init"] = time.perf_counter() - t0
    ctx = ctypes.c_void_p()
    t0 = time.perf_counter()
    assert lib.lbf_ctx_create(ctypes.c_uint32(1), ctypes.byref(ctx)) == 0
    t["ctx_create"] = time.perf_counter() - t0
    data = (ctypes.c_uint8 * 262144)()
    out = (ctypes.c_uint8 * 20)()
    for k in ("first_hash", "second_hash"):
        t0 = time.perf_counter()
        assert lib.lbf_sha1_one(ctx, data, ctypes.c_uint32(262144), out) == 0
        t[k] = time.perf_counter() - t0
    t0 = time.perf_counter()
    lib.lbf_ctx_destroy(ctx)
    t["ctx_destroy"] = time.perf_counter() - t0
    print({k: round(v * 1e3, 1) for k, v in t.items()}, "ms", "slot_mb", os.environ.get("LBF_SLOT_MB", "512"))


if __name__ == "__main__":
    main()
