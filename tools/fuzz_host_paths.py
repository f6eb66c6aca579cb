#!/usr/bin/env python3
"""Randomised fuzz of the host-side paths around the kernels (diagnostic).

tools/fuzz_gpu.py varies the kernels; this varies what feeds them: staging slot
sizes (1, 3, 16, 512 MiB, so batches split into many groups and chunks larger
than a slot take the oversize path), chunk sizes up to 40 MiB, memory vs file
sources (pread), truncated and missing files in verify mode, device-pointer
batches, memory registered with the context (the direct route), and (mode 7)
multi-file batches (lbf_files_ranges) over 2-40 files, some missing in verify
mode, with a random LBF_FILES_WINDOW so floods run in windows of files.  The copy-thread count is process-wide (LBF_COPY_THREADS), so run the
tool once per setting.  Everything is checked against the oracle restatement.

Usage: LBF_COPY_THREADS=3 python tools/fuzz_host_paths.py [--seconds 60] [--seed 1]
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (first: one HIP runtime per process)

from bitflood_amd import ChunkHasher, DeviceBuffer  # noqa: E402
from bitflood_amd import _capi  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402

THREADS = min(16, os.cpu_count() or 1)
SLOTS_MB = [1, 3, 16, 512]
DIAG = False


def draw_table(rng, span):
    if rng.random() < 0.15:  # a few big chunks (oversize with small slots)
        n = int(rng.integers(1, 6))
        sizes = rng.integers(0, 40 << 20, n)
    else:
        n = int(rng.integers(1, 1500))
        sizes = np.where(rng.random(n) < 0.5, rng.integers(0, 300, n), rng.integers(0, 512 << 10, n))
    sizes = np.minimum(sizes, span).astype(np.uint32)
    if rng.random() < 0.3:  # contiguous file chunking
        cs = int(rng.choice([4096, 65536, 262144, 1 << 20, 3 << 20]))
        total = int(rng.integers(1, span + 1))
        n = (total + cs - 1) // cs
        offs = np.arange(n, dtype=np.uint64) * np.uint64(cs)
        sizes = np.minimum(cs, total - offs).astype(np.uint32)
        return offs, sizes
    offs = np.array([rng.integers(0, span - int(s) + 1) for s in sizes], dtype=np.uint64)
    if rng.random() < 0.5:
        offs &= ~np.uint64(15)
    return offs, sizes


def registered_case(rng, slot, mode, orc, h, pool):
    start = int(rng.integers(0, 8192)) if rng.random() < 0.5 else 0
    src = pool[start:]
    offs, sizes = draw_table(rng, src.size)
    want = orc.sha1_batch(src, offs, sizes, nthreads=THREADS)
    n = offs.size
    h.register_host(src)
    try:
        if mode == 5:
            return slot, mode, n, bool(np.array_equal(h.hash_chunks(src, offs, sizes), want))
        exp = want.copy()
        bad = rng.random(n) < 0.1
        exp[bad, rng.integers(0, 20)] ^= np.uint8(1 << int(rng.integers(0, 8)))
        return slot, mode, n, bool(np.array_equal(h.verify_chunks(src, offs, sizes, exp), ~bad))
    finally:
        h.unregister_host(src)


def files_case(rng, slot, orc, h, pool, tmpdir):
    """Mode 7: one lbf_files_ranges call over k files cut from the pool, chunks
    listed in a shuffled order, with LBF_FILES_WINDOW drawn per case (read by
    the library on every call), hash or verify (a few files missing)."""
    k = int(rng.integers(2, 41))
    lo = int(rng.integers(0, pool.size // 2))
    cuts = np.sort(rng.integers(lo, min(pool.size, lo + (64 << 20)) + 1, k + 1))
    paths, fo, offs, sizes, srcs = [], [], [], [], []
    for f in range(k):
        data = pool[cuts[f]:cuts[f + 1]]
        p = os.path.join(tmpdir, f"m{f:02d}.bin")
        data.tofile(p)
        paths.append(p)
        cs = int(rng.choice([4096, 65536, 262144, 1 << 20]))
        for o in range(0, data.size, cs):
            fo.append(f)
            offs.append(o)
            sizes.append(min(cs, data.size - o))
            srcs.append(int(cuts[f]) + o)
    n = len(fo)
    if n == 0:
        return slot, 7, 0, True
    order = rng.permutation(n)
    fo, offs, sizes, srcs = [np.array(x)[order] for x in (fo, offs, sizes, srcs)]
    want = orc.sha1_batch(pool, srcs.astype(np.uint64), sizes.astype(np.uint32), nthreads=THREADS)
    os.environ["LBF_FILES_WINDOW"] = str(int(rng.integers(1, k + 3)))
    try:
        if rng.random() < 0.5:
            ok = bool(np.array_equal(h.hash_files(paths, fo, offs, sizes), want))
        else:
            gone = rng.random(k) < 0.2
            for f in np.nonzero(gone)[0]:
                os.remove(paths[f])
            exp = want.copy()
            bad = rng.random(n) < 0.1
            exp[bad, 0] ^= np.uint8(1)
            expect = ~bad & ~gone[fo]
            ok = bool(np.array_equal(h.verify_files(paths, fo, offs, sizes, exp), expect))
    finally:
        os.environ.pop("LBF_FILES_WINDOW", None)
        for p in paths:
            if os.path.exists(p):
                os.remove(p)
    return slot, 7, n, ok


def one_case(seed, orc, hashers, pool, path, tmpdir):
    rng = np.random.default_rng(seed)
    slot = int(rng.choice(SLOTS_MB))
    h = hashers[slot]
    # 0 mem hash, 1 mem verify, 2 file hash, 3 file verify, 4 device ptrs,
    # 5/6 mem hash/verify from a registered source (lbf_host_register) that
    # starts at a random byte of the pool, 7 multi-file batches in windows
    mode = int(rng.integers(0, 8))
    if mode == 7:
        return files_case(rng, slot, orc, h, pool, tmpdir)
    if mode >= 5:
        return registered_case(rng, slot, mode, orc, h, pool)
    offs, sizes = draw_table(rng, pool.size)
    want = orc.sha1_batch(pool, offs, sizes, nthreads=THREADS)
    n = offs.size
    if mode == 0:
        return slot, mode, n, bool(np.array_equal(h.hash_chunks(pool, offs, sizes), want))
    if mode == 2:
        return slot, mode, n, bool(np.array_equal(h.hash_file(path, offs, sizes), want))
    if mode == 4:
        bufs = [DeviceBuffer(pool.size), DeviceBuffer(max(8, n * 8)), DeviceBuffer(max(4, n * 4)),
                DeviceBuffer(n * 20)]
        try:
            bufs[0].upload(pool)
            bufs[1].upload(offs)
            bufs[2].upload(sizes)
            _capi.check(_capi.load().lbf_sha1_batch(h._h, bufs[0].ptr, pool.size, bufs[1].ptr, bufs[2].ptr, n,
                                                    bufs[3].ptr, _capi.LBF_DEVICE_PTR))
            got = bufs[3].download(n * 20).reshape(n, 20)
        finally:
            for b in bufs:
                b.free()
        return slot, mode, n, bool(np.array_equal(got, want))
    exp = want.copy()
    bad = rng.random(n) < 0.1
    exp[bad, rng.integers(0, 20)] ^= np.uint8(1 << int(rng.integers(0, 8)))
    if mode == 1:
        return slot, mode, n, bool(np.array_equal(h.verify_chunks(pool, offs, sizes, exp), ~bad))
    # file verify: sometimes against a truncated copy (chunks past the cut are '0')
    cut = pool.size if rng.random() < 0.5 else int(rng.integers(0, pool.size + 1))
    vpath = path
    if cut < pool.size:
        vpath = os.path.join(tmpdir, "cut.bin")
        with open(vpath, "wb") as f:
            f.write(pool[:cut].tobytes())
    # Flood.cpp:259-275: a chunk is '1' when fseek succeeds (it does past EOF
    # too), fread returns all its bytes (0 of 0 for an empty chunk) and the hash
    # matches -- so an empty chunk past the cut still verifies
    expect = ~bad & ((offs + sizes.astype(np.uint64) <= np.uint64(cut)) | (sizes == 0))
    got = h.verify_file(vpath, offs, sizes, exp)
    if DIAG and not np.array_equal(got, expect):
        for k in np.nonzero(got != expect)[0][:10]:
            print(json.dumps({"chunk": int(k), "off": int(offs[k]), "size": int(sizes[k]), "cut": cut,
                              "corrupted": bool(bad[k]), "got": bool(got[k]), "expect": bool(expect[k])}))
        print(json.dumps({"n_mismatch": int((got != expect).sum()), "n": n, "cut": cut, "file_size": pool.size}))
    return slot, mode, n, bool(np.array_equal(got, expect))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--replay", type=int, default=None, help="re-run one case seed, print mismatches")
    a = ap.parse_args()
    global DIAG
    DIAG = a.replay is not None
    orc = Oracle()
    pool = orc.synth(0xF0F0, 0, (96 << 20) + 12345, nthreads=THREADS)
    tmpdir = tempfile.mkdtemp(prefix="lbf_fuzz_")
    path = os.path.join(tmpdir, "pool.bin")
    with open(path, "wb") as f:
        f.write(pool.tobytes())
    hashers = {}
    for mb in SLOTS_MB:
        os.environ["LBF_SLOT_MB"] = str(mb)
        hashers[mb] = ChunkHasher(device_mask=1)
    os.environ.pop("LBF_SLOT_MB", None)
    t0, k, stats, rc = time.time(), 0, {}, 0
    try:
        if a.replay is not None:
            print(json.dumps({"replay": a.replay, "result": one_case(a.replay, orc, hashers, pool, path, tmpdir)}))
            a.seconds = 0
        while time.time() - t0 < a.seconds:
            seed = a.seed * 1_000_003 + k
            slot, mode, n, ok = one_case(seed, orc, hashers, pool, path, tmpdir)
            stats[f"slot{slot}m{mode}"] = stats.get(f"slot{slot}m{mode}", 0) + 1
            if not ok:
                print(json.dumps({"FAIL": True, "seed": seed, "slot_mb": slot, "mode": mode, "n": n}), flush=True)
                rc = 1
                break
            k += 1
            if k % 25 == 0:
                print(f"{k} cases ok ({time.time() - t0:.0f} s)", flush=True)
    finally:
        for h in hashers.values():
            h.close()
        for f in os.listdir(tmpdir):
            os.remove(os.path.join(tmpdir, f))
        os.rmdir(tmpdir)
    if rc == 0:
        print(json.dumps({"cases": k, "seconds": round(time.time() - t0, 1), "all_ok": True,
                          "copy_threads": os.environ.get("LBF_COPY_THREADS", "8"), "per_slot_mode": stats}))
    return rc


if __name__ == "__main__":
    sys.exit(main())
