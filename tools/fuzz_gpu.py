#!/usr/bin/env python3
"""Randomised GPU-vs-oracle fuzz of every kernel variant (diagnostic, not a test).

Each case draws a kernel variant, a chunk-size mix (tiny, around the 55/56/64-byte
padding boundaries, page-sized, up to 1 MiB), a layout (aligned, unaligned,
overlapping, zero-size chunks) and a mode (hash, verify with random corruptions
of data or expected digests, device-resident uniform launch with a random
first chunk) and checks the GPU result against the oracle restatement
(oracle/sha1_oracle.c, test infrastructure).  Stops at the first mismatch and
prints the case seed so it can be replayed with --seed S --cases 1.

Usage: python tools/fuzz_gpu.py [--seconds 90] [--seed 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (first: one HIP runtime per process)

from bitflood_amd import ChunkHasher, DeviceBuffer  # noqa: E402
from bitflood_amd import hashing as H  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402

# Shipped variants; with LBF_LIB pointing at the A/B library of
# tools/experimental/ (make -C tools/experimental) LBF_FUZZ_ALL=1 adds the rest.
VARIANTS = list(range(1, 13)) if os.environ.get("LBF_FUZZ_ALL") else [1, 7, 10, 11, 12]
if os.environ.get("LBF_FUZZ_VARIANTS"):  # e.g. "7,37" for an A/B variant of the experimental library
    VARIANTS = [int(x) for x in os.environ["LBF_FUZZ_VARIANTS"].split(",")]
THREADS = min(16, os.cpu_count() or 1)


def draw_sizes(rng, n):
    kind = rng.integers(0, 5)
    if kind == 0:  # around the padding boundaries
        base = rng.integers(0, 64, n) + 64 * rng.integers(0, 40, n)
    elif kind == 1:  # tiny
        base = rng.integers(0, 130, n)
    elif kind == 2:  # page-ish
        base = rng.integers(1, 9, n) * 4096 + rng.integers(-3, 4, n)
    elif kind == 3:  # large, ragged
        base = rng.integers(0, 1 << 20, n)
    else:  # uniform chunk size with a short tail
        cs = int(rng.choice([4096, 65536, 262144]))
        base = np.full(n, cs)
        base[-1] = rng.integers(0, cs + 1)
    return np.clip(base, 0, 1 << 20).astype(np.uint32), int(kind)


def one_case(seed, orc, hasher, pool):
    rng = np.random.default_rng(seed)
    v = int(rng.choice(VARIANTS))
    H.set_kernel_variant(v)
    mode = int(rng.integers(0, 3))  # 0 hash, 1 verify, 2 device uniform
    if mode == 2:
        cs = int(rng.choice([64, 100, 4096, 65536, 262144, 1 << 20]))
        total = int(rng.integers(1, min(pool.size, 64 * cs * 64) + 1))
        nchunks = (total + cs - 1) // cs
        first = int(rng.integers(0, nchunks))
        n = int(rng.integers(1, nchunks - first + 1))
        buf = DeviceBuffer(total)
        dig = DeviceBuffer(n * 20)
        try:
            buf.upload(pool[:total])
            H.uniform_launch(buf, total, cs, first, n, dig)
            H.synchronize()
            got = dig.download(n * 20).reshape(n, 20)
        finally:
            buf.free()
            dig.free()
        offs = np.arange(first, first + n, dtype=np.uint64) * np.uint64(cs)
        sizes = np.minimum(cs, total - offs).astype(np.uint32)
        want = orc.sha1_batch(pool, offs, sizes, nthreads=THREADS)
        return v, mode, n, bool(np.array_equal(got, want))
    n = int(rng.integers(1, 6000))
    sizes, kind = draw_sizes(rng, n)
    span = pool.size
    offs = np.array([rng.integers(0, span - int(s) + 1) for s in sizes], dtype=np.uint64)
    if rng.random() < 0.5:
        offs &= ~np.uint64(15)  # aligned starts
    want = orc.sha1_batch(pool, offs, sizes, nthreads=THREADS)
    if mode == 0:
        got = hasher.hash_chunks(pool, offs, sizes)
        return v, mode, n, bool(np.array_equal(got, want))
    exp = want.copy()
    bad = rng.random(n) < 0.1
    exp[bad, rng.integers(0, 20)] ^= np.uint8(1 << int(rng.integers(0, 8)))
    ver = hasher.verify_chunks(pool, offs, sizes, exp)
    return v, mode, n, bool(np.array_equal(ver, ~bad))


def replay(seed, orc, hasher, pool, repeats):
    """Re-run one failing case and say where it differs: hash vs verify, which
    chunks, their sizes and alignment, whether other variants agree, and whether
    the result repeats."""
    rng = np.random.default_rng(seed)
    v = int(rng.choice(VARIANTS))
    mode = int(rng.integers(0, 3))
    print(json.dumps({"seed": seed, "variant": v, "mode": mode}), flush=True)
    if mode == 2:
        print("uniform-mode replay: rerun one_case", one_case(seed, orc, hasher, pool), flush=True)
        return
    n = int(rng.integers(1, 6000))
    sizes, kind = draw_sizes(rng, n)
    offs = np.array([rng.integers(0, pool.size - int(s) + 1) for s in sizes], dtype=np.uint64)
    if rng.random() < 0.5:
        offs &= ~np.uint64(15)
    want = orc.sha1_batch(pool, offs, sizes, nthreads=THREADS)
    exp = want.copy()
    bad = np.zeros(n, bool)
    if mode == 1:
        bad = rng.random(n) < 0.1
        exp[bad, rng.integers(0, 20)] ^= np.uint8(1 << int(rng.integers(0, 8)))
    print(json.dumps({"n": n, "kind": kind, "aligned16": int((offs % 16 == 0).sum()),
                      "size_min": int(sizes.min()), "size_max": int(sizes.max())}), flush=True)
    for vv in [v] + [x for x in VARIANTS if x != v]:
        H.set_kernel_variant(vv)
        for r in range(repeats if vv == v else 1):
            got = hasher.hash_chunks(pool, offs, sizes)
            hbad = np.nonzero((got != want).any(axis=1))[0]
            ver = hasher.verify_chunks(pool, offs, sizes, exp)
            vbad = np.nonzero(ver != ~bad)[0]
            info = {"variant": vv, "rep": r, "hash_mismatch": hbad[:8].tolist(), "n_hash_mismatch": int(hbad.size),
                    "verify_mismatch": vbad[:8].tolist(), "n_verify_mismatch": int(vbad.size)}
            for k in list(hbad[:3]) + list(vbad[:3]):
                info[f"chunk{k}"] = {"size": int(sizes[k]), "off_mod16": int(offs[k] % 16), "corrupted": bool(bad[k]),
                                     "group_pos": int(k % 128)}
            print(json.dumps(info), flush=True)
    H.set_kernel_variant(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=90)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cases", type=int, default=1 << 30)
    ap.add_argument("--replay", type=int, default=None, help="re-run one case seed with diagnostics")
    ap.add_argument("--repeats", type=int, default=3)
    a = ap.parse_args()
    orc = Oracle()
    pool = orc.synth(0xF022, 0, 160 << 20, nthreads=THREADS)
    if a.replay is not None:
        with ChunkHasher(device_mask=1) as hasher:
            replay(a.replay, orc, hasher, pool, a.repeats)
        return 0
    t0 = time.time()
    k = 0
    stats = {}
    with ChunkHasher(device_mask=1) as hasher:
        while k < a.cases and time.time() - t0 < a.seconds:
            seed = a.seed * 1_000_003 + k
            v, mode, n, ok = one_case(seed, orc, hasher, pool)
            stats[(v, mode)] = stats.get((v, mode), 0) + 1
            if not ok:
                print(json.dumps({"FAIL": True, "seed": seed, "variant": v, "mode": mode, "n": n}), flush=True)
                H.set_kernel_variant(0)
                return 1
            k += 1
            if k % 25 == 0:
                print(f"{k} cases ok ({time.time() - t0:.0f} s)", flush=True)
    H.set_kernel_variant(0)
    print(json.dumps({"cases": k, "seconds": round(time.time() - t0, 1), "all_ok": True,
                      "per_variant_mode": {f"v{v}m{m}": c for (v, m), c in sorted(stats.items())}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
