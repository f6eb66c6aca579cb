#!/usr/bin/env python3
"""Disk-path rate of the encoder (diagnostic; DESIGN.md §5 "PCIe-inclusive").

The path north_star names starts at file bytes and ends at digests in a flood
file.  This writes the C2 file (4 GiB synthetic, seed 0x5EED, 256 KiB chunks)
to local storage, then times:
  1. ChunkHasher.hash_file: lbf_file_ranges, pread straight into pinned staging,
     H2D, kernel, D2H (page-cache warm after the write; no root to drop caches);
  2. the lbf_encoder CLI end to end (process start, HIP init, EncodeFile, the
     flood-file XML write): the test_encoder.cpp command line.
Both outputs are checked against the C2 golden (SHA-1 of the 16,384
concatenated raw digests, tests/golden/c2.json).

Usage: python tools/file_rate.py [--dir DIR] [--keep]
"""
import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (first: one HIP runtime per process)

from bitflood_amd import ChunkHasher, b64_27_decode, chunk_table  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402

GIB = 1 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", tempfile.gettempdir()))
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    c2 = json.load(open(os.path.join(ROOT, "tests", "golden", "c2.json")))
    size, cs = c2["size"], c2["chunk_size"]
    path = os.path.join(a.dir, "lbf_c2.bin")
    xml = os.path.join(a.dir, "lbf_c2.flood")
    orc = Oracle()
    t0 = time.perf_counter()
    with open(path, "wb") as f:
        step = 512 << 20
        for off in range(0, size, step):
            f.write(orc.synth(c2["seed"], off, min(step, size - off), nthreads=16).tobytes())
    t_write = time.perf_counter() - t0
    out = {"file_bytes": size, "chunk_size": cs, "write_s": round(t_write, 2), "dir": a.dir}
    try:
        offs, sizes = chunk_table(size, cs)
        with ChunkHasher(device_mask=1) as h:
            h.hash_file(path, offs[:64], sizes[:64])  # warm: kernels loaded, small staging
            rates = []
            for _ in range(3):
                t0 = time.perf_counter()
                d = h.hash_file(path, offs, sizes)
                rates.append(size / GIB / (time.perf_counter() - t0))
        # the first full pass grows the pinned staging to 3 x 512 MiB inside the timing
        out["hash_file_first_gibs"] = round(rates[0], 2)
        out["hash_file_steady_gibs"] = [round(r, 2) for r in rates[1:]]
        out["hash_file_parity"] = hashlib.sha1(d.tobytes()).hexdigest() == c2["sha1_of_concat_raw_digests_hex"]
        enc = os.path.join(ROOT, "bitflood_amd", "lib", "lbf_encoder")
        t0 = time.perf_counter()
        r = subprocess.run([enc, path, "http://127.0.0.1:10101/", xml], capture_output=True, text=True)
        t_cli = time.perf_counter() - t0
        out["cli_rc"] = r.returncode
        out["cli_s"] = round(t_cli, 3)
        out["cli_gibs"] = round(size / GIB / t_cli, 2)
        # fixed cost of the CLI (process start, HIP init, context and staging
        # allocation) from a one-chunk file
        tiny = os.path.join(a.dir, "lbf_tiny.bin")
        with open(tiny, "wb") as f:
            f.write(orc.synth(c2["seed"], 0, cs).tobytes())
        t0 = time.perf_counter()
        r2 = subprocess.run([enc, tiny, "http://127.0.0.1:10101/", xml + ".tiny"], capture_output=True, text=True)
        out["cli_fixed_s"] = round(time.perf_counter() - t0, 3)
        out["cli_marginal_gibs"] = round(size / GIB / max(1e-9, t_cli - out["cli_fixed_s"]), 2)
        for p in (tiny, xml + ".tiny"):
            if os.path.exists(p):
                os.remove(p)
        assert r2.returncode == 0, r2.stderr
        hashes = re.findall(r'hash="([A-Za-z0-9+/]{27})"', open(xml).read())
        raw = b"".join(b64_27_decode(s) for s in hashes)
        out["cli_chunks"] = len(hashes)
        out["cli_parity"] = hashlib.sha1(raw).hexdigest() == c2["sha1_of_concat_raw_digests_hex"]
        out["cli_matches_hash_file"] = raw == d.tobytes()
    finally:
        if not a.keep:
            for p in (path, xml):
                if os.path.exists(p):
                    os.remove(p)
    print(json.dumps(out), flush=True)
    return 0 if out.get("hash_file_parity") and out.get("cli_parity") else 1


if __name__ == "__main__":
    sys.exit(main())
