#!/usr/bin/env python3
"""Randomised fuzz of the C++ layer through its two CLIs (diagnostic).

Each case writes a random file (empty, tiny, around chunk multiples, up to
48 MiB), encodes it with lbf_encoder (test_encoder.cpp's command line) at a
random chunk size, and checks the flood file against hashlib: every chunk's
index, size and 27-char hash, the File size attribute.  Then it damages the
file (flipped bytes, a truncation, an appended tail, deletion, or nothing) and
checks lbf_verify's chunkmap, verified count, to_download count and content
hash against what Flood.cpp:220-299 implies for those bytes.

Usage: python tools/fuzz_cli.py [--seconds 120] [--seed 1]
"""
import argparse
import base64
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "bitflood_amd", "lib")
ENCODER = os.path.join(LIB, "lbf_encoder")
VERIFY = os.path.join(LIB, "lbf_verify")


def b64_27(d: bytes) -> str:
    return base64.b64encode(d).decode().rstrip("=")


def one_case(seed, tmp):
    rng = np.random.default_rng(seed)
    cs = int(rng.choice([1, 7, 55, 56, 64, 100, 4096, 65536, 262144, 1 << 20, (3 << 20) + 17]))
    kind = int(rng.integers(0, 4))
    if kind == 0:
        size = int(rng.integers(0, 3))
    elif kind == 1:
        size = int(rng.integers(0, 200))
    elif kind == 2:
        size = max(0, cs * int(rng.integers(1, 9)) + int(rng.integers(-2, 3)))
    else:
        size = int(rng.integers(0, 48 << 20))
    size = min(size, cs * 40000)  # bound the chunk count
    data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    name = "f.bin"
    fpath = os.path.join(tmp, name)
    with open(fpath, "wb") as f:
        f.write(data)
    r = subprocess.run([ENCODER, name, "http://127.0.0.1:10101/", "f.flood", "--chunksize", str(cs)],
                       cwd=tmp, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"stage": "encode", "rc": r.returncode, "err": r.stderr[-300:], "size": size, "cs": cs}
    xml = open(os.path.join(tmp, "f.flood")).read()
    chunks = [(int(i), int(s), h) for h, i, s in
              re.findall(r'<Chunk hash="([^"]+)" index="(\d+)" size="(\d+)" weight="0"/>', xml)]
    n = (size + cs - 1) // cs
    want = [(i, min(cs, size - i * cs), b64_27(hashlib.sha1(data[i * cs:(i + 1) * cs]).digest())) for i in range(n)]
    if chunks != want:
        bad = [k for k in range(min(len(chunks), len(want))) if chunks[k] != want[k]]
        return {"stage": "encode_chunks", "size": size, "cs": cs, "n_got": len(chunks), "n_want": n, "first_bad": bad[:3]}
    m = re.search(r'<File name="([^"]+)" size="(\d+)"', xml)
    if not m or m.group(1) != name or int(m.group(2)) != size:
        return {"stage": "encode_file_attr", "size": size, "cs": cs, "got": m.groups() if m else None}
    # damage, then verify (Flood.cpp:259-275: '1' iff the chunk's bytes are all present and hash equal)
    dmg = int(rng.integers(0, 5))
    new = bytearray(data)
    if dmg == 1 and size:
        for _ in range(int(rng.integers(1, 6))):
            new[int(rng.integers(0, size))] ^= 1 << int(rng.integers(0, 8))
    elif dmg == 2:
        new = new[:int(rng.integers(0, size + 1))]
    elif dmg == 3:
        new += bytes(rng.integers(0, 256, int(rng.integers(1, 5000)), dtype=np.uint8))
    if dmg == 4:
        os.remove(fpath)
    else:
        with open(fpath, "wb") as f:
            f.write(bytes(new))
    r = subprocess.run([VERIFY, "f.flood", "--no-resolve"], cwd=tmp, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"stage": "verify", "rc": r.returncode, "err": r.stderr[-300:], "size": size, "cs": cs, "dmg": dmg}
    lines = dict(line.split(" ", 1) for line in r.stdout.strip().splitlines())
    if dmg == 4:
        cmap = "0" * n
    else:
        cmap = "".join("1" if i * cs + w[1] <= len(new) and bytes(new[i * cs:i * cs + w[1]]) == data[i * cs:i * cs + w[1]]
                       else "0" for i, w in enumerate(want))
    content = b64_27(hashlib.sha1((name + "".join(w[2] for w in want)).encode()).digest())
    got_line = lines.get(name, "0 0" if n == 0 else "")
    want_line = f"{n} {cmap.count('1')} {cmap}"
    if got_line.strip() != want_line.strip() or lines.get("content_hash") != content or \
            int(lines.get("to_download", -1)) != cmap.count("0"):
        return {"stage": "verify_map", "size": size, "cs": cs, "dmg": dmg, "got": got_line[:80],
                "want": want_line[:80], "content_ok": lines.get("content_hash") == content,
                "to_download": lines.get("to_download")}
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--replay", type=int, default=None)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="lbf_cli_fuzz_")
    t0, k, rc = time.time(), 0, 0
    try:
        seeds = [a.replay] if a.replay is not None else None
        while (seeds and k < 1) or (not seeds and time.time() - t0 < a.seconds):
            seed = seeds[0] if seeds else a.seed * 1_000_003 + k
            fail = one_case(seed, tmp)
            if fail:
                print(json.dumps({"FAIL": True, "seed": seed, **fail}), flush=True)
                rc = 1
                break
            k += 1
            if k % 10 == 0:
                print(f"{k} cases ok ({time.time() - t0:.0f} s)", flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if rc == 0:
        print(json.dumps({"cases": k, "seconds": round(time.time() - t0, 1), "all_ok": True}))
    return rc


if __name__ == "__main__":
    sys.exit(main())
