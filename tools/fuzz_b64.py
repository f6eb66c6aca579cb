#!/usr/bin/env python3
"""Randomised fuzz of the wire-form entry points (diagnostic, not a test).

Each case is a batch of 1-64 chunks of 0 B to 300 KiB.  The texts are the
encoder's (tests/test_gpu_b64.py xmlrpc_text, base64.h:154-210) or that text
perturbed in one of the ways the parity test uses: junk or '=' inserted,
characters dropped, truncation, an alphabet character flipped, '=' / junk /
an alphabet character in place of a group character or a separator -- so both
the one-pass decode and the general one are hit, and chunks that go from one
to the other share a batch.  lbf_b64_verify_batch's bytes, lengths and
verdicts must equal the Python restatement of xmlrpc++'s decoder (b64get),
and lbf_verify_encode_b64_batch's text must equal xmlrpc_text.  Stops at the
first mismatch and prints the case seed (--seed S --cases 1 replays it).

Usage: python tools/fuzz_b64.py [--seconds 90] [--seed 1]
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (first: one HIP runtime per process)

from bitflood_amd import ChunkHasher  # noqa: E402
from tests.test_gpu_b64 import _DEC, SKIP, b64get, xmlrpc_text  # noqa: E402

JUNK = np.array([c for c in range(256) if _DEC[c] == SKIP], dtype=np.uint8)


def perturb(rng, t):
    t = bytearray(t)
    kind = int(rng.integers(0, 10))
    if kind == 0 or not t:
        pass
    elif kind == 1:
        for _ in range(int(rng.integers(1, 6))):
            t.insert(int(rng.integers(0, len(t) + 1)), int(rng.choice(JUNK)))
    elif kind == 2:
        t.insert(int(rng.integers(0, len(t) + 1)), ord("="))
    elif kind == 3:
        del t[int(rng.integers(0, len(t)))]
    elif kind == 4:
        t = t[:int(rng.integers(0, len(t) + 1))]
    elif kind == 5:
        j = int(rng.integers(0, len(t)))
        if _DEC[t[j]] < 64:
            t[j] = ord("A") if t[j] != ord("A") else ord("B")
    elif kind == 6:
        t[int(rng.integers(0, len(t)))] = ord("=")
    elif kind == 7:
        t[int(rng.integers(0, len(t)))] = int(rng.choice(JUNK))
    elif kind == 8 and b" " in t:
        seps = [j for j, c in enumerate(t) if c == ord(" ")]
        t[seps[int(rng.integers(0, len(seps)))]] = ord("Q")
    return bytes(t), kind


def one_case(h, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 65))
    big = rng.random() < 0.2
    sizes = [int(rng.integers(0, 300 * 1024 if big and k % 8 == 0 else 4096)) for k in range(n)]
    datas = [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]
    texts, kinds = zip(*[perturb(rng, xmlrpc_text(d)) for d in datas])
    align = int(rng.choice([1, 4, 16]))
    toffs, pos, buf = [], int(rng.integers(0, 16)), bytearray()
    buf += b"\0" * pos
    for t in texts:
        pad = (-pos) % align
        buf += b"\0" * pad
        pos += pad
        toffs.append(pos)
        buf += t
        pos += len(t)
    text = np.frombuffer(bytes(buf) + b"\0", dtype=np.uint8)
    exp = np.frombuffer(b"".join(hashlib.sha1(d).digest() for d in datas), dtype=np.uint8).reshape(-1, 20)
    ooff = np.zeros(n, dtype=np.uint64)
    o = int(rng.integers(0, 16))
    for k, s in enumerate(sizes):
        ooff[k] = o
        o += s + int(rng.integers(0, 20))
    out = np.zeros(o + 1, dtype=np.uint8)
    ver, dec = h.verify_b64(text, toffs, [len(t) for t in texts], sizes, exp, out, ooff)
    for k in range(n):
        w = b64get(texts[k])
        cap = sizes[k]
        want_len = len(w) if len(w) <= cap else cap + 1
        got = out[int(ooff[k]):int(ooff[k]) + min(len(w), cap)].tobytes()
        if int(dec[k]) != want_len or got != w[:cap] or bool(ver[k]) != (w == datas[k]):
            return {"chunk": k, "kind": kinds[k], "size": cap, "text_len": len(texts[k]), "got_len": int(dec[k]),
                    "want_len": want_len, "verdict": bool(ver[k])}
    # the sender's side over the same chunks (a few expected digests wrong)
    bad = rng.random(n) < 0.1
    exp2 = exp.copy()
    exp2[bad, 0] ^= 1
    data = np.frombuffer(b"".join(datas) + b"\0", dtype=np.uint8)
    offs = np.cumsum([0] + sizes[:-1]).astype(np.uint64)
    v2, enc = h.verify_encode_b64(data, offs, sizes, exp2)
    for k in range(n):
        want = xmlrpc_text(datas[k])
        if enc[k] != want or bool(v2[k]) == bool(bad[k]):
            first = next((j for j in range(min(len(want), len(enc[k]))) if enc[k][j] != want[j]), None)
            return {"chunk": k, "side": "encode", "size": sizes[k], "n": n, "text_len": len(want),
                    "got_len": len(enc[k]), "first_diff": first,
                    "got": enc[k][first - 8:first + 24].decode("latin1") if first is not None else None,
                    "want": want[first - 8:first + 24].decode("latin1") if first is not None else None,
                    "verdict": bool(v2[k]), "expected_bad": bool(bad[k])}
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=90)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cases", type=int, default=0)
    a = ap.parse_args()
    t0, cases, chunks = time.time(), 0, 0
    with ChunkHasher(device_mask=1) as h:
        seed = a.seed
        while (a.cases and cases < a.cases) or (not a.cases and time.time() - t0 < a.seconds):
            bad = one_case(h, seed)
            if bad:
                print(json.dumps({"all_ok": False, "seed": seed, **bad}), flush=True)
                sys.exit(1)
            cases += 1
            seed += 1
            if cases % 50 == 0:
                print(f"{cases} cases ok ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
    print(json.dumps({"all_ok": True, "cases": cases, "first_seed": a.seed, "seconds": round(time.time() - t0, 1)}))


if __name__ == "__main__":
    main()
