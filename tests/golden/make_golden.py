#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

The expected digests come from Python's hashlib.sha1 + base64 -- an SHA-1
implementation independent of both the reference (Crypto++ 5.2.1) and of this
repo's oracle/ restatement.  The reference itself could not be built or run
(SURVEY.md §8c), so these fixtures plus the Crypto++ known-answer tests
(cpp/extern/crypto++/5.2.1/TestVectors/sha.txt:1-11) are what pin parity.

Synthetic inputs use the counter-mode splitmix64 stream defined in
oracle/sha1_oracle.c (oracle_synth_word) and in the device fill kernel; small
streams are generated here with numpy, the 4 GiB C2 stream with the oracle's
C filler (cross-checked against numpy on a prefix before use).

Run:  python tests/golden/make_golden.py          (takes ~1 minute)
      python tests/golden/make_golden.py --ranks  (c2_ranks.json: the 8 weak-scaled C2 shards, ~5 minutes)
      python tests/golden/make_golden.py --big    (c3.json, c4.json: 64 GiB + 256 GiB, ~1 hour)
"""
import base64
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

M64 = (1 << 64) - 1
G = 0x9E3779B97F4A7C15
SEED_MUL = 0xD1B54A32D192ED03
SEED_C = 0x5EED


def b64_27(digest: bytes) -> str:
    # BaseN_Encoder(alphabet, 6) without padding == standard base64 minus '='
    # (cpp/extern/crypto++/5.2.1/basecode.cpp:39-104, cpp/src/Encoder.cpp:104-120)
    s = base64.b64encode(digest).decode().rstrip("=")
    assert len(s) == 27
    return s


def synth_np(seed: int, start: int, length: int) -> bytes:
    """numpy restatement of oracle_synth_fill (little-endian u64 words)."""
    if length == 0:
        return b""
    w0 = start >> 3
    w1 = (start + length + 7) >> 3
    k = np.arange(w0, w1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64((seed * SEED_MUL) & M64) + (k + np.uint64(1)) * np.uint64(G)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    raw = z.astype("<u8").tobytes()
    off = start - (w0 << 3)
    return raw[off:off + length]


def load_oracle():
    path = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not os.path.exists(path):
        os.system(f"make -s -C {os.path.join(ROOT, 'oracle')}")
    lib = ctypes.CDLL(path)
    lib.oracle_synth_fill_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_int]
    return lib


def synth_c(lib, seed, start, length):
    buf = np.empty(length, dtype=np.uint8)
    lib.oracle_synth_fill_mt(buf.ctypes.data, length, seed, start, os.cpu_count() or 1)
    return buf


def chunk_digests(data, chunk_size):
    n = (len(data) + chunk_size - 1) // chunk_size
    out = []
    mv = memoryview(data)
    for i in range(n):
        out.append(hashlib.sha1(mv[i * chunk_size:(i + 1) * chunk_size]).digest())
    return out


def stream_digests(lib, seed, start, size, cs, slab=256 << 20, workers=None):
    """Raw SHA-1 digests of every cs-byte chunk of stream `seed` bytes
    [start, start+size), slab-parallel (ctypes and hashlib release the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    assert slab % cs == 0 and size % cs == 0

    def one(s0):
        ln = min(slab, size - s0)
        buf = np.empty(ln, dtype=np.uint8)
        lib.oracle_synth_fill_mt(buf.ctypes.data, ln, seed, start + s0, 1)
        mv = memoryview(buf)
        return [hashlib.sha1(mv[j:j + cs]).digest() for j in range(0, ln, cs)]

    with ThreadPoolExecutor(max_workers=workers or os.cpu_count() or 1) as ex:
        parts = list(ex.map(one, range(0, size, slab)))
    return [d for part in parts for d in part]


def dod(digests):
    h = hashlib.sha1()
    for d in digests:
        h.update(d)
    return h.hexdigest()


def big(lib):
    """C3 and C4 at full size: digest-of-digests per file /
    per 8-GPU shard plus sampled chunk strings."""
    gib = 1 << 30
    cs = 262144
    files, allh = [], hashlib.sha1()
    for f in range(64):
        d = stream_digests(lib, f, 0, gib, cs)
        for x in d:
            allh.update(x)
        files.append({"seed": f, "n_chunks": len(d), "sha1_of_concat_raw_digests_hex": dod(d),
                      "first_b64": b64_27(d[0]), "last_b64": b64_27(d[-1])})
        print(f"  C3 file {f}", end="\r", file=sys.stderr)
    write("c3.json", {
        "config": "C3: 64 files x 1 GiB (file f = stream seed f from byte 0), 256 KiB chunks",
        "file_size": gib, "chunk_size": cs, "files": files,
        "sha1_of_all_digests_in_file_order_hex": allh.hexdigest(),
    })
    cs = 1 << 20
    shard = 32 * gib
    shards = []
    for r in range(8):
        d = stream_digests(lib, SEED_C, r * shard, shard, cs)
        shards.append({"rank": r, "first_chunk": r * (shard // cs), "n_chunks": len(d),
                       "sha1_of_concat_raw_digests_hex": dod(d),
                       "samples_b64": {str(i): b64_27(d[i]) for i in (0, 1, 12345, len(d) - 1)}})
        print(f"  C4 shard {r}", end="\r", file=sys.stderr)
    write("c4.json", {
        "config": "C4: one 256 GiB file (stream seed 0x5EED), 1 MiB chunks, 8 contiguous shards of 32 GiB",
        "seed": SEED_C, "size": 8 * shard, "chunk_size": cs, "shards": shards,
    })


def ranks(lib, world=8):
    """The weak-scaled C2 stream bench.py hashes at N GPUs: rank r hashes bytes
    [r*4 GiB, (r+1)*4 GiB) of stream 0x5EED at 256 KiB chunks, for r < world.
    Rank 0 is C2 itself (cross-checked against c2.json)."""
    size, cs = 4 << 30, 262144
    out = []
    for r in range(world):
        d = stream_digests(lib, SEED_C, r * size, size, cs)
        out.append({"rank": r, "first_chunk": r * (size // cs), "n_chunks": len(d),
                    "sha1_of_concat_raw_digests_hex": dod(d),
                    "samples_b64": {str(i): b64_27(d[i]) for i in (0, 1, 8191, len(d) - 1)}})
        print(f"  C2 rank {r}", end="\r", file=sys.stderr)
    with open(os.path.join(HERE, "c2.json")) as f:
        assert json.load(f)["sha1_of_concat_raw_digests_hex"] == out[0]["sha1_of_concat_raw_digests_hex"]
    write("c2_ranks.json", {
        "config": "bench.py weak scaling: rank r hashes bytes [r*4GiB,(r+1)*4GiB) of stream 0x5EED, 256 KiB chunks",
        "seed": SEED_C, "bytes_per_rank": size, "chunk_size": cs, "ranks": out,
    })


def write(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", name)


def main():
    lib = load_oracle()

    # -- 1. known-answer tests ------------------------------------------------
    kats = []
    msgs = [
        ("empty", b""),
        ("abc", b"abc"),  # sha.txt:3-4
        ("nist448", b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"),  # sha.txt:6-7
        ("a_x_1e6", b"a" * 1000000),  # sha.txt:9-10 (r15625 x 64 'a')
        ("zeros_256KiB", bytes(262144)),
        ("zeros_64KiB", bytes(65536)),
    ]
    for name, m in msgs:
        d = hashlib.sha1(m).digest()
        kats.append({"name": name, "hex": d.hex(), "b64_27": b64_27(d),
                     "len": len(m), "fill": (m[:1].decode() if m else ""),
                     "text": (m.decode() if len(m) <= 64 else None)})
    write("kat.json", {"source": "hashlib; hex column equals Crypto++ KATs sha.txt:1-11",
                       "kats": kats})

    # -- 2. synthetic stream cross-check (numpy vs oracle C) ------------------
    for seed, start, ln in [(SEED_C, 0, 4096), (7, 13, 1000), (123456789, 1 << 33, 777)]:
        a = synth_np(seed, start, ln)
        b = synth_c(lib, seed, start, ln).tobytes()
        assert a == b, ("synth mismatch", seed, start, ln)
    stream_probe = {"seed": SEED_C, "first32_hex": synth_np(SEED_C, 0, 32).hex(),
                    "at_1GiB_hex": synth_np(SEED_C, 1 << 30, 32).hex(),
                    "seed7_off13_hex": synth_np(7, 13, 19).hex()}

    # -- 3. tails: last chunk sizes 1,55,56,63,64,65 and sub-block chunk sizes --
    tails = []
    for tail in [1, 55, 56, 63, 64, 65, 119, 120, 127, 128]:
        cs = 4096
        size = 3 * cs + tail
        seed = 1000 + tail
        data = synth_np(seed, 0, size)
        tails.append({"seed": seed, "size": size, "chunk_size": cs,
                      "b64": [b64_27(d) for d in chunk_digests(data, cs)]})
    for cs in [1, 55, 56, 57, 63, 64, 65, 100]:
        seed = 2000 + cs
        size = 5 * cs + (cs // 3)
        data = synth_np(seed, 0, size)
        tails.append({"seed": seed, "size": size, "chunk_size": cs,
                      "b64": [b64_27(d) for d in chunk_digests(data, cs)]})

    # -- 4. ragged batch over one buffer: random offsets (misaligned) / sizes --
    rng = np.random.default_rng(20041015)
    buf_len = 4 << 20
    buf = synth_np(7, 0, buf_len)
    specials = [0, 1, 2, 3, 4, 5, 54, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129,
                4095, 4096, 4097, 65535, 65536, 65537, 262143, 262144]
    sizes = specials + [int(s) for s in rng.integers(0, 300000, size=64 - len(specials))]
    offsets = []
    for i, s in enumerate(sizes):
        if i % 3 == 0:
            o = int(rng.integers(0, (buf_len - s) // 64)) * 64  # 64-B aligned
        else:
            o = int(rng.integers(0, buf_len - s + 1))  # anywhere
        offsets.append(o)
    ragged = {"seed": 7, "buf_len": buf_len, "offsets": offsets, "sizes": sizes,
              "hex": [hashlib.sha1(buf[o:o + s]).hexdigest() for o, s in zip(offsets, sizes)]}

    write("synthetic.json", {"stream_probe": stream_probe, "tails": tails, "ragged": ragged})

    # -- 5. C1: one 16 MiB file, 64 KiB chunks (256 digests, full list) ------
    c1 = synth_np(SEED_C, 0, 16 << 20)
    c1d = chunk_digests(c1, 65536)
    odd = synth_np(SEED_C + 1, 0, (16 << 20) + 12345)
    oddd = chunk_digests(odd, 262144)
    write("c1.json", {
        "config": "C1: one 16 MiB file (seed 0x5EED), 64 KiB chunks",
        "seed": SEED_C, "size": 16 << 20, "chunk_size": 65536,
        "b64": [b64_27(d) for d in c1d],
        "odd_tail": {"seed": SEED_C + 1, "size": (16 << 20) + 12345, "chunk_size": 262144,
                     "b64": [b64_27(d) for d in oddd]},
    })

    # -- 6. C2: one 4 GiB file, 256 KiB chunks: samples + digest of digests --
    size = 4 << 30
    cs = 262144
    n = size // cs
    slab = 256 << 20
    h = hashlib.sha1()
    sample_idx = [0, 1, 2, 3, 63, 64, 1000, 4095, 4096, 8191, 8192, 12345, 16382, 16383]
    samples = {}
    chk = synth_c(lib, SEED_C, 0, 4096).tobytes()
    assert chk == synth_np(SEED_C, 0, 4096)
    for s0 in range(0, size, slab):
        data = synth_c(lib, SEED_C, s0, slab)
        mv = memoryview(data)
        for j in range(slab // cs):
            d = hashlib.sha1(mv[j * cs:(j + 1) * cs]).digest()
            h.update(d)
            gi = s0 // cs + j
            if gi in sample_idx:
                samples[str(gi)] = b64_27(d)
        print(f"  C2 {s0 >> 20} MiB", end="\r", file=sys.stderr)
    write("c2.json", {
        "config": "C2: one 4 GiB file (seed 0x5EED), 256 KiB chunks",
        "seed": SEED_C, "size": size, "chunk_size": cs, "n_chunks": n,
        "samples_b64": samples,
        "sha1_of_concat_raw_digests_hex": h.hexdigest(),
    })


if __name__ == "__main__":
    if "--big" in sys.argv:
        big(load_oracle())
    elif "--ranks" in sys.argv:
        ranks(load_oracle())
    else:
        main()
