"""Full-size parity for the C3 and C4 configurations, entirely
in HBM, against the hashlib goldens of tests/golden/make_golden.py --big.

C3: 64 files x 1 GiB at 256 KiB chunks (file f = synthetic stream seed f).  The
files lie back to back in one 64 GiB buffer, so one uniform launch over it
produces exactly the per-file chunk sequence EncodeFile emits.
C4: one 256 GiB file at 1 MiB chunks, sharded 8 ways (32 GiB each); every shard
is generated and hashed on this one GPU in turn, i.e. what each of the 8 ranks
of the multi-GPU run computes.
"""
import hashlib

import numpy as np
import pytest

from bitflood_amd import DeviceBuffer, b64_27
from bitflood_amd import hashing as H

pytestmark = pytest.mark.gpu
GIB = 1 << 30


@pytest.fixture(params=[0, 1, 7, 10, 11, 12], ids=["auto", "lane", "pc4b64", "pcx5", "lds2", "pc4x2"])
def variant(request):
    H.set_kernel_variant(request.param)
    yield request.param
    H.set_kernel_variant(0)


@pytest.fixture(scope="module")
def c3_buffer(golden):
    c3 = golden("c3.json")
    fs = c3["file_size"]
    buf = DeviceBuffer(64 * fs)
    for f in c3["files"]:
        buf.fill_synthetic(f["seed"], start=0, nbytes=fs, offset=f["seed"] * fs)
    H.synchronize()
    yield c3, buf
    buf.free()


def test_c3_multi_file_flood(variant, c3_buffer):
    c3, buf = c3_buffer
    fs, cs = c3["file_size"], c3["chunk_size"]
    per = fs // cs
    n = 64 * per
    dig = DeviceBuffer(n * 20)
    try:
        H.uniform_launch(buf, 64 * fs, cs, 0, n, dig)
        H.synchronize()
        d = dig.download(n * 20).reshape(64, per, 20)
        assert hashlib.sha1(d.tobytes()).hexdigest() == c3["sha1_of_all_digests_in_file_order_hex"]
        for f in c3["files"]:
            k = f["seed"]
            assert hashlib.sha1(d[k].tobytes()).hexdigest() == f["sha1_of_concat_raw_digests_hex"], k
            assert b64_27(bytes(d[k, 0])) == f["first_b64"]
            assert b64_27(bytes(d[k, -1])) == f["last_b64"]
    finally:
        dig.free()


def test_c3_verify_flags_corruption(c3_buffer):
    """Verify mode at C3 scale: expected digests with a few flipped bytes give
    exactly those verdicts 0."""
    c3, buf = c3_buffer
    fs, cs = c3["file_size"], c3["chunk_size"]
    n = 64 * (fs // cs)
    dig, ver = DeviceBuffer(n * 20), DeviceBuffer(n)
    try:
        H.uniform_launch(buf, 64 * fs, cs, 0, n, dig)
        H.synchronize()
        exp = dig.download(n * 20).reshape(n, 20).copy()
        bad = np.array([0, 1, 4095, 4096, 131071, n - 1])
        exp[bad, 7] ^= 0x40
        dig.upload(exp.reshape(-1))
        H.uniform_launch(buf, 64 * fs, cs, 0, n, None, expected=dig, verdicts=ver)
        H.synchronize()
        v = ver.download(n)
        assert set(np.flatnonzero(v == 0).tolist()) == set(bad.tolist())
    finally:
        dig.free()
        ver.free()


def test_c4_all_shards(golden):
    """Every 32 GiB shard of the 256 GiB C4 file (automatic kernel choice: pc4x2
    at 32,768 chunks), plus one shard through the other kernels."""
    c4 = golden("c4.json")
    cs = c4["chunk_size"]
    shard_bytes = c4["size"] // 8
    buf = DeviceBuffer(shard_bytes)
    n = shard_bytes // cs
    dig = DeviceBuffer(n * 20)
    try:
        for sh in c4["shards"]:
            assert sh["n_chunks"] == n
            buf.fill_synthetic(c4["seed"], start=sh["first_chunk"] * cs)
            for v in ([0, 1, 7, 10, 11, 12] if sh["rank"] == 5 else [0]):
                H.set_kernel_variant(v)
                H.uniform_launch(buf, shard_bytes, cs, 0, n, dig)
                H.synchronize()
                d = dig.download(n * 20).reshape(n, 20)
                assert hashlib.sha1(d.tobytes()).hexdigest() == sh["sha1_of_concat_raw_digests_hex"], (sh["rank"], v)
                for k, s in sh["samples_b64"].items():
                    assert b64_27(bytes(d[int(k)])) == s
    finally:
        H.set_kernel_variant(0)
        buf.free()
        dig.free()


@pytest.mark.timeout(900)
def test_c3_encode_file_cli_64_files(golden, tmp_path):
    """C3 end to end through the C++ product path: lbf_encoder (test_encoder's
    port) with the 64 x 1 GiB files of c3.json on disk (or /dev/shm), i.e.
    Encoder::EncodeFile over 64 files (Encoder.cpp:17-102, batched over files),
    then the flood file's 262,144 chunk strings are checked against the hashlib
    goldens, and lbf_verify (Flood::SetupFilesAndChunks over the 64 files)
    finds every chunk present."""
    import base64
    import json
    import os
    import re
    import shutil
    import subprocess
    import tempfile
    c3 = golden("c3.json")
    fs = c3["file_size"]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "bitflood_amd", "lib")
    shm_free = shutil.disk_usage("/dev/shm").free if os.path.isdir("/dev/shm") else 0
    base = "/dev/shm" if shm_free > 80 * GIB else str(tmp_path)
    d = tempfile.mkdtemp(prefix="lbf_c3_", dir=base)
    try:
        buf = DeviceBuffer(fs)
        try:
            names = []
            for f in c3["files"]:
                buf.fill_synthetic(f["seed"], start=0)
                H.synchronize()
                name = f"f{f['seed']:02d}.bin"
                buf.download(fs).tofile(os.path.join(d, name))
                names.append(name)
        finally:
            buf.free()
        # twice: the first run is also the first read of the files just written, which the kernel serves at
        # ~14 GiB/s whoever reads (tools/c3_e2e_probe.py); the second is EncodeFile's own rate
        for run in ("first read", "pages read before"):
            out = subprocess.run([os.path.join(lib, "lbf_encoder"), *names, "http://127.0.0.1:10101/", "c3.flood",
                                  "--time"], cwd=d, capture_output=True, text=True, timeout=600)
            assert out.returncode == 0, out.stderr
            t = json.loads(out.stdout.strip().splitlines()[-1])
            print(f"C3 EncodeFile ({run}):", json.dumps(t), f"{t['bytes'] / GIB / t['encode_s']:.1f} GiB/s")
        xml = open(os.path.join(d, "c3.flood")).read()
        files = re.findall(r'<File name="([^"]+)" size="(\d+)">(.*?)</File>', xml, re.S)
        assert [n for n, _, _ in files] == sorted(names)
        allh = hashlib.sha1()
        for (name, size, body), f in zip(files, c3["files"]):
            assert int(size) == fs
            hashes = re.findall(r'<Chunk hash="([^"]+)" index="(\d+)" size="(\d+)" weight="0"/>', body)
            assert [int(i) for _, i, _ in hashes] == list(range(fs // c3["chunk_size"]))
            raw = b"".join(base64.b64decode(h + "=") for h, _, _ in hashes)
            allh.update(raw)
            assert hashlib.sha1(raw).hexdigest() == f["sha1_of_concat_raw_digests_hex"], name
            assert hashes[0][0] == f["first_b64"] and hashes[-1][0] == f["last_b64"]
        assert allh.hexdigest() == c3["sha1_of_all_digests_in_file_order_hex"]
        v = subprocess.run([os.path.join(lib, "lbf_verify"), "c3.flood", "--no-resolve"], cwd=d,
                           capture_output=True, text=True, timeout=600)
        assert v.returncode == 0, v.stderr
        lines = dict(line.split(" ", 1) for line in v.stdout.strip().splitlines())
        assert lines["to_download"] == "0"
        for n in names:
            assert lines[n].startswith("4096 4096 ")
    finally:
        shutil.rmtree(d, ignore_errors=True)
