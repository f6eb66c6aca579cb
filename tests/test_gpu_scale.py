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


@pytest.fixture(params=[0, 1, 7, 10, 11], ids=["auto", "lane", "pc4b64", "pcx5", "lds2"])
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
    """Every 32 GiB shard of the 256 GiB C4 file (automatic kernel choice: pcx5
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
            for v in ([0, 1, 7, 11] if sh["rank"] == 5 else [0]):
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
