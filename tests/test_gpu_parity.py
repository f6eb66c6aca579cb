"""Parity of the MI355X chunk-hash kernels against the oracle and the golden fixtures.

Bit-exact: SHA-1 digests are integer/byte results, so every comparison is
equality.  Small cases go through the oracle (oracle/sha1_oracle.c) on the same
seeded bytes; full-size C2 (4 GiB at 256 KiB chunks) is checked through
size-independent properties against hashlib goldens: the SHA-1 of the 16,384
concatenated raw digests, sampled chunk strings, and a verify round trip.
"""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

from bitflood_amd import ChunkHasher, DeviceBuffer, b64_27, chunk_table
from bitflood_amd import hashing as H

pytestmark = pytest.mark.gpu
SEED_C = 0x5EED

# the shipped kernel variants (bitflood_amd/csrc/sha1_kernels.hip): 1 = one chunk
# per lane ("lane", the simple baseline), 7 = one consumer + two producer waves
# per 64 chains with the W+K schedule double-buffered in registers as 8-byte
# pairs ("pc4b64", <= 16 K chains), 10 = two consumer/producer pairs per CU
# with the round constants split and words 0..15 from the raw block ("pcx5",
# 16-32 K chains until round 3), 11 = one chunk per lane with LDS-DMA staging
# of whole 128-byte lines ("lds2", many chains), 12 = two pc4 groups in one
# 6-wave workgroup, producers two to a SIMD ("pc4x2", 16-32 K chains since
# round 3).  The superseded variants live only in the A/B library of
# tools/experimental/ (make -C tools/experimental).
VARIANTS = [1, 7, 10, 11, 12]


@pytest.fixture(params=VARIANTS, ids=lambda v: {1: "lane", 7: "pc4b64", 10: "pcx5", 11: "lds2", 12: "pc4x2"}[v])
def variant(request):
    H.set_kernel_variant(request.param)
    yield request.param
    H.set_kernel_variant(0)


def _kat_message(k):
    if k["text"] is not None:
        return k["text"].encode()
    if k["name"] == "a_x_1e6":
        return b"a" * k["len"]
    return bytes(k["len"])


def test_kats(variant, hasher, golden):
    for k in golden("kat.json")["kats"]:
        m = _kat_message(k)
        assert hasher.sha1(m).hex() == k["hex"], k["name"]
        assert hasher.base64_encode(m) == k["b64_27"], k["name"]


def test_hmac_sha1_kats_through_batches(variant, hasher):
    """Crypto++'s HMAC(SHA-1) known answers (TestVectors/hmac.txt) as three
    batched SHA-1 passes on the GPU: each message of a stage packed back to
    back in one buffer at its natural, unaligned offset."""
    from tests.test_oracle import hmac_sha1_cases

    def sha1_many(msgs):
        if not msgs:
            return []
        buf = np.frombuffer(b"".join(msgs), dtype=np.uint8)
        sizes = np.array([len(m) for m in msgs], dtype=np.uint32)
        offs = np.concatenate([[0], np.cumsum(sizes[:-1], dtype=np.uint64)]).astype(np.uint64)
        return list(hasher.hash_chunks(buf, offs, sizes))

    for name, got, want in hmac_sha1_cases(sha1_many):
        assert got == want, name


def test_tails(variant, hasher, oracle, golden):
    for t in golden("synthetic.json")["tails"]:
        data = oracle.synth(t["seed"], 0, t["size"])
        assert hasher.encode_buffer(data, t["chunk_size"]) == t["b64"], (t["size"], t["chunk_size"])


def test_ragged_misaligned(variant, hasher, oracle, golden):
    r = golden("synthetic.json")["ragged"]
    buf = oracle.synth(r["seed"], 0, r["buf_len"])
    got = hasher.hash_chunks(buf, r["offsets"], r["sizes"])
    assert [bytes(d).hex() for d in got] == r["hex"]


def test_random_batch_vs_oracle(variant, hasher, oracle):
    rng = np.random.default_rng(11)
    buf = oracle.synth(12, 0, 24 << 20)
    n = 3000
    sizes = rng.integers(0, 70000, n).astype(np.uint32)
    sizes[:40] = np.arange(40) * 3  # tiny, every residue class around 0..117
    offs = np.array([rng.integers(0, buf.size - s + 1) for s in sizes], dtype=np.uint64)
    offs[::2] &= ~np.uint64(63)  # half aligned, half anywhere
    got = hasher.hash_chunks(buf, offs, sizes)
    want = oracle.sha1_batch(buf, offs, sizes, nthreads=os.cpu_count() or 1)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]} sizes {sizes[bad[:5]]}"


@pytest.mark.parametrize("n", [1, 2, 63, 65, 127, 129])
def test_partial_waves_hash_and_verify(variant, hasher, oracle, n):
    """Waves with idle lanes (n not a multiple of 64): those lanes run a copy of
    their wave's first chain and write nothing (kern_common.hpp chain_info).
    The first chain of each wave is made the longest, or unaligned, so that a
    copy that leaked into a result or outlived the real chains would show."""
    rng = np.random.default_rng(1000 + n)
    buf = oracle.synth(31, 0, 4 << 20)
    sizes = rng.integers(0, 150000, n).astype(np.uint32)
    offs = np.array([rng.integers(0, buf.size - s + 1) for s in sizes], dtype=np.uint64) & ~np.uint64(15)
    for w0 in range(0, n, 64):
        sizes[w0] = 200000 + w0
        offs[w0] = 4096 * (w0 // 64) + (w0 // 64) % 2 * 5  # odd waves: first chain unaligned
    want = oracle.sha1_batch(buf, offs, sizes)
    got = hasher.hash_chunks(buf, offs, sizes)
    assert np.array_equal(got, want)
    exp = want.copy()
    exp[-1, 7] ^= 0x10
    v = hasher.verify_chunks(buf, offs, sizes, exp)
    assert v[:-1].all() and not v[-1]


@pytest.mark.parametrize("long_group", [0, 1])
def test_groups_of_one_workgroup_with_different_step_counts(variant, hasher, oracle, long_group):
    """Chains 0..63 and 64..127 share a workgroup in pc4x2 (12) and pcx5 (10):
    one group's chains a few blocks long, the other's thousands.  Every wave of
    the workgroup passes the longer group's barriers; the short group's chains
    must still end at their own last block."""
    rng = np.random.default_rng(77 + long_group)
    buf = oracle.synth(37, 0, 8 << 20)
    n = 256  # two pc4x2 workgroups
    sizes = rng.integers(0, 300, n).astype(np.uint32)
    for w in range(0, n, 128):
        lo = w + 64 * long_group
        sizes[lo:lo + 64] = rng.integers(200000, 260000, 64)
    offs = np.array([rng.integers(0, buf.size - s + 1) for s in sizes], dtype=np.uint64)
    want = oracle.sha1_batch(buf, offs, sizes)
    assert np.array_equal(hasher.hash_chunks(buf, offs, sizes), want)
    v = hasher.verify_chunks(buf, offs, sizes, want)
    assert v.all()


def test_empty_inputs(variant, hasher):
    assert hasher.sha1(b"").hex() == "da39a3ee5e6b4b0d3255bfef95601890afd80709"
    out = hasher.hash_chunks(np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32))
    assert out.shape == (0, 20)
    # zero-size chunk anywhere in a batch
    d = hasher.hash_chunks(np.arange(100, dtype=np.uint8), [0, 100, 5], [0, 0, 1])
    assert bytes(d[0]) == bytes(d[1]) == hashlib.sha1(b"").digest()
    assert bytes(d[2]) == hashlib.sha1(bytes([5])).digest()


def test_c1(variant, hasher, oracle, golden):
    c1 = golden("c1.json")
    data = oracle.synth(c1["seed"], 0, c1["size"])
    assert hasher.encode_buffer(data, c1["chunk_size"]) == c1["b64"]
    o = c1["odd_tail"]
    data = oracle.synth(o["seed"], 0, o["size"])
    assert hasher.encode_buffer(data, o["chunk_size"]) == o["b64"]


def test_verify_round_trip(variant, hasher, oracle):
    data = oracle.synth(21, 0, 8 << 20)
    offs, sizes = chunk_table(data.size, 65536)
    exp = hasher.hash_chunks(data, offs, sizes)
    assert hasher.verify_chunks(data, offs, sizes, exp).all()
    bad_data = data.copy()
    for idx in [0, 17, 127]:
        bad_data[idx * 65536 + 1000] ^= 0x40
    v = hasher.verify_chunks(bad_data, offs, sizes, exp)
    assert np.nonzero(~v)[0].tolist() == [0, 17, 127]
    exp2 = exp.copy()
    exp2[5, 19] ^= 1
    v = hasher.verify_chunks(data, offs, sizes, exp2)
    assert np.nonzero(~v)[0].tolist() == [5]


def test_small_slots_and_oversize_chunks(variant, oracle, monkeypatch):
    """Force many staging groups (1 MiB slots) and the oversize-chunk path."""
    with monkeypatch.context() as m:  # read at context creation only
        m.setenv("LBF_SLOT_MB", "1")
        h = ChunkHasher()
    try:
        data = oracle.synth(31, 0, 9 << 20)
        offs = np.array([0, 3, 1 << 20, (1 << 20) + 7, 5 << 20, 100], dtype=np.uint64)
        sizes = np.array([1 << 20, (1 << 20) - 3, (3 << 20) + 5, 65, 4 << 20, 1], dtype=np.uint32)
        got = h.hash_chunks(data, offs, sizes)
        want = oracle.sha1_batch(data, offs, sizes)
        assert np.array_equal(got, want)
        offs, sizes = chunk_table(data.size, 300001)
        assert np.array_equal(h.hash_chunks(data, offs, sizes), oracle.sha1_batch(data, offs, sizes))
    finally:
        h.close()


@pytest.mark.parametrize("slots", ["2", "3", "5"])
def test_staging_slot_counts(slots, oracle, monkeypatch):
    """LBF_SLOTS round-robin staging: a 200 MiB job is split into quarter-span
    groups (>= 32 MiB each), so every slot is reused; ragged and unaligned
    chunks straddle the group edges.  Hash and verify both match the oracle."""
    with monkeypatch.context() as m:
        m.setenv("LBF_SLOTS", slots)
        h = ChunkHasher(device_mask=1)
    try:
        data = oracle.synth(47, 0, 200 << 20, nthreads=8)
        offs, sizes = chunk_table(data.size - 5, 262144 + 13)
        offs = offs + np.uint64(5)
        want = oracle.sha1_batch(data, offs, sizes, nthreads=8)
        assert np.array_equal(h.hash_chunks(data, offs, sizes), want)
        bad = data.copy()
        flipped = [0, len(sizes) // 2, len(sizes) - 1]
        for i in flipped:
            bad[int(offs[i]) + int(sizes[i]) - 1] ^= 0x01
        v = h.verify_chunks(bad, offs, sizes, want)
        assert np.nonzero(~v)[0].tolist() == flipped
    finally:
        h.close()


def test_device_fill_matches_oracle_stream(oracle):
    buf = DeviceBuffer(1 << 20)
    try:
        buf.fill_synthetic(SEED_C, start=1 << 30)
        got = buf.download()
        assert np.array_equal(got, oracle.synth(SEED_C, 1 << 30, 1 << 20))
        buf.fill_synthetic(7, start=16, nbytes=1001)
        got = buf.download(1001)
        assert np.array_equal(got, oracle.synth(7, 16, 1001))
    finally:
        buf.free()


def test_device_ptr_batch(variant, hasher, oracle):
    from bitflood_amd import _capi
    data = oracle.synth(41, 0, 1 << 20)
    offs = np.array([0, 64, 129, 4096, 70000], dtype=np.uint64)
    sizes = np.array([64, 65, 1000, 60000, 300000], dtype=np.uint32)
    d_data, d_off, d_size, d_out = (DeviceBuffer(data.size), DeviceBuffer(40), DeviceBuffer(20),
                                    DeviceBuffer(100))
    try:
        d_data.upload(data)
        d_off.upload(offs)
        d_size.upload(sizes)
        _capi.check(_capi.load().lbf_sha1_batch(hasher._h, d_data.ptr, data.size, d_off.ptr, d_size.ptr, 5,
                                                d_out.ptr, _capi.LBF_DEVICE_PTR))
        got = d_out.download(100).reshape(5, 20)
        assert np.array_equal(got, oracle.sha1_batch(data, offs, sizes))
    finally:
        for b in (d_data, d_off, d_size, d_out):
            b.free()


@pytest.mark.parametrize("n", [20000, 20064])
def test_uniform_ragged_chain_count_between_16k_and_32k(variant, oracle, n):
    """Chain counts where the automatic choice is pc4x2, with a short last
    chunk.  pc4x2 takes 128 chains per workgroup, two groups of 64.  At 20,000
    = 156 x 128 + 32 the last workgroup's group 0 has 32 chains and group 1
    none; at 20,064 = 156 x 128 + 96 group 0 is full and group 1 has 32
    (ADVICE r03).  Device-resident, every digest against the oracle."""
    cs = 4096
    n_bytes = (n - 1) * cs + 1000
    buf = DeviceBuffer(n_bytes)
    dig = DeviceBuffer(n * 20)
    try:
        buf.fill_synthetic(91)
        H.uniform_launch(buf, n_bytes, cs, 0, n, dig)
        H.synchronize()
        got = dig.download(n * 20).reshape(n, 20)
        want = oracle.encode_buffer(oracle.synth(91, 0, n_bytes), cs)
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"
    finally:
        buf.free()
        dig.free()


def test_uniform_partial_last_chunk(variant, oracle):
    n_bytes = (5 << 20) + 12345
    buf = DeviceBuffer(n_bytes)
    dig = DeviceBuffer(21 * 20)
    try:
        buf.fill_synthetic(77)
        n = (n_bytes + 262143) // 262144
        H.uniform_launch(buf, n_bytes, 262144, 0, n, dig)
        H.synchronize()
        got = dig.download(n * 20).reshape(n, 20)
        want = oracle.encode_buffer(oracle.synth(77, 0, n_bytes), 262144)
        assert np.array_equal(got, want)
        # sub-range launch (first_chunk > 0) as a sharded rank would issue it
        H.uniform_launch(buf, n_bytes, 262144, 7, n - 7, dig)
        H.synchronize()
        assert np.array_equal(dig.download((n - 7) * 20).reshape(n - 7, 20), want[7:])
    finally:
        buf.free()
        dig.free()


def test_c2_full_size_device_resident(variant, golden, oracle):
    """C2: one 4 GiB file, 256 KiB chunks, entirely in HBM."""
    c2 = golden("c2.json")
    size, cs, n = c2["size"], c2["chunk_size"], c2["n_chunks"]
    buf = DeviceBuffer(size)
    dig = DeviceBuffer(n * 20)
    ver = DeviceBuffer(n)
    try:
        buf.fill_synthetic(c2["seed"])
        H.uniform_launch(buf, size, cs, 0, n, dig)
        H.synchronize()
        d = dig.download(n * 20).reshape(n, 20)
        assert hashlib.sha1(d.tobytes()).hexdigest() == c2["sha1_of_concat_raw_digests_hex"]
        for k, v in c2["samples_b64"].items():
            assert b64_27(bytes(d[int(k)])) == v
        # spot-check against the oracle on device-generated bytes
        for i in [5, 9000]:
            chunk = buf.download(cs, offset=i * cs)
            assert oracle.sha1(chunk) == bytes(d[i])
        # verify mode against the just-computed digests: every verdict 1
        H.uniform_launch(buf, size, cs, 0, n, None, expected=dig, verdicts=ver)
        H.synchronize()
        assert ver.download(n).all()
    finally:
        buf.free()
        dig.free()
        ver.free()


def test_hash_and_verify_file(hasher, oracle, tmp_path):
    """lbf_file_ranges through the Python face: EncodeFile's fread loop
    (Encoder.cpp:54-72) and the resume verify (Flood.cpp:259-275) on a real file,
    including a truncated copy (short chunks verify False) and a missing file."""
    data = oracle.synth(31, 0, (9 << 20) + 777)
    path = tmp_path / "f.bin"
    path.write_bytes(data.tobytes())
    offs, sizes = chunk_table(data.size, 262144)
    want = oracle.sha1_batch(data, offs, sizes)
    got = hasher.hash_file(str(path), offs, sizes)
    assert np.array_equal(got, want)
    assert hasher.verify_file(str(path), offs, sizes, want).all()
    cut = 5 * 262144 + 100
    short = tmp_path / "short.bin"
    short.write_bytes(data[:cut].tobytes())
    v = hasher.verify_file(str(short), offs, sizes, want)
    assert v.tolist() == [True] * 5 + [False] * (offs.size - 5)
    assert not hasher.verify_file(str(tmp_path / "missing.bin"), offs, sizes, want).any()
    with pytest.raises(Exception):
        hasher.hash_file(str(short), offs, sizes)


@pytest.mark.parametrize("extra", [1, 2, 4095, 4097])
def test_staging_split_covers_tail(hasher, oracle, extra):
    """A staging group of 3 x 8 MiB + `extra` bytes is copied by 3 host threads;
    the split must cover the tail bytes (floor(len/3) is a page multiple for
    small `extra`, which once left the last bytes uncopied: hash mode failed with
    LBF_ERR_IO and verify mode returned false mismatches).  Found by
    tools/fuzz_gpu.py seed 23006099."""
    n = 3 * (8 << 20) + extra
    data = oracle.synth(57, 0, n)
    offs = np.array([0, n - 100, 5], dtype=np.uint64)
    sizes = np.array([n, 100, n - 5], dtype=np.uint32)
    want = oracle.sha1_batch(data, offs, sizes)
    assert np.array_equal(hasher.hash_chunks(data, offs, sizes), want)
    assert hasher.verify_chunks(data, offs, sizes, want).all()


def test_verify_file_empty_chunk_past_eof(hasher, tmp_path):
    """Flood.cpp:259-275: fseek past EOF succeeds and fread of 0 bytes returns 0,
    so an empty chunk past the end of an existing file verifies ('1'); with no file
    (fopen fails) nothing does."""
    path = tmp_path / "short.bin"
    path.write_bytes(b"x" * 1000)
    empty = hashlib.sha1(b"").digest()
    offs = np.array([0, 5000, 999], dtype=np.uint64)
    sizes = np.array([0, 0, 2], dtype=np.uint32)
    exp = np.frombuffer(empty * 3, np.uint8).reshape(3, 20)
    assert hasher.verify_file(str(path), offs, sizes, exp).tolist() == [True, True, False]
    assert not hasher.verify_file(str(tmp_path / "missing.bin"), offs, sizes, exp).any()


def test_chunk_over_512_mib_bit_length_high_word(oracle):
    """A chunk of 2^29 bytes or more has a non-zero high word of the 64-bit bit
    length in the final block (iterhash.h:30-31,106-121: GetBitCountHi); no
    configuration's chunk reaches that size, so pin it once on the device path."""
    n_bytes = (512 << 20) + 100
    buf = DeviceBuffer(n_bytes)
    dig = DeviceBuffer(20)
    try:
        buf.fill_synthetic(91)
        H.uniform_launch(buf, n_bytes, n_bytes, 0, 1, dig)
        H.synchronize()
        got = dig.download(20).tobytes()
    finally:
        buf.free()
        dig.free()
    assert got == hashlib.sha1(oracle.synth(91, 0, n_bytes, nthreads=8).tobytes()).digest()


def test_more_chunks_than_one_group_holds(hasher, oracle):
    """150,000 small chunks in one call: more than a staging group's 65,536
    descriptors, so the job spans several groups by count, not by bytes; sizes
    0..600 cover every padding case, offsets are unaligned; hash and verify."""
    rng = np.random.default_rng(150000)
    n = 150000
    sizes = rng.integers(0, 601, n).astype(np.uint32)
    buf = oracle.synth(67, 0, int(sizes.sum()) + 4096, nthreads=8)
    offs = np.concatenate([[0], np.cumsum(sizes[:-1], dtype=np.uint64)]).astype(np.uint64) + np.uint64(3)
    want = oracle.sha1_batch(buf, offs, sizes, nthreads=8)
    got = hasher.hash_chunks(buf, offs, sizes)
    bad = np.flatnonzero((got != want).any(axis=1))
    assert bad.size == 0, bad[:10]
    exp = want.copy()
    flips = [0, 65535, 65536, 131072, n - 1]
    exp[flips, 11] ^= 0x80
    assert np.flatnonzero(~hasher.verify_chunks(buf, offs, sizes, exp)).tolist() == flips


def test_unsorted_overlapping_duplicate_table(hasher, oracle):
    """The staging sorts descriptors by offset and packs them as joined runs
    (lbf_capi.cpp worker_run); results must land at the caller's indices:
    a descending table, exact duplicates, chunks nested in others, chunks far
    apart, and empty chunks anywhere, in hash and verify mode."""
    buf = oracle.synth(71, 0, 64 << 20, nthreads=8)
    rng = np.random.default_rng(71)
    offs = list(range((60 << 20), 0, -(3 << 20)))          # descending, 3 MiB apart
    sizes = [1 << 20] * len(offs)
    offs += [5, 5, 5 + 4096, 1000, 63 << 20]                   # duplicates, nested, far
    sizes += [70000, 70000, 100, 0, (1 << 20) - 1]
    offs += [int(x) for x in rng.integers(0, 60 << 20, 500)]  # random, overlapping
    sizes += [int(x) for x in rng.integers(0, 300000, 500)]
    offs = np.array(offs, dtype=np.uint64)
    sizes = np.array(sizes, dtype=np.uint32)
    want = oracle.sha1_batch(buf, offs, sizes, nthreads=8)
    assert np.array_equal(hasher.hash_chunks(buf, offs, sizes), want)
    exp = want.copy()
    flips = [0, 7, 21, 22, 300, len(offs) - 1]
    exp[flips, 19] ^= 1
    assert np.flatnonzero(~hasher.verify_chunks(buf, offs, sizes, exp)).tolist() == flips


def test_hash_and_verify_many_files_one_batch(hasher, oracle, tmp_path):
    """lbf_files_ranges: EncodeFile's and _SetupFilesAndChunks' loops over a
    flood's files (Encoder.cpp:40-79, Flood.cpp:239-287) as ONE batch.  40 files
    of assorted sizes (empty, sub-chunk, ragged tails), descriptors interleaved
    across files; verify with a truncated file, a missing file (all '0', its
    empty chunk too) and a flipped byte."""
    rng = np.random.default_rng(40)
    cs = 65536 + 13
    paths, datas = [], []
    for f in range(40):
        size = int(rng.choice([0, 1, 100, cs, 3 * cs + 7, int(rng.integers(0, 2 << 20))]))
        d = oracle.synth(500 + f, 0, size)
        p = tmp_path / f"f{f:02d}.bin"
        p.write_bytes(d.tobytes())
        paths.append(str(p))
        datas.append(d)
    file_of, offs, sizes = [], [], []
    for f, d in enumerate(datas):
        o, s = chunk_table(d.size, cs)
        if d.size == 0:  # an empty file still contributes an empty chunk here
            o, s = np.zeros(1, np.uint64), np.zeros(1, np.uint32)
        file_of += [f] * o.size
        offs += o.tolist()
        sizes += s.tolist()
    perm = rng.permutation(len(offs))  # interleave files and chunks
    file_of = np.array(file_of, np.uint32)[perm]
    offs = np.array(offs, np.uint64)[perm]
    sizes = np.array(sizes, np.uint32)[perm]
    want = np.stack([oracle.sha1(datas[f][o:o + s].tobytes()) if s else oracle.sha1(b"")
                     for f, o, s in zip(file_of, offs.astype(np.int64), sizes.astype(np.int64))]).view(np.uint8)
    want = want.reshape(-1, 20)
    assert np.array_equal(hasher.hash_files(paths, file_of, offs, sizes), want)
    assert hasher.verify_files(paths, file_of, offs, sizes, want).all()
    # damage: file 3 truncated to half, file 7 missing, one byte of file 11 flipped
    big = [f for f in range(40) if datas[f].size > 2 * cs][:3]
    t, m, x = big
    cut = datas[t].size // 2
    open(paths[t], "wb").write(datas[t][:cut].tobytes())
    import os as _os
    _os.remove(paths[m])
    bad = datas[x].copy()
    bad[cs + 5] ^= 1
    open(paths[x], "wb").write(bad.tobytes())
    v = hasher.verify_files(paths, file_of, offs, sizes, want)
    exp_v = np.ones(len(offs), bool)
    exp_v[(file_of == t) & (offs.astype(np.int64) + sizes > cut) & (sizes > 0)] = False
    exp_v[file_of == m] = False
    exp_v[(file_of == x) & (offs == np.uint64(cs))] = False
    assert np.array_equal(v, exp_v)
    with pytest.raises(Exception):
        hasher.hash_files(paths, file_of, offs, sizes)  # a missing file fails hash mode


def test_launch_refuses_device_arrays_too_small(hasher, oracle):
    """A device array the caller passes must fit its allocation: a launch that
    would write past a digest / verdict array (or read past the region or the
    chunk table) is refused before any kernel runs, since an out-of-bounds
    write is a GPU fault.  Arrays of exactly the right size are accepted."""
    from bitflood_amd import LbfError
    from bitflood_amd import _capi
    cs, n = 4096, 100
    buf, dig, small = DeviceBuffer(n * cs), DeviceBuffer(n * 20), DeviceBuffer(20 * 10)
    offs, sizes = DeviceBuffer(8 * n), DeviceBuffer(4 * (n - 1))
    try:
        buf.fill_synthetic(93)
        for call, what in [
                (lambda: H.uniform_launch(buf, n * cs, cs, 0, n, small), "digests"),
                (lambda: H.uniform_launch(buf.ptr + cs, n * cs, cs, 0, n, dig), "region"),
                (lambda: H.batch_launch(buf, offs, sizes, n, dig), "sizes"),
                (lambda: _capi.check(_capi.load().lbf_fill_synthetic(buf.ptr + 16, n * cs, 1, 0, None)),
                 "lbf_fill_synthetic")]:
            with pytest.raises(LbfError) as e:
                call()
            assert e.value.status == _capi.LBF_ERR_INVALID and what in str(e.value), str(e.value)
        # exact sizes pass, and the digests are right
        H.uniform_launch(buf, n * cs, cs, 0, n, dig)
        H.synchronize()
        want = oracle.encode_buffer(oracle.synth(93, 0, n * cs), cs)
        assert np.array_equal(dig.download(n * 20).reshape(n, 20), want)
    finally:
        for b in (buf, dig, small, offs, sizes):
            b.free()
