"""Pin the CPU oracle (oracle/sha1_oracle.c) before trusting it as the checker.

Anchors: Crypto++ SHA-1 KATs (cpp/extern/crypto++/5.2.1/TestVectors/sha.txt:1-11)
and its HMAC(SHA-1) KATs (TestVectors/hmac.txt, two SHA-1 passes each),
hashlib-generated golden fixtures (tests/golden/make_golden.py), and for the
27-char rendering (basecode.cpp:39-104 without padding) Crypto++'s own expected
base64 output (validat1.cpp ValidateBaseCode, tests/golden/cryptopp521_base64.json)
plus Python's base64.
"""
import base64
import hashlib
import json
import os

import numpy as np
import pytest

SEED_C = 0x5EED
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _kat_message(k):
    if k["text"] is not None:
        return k["text"].encode()
    if k["name"] == "a_x_1e6":
        return b"a" * k["len"]
    return bytes(k["len"])


def test_kats(oracle, golden):
    for k in golden("kat.json")["kats"]:
        m = _kat_message(k)
        d = oracle.sha1(m)
        assert d.hex() == k["hex"], k["name"]
        assert oracle.base64_encode(m) == k["b64_27"], k["name"]


def test_crypto_pp_kat_hex_column(golden):
    # sha.txt:3-10 / validat3.cpp:171-176 digests, verbatim upper-case hex
    ref = {"abc": "A9993E364706816ABA3E25717850C26C9CD0D89D",
           "nist448": "84983E441C3BD26EBAAE4AA1F95129E5E54670F1",
           "a_x_1e6": "34AA973CD4C4DAA4F61EEB2BDBAD27316534016F"}
    got = {k["name"]: k["hex"].upper() for k in golden("kat.json")["kats"]}
    for name, hexd in ref.items():
        assert got[name] == hexd


def test_incremental_update_matches_one_shot(oracle):
    """iterhash.cpp:9-63 left-over handling: any split of Update calls gives the same digest."""
    rng = np.random.default_rng(1)
    for n in [0, 1, 55, 56, 63, 64, 65, 127, 128, 129, 1000, 4097]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        want = hashlib.sha1(data).digest()
        assert oracle.sha1(data) == want
        for _ in range(3):
            splits = sorted(rng.integers(0, n + 1, size=int(rng.integers(0, 6))).tolist())
            assert oracle.sha1_incremental(data, splits) == want


def _cryptopp_base64_stream():
    """Crypto++ 5.2.1's own expected Base64Encoder output for bytes 0..254
    (validat1.cpp, ValidateBaseCode; tests/golden/make_cryptopp_base64_fixture.py),
    line breaks removed."""
    with open(os.path.join(GOLDEN, "cryptopp521_base64.json")) as f:
        return json.load(f)["base64_with_linebreaks"].replace("\n", "")


def cryptopp_windows():
    """20-byte windows of bytes 0..254 whose 27-char rendering is a slice of
    Crypto++'s own expected output: the window must start on a 3-byte group
    (chars 4k..) and the byte after it must be < 64, so that the 27th char of
    the stream carries the window's last 4 bits followed by two zero bits, as
    the unpadded 27th char does (basecode.cpp:39-104)."""
    s = _cryptopp_base64_stream()
    return [(bytes(range(3 * k, 3 * k + 20)), s[4 * k:4 * k + 27]) for k in range(15) if 3 * k + 20 < 64]


def test_b64_27_restatement_matches_cryptopp_vector(oracle):
    w = cryptopp_windows()
    assert len(w) == 15
    for d, want in w:
        assert oracle.b64_27(d) == want
    # and the stream itself is what Python's codec gives for 0..254
    assert _cryptopp_base64_stream() == base64.b64encode(bytes(range(255))).decode()


def hmac_sha1_cases(sha1_many):
    """Crypto++'s HMAC(SHA-1) known answers (TestVectors/hmac.txt, RFC 2202;
    tests/golden/make_cryptopp_hmac_fixture.py) computed through `sha1_many`
    (list of messages -> list of 20-byte digests): SHA-1 of a long key, then
    SHA1((K ^ ipad) || m) and SHA1((K ^ opad) || inner), each stage one batch.
    Returns [(name, got, want)]."""
    with open(os.path.join(GOLDEN, "cryptopp521_hmac_sha1.json")) as f:
        cases = json.load(f)["cases"]
    keys = [bytes.fromhex(c["key"]) for c in cases]
    long_ = [i for i, k in enumerate(keys) if len(k) > 64]
    for i, d in zip(long_, sha1_many([keys[i] for i in long_])):
        keys[i] = bytes(d)
    keys = [k.ljust(64, b"\0") for k in keys]
    inner = sha1_many([bytes(b ^ 0x36 for b in k) + bytes.fromhex(c["message"]) for k, c in zip(keys, cases)])
    outer = sha1_many([bytes(b ^ 0x5C for b in k) + bytes(d) for k, d in zip(keys, inner)])
    return [(c["name"], bytes(o).hex(), c["digest"]) for c, o in zip(cases, outer)]


def test_oracle_reproduces_cryptopp_hmac_sha1_kats(oracle):
    got = hmac_sha1_cases(lambda ms: [oracle.sha1(m) for m in ms])
    assert len(got) == 7
    for name, g, want in got:
        assert g == want, name


def test_b64_27_restatement(oracle):
    rng = np.random.default_rng(2)
    for _ in range(200):
        d = rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
        want = base64.b64encode(d).decode().rstrip("=")
        assert oracle.b64_27(d) == want
        assert len(want) == 27


def test_synthetic_stream_probe(oracle, golden):
    sp = golden("synthetic.json")["stream_probe"]
    assert oracle.synth(SEED_C, 0, 32).tobytes().hex() == sp["first32_hex"]
    assert oracle.synth(SEED_C, 1 << 30, 32).tobytes().hex() == sp["at_1GiB_hex"]
    assert oracle.synth(7, 13, 19).tobytes().hex() == sp["seed7_off13_hex"]
    a = oracle.synth(99, 5, 100003, nthreads=1)
    b = oracle.synth(99, 5, 100003, nthreads=4)
    assert np.array_equal(a, b)


def test_tails_golden(oracle, golden):
    for t in golden("synthetic.json")["tails"]:
        data = oracle.synth(t["seed"], 0, t["size"])
        got = [oracle.b64_27(bytes(d)) for d in oracle.encode_buffer(data, t["chunk_size"])]
        assert got == t["b64"], (t["size"], t["chunk_size"])


def test_ragged_golden(oracle, golden):
    r = golden("synthetic.json")["ragged"]
    buf = oracle.synth(r["seed"], 0, r["buf_len"])
    got = oracle.sha1_batch(buf, r["offsets"], r["sizes"], nthreads=4)
    assert [bytes(d).hex() for d in got] == r["hex"]


def test_c1_golden(oracle, golden):
    c1 = golden("c1.json")
    data = oracle.synth(c1["seed"], 0, c1["size"])
    got = [oracle.b64_27(bytes(d)) for d in oracle.encode_buffer(data, c1["chunk_size"])]
    assert len(got) == 256
    assert got == c1["b64"]
    o = c1["odd_tail"]
    data = oracle.synth(o["seed"], 0, o["size"])
    got = [oracle.b64_27(bytes(d)) for d in oracle.encode_buffer(data, o["chunk_size"])]
    assert got == o["b64"]


def test_encode_file_fread_path(oracle, tmp_path):
    """Encoder.cpp:40-79 restated with fread: empty file -> 0 chunks, short tail kept."""
    p = tmp_path / "f.bin"
    data = oracle.synth(3, 0, 3 * 4096 + 17)
    p.write_bytes(data.tobytes())
    out = np.zeros((8, 20), dtype=np.uint8)
    sizes = np.zeros(8, dtype=np.uint32)
    n = oracle.lib.oracle_encode_file(str(p).encode(), 4096, out.ctypes.data, 8, sizes.ctypes.data)
    assert n == 4
    assert sizes[:4].tolist() == [4096, 4096, 4096, 17]
    for i in range(4):
        assert bytes(out[i]) == hashlib.sha1(data[i * 4096:(i + 1) * 4096].tobytes()).digest()
    e = tmp_path / "empty.bin"
    e.write_bytes(b"")
    assert oracle.lib.oracle_encode_file(str(e).encode(), 4096, out.ctypes.data, 8, None) == 0
    assert oracle.lib.oracle_encode_file(str(tmp_path / "missing").encode(), 4096, out.ctypes.data, 8, None) == -1


@pytest.mark.slow
def test_c2_digest_of_digests(oracle, golden):
    """Full C2 (4 GiB, 256 KiB chunks) through the oracle, multithreaded: the
    SHA-1 of the 16,384 concatenated raw digests equals the hashlib golden."""
    c2 = golden("c2.json")
    nt = os.cpu_count() or 1
    data = oracle.synth(c2["seed"], 0, c2["size"], nthreads=nt)
    n = c2["n_chunks"]
    offs = np.arange(n, dtype=np.uint64) * np.uint64(c2["chunk_size"])
    sizes = np.full(n, c2["chunk_size"], dtype=np.uint32)
    d = oracle.sha1_batch(data, offs, sizes, nthreads=nt)
    del data
    assert hashlib.sha1(d.tobytes()).hexdigest() == c2["sha1_of_concat_raw_digests_hex"]
    for k, v in c2["samples_b64"].items():
        assert oracle.b64_27(bytes(d[int(k)])) == v


from hypothesis import given, settings, strategies as st  # noqa: E402


@settings(max_examples=200, deadline=None)
@given(st.binary(min_size=0, max_size=1200))
def test_sha1_property_vs_hashlib(oracle, data):
    """Property: the restatement equals an independent SHA-1 (hashlib) on any bytes,
    and its base64-27 string is hashlib's digest in unpadded standard base64."""
    want = hashlib.sha1(data).digest()
    assert oracle.sha1(data) == want
    assert oracle.base64_encode(data) == base64.b64encode(want).decode().rstrip("=")


@settings(max_examples=60, deadline=None)
@given(st.lists(st.integers(min_value=0, max_value=700), min_size=1, max_size=24), st.integers(0, 2**31 - 1))
def test_sha1_batch_property_ragged(oracle, sizes, seed):
    """Property: the batch entry point over a ragged, overlapping-free chunk table at
    arbitrary (unaligned) offsets equals hashlib chunk by chunk."""
    rng = np.random.default_rng(seed)
    gaps = rng.integers(0, 17, len(sizes))
    offs, pos = [], 0
    for g, s in zip(gaps, sizes):
        pos += int(g)
        offs.append(pos)
        pos += s
    base = rng.integers(0, 256, pos + 1, dtype=np.uint8)
    got = oracle.sha1_batch(base, np.array(offs, np.uint64), np.array(sizes, np.uint32))
    for k, (o, s) in enumerate(zip(offs, sizes)):
        assert bytes(got[k]) == hashlib.sha1(base[o:o + s].tobytes()).digest()


# --------------------------------------------------------------------------- the timed CPU comparator
def test_unrolled_comparator_kats_and_hmac(oracle, golden):
    """oracle/sha1_unrolled.c, the reference-shaped comparator that bench.py's
    cpu_baseline times, answers the Crypto++ SHA-1 and HMAC(SHA-1) KATs."""
    for k in golden("kat.json")["kats"]:
        assert oracle.sha1_unrolled(_kat_message(k)).hex() == k["hex"], k["name"]
    for name, g, want in hmac_sha1_cases(lambda ms: [oracle.sha1_unrolled(m) for m in ms]):
        assert g == want, name


def test_unrolled_comparator_tails_ragged_c1(oracle, golden):
    """Same goldens as the checker: the padding tails, the ragged batch (unaligned
    offsets, threaded) and C1 in full."""
    for t in golden("synthetic.json")["tails"]:
        data = oracle.synth(t["seed"], 0, t["size"])
        n = (t["size"] + t["chunk_size"] - 1) // t["chunk_size"]
        offs = np.arange(n, dtype=np.uint64) * np.uint64(t["chunk_size"])
        sizes = np.minimum(t["chunk_size"], t["size"] - offs.astype(np.int64)).astype(np.uint32)
        got = [oracle.b64_27(bytes(d)) for d in oracle.sha1_batch_unrolled(data, offs, sizes)]
        assert got == t["b64"], (t["size"], t["chunk_size"])
    r = golden("synthetic.json")["ragged"]
    buf = oracle.synth(r["seed"], 0, r["buf_len"])
    got = oracle.sha1_batch_unrolled(buf, r["offsets"], r["sizes"], nthreads=4)
    assert [bytes(d).hex() for d in got] == r["hex"]
    c1 = golden("c1.json")
    data = oracle.synth(c1["seed"], 0, c1["size"])
    n = c1["size"] // c1["chunk_size"]
    offs = np.arange(n, dtype=np.uint64) * np.uint64(c1["chunk_size"])
    got = oracle.sha1_batch_unrolled(data, offs, np.full(n, c1["chunk_size"], np.uint32), nthreads=3)
    assert [oracle.b64_27(bytes(d)) for d in got] == c1["b64"]


@settings(max_examples=200, deadline=None)
@given(st.binary(min_size=0, max_size=1200))
def test_unrolled_comparator_equals_checker(oracle, data):
    assert oracle.sha1_unrolled(data) == oracle.sha1(data) == hashlib.sha1(data).digest()
