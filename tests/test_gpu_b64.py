"""The receiver's base64 decode + verify on the device (lbf_b64_verify_batch).

A SendChunk frame carries the chunk as XML-RPC base64 text
(/root/reference/cpp/src/ChunkMethods.cpp:141-163), written by xmlrpc++ 0.7's
encoder with a newline after every 18 groups (base64.h:154-210; the frame turns
it into a space, PeerConnection.cpp:132-156) and read back by its decoder
(base64.h:215-330).  `b64get` below restates that decoder in Python (the same
rules bitflood_amd/host/PeerWire.cpp Base64Get restates in C++); the GPU's
decoded bytes, lengths and verdicts must equal it on well-formed frames of
every size up to a full C5 chunk and on texts with junk characters, '='
anywhere, dropped characters and truncation.
"""
import base64
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EQ, SKIP = 64, 255
_DEC = np.full(256, SKIP, dtype=np.int16)
for _i, _c in enumerate(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"):
    _DEC[_c] = _i
_DEC[ord("=")] = EQ


def b64get(text: bytes) -> bytes:
    """xmlrpc++ 0.7 base64 decode (base64.h:215-330): skip characters outside
    the alphabet; take the rest four at a time; a group holding '=' ends the
    data ("xx==" one byte, "xxx=" two); an incomplete last group is dropped."""
    v = _DEC[np.frombuffer(text, dtype=np.uint8)]
    s = v[v != SKIP]
    out = bytearray()
    i = 0
    while True:
        if i >= len(s) or s[i] == EQ:
            return bytes(out)
        if i + 1 >= len(s) or s[i + 1] == EQ:
            return bytes(out)
        c0, c1 = int(s[i]), int(s[i + 1])
        if i + 2 >= len(s):
            return bytes(out)
        c2 = int(s[i + 2])
        if c2 == EQ:
            out.append(((c0 << 2) | (c1 >> 4)) & 255)
            return bytes(out)
        if i + 3 >= len(s):
            return bytes(out)
        c3 = int(s[i + 3])
        if c3 == EQ:
            out += bytes([((c0 << 2) | (c1 >> 4)) & 255, ((c1 << 4) | (c2 >> 2)) & 255])
            return bytes(out)
        out += bytes([((c0 << 2) | (c1 >> 4)) & 255, ((c1 << 4) | (c2 >> 2)) & 255, ((c2 << 6) | c3) & 255])
        i += 4


def xmlrpc_text(data: bytes) -> bytes:
    """The payload text of a SendChunk frame: base64 with a newline after
    every 18th complete group (base64.h:197-205), CR/LF framed as spaces."""
    s = base64.b64encode(data)
    full = len(data) // 3
    parts = []
    for g in range(len(s) // 4):
        parts.append(s[4 * g:4 * g + 4])
        if g < full and g % 18 == 17:
            parts.append(b" ")
    return b"".join(parts)


def _batch(hasher, texts, datas, align=16, shift=0, with_out=True, sizes=None):
    """One lbf_b64_verify_batch over texts[i] (expected: datas[i])."""
    toffs, chunks, pos = [], [], 0
    for t in texts:
        pos = (pos + align - 1) // align * align + shift
        toffs.append(pos)
        chunks.append((pos, t))
        pos += len(t)
    text = np.zeros(pos + 1, dtype=np.uint8)
    for p, t in chunks:
        text[p:p + len(t)] = np.frombuffer(t, dtype=np.uint8)
    esz = np.array([len(d) for d in datas] if sizes is None else sizes, dtype=np.uint32)
    exp = np.frombuffer(b"".join(hashlib.sha1(d).digest() for d in datas), dtype=np.uint8).reshape(-1, 20)
    out = ooff = None
    if with_out:
        ooff = np.zeros(len(texts), dtype=np.uint64)
        o = 0
        for i, s in enumerate(esz):
            ooff[i] = o
            o += (int(s) + 15) // 16 * 16
        out = np.zeros(max(o, 1), dtype=np.uint8)
    ver, dec = hasher.verify_b64(text, toffs, [len(t) for t in texts], esz, exp, out, ooff)
    return ver, dec, out, ooff, esz


@pytest.mark.parametrize("align,shift", [(16, 0), (16, 3), (1, 0)])
def test_well_formed_frames_every_size(hasher, align, shift):
    rng = np.random.default_rng(11 + shift)
    sizes = [0, 1, 2, 3, 4, 53, 54, 55, 56, 57, 63, 64, 65, 1000, 4095, 65536, 65539, 262144, 262147]
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sizes]
    texts = [xmlrpc_text(d) for d in datas]
    ver, dec, out, ooff, esz = _batch(hasher, texts, datas, align, shift)
    assert ver.all(), np.nonzero(~ver)[0]
    assert list(dec) == sizes
    for i, d in enumerate(datas):
        assert out[int(ooff[i]):int(ooff[i]) + len(d)].tobytes() == d, i
        if len(d) < 8192:
            assert b64get(texts[i]) == d  # the restatement agrees with Python's codec


def test_perturbed_texts_match_the_reference_decoder(hasher):
    """Junk characters anywhere, '=' anywhere, characters dropped, truncation,
    and replacements that keep the encoder's length ('=', junk or an alphabet
    character in place of another, so the one-pass decode reads them and must
    hand the chunk back): the device's bytes and lengths equal b64get's, and a
    verdict is 1 exactly when the decoded bytes are the original chunk."""
    rng = np.random.default_rng(5)
    junk = [c for c in range(256) if _DEC[c] == SKIP]
    texts, datas, wants = [], [], []
    for case in range(540):
        n = int(rng.integers(0, 3000))
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        t = bytearray(xmlrpc_text(d))
        kind = case % 9
        if kind == 1 and t:  # junk inserted
            for _ in range(int(rng.integers(1, 20))):
                t.insert(int(rng.integers(0, len(t) + 1)), int(rng.choice(junk)))
        elif kind == 2 and t:  # '=' somewhere
            t.insert(int(rng.integers(0, len(t) + 1)), ord("="))
        elif kind == 3 and t:  # characters dropped
            for _ in range(int(rng.integers(1, 4))):
                if t:
                    del t[int(rng.integers(0, len(t)))]
        elif kind == 4:  # truncated
            t = t[:int(rng.integers(0, len(t) + 1))]
        elif kind == 5 and t:  # a character flipped to another alphabet character
            j = int(rng.integers(0, len(t)))
            if _DEC[t[j]] < 64:
                t[j] = b"A"[0] if t[j] != b"A"[0] else b"B"[0]
        elif kind == 6 and len(t) > 4:  # '=' in place of a character before the last group
            t[int(rng.integers(0, len(t) - 4))] = ord("=")
        elif kind == 7 and t:  # junk in place of a character
            t[int(rng.integers(0, len(t)))] = int(rng.choice(junk))
        elif kind == 8 and b" " in t:  # an alphabet character in place of a separator
            seps = [j for j, c in enumerate(t) if c == ord(" ")]
            t[seps[int(rng.integers(0, len(seps)))]] = ord("Q")
        texts.append(bytes(t))
        datas.append(d)
        wants.append(b64get(bytes(t)))
    ver, dec, out, ooff, esz = _batch(hasher, texts, datas, align=1, shift=0)
    for i, (d, w) in enumerate(zip(datas, wants)):
        cap = len(d)
        assert int(dec[i]) == (len(w) if len(w) <= cap else cap + 1), (i, len(w), cap, int(dec[i]))
        got = out[int(ooff[i]):int(ooff[i]) + min(len(w), cap)].tobytes()
        assert got == w[:cap], i
        assert bool(ver[i]) == (w == d), i


def test_longer_text_and_no_output_buffer(hasher):
    """A text that decodes to more than the chunk's size fails the size check
    (ChunkMethods.cpp:156) and reports size + 1; without `out` only the
    verdicts and lengths come back."""
    rng = np.random.default_rng(7)
    d = rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    longer = xmlrpc_text(d + b"xyz")
    shorter = xmlrpc_text(d[:-3])
    ver, dec, *_ = _batch(hasher, [longer, shorter, xmlrpc_text(d)], [d, d, d], with_out=False)
    assert list(ver) == [False, False, True]
    assert list(dec) == [5001, 4997, 5000]


def test_many_chunks_in_one_call(hasher, oracle):
    """A C5-shaped batch: 300 frames of 64 KiB from the synthetic stream, every
    tenth corrupted by one flipped alphabet character."""
    cs, n = 65536, 300
    data = oracle.synth(0x5EED, 0, cs * n, nthreads=8)
    datas = [data[i * cs:(i + 1) * cs].tobytes() for i in range(n)]
    texts = [bytearray(xmlrpc_text(x)) for x in datas]
    for i in range(0, n, 10):
        j = 100 + i if texts[i][100 + i] != ord(" ") else 101 + i  # an alphabet character, not a separator
        texts[i][j] = ord("A") if texts[i][j] != ord("A") else ord("B")
    ver, dec, out, ooff, esz = _batch(hasher, [bytes(t) for t in texts], datas)
    assert [bool(v) for v in ver] == [i % 10 != 0 for i in range(n)]
    assert (dec == cs).all()
    for i in range(1, n, 37):
        if i % 10:  # the corrupted ones decode to other bytes, as they should
            assert out[int(ooff[i]):int(ooff[i]) + cs].tobytes() == datas[i], i


def test_sender_encode_matches_xmlrpc_text(hasher):
    """lbf_verify_encode_b64_batch: the text equals the encoder's (base64.h:154-210,
    spaces for the frame's newlines) at every size and alignment, and the
    verdicts mark the chunks whose expected digest is wrong."""
    rng = np.random.default_rng(21)
    sizes = [0, 1, 2, 3, 4, 53, 54, 55, 56, 57, 63, 64, 65, 1000, 4095, 65536, 65539, 262144, 262147]
    offs, pos = [], 0
    for k, n in enumerate(sizes):
        pos += k % 5  # ragged starts
        offs.append(pos)
        pos += n
    data = rng.integers(0, 256, pos, dtype=np.uint8)
    datas = [data[o:o + n].tobytes() for o, n in zip(offs, sizes)]
    exp = np.frombuffer(b"".join(hashlib.sha1(d).digest() for d in datas), dtype=np.uint8).reshape(-1, 20).copy()
    exp[3, 0] ^= 1
    ver, texts = hasher.verify_encode_b64(data, offs, sizes, exp)
    assert [bool(v) for v in ver] == [i != 3 for i in range(len(sizes))]
    for i, d in enumerate(datas):
        assert texts[i] == xmlrpc_text(d), (i, len(d))
    # round trip through the receiver's device decode
    rv, rs, out, ooff, _ = _batch(hasher, texts, datas)
    assert rv.all() and list(rs) == sizes


def test_outputs_touch_nothing_outside_their_slots(hasher):
    """Both entry points copy results back slot by slot (touching slots merged):
    the bytes of `out` / `text` before the first slot, between slots and after
    the last stay as they were, whatever the slots' alignment (the device
    copies keep it mod 16)."""
    rng = np.random.default_rng(3)
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (1000, 77, 4099)]
    exp = np.frombuffer(b"".join(hashlib.sha1(d).digest() for d in datas), dtype=np.uint8).reshape(-1, 20)
    texts = [xmlrpc_text(d) for d in datas]
    for first in (5, 16, 27):
        # decode: out slots from `first` on, sentinel everywhere else
        ooff = np.array([first, first + 1100, first + 1200], dtype=np.uint64)
        out = np.full(first + 1200 + 4099 + 40, 0xAB, dtype=np.uint8)
        toffs, pos, buf = [], 3, bytearray(b"\0" * 3)
        for t in texts:
            toffs.append(pos)
            buf += t
            pos += len(t)
        text = np.frombuffer(bytes(buf), dtype=np.uint8)
        esz = [len(d) for d in datas]
        ver, dec = hasher.verify_b64(text, toffs, [len(t) for t in texts], esz, exp, out, ooff)
        assert ver.all()
        assert (out[:first] == 0xAB).all() and (out[first + 1200 + 4099:] == 0xAB).all()
        for i, d in enumerate(datas):
            assert out[int(ooff[i]):int(ooff[i]) + len(d)].tobytes() == d
        # encode: text slots from `first` on
        lens = [len(t) for t in texts]
        tslot = np.array([first, first + lens[0] + 9, first + lens[0] + lens[1] + 20], dtype=np.uint64)
        tbuf = np.full(int(tslot[-1]) + lens[2] + 40, 0xCD, dtype=np.uint8)
        data = np.frombuffer(b"".join(datas), dtype=np.uint8)
        offs = np.array([0, 1000, 1077], dtype=np.uint64)
        sz = np.array(esz, dtype=np.uint32)
        v = np.zeros(3, dtype=np.uint8)
        e = np.ascontiguousarray(exp)
        assert hasher._lib.lbf_verify_encode_b64_batch(hasher._h, data.ctypes.data, data.size, offs.ctypes.data,
                                                       sz.ctypes.data, 3, e.ctypes.data, v.ctypes.data,
                                                       tbuf.ctypes.data, tbuf.size, tslot.ctypes.data) == 0
        assert v.all()
        assert (tbuf[:first] == 0xCD).all() and (tbuf[int(tslot[-1]) + lens[2]:] == 0xCD).all()
        for i, t in enumerate(texts):
            assert tbuf[int(tslot[i]):int(tslot[i]) + len(t)].tobytes() == t


def _encoder_layout_sizes():
    """Chunk sizes whose text exercises every length form of the encoder's
    layout and the one-pass kernels' tiles (encode 112 lines = 6,048 bytes =
    8,176 characters, decode 72 lines = 3,888 bytes = 5,256 characters; 64
    lines = 3,456 bytes, round 5's first tile): no tail, one or two tail
    bytes, a padded last group that is the 18th of its line (length 73q + 72:
    52, 53, 106, 107, ...), a text that ends with a separator (54k bytes), tile
    edges, a C5 chunk."""
    s = {0, 1, 2, 3, 51, 52, 53, 54, 55, 105, 106, 107, 108, 161, 162}
    for tile, ks in ((3456, (1, 2, 3, 76)), (6048, (1, 2, 43)), (3888, (1, 2, 67))):
        for k in ks:
            for d in (-3, -2, -1, 0, 1, 2, 3):
                s.add(tile * k + d)
    for g in (17, 35, 18 * 64 - 1, 18 * 64 + 17, 18 * 200 + 17):  # full groups = 18q + 17
        s.update({3 * g + 1, 3 * g + 2})
    s.update({65536, 262144, 262145, 262146})
    return sorted(s)


@pytest.mark.parametrize("align,shift", [(16, 0), (16, 5), (4, 2)])
def test_one_pass_takes_every_encoder_layout(hasher, align, shift):
    """Every text the encoder writes takes the one-pass kernel (the general
    decode sees none of them), including a padded last group that is the 18th
    of its line (such lengths, 73q + 72, went to the general
    kernel before), at aligned and unaligned text and output slots; bytes,
    lengths and verdicts equal the reference decoder's.  Damaged texts of the
    same lengths go to the general kernel."""
    rng = np.random.default_rng(40 + shift)
    sizes = _encoder_layout_sizes()
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sizes]
    texts = [xmlrpc_text(d) for d in datas]
    for d, t in zip(datas, texts):
        if len(t) % 73 == 72:
            assert t[-1:] == b"=", len(d)  # the form ADVICE r04 named: a padded group ends the line
    s0 = hasher.b64_stats()
    ver, dec, out, ooff, esz = _batch(hasher, texts, datas, align, shift)
    s1 = hasher.b64_stats()
    assert ver.all(), [sizes[i] for i in np.nonzero(~ver)[0]]
    assert list(dec) == sizes
    for i, d in enumerate(datas):
        assert out[int(ooff[i]):int(ooff[i]) + len(d)].tobytes() == d, sizes[i]
    assert s1["one_pass"] - s0["one_pass"] == len(sizes) and s1["general"] == s0["general"]
    # one alphabet character of each non-empty text replaced by junk: same lengths, general path, verdict 0
    bad = [bytearray(t) for t in texts]
    for t in bad:
        if t:
            alpha = [j for j, c in enumerate(t) if _DEC[c] < 64]
            t[alpha[int(rng.integers(0, len(alpha)))]] = ord("*")
    ver, dec, *_ = _batch(hasher, [bytes(t) for t in bad], datas, align, shift)
    s2 = hasher.b64_stats()
    nonempty = sum(1 for t in texts if t)
    assert s2["general"] - s1["general"] == nonempty
    for i, t in enumerate(bad):
        w = b64get(bytes(t))
        assert int(dec[i]) == (len(w) if len(w) <= sizes[i] else sizes[i] + 1), sizes[i]
        assert bool(ver[i]) == (w == datas[i]), sizes[i]


@pytest.mark.parametrize("one_pass", [True, False])
def test_gaps_between_slots_are_never_written(hasher, one_pass):
    """the decoded bytes come back slot by slot, so bytes of
    `out` between slots keep the caller's data (a shared or file-mapped arena),
    and a slot's bytes past a short decode are zeros, never another batch's
    device bytes.  Same for the encoder's text slots."""
    rng = np.random.default_rng(9)
    sizes = [5000, 3456, 77, 262144, 1]
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sizes]
    texts = [xmlrpc_text(d) for d in datas]
    texts[2] = xmlrpc_text(datas[2][:40])  # short: decodes to 40 of 77 bytes
    if not one_pass:
        texts = [b"\x01" + t for t in texts]  # junk in front: the general kernel decodes them all
    # a previous call leaves other bytes in the device scratch
    _batch(hasher, [xmlrpc_text(bytes([0xEE]) * 300000)], [bytes([0xEE]) * 300000])
    gaps = [7, 0, 100, 13, 3]  # bytes before each slot
    ooff, pos = [], 0
    for g, n in zip(gaps, sizes):
        pos += g
        ooff.append(pos)
        pos += n
    out = np.full(pos + 9, 0x5A, dtype=np.uint8)
    toffs, buf = [], bytearray()
    for t in texts:
        toffs.append(len(buf))
        buf += t
    exp = np.frombuffer(b"".join(hashlib.sha1(d).digest() for d in datas), dtype=np.uint8).reshape(-1, 20)
    ver, dec = hasher.verify_b64(np.frombuffer(bytes(buf), np.uint8), toffs, [len(t) for t in texts], sizes, exp,
                                 out, np.array(ooff, dtype=np.uint64))
    assert list(ver) == [True, True, False, True, True]
    assert list(dec) == [5000, 3456, 40, 262144, 1]
    inside = np.zeros(out.size, dtype=bool)
    for o, n in zip(ooff, sizes):
        inside[o:o + n] = True
    assert (out[~inside] == 0x5A).all(), "a byte outside the slots was written"
    for i, (o, d) in enumerate(zip(ooff, datas)):
        got = out[o:o + sizes[i]].tobytes()
        assert got == (d if i != 2 else d[:40] + bytes(37)), i


def test_overlapping_slots_are_refused(hasher):
    """two chunks' results in one byte would race on the device;
    both entry points refuse overlapping output slots."""
    from bitflood_amd import LbfError
    d = bytes(range(200))
    t = xmlrpc_text(d)
    text = np.frombuffer(t + t, np.uint8)
    exp = np.frombuffer(hashlib.sha1(d).digest() * 2, np.uint8).reshape(2, 20)
    out = np.zeros(600, np.uint8)
    with pytest.raises(LbfError, match="overlaps"):
        hasher.verify_b64(text, [0, len(t)], [len(t)] * 2, [200, 200], exp, out, np.array([0, 199], np.uint64))
    ver, _ = hasher.verify_b64(text, [0, len(t)], [len(t)] * 2, [200, 200], exp, out, np.array([0, 200], np.uint64))
    assert ver.all()  # touching slots are fine
    data = np.frombuffer(d, np.uint8)
    offs = np.zeros(2, np.uint64)
    sz = np.array([200, 200], np.uint32)
    v = np.zeros(2, np.uint8)
    tbuf = np.zeros(1000, np.uint8)
    e = np.ascontiguousarray(exp)
    for tslot, rc_ok in (([0, len(t) - 1], False), ([0, len(t)], True)):
        ts = np.array(tslot, np.uint64)
        rc = hasher._lib.lbf_verify_encode_b64_batch(hasher._h, data.ctypes.data, data.size, offs.ctypes.data,
                                                     sz.ctypes.data, 2, e.ctypes.data, v.ctypes.data,
                                                     tbuf.ctypes.data, tbuf.size, ts.ctypes.data)
        assert (rc == 0) is rc_ok, rc


def test_chunks_past_the_32_bit_bound_are_refused(hasher):
    """the wire kernels keep a chunk's text and byte positions in
    32 bits, so chunks whose text or tile math would pass 2^32 are refused at
    the entry points (LBF_ERR_INVALID), before any copy: the buffers here are
    small, only their claimed lengths are large."""
    from bitflood_amd import _capi
    lib = _capi.load()
    small = np.zeros(256, np.uint8)
    zero64 = np.zeros(1, np.uint64)
    exp, ver = np.zeros(20, np.uint8), np.zeros(1, np.uint8)
    big = np.array([(1 << 30) + 1], np.uint32)
    rc = lib.lbf_verify_encode_b64_batch(hasher._h, small.ctypes.data, 2 << 30, zero64.ctypes.data, big.ctypes.data,
                                         1, exp.ctypes.data, ver.ctypes.data, small.ctypes.data, 4 << 30,
                                         zero64.ctypes.data)
    assert rc == _capi.LBF_ERR_INVALID and b"1 GiB" in lib.lbf_last_error()
    ok_size = np.array([100], np.uint32)
    for tlen, cap in (((3 << 29) + 1, ok_size), (ok_size, big)):
        tl = np.asarray(tlen, np.uint32).reshape(1)
        rc = lib.lbf_b64_verify_batch(hasher._h, small.ctypes.data, 4 << 30, zero64.ctypes.data, tl.ctypes.data, 1,
                                      np.asarray(cap, np.uint32).reshape(1).ctypes.data, exp.ctypes.data, None, 0,
                                      None, None, ver.ctypes.data)
        assert rc == _capi.LBF_ERR_INVALID and b"wire decode" in lib.lbf_last_error()
    # the bound is far above the reference's chunk sizes: a well-formed 4 MiB chunk still decodes
    data = bytes(np.random.default_rng(3).integers(0, 256, 4 << 20, dtype=np.uint8))
    ver, dec, *_ = _batch(hasher, [xmlrpc_text(data)], [data], with_out=False)
    assert list(ver) == [True] and list(dec) == [len(data)]
