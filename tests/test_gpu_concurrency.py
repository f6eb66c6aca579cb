"""Concurrent callers on one lbf_ctx, and several contexts at once.

The reference's Base64Encode builds its hasher on the stack per call, so any
number of threads may call it (/root/reference/cpp/src/Encoder.cpp:107-120;
SURVEY.md §8b).  The drop-in keeps that promise with one context per process
whose calls serialize on the context (lbf_capi.cpp run_job / run_device_job)
and a thread-local last-error string.  These tests hammer one context from
several host threads (ctypes drops the GIL for the call, so the calls really
overlap on the host) with a mix of hash, verify, one-buffer and file batches,
including failing calls, and check every result against hashlib bit for bit.
"""
import hashlib
import os
import threading

import numpy as np
import pytest

from bitflood_amd import ChunkHasher, LbfError, chunk_table

pytestmark = pytest.mark.gpu


def _table(rng, buf_len, n):
    sizes = rng.integers(0, 200000, n).astype(np.uint32)
    offs = np.array([rng.integers(0, buf_len - s + 1) for s in sizes], dtype=np.uint64)
    return offs, sizes


def _want(buf, offs, sizes):
    return np.frombuffer(b"".join(hashlib.sha1(buf[o:o + s].tobytes()).digest() for o, s in zip(offs, sizes)),
                         dtype=np.uint8).reshape(-1, 20)


def _run_threads(target, n):
    errors = []

    def wrap(t):
        try:
            target(t)
        except BaseException as e:  # collected, re-raised in the main thread
            errors.append((t, e))

    th = [threading.Thread(target=wrap, args=(t,)) for t in range(n)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not any(x.is_alive() for x in th), "a caller thread did not finish"
    assert not errors, errors[:3]


@pytest.mark.parametrize("workers", [1, 2])
def test_many_threads_one_context(tmp_path, monkeypatch, workers):
    monkeypatch.setenv("LBF_WORKERS_PER_DEVICE", str(workers))
    rng = np.random.default_rng(404 + workers)
    buf = rng.integers(0, 256, 24 << 20, dtype=np.uint8)
    path = tmp_path / "shared.bin"
    buf[: 8 << 20].tofile(path)
    file_offs, file_sizes = chunk_table(8 << 20, 65536)
    file_want = _want(buf, file_offs, file_sizes)
    with ChunkHasher() as h:
        assert h.num_workers == workers

        def caller(t):
            r = np.random.default_rng(1000 * workers + t)
            for it in range(6):
                kind = (t + it) % 4
                if kind == 0:  # hash batch, ragged and unaligned
                    offs, sizes = _table(r, buf.size, int(r.integers(1, 400)))
                    got = h.hash_chunks(buf, offs, sizes)
                    assert np.array_equal(got, _want(buf, offs, sizes)), (t, it)
                elif kind == 1:  # verify batch with some corrupted expectations
                    offs, sizes = _table(r, buf.size, int(r.integers(1, 300)))
                    exp = _want(buf, offs, sizes).copy()
                    bad = r.random(exp.shape[0]) < 0.3
                    exp[bad, int(r.integers(0, 20))] ^= 0x40
                    assert np.array_equal(h.verify_chunks(buf, offs, sizes, exp), ~bad), (t, it)
                elif kind == 2:  # Base64Encode-style single buffers
                    for _ in range(5):
                        o = int(r.integers(0, buf.size - 70000))
                        n = int(r.integers(0, 70000))
                        assert h.sha1(buf[o:o + n]) == hashlib.sha1(buf[o:o + n].tobytes()).digest(), (t, it)
                else:  # file batch, and a failing call whose message stays in this thread
                    assert np.array_equal(h.hash_file(str(path), file_offs, file_sizes), file_want), (t, it)
                    with pytest.raises(LbfError, match="outside"):
                        h.hash_chunks(buf[:1000], np.array([999], np.uint64), np.array([2], np.uint32))

        _run_threads(caller, 8)


def test_contexts_in_parallel():
    """Several contexts (each with its own staging and streams) used at once."""
    rng = np.random.default_rng(77)
    buf = rng.integers(0, 256, 16 << 20, dtype=np.uint8)
    offs, sizes = chunk_table(buf.size, 262144)
    want = _want(buf, offs, sizes)
    ctxs = [ChunkHasher() for _ in range(3)]
    try:
        def caller(t):
            for _ in range(4):
                assert np.array_equal(ctxs[t % 3].hash_chunks(buf, offs, sizes), want), t
                assert ctxs[t % 3].verify_chunks(buf, offs, sizes, want).all(), t

        _run_threads(caller, 6)
    finally:
        for c in ctxs:
            c.close()
