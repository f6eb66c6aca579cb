"""Python face of the MI355X chunk-hash path (over liblbfhash.so).

Mirrors the reference's hash entry points so tests read like the reference's
own call sites:

* ``base64_encode(data)`` == ``libBitFlood::Encoder::Base64Encode``
  (/root/reference/cpp/src/Encoder.cpp:107-120): SHA-1 rendered as the
  27-char unpadded base64 string.
* ``ChunkHasher.hash_chunks`` == the per-chunk hash loop of
  ``Encoder::EncodeFile`` (Encoder.cpp:54-72), batched.
* ``ChunkHasher.verify_chunks`` == the compare-with-flood-file verify of
  ``Flood::_SetupFilesAndChunks`` (Flood.cpp:259-275) and of
  ``ChunkMethodHandler::_HandleSendChunk`` (ChunkMethods.cpp:165-167).

All hashing runs on the GPU; there is no CPU path in this module.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _capi
from ._capi import LBF_DEVICE_PTR, LBF_HOST_PTR, LbfError, check, load

DIGEST = 20
# A valid one-byte host buffer that lives as long as the process: the base
# pointer for batches over empty data (every chunk then has size 0, so nothing
# is read from it, but the library still gets a real address).
_EMPTY = (ctypes.c_uint8 * 1)()


def b64_27(digest: bytes) -> str:
    """20-byte digest -> 27-char string (basecode.cpp:39-104, no padding)."""
    if len(digest) != DIGEST:
        raise ValueError("digest must be 20 bytes")
    out = ctypes.create_string_buffer(28)
    load().lbf_b64_27(bytes(digest), out)
    return out.value.decode()


def b64_27_decode(s: str) -> bytes:
    raw = s.encode()
    out = (ctypes.c_uint8 * DIGEST)()
    check(load().lbf_b64_27_decode(raw, len(raw), out))
    return bytes(out)


def chunk_table(length: int, chunk_size: int, base_offset: int = 0):
    """Offsets/sizes of Encoder.cpp's fixed-size chunking of one file:
    chunk i = [i*cs, min((i+1)*cs, length)); an empty file has no chunks."""
    if chunk_size <= 0:
        raise ValueError("chunk_size must be positive")
    n = (length + chunk_size - 1) // chunk_size
    offs = np.arange(n, dtype=np.uint64) * np.uint64(chunk_size)
    sizes = np.full(n, chunk_size, dtype=np.uint32)
    if n:
        sizes[-1] = length - (n - 1) * chunk_size
    return offs + np.uint64(base_offset), sizes


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return np.frombuffer(memoryview(data), dtype=np.uint8)


class ChunkHasher:
    """An lbf_ctx: device buffers, streams and pinned staging on one or more GPUs."""

    def __init__(self, device_mask: int = 0):
        lib = load()
        h = ctypes.c_void_p()
        check(lib.lbf_ctx_create(device_mask, ctypes.byref(h)))
        self._h = h
        self._lib = lib
        self._registered = {}  # pointer -> array kept alive while pinned

    @property
    def num_devices(self) -> int:
        return self._lib.lbf_ctx_num_devices(self._h)

    @property
    def num_workers(self) -> int:
        return self._lib.lbf_ctx_num_workers(self._h)

    def worker_info(self, worker: int = 0) -> dict:
        """Device, its NUMA node, the node of the worker's pinned staging and the
        number of CPUs its host threads are bound to (see lbf_ctx_worker_info)."""
        v = [ctypes.c_int(-9) for _ in range(4)]
        check(self._lib.lbf_ctx_worker_info(self._h, worker, *[ctypes.byref(x) for x in v]))
        return dict(zip(["device", "numa_node", "staging_node", "bound_cpus"], [x.value for x in v]))

    def close(self) -> None:
        if self._h:
            self._lib.lbf_ctx_destroy(self._h)
            self._h = None
        self._registered = {}

    def staging_stats(self) -> dict:
        """Cumulative chunk bytes sent through pinned staging / straight from
        registered memory (lbf_ctx_staging_stats)."""
        st, di = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(self._lib.lbf_ctx_staging_stats(self._h, ctypes.byref(st), ctypes.byref(di)))
        return {"staged": st.value, "direct": di.value}

    def b64_stats(self) -> dict:
        """Chunks of verify_b64 calls so far by decode path: text with the
        encoder's own layout decoded in one pass, the rest by the general
        two-pass kernel (lbf_ctx_b64_stats)."""
        one, gen = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(self._lib.lbf_ctx_b64_stats(self._h, ctypes.byref(one), ctypes.byref(gen)))
        return {"one_pass": one.value, "general": gen.value}

    # -- caller-pinned sources (lbf_host_register) ---------------------------
    def register_host(self, data) -> None:
        """Pin `data` (a contiguous numpy array / buffer) for this context:
        batches over it then go to the GPU without the staging copy.  The array
        is kept alive until unregister_host / close."""
        if isinstance(data, np.ndarray) and not data.flags.c_contiguous:
            raise ValueError("register_host: the array must be C-contiguous (a copy would be pinned instead)")
        buf = _as_u8(data)
        if buf.size == 0:
            raise ValueError("register_host: empty buffer")
        check(self._lib.lbf_host_register(self._h, buf.ctypes.data, buf.size))
        self._registered[buf.ctypes.data] = buf

    def unregister_host(self, data) -> None:
        ptr = _as_u8(data).ctypes.data
        check(self._lib.lbf_host_unregister(self._h, ptr))
        self._registered.pop(ptr, None)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host-memory batches -------------------------------------------------
    def hash_chunks(self, data, offsets, sizes) -> np.ndarray:
        buf = _as_u8(data)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        szs = np.ascontiguousarray(sizes, dtype=np.uint32)
        if offs.shape != szs.shape:
            raise ValueError("offsets and sizes differ in length")
        n = offs.size
        out = np.zeros((n, DIGEST), dtype=np.uint8)
        if n == 0:
            return out
        base = buf.ctypes.data if buf.size else ctypes.addressof(_EMPTY)
        check(self._lib.lbf_sha1_batch(self._h, base, buf.size, offs.ctypes.data, szs.ctypes.data, n,
                                       out.ctypes.data, LBF_HOST_PTR))
        return out

    def verify_chunks(self, data, offsets, sizes, expected) -> np.ndarray:
        buf = _as_u8(data)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        szs = np.ascontiguousarray(sizes, dtype=np.uint32)
        exp = np.ascontiguousarray(expected, dtype=np.uint8).reshape(-1, DIGEST)
        n = offs.size
        if szs.size != n or exp.shape[0] != n:
            raise ValueError("offsets, sizes and expected differ in length")
        ver = np.zeros(n, dtype=np.uint8)
        if n == 0:
            return ver.astype(bool)
        base = buf.ctypes.data if buf.size else ctypes.addressof(_EMPTY)
        check(self._lib.lbf_verify_batch(self._h, base, buf.size, offs.ctypes.data, szs.ctypes.data, n,
                                         exp.ctypes.data, ver.ctypes.data, LBF_HOST_PTR))
        return ver.astype(bool)

    # -- chunks read straight from a file (lbf_file_ranges) ---------------------
    def hash_file(self, path: str, offsets, sizes) -> np.ndarray:
        """Digests of byte ranges of a file, pread into pinned staging: EncodeFile's
        fread -> Base64Encode loop (Encoder.cpp:54-72) as one call."""
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        szs = np.ascontiguousarray(sizes, dtype=np.uint32)
        if offs.shape != szs.shape:
            raise ValueError("offsets and sizes differ in length")
        out = np.zeros((offs.size, DIGEST), dtype=np.uint8)
        if offs.size:
            check(self._lib.lbf_file_ranges(self._h, os.fsencode(path), offs.ctypes.data, szs.ctypes.data,
                                            offs.size, None, out.ctypes.data))
        return out

    def verify_file(self, path: str, offsets, sizes, expected) -> np.ndarray:
        """Resume verify of a file (Flood.cpp:259-275): True where the chunk is present
        in full and matches; short or missing chunks are False, as the reference leaves
        them '0'."""
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        szs = np.ascontiguousarray(sizes, dtype=np.uint32)
        exp = np.ascontiguousarray(expected, dtype=np.uint8).reshape(-1, DIGEST)
        if szs.size != offs.size or exp.shape[0] != offs.size:
            raise ValueError("offsets, sizes and expected differ in length")
        ver = np.zeros(offs.size, dtype=np.uint8)
        if offs.size:
            check(self._lib.lbf_file_ranges(self._h, os.fsencode(path), offs.ctypes.data, szs.ctypes.data,
                                            offs.size, exp.ctypes.data, ver.ctypes.data))
        return ver.astype(bool)

    def _files_call(self, paths, file_of, offsets, sizes, expected):
        enc = [os.fsencode(p) for p in paths]
        arr = (ctypes.c_char_p * len(enc))(*enc)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        szs = np.ascontiguousarray(sizes, dtype=np.uint32)
        fo = np.ascontiguousarray(file_of, dtype=np.uint32)
        if not (offs.shape == szs.shape == fo.shape):
            raise ValueError("file_of, offsets and sizes differ in length")
        if expected is None:
            out = np.zeros((offs.size, DIGEST), dtype=np.uint8)
            exp_ptr = None
        else:
            exp = np.ascontiguousarray(expected, dtype=np.uint8).reshape(-1, DIGEST)
            if exp.shape[0] != offs.size:
                raise ValueError("expected differs in length")
            out = np.zeros(offs.size, dtype=np.uint8)
            exp_ptr = exp.ctypes.data
        if offs.size:
            check(self._lib.lbf_files_ranges(self._h, arr, len(enc), fo.ctypes.data, offs.ctypes.data,
                                             szs.ctypes.data, offs.size, exp_ptr, out.ctypes.data))
        return out

    def hash_files(self, paths, file_of, offsets, sizes) -> np.ndarray:
        """Digests of byte ranges of several files in one pipelined batch
        (lbf_files_ranges): chunk i = [offsets[i], +sizes[i]) of paths[file_of[i]]."""
        return self._files_call(paths, file_of, offsets, sizes, None)

    def verify_files(self, paths, file_of, offsets, sizes, expected) -> np.ndarray:
        """Resume verify over several files in one batch (Flood.cpp:239-287)."""
        return self._files_call(paths, file_of, offsets, sizes, expected).astype(bool)

    def verify_b64(self, text, text_offsets, text_lens, expected_sizes, expected, out=None, out_offsets=None):
        """The receiver's decode + verify on the device (lbf_b64_verify_batch,
        ChunkMethods.cpp:137-167 with xmlrpc++'s base64 decode): chunk i is
        the base64 text text[text_offsets[i], + text_lens[i]).  Returns
        (verdicts as bool, decoded lengths); with `out` (a uint8 array) and
        `out_offsets` the decoded bytes land at out[out_offsets[i], +
        expected_sizes[i])."""
        buf = _as_u8(text)
        toff = np.ascontiguousarray(text_offsets, dtype=np.uint64)
        tlen = np.ascontiguousarray(text_lens, dtype=np.uint32)
        esz = np.ascontiguousarray(expected_sizes, dtype=np.uint32)
        exp = np.ascontiguousarray(expected, dtype=np.uint8).reshape(-1, DIGEST)
        n = toff.size
        if not (tlen.size == esz.size == exp.shape[0] == n):
            raise ValueError("text_offsets, text_lens, expected_sizes and expected differ in length")
        ver = np.zeros(n, dtype=np.uint8)
        sizes = np.zeros(n, dtype=np.uint32)
        if n == 0:
            return ver.astype(bool), sizes
        ooff = None
        if out is not None:
            if not (isinstance(out, np.ndarray) and out.dtype == np.uint8 and out.flags.c_contiguous):
                raise ValueError("out must be a C-contiguous uint8 array")
            ooff = np.ascontiguousarray(out_offsets, dtype=np.uint64)
            if ooff.size != n:
                raise ValueError("out_offsets differs in length")
        base = buf.ctypes.data if buf.size else ctypes.addressof(_EMPTY)
        check(self._lib.lbf_b64_verify_batch(self._h, base, buf.size, toff.ctypes.data, tlen.ctypes.data, n,
                                             esz.ctypes.data, exp.ctypes.data,
                                             None if out is None else out.ctypes.data,
                                             0 if out is None else out.size,
                                             None if ooff is None else ooff.ctypes.data, sizes.ctypes.data,
                                             ver.ctypes.data))
        return ver.astype(bool), sizes

    def verify_encode_b64(self, data, offsets, sizes, expected):
        """The sender's verify + encode on the device
        (lbf_verify_encode_b64_batch, ChunkMethods.cpp:89-135 with xmlrpc++'s
        base64 encode): chunk i = data[offsets[i], + sizes[i]).  Returns
        (verdicts as bool, [text of chunk i as bytes])."""
        buf = _as_u8(data)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        sz = np.ascontiguousarray(sizes, dtype=np.uint32)
        exp = np.ascontiguousarray(expected, dtype=np.uint8).reshape(-1, DIGEST)
        n = offs.size
        if not (sz.size == exp.shape[0] == n):
            raise ValueError("offsets, sizes and expected differ in length")
        ver = np.zeros(n, dtype=np.uint8)
        if n == 0:
            return ver.astype(bool), []
        lens = [int(self._lib.lbf_b64_put_length(int(s))) for s in sz]
        toff = np.zeros(n, dtype=np.uint64)
        pos = 0
        for i, tl in enumerate(lens):
            toff[i] = pos
            pos += (tl + 15) // 16 * 16
        text = np.zeros(max(pos, 1), dtype=np.uint8)
        base = buf.ctypes.data if buf.size else ctypes.addressof(_EMPTY)
        check(self._lib.lbf_verify_encode_b64_batch(self._h, base, buf.size, offs.ctypes.data, sz.ctypes.data, n,
                                                    exp.ctypes.data, ver.ctypes.data, text.ctypes.data, text.size,
                                                    toff.ctypes.data))
        return ver.astype(bool), [text[int(toff[i]):int(toff[i]) + lens[i]].tobytes() for i in range(n)]

    def sha1(self, data) -> bytes:
        buf = _as_u8(data)
        out = (ctypes.c_uint8 * DIGEST)()
        base = buf.ctypes.data if buf.size else ctypes.addressof(_EMPTY)
        check(self._lib.lbf_sha1_one(self._h, base, buf.size, out))
        return bytes(out)

    def base64_encode(self, data) -> str:
        """Encoder::Base64Encode(data, size, out) (Encoder.cpp:107-120)."""
        return b64_27(self.sha1(data))

    def encode_buffer(self, data, chunk_size: int) -> list[str]:
        """Per-chunk hash strings of one in-memory file (Encoder.cpp:54-72)."""
        buf = _as_u8(data)
        offs, sizes = chunk_table(buf.size, chunk_size)
        return [b64_27(bytes(d)) for d in self.hash_chunks(buf, offs, sizes)]


# ---------------------------------------------------------------------------
# Device-resident helpers (bench.py, parity tests at full size)
# ---------------------------------------------------------------------------
class DeviceBuffer:
    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(load().lbf_dev_malloc(ctypes.byref(p), self.nbytes))
        self.ptr = p.value

    def free(self):
        if self.ptr:
            check(load().lbf_dev_free(self.ptr))
            self.ptr = None

    def _range(self, offset: int, nbytes: int, what: str):
        if not self.ptr:
            raise ValueError(f"{what}: buffer already freed")
        if offset < 0 or nbytes < 0 or offset + nbytes > self.nbytes:
            raise ValueError(f"{what}: [{offset}, {offset + nbytes}) outside the {self.nbytes}-byte buffer")

    def upload(self, host: np.ndarray, offset: int = 0):
        host = np.ascontiguousarray(host)
        self._range(offset, host.nbytes, "upload")
        check(load().lbf_memcpy_h2d(self.ptr + offset, host.ctypes.data, host.nbytes))

    def download(self, nbytes: int | None = None, offset: int = 0, dtype=np.uint8) -> np.ndarray:
        nbytes = self.nbytes - offset if nbytes is None else nbytes
        self._range(offset, nbytes, "download")
        out = np.empty(nbytes, dtype=np.uint8)
        check(load().lbf_memcpy_d2h(out.ctypes.data, self.ptr + offset, nbytes))
        return out.view(dtype)

    def download_into(self, out: np.ndarray, offset: int = 0) -> None:
        """Copy out.nbytes bytes from this buffer at `offset` into the existing
        C-contiguous host array `out`."""
        if not isinstance(out, np.ndarray) or not out.flags.c_contiguous:
            raise ValueError("download_into: out must be a C-contiguous numpy array")
        self._range(offset, out.nbytes, "download_into")
        if out.nbytes:
            check(load().lbf_memcpy_d2h(out.ctypes.data, self.ptr + offset, out.nbytes))

    def fill_synthetic(self, seed: int, start: int = 0, nbytes: int | None = None, stream=None, offset: int = 0):
        """Bytes [start, start+nbytes) of synthetic stream `seed` into this
        buffer at byte `offset` (16-byte aligned)."""
        nbytes = self.nbytes - offset if nbytes is None else nbytes
        self._range(offset, nbytes, "fill_synthetic")
        check(load().lbf_fill_synthetic(self.ptr + offset, nbytes, seed, start, stream))


def uniform_launch(base: DeviceBuffer | int, length: int, chunk_size: int, first: int, n: int,
                   digests: DeviceBuffer | int | None, expected=None, verdicts=None, stream=None):
    p = lambda x: None if x is None else (x.ptr if isinstance(x, DeviceBuffer) else x)  # noqa: E731
    check(load().lbf_sha1_uniform_launch(p(base), length, chunk_size, first, n, p(digests), p(expected),
                                         p(verdicts), stream))


def batch_launch(base, offsets, sizes, n, digests, expected=None, verdicts=None, stream=None):
    p = lambda x: None if x is None else (x.ptr if isinstance(x, DeviceBuffer) else x)  # noqa: E731
    check(load().lbf_sha1_launch(p(base), p(offsets), p(sizes), n, p(digests), p(expected), p(verdicts),
                                 stream))


def synchronize():
    check(load().lbf_device_synchronize())


def set_kernel_variant(v: int):
    check(load().lbf_set_kernel_variant(v))


__all__ = ["ChunkHasher", "DeviceBuffer", "LbfError", "b64_27", "b64_27_decode", "chunk_table",
           "uniform_launch", "batch_launch", "synchronize", "set_kernel_variant", "LBF_DEVICE_PTR",
           "_capi"]
