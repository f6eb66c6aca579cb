"""ctypes wrapper of oracle/build/liboracle.so -- TEST INFRASTRUCTURE (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")

_c = ctypes


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        lib = ctypes.CDLL(path)
        lib.oracle_sha1.argtypes = [_c.c_void_p, _c.c_uint32, _c.c_void_p]
        lib.oracle_sha1_init.argtypes = [_c.c_void_p]
        lib.oracle_sha1_update.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_uint32]
        lib.oracle_sha1_final.argtypes = [_c.c_void_p, _c.c_void_p]
        lib.oracle_b64_27.argtypes = [_c.c_void_p, _c.c_char_p]
        lib.oracle_base64_encode.argtypes = [_c.c_void_p, _c.c_uint32, _c.c_char_p]
        lib.oracle_encode_buffer.argtypes = [_c.c_void_p, _c.c_uint64, _c.c_uint32, _c.c_void_p]
        lib.oracle_encode_buffer.restype = _c.c_uint64
        lib.oracle_encode_file.argtypes = [_c.c_char_p, _c.c_uint32, _c.c_void_p, _c.c_uint64, _c.c_void_p]
        lib.oracle_encode_file.restype = _c.c_int64
        lib.oracle_sha1_batch.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_uint64, _c.c_void_p,
                                          _c.c_int]
        lib.oracle_synth_word.argtypes = [_c.c_uint64, _c.c_uint64]
        lib.oracle_synth_word.restype = _c.c_uint64
        lib.oracle_synth_fill.argtypes = [_c.c_void_p, _c.c_uint64, _c.c_uint64, _c.c_uint64]
        lib.oracle_synth_fill_mt.argtypes = [_c.c_void_p, _c.c_uint64, _c.c_uint64, _c.c_uint64, _c.c_int]
        # oracle/sha1_unrolled.c: the reference-shaped comparator bench.py times
        lib.unrolled_sha1.argtypes = [_c.c_void_p, _c.c_uint32, _c.c_void_p]
        lib.unrolled_sha1_batch.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_uint64, _c.c_void_p,
                                            _c.c_int]
        lib.unrolled_clock_probe.argtypes = [_c.c_uint64]
        lib.unrolled_clock_probe.restype = _c.c_uint64
        lib.unrolled_encode_file.argtypes = [_c.c_char_p, _c.c_uint32, _c.c_void_p, _c.c_uint64]
        lib.unrolled_encode_file.restype = _c.c_int64
        self.lib = lib

    @staticmethod
    def _ptr(a: np.ndarray):
        return a.ctypes.data if a.size else None

    def sha1(self, data) -> bytes:
        buf = np.frombuffer(memoryview(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        out = (_c.c_uint8 * 20)()
        self.lib.oracle_sha1(self._ptr(buf), buf.size, out)
        return bytes(out)

    def sha1_incremental(self, data: bytes, splits) -> bytes:
        ctx = (_c.c_uint8 * 128)()
        self.lib.oracle_sha1_init(ctx)
        pos = 0
        for s in list(splits) + [len(data)]:
            piece = data[pos:s]
            self.lib.oracle_sha1_update(ctx, piece, len(piece))
            pos = s
        out = (_c.c_uint8 * 20)()
        self.lib.oracle_sha1_final(ctx, out)
        return bytes(out)

    def b64_27(self, digest: bytes) -> str:
        out = _c.create_string_buffer(28)
        self.lib.oracle_b64_27(digest, out)
        return out.value.decode()

    def base64_encode(self, data) -> str:
        buf = np.frombuffer(memoryview(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        out = _c.create_string_buffer(28)
        self.lib.oracle_base64_encode(self._ptr(buf), buf.size, out)
        return out.value.decode()

    def encode_buffer(self, data: np.ndarray, chunk_size: int) -> np.ndarray:
        n = (data.size + chunk_size - 1) // chunk_size
        out = np.zeros((max(n, 1), 20), dtype=np.uint8)
        got = self.lib.oracle_encode_buffer(self._ptr(data), data.size, chunk_size, out.ctypes.data)
        return out[:got]

    def sha1_batch(self, base: np.ndarray, offsets, sizes, nthreads: int = 1) -> np.ndarray:
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        szs = np.ascontiguousarray(sizes, dtype=np.uint32)
        out = np.zeros((offs.size, 20), dtype=np.uint8)
        if offs.size:
            self.lib.oracle_sha1_batch(self._ptr(base), offs.ctypes.data, szs.ctypes.data, offs.size,
                                       out.ctypes.data, nthreads)
        return out

    def sha1_unrolled(self, data) -> bytes:
        buf = np.frombuffer(memoryview(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        out = (_c.c_uint8 * 20)()
        self.lib.unrolled_sha1(self._ptr(buf), buf.size, out)
        return bytes(out)

    def sha1_batch_unrolled(self, base: np.ndarray, offsets, sizes, nthreads: int = 1) -> np.ndarray:
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        szs = np.ascontiguousarray(sizes, dtype=np.uint32)
        out = np.zeros((offs.size, 20), dtype=np.uint8)
        if offs.size:
            self.lib.unrolled_sha1_batch(self._ptr(base), offs.ctypes.data, szs.ctypes.data, offs.size,
                                         out.ctypes.data, nthreads)
        return out

    def clock_ghz(self, iters: int = 200_000_000) -> float:
        """Approximate clock of the calling core (dependent-add chain, one per cycle)."""
        import time
        t0 = time.perf_counter()
        self.lib.unrolled_clock_probe(iters)
        return iters / (time.perf_counter() - t0) / 1e9

    def synth(self, seed: int, start: int, length: int, nthreads: int = 1) -> np.ndarray:
        out = np.empty(length, dtype=np.uint8)
        if length:
            if nthreads > 1:
                self.lib.oracle_synth_fill_mt(out.ctypes.data, length, seed, start, nthreads)
            else:
                self.lib.oracle_synth_fill(out.ctypes.data, length, seed, start)
        return out
