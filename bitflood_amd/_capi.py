"""ctypes binding of include/lbf_hash.h (liblbfhash.so).

The library is built in-tree by __graft_entry__.build() / `make -C
bitflood_amd/csrc`.  torch is imported first when it is available so that the
process has exactly one HIP runtime: torch's bundled libamdhip64 and
/opt/rocm's share the soname libamdhip64.so.7, and whichever loads first
serves both.  There is no CPU fallback: when the library is missing this
module raises, and when no GPU is visible lbf_ctx_create fails with
LBF_ERR_NO_DEVICE.
"""
from __future__ import annotations

import ctypes
import os
import re

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
# LBF_LIB: tools only (tools/sweep_variants.py, tools/fuzz_gpu.py) point it at
# the A/B library of tools/experimental/ (`make -C tools/experimental`) that
# also carries the superseded kernel variants; the product loads the shipped one.
LIB_PATH = os.environ.get("LBF_LIB") or os.path.join(_HERE, "lib", "liblbfhash.so")
HEADER_PATH = os.path.join(_REPO, "include", "lbf_hash.h")

LBF_OK = 0
LBF_ERR_INVALID = -1
LBF_ERR_NO_DEVICE = -2
LBF_ERR_HIP = -3
LBF_ERR_NOMEM = -4
LBF_ERR_IO = -5
LBF_HOST_PTR = 0
LBF_DEVICE_PTR = 1

_u8p = ctypes.POINTER(ctypes.c_uint8)
_c = ctypes
_SIGS = {
    "lbf_abi_version": (_c.c_int, []),
    "lbf_last_error": (_c.c_char_p, []),
    "lbf_device_count": (_c.c_int, [_c.POINTER(_c.c_int)]),
    "lbf_ctx_create": (_c.c_int, [_c.c_uint32, _c.POINTER(_c.c_void_p)]),
    "lbf_ctx_destroy": (None, [_c.c_void_p]),
    "lbf_ctx_num_devices": (_c.c_int, [_c.c_void_p]),
    "lbf_ctx_num_workers": (_c.c_int, [_c.c_void_p]),
    "lbf_ctx_worker_info": (_c.c_int, [_c.c_void_p, _c.c_int, _c.POINTER(_c.c_int), _c.POINTER(_c.c_int),
                                       _c.POINTER(_c.c_int), _c.POINTER(_c.c_int)]),
    "lbf_sha1_batch": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_uint64, _c.c_void_p, _c.c_void_p,
                                  _c.c_uint64, _c.c_void_p, _c.c_int]),
    "lbf_verify_batch": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_uint64, _c.c_void_p, _c.c_void_p,
                                    _c.c_uint64, _c.c_void_p, _c.c_void_p, _c.c_int]),
    "lbf_host_register": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_uint64]),
    "lbf_host_unregister": (_c.c_int, [_c.c_void_p, _c.c_void_p]),
    "lbf_ctx_staging_stats": (_c.c_int, [_c.c_void_p, _c.POINTER(_c.c_uint64), _c.POINTER(_c.c_uint64)]),
    "lbf_ctx_b64_stats": (_c.c_int, [_c.c_void_p, _c.POINTER(_c.c_uint64), _c.POINTER(_c.c_uint64)]),
    "lbf_sha1_one": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_uint32, _c.c_void_p]),
    "lbf_verify_encode_b64_batch": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_uint64, _c.c_void_p, _c.c_void_p,
                                               _c.c_uint64, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_uint64,
                                               _c.c_void_p]),
    "lbf_b64_put_length": (_c.c_uint64, [_c.c_uint64]),
    "lbf_b64_verify_batch": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_uint64, _c.c_void_p, _c.c_void_p,
                                        _c.c_uint64, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_uint64,
                                        _c.c_void_p, _c.c_void_p, _c.c_void_p]),
    "lbf_file_ranges": (_c.c_int, [_c.c_void_p, _c.c_char_p, _c.c_void_p, _c.c_void_p, _c.c_uint64,
                                   _c.c_void_p, _c.c_void_p]),
    "lbf_files_ranges": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_uint32, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                    _c.c_uint64, _c.c_void_p, _c.c_void_p]),
    "lbf_b64_27": (None, [_c.c_void_p, _c.c_char_p]),
    "lbf_b64_27_decode": (_c.c_int, [_c.c_char_p, _c.c_size_t, _c.c_void_p]),
    "lbf_sha1_launch": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_uint64, _c.c_void_p,
                                   _c.c_void_p, _c.c_void_p, _c.c_void_p]),
    "lbf_sha1_uniform_launch": (_c.c_int, [_c.c_void_p, _c.c_uint64, _c.c_uint32, _c.c_uint64,
                                           _c.c_uint64, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                           _c.c_void_p]),
    "lbf_set_kernel_variant": (_c.c_int, [_c.c_int]),
    "lbf_get_kernel_variant": (_c.c_int, []),
    "lbf_kernel_for": (_c.c_int, [_c.c_uint64]),
    "lbf_fill_synthetic": (_c.c_int, [_c.c_void_p, _c.c_uint64, _c.c_uint64, _c.c_uint64, _c.c_void_p]),
    "lbf_dev_malloc": (_c.c_int, [_c.POINTER(_c.c_void_p), _c.c_uint64]),
    "lbf_dev_free": (_c.c_int, [_c.c_void_p]),
    "lbf_memcpy_h2d": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_uint64]),
    "lbf_memcpy_d2h": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_uint64]),
    "lbf_set_device": (_c.c_int, [_c.c_int]),
    "lbf_device_synchronize": (_c.c_int, []),
    "lbf_stream_create": (_c.c_int, [_c.POINTER(_c.c_void_p)]),
    "lbf_stream_destroy": (_c.c_int, [_c.c_void_p]),
    "lbf_stream_synchronize": (_c.c_int, [_c.c_void_p]),
    "lbf_time_uniform": (_c.c_int, [_c.c_void_p, _c.c_uint64, _c.c_uint32, _c.c_uint64, _c.c_uint64,
                                    _c.c_void_p, _c.c_int, _c.c_void_p, _c.POINTER(_c.c_float)]),
}

_lib = None


class LbfError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"lbf status {status}: {msg}")
        self.status = status


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function the public header declares (used by the ABI test)."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lbf_[a-z0-9_]+)\s*\(", text)))


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LbfError(LBF_ERR_INVALID,
                       f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # an A/B build of an earlier round (LBF_LIB, tools only) may lack
            # entry points added since; the shipped library must have them all
            if "LBF_LIB" in os.environ:
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != LBF_OK:
        msg = load().lbf_last_error()
        raise LbfError(rc, msg.decode() if msg else "")


def device_count() -> int:
    n = ctypes.c_int(0)
    check(load().lbf_device_count(ctypes.byref(n)))
    return n.value
