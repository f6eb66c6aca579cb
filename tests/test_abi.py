"""The C-ABI library loads and exports every symbol include/lbf_hash.h declares.

CPU-only checks: no hashing happens here (there is no CPU hashing path); the
GPU-less behaviour tested is that the context refuses to start loudly.
"""
import base64
import ctypes
import os
import subprocess

import numpy as np
import pytest

from bitflood_amd import _capi


def test_library_exports_every_header_symbol():
    lib = _capi.load()
    syms = _capi.header_symbols()
    assert "lbf_sha1_batch" in syms and "lbf_verify_batch" in syms and "lbf_b64_27" in syms
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the binding covers the whole header
    assert sorted(_capi._SIGS) == syms


def test_exported_symbols_are_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    names = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for s in _capi.header_symbols():
        assert s in names, f"{s} not exported with C linkage"


def test_abi_version():
    assert _capi.load().lbf_abi_version() == 1


def test_b64_27_product_matches_cryptopp_vector():
    """The product's rendering (lbf_b64_27, host code of liblbfhash.so) and its
    inverse against Crypto++ 5.2.1's own expected base64 output
    (tests/test_oracle.py explains which 20-byte windows it pins)."""
    from bitflood_amd import b64_27, b64_27_decode
    from tests.test_oracle import cryptopp_windows
    for d, want in cryptopp_windows():
        assert b64_27(d) == want
        assert b64_27_decode(want) == d


def test_b64_27_host_formatting_matches_python():
    from bitflood_amd import b64_27, b64_27_decode
    rng = np.random.default_rng(5)
    for _ in range(100):
        d = rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
        s = b64_27(d)
        assert s == base64.b64encode(d).decode().rstrip("=")
        assert b64_27_decode(s) == d


def test_b64_27_decode_rejects_malformed():
    from bitflood_amd import LbfError, b64_27_decode
    good = "qZk+NkcGgWq6PiVxeFDCbJzQ2J0"
    assert b64_27_decode(good).hex() == "a9993e364706816aba3e25717850c26c9cd0d89d"
    for bad in [good[:-1], good + "A", good[:-1] + "1", good[:5] + "*" + good[6:], ""]:
        with pytest.raises(LbfError):
            b64_27_decode(bad)


@pytest.mark.skipif(_capi.device_count() > 0, reason="only meaningful without a GPU")
def test_no_gpu_fails_loudly():
    from bitflood_amd import ChunkHasher, LbfError
    with pytest.raises(LbfError) as ei:
        ChunkHasher()
    assert ei.value.status == _capi.LBF_ERR_NO_DEVICE
    assert "no CPU fallback" in str(ei.value)


def test_shipped_kernel_variants_only():
    """The product library carries the five shipped kernels (1 lane, 7 pc4/b64,
    10 pcx5, 11 lds2, 12 pc4x2); the superseded ones exist only in the A/B library of tools/experimental/."""
    lib = _capi.load()
    try:
        for v in (0, 1, 7, 10, 11, 12):
            assert lib.lbf_set_kernel_variant(v) == _capi.LBF_OK, v
        for v in (2, 3, 4, 5, 6, 8, 9, 13, -1):
            assert lib.lbf_set_kernel_variant(v) == _capi.LBF_ERR_INVALID, v
        # automatic choice by chain count
        lib.lbf_set_kernel_variant(0)
        assert [lib.lbf_kernel_for(n) for n in (1, 16384, 16385, 32768, 32769, 1 << 20)] == [7, 7, 12, 12, 11, 11]
    finally:
        lib.lbf_set_kernel_variant(0)


def test_kernels_compiled_for_gfx950():
    blob = open(_capi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_header_is_plain_c(tmp_path):
    """include/lbf_hash.h compiles as C99 with warnings as errors, links against
    liblbfhash.so from a C program, and behaves (tests/c/c_abi_check.c)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "c_abi_check"
    libdir = os.path.dirname(_capi.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
                    "-I", os.path.join(root, "include"), os.path.join(root, "tests", "c", "c_abi_check.c"),
                    "-L", libdir, "-llbfhash", f"-Wl,-rpath,{libdir}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert r.stdout.startswith("ok:")
