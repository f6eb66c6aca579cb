"""Compile-time checks on the gfx950 code (CPU only: hipcc cross-compiles).

The LDS-DMA primitive dma16 (bitflood_amd/csrc/kern_common.hpp) writes M0 in
inline asm.  M0 must be declared clobbered, or the compiler may reuse an M0
value it set before the asm.  tests/c/m0_clobber_probe.hip puts dma16 between
two compiler-generated LDS DMAs with the same LDS base; the second must get its
own `s_mov_b32 m0`.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CSRC = os.path.join(ROOT, "bitflood_amd", "csrc")

pytestmark = pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="no hipcc")


def _isa(src, tmp_path, name):
    out = tmp_path / name
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                        "-I" + CSRC, "--offload-device-only", "-S", "-o", str(out), src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return [ln.strip() for ln in out.read_text().splitlines() if ln.strip() and not ln.strip().startswith((".", ";"))]


def test_dma16_m0_clobber_forces_reinit(tmp_path):
    ins = _isa(os.path.join(ROOT, "tests", "c", "m0_clobber_probe.hip"), tmp_path, "probe.s")
    seq = [i for i in ins if i.startswith("s_mov_b32 m0") or i.startswith("global_load_lds")]
    assert len([i for i in seq if i.startswith("global_load_lds")]) == 3, seq
    # every LDS DMA is directly preceded by its own M0 write
    for k, i in enumerate(seq):
        if i.startswith("global_load_lds"):
            assert k > 0 and seq[k - 1].startswith("s_mov_b32 m0"), seq


def test_shipped_kernels_write_m0_only_in_dma16(tmp_path):
    """No compiler-generated M0 user exists in the shipped kernels: every M0
    write is the dma16 asm (`s_mov_b32 m0, sN` followed by the DMA)."""
    ins = _isa(os.path.join(CSRC, "sha1_kernels.hip"), tmp_path, "k.s")
    m0 = [k for k, i in enumerate(ins) if re.search(r"\bm0\b", i)]
    assert m0, "expected the LDS-DMA kernels to set M0"
    for k in m0:
        assert ins[k].startswith("s_mov_b32 m0, s"), ins[k]
        assert ins[k + 1] == "s_nop 0" and ins[k + 2].startswith("global_load_lds_dwordx4"), ins[k:k + 3]
