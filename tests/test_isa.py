"""Compile-time checks on the gfx950 code (CPU only: hipcc cross-compiles).

The shipped kernels' instruction streams are pinned by per-kernel digests
(tests/golden/isa_shipped.json, tools/isa_digest.py): moving the superseded
variants out to tools/experimental/ (VERDICT r03 "Next round" #2) had to leave
them unchanged, and any later change to a shipped kernel re-records them on
purpose.

The LDS-DMA primitive dma16 (bitflood_amd/csrc/kern_common.hpp) writes M0 in
inline asm.  M0 must be declared clobbered, or the compiler may reuse an M0
value it set before the asm.  tests/c/m0_clobber_probe.hip puts dma16 between
two compiler-generated LDS DMAs with the same LDS base; the second must get its
own `s_mov_b32 m0`.
"""
import ctypes
import json
import os
import re
import shutil
import subprocess
import sys

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


@pytest.fixture(scope="module")
def shipped_asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "k.s"
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                        "-I" + CSRC, "--offload-device-only", "-S", "-o", str(out),
                        os.path.join(CSRC, "sha1_kernels.hip")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_text()


def test_shipped_kernels_write_m0_only_in_dma16(shipped_asm):
    """No compiler-generated M0 user exists in the shipped kernels: every M0
    write is the dma16 asm (`s_mov_b32 m0, sN` followed by the DMA)."""
    ins = [ln.strip() for ln in shipped_asm.splitlines() if ln.strip() and not ln.strip().startswith((".", ";"))]
    m0 = [k for k, i in enumerate(ins) if re.search(r"\bm0\b", i)]
    assert m0, "expected the LDS-DMA kernels to set M0"
    for k in m0:
        assert ins[k].startswith("s_mov_b32 m0, s"), ins[k]
        assert ins[k + 1] == "s_nop 0" and ins[k + 2].startswith("global_load_lds_dwordx4"), ins[k:k + 3]


def test_shipped_kernel_isa_matches_recorded_digests(shipped_asm):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_digest
    import hashlib
    got = {k: {"instructions": len(v), "sha256": hashlib.sha256("\n".join(v).encode()).hexdigest()}
           for k, v in isa_digest.kernels(shipped_asm).items()}
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "isa_shipped.json")))["kernels"]
    assert sorted(got) == sorted(want)
    for k in want:
        assert got[k] == want[k], k


def test_shipped_sources_carry_no_experimental_variants():
    for name in os.listdir(CSRC):
        if name.endswith((".hip", ".hpp", ".cpp")):
            text = open(os.path.join(CSRC, name)).read()
            assert "LBF_EXPERIMENTAL_VARIANTS" not in text, name
            for k in ("sha1_pc_kernel", "sha1_pc2_kernel", "sha1_lds_kernel", "sha1_pcx4_kernel",
                      "sha1_pc4x2_diag_kernel"):
                assert k + "<" not in text and k + "(" not in text, (name, k)


def test_experimental_library_registers_exactly_its_table():
    """tools/experimental builds the A/B library from the shipped objects plus
    the superseded kernels; lbf_set_kernel_variant accepts a variant only if it
    has a launcher there (variant 24 used to be accepted and then
    silently fall back to the lane kernel)."""
    r = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "tools", "experimental")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "experimental", "liblbfhash.so"))
    accepted = [v for v in range(-1, 45) if lib.lbf_set_kernel_variant(v) == 0]
    lib.lbf_set_kernel_variant(0)
    # 37-39: round 6's A/Bs (pc4 with a barrier every second step; one pc4x2 group per workgroup)
    assert accepted == [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 25, 26,
                        27, 28, 34, 35, 36, 37, 38, 39]
