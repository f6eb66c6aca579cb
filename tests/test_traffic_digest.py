"""roofline.traffic is tied to the machine code that was profiled (VERDICT r04
weak #6): profiles/pmc_traffic.json entries carry the profiled kernel's code
digest, and bench.py cites an entry only while the library it loaded carries
the same bytes for that kernel.  CPU only: the digests are read out of the
built .so (bitflood_amd/kernel_digest.py), no GPU call."""
import json
import os

import pytest

import bench
from bitflood_amd import _capi
from bitflood_amd import kernel_digest as KD

LIB = _capi.LIB_PATH
SHIPPED = ["sha1_pc4_kernel<true, 2, 8>", "sha1_pc4x2_kernel<true>", "sha1_lds2_kernel<true>",
           "sha1_lane_kernel<true>", "sha1_pcx5_kernel<true, 64>", "b64_encode_kernel", "b64_decode_kernel",
           "b64_decode_canon_kernel"]


@pytest.fixture(scope="module")
def digests():
    if not os.path.exists(LIB):
        pytest.skip("liblbfhash.so not built")
    return KD.kernel_digests(LIB)


def test_every_shipped_kernel_has_a_digest(digests):
    for k in SHIPPED:
        sym = KD.symbol_for(digests, k)
        assert sym, k
        assert len(digests[sym]) == 64
    # the demangled form rocprofv3 prints resolves to the same symbol
    assert (KD.symbol_for(digests, "void lbf::(anonymous namespace)::sha1_pc4_kernel<true, 2, 8>(lbf::ChunkParams)")
            == KD.symbol_for(digests, "sha1_pc4_kernel<true, 2, 8>"))
    # template arguments are part of the match: <false, ...> is another kernel
    assert KD.symbol_for(digests, "sha1_pc4_kernel<false, 2, 8>") != KD.symbol_for(digests, SHIPPED[0])
    assert KD.symbol_for(digests, "sha1_pc4_kernel<true, 4>") is None  # superseded, not shipped


def test_bench_reads_the_loaded_librarys_digest(digests):
    sym, sha = bench.kernel_code_digest("sha1_pc4_kernel<true, 2, 8>")
    assert sym and sha == digests[sym]


def _entry(sha, **kw):
    e = {"file_bytes": 4 << 30, "chunk_size": 262144, "hbm_bytes_per_launch": 4296004394.0,
         "source": "profiles/rXX/c2/summary.json",
         "kernel": "void lbf::(anonymous namespace)::sha1_pc4_kernel<true, 2, 8>(lbf::ChunkParams)"}
    if sha is not None:
        e["code_sha256"] = sha
    e.update(kw)
    return e


def _lookup(tmp_path, entries, code_sha, kernel="sha1_pc4_kernel<true, 2, 8>", size=4 << 30):
    p = tmp_path / "pmc_traffic.json"
    p.write_text(json.dumps({"entries": entries}))
    return bench.traffic_from_profiles(size, 262144, kernel, code_sha, path=str(p))


def test_matching_digest_gives_the_recorded_traffic(tmp_path):
    t, src, why = _lookup(tmp_path, [_entry("ab" * 32)], "ab" * 32)
    assert t == 4296004394.0 and "ab" * 8 in src and why is None


def test_changed_kernel_gets_null(tmp_path):
    t, src, why = _lookup(tmp_path, [_entry("ab" * 32)], "cd" * 32)
    assert t is None and src is None and "not the code that was profiled" in why


def test_record_without_digest_gets_null(tmp_path):
    t, _, why = _lookup(tmp_path, [_entry(None)], "ab" * 32)
    assert t is None and "no machine-code digest" in why


def test_unreadable_library_gets_null(tmp_path):
    t, _, why = _lookup(tmp_path, [_entry("ab" * 32)], None)
    assert t is None and "could not be read" in why


def test_other_size_gets_null(tmp_path):
    t, _, why = _lookup(tmp_path, [_entry("ab" * 32)], "ab" * 32, size=8 << 30)
    assert t is None and "no PMC record" in why


def test_an_older_record_is_skipped_for_the_matching_one(tmp_path):
    t, _, why = _lookup(tmp_path, [_entry("cd" * 32, hbm_bytes_per_launch=1.0), _entry("ab" * 32)], "ab" * 32)
    assert t == 4296004394.0 and why is None


@pytest.mark.parametrize("kernel,size,cs", [("sha1_lds2_kernel<true>", 64 << 30, 262144),
                                            ("sha1_pc4x2_kernel<true>", 32 << 30, 1 << 20)])
def test_other_configs_entry_cites_traffic_by_digest(tmp_path, digests, kernel, size, cs):
    """other_configs' C3 and C4 records take their traffic
    through the same digest rule as the main line."""
    sym = KD.symbol_for(digests, kernel)
    rec = {"file_bytes": size, "chunk_size": cs, "hbm_bytes_per_launch": size * 1.001, "source": "profiles/x.json",
           "kernel": f"void lbf::(anonymous namespace)::{kernel}(lbf::ChunkParams)"}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"entries": [dict(rec, code_sha256=digests[sym])]}))
    e = bench.config_entry("Cx", size, cs, 10.0, True, "g", kernel, pmc_path=str(p))
    assert e["traffic"] == size * 1.001 and e["traffic_ratio"] == 1.001 and e["traffic_null_reason"] is None
    assert e["kernel_code_sha256"] == digests[sym] and e["kernel_symbol"] == sym
    p.write_text(json.dumps({"entries": [dict(rec, code_sha256="ef" * 32)]}))
    e = bench.config_entry("Cx", size, cs, 10.0, True, "g", kernel, pmc_path=str(p))
    assert e["traffic"] is None and "not the code that was profiled" in e["traffic_null_reason"]


@pytest.mark.parametrize("kernel,size,cs", [("sha1_pc4_kernel<true, 2, 8>", 4 << 30, 262144),
                                            ("sha1_lds2_kernel<true>", 64 << 30, 262144),
                                            ("sha1_pc4x2_kernel<true>", 32 << 30, 1 << 20)])
def test_committed_records_match_the_shipped_library(digests, kernel, size, cs):
    """The committed C2, C3 and C4 records were profiled on the code this tree
    ships (the round-end bench line carries their traffic only then)."""
    sym = KD.symbol_for(digests, kernel)
    t, src, why = bench.traffic_from_profiles(size, cs, kernel, digests[sym])
    assert t is not None, why
    assert 1.0 <= t / size < 1.03, (t, src)


def test_descriptor_is_part_of_the_digest(digests):
    """the digest covers the kernel descriptor (VGPR/SGPR counts,
    LDS size), not only the instructions."""
    with open(LIB, "rb") as f:
        blob = f.read()
    co = KD._code_objects(blob)[0]
    funcs = KD._elf_functions(co)
    sym = KD.symbol_for(digests, "sha1_pc4_kernel<true, 2, 8>")
    code = funcs[sym]
    kd = bytearray(code[-64:])
    # compute_pgm_rsrc1 (VGPR/SGPR granules) sits at byte 48 of the descriptor
    assert int.from_bytes(kd[48:52], "little") & 63 > 0
    assert kd[16:24] == bytes(8)  # the code-entry offset is left out


def test_compressed_bundle_is_reported(tmp_path):
    p = tmp_path / "fake.so"
    p.write_bytes(b"\x7fELF" + b"\0" * 64 + b"CCOB" + b"\0" * 64)
    with pytest.raises(KD.CompressedBundle):
        KD.kernel_digests(str(p))
