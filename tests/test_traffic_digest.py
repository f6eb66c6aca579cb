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


def test_committed_c2_record_matches_the_shipped_library(digests):
    """The committed C2 record was profiled on the code this tree ships (the
    round-end bench line carries its traffic only then)."""
    d = json.load(open(os.path.join(bench.ROOT, "profiles", "pmc_traffic.json")))
    sym = KD.symbol_for(digests, "sha1_pc4_kernel<true, 2, 8>")
    c2 = [e for e in d["entries"] if e["file_bytes"] == 4 << 30 and e.get("chunk_size") == 262144
          and "sha1_pc4_kernel<true, 2, 8>" in e["kernel"] and e.get("code_sha256")]
    assert c2, "no C2 record with a code digest"
    assert any(e["code_sha256"] == digests[sym] for e in c2)
