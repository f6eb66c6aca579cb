"""The C++ libBitFlood layer: flood-file format (CPU), the test_encoder port and
the resume-verify CLI (GPU), and the C++ API tests in lbf_gpu_tests (GPU).

Expected flood-file bytes are built here from the golden chunk strings with the
Xerces 2.6 DOMWriter pretty-print restatement of tests/domwriter.py, whose
layout rules tests/test_floodfile_format.py pins against Xerces' own expected
output (a fixture the reference holds).  No flood file exists in the
reference, so attribute order and escaping rest on code reading (SURVEY.md §4,
§8f).
"""
import base64
import json
import hashlib
import os
import subprocess

import numpy as np
import pytest

from bitflood_amd import _capi
from tests.c5_pair import run_pair
from tests.domwriter import pretty

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "bitflood_amd", "lib")
ENCODER = os.path.join(LIB, "lbf_encoder")
VERIFY = os.path.join(LIB, "lbf_verify")


def expected_xml(files, trackers) -> str:
    """files: list of (name, size, [(hash, index, size, weight)]) in map order.
    The tree FloodFile::ToXML builds (FloodFile.cpp:42-142), written by the
    DOMWriter restatement that tests/test_floodfile_format.py pins against
    Xerces' own expected output; attributes in name order."""
    file_nodes = []
    for name, size, chunks in sorted(files, key=lambda f: f[0].encode()):
        kids = [("Chunk", [("hash", h), ("index", str(i)), ("size", str(s)), ("weight", str(w))], [])
                for h, i, s, w in chunks]
        file_nodes.append(("File", [("name", name), ("size", str(size))], kids))
    tracker_nodes = [("Tracker", [("host", host), ("port", str(port))], []) for host, port in trackers]
    return pretty(("BitFlood", [], [("FileInfo", [], file_nodes)] + tracker_nodes))


def b64_27(d: bytes) -> str:
    return base64.b64encode(d).decode().rstrip("=")


def test_flood_file_format_unit():
    out = subprocess.run([os.path.join(LIB, "lbf_host_tests")], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert "host_tests OK" in out.stdout


def xmlrpc_base64(data: bytes) -> str:
    """xmlrpc++ 0.7 base64 (base64.h:154-210) restated on Python's codec: a
    newline after every 18th complete 4-char group, none after a padded one."""
    s = base64.b64encode(data).decode()
    full = len(data) // 3
    out = []
    for g in range(0, len(s) // 4):
        out.append(s[4 * g:4 * g + 4])
        if g < full and g % 18 == 17:
            out.append("\n")
    return "".join(out)


def test_peer_wire_base64_vectors(tmp_path):
    rng = np.random.default_rng(5)
    lines = []
    for n in [0, 1, 2, 3, 4, 53, 54, 55, 56, 107, 108, 109, 162, 1000, 4096, 65536]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        lines.append(f"{d.hex() or '-'} {xmlrpc_base64(d).replace(chr(10), chr(92) + 'n')}")
    p = tmp_path / "vec.txt"
    p.write_text("\n".join(lines) + "\n")
    out = subprocess.run([os.path.join(LIB, "lbf_host_tests"), "--wire-vectors", str(p)],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert f"wire_vectors OK {len(lines)}" in out.stdout


@pytest.mark.skipif(_capi.device_count() > 0, reason="only meaningful without a GPU")
def test_loopback_needs_gpu():
    out = subprocess.run([os.path.join(LIB, "lbf_loopback"), "--size", "100000"], capture_output=True, text=True)
    assert out.returncode == 2 and "no CPU fallback" in out.stderr


def _loopback(tmp_path, size, cs, window, batch, corrupt, synthetic=False, threads=None, timeout=600, register=True,
              extra=(), shape="one process"):
    """shape "one process": both peers as threads of one lbf_loopback (--role
    both); "two processes": the reference's shape, a seeder process and a
    leecher process (tests/c5_pair.py), each with its own HIP runtime."""
    opts = ["--size", str(size), "--chunksize", str(cs), "--window", str(window),
            "--batch", str(batch), "--corrupt", str(corrupt)] + list(extra)
    if synthetic:
        opts.append("--synthetic")
    if threads:
        opts += ["--threads", str(threads)]
    if not register:
        opts.append("--no-register")
    if shape == "two processes":
        r, _, _ = run_pair(opts, str(tmp_path / "c5"), timeout=timeout)
        assert r["pids"]["seeder"] != r["pids"]["leecher"]
        assert not os.path.exists(tmp_path / "c5"), "the two peers left files behind"
    else:
        out = subprocess.run([os.path.join(LIB, "lbf_loopback")] + opts + ["--dir", str(tmp_path / "c5")],
                             capture_output=True, text=True, timeout=timeout)
        assert out.returncode == 0, out.stderr + out.stdout
        r = json.loads(out.stdout.strip().splitlines()[-1])
        assert r["role"] == "both"
        r["process_shape"] = "one process"
    assert r["resume_verify_complete"] and r["files_identical"]
    assert r["arenas_registered"] is register
    n = (size + cs - 1) // cs
    assert r["chunks"] == n
    if corrupt:
        assert r["corrupted_sent"] == n // corrupt
        assert r["leecher"]["rejected"] == r["corrupted_sent"]
    else:
        assert r["leecher"]["rejected"] == 0
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("size,cs,window,batch,corrupt,synthetic", [
    (64 << 20, 262144, 64, 16, 0, False),                 # C5 chunk size, small file
    ((16 << 20) + 12345, 65536, 512, 128, 7, False),      # odd tail, wire corruption every 7th chunk
    ((16 << 20) + 12345, 65536 + 3, 512, 128, 7, True),   # generated seeder, chunks off the 8-byte grid
    (3 * 262144 + 1, 262144, 1, 1, 0, False),             # one chunk in flight, batch of one
    (65537, 4096, 1, 3, 1, False),                        # every chunk corrupted on its first send
    (65537, 4096, 1, 3, 1, True),
    (0, 1000, 1024, 512, 0, False),                       # empty file: no chunks, nothing to create
    (0, 1000, 1024, 512, 0, True),
])
def test_loopback_two_peers(tmp_path, size, cs, window, batch, corrupt, synthetic):
    """C5 shape: seeder and leecher over 127.0.0.1 speaking the reference's frames;
    every arrival is GPU-verified before it is written; a corrupted arrival is
    rejected and fetched again; the written file passes the resume verify and
    equals the source (a file, or with --synthetic the generated stream) byte
    for byte."""
    _loopback(tmp_path, size, cs, window, batch, corrupt, synthetic)


@pytest.mark.gpu
@pytest.mark.parametrize("size,cs,window,batch,corrupt,synthetic,extra", [
    (64 << 20, 262144, 64, 16, 0, False, []),
    ((16 << 20) + 12345, 65536, 512, 128, 7, False, []),                 # file seeder, odd tail, wire errors
    ((16 << 20) + 12345, 65536 + 3, 512, 128, 7, True, []),              # generated seeder, off the 8-byte grid
    (65537, 4096, 1, 3, 1, True, []),                                    # every chunk corrupted once
    (0, 1000, 1024, 512, 0, True, []),                                   # empty file
    ((32 << 20) + 12345, 65536, 512, 128, 7, True, ["--gpu-encode", "--seeder-workers", "2"]),
    ((32 << 20) + 12345, 65536, 512, 128, 7, False, ["--verifiers", "1", "--cpu-decode", "--no-register"]),
])
def test_loopback_two_processes(tmp_path, size, cs, window, batch, corrupt, synthetic, extra):
    """The reference's process shape: seeder and leecher are
    separate processes sharing the GPU, each with its own HIP runtime, GPU
    contexts and pinned arenas (neither sees the other's registrations).  Same
    end state as the one-process harness: the written file equals the source,
    every corrupted arrival is rejected and fetched again."""
    register = "--no-register" not in extra
    r = _loopback(tmp_path, size, cs, window, batch, corrupt, synthetic, register=register,
                  extra=[e for e in extra if e != "--no-register"], shape="two processes")
    assert r["seeder"]["sent"] >= r["chunks"]


def test_loopback_role_options_checked_before_the_gpu(tmp_path):
    """--role errors are reported before any GPU call (CPU-only host)."""
    lb = os.path.join(LIB, "lbf_loopback")
    for args, msg in [(["--role", "leecher", "--dir", str(tmp_path)], "needs --port"),
                      (["--role", "seeder"], "needs --dir"),
                      (["--role", "peer"], "--role takes"),
                      (["--role", "seeder", "--dir", str(tmp_path), "--port", "70000"], "--port must be"),
                      (["--role", "seeder", "--dir", str(tmp_path), "--port", "-1"], "--port must be")]:
        out = subprocess.run([lb] + args, capture_output=True, text=True, timeout=60)
        assert out.returncode == 2 and msg in out.stderr, (args, out.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("extra,synthetic", [
    (["--verifiers", "1", "--cpu-decode"], False),                         # round 3's shape
    (["--verifiers", "1", "--pipelined-seeder"], True),
    (["--verifiers", "4"], True),                                          # four leecher contexts side by side
    (["--verifiers", "3", "--pipelined-seeder", "--cpu-decode"], False),
    (["--verifiers", "2", "--cpu-decode"], True),                          # the host decode with two verifiers
    (["--verifiers", "1"], False),
    (["--verifiers", "2", "--gpu-encode"], True),                          # the seeder's encode on the GPU too
    (["--verifiers", "1", "--gpu-encode", "--pipelined-seeder", "--cpu-decode"], True),
    (["--verifiers", "2", "--seeder-workers", "2"], True),                # two seeder workers, each its own context
    (["--verifiers", "2", "--seeder-workers", "3", "--pipelined-seeder"], False),
    (["--verifiers", "2", "--seeder-workers", "2", "--gpu-encode"], True),
])
def test_loopback_verifier_counts(tmp_path, extra, synthetic):
    """The leecher's verifiers (each with its own GPU context and a copy of the
    chunk table), its base64 decode on the GPU (the default) or on the host,
    and the seeder's verify/encode stages: same end state for every
    combination -- the written file equals the source, every corrupted
    arrival is rejected and fetched again."""
    r = _loopback(tmp_path, (32 << 20) + 12345, 65536, 512, 128, 7, synthetic, extra=extra)
    assert r["verifiers"] == int(extra[1]) and r["seeder_pipelined"] is ("--pipelined-seeder" in extra)
    assert r["gpu_decode"] is ("--cpu-decode" not in extra)
    assert r["gpu_encode"] is ("--gpu-encode" in extra)
    assert r["seeder_workers"] == (int(extra[extra.index("--seeder-workers") + 1]) if "--seeder-workers" in extra else 1)


@pytest.mark.gpu
def test_loopback_staged_arenas(tmp_path):
    """The leecher's arenas are registered with its context by default, so its
    verifies copy them straight to HBM (lbf_host_register); --no-register sends
    them through the context's staging instead.  Same results either way."""
    _loopback(tmp_path, (16 << 20) + 12345, 65536, 512, 128, 7, register=False)


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("shape", ["two processes", "one process"])
def test_c5_full_size_16gib(tmp_path, shape):
    """C5 at its stated workload (BASELINE.json configs[4]): 16 GiB at the
    test_encoder default of 256 KiB chunks, i.e. 65,536 chunks, each verified on
    the GPU on receipt (ChunkMethods.cpp:137-225) before it is written, with
    every 1000th chunk corrupted on the wire once.  The seeder serves the
    generated stream (no 16 GiB seeder file); the leecher's 16 GiB file must pass
    the resume verify and equal the stream.  "two processes" is the config's own
    shape (two test_client processes): each peer a fresh process
    with its own HIP runtime on the one GPU; "one process" is the threaded
    harness.  Not in the harness, on purpose: the
    tracker hop (test_tracker.cpp:27-75, TrackerMethods.cpp:26-44), the
    NotifyHaveChunk broadcast (ChunkMethods.cpp:202-211) and the 100 ms loop
    pacing (test_client.cpp:72-76) -- control plane, not the hash path."""
    r = _loopback(tmp_path, 16 << 30, 262144, 4096, 1024, 1000, synthetic=True, threads=16, timeout=840, shape=shape)
    print(f"C5 16 GiB ({shape}):", json.dumps({k: r[k] for k in (
        "seconds", "payload_gibs", "wire_gibs", "verify_latency_us", "accept_latency_us", "leecher", "seeder",
        "encode_flood_s", "process_shape")}))
    assert r["chunks"] == 65536 and r["corrupted_sent"] == 65
    # Latency at the default 10 ms batch deadline: verify =
    # frame arrival -> GPU verdict (before the disk write), accept = arrival ->
    # chunk written and marked.  With two verifiers and the GPU decode (the
    # defaults since round 4) five fresh-box runs measured verify p90 8.6-8.7
    # and p99 10.8-11.4 ms (worst arrival 18.5-19.7 ms), accept p90 11.5 and
    # p99 14.7-15.7 ms (profiles/r04/b64/c5_ab_pool.jsonl, r04/s14/).  The
    # bounds sit at about 3x the p90 and 4.5x the p99; the session-3 tree
    # (verify p90 180, p99 252 ms, profiles/r03/suite_s3_failed_c5_p99.txt)
    # and round 3's shipped shape (p99 up to 60 ms) fail them.
    assert r["deadline_ms"] == 10 and r["verifiers"] == 2 and r["gpu_decode"] is True
    v, a = r["verify_latency_us"], r["accept_latency_us"]
    assert v["p90"] < 25_000 and v["p99"] < 50_000, v
    assert a["p90"] < 30_000 and a["p99"] < 60_000, a


@pytest.mark.gpu
def test_per_chunk_base64encode_resume_loop_cost(tmp_path):
    """The reference's resume verify unchanged (Flood.cpp:259-275: Base64Encode
    once per chunk) over a 64 MiB file at 256 KiB chunks, against the batched
    Flood::SetupFilesAndChunks and the same loop on one host core
    (tests/c/per_chunk_resume.cpp).  All three must give the same chunkmap;
    the times are printed for INTEGRATION.md (VERDICT r03 "Next round" #3)."""
    exe = os.path.join(ROOT, "tests", "c", "build", "per_chunk_resume")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "c")])
    r = subprocess.run([exe, str(tmp_path), "64", "256"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr[-2000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    print("per-chunk resume loop:", json.dumps(out))
    assert out["chunkmaps_equal"] is True and out["chunks"] == 256
    # the batched call beats the per-chunk loop it replaces
    assert out["batched_setup_files_and_chunks_s"] < out["per_chunk_base64encode_gpu_s"]


def test_expected_xml_helper_matches_cpp_unit_case():
    # the same model as host_tests.cpp kExpected, built by the Python restatement
    x = expected_xml([("a.bin", 70000, [("LgAPp+hXWcf0wlTU2cM+9IHkWac", 0, 65536, 0),
                                         ("qZk+NkcGgWq6PiVxeFDCbJzQ2J0", 1, 4464, 0)]),
                      ('b&c"<d>\n.bin', 0, [])], [("127.0.0.1", 10101)])
    assert x.startswith('\n<BitFlood>\n\n  <FileInfo>\n    <File name="a.bin" size="70000">')
    assert '<File name="b&amp;c&quot;&lt;d>&#xA;.bin" size="0"/>' in x
    assert x.endswith('\n\n  <Tracker host="127.0.0.1" port="10101"/>\n\n</BitFlood>')


@pytest.mark.skipif(_capi.device_count() > 0, reason="only meaningful without a GPU")
def test_encoder_cli_fails_loudly_without_gpu(tmp_path):
    f = tmp_path / "x.bin"
    f.write_bytes(b"abc")
    out = subprocess.run([ENCODER, str(f), "http://127.0.0.1:10101/", str(tmp_path / "x.flood")],
                         capture_output=True, text=True)
    assert out.returncode == 2
    assert "no CPU fallback" in out.stderr


def test_encoder_cli_usage():
    out = subprocess.run([ENCODER, "only-one-arg"], capture_output=True, text=True)
    assert out.returncode == 1
    assert "three arguments" in out.stderr


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("crlf", [False, True])
def test_encoder_cli_c1(tmp_path, oracle, golden, crlf):
    """C1: one 16 MiB file at 64 KiB chunks -> flood file, byte-exact."""
    c1 = golden("c1.json")
    (tmp_path / "c1.bin").write_bytes(oracle.synth(c1["seed"], 0, c1["size"]).tobytes())
    args = [ENCODER, "c1.bin", "http://127.0.0.1:10101/", "c1.flood", "--chunksize", str(c1["chunk_size"])]
    if crlf:
        args.append("--crlf")
    out = subprocess.run(args, cwd=tmp_path, capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    chunks = [(h, i, c1["chunk_size"], 0) for i, h in enumerate(c1["b64"])]
    want = expected_xml([("c1.bin", c1["size"], chunks)], [("127.0.0.1", 10101)])
    if crlf:
        want = want.replace("\n", "\r\n")
    assert (tmp_path / "c1.flood").read_bytes() == want.encode()


@pytest.mark.gpu
def test_encoder_cli_default_chunksize_odd_tail(tmp_path, oracle, golden):
    o = golden("c1.json")["odd_tail"]
    (tmp_path / "odd.bin").write_bytes(oracle.synth(o["seed"], 0, o["size"]).tobytes())
    out = subprocess.run([ENCODER, "odd.bin", "http://localhost:4000/", "odd.flood"], cwd=tmp_path,
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    n = len(o["b64"])
    sizes = [262144] * (n - 1) + [o["size"] - 262144 * (n - 1)]
    chunks = [(h, i, sizes[i], 0) for i, h in enumerate(o["b64"])]
    assert (tmp_path / "odd.flood").read_text() == expected_xml([("odd.bin", o["size"], chunks)],
                                                                [("localhost", 4000)])


@pytest.mark.gpu
def test_encoder_cli_empty_file(tmp_path):
    (tmp_path / "empty.bin").write_bytes(b"")
    out = subprocess.run([ENCODER, "empty.bin", "http://127.0.0.1:1/", "e.flood"], cwd=tmp_path,
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert (tmp_path / "e.flood").read_text() == expected_xml([("empty.bin", 0, [])], [("127.0.0.1", 1)])


@pytest.mark.gpu
def test_verify_cli_resume(tmp_path, oracle):
    """Flood.cpp:220-299 batched: intact -> all '1'; a flipped byte, a
    truncated tail and a missing file -> '0' exactly there."""
    cs = 65536
    data = oracle.synth(77, 0, 10 * cs + 999)
    (tmp_path / "f.bin").write_bytes(data.tobytes())
    assert subprocess.run([ENCODER, "f.bin", "http://127.0.0.1:10101/", "f.flood", "--chunksize", str(cs)],
                          cwd=tmp_path).returncode == 0

    def verify():
        out = subprocess.run([VERIFY, "f.flood", "--no-resolve"], cwd=tmp_path, capture_output=True, text=True)
        assert out.returncode == 0, out.stderr
        lines = dict(line.split(" ", 1) for line in out.stdout.strip().splitlines())
        return lines

    r = verify()
    assert r["f.bin"] == "11 11 " + "1" * 11
    # content hash: Base64Encode(name + every chunk hash), FloodFile.cpp:324-349
    hashes = [b64_27(hashlib.sha1(data[i * cs:(i + 1) * cs].tobytes()).digest()) for i in range(11)]
    want = b64_27(hashlib.sha1(("f.bin" + "".join(hashes)).encode()).digest())
    assert r["content_hash"] == want
    assert r["to_download"] == "0"

    bad = data.copy()
    bad[3 * cs + 5] ^= 0xFF
    (tmp_path / "f.bin").write_bytes(bad[: 8 * cs + 10].tobytes())  # corrupt chunk 3, cut inside chunk 8
    r = verify()
    assert r["f.bin"] == "11 7 " + "111011110" + "00"
    assert r["to_download"] == "4"
    os.remove(tmp_path / "f.bin")
    r = verify()
    assert r["f.bin"] == "11 0 " + "0" * 11


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["default", "--ref-u32-size", "--true-size"])
def test_encoder_cli_file_past_4gib(tmp_path, form):
    """A 4 GiB + 12,345 B sparse file at 256 KiB chunks through EncodeFile and the
    resume verify.  The flood file's size attribute is the reference's wrapped
    U32 (Encoder.cpp:42,59,76: 12345) unless --true-size; either way lbf_verify
    reads it back and lays chunk 16,384 out at byte 4 GiB (the reference's U32
    offset would be 0), so damaging exactly that chunk flips exactly its bit."""
    cs, size = 262144, (4 << 30) + 12345
    n = size // cs + 1
    f = tmp_path / "big.bin"
    rng = np.random.default_rng(4)
    marks = {0: rng.integers(0, 256, 1000, dtype=np.uint8), 8192 * cs + 77: rng.integers(0, 256, 5000, dtype=np.uint8),
             (n - 2) * cs + cs - 300: rng.integers(0, 256, 300, dtype=np.uint8),
             (n - 1) * cs: rng.integers(0, 256, 12345, dtype=np.uint8)}
    with open(f, "wb") as fh:
        fh.truncate(size)
        for off, b in marks.items():
            fh.seek(off)
            fh.write(b.tobytes())

    def chunk_hash(k):
        b = bytearray(min(cs, size - k * cs))
        for off, m in marks.items():
            lo, hi = max(off, k * cs), min(off + m.size, k * cs + len(b))
            if lo < hi:
                b[lo - k * cs:hi - k * cs] = m[lo - off:hi - off].tobytes()
        return b64_27(hashlib.sha1(bytes(b)).digest())

    args = [ENCODER, "big.bin", "http://127.0.0.1:10101/", "big.flood"] + ([] if form == "default" else [form])
    out = subprocess.run(args, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    xml = (tmp_path / "big.flood").read_text()
    want_size = size if form == "--true-size" else size % (1 << 32)
    assert f'<File name="big.bin" size="{want_size}">' in xml
    assert xml.count("<Chunk ") == n
    zero = b64_27(hashlib.sha1(bytes(cs)).digest())
    for k in (0, 1, 8192, 8193, n - 2, n - 1):
        want = chunk_hash(k)
        assert f'<Chunk hash="{want}" index="{k}" size="{min(cs, size - k * cs)}" weight="0"/>' in xml, k
    assert xml.count(f'hash="{zero}"') == n - 4  # every chunk without a mark is zeros

    def verify():
        r = subprocess.run([VERIFY, "big.flood", "--no-resolve"], cwd=tmp_path, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr
        return dict(line.split(" ", 1) for line in r.stdout.strip().splitlines())

    assert verify()["big.bin"] == f"{n} {n} " + "1" * n
    with open(f, "r+b") as fh:  # one byte of the chunk that starts at 4 GiB
        fh.seek((n - 1) * cs + 6000)
        fh.write(b"\xff" if marks[(n - 1) * cs][6000] != 0xFF else b"\x00")
    assert verify()["big.bin"] == f"{n} {n - 1} " + "1" * (n - 1) + "0"


@pytest.mark.gpu
def test_cpp_api_gpu_suite(tmp_path):
    out = subprocess.run([os.path.join(LIB, "lbf_gpu_tests"), str(tmp_path)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr + out.stdout
    assert "gpu_tests OK" in out.stdout


def test_wire_and_floodfile_parsers_fuzz_asan(tmp_path):
    """Mutated peer frames and flood files through the parsers in an
    ASAN/UBSan build of the host code (tools/fuzz_wire.cpp)."""
    src = [os.path.join(ROOT, "tools", "fuzz_wire.cpp")] + [
        os.path.join(ROOT, "bitflood_amd", "host", f) for f in ("PeerWire.cpp", "FloodFile.cpp", "Encoder.cpp", "Flood.cpp")]
    exe = str(tmp_path / "fuzz_wire")
    cc = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                         "-I" + os.path.join(ROOT, "include"), *src, "-L" + LIB, "-llbfhash", "-Wl,-rpath," + LIB,
                         "-lpthread", "-o", exe], capture_output=True, text=True)
    if cc.returncode != 0 and "sanitizer" in cc.stderr:
        pytest.skip("no sanitizer runtime: " + cc.stderr[-200:])
    assert cc.returncode == 0, cc.stderr
    out = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=300,
                         env={**os.environ, "UBSAN_OPTIONS": "halt_on_error=1", "ASAN_OPTIONS": "detect_leaks=0"})
    assert out.returncode == 0, out.stderr[-3000:]
    assert "fuzz_wire OK 20000" in out.stdout
