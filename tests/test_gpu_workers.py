"""The multi-worker host path of lbf_ctx on one GPU, and its error paths.

On an 8-GPU node every EncodeFile / SetupFilesAndChunks runs through
run_job's multi-worker branch (bitflood_amd/csrc/lbf_capi.cpp): contiguous
index ranges, one host thread, one set of staging slots per worker, the first
failing worker's status and message returned (the reference's one-thread loop
it replaces: /root/reference/cpp/src/Encoder.cpp:40-79, Flood.cpp:243-285).
LBF_WORKERS_PER_DEVICE=k gives a context k workers on the one GPU of a test
box, so that branch runs here exactly as it would with one worker per device.
Results are compared with the oracle, bit for bit.
"""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from bitflood_amd import ChunkHasher, LbfError, chunk_table
from bitflood_amd import _capi

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "bitflood_amd", "lib")


def _ctx(monkeypatch, **env):
    with monkeypatch.context() as m:  # read at context creation only
        for k, v in env.items():
            m.setenv(k, str(v))
        return ChunkHasher()


def _mixed_table(rng, buf_len, n):
    """Ragged, unaligned chunks plus a few larger than a 2 MiB slot."""
    sizes = rng.integers(0, 300000, n).astype(np.uint32)
    sizes[:20] = np.arange(20) * 7
    sizes[[50, 51, 300]] = [3 << 20, (2 << 20) + 1, 5 << 20]  # oversize: dedicated buffers
    offs = np.array([rng.integers(0, buf_len - s + 1) for s in sizes], dtype=np.uint64)
    offs[::3] &= ~np.uint64(4095)
    return offs, sizes


@pytest.mark.parametrize("workers", [2, 8])
def test_multi_worker_hash_and_verify_memory(workers, oracle, monkeypatch):
    h = _ctx(monkeypatch, LBF_WORKERS_PER_DEVICE=workers, LBF_SLOT_MB=2)
    try:
        assert h.num_workers == workers and h.num_devices == 1
        rng = np.random.default_rng(100 + workers)
        buf = oracle.synth(61, 0, 48 << 20, nthreads=8)
        offs, sizes = _mixed_table(rng, buf.size, 900)
        want = oracle.sha1_batch(buf, offs, sizes, nthreads=8)
        got = h.hash_chunks(buf, offs, sizes)
        bad = np.flatnonzero((got != want).any(axis=1))
        assert bad.size == 0, bad[:10]
        flips = [0, 51, 299, 300, 450, 899]
        exp = want.copy()
        exp[flips, 3] ^= 0x10
        v = h.verify_chunks(buf, offs, sizes, exp)
        assert np.flatnonzero(~v).tolist() == flips
    finally:
        h.close()


@pytest.mark.parametrize("workers", [2, 8])
def test_multi_worker_file_paths(workers, oracle, monkeypatch, tmp_path):
    """lbf_file_ranges split over workers: hash, resume verify of an intact and
    of a truncated file (short chunks verdict 0), and hash mode on the
    truncated file failing with the failing worker's LBF_ERR_IO."""
    h = _ctx(monkeypatch, LBF_WORKERS_PER_DEVICE=workers, LBF_SLOT_MB=4)
    try:
        data = oracle.synth(62, 0, (40 << 20) + 4321, nthreads=8)
        path = tmp_path / "f.bin"
        path.write_bytes(data.tobytes())
        offs, sizes = chunk_table(data.size, 262144 + 7)
        want = oracle.sha1_batch(data, offs, sizes, nthreads=8)
        assert np.array_equal(h.hash_file(str(path), offs, sizes), want)
        assert h.verify_file(str(path), offs, sizes, want).all()
        cut = int(offs[100]) + 5
        short = tmp_path / "short.bin"
        short.write_bytes(data[:cut].tobytes())
        v = h.verify_file(str(short), offs, sizes, want)
        assert v.tolist() == [True] * 100 + [False] * (offs.size - 100)
        with pytest.raises(LbfError) as ei:
            h.hash_file(str(short), offs, sizes)
        assert ei.value.status == _capi.LBF_ERR_IO
        msg = str(ei.value)
        assert "worker" in msg and "device 0" in msg and "chunk 100 could not be read in full" in msg, msg
        # the same context keeps working after the failed job
        o2, s2 = chunk_table(cut, 65536)
        assert np.array_equal(h.hash_file(str(short), o2, s2), oracle.sha1_batch(data[:cut], o2, s2))
    finally:
        h.close()


@pytest.mark.parametrize("kind", ["hip", "throw"])
@pytest.mark.parametrize("workers,fault_worker", [(1, 0), (4, 3)])
def test_injected_fault_drains_before_next_job(workers, fault_worker, kind, oracle, monkeypatch):
    """A failure in the middle of a job (LBF_TEST_FAULT_GROUP: the worker's
    third staging group fails after two are in flight) returns LBF_ERR_HIP for
    a HIP-side error, LBF_ERR_NOMEM for a host exception (which must not cross
    the C ABI); every slot is drained either way, so the next, smaller job on
    the same context gets exactly its own results (a stale pending
    group used to be finalized into the next job's arrays)."""
    h = _ctx(monkeypatch, LBF_WORKERS_PER_DEVICE=workers, LBF_SLOT_MB=8, LBF_TEST_FAULT_GROUP=2,
             LBF_TEST_FAULT_WORKER=fault_worker, LBF_TEST_FAULT_KIND=kind)
    try:
        big = oracle.synth(63, 0, 96 << 20, nthreads=8)
        offs, sizes = chunk_table(big.size, 65536)
        with pytest.raises(LbfError) as ei:
            h.hash_chunks(big, offs, sizes)
        if kind == "hip":
            assert ei.value.status == _capi.LBF_ERR_HIP and "injected fault" in str(ei.value)
        else:
            assert ei.value.status == _capi.LBF_ERR_NOMEM and "host allocation failed while staging" in str(ei.value)
        if workers > 1:
            assert f"worker {fault_worker} " in str(ei.value)
        small = oracle.synth(64, 0, (3 << 20) + 99)
        o2, s2 = chunk_table(small.size, 100003)
        assert np.array_equal(h.hash_chunks(small, o2, s2), oracle.sha1_batch(small, o2, s2))
        exp = oracle.sha1_batch(small, o2, s2)
        exp[7, 0] ^= 1
        assert np.flatnonzero(~h.verify_chunks(small, o2, s2, exp)).tolist() == [7]
        # and the big job itself, now that the one-shot fault is spent
        assert np.array_equal(h.hash_chunks(big, offs, sizes), oracle.sha1_batch(big, offs, sizes, nthreads=8))
    finally:
        h.close()


def test_numa_placement(monkeypatch):
    """Each worker's pinned staging sits on its GPU's NUMA node and its host
    threads are bound to that node's CPUs."""
    h = _ctx(monkeypatch, LBF_WORKERS_PER_DEVICE=2)
    try:
        data = np.arange(64 << 20, dtype=np.uint64).view(np.uint8)
        offs, sizes = chunk_table(data.size, 1 << 20)
        h.hash_chunks(data, offs, sizes)  # allocates the data slots
        for w in range(h.num_workers):
            info = h.worker_info(w)
            print("worker", w, info)
            assert info["device"] == 0
            bus_node = _sysfs_gpu_node()
            if bus_node is None or bus_node < 0:
                assert info["numa_node"] == -1
                continue
            assert info["numa_node"] == bus_node
            assert info["bound_cpus"] > 0
            assert info["staging_node"] == bus_node, info
    finally:
        h.close()


def test_numa_placement_off():
    """LBF_NUMA=0: no node, no binding (read once per process, so a child)."""
    code = ("import torch, json; from bitflood_amd import ChunkHasher\n"
            "h = ChunkHasher(); print(json.dumps(h.worker_info(0))); h.close()")
    out = subprocess.run(["python", "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120,
                         env={**os.environ, "LBF_NUMA": "0"})
    assert out.returncode == 0, out.stderr
    info = json.loads(out.stdout.strip().splitlines()[-1])
    assert info["numa_node"] == -1 and info["bound_cpus"] == 0, info


def _sysfs_gpu_node():
    """NUMA node of GPU 0 from sysfs, read independently of the library."""
    out = subprocess.run(["rocm-smi", "--showbus"], capture_output=True, text=True)
    for line in out.stdout.splitlines():
        if "PCI Bus" in line and "GPU[0]" in line:
            bus = line.split("PCI Bus:")[1].strip().lower()
            try:
                return int(open(f"/sys/bus/pci/devices/{bus}/numa_node").read())
            except OSError:
                return None
    return None


@pytest.mark.parametrize("workers", [2, 8])
def test_encode_file_cli_multi_worker(workers, tmp_path, oracle, golden):
    """Encoder::EncodeFile (Encoder.cpp:17-102) through the test_encoder port
    with the process-wide context split over `workers` workers: the C1 flood
    file's chunk hashes equal the goldens; the resume-verify CLI agrees."""
    from tests.test_host_cpp import expected_xml
    c1 = golden("c1.json")
    (tmp_path / "c1.bin").write_bytes(oracle.synth(c1["seed"], 0, c1["size"]).tobytes())
    env = {**os.environ, "LBF_WORKERS_PER_DEVICE": str(workers), "LBF_SLOT_MB": "2"}
    # --devices 1: Encoder::SetDeviceMask(1) before first use, then k workers on device 0
    out = subprocess.run([os.path.join(LIB, "lbf_encoder"), "c1.bin", "http://127.0.0.1:10101/", "c1.flood",
                          "--chunksize", str(c1["chunk_size"]), "--devices", "1"], cwd=tmp_path, capture_output=True,
                         text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stderr
    chunks = [(hh, i, c1["chunk_size"], 0) for i, hh in enumerate(c1["b64"])]
    assert (tmp_path / "c1.flood").read_text() == expected_xml([("c1.bin", c1["size"], chunks)],
                                                               [("127.0.0.1", 10101)])
    data = (tmp_path / "c1.bin").read_bytes()
    bad = bytearray(data)
    bad[37 * c1["chunk_size"] + 3] ^= 1
    (tmp_path / "c1.bin").write_bytes(bytes(bad))
    out = subprocess.run([os.path.join(LIB, "lbf_verify"), "c1.flood", "--no-resolve", "--devices", "1"], cwd=tmp_path,
                         capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = dict(line.split(" ", 1) for line in out.stdout.strip().splitlines())
    n = len(c1["b64"])
    assert lines["c1.bin"] == f"{n} {n - 1} " + "1" * 37 + "0" + "1" * (n - 38)
    assert hashlib.sha1(data).hexdigest() != hashlib.sha1(bytes(bad)).hexdigest()
