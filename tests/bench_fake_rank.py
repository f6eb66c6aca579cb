"""bench.py's own main() on a CPU-only host, for tests/test_bench_spawn.py.

TEST INFRASTRUCTURE.  This container has no GPU, so the few device calls
bench.main() makes are pointed at host stand-ins before it runs: device
buffers are numpy arrays, the chunk-hash launch and the lbf_ctx host-memory
batches hash with the oracle, HIP events read the host clock.  Everything
else -- the spawner's environment, the process group, every collective and
the assembly of rank 0's JSON line (roofline, cpu_baseline, parity, e2e,
e2e_inprocess) -- is bench.py's code as the driver runs it, so the test can
check the key set of an N>1 line.

Run as a rank by bench.spawn_ranks(n, argv, script=<this file>).
"""
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import bitflood_amd  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402

ORC = Oracle()
NDEV = int(os.environ.get("FAKE_NDEV", "1"))


class FakeDeviceBuffer:
    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.arr = np.zeros(self.nbytes, dtype=np.uint8)
        self.ptr = 1

    def free(self):
        self.arr, self.ptr = None, None

    def fill_synthetic(self, seed, start=0, nbytes=None, stream=None, offset=0):
        nbytes = self.nbytes - offset if nbytes is None else nbytes
        self.arr[offset:offset + nbytes] = ORC.synth(seed, start, nbytes)

    def download(self, nbytes=None, offset=0, dtype=np.uint8):
        nbytes = self.nbytes - offset if nbytes is None else nbytes
        return self.arr[offset:offset + nbytes].copy().view(dtype)

    def download_into(self, out, offset=0):
        out[...] = self.arr[offset:offset + out.nbytes].view(out.dtype).reshape(out.shape)


def _uniform(data, length, cs, first, n):
    offs = (np.arange(n, dtype=np.uint64) + np.uint64(first)) * np.uint64(cs)
    sizes = np.minimum(np.uint64(cs), np.uint64(length) - offs).astype(np.uint32)
    return ORC.sha1_batch(data, offs, sizes, nthreads=2)


def fake_uniform_launch(base, length, cs, first, n, digests, expected=None, verdicts=None, stream=None):
    d = _uniform(base.arr, length, cs, first, n)
    digests.arr[:n * 20] = d.reshape(-1)


class FakeLib:
    @staticmethod
    def lbf_kernel_for(n):
        return 7 if n <= 16384 else (12 if n <= 32768 else 11)


fake_H = types.SimpleNamespace(uniform_launch=fake_uniform_launch, load=lambda: FakeLib(),
                               synchronize=lambda: None, set_kernel_variant=lambda v: None)


class FakeChunkHasher:
    def __init__(self, device_mask=0):
        self.num_devices = NDEV if device_mask == 0 else bin(device_mask).count("1")
        self.num_workers = self.num_devices
        self._direct = 0
        self._registered = set()

    def hash_chunks(self, data, offsets, sizes):
        if data.ctypes.data in self._registered:
            self._direct += int(np.asarray(sizes, dtype=np.uint64).sum())
        return ORC.sha1_batch(data, offsets, sizes, nthreads=2)

    def worker_info(self, w=0):
        return {"device": w, "numa_node": 0, "staging_node": 0, "bound_cpus": 1}

    def register_host(self, data):
        self._registered.add(data.ctypes.data)

    def unregister_host(self, data):
        self._registered.discard(data.ctypes.data)

    def staging_stats(self):
        return {"staged": 0, "direct": self._direct}

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class FakeEvent:
    def __init__(self, enable_timing=False):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


def install():
    torch.cuda.device_count = lambda: NDEV
    torch.cuda.set_device = lambda d: None
    torch.cuda.current_device = lambda: 0
    torch.cuda.synchronize = lambda *a: None
    torch.cuda.current_stream = lambda *a: types.SimpleNamespace(cuda_stream=None)
    torch.cuda.Event = FakeEvent
    bench.DeviceBuffer = FakeDeviceBuffer
    bench.H = fake_H
    bitflood_amd.ChunkHasher = FakeChunkHasher
    if os.environ.get("FAKE_CPU_BASELINE_FAILS") == "1":
        def failing_cpu_baseline(*a, **k):
            raise OSError("injected: the host comparator cannot run")
        bench.cpu_baseline = failing_cpu_baseline


if __name__ == "__main__":
    install()
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
    bench.main()
