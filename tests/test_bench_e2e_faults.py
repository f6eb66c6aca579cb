"""bench.py's host-memory leg (e2e_leg) must not take the line down with it.

At N > 1 the device-resident `value` is measured first, then every rank runs
the copy-inclusive passes together.  A rank whose context, pass or
registration fails must record the failure and still take part in every
collective, so the other ranks finish and rank 0 prints the line.  On CPU the
GPU context cannot be created, which is itself the failure under test; the
two-rank case swaps in a fake hasher (the oracle standing in for the GPU on
rank 0, an injected failure on rank 1)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_e2e_leg_without_gpu_records_the_error():
    data = np.zeros(1 << 20, dtype=np.uint8)
    r = bench.e2e_leg(data, 262144, 0, 1)
    assert r["error"] and r["error"].startswith("lbf_ctx_create")
    assert r["pageable_agg"] == 0.0 and r["registered_agg"] == 0.0
    assert r["digests"] is None and r["registered_equal"] is False


class _FakeHasher:
    """ChunkHasher's surface as e2e_leg uses it; fails on call `fail_at` if set."""
    fail_at = None

    def __init__(self, device_mask=0):
        from tests.oracle_lib import Oracle
        self.orc = Oracle()
        self.calls = 0
        self.direct = 0

    def hash_chunks(self, data, offs, sizes):
        self.calls += 1
        if self.fail_at is not None and self.calls >= self.fail_at:
            raise RuntimeError("injected staging failure")
        return self.orc.sha1_batch(data, offs, sizes)

    def worker_info(self, w=0):
        return {"device": 0, "numa_node": 0, "staging_node": 0, "bound_cpus": 1}

    def register_host(self, data):
        pass

    def unregister_host(self, data):
        pass

    def staging_stats(self):
        return {"staged": 0, "direct": self.direct}

    def close(self):
        pass


def _rank(rank, world, port, out_dir, fail_rank, fail_at):
    import torch.distributed as dist

    import bitflood_amd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class Fake(_FakeHasher):
        pass
    Fake.fail_at = fail_at if rank == fail_rank else None
    bitflood_amd.ChunkHasher = Fake  # e2e_leg imports it from the package at call time
    data = np.arange(3 * 65536 + 77, dtype=np.uint32).view(np.uint8)[: 3 * 65536 + 77].copy()
    r = bench.e2e_leg(data, 65536, 0, world)
    np.save(os.path.join(out_dir, f"d{rank}.npy"), r["digests"] if r["digests"] is not None else np.zeros(0))
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(f"{r['error']}|{r['pageable_agg']}|{r['registered_agg']}|{r['registered_equal']}")
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path, fail_rank, fail_at):
    mp.spawn(_rank, args=(2, _free_port(), str(tmp_path), fail_rank, fail_at), nprocs=2, join=True)
    out = []
    for r in range(2):
        err, pag, reg, eq = open(tmp_path / f"r{r}.txt").read().split("|")
        out.append((err, float(pag), float(reg), eq == "True", np.load(tmp_path / f"d{r}.npy")))
    return out


def test_e2e_leg_all_ranks_ok_gloo(tmp_path):
    (e0, p0, g0, q0, d0), (e1, p1, g1, q1, d1) = _run(tmp_path, fail_rank=-1, fail_at=None)
    assert e0 == "None" and e1 == "None"
    assert p0 > 0 and g0 > 0 and q0 and q1
    assert d0.shape == (4, 20) and np.array_equal(d0, d1)


def test_e2e_leg_one_rank_fails_mid_leg_the_others_finish(tmp_path):
    # rank 1 fails on its third hash call (the second pageable pass): both ranks
    # return, rank 0 keeps its digests, and the aggregate of the passes rank 1
    # missed reads 0 rather than hanging
    (e0, p0, g0, q0, d0), (e1, p1, g1, q1, d1) = _run(tmp_path, fail_rank=1, fail_at=3)
    assert e0 == "None"
    assert e1.startswith("hash pass: RuntimeError: injected staging failure")
    assert d0.shape == (4, 20) and q0
    assert g0 == 0.0 and g1 == 0.0  # the registered passes: rank 1 reported an infinite time
    assert p0 > 0  # the first pageable pass completed on both ranks


def test_e2e_leg_one_rank_fails_its_first_pass(tmp_path):
    (e0, p0, g0, q0, d0), (e1, p1, g1, q1, d1) = _run(tmp_path, fail_rank=0, fail_at=1)
    assert e0.startswith("warm pass: RuntimeError")
    assert e1 == "None" and d1.shape == (4, 20)
    assert p1 == 0.0 and g1 == 0.0
