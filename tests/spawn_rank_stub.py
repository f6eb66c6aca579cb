"""A rank process for tests/test_bench_spawn.py: what bench.py's rank does,
with the oracle standing in for the GPU (this container has none).

It reads the environment bench.spawn_ranks() sets, forms the process group
through bench.dist_setup's contract (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*,
LBF_BENCH_BACKEND), hashes its contiguous shard of a small synthetic file,
checks it against hashlib, all-gathers the flags with bench.gather_ints and
the timings with bench.gather_floats / max_over_ranks, and rank 0 prints one
JSON line.  STUB_FAIL_RANK=r makes rank r exit 3 before joining the group."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from bitflood_amd.sharding import max_over_ranks, shard_range  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if int(os.environ.get("STUB_FAIL_RANK", "-1")) == rank:
        sys.exit(3)
    dist.init_process_group(os.environ["LBF_BENCH_BACKEND"], rank=rank, world_size=world)
    orc = Oracle()
    cs, per = 4096, 24
    first, last = shard_range(world * per, rank, world)
    t0 = time.perf_counter()
    data = orc.synth(0x5EED, first * cs, (last - first) * cs)
    d = orc.encode_buffer(data, cs)
    ok = all(bytes(d[i]) == hashlib.sha1(data[i * cs:(i + 1) * cs].tobytes()).digest() for i in range(len(d)))
    flags = bench.gather_ints(int(ok), world)
    firsts = bench.gather_ints(first, world)
    local = bench.gather_ints(int(os.environ["LOCAL_RANK"]), world)
    t = max_over_ranks(time.perf_counter() - t0, world)
    hashes = bench.gather_ints(bench.slice_hash(d), world)
    if rank == 0:
        full = orc.encode_buffer(orc.synth(0x5EED, 0, world * per * cs), cs)
        want = [bench.slice_hash(full[r * per:(r + 1) * per]) for r in range(world)]
        print(json.dumps({"n_gpus": world, "per_rank": flags, "first_chunk_per_rank": firsts,
                          "local_rank": local, "max_s": t, "slice_hash_ok": hashes == want,
                          "master": [os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"]],
                          "backend": os.environ["LBF_BENCH_BACKEND"],
                          "launcher": os.environ.get("LBF_BENCH_LAUNCHER")}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    np.zeros(1)


if __name__ == "__main__":
    main()
