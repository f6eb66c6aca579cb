"""bench.py's collectives through RCCL on the 1-GPU box (VERDICT r03 "Next round" #1).

Every N>1 run before round 4 formed its process group with gloo (more ranks
than GPUs on the test boxes), so the `nccl` branch of bench.init_group and the
cuda-tensor collectives behind bench._gather, sharding.max_over_ranks and
sharding.gather_digests had never executed -- and they are what the driver's
8-GPU run uses.  A one-rank RCCL group runs all of them on one GPU:

* the helpers themselves, in a fresh process (int64 and float64 all-gathers,
  the MAX all-reduce, a uint8 digest all-gather, barrier, destroy);
* bench.py end to end with LBF_BENCH_FORM_GROUP=1: one rank takes the N>1
  route (device-resident timing, e2e, e2e_inprocess, cpu_baseline) with every
  collective on RCCL.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

_CHILD = r'''
import json, os, sys
sys.path.insert(0, {root!r})
import numpy as np
import torch
import torch.distributed as dist
import bench
from bitflood_amd.sharding import gather_digests, max_over_ranks
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[1])
torch.cuda.set_device(0)
bench.init_group("nccl", 0, 1, 0)
out = {{"grouped": bench.grouped(), "backend": bench.backend_name()}}
out["ints"] = bench.gather_ints(-(1 << 40) - 7, 1)
out["floats"] = bench.gather_floats(3.25, 1)
out["max"] = max_over_ranks(1.5, 1)
bench.barrier(1)
d = np.random.default_rng(5).integers(0, 256, size=(37, 20), dtype=np.uint8)
out["digests_equal"] = bool(np.array_equal(gather_digests(d, 37, 1), d))
dist.destroy_process_group()
out["grouped_after"] = bench.grouped()
print(json.dumps(out), flush=True)
'''


def test_one_rank_rccl_group_runs_the_bench_collectives(tmp_path):
    import bench
    script = tmp_path / "child.py"
    script.write_text(_CHILD.format(root=ROOT))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, str(script), str(bench._free_port())], env=env, capture_output=True,
                       text=True, timeout=180, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert out == {"grouped": True, "backend": "nccl", "ints": [-(1 << 40) - 7], "floats": [3.25], "max": 1.5,
                   "digests_equal": True, "grouped_after": False}, out


def test_bench_one_rank_rccl_group_takes_the_n_rank_route(oracle):
    import bench
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LBF_BENCH_BACKEND")}
    env.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(bench._free_port()),
               LBF_BENCH_FORM_GROUP="1")
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
            "--file-gib", "0.25", "--cpu-min-s", "0.5"]
    p = subprocess.run(args, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["ranks"]["process_group"] == "nccl" and out["n_gpus"] == 1
    for k in ("roofline", "cpu_baseline", "parity", "e2e", "e2e_inprocess"):
        assert k in out, k
    assert "other_configs" not in out  # the N>1 route
    cs, n = 262144, 1024
    data = oracle.synth(0x5EED, 0, n * cs, nthreads=8)
    want = oracle.sha1_batch(data, np.arange(n, dtype=np.uint64) * np.uint64(cs), np.full(n, cs, np.uint32),
                             nthreads=8)
    import hashlib
    assert out["digest_check"] == hashlib.sha1(want.tobytes()).hexdigest()
    assert out["e2e"]["parity_per_rank"] == [1] and out["e2e"]["failed_per_rank"] == [0]
    assert out["e2e_inprocess"].get("parity") is True, out["e2e_inprocess"]
    assert out["cpu_baseline"]["parity_vs_gpu"] is True and out["cpu_baseline"]["value"] > 0
