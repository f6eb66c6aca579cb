"""bench.py's multi-rank flow on the GPU box, launched the way a driver runs it:
`python bench.py --gpus 2` with no launcher (bench.py starts its own ranks).
With one GPU the two ranks share it under gloo (a rehearsal); what is checked
is the flow: two ranks, each rank's device-resident digests equal the oracle
on its shard, and the N-rank host-memory legs (e2e, e2e_inprocess) report
parity, and rank 0's cpu_baseline is in the line.  Small shards (256 MiB per
rank) keep it to seconds."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_bench_self_launched_two_ranks(oracle):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["LBF_BENCH_BACKEND"] = "gloo"
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
            "--file-gib", "0.25", "--cpu-min-s", "0.5"]
    p = subprocess.run(args, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["ranks"]["launcher"] == "bench.py" and len(out["ranks"]["kernel_ms_per_rank"]) == 2
    assert out["parity"]["per_rank"] == [-1, -1]  # no golden at this size; checked against the oracle below
    cs, per = 262144, 1024
    # rank 0's digests: chunks [0, 1024) of the 2 x 256 MiB stream
    data = oracle.synth(0x5EED, 0, per * cs, nthreads=8)
    want = oracle.sha1_batch(data, np.arange(per, dtype=np.uint64) * np.uint64(cs), np.full(per, cs, np.uint32),
                             nthreads=8)
    assert out["digest_check"] == hashlib.sha1(want.tobytes()).hexdigest()
    e2e = out["e2e"]
    assert e2e["parity_per_rank"] == [1, 1] and e2e["bytes_per_rank"] == per * cs
    assert e2e["pageable"]["aggregate_gibs"] > 0 and len(e2e["registered"]["per_rank_gibs"]) == 2
    inproc = out["e2e_inprocess"]
    assert "error" not in inproc, inproc
    assert inproc["parity"] is True and inproc["parity_per_slice"] == [1, 1] and inproc["bytes"] == 2 * per * cs
    # the CPU comparator is in the N>1 line too, timed by rank 0 after the other rank finished
    cb = out["cpu_baseline"]
    assert cb["parity_vs_gpu"] is True and cb["value"] > 0 and "rank 0 alone" in cb["when"]
