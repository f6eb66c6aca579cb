"""Many-file batches against the process's descriptor limit.

EncodeFile / SetupFilesAndChunks hand a whole flood to one lbf_files_ranges
call.  The reference opens one file at a time (Encoder.cpp:40-79,
Flood.cpp:239-287), so a flood with more files than RLIMIT_NOFILE must still
hash, and verify must never turn "too many open files" into verdict 0 (which
would queue intact chunks for re-download and overwrite).  The call now runs
one job per window of files (a quarter of the soft limit, LBF_FILES_WINDOW
overrides) and reports EMFILE/ENFILE as LBF_ERR_IO."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, resource, sys
sys.path.insert(0, {root!r})
import numpy as np
from bitflood_amd import ChunkHasher, LbfError
resource.setrlimit(resource.RLIMIT_NOFILE, ({soft}, resource.getrlimit(resource.RLIMIT_NOFILE)[1]))
d = {tmp!r}
paths = [os.path.join(d, f"f{{i:03d}}.bin") for i in range({nfiles})]
sizes_of = json.load(open(os.path.join(d, "sizes.json")))
fo, offs, szs = [], [], []
for f, sz in enumerate(sizes_of):   # chunks listed file-major but interleaved in pairs
    for k in range((sz + {cs} - 1) // {cs}):
        fo.append(f); offs.append(k * {cs}); szs.append(min({cs}, sz - k * {cs}))
order = np.random.default_rng(5).permutation(len(fo))
fo, offs, szs = [np.array(x)[order] for x in (fo, offs, szs)]
out = {{}}
with ChunkHasher() as h:
    try:
        dig = h.hash_files(paths, fo, offs, szs)
        out["hash"] = [bytes(x).hex() for x in dig]
    except LbfError as e:
        out["hash_error"] = str(e)
    exp = np.frombuffer(bytes.fromhex("".join(out.get("hash", ["00" * 20] * len(fo)))), np.uint8).reshape(-1, 20)
    os.rename(paths[3], paths[3] + ".gone")   # one file missing: its chunks '0'
    try:
        out["verify"] = h.verify_files(paths, fo, offs, szs, exp).astype(int).tolist()
    except LbfError as e:
        out["verify_error"] = str(e)
    os.rename(paths[3] + ".gone", paths[3])
out["fo"] = fo.tolist(); out["offs"] = offs.tolist(); out["szs"] = szs.tolist()
print(json.dumps(out))
'''


def _files(tmp_path, nfiles, cs):
    rng = np.random.default_rng(9)
    sizes = [int(rng.integers(0, 3 * cs + 50)) for _ in range(nfiles)]
    for i, sz in enumerate(sizes):
        (tmp_path / f"f{i:03d}.bin").write_bytes(rng.integers(0, 256, sz, dtype=np.uint8).tobytes())
    (tmp_path / "sizes.json").write_text(json.dumps(sizes))
    return sizes


def _run(tmp_path, nfiles, cs, soft, env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    code = CHILD.format(root=ROOT, soft=soft, tmp=str(tmp_path), nfiles=nfiles, cs=cs)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_more_files_than_descriptor_limit(tmp_path):
    """400 files under a soft limit of 128 descriptors: windows of 32 files,
    hash equals hashlib chunk by chunk, verify gives '1' everywhere but on the
    missing file."""
    nfiles, cs = 400, 4096
    _files(tmp_path, nfiles, cs)
    out = _run(tmp_path, nfiles, cs, 128)
    assert "hash_error" not in out and "verify_error" not in out, out
    for k, (f, o, s) in enumerate(zip(out["fo"], out["offs"], out["szs"])):
        data = (tmp_path / f"f{f:03d}.bin").read_bytes()[o:o + s]
        assert out["hash"][k] == hashlib.sha1(data).hexdigest(), k
        assert out["verify"][k] == (0 if f == 3 else 1), k


@pytest.mark.gpu
def test_emfile_is_an_error_not_verdict_zero(tmp_path):
    """With the window forced above the limit, open() fails with EMFILE partway:
    hash and verify both fail loudly (LBF_ERR_IO, 'too many open files')."""
    nfiles, cs = 300, 4096
    _files(tmp_path, nfiles, cs)
    out = _run(tmp_path, nfiles, cs, 128, {"LBF_FILES_WINDOW": "100000"})
    assert "too many open files" in out.get("hash_error", ""), out.keys()
    assert "too many open files" in out.get("verify_error", ""), out.keys()
