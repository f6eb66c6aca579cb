"""The shipped library's Makefile rebuilds an object whenever any header it
can include changes (kern_b64.hpp was missing from HDRS,
so an incremental make after editing the wire kernels kept a stale object).
CPU only: reads make's database, builds nothing."""
import glob
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bitflood_amd", "csrc")


def _prereqs(target):
    db = subprocess.run(["make", "-p", "-n", "-q", "-C", CSRC], capture_output=True, text=True).stdout
    for line in db.splitlines():
        if line.startswith(target + ":"):
            return set(line.split(":", 1)[1].split())
    raise AssertionError(f"{target} not in make's database")


def test_every_header_is_a_prerequisite_of_both_objects():
    headers = {os.path.basename(p) for p in glob.glob(os.path.join(CSRC, "*.hpp"))}
    assert "kern_b64.hpp" in headers
    for obj in ("../lib/sha1_kernels.o", "../lib/lbf_capi.o"):
        pre = _prereqs(obj)
        assert headers <= pre, (obj, headers - pre)
        assert "../../include/lbf_hash.h" in pre
