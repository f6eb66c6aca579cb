#!/usr/bin/env python3
"""Per-kernel digests of the gfx950 ISA of a HIP source (instruction lines only).

    python tools/isa_digest.py [SRC] [--record tests/golden/isa_shipped.json]

Compiles SRC (default: the shipped bitflood_amd/csrc/sha1_kernels.hip) with the
shipped flags to device assembly, splits it into kernels at their `.type ...,
@function` / `.Lfunc_end` markers and hashes each kernel's instruction stream
(directives, labels' own names and comments dropped; branch targets renamed to
their order of appearance, so a renumbered label is not a change).  tests/test_isa.py
compares the shipped kernels with the recorded digests: a refactor that moves
code between files must leave them unchanged.
"""
import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CSRC = os.path.join(ROOT, "bitflood_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def compile_s(src, out, extra=()):
    r = subprocess.run([HIPCC, *FLAGS, *extra, "--offload-device-only", "-S", "-o", out, src],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-3000:])


def kernels(asm_text):
    """{mangled kernel name: [normalised instruction lines]}"""
    out, cur, name = {}, None, None
    for raw in asm_text.splitlines():
        line = raw.split(";")[0].rstrip()
        s = line.strip()
        if not s:
            continue
        m = re.match(r"\.type\s+([\w.$]+),@function", s)
        if m:
            name, cur = m.group(1), []
            continue
        if name is None:
            continue
        if s.startswith(".Lfunc_end"):
            out[name] = cur
            name, cur = None, None
            continue
        if s.startswith("."):
            if s.endswith(":"):
                cur.append("<label>")
            continue
        if s.endswith(":"):
            continue  # the kernel's own symbol
        cur.append(s)
    # branch targets by order of first appearance
    for k, ins in out.items():
        ren = {}

        def sub(m):
            return ren.setdefault(m.group(0), f".L{len(ren)}")
        out[k] = [re.sub(r"\.LBB\d+_\d+", sub, i) for i in ins]
    return out


def digests(src, extra=()):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        compile_s(src, out, extra)
        ks = kernels(open(out).read())
    return {k: {"instructions": len(v), "sha256": hashlib.sha256("\n".join(v).encode()).hexdigest()}
            for k, v in sorted(ks.items())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="?", default=os.path.join(CSRC, "sha1_kernels.hip"))
    ap.add_argument("--record", help="write the digests to this JSON file")
    a = ap.parse_args()
    d = digests(a.src)
    if a.record:
        with open(a.record, "w") as f:
            json.dump({"source": os.path.relpath(a.src, ROOT), "hipcc_flags": FLAGS[:3], "kernels": d}, f,
                      indent=1, sort_keys=True)
            f.write("\n")
    json.dump(d, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
