"""INTEGRATION.md's reference-side shim is real code.

The shim (a replacement `cpp/src/Encoder.cpp` over the C ABI) is compiled,
syntax only, against this repo's mirror of the reference headers
(include/libBitFlood/, same names and types as cpp/src/*.H) and
include/lbf_hash.h, with a stand-in for the reference's precompiled-header
include.  No GPU needed.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integration_shim_compiles(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"```cpp\n(// cpp/src/Encoder.cpp \(replacement\).*?)```", text, re.S)
    assert m, "shim block not found in INTEGRATION.md"
    (tmp_path / "Encoder_shim.cpp").write_text(m.group(1))
    (tmp_path / "stdafx.H").write_text("#pragma once\n#include <algorithm>\n#include <string>\n#include <vector>\n")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", f"-I{tmp_path}",
                        "-I" + os.path.join(ROOT, "include", "libBitFlood"), "-I" + os.path.join(ROOT, "include"),
                        str(tmp_path / "Encoder_shim.cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    for sym in ("lbf_files_ranges", "lbf_sha1_one", "lbf_b64_27", "lbf_ctx_create"):
        assert sym in m.group(1)
