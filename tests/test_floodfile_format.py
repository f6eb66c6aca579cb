"""Flood-file layout pinned by a fixture the reference holds.

The reference writes flood files with its vendored Xerces-C 2.6.0 DOMWriter
(cpp/src/FloodFile.cpp:42-142).  No flood file exists in the reference, but
Xerces' own test suite holds DOMWriter pretty-print output
(cpp/extern/xercesc++/2.6.0/tests/DOM/Normalizer/expectedOutput), extracted
as data by tests/golden/make_xerces_fixture.py.  Every element-only document
there must come out of the restatement (tests/domwriter.py) byte for byte;
the C++ writer is then checked against the same restatement
(tests/test_host_cpp.py, host_tests.cpp).  This pins the layout -- newlines,
indentation, blank lines, "/>" -- by the reference's own fixture.  The
attribute order follows from the reference's setAttribute calls, which are in
name order already (FloodFile.cpp:74-75,95-98,115-116), so sorted and
insertion order agree; only the escapes rest on code reading (no fixture holds
a character that needs one).
"""
import json
import os

from tests.domwriter import parse, pretty

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "xerces260_domwriter_pretty.json")


def test_domwriter_restatement_reproduces_xerces_fixture():
    fx = json.load(open(GOLDEN))
    assert fx["source"].endswith("tests/DOM/Normalizer/expectedOutput")
    assert len(fx["docs"]) >= 10
    depths = set()
    for doc in fx["docs"]:
        tree = parse(doc)
        assert pretty(tree) == doc

        def depth(n, d=0):
            return max([d] + [depth(k, d + 1) for k in n[2]])
        depths.add(depth(tree))
    assert max(depths) >= 3  # a flood file nests to level 3 (BitFlood/FileInfo/File/Chunk)


def test_restatement_is_the_flood_layout():
    # the flood-file builder used against the C++ writer is this same pretty()
    from tests.test_host_cpp import expected_xml
    x = expected_xml([("a.bin", 70000, [("LgAPp+hXWcf0wlTU2cM+9IHkWac", 0, 65536, 0)]), ("e.bin", 0, [])],
                     [("127.0.0.1", 10101)])
    assert x == pretty(parse(x))
    assert x == ('\n<BitFlood>\n\n  <FileInfo>\n    <File name="a.bin" size="70000">\n      <Chunk '
                 'hash="LgAPp+hXWcf0wlTU2cM+9IHkWac" index="0" size="65536" weight="0"/>\n    </File>\n'
                 '    <File name="e.bin" size="0"/>\n  </FileInfo>\n\n  <Tracker host="127.0.0.1" port="10101"/>'
                 '\n\n</BitFlood>')
