"""Extract tests/golden/xerces260_domwriter_pretty.json (run in the build
container, where /root/reference exists).

The reference vendors Xerces-C 2.6.0, whose DOMWriter with
format-pretty-print writes bitflood's flood files (cpp/src/FloodFile.cpp:42-142,
writeToString(*rootElem)).  Xerces' own DOM test suite holds the expected
pretty-printed output of its Normalizer test
(cpp/extern/xercesc++/2.6.0/tests/DOM/Normalizer/expectedOutput, written by
Normalizer.cpp:204-213 with format-pretty-print on).  This keeps the documents
of that file that hold only elements and attributes -- the shape of a flood
file -- as data, byte for byte after their XML declaration, so the test suite
can pin the layout rules (newline + 2-space indent per level, a blank line
before level-1 elements and before the root's end tag, "/>" for childless
elements) without the reference present.
"""
import json
import os
import re

SRC = "/root/reference/cpp/extern/xercesc++/2.6.0/tests/DOM/Normalizer/expectedOutput"
DECL = '<?xml version="1.0" encoding="UTF-8" standalone="no" ?>'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "xerces260_domwriter_pretty.json")


def main():
    text = open(SRC, encoding="utf-8").read()
    docs = []
    for part in text.split(DECL)[1:]:
        root = re.match(r"\s*<([^\s/>]+)", part).group(1)
        end = part.find("\n</" + root + ">")
        if end < 0:
            continue
        body = part[: end + len(root) + 4]
        stripped = re.sub(r"<[^>]*>", "", body)
        if "<!--" in body or "<![CDATA[" in body or stripped.strip():
            continue  # comments, CDATA or text: not a flood file's shape
        docs.append(body)
    json.dump({"source": SRC.replace("/root/reference/", ""), "declaration": DECL,
               "note": "each doc is the bytes after the XML declaration, up to the root's end tag",
               "docs": docs}, open(OUT, "w"), indent=1)
    print(f"{len(docs)} element-only documents -> {OUT}")


if __name__ == "__main__":
    main()
