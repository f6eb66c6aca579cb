"""Test-side restatement of Xerces-C 2.6.0's DOMWriter pretty-print for
element-only trees -- the shape of a bitflood flood file, which the reference
writes with DOMWriter + format-pretty-print, writeToString(*rootElem)
(cpp/src/FloodFile.cpp:42-142).

Rules (DOMWriterImpl.cpp, citations as in bitflood_amd/host/FloodFile.cpp):
  - every start tag begins a new line indented 2 spaces per level
    (:970-981, printIndent :1773-1788), with one extra blank line at level 1;
  - a childless element closes with "/>" (:1198-1210);
  - otherwise the end tag goes on its own line at the element's indent, with
    one extra blank line for the root (level 0) (:1171-1191);
  - attribute values escape & < " and LF, LF as "&#xA;" (XMLFormatter.cpp:78-84,
    562-581), in the order given (a flood file's non-namespace attributes come
    sorted by name: DOMAttrMapImpl.cpp:111-150).
tests/test_floodfile_format.py pins these rules against Xerces' own expected
output (tests/golden/xerces260_domwriter_pretty.json), and tests/test_host_cpp.py
checks the C++ writer against flood files built here.  A node is
(name, [(attr, value), ...], [children]).
"""
import re


def escape_attr(v: str) -> str:
    return v.replace("&", "&amp;").replace("<", "&lt;").replace('"', "&quot;").replace("\n", "&#xA;")


def pretty(node, level: int = 0) -> str:
    name, attrs, kids = node
    out = ("\n" if level == 1 else "") + "\n" + "  " * level + "<" + name
    out += "".join(f' {k}="{escape_attr(v)}"' for k, v in attrs)
    if not kids:
        return out + "/>"
    out += ">" + "".join(pretty(k, level + 1) for k in kids)
    return out + ("\n" if level == 0 else "") + "\n" + "  " * level + "</" + name + ">"


_TAG = re.compile(r"<(/?)([^\s/>]+)((?:\s+[^\s=]+=\"[^\"]*\")*)\s*(/?)>")
_ATTR = re.compile(r"([^\s=]+)=\"([^\"]*)\"")


def parse(xml: str):
    """Element-only XML (no text, comments or CDATA) -> node tree; attribute
    values are taken as written (the fixtures hold no escapes)."""
    stack, root, pos = [], None, 0
    for m in _TAG.finditer(xml):
        if xml[pos:m.start()].strip():
            raise ValueError("text content: not element-only")
        pos = m.end()
        closing, name, attrs, empty = m.groups()
        if closing:
            node = stack.pop()
            assert node[0] == name, (node[0], name)
            continue
        node = (name, _ATTR.findall(attrs), [])
        if stack:
            stack[-1][2].append(node)
        else:
            root = node
        if not empty:
            stack.append(node)
    if stack or xml[pos:].strip():
        raise ValueError("unbalanced or trailing text")
    return root
