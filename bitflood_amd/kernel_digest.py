"""Digests of the gfx950 machine code a built library actually carries.

A HIP shared library holds its device code as clang offload bundles in the
host ELF (`__CLANG_OFFLOAD_BUNDLE__`, one per translation unit); each bundle
entry for `hipv4-amdgcn-amd-amdhsa--gfx950` is an AMDGPU code object, itself
an ELF whose symbol table gives every kernel's bytes.  kernel_digests(path)
returns {mangled kernel symbol: sha256 of its machine code}, read from the
file with no tool and no GPU.

Used to tie a recorded measurement to the code it measured:
tools/pmc_traffic.py --record stores the profiled kernel's digest beside its
PMC traffic in profiles/pmc_traffic.json, and bench.py reports that traffic
only while the library it loaded carries the same bytes for that kernel
(a changed kernel under an unchanged template name must
not keep citing the old counters).
"""
import hashlib
import re
import struct

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_CCOB = b"CCOB"  # a compressed offload bundle (clang --offload-compress)
_TARGET = b"amdgcn-amd-amdhsa--gfx950"


class CompressedBundle(ValueError):
    """The library's device code sits in compressed offload bundles, which this
    reader does not inflate: no digest can be given."""


def _code_objects(blob):
    """The gfx950 code objects of every uncompressed offload bundle in blob."""
    out = []
    at = blob.find(_MAGIC)
    while at >= 0:
        p = at + len(_MAGIC)
        (n,) = struct.unpack_from("<Q", blob, p)
        p += 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            p += 24
            triple = blob[p:p + tlen]
            p += tlen
            if triple.endswith(_TARGET) and size:
                out.append(blob[at + off:at + off + size])
        at = blob.find(_MAGIC, at + len(_MAGIC))
    return out


# The kernel descriptor (<kernel>.kd, 64 bytes): LDS and scratch sizes,
# kernarg size, the compute_pgm_rsrc1/2/3 words (VGPR/SGPR counts, wave
# limits), properties.  Bytes 16..24 hold the code's offset from the
# descriptor, which moves whenever anything else in the object changes size,
# so they are left out.
_KD_SIZE = 64
_KD_ENTRY = slice(16, 24)


def _elf_functions(co):
    """{symbol: machine-code bytes + its kernel descriptor's bytes (entry offset
    zeroed)} for the STT_FUNC symbols of an ELF64 code object: two builds whose
    instructions match but whose register counts, LDS size or wave limits
    differ get different digests."""
    if co[:4] != b"\x7fELF" or co[4] != 2:
        raise ValueError("not an ELF64 code object")
    e_shoff, = struct.unpack_from("<Q", co, 0x28)
    e_shentsize, e_shnum = struct.unpack_from("<HH", co, 0x3A)
    secs = []
    for i in range(e_shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", co, e_shoff + i * e_shentsize)
        secs.append((typ, addr, off, size, link, entsize))
    funcs, kds = {}, {}
    for typ, _, off, size, link, entsize in secs:
        if typ != 2:  # SHT_SYMTAB
            continue
        stroff = secs[link][2]
        for k in range(size // entsize):
            st_name, st_info, _, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", co, off + k * entsize)
            if not st_size or st_shndx >= len(secs):
                continue
            kind = st_info & 0xF
            if kind not in (1, 2):  # STT_OBJECT (descriptors), STT_FUNC (code)
                continue
            end = co.index(b"\0", stroff + st_name)
            sym = co[stroff + st_name:end].decode()
            _, saddr, soff, _, _, _ = secs[st_shndx]
            start = soff + (st_value - saddr)
            if kind == 2:
                funcs[sym] = co[start:start + st_size]
            elif sym.endswith(".kd") and st_size == _KD_SIZE:
                kd = bytearray(co[start:start + st_size])
                kd[_KD_ENTRY] = bytes(_KD_ENTRY.stop - _KD_ENTRY.start)
                kds[sym[:-3]] = bytes(kd)
    return {sym: code + kds.get(sym, b"") for sym, code in funcs.items()}


def kernel_digests(path):
    """{mangled kernel symbol: sha256 hex of its gfx950 machine code and kernel
    descriptor} for the library at path; CompressedBundle if the device code is
    compressed.  A symbol found in two code objects with different bytes
    maps to None (ambiguous)."""
    with open(path, "rb") as f:
        blob = f.read()
    out = {}
    cos = _code_objects(blob)
    if not cos and _CCOB in blob:
        raise CompressedBundle(f"{path}: device code in compressed offload bundles (CCOB), not read here")
    for co in cos:
        for sym, code in _elf_functions(co).items():
            d = hashlib.sha256(code).hexdigest()
            out[sym] = d if out.get(sym, d) == d else None
    return out


def find_kernel(digests, demangled_fragment, template_args=None):
    """The mangled symbols whose name holds every piece of a demangled kernel
    name like 'sha1_pc4_kernel<true, 2, 8>': the identifier, and (optionally)
    the template arguments in Itanium form (Lb1E Li2E Li8E)."""
    ident = demangled_fragment.split("<")[0].strip()
    hits = [s for s in digests if f"{len(ident)}{ident}" in s]
    if template_args is not None:
        hits = [s for s in hits if _itanium_args(template_args) in s]
    return hits


def _itanium_args(args):
    enc = []
    for a in args:
        if a is True or a == "true":
            enc.append("Lb1E")
        elif a is False or a == "false":
            enc.append("Lb0E")
        else:
            enc.append(f"Li{int(a)}E")
    return "I" + "".join(enc) + "E"


def symbol_for(digests, demangled):
    """The one mangled symbol for a demangled kernel name ('sha1_pc4_kernel<true, 2, 8>', with or without its
    namespace, return type and parameter list), or None."""
    m = re.search(r"(\w+)\s*(<[^<>]*>)?\s*(\([^()]*\))?\s*$", demangled.strip())
    if not m:
        return None
    ident, targs = m.group(1), m.group(2)
    args = None if targs is None else [a.strip() for a in targs[1:-1].split(",") if a.strip()]
    hits = find_kernel(digests, ident, args)
    return hits[0] if len(hits) == 1 else None
