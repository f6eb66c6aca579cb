#!/usr/bin/env python3
"""What HIP reports about host memory pinned with hipHostRegister (diagnostic,
GPU box): for a whole-buffer registration, a sub-range registration and a
hipHostMalloc buffer, print hipPointerGetAttributes (type, host and device
pointers), hipMemGetAddressRange and hipMemPtrGetInfo on the host pointer, an
interior pointer and the device pointer.  lbf_host_register needs the extent
of the pinned allocation holding a caller's range."""
import ctypes
import json
import mmap

import torch  # noqa: F401  (loads libamdhip64 first)

hip = ctypes.CDLL("libamdhip64.so")
MIB = 1 << 20


class Attr(ctypes.Structure):  # hipPointerAttribute_t (ROCm 6+/7 layout)
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


hsa = ctypes.CDLL("libhsa-runtime64.so.1")


class HsaInfo(ctypes.Structure):  # hsa_amd_pointer_info_t (hsa_ext_amd.h)
    _fields_ = [("size", ctypes.c_uint32), ("type", ctypes.c_int), ("agentBaseAddress", ctypes.c_void_p),
                ("hostBaseAddress", ctypes.c_void_p), ("sizeInBytes", ctypes.c_size_t), ("userData", ctypes.c_void_p),
                ("agentOwner", ctypes.c_uint64), ("global_flags", ctypes.c_uint32)]


def q(p):
    out = {}
    info = HsaInfo()
    info.size = ctypes.sizeof(HsaInfo)
    rc = hsa.hsa_amd_pointer_info(ctypes.c_void_p(p), ctypes.byref(info), None, None, None)
    out["hsa"] = [rc, info.type, (info.hostBaseAddress or 0) - p if info.hostBaseAddress else None,
                  (info.agentBaseAddress or 0) - p if info.agentBaseAddress else None, info.sizeInBytes]
    for name, code, ctype in (("buffer_id", 7, ctypes.c_uint64), ("range_start", 11, ctypes.c_void_p),
                              ("range_size", 12, ctypes.c_size_t), ("mapped", 13, ctypes.c_int)):
        v = ctype()
        rc = hip.hipPointerGetAttribute(ctypes.byref(v), code, ctypes.c_void_p(p))
        val = v.value
        if name == "range_start" and val:
            val = val - p
        out[name] = [rc, val]
    hip.hipGetLastError()
    a = Attr()
    out["attr_rc"] = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    out["type"], out["dev_ptr_minus_p"] = a.type, (a.devicePointer or 0) - p
    out["host_ptr_minus_p"] = (a.hostPointer or 0) - p
    for name, ptr in (("host", p), ("dev", a.devicePointer or 0)):
        b, sz = ctypes.c_void_p(), ctypes.c_size_t()
        rc = hip.hipMemGetAddressRange(ctypes.byref(b), ctypes.byref(sz), ctypes.c_void_p(ptr))
        out[f"range_{name}"] = [rc, (b.value or 0) - p if b.value else None, sz.value]
        s2 = ctypes.c_size_t()
        rc2 = hip.hipMemPtrGetInfo(ctypes.c_void_p(ptr), ctypes.byref(s2))
        out[f"ptrinfo_{name}"] = [rc2, s2.value]
    hip.hipGetLastError()
    return out


res = {}
mm = mmap.mmap(-1, 8 * MIB)
buf = (ctypes.c_uint8 * (8 * MIB)).from_buffer(mm)
base = ctypes.addressof(buf)
assert hip.hipHostRegister(ctypes.c_void_p(base), 3 * MIB + 12345, 0) == 0
res["registered_whole_3MiB+12345"] = {"base": q(base), "interior": q(base + MIB + 100), "last": q(base + 3 * MIB + 12344),
                                      "past": q(base + 3 * MIB + 4096 * 4)}
hip.hipHostUnregister(ctypes.c_void_p(base))
res["after_unregister"] = q(base)
p = ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(p), 8 * MIB, 0) == 0
res["hostmalloc_8MiB"] = {"base": q(p.value), "interior": q(p.value + 3 * MIB + 7)}
# two registrations with pageable memory between them
assert hip.hipHostRegister(ctypes.c_void_p(base), MIB, 0) == 0
assert hip.hipHostRegister(ctypes.c_void_p(base + 2 * MIB), MIB, 0) == 0
res["two_regs"] = {"first": q(base + 100), "middle": q(base + MIB + 100), "second": q(base + 2 * MIB + 100)}
hip.hipHostUnregister(ctypes.c_void_p(base))
hip.hipHostUnregister(ctypes.c_void_p(base + 2 * MIB))
hip.hipHostFree(p)
print(json.dumps(res, indent=1))
