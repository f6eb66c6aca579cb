#!/usr/bin/env python3
"""Does pinning a pageable job on the fly beat the staging memcpy? (VERDICT r04
next #4; diagnostic, GPU box.)

For one pageable host buffer per size (64 MiB, 1 GiB, 4 GiB at 256 KiB chunks),
all in one process and lease, best of 3 after a warm pass:
  staged        hash_chunks on the pageable buffer (memcpy into pinned staging, H2D)
  reg_whole     lbf_host_register of the whole buffer + hash_chunks (direct H2D) +
                lbf_host_unregister, all inside the timing
  reg_pipelined pieces of --piece-mib: a helper thread registers piece k+1 (and
                unregisters piece k-1) while piece k is hashed straight from
                pinned memory; registration and hashing timed together
  autopin       the library's own on-the-fly pinning (lbf_capi.cpp AutoPin; the
                default since round 5): the job's span registered in one piece
  registered    the buffer registered outside the timing (what a caller that
                reuses its buffer gets: the ceiling of the pinned routes)
plus the cost of pinning and unpinning alone (GiB/s of hipHostRegister /
hipHostUnregister through lbf_host_register).  One JSON line.

    python tools/autopin_probe.py [--piece-mib 256] [--sizes 64,1024,4096]
"""
import argparse
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime per process, loaded first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bitflood_amd import ChunkHasher, chunk_table  # noqa: E402

CS = 262144


def best_of(n, fn):
    best = 1e9
    for _ in range(n):
        t = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--piece-mib", type=int, default=256)
    ap.add_argument("--sizes", default="64,1024,4096")
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    page = os.sysconf("SC_PAGESIZE")
    # page-aligned (mmap), so pieces of whole pages never share one (lbf_host_register pins whole pages)
    import mmap
    _mm = mmap.mmap(-1, max(sizes) << 20)
    big = np.frombuffer(_mm, dtype=np.uint8)
    big[:] = np.random.default_rng(7).integers(0, 256, size=big.size, dtype=np.uint8)
    out = {"piece_mib": a.piece_mib, "gibs": {}, "pin": {}}
    with ChunkHasher(device_mask=1) as h:
        for mib in sizes:
            data = big[:mib << 20]
            offs, sizes_ = chunk_table(data.size, CS)
            want_last = hashlib.sha1(data[int(offs[-1]):].tobytes()).digest()
            r = {}
            os.environ["LBF_AUTOPIN"] = "0"  # the staging memcpy
            got = h.hash_chunks(data, offs, sizes_)  # warm
            assert bytes(got[-1]) == want_last
            r["staged"] = best_of(3, lambda: h.hash_chunks(data, offs, sizes_))

            def whole():
                h.register_host(data)
                g = h.hash_chunks(data, offs, sizes_)
                h.unregister_host(data)
                assert bytes(g[-1]) == want_last
            r["reg_whole"] = best_of(3, whole)

            piece = max(page, (a.piece_mib << 20) // page * page)
            bounds = [(p, min(p + piece, data.size)) for p in range(0, data.size, piece)]
            views = [data[lo:hi] for lo, hi in bounds]
            tabs = [chunk_table(v.size, CS) for v in views]

            def pipelined():
                ready = [threading.Event() for _ in views]
                done = [threading.Event() for _ in views]

                def helper():
                  try:
                    for k, v in enumerate(views):
                        h.register_host(v)
                        ready[k].set()
                        if k >= 1:  # unpin the piece before the one just pinned, once it is hashed
                            done[k - 1].wait()
                            h.unregister_host(views[k - 1])
                    done[-1].wait()
                    h.unregister_host(views[-1])
                  except Exception as e:  # the main thread times out on ready[] and reports
                    print(f"helper: {e}", file=sys.stderr, flush=True)
                th = threading.Thread(target=helper)
                th.start()
                last = None
                for k, v in enumerate(views):
                    if not ready[k].wait(timeout=60):
                        raise RuntimeError("the pinning helper stopped")
                    last = h.hash_chunks(v, *tabs[k])
                    done[k].set()
                th.join()
                assert bytes(last[-1]) == want_last
            r["reg_pipelined"] = best_of(3, pipelined)

            os.environ["LBF_AUTOPIN"] = "1"  # the library's default: the whole span in one registration
            s0 = h.staging_stats()
            g = h.hash_chunks(data, offs, sizes_)
            assert bytes(g[-1]) == want_last
            r["autopin"] = best_of(3, lambda: h.hash_chunks(data, offs, sizes_))
            autopin_direct = (h.staging_stats()["direct"] - s0["direct"]) / (4 * data.size)
            os.environ["LBF_AUTOPIN"] = "0"
            r["staged_again"] = best_of(3, lambda: h.hash_chunks(data, offs, sizes_))

            t = time.perf_counter()
            h.register_host(data)
            reg_s = time.perf_counter() - t
            s0 = h.staging_stats()
            r["registered"] = best_of(3, lambda: h.hash_chunks(data, offs, sizes_))
            direct = h.staging_stats()["direct"] - s0["direct"]
            t = time.perf_counter()
            h.unregister_host(data)
            unreg_s = time.perf_counter() - t
            out["gibs"][mib] = {k: round(data.size / v / 2**30, 2) for k, v in r.items()}
            out["pin"][mib] = {"register_s": round(reg_s, 4), "unregister_s": round(unreg_s, 4),
                               "register_gibs": round(data.size / reg_s / 2**30, 1),
                               "unregister_gibs": round(data.size / unreg_s / 2**30, 1),
                               "registered_direct_fraction": round(direct / (3 * data.size), 3),
                               "autopin_direct_fraction": round(autopin_direct, 3)}
            print(json.dumps({mib: out["gibs"][mib], "pin": out["pin"][mib]}), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
