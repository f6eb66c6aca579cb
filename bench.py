#!/usr/bin/env python3
"""bench.py -- device-resident chunk-hash throughput (BASELINE.json metric).

Workload per GPU (configs[1], "C2"): one 4 GiB synthetic file at 256 KiB chunks
(16,384 chunks), bytes generated directly in HBM before timing.  One step = one
launch of the chunk-hash kernel over the whole batch (SHA-1 of every chunk,
20-byte digests written to HBM).  With N GPUs each rank hashes its own 4 GiB
shard of an N x 4 GiB file (weak scaling, contiguous chunk ranges, no data-path
collective; the only collectives are the timing barrier and the max-over-ranks
reduction).

--config c4: the C4 shard instead (configs[3]): 32 GiB at 1 MiB chunks per rank,
rank r = shard r of the 256 GiB file.

Every rank checks its own digests against the committed golden for its shard
(tests/golden/c2_ranks.json, c4.json) and the pass flags are gathered into the
line, so a multi-GPU run validates itself.

Launch:  python bench.py [--gpus N --steps K --warmup W] [--config c2|c4]
   N>1, either way:
     python bench.py --gpus N ...              (bench.py starts the N rank processes itself)
     python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
   Rank 0 prints ONE JSON line.  The process group is RCCL ("nccl"); with more
   ranks than visible GPUs (rehearsals on a small box) the self-launch uses gloo
   and the line says so (LBF_BENCH_BACKEND overrides).

LBF_BENCH_FORM_GROUP=1 at --gpus 1: rank 0 forms a one-rank process group
(RCCL unless LBF_BENCH_BACKEND says otherwise) and takes the N>1 route below,
so every collective of the N-GPU line runs on a 1-GPU box (tests/test_gpu_nccl.py).

N>1 also measures, after the timed region:
  * e2e: every rank hashes (the first 4 GiB of) its shard from host memory at
    the same moment, pageable and then registered, through its own NUMA-local
    lbf_ctx -- the copy-inclusive rate of north_star at N ranks;
  * e2e_inprocess: rank 0 alone, after the others have finished, hashes one
    registered N x 4 GiB host buffer through ONE lbf_ctx over every visible
    device (Encoder::EncodeFile's shape on an N-GPU node).
At every N rank 0 then times cpu_baseline (the reference encoder's hash on the
host's usable cores, same stream) once the GPU legs are over.
"""
import math
import argparse
import hashlib
import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (first: one HIP runtime per process)

from bitflood_amd import DeviceBuffer, b64_27  # noqa: E402
from bitflood_amd import hashing as H  # noqa: E402
from bitflood_amd.sharding import max_over_ranks, shard_range  # noqa: E402

GIB = 1 << 30
SEED_C = 0x5EED
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, MI355X_MICROARCH.md "Chip-level parameters"
CLOCK_HZ = 2.4e9       # MI355X max engine clock, MI355X_MICROARCH.md (chip table)
N_SIMDS = 1024         # 256 CUs x 4 SIMDs
# kernel variant -> uniform-mode kernel symbol (profiles/pmc_traffic.json "kernel")
KERNELS = {1: "sha1_lane_kernel<true>", 2: "sha1_pc_kernel<true, 2>", 3: "sha1_lds_kernel<true, 2>",
           4: "sha1_pc2_kernel<true>", 5: "sha1_pc_kernel<true, 2, 2>",
           6: "sha1_pc4_kernel<true, 4>", 7: "sha1_pc4_kernel<true, 2, 8>", 8: "sha1_pc4_kernel<true, 1>",
           9: "sha1_pcx4_kernel<true, 40>", 10: "sha1_pcx5_kernel<true, 64>",
           11: "sha1_lds2_kernel<true>", 12: "sha1_pc4x2_kernel<true>"}
# Issue floors per 64-byte block (tools/gen_round_order.py, tools/probe_lds_lanes.hip):
#  pc2/pc4/pc4x2 consumer: 80 rounds x 5 VALU at one issue per 4.09 cycles -- the chain's own
#    arithmetic alone (its 20 schedule loads and the barrier are not counted)
#  pc/pcx2 consumer: the two-add3 round form with K in a VGPR (23.2 cycles per round measured)
#  fused lane/lds: 613 VALU; a lone wave issues one per 4.09 cycles, a SIMD retires one per 4
PC2_CYCLES_PER_BLOCK = 80 * 5 * 4.09
PC_CYCLES_PER_BLOCK = 80 * 23.2
#  pcx4 consumer: rounds 0..39 in the two-add3 form, 40..79 with W+K
PCX4_CYCLES_PER_BLOCK = 40 * 23.2 + 40 * 5 * 4.09
#  pcx5 consumer: rounds 0..63 in the two-add3 form, 64..79 with W+K (the producer
#    byte-swaps words 0..15 since round 2)
PCX5_CYCLES_PER_BLOCK = 64 * 23.2 + 16 * 5 * 4.09
FUSED_VALU_PER_BLOCK = 613
# bytes per rank of the N>1 copy-inclusive leg (the whole C2 shard; C4's first 4 GiB)
E2E_SLICE_BYTES = 4 * GIB


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c2", "c4"], default="c2",
                    help="c2: 4 GiB at 256 KiB per GPU (configs[1]); c4: 32 GiB at 1 MiB per GPU (configs[3])")
    ap.add_argument("--chunk-size", type=int, default=0, help="override the config's chunk size")
    ap.add_argument("--file-gib", type=float, default=0.0, help="override the config's bytes per GPU per step")
    ap.add_argument("--variant", type=int, default=0, help="kernel variant (0 = automatic)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every CPU this process may use (affinity, capped by the cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-min-s", type=float, default=3.0,
                    help="cpu_baseline: seconds each multi-thread rate is timed over (>= 3 s by default, so a cgroup "
                         "quota's per-period burst cannot inflate it)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host->device->host rate")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the device-resident C3 and C4 measurements that follow the main line at N=1")
    ap.add_argument("--no-inproc", action="store_true",
                    help="N>1: skip the single-process all-device host-memory leg (e2e_inprocess)")
    a = ap.parse_args()
    a.chunk_size = a.chunk_size or {"c2": 262144, "c4": 1 << 20}[a.config]
    a.file_gib = a.file_gib or {"c2": 4.0, "c4": 32.0}[a.config]
    return a


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(base, n, port, backend=None):
    """The environment of each of n self-launched ranks: what torch.distributed.run
    would export (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*), one node."""
    common = dict(base, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                  LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", LBF_BENCH_LAUNCHER="bench.py")
    if backend:
        common["LBF_BENCH_BACKEND"] = backend
    return [dict(common, RANK=str(r), LOCAL_RANK=str(r)) for r in range(n)]


def spawn_ranks(n, argv, script=None, python=None, env=None, grace_s=15.0):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes of
    this script and wait for them.  The parent makes no GPU call (importing
    torch and counting devices do not initialise HIP on this image) and never
    execs: the ranks are children.  Rank 0 inherits stdout and prints the one
    JSON line; the other ranks' stdout goes to stderr.  If a rank fails, the
    others are stopped (by PID) and its exit status is returned."""
    import signal
    import subprocess
    base = dict(os.environ if env is None else env)
    backend = None
    if "LBF_BENCH_BACKEND" not in base:
        ndev = torch.cuda.device_count()
        if ndev < n:
            # RCCL refuses two ranks on one device: a rehearsal on a small box
            backend = "gloo"
            print(f"bench.py: {n} ranks on {ndev} visible GPU(s): process group gloo (rehearsal)", file=sys.stderr)
    envs = rank_env(base, n, _free_port(), backend)
    cmd = [python or sys.executable, script or os.path.abspath(__file__)] + list(argv)
    procs = []
    try:
        for r in range(n):
            procs.append(subprocess.Popen(cmd, env=envs[r], stdout=subprocess.PIPE if r == 0 else sys.stderr))
    except BaseException:
        for p in procs:
            p.kill()
        raise

    def relay(pipe):
        # rank 0's JSON line to stdout; anything else it prints (gloo's C++
        # connection notice goes to stdout) to stderr, so stdout stays one line
        for raw in iter(pipe.readline, b""):
            line = raw.decode(errors="replace")
            dst = sys.stdout if line.lstrip().startswith("{") else sys.stderr
            dst.write(line)
            dst.flush()

    import threading
    relay_t = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    relay_t.start()

    def stop_all(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    old = signal.signal(signal.SIGTERM, lambda *a: (stop_all(), sys.exit(143)))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print(f"bench.py: rank {procs.index(p)} exited with {c}; stopping the others", file=sys.stderr)
                    stop_all()
                    deadline = time.time() + grace_s
                    for q in live:
                        try:
                            q.wait(timeout=max(0.1, deadline - time.time()))
                        except subprocess.TimeoutExpired:
                            q.kill()
            time.sleep(0.1)
    finally:
        signal.signal(signal.SIGTERM, old)
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        relay_t.join(timeout=10)
    return rc


class _stdout_to_stderr:
    """File descriptor 1 redirected to 2 while in scope (C and C++ writers included)."""

    def __enter__(self):
        import ctypes
        self._libc = ctypes.CDLL(None)
        sys.stdout.flush()
        self._libc.fflush(None)
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        self._libc.fflush(None)
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


def init_group(backend, rank, world, dev):
    """The process group of one rank: RCCL ("nccl") bound to its device, or gloo.
    gloo's C++ side prints its "[Gloo] Rank r is connected to ..." notice on
    stdout, where the launcher collects the one JSON line: while the group
    forms, the process's stdout points at stderr."""
    import torch.distributed as dist
    with _stdout_to_stderr():
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)


def grouped():
    """True while a process group is formed: the collectives below then run
    through it even at world 1 (LBF_BENCH_FORM_GROUP)."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        # only reachable under an outside launcher whose world differs from --gpus:
        # refuse rather than print a line whose n_gpus is not what was asked for
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher's WORLD_SIZE is {world}")
    ndev = max(1, torch.cuda.device_count())
    # one rank per GPU; more ranks than GPUs only for rehearsals of the
    # multi-rank flow on a small box (process group gloo)
    dev = local % ndev
    torch.cuda.set_device(dev)
    if world > 1 or os.environ.get("LBF_BENCH_FORM_GROUP") == "1":
        backend = os.environ.get("LBF_BENCH_BACKEND")
        if backend is None:
            # the self-launch's rule under an outside launcher too: RCCL refuses
            # two ranks on one device, so more ranks than GPUs rehearse on gloo
            backend = "gloo" if world > ndev else "nccl"
            if backend == "gloo" and rank == 0:
                print(f"bench.py: {world} ranks on {ndev} visible GPU(s): process group gloo (rehearsal)",
                      file=sys.stderr)
        init_group(backend, rank, world, dev)
    return rank, world, local, dev, ndev


def backend_name():
    import torch.distributed as dist
    return str(dist.get_backend())


def under_profiler():
    """rocprofv3's preloaded tool library is in this process (the preload is
    what initialises the GPU before the program starts)."""
    return "rocprof" in os.environ.get("LD_PRELOAD", "")


def barrier(world):
    if grouped():
        import torch.distributed as dist
        dist.barrier()


DIGEST_ERRORS = {}  # kernel -> why its digest could not be read (traffic_null_reason)


def kernel_code_digest(kernel, lib_path=None):
    """(mangled symbol, sha256 of its gfx950 machine code and descriptor) of
    `kernel` (e.g. 'sha1_pc4_kernel<true, 2, 8>') in the library this process
    loaded (bitflood_amd/kernel_digest.py reads the code object out of the
    .so), or (None, None) when it cannot be found; the reason is kept in
    DIGEST_ERRORS[kernel]."""
    from bitflood_amd import _capi
    from bitflood_amd import kernel_digest as KD
    try:
        d = KD.kernel_digests(lib_path or _capi.LIB_PATH)
        sym = KD.symbol_for(d, kernel)
        if sym and d.get(sym):
            return sym, d[sym]
        DIGEST_ERRORS[kernel] = f"{kernel} not found (or ambiguous) in the loaded library's gfx950 code objects"
    except KD.CompressedBundle as e:
        DIGEST_ERRORS[kernel] = f"compressed bundle: {e}"
    except (OSError, ValueError, IndexError, struct.error) as e:
        DIGEST_ERRORS[kernel] = f"{type(e).__name__}: {e}"
    return None, None


def traffic_from_profiles(file_bytes, chunk_size, kernel, code_sha=None, path=None):
    """HBM bytes per launch measured with rocprofv3 PMC (FETCH_SIZE x2, gfx950
    correction), recorded by tools/pmc_traffic.py --record for
    this workload size and this kernel.  A static lookup, not a measurement of
    this run, so it is tied to the code it measured: an entry counts only when
    its recorded machine-code digest (`code_sha256`, the profiled library's
    bytes for that kernel) equals `code_sha`, the digest of the kernel in the
    library this run loaded.  Returns (bytes, source, None) or
    (None, None, reason)."""
    p = path or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError) as e:
        return None, None, f"no traffic record ({type(e).__name__})"
    reason = f"no PMC record for {kernel} at {file_bytes} B / {chunk_size} B chunks"
    for e in d.get("entries", [d]):
        if not (int(e.get("file_bytes", -1)) == int(file_bytes) and int(e.get("chunk_size", 262144)) == chunk_size
                and kernel in e.get("kernel", "")):
            continue
        rec = e.get("code_sha256")
        if not rec:
            reason = f"the PMC record for {kernel} ({e.get('source')}) carries no machine-code digest"
            continue
        if code_sha is None:
            reason = f"the loaded library's code for {kernel} could not be read"
            if DIGEST_ERRORS.get(kernel):
                reason += f" ({DIGEST_ERRORS[kernel]})"
            continue
        if rec != code_sha:
            reason = (f"the loaded library's {kernel} is not the code that was profiled ({e.get('source')}: "
                      f"sha256 {rec[:16]}..., loaded {code_sha[:16]}...)")
            continue
        src = e.get("source", p)
        b = e.get("bench_same_session")
        if b and e.get("trace_timed_median_ns"):
            src += (f" (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of this kernel at this size; recorded in one lease "
                    f"with an unprofiled bench line of ms_per_step {b['ms_per_step']} and a kernel trace whose "
                    f"timed dispatches have median {e['trace_timed_median_ns'] / 1e6:.4f} ms; machine code "
                    f"sha256 {rec[:16]}... equal to the loaded library's; a lookup, not this run's counters)")
        else:
            src += (f" (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, same kernel, size and machine code sha256 "
                    f"{rec[:16]}...; a recorded lookup, not this run's counters)")
        return float(e["hbm_bytes_per_launch"]), src, None
    return None, None, reason


def _cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else int(q) / int(per)
    except Exception:
        return None


def _numa_nodes():
    out = {}
    base = "/sys/devices/system/node"
    try:
        for n in sorted(os.listdir(base)):
            if n.startswith("node") and n[4:].isdigit():
                out[n] = open(os.path.join(base, n, "cpulist")).read().strip()
    except Exception:
        pass
    return out


def host_cpus():
    """The CPUs this process can actually use: its affinity mask, capped by the
    cgroup CPU quota (a GPU box grants 16 CPUs of a 256-CPU host per GPU)."""
    affinity = len(os.sched_getaffinity(0))
    quota = _cgroup_cpu_quota()
    usable = min(affinity, math.ceil(quota)) if quota else affinity
    return affinity, quota, usable


def cpu_baseline(args, stream_start, n_chunks_sample, gpu_digests_sample):
    """The reference encoder's hash on the host cores, over a bounded sample of
    the same synthetic bytes.  `value` times oracle/sha1_unrolled.c: portable C
    -O2 in the shape of the reference's Crypto++ 5.2.1 Transform (80 unrolled
    rounds, rolling W[i&15]; sha.cpp:34-69), the speed the reference itself
    compiles to.  kind="port": building the reference was denied (SURVEY.md
    §8c).  The checker oracle's loop form (oracle/sha1_oracle.c, ~1.5x slower)
    is kept as `loop_form`.  Threads: every CPU the process may use (SURVEY.md
    §8d (ii)), i.e. its affinity mask capped by the cgroup CPU quota; the
    reference encoder itself is one thread (Encoder.cpp:40-79), timed as
    `single_thread_value`."""
    from tests.oracle_lib import Oracle
    orc = Oracle()
    cs = args.chunk_size
    nbytes = n_chunks_sample * cs
    affinity, quota, usable = host_cpus()
    threads = args.cpu_threads or usable
    data = orc.synth(SEED_C, stream_start, nbytes, nthreads=threads)
    offs = np.arange(n_chunks_sample, dtype=np.uint64) * np.uint64(cs)
    sizes = np.full(n_chunks_sample, cs, dtype=np.uint32)
    clock0 = orc.clock_ghz()

    def rate(fn, nthreads, n=n_chunks_sample, min_s=3.0, max_reps=20):
        reps, t = 0, 0.0
        d = None
        while reps == 0 or (t < min_s and reps < max_reps):
            t0 = time.perf_counter()
            d = fn(data, offs[:n], sizes[:n], nthreads=nthreads)
            t += time.perf_counter() - t0
            reps += 1
        return reps * n * cs / GIB / t, reps, d

    # all usable host cores, chunk-parallel; >= 3 s, so a
    # cgroup quota's per-period burst cannot inflate it
    min_s = args.cpu_min_s
    mt_gibs, reps, d_mt = rate(orc.sha1_batch_unrolled, threads, min_s=min_s, max_reps=400)
    # one thread per CPU of the affinity mask (256 on a GPU box): what the quota
    # lets through over the same >= 3 s
    aff_gibs = (rate(orc.sha1_batch_unrolled, affinity, min_s=min_s, max_reps=400)[0] if affinity != threads
                else mt_gibs)
    # one thread, like Encoder.cpp:40-79 (a quarter of the sample)
    n1 = max(1, n_chunks_sample // 4)
    st_gibs, _, d_1 = rate(orc.sha1_batch_unrolled, 1, n=n1, min_s=0.0, max_reps=1)
    clock1 = orc.clock_ghz()
    # the checker's loop form, for continuity with round 1-2 lines
    loop_mt = rate(orc.sha1_batch, threads, min_s=min_s / 2, max_reps=10)
    loop_st = rate(orc.sha1_batch, 1, n=n1 // 2 or 1, min_s=0.0, max_reps=1)
    # fread-inclusive single-thread encode of the same bytes as a file, as
    # Encoder::EncodeFile does it (one chunk buffer, fread + hash per chunk);
    # the file is page-cache warm, written just before
    import tempfile
    fread = None
    with tempfile.NamedTemporaryFile(prefix="lbf_cpu_sample_", dir=os.environ.get("TMPDIR", "/tmp")) as f:
        data[: n1 * cs].tofile(f.name)
        dig = np.zeros((n1, 20), dtype=np.uint8)
        t0 = time.perf_counter()
        got = orc.lib.unrolled_encode_file(f.name.encode(), cs, dig.ctypes.data, n1)
        t_f = time.perf_counter() - t0
        if got == n1:
            fread = {"value": round(n1 * cs / GIB / t_f, 3), "unit": "GiB/s",
                     "sample": f"{n1} x {cs // 1024} KiB chunks from a page-cached file, 1 thread",
                     "parity_vs_gpu": bool(np.array_equal(dig, gpu_digests_sample[:n1]))}
    parity = bool(np.array_equal(d_mt, gpu_digests_sample) and np.array_equal(d_1, gpu_digests_sample[:n1])
                  and np.array_equal(loop_mt[2], gpu_digests_sample))
    # value: the faster of the two thread counts, so the comparator is never the
    # weaker one; cores says which
    best_gibs, best_threads = max((mt_gibs, threads), (aff_gibs, affinity))
    return {
        "value": round(best_gibs, 3), "unit": "GiB/s", "cores": best_threads, "kind": "port",
        "implementation": "oracle/sha1_unrolled.c: unrolled 80-round Transform in Crypto++ 5.2.1's shape "
                          "(sha.cpp:34-69), gcc -O2, portable C, no SHA-NI",
        "sample": f"{n_chunks_sample} x {cs // 1024} KiB chunks ({nbytes / GIB:.2f} GiB) of the same stream, "
                  f"passes for >= {min_s:g} s on {threads} threads ({reps} passes) and on {affinity}; single-thread pass "
                  f"over {n1} chunks",
        "usable_threads_value": round(mt_gibs, 3),
        "single_thread_value": round(st_gibs, 3),
        "affinity_threads_value": round(aff_gibs, 3),
        "single_thread_fread_encode": fread,
        "loop_form": {"value": round(loop_mt[0], 3), "single_thread_value": round(loop_st[0], 3),
                      "implementation": "oracle/sha1_oracle.c (the parity checker: rounds as a loop)"},
        "host": {**_host_desc(), "affinity_cores": affinity, "cgroup_cpu_quota": quota, "usable_cores": usable,
                 "numa_nodes": _numa_nodes(),
                 "clock_ghz_measured": [round(clock0, 3), round(clock1, 3)],
                 "clock_note": "one core, dependent-add chain (oracle unrolled_clock_probe), before and after "
                               "the multi-thread passes"},
        "parity_vs_gpu": parity,
    }


def _host_desc():
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    out = {"cpu_model": model, "os_cpu_count": os.cpu_count()}
    try:
        khz = int(open("/sys/devices/system/cpu/cpu0/cpufreq/cpuinfo_max_freq").read())
        out["cpufreq_max_ghz"] = round(khz / 1e6, 3)
    except Exception:
        pass
    return out


def compute_floor_ms(variant, cs, n_chunks):
    """Lower bound on one launch from instruction issue alone (SHA-1 is a serial
    chain per chunk, so few chunks are bound by one chain's issue rate)."""
    blocks = (cs + 9 + 63) // 64  # compressions per chunk incl. padding
    if variant in (4, 6, 7, 8, 12):
        return blocks * PC2_CYCLES_PER_BLOCK / CLOCK_HZ * 1e3
    if variant in (2, 5):
        return blocks * PC_CYCLES_PER_BLOCK / CLOCK_HZ * 1e3
    if variant == 9:
        return blocks * PCX4_CYCLES_PER_BLOCK / CLOCK_HZ * 1e3
    if variant == 10:
        return blocks * PCX5_CYCLES_PER_BLOCK / CLOCK_HZ * 1e3
    chain = blocks * FUSED_VALU_PER_BLOCK * 4.09 / CLOCK_HZ
    chip = n_chunks / 64 * blocks * FUSED_VALU_PER_BLOCK * 4.0 / (N_SIMDS * CLOCK_HZ)
    return max(chain, chip) * 1e3


def e2e_leg(host_data, cs, dev, world):
    """Host bytes in -> host digests out through this rank's lbf_ctx (pinned,
    NUMA-local staging on its GPU), from pageable memory and then from the same
    memory registered with the context (lbf_host_register: straight to HBM, no
    staging memcpy).  The PCIe-inclusive rate of north_star; never `value`.

    With world > 1 every rank runs each pass at the same moment (a barrier
    before each), so the aggregate world x bytes / slowest rank is what N GPUs
    pull over their links and host DRAM together.  Best of 3 passes per route,
    after one untimed pass that sizes the context's pinned staging.

    A failure on this rank (its context, a pass, the registration) is kept in
    `error` and never raised: the rank still takes part in every collective
    (a failed pass reports an infinite time, so the aggregate reads 0), so the
    other ranks finish and the line -- whose device-resident `value` was
    measured before this leg -- is still printed."""
    from bitflood_amd import ChunkHasher, chunk_table
    offs, sizes = chunk_table(host_data.size, cs)
    gib = host_data.size / GIB
    err = []

    def attempt(fn, what):
        if err:
            return None
        try:
            return fn()
        except Exception as e:  # recorded, see above
            err.append(f"{what}: {type(e).__name__}: {e}")
            return None

    def passes(h, k=3):
        best_agg, best_own, d = 0.0, float("inf"), None
        for _ in range(k):
            barrier(world)
            t0 = time.perf_counter()
            d = attempt(lambda: h.hash_chunks(host_data, offs, sizes), "hash pass")
            t = time.perf_counter() - t0 if not err else float("inf")
            t_max = max_over_ranks(t, world)
            best_agg = max(best_agg, world * gib / t_max)
            best_own = min(best_own, t)
        return best_agg, gib / best_own, d

    h = attempt(lambda: ChunkHasher(device_mask=1 << dev), "lbf_ctx_create")
    placement = {"device": dev, "numa_node": -1, "staging_node": -1, "bound_cpus": 0}
    reg_s, s0, s1, registered = 0.0, {"direct": 0}, {"direct": 0}, False
    fresh = None
    try:
        attempt(lambda: h.hash_chunks(host_data, offs, sizes), "warm pass")  # sizes the staging to this job
        pag_agg, pag_own, d_pag = passes(h)  # the default route: the staging memcpy (LBF_AUTOPIN unset)
        # Opt-in on-the-fly pinning (LBF_AUTOPIN=1; the default in round 5, off
        # since round 6) on a fresh copy of the bytes: the first pass pays the
        # first registration of those pages (tools/register_cost.py: ~21 GiB/s
        # of touched memory), later passes re-register what HIP already knows
        fresh = attempt(lambda: host_data.copy(), "fresh copy")
        old = os.environ.get("LBF_AUTOPIN")
        os.environ["LBF_AUTOPIN"] = "1"
        try:
            barrier(world)
            t0 = time.perf_counter()
            d_ap = attempt(lambda: h.hash_chunks(fresh, offs, sizes), "first on-the-fly pass")
            t = time.perf_counter() - t0 if not err else float("inf")
            ap_first_agg, ap_first_own = world * gib / max_over_ranks(t, world), gib / t
            ap_agg, ap_own, d_ap2 = passes(h)
        finally:
            if old is None:
                os.environ.pop("LBF_AUTOPIN", None)
            else:
                os.environ["LBF_AUTOPIN"] = old
        placement = attempt(lambda: h.worker_info(0), "worker_info") or placement
        t0 = time.perf_counter()
        registered = attempt(lambda: h.register_host(host_data) or True, "lbf_host_register") or False
        reg_s = time.perf_counter() - t0
        s0 = attempt(lambda: h.staging_stats(), "staging_stats") or s0
        reg_agg, reg_own, d_reg = passes(h)
        s1 = attempt(lambda: h.staging_stats(), "staging_stats") or s1
    finally:
        if h is not None:
            if registered:
                try:
                    h.unregister_host(host_data)
                except Exception as e:
                    err.append(f"lbf_host_unregister: {type(e).__name__}: {e}")
            h.close()
    del fresh
    return {"pageable_agg": pag_agg, "pageable_own": pag_own,
            "autopin_agg": ap_agg, "autopin_own": ap_own, "autopin_first_agg": ap_first_agg,
            "autopin_first_own": ap_first_own,
            "autopin_equal": d_ap is not None and d_ap2 is not None and bool(np.array_equal(d_ap, d_pag))
            and bool(np.array_equal(d_ap2, d_pag)),
            "registered_agg": reg_agg, "registered_own": reg_own, "register_s": reg_s,
            "direct_fraction": (s1["direct"] - s0["direct"]) / max(1, 3 * host_data.size),
            "digests": d_pag, "registered_equal": d_reg is not None and bool(np.array_equal(d_reg, d_pag)),
            "placement": placement, "error": err[0] if err else None}


def inproc_leg(buf, slice_bytes, cs, shard_starts, slice_hashes):
    """EncodeFile's shape on an N-GPU node: ONE process, ONE lbf_ctx over the
    run's N devices (the first N visible; all of them on a rehearsal with fewer
    GPUs than ranks), lbf_sha1_batch on one N x slice_bytes host buffer (slice r
    = the bytes rank r hashed in its e2e leg), registered, then pageable.  Run
    by rank 0 after the other ranks have finished.  `buf` (a device buffer of
    at least slice_bytes) generates each slice; parity: slice r's digests must
    hash to rank r's reported slice hash (its device-resident digests, which
    were checked against the golden of its shard)."""
    from bitflood_amd import ChunkHasher, chunk_table
    world = len(shard_starts)
    total = world * slice_bytes
    big = np.empty(total, dtype=np.uint8)
    for r, start in enumerate(shard_starts):
        buf.fill_synthetic(SEED_C, start=start, nbytes=slice_bytes)
        H.synchronize()
        buf.download_into(big[r * slice_bytes:(r + 1) * slice_bytes])
    offs, sizes = chunk_table(total, cs)
    per_slice = slice_bytes // cs
    gib = total / GIB

    def best(h, k):
        t, d = float("inf"), None
        for _ in range(k):
            t0 = time.perf_counter()
            d = h.hash_chunks(big, offs, sizes)
            t = min(t, time.perf_counter() - t0)
        return gib / t, d

    # the N GPUs the ranks ran on, not every GPU the node has (N=2 on an 8-GPU node)
    use = min(world, max(1, torch.cuda.device_count()))
    with ChunkHasher(device_mask=(1 << use) - 1) as h:
        info = [h.worker_info(w) for w in range(h.num_workers)]
        ndev = h.num_devices
        h.hash_chunks(big, offs, sizes)  # warm: every worker's staging and device slots
        s0 = h.staging_stats()
        pag, d_pag = best(h, 2)
        # the pageable passes' route: the staging memcpy by default (0 here);
        # with LBF_AUTOPIN=1, pinned on the fly for the whole job (one
        # registration shared by every worker)
        pag_direct = (h.staging_stats()["direct"] - s0["direct"]) / (2 * total)
        t0 = time.perf_counter()
        h.register_host(big)
        reg_s = time.perf_counter() - t0
        try:
            reg, d_reg = best(h, 3)
            st = h.staging_stats()
        finally:
            h.unregister_host(big)
    del big
    ok = [int(slice_hash(d_reg[r * per_slice:(r + 1) * per_slice]) == slice_hashes[r]) for r in range(world)]
    return {
        "what": f"one process, one lbf_ctx over {use} device(s), lbf_sha1_batch on one host buffer of "
                f"{world} x {slice_bytes / GIB:g} GiB (slice r = rank r's e2e bytes)",
        "devices": ndev, "workers": len(info), "workers_per_device": int(os.environ.get("LBF_WORKERS_PER_DEVICE", "1")),
        "bytes": total, "chunk_size": cs,
        "registered_gibs": round(reg, 3), "register_s": round(reg_s, 4), "pageable_gibs": round(pag, 3),
        "pageable_direct_fraction": round(pag_direct, 4),
        "direct_bytes": st["direct"],
        "parity_per_slice": ok, "parity": all(ok) and bool(np.array_equal(d_reg, d_pag)),
        "placement": info,
    }


def slice_hash(digests):
    """56-bit fingerprint of a digest slice (fits an int64 all-gather)."""
    return int.from_bytes(hashlib.sha1(np.ascontiguousarray(digests).tobytes()).digest()[:7], "big")


def golden_for_rank(args, rank, file_bytes):
    """The committed golden of this rank's shard, or (None, None)."""
    g = os.path.join(ROOT, "tests", "golden")
    try:
        if args.config == "c2" and (file_bytes, args.chunk_size) == (4 * GIB, 262144):
            d = json.load(open(os.path.join(g, "c2_ranks.json")))
            return next((r for r in d["ranks"] if r["rank"] == rank), None), "tests/golden/c2_ranks.json"
        if args.config == "c4" and (file_bytes, args.chunk_size) == (32 * GIB, 1 << 20):
            d = json.load(open(os.path.join(g, "c4.json")))
            return next((r for r in d["shards"] if r["rank"] == rank), None), "tests/golden/c4.json"
    except OSError:
        pass
    return None, None


def check_golden(gold, digests):
    """1 = this rank's digests match its golden shard, 0 = mismatch, -1 = no golden."""
    if gold is None:
        return -1
    ok = hashlib.sha1(digests.tobytes()).hexdigest() == gold["sha1_of_concat_raw_digests_hex"]
    ok = ok and digests.shape[0] == gold["n_chunks"]
    for k, v in gold.get("samples_b64", {}).items():
        ok = ok and b64_27(bytes(digests[int(k)])) == v
    return 1 if ok else 0


def config_entry(name, length, cs, ms, ok, gold, kernel, pmc_path=None):
    """One other_configs record: rate, HBM fraction and, through the same rule
    as the main line (traffic_from_profiles), the PMC traffic recorded for
    this kernel's machine code at this size, or null with the reason."""
    code_sym, code_sha = kernel_code_digest(kernel)
    traffic, src, why = traffic_from_profiles(length, cs, kernel, code_sha, path=pmc_path)
    return {"workload": name, "bytes": length, "chunk_size": cs, "chunks": length // cs, "kernel": kernel,
            "ms_per_launch": round(ms, 4), "gibs": round(length / GIB / (ms / 1e3), 1),
            "hbm_frac": round(length / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": traffic, "traffic_ratio": round(traffic / length, 5) if traffic else None,
            "traffic_source": src, "traffic_null_reason": why,
            "kernel_code_sha256": code_sha, "kernel_symbol": code_sym, "golden": gold, "parity": ok}


def other_configs():
    """C3 and C4 (BASELINE.json configs[2], configs[3] per GPU), device-resident,
    measured after the main line at N=1 and checked against their goldens:
    secondary numbers for DESIGN.md §5, never `value`.  A failure is recorded,
    not raised."""
    g = os.path.join(ROOT, "tests", "golden")
    res = {}
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream

    def timed(buf, length, cs, n, dig, reps=3):
        H.uniform_launch(buf, length, cs, 0, n, dig, stream=sptr)  # warm-up
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            H.uniform_launch(buf, length, cs, 0, n, dig, stream=sptr)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    def entry(name, length, cs, ms, ok, gold):
        return config_entry(name, length, cs, ms, ok, gold, KERNELS.get(H.load().lbf_kernel_for(length // cs), "?"))

    for name in ("C3", "C4"):
        buf = dig = None
        try:
            if name == "C3":
                c3 = json.load(open(os.path.join(g, "c3.json")))
                fs, cs = c3["file_size"], c3["chunk_size"]
                length = fs * len(c3["files"])
                buf = DeviceBuffer(length)
                for f in range(len(c3["files"])):  # file f = stream seed f from byte 0
                    buf.fill_synthetic(f, start=0, nbytes=fs, stream=sptr, offset=f * fs)
                n = length // cs
                dig = DeviceBuffer(n * 20)
                ms = timed(buf, length, cs, n, dig)
                d = dig.download(n * 20)
                ok = hashlib.sha1(d.tobytes()).hexdigest() == c3["sha1_of_all_digests_in_file_order_hex"]
                res[name] = entry("C3: 64 files x 1 GiB, 256 KiB chunks, one launch", length, cs, ms, ok,
                                  "tests/golden/c3.json")
            else:
                c4 = json.load(open(os.path.join(g, "c4.json")))
                cs, length = c4["chunk_size"], 32 * GIB
                gold = next(r for r in c4["shards"] if r["rank"] == 0)
                buf = DeviceBuffer(length)
                buf.fill_synthetic(SEED_C, start=0, stream=sptr)
                n = length // cs
                dig = DeviceBuffer(n * 20)
                ms = timed(buf, length, cs, n, dig)
                ok = check_golden(gold, dig.download(n * 20).reshape(n, 20)) == 1
                res[name] = entry("C4 per GPU: shard 0 (32 GiB) of the 256 GiB file, 1 MiB chunks", length, cs, ms,
                                  ok, "tests/golden/c4.json shard 0")
        except Exception as e:  # recorded in the line; the main measurement stands
            res[name] = {"error": f"{type(e).__name__}: {e}"}
        finally:
            for b in (buf, dig):
                if b is not None:
                    b.free()
    return res


def _gather(x, world, dtype):
    if not grouped():
        return [x]
    import torch.distributed as dist
    backend = dist.get_backend()
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=dtype, device=dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.item() for p in parts]


def gather_ints(x, world):
    return [int(v) for v in _gather(int(x), world, torch.int64)]


def gather_floats(x, world):
    return [float(v) for v in _gather(float(x), world, torch.float64)]


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        if under_profiler():
            # the profiler's preload has initialised the GPU in this process: a
            # launcher here would start GPU children from it (not allowed)
            raise SystemExit("bench.py: --gpus N without a launcher starts its own rank processes, which is not "
                             "allowed under rocprofv3; profile one rank per process instead (torch.distributed.run "
                             "with rocprofv3 inside each rank, or --gpus 1)")
        # no outside launcher: start the N ranks here (children, never exec)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    rank, world, local, dev, ndev = dist_setup(args)
    multi = grouped()  # world > 1, or a one-rank group (LBF_BENCH_FORM_GROUP)
    if args.variant:
        H.set_kernel_variant(args.variant)
    cs = args.chunk_size
    file_bytes = int(args.file_gib * GIB)
    n_chunks = (file_bytes + cs - 1) // cs
    # this rank's contiguous shard of the N x file_bytes file (weak scaling)
    first, last = shard_range(world * n_chunks, rank, world)
    stream_start = first * cs

    buf = DeviceBuffer(file_bytes)
    dig = DeviceBuffer(n_chunks * 20)
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream
    buf.fill_synthetic(SEED_C, start=stream_start, stream=sptr)
    torch.cuda.synchronize()

    def step():
        H.uniform_launch(buf, file_bytes, cs, 0, n_chunks, dig, stream=sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    # HIP events recorded on the stream the kernels run on (torch's current stream)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    wall = t1 - t0
    ev_ms = e0.elapsed_time(e1)
    t_max = max_over_ranks(wall, world)
    ev_max = max_over_ranks(ev_ms, world)
    per_rank_kernel_ms = [round(x / args.steps, 4) for x in gather_floats(ev_ms, world)]

    total_bytes = world * file_bytes * args.steps
    value = total_bytes / GIB / t_max
    launch_s = ev_max / 1e3 / args.steps
    achieved_gbs = file_bytes / launch_s / 1e9

    digests = dig.download(n_chunks * 20).reshape(n_chunks, 20)
    # every rank checks its own shard against the committed golden
    gold, gold_path = golden_for_rank(args, rank, file_bytes)
    per_rank = gather_ints(check_golden(gold, digests), world)
    per_rank_dev = gather_ints(dev, world)

    # N>1: the copy-inclusive rate with every rank pulling from host memory at once
    e2e_multi = None
    n_slice = min(file_bytes, E2E_SLICE_BYTES) // cs  # whole chunks only
    slice_bytes = n_slice * cs
    if multi:
        # the host slice, then free the shard's HBM before the host-memory legs:
        # with ranks sharing a GPU (rehearsals: 8 x 32 GiB of C4 on one card)
        # their contexts' device slots would not fit beside it
        host = buf.download(slice_bytes) if not args.no_e2e else None
        buf.free()
        buf = None
    if multi and not args.no_e2e and n_slice:
        r = e2e_leg(host, cs, dev, world)
        del host
        ok = int(np.array_equal(r["digests"], digests[:n_slice]) and r["registered_equal"] and r["autopin_equal"])
        g = {k: gather_floats(r[k], world)
             for k in ("pageable_own", "autopin_own", "autopin_first_own", "registered_own", "register_s")}
        e2e_multi = {
            "what": f"every rank hashes the first {slice_bytes / GIB:g} GiB of its shard from host memory at the "
                    "same moment through its own lbf_ctx (NUMA-local pinned staging): pageable (the default route, "
                    "the staging memcpy), pinned on the fly (opt-in, on a fresh copy: its first pass, then best of "
                    "3), then registered; best of 3 synchronized passes",
            "bytes_per_rank": slice_bytes, "chunk_size": cs,
            "pageable": {"aggregate_gibs": round(r["pageable_agg"], 3),
                         "per_rank_gibs": [round(x, 3) for x in g["pageable_own"]],
                         "route": "the staging memcpy into NUMA-local pinned slots (the default)"},
            "autopin": {"aggregate_gibs": round(r["autopin_agg"], 3),
                        "per_rank_gibs": [round(x, 3) for x in g["autopin_own"]],
                        "first_pass_aggregate_gibs": round(r["autopin_first_agg"], 3),
                        "first_pass_per_rank_gibs": [round(x, 3) for x in g["autopin_first_own"]],
                        "route": "pinned on the fly (LBF_AUTOPIN=1, opt-in since round 6): the first pass pays "
                                 "the first registration of the pages"},
            "registered": {"aggregate_gibs": round(r["registered_agg"], 3),
                           "per_rank_gibs": [round(x, 3) for x in g["registered_own"]],
                           "register_s_per_rank": [round(x, 4) for x in g["register_s"]],
                           "direct_fraction_rank0": round(r["direct_fraction"], 4)},
            "parity_per_rank": gather_ints(ok, world),
            "numa_per_rank": [{"device": d, "numa_node": n, "staging_node": s} for d, n, s in zip(
                per_rank_dev, gather_ints(r["placement"]["numa_node"], world),
                gather_ints(r["placement"]["staging_node"], world))],
        }
        e2e_multi["parity"] = all(x == 1 for x in e2e_multi["parity_per_rank"])
        e2e_multi["failed_per_rank"] = gather_ints(r["error"] is not None, world)
        if r["error"]:
            e2e_multi["error_rank0"] = r["error"]
    slice_hashes = gather_ints(slice_hash(digests[:n_slice]), world)
    gpu0_numa = None
    shard_starts = [shard_range(world * n_chunks, q, world)[0] * cs for q in range(world)]

    variant = H.load().lbf_kernel_for(n_chunks)
    floor_ms = compute_floor_ms(variant, cs, n_chunks)
    kernel = KERNELS.get(variant, str(variant))
    code_sym, code_sha = kernel_code_digest(kernel)
    traffic, traffic_src, traffic_null = traffic_from_profiles(file_bytes, cs, kernel, code_sha)
    out = None
    if rank == 0:
        c2 = (file_bytes, cs) == (4 * GIB, 262144)
        c4 = (file_bytes, cs) == (32 * GIB, 1 << 20)
        workload = ("C2 per GPU: one 4 GiB file, 256 KiB chunks, SHA-1 -> 20 B digest per chunk "
                    "(BASELINE.json configs[1]); N GPUs = N x 4 GiB file, contiguous chunk shards" if c2 else
                    "C4 per GPU: a 32 GiB shard of the 256 GiB file at 1 MiB chunks, SHA-1 -> 20 B digest per "
                    "chunk (BASELINE.json configs[3]); rank r hashes shard r" if c4 else
                    f"custom per GPU: {file_bytes / GIB:g} GiB file, {cs // 1024} KiB chunks, SHA-1 -> 20 B "
                    f"digest per chunk; N GPUs = N such shards")
        out = {
            "metric": "GiB/s device-resident chunk hashing, 256 KiB chunks, at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: counter-mode splitmix64 stream seed 0x5EED generated in HBM "
                    f"(rank r hashes bytes [r*{file_bytes / GIB:g}GiB,(r+1)*{file_bytes / GIB:g}GiB) of it)",
            "config": {
                "workload": workload,
                "file_bytes_per_gpu": file_bytes,
                "chunk_size": cs,
                "chunks_per_gpu": n_chunks,
                "kernel": kernel,
                "parallelism": f"chunk-shard x{world} (no data-path collective)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_null_reason": traffic_null,
                "kernel_code_sha256": code_sha,
                "kernel_symbol": code_sym,
                "kernel_ms": round(launch_s * 1e3, 4),
                "algorithmic_bytes_per_launch": file_bytes,
                # what the HBM fraction can reach at all: SHA-1 is a serial chain per
                # chunk, so with this many chunks the launch cannot beat the chain's
                # instruction-issue floor
                "ceiling_frac": round(file_bytes / (floor_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "ceiling_reason": (f"{n_chunks} serial SHA-1 chains: the issue floor below ({floor_ms:.3f} ms) "
                                   "bounds the launch, not HBM"),
                "per": "GPU (the slowest rank's HIP-event launch time)",
                # all N GPUs together: N shards in the slowest rank's launch time,
                # against N x the HBM peak
                "aggregate_achieved": round(world * achieved_gbs, 2),
                "aggregate_peak": world * HBM_PEAK_GBS,
            },
            # SHA-1 is integer VALU work on a serial chain per chunk: the binding
            # limit is instruction issue, not HBM.
            "compute_floor": {
                "bound": "per-chain issue" if variant in (2, 4, 5, 6, 7, 8, 9, 10, 12) else "valu",
                "floor_ms": round(floor_ms, 4),
                "frac": round(floor_ms / (launch_s * 1e3), 4),
                "clock_ghz": CLOCK_HZ / 1e9,
            },
            "digest_check": hashlib.sha1(digests.tobytes()).hexdigest(),
            "parity": {
                "golden": gold_path,
                "per_rank": per_rank,  # 1 match, 0 mismatch, -1 no golden for that shard
                "all_ranks_match_golden": all(x == 1 for x in per_rank),
            },
            "ranks": {
                "launcher": os.environ.get("LBF_BENCH_LAUNCHER", "torch.distributed.run" if world > 1 else "none"),
                "process_group": backend_name() if multi else None,
                "visible_gpus": ndev,
                "device_per_rank": per_rank_dev,
                "kernel_ms_per_rank": per_rank_kernel_ms,
                "rehearsal": world > ndev,
            },
        }
        if world > ndev:
            out["ranks"]["note"] = (f"{world} ranks share {ndev} GPU(s): a rehearsal of the N-rank flow; their "
                                    "launches queue on the shared device, so value is not an N-GPU rate")
        if e2e_multi is not None:
            out["e2e"] = e2e_multi
        if not multi:
            if not args.no_e2e:
                # the whole file, copied back from HBM into pageable host memory
                host_file = buf.download(file_bytes)
                r = e2e_leg(host_file, cs, dev, 1)
                del host_file
                out["e2e_host_to_host_gibs"] = round(r["pageable_own"], 3)
                out["e2e_route"] = ("pageable memory through the staging memcpy into NUMA-local pinned slots (the "
                                    "default; on-the-fly pinning is opt-in since round 6, DESIGN.md §9 item 6)")
                out["e2e_autopin"] = {"gibs": round(r["autopin_own"], 3),
                                      "first_pass_gibs": round(r["autopin_first_own"], 3),
                                      "parity": r["autopin_equal"],
                                      "route": "a fresh copy of the bytes pinned on the fly (LBF_AUTOPIN=1): its "
                                               "first pass, which pays the pages' first registration, then best "
                                               "of 3"}
                out["e2e_bytes"] = file_bytes
                out["e2e_parity"] = bool(np.array_equal(r["digests"], digests))
                out["e2e_staging"] = r["placement"]
                out["e2e_registered"] = {"gibs": round(r["registered_own"], 3), "register_s": round(r["register_s"], 4),
                                         "direct_fraction": round(r["direct_fraction"], 4),
                                         "parity": r["registered_equal"]}
                if r["error"]:
                    out["e2e_error"] = r["error"]
                gpu0_numa = r["placement"]["numa_node"]
        out["first_chunk_b64"] = b64_27(bytes(digests[0]))
    if multi:
        import torch.distributed as dist
        barrier(world)  # every rank's e2e leg has ended before rank 0 goes on alone
        dist.destroy_process_group()
    if rank == 0 and multi and not args.no_e2e and not args.no_inproc and n_slice:
        gen = None
        try:
            gen = DeviceBuffer(slice_bytes)
            out["e2e_inprocess"] = inproc_leg(gen, slice_bytes, cs, shard_starts, slice_hashes)
        except Exception as e:  # recorded in the line; the main measurement stands
            out["e2e_inprocess"] = {"error": f"{type(e).__name__}: {e}"}
        finally:
            if gen is not None:
                gen.free()
    if buf is not None:
        buf.free()
    dig.free()
    if rank == 0 and not multi and not args.no_other_configs and args.config == "c2":
        out["other_configs"] = other_configs()
    if rank == 0 and not args.no_cpu_baseline:
        # at every N, rank 0 alone once the GPU legs are over (the other ranks
        # have left the group), on the same stream as its shard
        sample = min(n_chunks, max(1, GIB // cs))
        try:
            cb = cpu_baseline(args, stream_start, sample, digests[:sample])
        except Exception as e:  # a host-side failure must not cost the line its device-resident value
            cb = {"value": None, "unit": "GiB/s", "cores": None, "kind": "port",
                  "error": f"{type(e).__name__}: {e}", "host": {}}
        if e2e_multi is not None:
            gpu0_numa = e2e_multi["numa_per_rank"][0]["numa_node"]
        if gpu0_numa is not None:
            cb["host"]["gpu0_numa_node"] = gpu0_numa
        cb["when"] = ("after the timed region and the host-memory legs, rank 0 alone"
                      + ("" if world == 1 else " (rank 1 has finished)" if world == 2 else
                         f" (ranks 1-{world - 1} have finished)"))
        out["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
