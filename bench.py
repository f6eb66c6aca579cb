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
   N>1:  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
Rank 0 prints ONE JSON line.
"""
import math
import argparse
import hashlib
import json
import os
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
           6: "sha1_pc4_kernel<true, 4>", 7: "sha1_pc4_kernel<true, 2>", 8: "sha1_pc4_kernel<true, 1>",
           9: "sha1_pcx4_kernel<true, 40>", 10: "sha1_pcx5_kernel<true, 64>",
           11: "sha1_lds2_kernel<true>"}
# Issue floors per 64-byte block (tools/gen_round_order.py, tools/probe_lds_lanes.hip):
#  pc2/pc4 consumer: 80 rounds x 5 VALU at one issue per 4.09 cycles -- the chain's own
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
    ap.add_argument("--no-e2e", action="store_true", help="skip the host->device->host rate")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the device-resident C3 and C4 measurements that follow the main line at N=1")
    a = ap.parse_args()
    a.chunk_size = a.chunk_size or {"c2": 262144, "c4": 1 << 20}[a.config]
    a.file_gib = a.file_gib or {"c2": 4.0, "c4": 32.0}[a.config]
    return a


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        # one rank per GPU; more ranks than GPUs only for rehearsals of the
        # multi-rank flow on a small box (LBF_BENCH_BACKEND=gloo)
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        backend = os.environ.get("LBF_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    else:
        torch.cuda.set_device(0)
    if args.gpus != world:
        if rank == 0:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}", file=sys.stderr)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def traffic_from_profiles(file_bytes, chunk_size, kernel):
    """HBM bytes per launch measured with rocprofv3 PMC (FETCH_SIZE x2, gfx950
    correction), recorded by tools/pmc_traffic.py --record for
    this workload size and this kernel.  A static lookup, not a measurement of
    this run: it goes null when the kernel or the size differ."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        for e in d.get("entries", [d]):
            if (int(e.get("file_bytes", -1)) == int(file_bytes) and int(e.get("chunk_size", 262144)) == chunk_size
                    and kernel in e.get("kernel", "")):
                return float(e["hbm_bytes_per_launch"]), e.get("source", p)
    except Exception:
        pass
    return None, None


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
    """The oracle restatement of the reference encoder hash (portable C -O2,
    oracle/sha1_oracle.c) on the host cores, over a bounded sample of the same
    synthetic bytes.  kind="port": building the reference was denied
    (SURVEY.md §8c).  Threads: every CPU the process may use (SURVEY.md §8d
    (ii)), i.e. its affinity mask capped by the cgroup CPU quota; the same
    sample on one thread per affinity CPU shows what the quota allows."""
    from tests.oracle_lib import Oracle
    orc = Oracle()
    cs = args.chunk_size
    nbytes = n_chunks_sample * cs
    affinity, quota, usable = host_cpus()
    threads = args.cpu_threads or usable
    data = orc.synth(SEED_C, stream_start, nbytes, nthreads=threads)
    offs = np.arange(n_chunks_sample, dtype=np.uint64) * np.uint64(cs)
    sizes = np.full(n_chunks_sample, cs, dtype=np.uint32)

    def rate(nthreads, min_s=3.0, max_reps=20):
        reps, t = 0, 0.0
        d = None
        while t < min_s and reps < max_reps:
            t0 = time.perf_counter()
            d = orc.sha1_batch(data, offs, sizes, nthreads=nthreads)
            t += time.perf_counter() - t0
            reps += 1
        return reps * nbytes / GIB / t, reps, d

    # all usable host cores, chunk-parallel
    mt_gibs, reps, d_mt = rate(threads)
    # one thread per CPU of the affinity mask (256 on a GPU box): what the quota lets through
    aff_gibs = rate(affinity, min_s=1.0, max_reps=3)[0] if affinity != threads else mt_gibs
    # one thread, like Encoder.cpp:40-79 (bounded to 1/4 of the sample)
    n1 = max(1, n_chunks_sample // 4)
    t0 = time.perf_counter()
    d_1 = orc.sha1_batch(data, offs[:n1], sizes[:n1], nthreads=1)
    t_1 = time.perf_counter() - t0
    st_gibs = n1 * cs / GIB / t_1
    # fread-inclusive single-thread encode of the same bytes as a file, as
    # Encoder::EncodeFile does it (one chunk buffer, fread + hash per chunk;
    # oracle_encode_file); the file is page-cache warm, written just before
    import tempfile
    fread = None
    with tempfile.NamedTemporaryFile(prefix="lbf_cpu_sample_", dir=os.environ.get("TMPDIR", "/tmp")) as f:
        data[: n1 * cs].tofile(f.name)
        dig = np.zeros((n1, 20), dtype=np.uint8)
        t0 = time.perf_counter()
        got = orc.lib.oracle_encode_file(f.name.encode(), cs, dig.ctypes.data, n1, None)
        t_f = time.perf_counter() - t0
        if got == n1:
            fread = {"value": round(n1 * cs / GIB / t_f, 3), "unit": "GiB/s",
                     "sample": f"{n1} x {cs // 1024} KiB chunks from a page-cached file, 1 thread",
                     "parity_vs_gpu": bool(np.array_equal(dig, gpu_digests_sample[:n1]))}
    parity = bool(np.array_equal(d_mt, gpu_digests_sample) and np.array_equal(d_1, gpu_digests_sample[:n1]))
    return {
        "value": round(mt_gibs, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "sample": f"{n_chunks_sample} x {cs // 1024} KiB chunks ({nbytes / GIB:.2f} GiB) of the same stream, "
                  f"{reps} pass(es) on {threads} threads; single-thread pass over {n1} chunks",
        "single_thread_value": round(st_gibs, 3),
        "affinity_threads_value": round(aff_gibs, 3),
        "single_thread_fread_encode": fread,
        "host": {**_host_desc(), "affinity_cores": affinity, "cgroup_cpu_quota": quota, "usable_cores": usable,
                 "numa_nodes": _numa_nodes()},
        "parity_vs_gpu": parity,
    }, data


def _host_desc():
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"cpu_model": model, "os_cpu_count": os.cpu_count()}


def compute_floor_ms(variant, cs, n_chunks):
    """Lower bound on one launch from instruction issue alone (SHA-1 is a serial
    chain per chunk, so few chunks are bound by one chain's issue rate)."""
    blocks = (cs + 9 + 63) // 64  # compressions per chunk incl. padding
    if variant in (4, 6, 7, 8):
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


def e2e_rate(host_data, cs):
    """Host bytes in -> host digests out through the lbf_ctx pinned pipeline
    (PCIe-inclusive rate for DESIGN.md; never the headline value), from
    pageable memory and from the same memory registered with the context."""
    from bitflood_amd import ChunkHasher, chunk_table
    offs, sizes = chunk_table(host_data.size, cs)
    with ChunkHasher(device_mask=1) as h:
        # warm: one untimed pass sizes the context's pinned staging to this job
        # (it grows on demand; tools/file_rate.py reports the one-shot cost)
        h.hash_chunks(host_data, offs, sizes)
        t = float("inf")
        for _ in range(3):  # best of 3: a lone pass swings with the host's other tenants
            t0 = time.perf_counter()
            d = h.hash_chunks(host_data, offs, sizes)
            t = min(t, time.perf_counter() - t0)
        placement = h.worker_info(0)
        # The same bytes from caller memory registered with the context
        # (lbf_host_register): straight to HBM with ordered copies, no staging
        # memcpy.  Pinning is a one-off cost of a reused buffer, reported apart.
        t0 = time.perf_counter()
        h.register_host(host_data)
        reg_s = time.perf_counter() - t0
        s0 = h.staging_stats()
        t_reg = float("inf")
        try:
            for _ in range(3):
                t0 = time.perf_counter()
                d_reg = h.hash_chunks(host_data, offs, sizes)
                t_reg = min(t_reg, time.perf_counter() - t0)
            s1 = h.staging_stats()
        finally:
            h.unregister_host(host_data)
    registered = {"gibs": round(host_data.size / GIB / t_reg, 3), "register_s": round(reg_s, 4),
                  "direct_fraction": round((s1["direct"] - s0["direct"]) / max(1, 3 * host_data.size), 4),
                  "parity": bool(np.array_equal(d_reg, d))}
    return host_data.size / GIB / t, d, placement, registered


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
        return {"workload": name, "bytes": length, "chunk_size": cs, "chunks": length // cs,
                "kernel": KERNELS.get(H.load().lbf_kernel_for(length // cs), "?"), "ms_per_launch": round(ms, 4),
                "gibs": round(length / GIB / (ms / 1e3), 1),
                "hbm_frac": round(length / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4), "golden": gold, "parity": ok}

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


def gather_ints(x, world):
    if world == 1:
        return [int(x)]
    import torch.distributed as dist
    backend = dist.get_backend()
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [int(p.item()) for p in parts]


def main():
    args = parse()
    rank, world, local = dist_setup(args)
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

    total_bytes = world * file_bytes * args.steps
    value = total_bytes / GIB / t_max
    launch_s = ev_max / 1e3 / args.steps
    achieved_gbs = file_bytes / launch_s / 1e9

    digests = dig.download(n_chunks * 20).reshape(n_chunks, 20)
    # every rank checks its own shard against the committed golden
    gold, gold_path = golden_for_rank(args, rank, file_bytes)
    per_rank = gather_ints(check_golden(gold, digests), world)
    variant = H.load().lbf_kernel_for(n_chunks)
    floor_ms = compute_floor_ms(variant, cs, n_chunks)
    kernel = KERNELS.get(variant, str(variant))
    traffic, traffic_src = traffic_from_profiles(file_bytes, cs, kernel)
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
                "traffic_source": traffic_src and f"{traffic_src} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, same "
                                                  "kernel and size; a recorded lookup, not this run's counters)",
                "kernel_ms": round(launch_s * 1e3, 4),
                "algorithmic_bytes_per_launch": file_bytes,
                # what the HBM fraction can reach at all: SHA-1 is a serial chain per
                # chunk, so with this many chunks the launch cannot beat the chain's
                # instruction-issue floor
                "ceiling_frac": round(file_bytes / (floor_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "ceiling_reason": (f"{n_chunks} serial SHA-1 chains: the issue floor below ({floor_ms:.3f} ms) "
                                   "bounds the launch, not HBM"),
            },
            # SHA-1 is integer VALU work on a serial chain per chunk: the binding
            # limit is instruction issue, not HBM.
            "compute_floor": {
                "bound": "per-chain issue" if variant in (2, 4, 5, 6, 7, 8, 9, 10) else "valu",
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
        }
        if world == 1 and not args.no_cpu_baseline:
            sample = min(n_chunks, max(1, GIB // cs))
            cb, host = cpu_baseline(args, stream_start, sample, digests[:sample])
            out["cpu_baseline"] = cb
            if not args.no_e2e:
                # the whole file, copied back from HBM into pageable host memory
                host_file = buf.download(file_bytes)
                rate, d_e2e, placement, registered = e2e_rate(host_file, cs)
                del host_file
                out["e2e_host_to_host_gibs"] = round(rate, 3)
                out["e2e_bytes"] = file_bytes
                out["e2e_parity"] = bool(np.array_equal(d_e2e, digests))
                out["e2e_staging"] = placement
                out["e2e_registered"] = registered
                cb["host"]["gpu0_numa_node"] = placement["numa_node"]
        out["first_chunk_b64"] = b64_27(bytes(digests[0]))
    buf.free()
    dig.free()
    if rank == 0 and world == 1 and not args.no_other_configs and args.config == "c2":
        out["other_configs"] = other_configs()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
