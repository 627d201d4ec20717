#!/usr/bin/env python3
"""Headline benchmark: CRC32C GiB/s over device-resident item batches.

Workload (BASELINE.json configs[1], per GPU): 1 Mi items x 4096 B, contiguous,
stride 4096, random bytes; one step = one crc32c_batch() over the whole batch
(K1 kernel).  With N GPUs every rank checksums its own 1 Mi items (BASELINE
config 4 at N = 8: 8 Mi items), so per-GPU work is fixed ("scaling": "weak");
the ranks share nothing but the timing barrier (no data-path collective).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints one JSON line.  `value` = all ranks' bytes / max-over-ranks time.
`roofline.achieved` = algorithmic bytes per launch (sum of span lengths) / the
average kernel duration measured with HIP events on the launch stream.
`cpu_baseline` = the reference crc32c.c (compiled under oracle/_ref) on the
host cores, rank 0, on a bounded sample of the same items; its CRCs are also
compared with the GPU's for those items.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

import torch  # load torch (and its HIP runtime) before the library

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from memcached_amd import _lib  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md chip table (spec)
ITEM_BYTES = 4096
ITEMS_PER_GPU = 1 << 20


def shard(n_total: int, rank: int, world: int):
    """Contiguous, byte-balanced shard of equal-size items for `rank`."""
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi


def dist_setup(n_gpus: int, backend: str = "nccl"):
    """One process per GPU; RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the
    launcher.  The process group only carries the timing barrier and the
    max-over-ranks reduction ("nccl" is RCCL on ROCm; "gloo" for CPU tests)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    if backend == "nccl":
        torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed(step, steps: int, world: int, sync=torch.cuda.synchronize):
    """Barrier + sync, run `steps` steps, sync + barrier; max wall time over ranks."""
    barrier(world)
    sync()
    t0 = time.perf_counter()
    r = step(steps)
    sync()
    barrier(world)
    return max_over_ranks(time.perf_counter() - t0, world), r


def splitmix64_bytes(nbytes: int, seed: int, chunk_words: int = 1 << 26, device: str = "cuda") -> torch.Tensor:
    """SURVEY.md 8(d) config 2 input: little-endian splitmix64(seed) words,
    word i = mix(seed + (i + 1) * golden), generated on the device in chunks."""
    assert nbytes % 8 == 0
    words = torch.empty(nbytes // 8, dtype=torch.int64, device=device)
    golden = 0x9E3779B97F4A7C15 - (1 << 64)  # as int64 (wrapping arithmetic)
    m1, m2 = 0xBF58476D1CE4E5B9 - (1 << 64), 0x94D049BB133111EB - (1 << 64)

    def srl(x, k):  # logical shift right on int64
        return (x >> k) & ((1 << (64 - k)) - 1)

    for lo in range(0, words.numel(), chunk_words):
        hi = min(lo + chunk_words, words.numel())
        z = torch.arange(lo + 1, hi + 1, dtype=torch.int64, device=device) * golden + seed
        z = (z ^ srl(z, 30)) * m1
        z = (z ^ srl(z, 27)) * m2
        words[lo:hi] = z ^ srl(z, 31)
    return words.view(torch.uint8)


def make_batch(n: int, seed: int, fill: str = "splitmix", device: str = "cuda"):
    if fill == "splitmix":
        data = splitmix64_bytes(n * ITEM_BYTES, seed, device=device)
    else:
        g = torch.Generator(device=device).manual_seed(seed)
        data = torch.randint(0, 256, (n * ITEM_BYTES,), dtype=torch.uint8, device=device, generator=g)
    out = torch.empty(n, dtype=torch.int32, device=device)
    spans = _lib.Spans(data.data_ptr(), data.numel(), None, ITEM_BYTES, None, ITEM_BYTES, None,
                       out.data_ptr(), n)
    return data, out, spans


def run_steps(spans, steps: int, stream, per_launch: bool = False):
    """Enqueue `steps` launches back to back on `stream`.  Events: one pair
    around all of them (default; sum of elapsed / steps = average launch
    duration), or one pair per launch (`per_launch`)."""
    flags = _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC
    npairs = steps if per_launch else 1
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(npairs)]
    for i in range(steps):
        if per_launch or i == 0:
            evs[i if per_launch else 0][0].record(stream)
        _lib.check(_lib.lib.crc32c_batch(ctypes.byref(spans), flags, ctypes.c_void_p(stream.cuda_stream)))
        if per_launch or i == steps - 1:
            evs[i if per_launch else 0][1].record(stream)
    return evs


def settle(step, ms: float) -> int:
    """Repeat `step` (in batches of 8) for `ms` of wall time before any
    warmup or timed step.  After idle the MI355X clock ramps over the first
    tens of launches (profiles/r01_ablations/k1_clock_ramp_800_launches.log:
    the first 20 launches average 1-2 % slower than the steady state), so a
    short warmup alone times part of the ramp.  Returns the launches run."""
    if ms <= 0:
        return 0
    n, t0 = 0, time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        step(8)
        torch.cuda.synchronize()
        n += 8
    return n


def cpu_topology():
    """Physical cores among the CPUs this process may run on: one logical CPU
    per (package, core) pair, from /sys topology.  Returns (cpus, sockets,
    logical count, model name)."""
    logical = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count()))
    first, pkgs = {}, set()
    for c in logical:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            key = (int(open(base + "physical_package_id").read()), int(open(base + "core_id").read()))
        except (OSError, ValueError):
            key = (0, c)
        pkgs.add(key[0])
        first.setdefault(key, c)
    model = "unknown CPU"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return sorted(first.values()), len(pkgs), len(logical), model


def cpu_baseline(data: torch.Tensor, out: torch.Tensor):
    """Reference crc32c.c on the host cores over the whole batch: one pthread
    per physical core (pinned, static contiguous split, best of 10 after a
    warm-up pass), plus the 1-core and 16-thread figures (16 = one GPU's share
    of the box's CPUs)."""
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")
    if not os.path.exists(ref):
        return {"value": None, "unit": "GiB/s", "cores": 0, "kind": "reference",
                "sample": "oracle/_ref/libref_crc32c.so missing (build in the container with /root/reference)"}
    import numpy as np
    lib = ctypes.CDLL(ref)
    lib.ref_crc32c_init()
    lib.ref_crc32c_batch_timed_cpus.restype = ctypes.c_double
    lib.ref_crc32c_batch_timed_cpus.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                                ctypes.c_void_p]
    n = out.numel()
    host = data[: n * ITEM_BYTES].cpu().numpy()
    crc = np.empty(n, np.uint32)
    cpus, sockets, nlogical, model = cpu_topology()
    cores = len(cpus)
    cpu_arr = np.asarray(cpus, np.int32)

    def rate(threads, passes, items):
        best = 0.0
        pin = cpu_arr.ctypes.data if threads <= cores else None
        lib.ref_crc32c_batch_timed_cpus(host.ctypes.data, None, None, ITEM_BYTES, ITEM_BYTES, items, threads,
                                        crc.ctypes.data, pin)
        for _ in range(passes):
            t = lib.ref_crc32c_batch_timed_cpus(host.ctypes.data, None, None, ITEM_BYTES, ITEM_BYTES, items, threads,
                                                crc.ctypes.data, pin)
            best = max(best, items * ITEM_BYTES / t / 2**30)
        return best

    one = rate(1, 3, min(n, 1 << 16))   # 1 core: the first 256 MiB, best of 3
    sixteen = rate(min(16, cores), 5, n)
    resident = rate(cores, 10, n)
    # NUMA-local: each pinned thread first copies its share into memory it
    # first-touches (its own node), then the shares are checksummed in parallel
    lib.ref_crc32c_batch_local.restype = ctypes.c_double
    lib.ref_crc32c_batch_local.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    crc[:] = 0
    local = n * ITEM_BYTES / lib.ref_crc32c_batch_local(host.ctypes.data, ITEM_BYTES, ITEM_BYTES, n, cores,
                                                         crc.ctypes.data, cpu_arr.ctypes.data, 10) / 2**30
    gpu = out[:n].cpu().numpy().view(np.uint32)
    return {"value": round(max(local, resident), 2), "unit": "GiB/s", "cores": cores, "kind": "reference",
            "sample": f"the whole GPU batch ({n} x {ITEM_BYTES} B, {n * ITEM_BYTES / 2**30:.0f} GiB) in host memory, "
                      f"reference crc32c.c (hw dispatch) per item as storage.c:567, one pinned pthread per physical "
                      f"core ({cores} cores, {sockets} socket(s), {nlogical} logical CPUs), static contiguous split, "
                      f"best of 10: {local:.2f} GiB/s with each thread's share in memory it first-touched (NUMA-local), "
                      f"{resident:.2f} GiB/s over the batch as copied from the GPU (one node); 16 threads: "
                      f"{sixteen:.2f} GiB/s; 1 core: {one:.2f} GiB/s (first 65536 items); {model}",
            "numa_local": round(local, 2), "resident": round(resident, 2), "one_core": round(one, 2),
            "sixteen_threads": round(sixteen, 2), "sockets": sockets, "cpu_model": model,
            "gpu_match": bool((gpu == crc).all())}


def zipf_lens(n: int, seed: int = 7):
    """BASELINE config 3 sizes: 44 classes 64 * 1.25^k <= 1 MiB, Zipf s = 1 over
    class rank (rank 1 = smallest), length uniform within +-half a class step."""
    import numpy as np
    rng = np.random.default_rng(seed)
    classes = 64 * 1.25 ** np.arange(44)
    classes = classes[classes <= 1 << 20]
    p = 1.0 / np.arange(1, classes.size + 1)
    k = rng.choice(classes.size, n, p=p / p.sum())
    step = classes[k] * 0.125
    return np.clip(classes[k] + rng.uniform(-step, step), 1, 1 << 20).astype(np.uint32)


_KEEP = []  # device tensors whose raw pointers a workload hands to the library


def workload_config3(args, rank, world):
    """1 Mi spans of Zipf sizes packed back to back at odd offsets (K2)."""
    import numpy as np
    lens = zipf_lens(args.items)
    offs = np.concatenate([[1], 1 + np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    total = int(offs[-1] + lens[-1] + 16)
    g = torch.Generator(device="cuda").manual_seed(3 + rank)
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda", generator=g)
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.empty(lens.size, dtype=torch.int32, device="cuda")
    spans = _lib.Spans(data.data_ptr(), total, d_offs.data_ptr(), 0, d_lens.data_ptr(), 0, None, out.data_ptr(),
                       lens.size)
    _KEEP.extend((data, d_offs, d_lens, out))  # the raw pointers in spans must outlive this frame
    return spans, int(lens.astype(np.uint64).sum()), {
        "workload": "BASELINE configs[2]: 1 Mi spans, Zipf sizes 64 B - 1 MiB (44 classes, s = 1), packed "
                    "back to back at odd offsets, K2 k_spans<unaligned>",
        "items_per_gpu": int(lens.size), "span_bytes_per_gpu": int(lens.astype(np.uint64).sum()),
        "items_le_4k_frac": round(float((lens <= 4096).mean()), 3)}


def run_verify_steps(args_v, steps: int, stream):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    base, size, region, offs, n, ok = args_v
    nbad = ctypes.c_uint64(0)
    for a, b in evs:
        a.record(stream)
        _lib.check(_lib.lib.crc32c_verify_items(base, size, region, offs, n, ok, ctypes.byref(nbad),
                                                _lib.CRC32C_DEVICE, ctypes.c_void_p(stream.cuda_stream)))
        b.record(stream)
    return evs, int(nbad.value)


def workload_config5(args, rank, world):
    """Extstore pages of packed 4165-byte item images, stored CRCs verified (K3).

    Pages: args.pages x 64 MiB, each 16 wbufs of 1007 items (key%07d, 4096-byte
    value, CAS) and a zero tail; 1 % of items get one flipped bit."""
    import numpy as np
    per_wbuf, ntotal, wbuf = 1007, 4165, 4 << 20
    nwb = args.pages * 16
    g = torch.Generator(device="cuda").manual_seed(5 + rank)
    data = torch.randint(0, 256, (nwb * wbuf,), dtype=torch.uint8, device="cuda", generator=g)
    wb = data.view(nwb, wbuf)
    wb[:, per_wbuf * ntotal:] = 0
    items = wb[:, : per_wbuf * ntotal].view(nwb, per_wbuf, ntotal)
    n = nwb * per_wbuf
    idx = torch.arange(n, device="cuda", dtype=torch.int64).view(nwb, per_wbuf)
    hdr = torch.zeros(nwb, per_wbuf, 67, dtype=torch.uint8, device="cuda")
    le = lambda v, k: torch.stack([(v >> (8 * i)) & 0xFF for i in range(k)], -1).to(torch.uint8)
    hdr[..., 24:28] = le(idx * 2654435761 & 0xFFFFFFFF, 4)        # time (hash)
    hdr[..., 32:36] = le(torch.full_like(idx, 4098), 4)            # nbytes (value + CRLF)
    hdr[..., 36] = 1                                               # refcount
    hdr[..., 38] = 2                                               # it_flags = ITEM_CAS
    hdr[..., 40] = 17                                              # slabs_clsid
    hdr[..., 41] = 10                                              # nkey
    hdr[..., 48:56] = le(idx + 1, 8)                               # CAS
    hdr[..., 56:59] = torch.tensor(list(b"key"), dtype=torch.uint8, device="cuda")
    for d in range(7):                                             # key%07d
        hdr[..., 65 - d] = (48 + (idx // 10 ** d) % 10).to(torch.uint8)
    hdr[..., 66] = 0
    items[..., :67] = hdr
    items[..., 4163] = 13
    items[..., 4164] = 10
    offs = (torch.arange(nwb, device="cuda", dtype=torch.int64)[:, None] * wbuf +
            torch.arange(per_wbuf, device="cuda", dtype=torch.int64)[None, :] * ntotal).reshape(-1).contiguous()
    # spill CRCs (storage.c:567) into exptime, computed by the span kernel
    span_offs = (offs + 32).contiguous()
    crc = torch.empty(n, dtype=torch.int32, device="cuda")
    sp = _lib.Spans(data.data_ptr(), data.numel(), span_offs.data_ptr(), 0, None, ntotal - 32, None,
                    crc.data_ptr(), n)
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), _lib.CRC32C_DEVICE, None))
    items[..., 28:32] = crc.view(torch.uint8).view(nwb, per_wbuf, 4)
    # inject one flipped bit into 1 % of items
    gen = torch.Generator(device="cuda").manual_seed(3)
    victims = torch.randperm(n, device="cuda", generator=gen)[: n // 100]
    pos = offs[victims] + 32 + torch.randint(0, ntotal - 32, (victims.numel(),), device="cuda", generator=gen)
    bit = torch.randint(0, 8, (victims.numel(),), device="cuda", generator=gen).to(torch.uint8)
    flat = data.view(-1)
    flat[pos] ^= (torch.ones_like(bit) << bit)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    _KEEP.extend((data, offs))  # the raw pointers below must outlive this frame
    return (data.data_ptr(), data.numel(), wbuf, offs.data_ptr(), n, ok.data_ptr()), ok, victims, \
        n * (ntotal - 32), {
            "workload": f"BASELINE configs[4]: {args.pages} x 64 MiB extstore pages, 16 wbufs x 1007 packed "
                        "4165-B item images each, stored CRC verified per item (K5 k_lines<verify>; other shapes "
                        "through the planned K3 path)",
            "pages_per_gpu": args.pages, "items_per_gpu": n, "span_bytes_per_gpu": n * (ntotal - 32),
            "injected_bad": int(victims.numel())}


def workload_pagesmix(args, rank, world):
    """Extstore pages of packed item images of mixed sizes, stored CRCs verified.

    Not a BASELINE config: a realistic page mix next to config 5's equal
    4165-B items.  Values are log-uniform 512 B - 64 KiB (extstore keeps items
    below ext_item_size = 512 B in RAM), key%07d keys, CAS; each 4 MiB wbuf is
    packed until the next item would not fit (extstore.c:591-670) and the rest
    zeroed; 1 % of items get one flipped bit."""
    import numpy as np
    wbuf, nwb = 4 << 20, args.pages * 16
    rng = np.random.default_rng(17 + rank)
    if args.workload == "mixed41":  # 2 KiB and 6 KiB values in turn: the average image is K5's ~4.2 KiB
        vals = np.broadcast_to(np.where(np.arange(1024) % 2, 2048, 6150), (nwb, 1024)).astype(np.int64)
    else:
        vals = np.exp(rng.uniform(np.log(512), np.log(65536), (nwb, 1024))).astype(np.int64)
    ntot = vals + 2 + 48 + 10 + 1 + 8                    # value + CRLF, header, key + NUL, CAS
    ends = np.cumsum(ntot, axis=1)
    keep = ends <= wbuf
    starts = ends - ntot
    offs_np = (np.arange(nwb, dtype=np.int64)[:, None] * wbuf + starts)[keep]
    ntot_np, vals_np = ntot[keep], vals[keep]
    n = int(offs_np.size)
    g = torch.Generator(device="cuda").manual_seed(9 + rank)
    data = torch.randint(0, 256, (nwb * wbuf,), dtype=torch.uint8, device="cuda", generator=g)
    wb = data.view(nwb, wbuf)
    for w, t in enumerate(np.where(keep, ends, 0).max(axis=1).tolist()):  # zero each wbuf's tail
        wb[w, t:] = 0
    offs = torch.from_numpy(offs_np).cuda()
    idx = torch.arange(n, device="cuda", dtype=torch.int64)
    nbytes = torch.from_numpy(vals_np + 2).cuda()
    le = lambda v, k: torch.stack([(v >> (8 * i)) & 0xFF for i in range(k)], -1).to(torch.uint8)
    hdr = torch.zeros(n, 67, dtype=torch.uint8, device="cuda")
    hdr[:, 24:28] = le(idx * 2654435761 & 0xFFFFFFFF, 4)          # time (hash)
    hdr[:, 32:36] = le(nbytes, 4)                                  # nbytes (value + CRLF)
    hdr[:, 36] = 1                                                 # refcount
    hdr[:, 38] = 2                                                 # it_flags = ITEM_CAS
    hdr[:, 40] = 17                                                # slabs_clsid
    hdr[:, 41] = 10                                                # nkey
    hdr[:, 48:56] = le(idx + 1, 8)                                 # CAS
    hdr[:, 56:59] = torch.tensor(list(b"key"), dtype=torch.uint8, device="cuda")
    for d in range(7):                                             # key%07d
        hdr[:, 65 - d] = (48 + (idx // 10 ** d) % 10).to(torch.uint8)
    flat = data.view(-1)
    flat[(offs[:, None] + torch.arange(67, device="cuda")[None, :]).reshape(-1)] = hdr.reshape(-1)
    end = offs + torch.from_numpy(ntot_np).cuda()
    flat[end - 2] = 13
    flat[end - 1] = 10
    # spill CRCs (storage.c:567) into exptime, computed by the span kernel
    span_offs = (offs + 32).contiguous()
    span_lens = torch.from_numpy((ntot_np - 32).astype(np.int32)).cuda()
    crc = torch.empty(n, dtype=torch.int32, device="cuda")
    sp = _lib.Spans(data.data_ptr(), data.numel(), span_offs.data_ptr(), 0, span_lens.data_ptr(), 0, None,
                    crc.data_ptr(), n)
    _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), _lib.CRC32C_DEVICE, None))
    flat[(offs[:, None] + 28 + torch.arange(4, device="cuda")[None, :]).reshape(-1)] = crc.view(torch.uint8)
    gen = torch.Generator(device="cuda").manual_seed(3)
    victims = torch.randperm(n, device="cuda", generator=gen)[: n // 100]
    span = span_lens[victims].to(torch.int64)
    pos = offs[victims] + 32 + (torch.rand(victims.numel(), device="cuda", generator=gen) * span).to(torch.int64)
    bit = torch.randint(0, 8, (victims.numel(),), device="cuda", generator=gen).to(torch.uint8)
    flat[pos] ^= (torch.ones_like(bit) << bit)
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    _KEEP.extend((data, offs))
    span_bytes = int((ntot_np - 32).sum())
    return (data.data_ptr(), data.numel(), wbuf, offs.data_ptr(), n, ok.data_ptr()), ok, victims, span_bytes, {
        "workload": f"{args.pages} x 64 MiB extstore pages of mixed items (values "
                    + ("2048 and 6150 B in turn" if args.workload == "mixed41" else "log-uniform 512 B - 64 KiB")
                    + f", mean item {int(ntot_np.mean())} B), packed per 4 MiB wbuf, stored CRC verified per item",
        "pages_per_gpu": args.pages, "items_per_gpu": n, "span_bytes_per_gpu": span_bytes,
        "items_le_4k_frac": round(float((ntot_np <= 4096).mean()), 3), "injected_bad": int(victims.numel())}


K1_LAYOUT = "pieces16-nt"  # K1's load shape since round 5 (crc32c_kernels.hip k_fixed)


def traffic_per_launch(items=ITEMS_PER_GPU, item_bytes=ITEM_BYTES):
    """HBM bytes per K1 launch from the committed rocprofv3 --pmc summaries:
    the newest profiles/*traffic*.json record of kernel k_fixed measured on
    this batch shape and K1 layout (files of other kernels, shapes or of the
    earlier K1 are skipped)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")), reverse=True):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        if (isinstance(rec, dict) and rec.get("kernel") == "k_fixed" and rec.get("k1_layout") == K1_LAYOUT
                and rec.get("items") == items
                and rec.get("item_bytes") == item_bytes and rec.get("hbm_bytes_per_launch")):
            return rec["hbm_bytes_per_launch"]
    return None


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 50 timed launches after 20 untimed ones -- the core clock takes
    # ~20 launches to settle (profiles/r01_ablations/k1_clock_ramp_800_launches.log)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=250.0,
                    help="before the warmup steps, repeat the step for this long (wall ms) so the GPU clock "
                         "leaves its idle ramp; not counted as warmup or timed steps (0 = off)")
    ap.add_argument("--items", type=int, default=ITEMS_PER_GPU, help="items per GPU (default: config 2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--events", default="region", choices=["region", "launch"],
                    help="HIP events around the timed launches (region) or around each launch")
    ap.add_argument("--fill", default="splitmix", choices=["splitmix", "randint"],
                    help="item bytes: splitmix64(42 + rank) words (SURVEY.md 8d) or torch.randint")
    ap.add_argument("--workload", default="config2",
                    choices=["config2", "config2r", "config3", "config5", "pagesmix", "mixed41", "pages", "pagesmixwalk",
                             "stamp", "host", "calls", "multi"],
                    help="config2 = headline; others are extra measurements (not the bench line)")
    ap.add_argument("--pages", type=int, default=1000, help="config5: 64 MiB pages per GPU")
    ap.add_argument("--span-len", type=int, default=4133, help="config2r: span length (stride = len + 32)")
    args = ap.parse_args(argv)
    if args.workload != "config2":
        return extra_workload(args)
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        # no launcher: one process drives the N devices itself
        return headline_devices(args)

    rank, world, local = dist_setup(args.gpus)
    if _lib.lib.crc32c_gpu_count() < 1:
        raise SystemExit("libmcrc32c.so sees no gfx950 device")
    n = args.items
    data, out, spans = make_batch(n, seed=42 + rank, fill=args.fill)
    stream = torch.cuda.current_stream()

    # clock settle, then the W warmup steps (the first launch also initialises
    # the library's device state and tables)
    settled = settle(lambda k: run_steps(spans, k, stream), args.settle_ms)
    for a, b in run_steps(spans, max(1, args.warmup), stream):
        pass
    torch.cuda.synchronize()

    per_launch = args.events == "launch"
    elapsed, evs = timed(lambda k: run_steps(spans, k, stream, per_launch), args.steps, world)

    kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    kernel_ms = max_over_ranks(kernel_ms, world)
    value = n * ITEM_BYTES * args.steps * world / elapsed / 2**30

    result = headline_result(args, value, elapsed, kernel_ms, world, settled,
                             f"items sharded across {world} rank(s), no collective on the data path")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the CPU leg runs at N = 1 only
        result["cpu_baseline"] = cpu_baseline(data, out)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def headline_result(args, value, elapsed, kernel_ms, n_gpus, settled, parallelism):
    """The bench line's fields (kernel_ms: the slowest device's average K1
    launch, HIP events on its launch stream)."""
    achieved = args.items * ITEM_BYTES / (kernel_ms * 1e-3) / 1e9
    return {
        "metric": "CRC32C GiB/s over device-resident item batches; % of HBM roofline",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle": {"ms": args.settle_ms, "launches": settled},
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic ({args.fill} bytes, seed 42 + rank), device-resident",
        "config": {
            "workload": "BASELINE configs[1]: 1 Mi items x 4096 B per GPU, stride 4096, one 32-lane group per "
                        "item (K1 k_fixed<slice-by-4, 32 lanes, 8 x 16-B pieces per lane at 512-B spacing, "
                        "non-temporal coalesced loads, half-item folds in the last-step tables, four items reduced per tree>)",
            "items_per_gpu": args.items,
            "item_bytes": ITEM_BYTES,
            "parallelism": parallelism,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic_per_launch(),
            "kernel_ms": round(kernel_ms, 4),
        },
    }


def headline_devices(args):
    """The headline on --gpus N devices from ONE process (bench.py started
    without a launcher, WORLD_SIZE unset): device g holds its own 1 Mi x 4 KiB
    shard (seed 42 + g, as rank g would) and K1 runs on every device, each on
    its own stream, the K launches of all devices enqueued before any is
    waited for.  The timed region is bracketed by a synchronize of every
    device; value = all devices' bytes / that wall time, kernel_ms = the
    slowest device's average launch.  No data-path collective, as with ranks."""
    ng = args.gpus
    vis = torch.cuda.device_count()  # (does not initialise the GPU)
    if vis < ng:
        raise SystemExit(f"bench.py: --gpus {ng} but only {vis} visible device(s); run with --gpus <= {vis}")
    if _lib.lib.crc32c_gpu_count() < ng:
        raise SystemExit(f"bench.py: --gpus {ng} but libmcrc32c.so sees {_lib.lib.crc32c_gpu_count()} gfx950 device(s)")
    devs = []
    for g in range(ng):
        torch.cuda.set_device(g)
        data, out, spans = make_batch(args.items, seed=42 + g, fill=args.fill, device=f"cuda:{g}")
        devs.append((g, data, out, spans, torch.cuda.Stream(device=g)))

    def launch(k, evs=None):
        flags = _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC
        for i in range(k):
            for g, data, out, sp, st in devs:
                torch.cuda.set_device(g)  # the library launches on the current device
                if evs is not None and i == 0:
                    evs[g][0].record(st)
                _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), flags, ctypes.c_void_p(st.cuda_stream)))
                if evs is not None and i == k - 1:
                    evs[g][1].record(st)

    def sync_all():
        for g, *_ in devs:
            torch.cuda.synchronize(g)

    settled = settle(lambda k: (launch(k), sync_all()), args.settle_ms)
    launch(max(1, args.warmup))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(ng)]
    sync_all()
    t0 = time.perf_counter()
    launch(args.steps, evs)
    sync_all()
    elapsed = time.perf_counter() - t0
    kms = [evs[g][0].elapsed_time(evs[g][1]) / args.steps for g in range(ng)]
    value = ng * args.items * ITEM_BYTES * args.steps / elapsed / 2**30
    result = headline_result(args, value, elapsed, max(kms), ng, settled,
                             f"items sharded across {ng} devices driven by one process (no launcher), one stream "
                             "each, no collective on the data path")
    result["kernel_ms_per_device"] = [round(x, 4) for x in kms]
    print(json.dumps(result), flush=True)
    return result


def workload_multi(args):
    """BASELINE configs[3] in one process: 1 Mi x 4 KiB items per GPU on the
    first --gpus devices (no collective; a shard per device).

    device: each device's shard resident in its HBM, K1 launched on every
            device (one stream each), all enqueued before any is waited for;
            value = all devices' bytes / wall time of the K steps.
    host:   the same bytes in one pinned host buffer, split by
            crc32c_batch_multi (crc32c_shard_cuts, one host thread per device,
            pinned H2D / kernel / D2H overlapped in two pipeline slots):
            the PCIe-inclusive rate.
    Both modes' CRCs must agree item for item."""
    import numpy as np
    ng = args.gpus
    if torch.cuda.device_count() < ng:
        raise SystemExit(f"--gpus {ng} but {torch.cuda.device_count()} visible devices")
    n = args.items
    flags = _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC
    dev = []
    for g in range(ng):
        torch.cuda.set_device(g)
        data = splitmix64_bytes(n * ITEM_BYTES, 42 + g, device=f"cuda:{g}")
        out = torch.empty(n, dtype=torch.int32, device=f"cuda:{g}")
        sp = _lib.Spans(data.data_ptr(), data.numel(), None, ITEM_BYTES, None, ITEM_BYTES, None, out.data_ptr(), n)
        dev.append((g, data, out, sp, torch.cuda.Stream(device=g)))

    def launch(k, evs=None):
        for i in range(k):
            for g, data, out, sp, st in dev:
                torch.cuda.set_device(g)
                if evs is not None and i == 0:
                    evs[g][0].record(st)
                _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), flags, ctypes.c_void_p(st.cuda_stream)))
                if evs is not None and i == k - 1:
                    evs[g][1].record(st)

    def sync_all():
        for g, *_ in dev:
            torch.cuda.synchronize(g)

    settled = settle(lambda k: (launch(k), sync_all()), args.settle_ms)
    launch(max(1, args.warmup))
    sync_all()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(ng)]
    t0 = time.perf_counter()
    launch(args.steps, evs)
    sync_all()
    el = time.perf_counter() - t0
    kms = [evs[g][0].elapsed_time(evs[g][1]) / args.steps for g in range(ng)]
    nbytes = ng * n * ITEM_BYTES
    res = {"device": {"gib_s": round(nbytes * args.steps / el / 2**30, 2), "ms_per_step": round(el / args.steps * 1e3, 4),
                      "kernel_ms_per_device": [round(x, 4) for x in kms],
                      "hbm_frac_per_device": [round(n * ITEM_BYTES / (x * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) for x in kms],
                      "settle_launches": settled}}
    # host-resident: the same bytes in one pinned buffer
    host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    for g, data, *_ in dev:
        host[g * n * ITEM_BYTES:(g + 1) * n * ITEM_BYTES].copy_(data)
    hout = np.empty(ng * n, np.uint32)
    hs = _lib.Spans(host.data_ptr(), nbytes, None, ITEM_BYTES, None, ITEM_BYTES, None, hout.ctypes.data, ng * n)
    _lib.check(_lib.lib.crc32c_batch_multi(ctypes.byref(hs), ng))  # warm-up (pipeline buffers)
    hsteps = max(1, min(args.steps, 5))
    t0 = time.perf_counter()
    for _ in range(hsteps):
        _lib.check(_lib.lib.crc32c_batch_multi(ctypes.byref(hs), ng))
    el = time.perf_counter() - t0
    res["host"] = {"gib_s": round(nbytes * hsteps / el / 2**30, 2), "gb_s": round(nbytes * hsteps / el / 1e9, 2),
                   "ms_per_step": round(el / hsteps * 1e3, 2), "steps": hsteps}
    want = np.concatenate([out.cpu().numpy().view(np.uint32) for _, _, out, _, _ in dev])
    res["crc_match"] = bool((want == hout).all())
    cuts = np.empty(ng + 1, np.uint64)
    _lib.check(_lib.lib.crc32c_shard_cuts(None, ITEM_BYTES, ng * n, ng, cuts.ctypes.data))
    res["config"] = {"workload": f"BASELINE configs[3] shape: {n} x {ITEM_BYTES} B items per GPU on {ng} GPU(s), "
                                 "one process; device-resident K1 on every device, and the same bytes in pinned host "
                                 "memory through crc32c_batch_multi (PCIe-inclusive)",
                     "items_per_gpu": n, "shard_cuts": [int(c) for c in cuts]}
    return res


def extra_workload(args):
    """Non-headline measurements; prints one JSON line per run."""
    if args.workload == "multi":  # one process drives every device (no torchrun)
        res = {"workload_kind": "multi", "n_gpus": args.gpus, "steps": args.steps}
        res.update(workload_multi(args))
        print(json.dumps(res), flush=True)
        return
    rank, world, local = dist_setup(args.gpus)
    stream = torch.cuda.current_stream()
    res = {"workload_kind": args.workload, "n_gpus": world, "steps": args.steps}
    if args.workload == "config3":
        if args.items == ITEMS_PER_GPU:
            args.items = 1 << 20
        spans, nbytes, cfg = workload_config3(args, rank, world)
        res["settle_launches"] = settle(lambda k: run_steps(spans, k, stream), args.settle_ms)
        run_steps(spans, max(1, args.warmup), stream)
        torch.cuda.synchronize()
        elapsed, evs = timed(lambda k: run_steps(spans, k, stream), args.steps, world)
        kms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
        res.update(config=cfg, kernel_ms=round(kms, 4), gib_s=round(nbytes * args.steps * world / elapsed / 2**30, 2),
                   hbm_frac=round(nbytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
    elif args.workload in ("config5", "pagesmix", "mixed41"):
        vargs, ok, victims, nbytes, cfg = (workload_config5 if args.workload == "config5" else
                                           workload_pagesmix)(args, rank, world)
        res["settle_launches"] = settle(lambda k: run_verify_steps(vargs, k, stream), args.settle_ms)
        run_verify_steps(vargs, max(1, args.warmup), stream)
        torch.cuda.synchronize()
        elapsed, (evs, nbad) = timed(lambda k: run_verify_steps(vargs, k, stream), args.steps, world)
        kms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
        bad_idx = torch.nonzero(ok == 0).flatten()
        exact = bool(nbad == victims.numel() and torch.equal(torch.sort(bad_idx)[0], torch.sort(victims)[0]))
        res.update(config=cfg, kernel_ms=round(kms, 4), gib_s=round(nbytes * args.steps * world / elapsed / 2**30, 2),
                   hbm_frac=round(nbytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), nbad=nbad,
                   detected_exactly_the_injected_items=exact)
    elif args.workload == "config2r":
        # SURVEY.md 8(d) config 2 variant: realistic 4133-B spans at stride 4165, start +32 (unaligned)
        n, sl = args.items, args.span_len
        g = torch.Generator(device="cuda").manual_seed(42 + rank)
        data = torch.randint(0, 256, (n * (sl + 32) + 64,), dtype=torch.uint8, device="cuda", generator=g)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        spans = _lib.Spans(data.data_ptr() + 32, data.numel() - 32, None, sl + 32, None, sl, None, out.data_ptr(), n)
        res["settle_launches"] = settle(lambda k: run_steps(spans, k, stream), args.settle_ms)
        run_steps(spans, max(1, args.warmup), stream)
        torch.cuda.synchronize()
        elapsed, evs = timed(lambda k: run_steps(spans, k, stream), args.steps, world)
        kms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
        nbytes = n * sl
        res.update(config={"workload": f"config 2 variant: {n} x {sl}-B spans at stride {sl + 32}, start +32 "
                                       "(K5 k_lines: 31-32 whole 128-B lines per span in one 4 KiB window, head and tail by the span's run lane)"},
                   kernel_ms=round(kms, 4), gib_s=round(nbytes * args.steps * world / elapsed / 2**30, 2),
                   hbm_frac=round(nbytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
    elif args.workload in ("pages", "pagesmixwalk", "stamp"):
        # pagesmixwalk: the mixed pages (workload_pagesmix) walked and verified on the device
        walk = args.workload != "stamp"
        vargs, ok, victims, nbytes, cfg = (workload_pagesmix if args.workload == "pagesmixwalk" else
                                           workload_config5)(args, rank, world)
        base, size, region, offs, n, okp = vargs
        nitems, nbad = ctypes.c_uint64(0), ctypes.c_uint64(0)
        sptr = ctypes.c_void_p(stream.cuda_stream)
        # walk outputs: at most one item more per wbuf than were written
        cap = n + size // region + 1
        woffs = torch.empty(cap, dtype=torch.int64, device="cuda")
        wok = torch.empty(cap, dtype=torch.uint8, device="cuda")

        def one():
            if walk:  # device walk + verify (storage.c:950-1070)
                _lib.check(_lib.lib.crc32c_verify_pages(base, size, region, woffs.data_ptr(), wok.data_ptr(), cap,
                                                        ctypes.byref(nitems), ctypes.byref(nbad),
                                                        _lib.CRC32C_DEVICE, sptr))
            else:  # spill CRCs stamped into every image (storage.c:567 per wbuf)
                _lib.check(_lib.lib.crc32c_stamp_items(base, size, region, offs, n, None, ctypes.byref(nbad),
                                                       _lib.CRC32C_DEVICE, sptr))

        def steps(k):
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
            for a, b in evs:
                a.record(stream)
                one()
                b.record(stream)
            return evs

        res["settle_launches"] = settle(steps, args.settle_ms)
        steps(max(1, args.warmup))
        torch.cuda.synchronize()
        elapsed, evs = timed(steps, args.steps, world)
        kms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
        cfg["workload"] += (" -- walked on the device (crc32c_verify_pages)" if walk
                            else " -- stamped (crc32c_stamp_items)")
        res.update(config=cfg, kernel_ms=round(kms, 4), gib_s=round(nbytes * args.steps * world / elapsed / 2**30, 2),
                   hbm_frac=round(nbytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), nbad=int(nbad.value),
                   nitems=int(nitems.value) if walk else n, items_written=n)
    elif args.workload == "calls":
        # Per-call latency of the integration's call shapes (INTEGRATION.md
        # 2-4): wall clock of synchronous calls, launch and sync included.
        import time

        import numpy as np
        args.pages = 1
        vargs, ok, victims, nbytes, cfg = workload_config5(args, rank, world)
        base, size, region, offs, n, okp = vargs
        nbad = ctypes.c_uint64(0)
        per_wbuf = 1007
        torch.cuda.synchronize()

        def per_call(fn, reps):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps * 1e6

        sptr = ctypes.c_void_p(stream.cuda_stream)
        stamp_us = per_call(lambda: _lib.check(_lib.lib.crc32c_stamp_items(
            base, region, region, offs, per_wbuf, None, ctypes.byref(nbad), _lib.CRC32C_DEVICE, sptr)), 200)
        verify64_us = per_call(lambda: _lib.check(_lib.lib.crc32c_verify_items(
            base, region, region, offs, 64, okp, ctypes.byref(nbad), _lib.CRC32C_DEVICE, sptr)), 200)
        host = np.frombuffer(bytearray(64 * 4165 + 64), dtype=np.uint8)
        hoffs = (np.arange(64, dtype=np.uint64) * 4165 + 32).astype(np.uint64)
        hout = np.empty(64, np.uint32)
        hs = _lib.Spans(host.ctypes.data, host.size, hoffs.ctypes.data, 0, None, 4133, None, hout.ctypes.data, 64)
        host64_us = per_call(lambda: _lib.check(_lib.lib.crc32c_batch(ctypes.byref(hs), 0, None)), 200)
        # 64 device spans by offsets (the read-back IO batch as raw spans)
        doffs64 = (torch.arange(64, device="cuda", dtype=torch.int64) * 4165 + 32).contiguous()
        dout64 = torch.empty(64, dtype=torch.int32, device="cuda")
        ds = _lib.Spans(base, region, doffs64.data_ptr(), 0, None, 4133, None, dout64.data_ptr(), 64)
        dev64_us = per_call(lambda: _lib.check(_lib.lib.crc32c_batch(ctypes.byref(ds), _lib.CRC32C_DEVICE, sptr)), 200)
        # host-resident item calls: one wbuf in page-locked
        # memory (crc32c_host_alloc / pin_memory) and in pageable memory
        wb_dev = _KEEP[-2][:region]  # (the config-5 page tensor; its first wbuf)
        wb_pin = wb_dev.cpu().pin_memory()
        wb_page = wb_dev.cpu().numpy().copy()
        hoffs_w = (np.arange(per_wbuf, dtype=np.uint64) * 4165).astype(np.uint64)
        hok = np.empty(per_wbuf, np.uint8)
        stamp_pin_us = per_call(lambda: _lib.check(_lib.lib.crc32c_stamp_items(
            wb_pin.data_ptr(), region, region, hoffs_w.ctypes.data, per_wbuf, None, ctypes.byref(nbad), 0, None)), 100)
        stamp_page_us = per_call(lambda: _lib.check(_lib.lib.crc32c_stamp_items(
            wb_page.ctypes.data, region, region, hoffs_w.ctypes.data, per_wbuf, None, ctypes.byref(nbad), 0, None)), 50)
        verify64_pin_us = per_call(lambda: _lib.check(_lib.lib.crc32c_verify_items(
            wb_pin.data_ptr(), region, region, hoffs_w.ctypes.data, 64, hok.ctypes.data, ctypes.byref(nbad), 0,
            None)), 200)
        # the compaction readback's shape (storage.c:950-1070, INTEGRATION.md
        # 3): one wbuf walked and verified, device-resident and page-locked
        nitems_w = ctypes.c_uint64(0)
        wcap = per_wbuf + 1
        d_woffs = torch.empty(wcap, dtype=torch.int64, device="cuda")
        d_wok = torch.empty(wcap, dtype=torch.uint8, device="cuda")
        h_woffs, h_wok = np.empty(wcap, np.uint64), np.empty(wcap, np.uint8)
        pages_wbuf_us = per_call(lambda: _lib.check(_lib.lib.crc32c_verify_pages(
            base, region, region, d_woffs.data_ptr(), d_wok.data_ptr(), wcap, ctypes.byref(nitems_w),
            ctypes.byref(nbad), _lib.CRC32C_DEVICE, sptr)), 200)
        pages_wbuf_pin_us = per_call(lambda: _lib.check(_lib.lib.crc32c_verify_pages(
            wb_pin.data_ptr(), region, region, h_woffs.ctypes.data, h_wok.ctypes.data, wcap, ctypes.byref(nitems_w),
            ctypes.byref(nbad), 0, None)), 100)
        pin64 = torch.from_numpy(host).pin_memory()
        hs_pin = _lib.Spans(pin64.data_ptr(), host.size, hoffs.ctypes.data, 0, None, 4133, None, hout.ctypes.data, 64)
        host64_pin_us = per_call(lambda: _lib.check(_lib.lib.crc32c_batch(ctypes.byref(hs_pin), 0, None)), 200)
        # host cost of enqueueing one asynchronous device batch (K1, 16 Ki x
        # 4 KiB of the page buffer), one thread, then 8 threads at once on
        # their own streams (the per-call device lookup takes no process-wide
        # lock: DESIGN.md section 6); ctypes releases the GIL during the call
        import threading
        n1 = 16384
        k1out = torch.empty(n1 * 8, dtype=torch.int32, device="cuda")

        def enqueue_loop(t, reps, st, times):
            sp1 = _lib.Spans(base, n1 * 4096, None, 4096, None, 4096, None, k1out.data_ptr() + 4 * n1 * t, n1)
            sp_ptr = ctypes.c_void_p(st.cuda_stream)
            flags = _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC
            t0 = time.perf_counter()
            for _ in range(reps):
                _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp1), flags, sp_ptr))
            times[t] = (time.perf_counter() - t0) / reps * 1e6

        streams = [torch.cuda.Stream() for _ in range(8)]
        enq = {}
        for nth in (1, 8):
            times = [0.0] * nth
            enqueue_loop(0, 10, streams[0], [0.0])  # (warm)
            torch.cuda.synchronize()
            ths = [threading.Thread(target=enqueue_loop, args=(t, 100, streams[t], times)) for t in range(nth)]
            w0 = time.perf_counter()
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            wall = time.perf_counter() - w0
            torch.cuda.synchronize()
            enq[nth] = (max(times), wall / (100 * nth) * 1e6)
        res.update(enqueue_async_us_1thread=round(enq[1][0], 2), enqueue_async_us_8threads=round(enq[8][0], 2),
                   enqueue_async_8threads_wall_us_per_call=round(enq[8][1], 2))
        res.update(config={"workload": "per-call latency, synchronous calls, one thread: stamp one 4 MiB wbuf of "
                                       "1007 images (device; host page-locked; host pageable), verify an IO batch "
                                       "of 64 images (device; host page-locked), CRC 64 x 4133-B spans in host "
                                       "memory (pageable: staged; page-locked: the coalescing queue) and in device "
                                       "memory, walk + verify one wbuf (device; host page-locked)"},
                   stamp_wbuf_us=round(stamp_us, 1), verify64_us=round(verify64_us, 1),
                   stamp_wbuf_host_pinned_us=round(stamp_pin_us, 1), stamp_wbuf_host_pageable_us=round(stamp_page_us, 1),
                   verify64_host_pinned_us=round(verify64_pin_us, 1),
                   host_batch64_us=round(host64_us, 1), host_batch64_pinned_us=round(host64_pin_us, 1),
                   device_batch64_us=round(dev64_us, 1),
                   pages_wbuf_us=round(pages_wbuf_us, 1), pages_wbuf_host_pinned_us=round(pages_wbuf_pin_us, 1),
                   stamp_wbuf_gb_s=round(per_wbuf * 4133 / (stamp_us * 1e-6) / 1e9, 1),
                   stamp_wbuf_host_pinned_gb_s=round(per_wbuf * 4133 / (stamp_pin_us * 1e-6) / 1e9, 1))
    else:  # host: pinned host memory -> H2D -> K1/K2 -> D2H through the library's host path
        import numpy as np
        n = args.items
        host = torch.empty(n * ITEM_BYTES, dtype=torch.uint8).pin_memory()
        g = torch.Generator().manual_seed(11)
        host.copy_(torch.randint(0, 256, (n * ITEM_BYTES,), dtype=torch.uint8, generator=g))
        out = np.empty(n, np.uint32)
        sp = _lib.Spans(host.data_ptr(), host.numel(), None, ITEM_BYTES, None, ITEM_BYTES, None,
                        out.ctypes.data, n)
        _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), 0, None))

        def steps(k):
            for _ in range(k):
                _lib.check(_lib.lib.crc32c_batch(ctypes.byref(sp), 0, None))

        elapsed, _ = timed(steps, args.steps, world, sync=lambda: None)
        res.update(config={"workload": f"{n} x {ITEM_BYTES} B items in pinned host memory; H2D over PCIe, "
                                       "K2 kernel, CRCs D2H (library host path, two pipeline slots)"},
                   gib_s=round(n * ITEM_BYTES * args.steps * world / elapsed / 2**30, 2),
                   gb_s=round(n * ITEM_BYTES * args.steps * world / elapsed / 1e9, 2))
    if rank == 0:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
