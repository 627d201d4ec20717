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


def make_batch(n: int, seed: int):
    g = torch.Generator(device="cuda").manual_seed(seed)
    data = torch.randint(0, 256, (n * ITEM_BYTES,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    spans = _lib.Spans(data.data_ptr(), data.numel(), None, ITEM_BYTES, None, ITEM_BYTES, None,
                       out.data_ptr(), n)
    return data, out, spans


def run_steps(spans, steps: int, stream):
    """Enqueue `steps` launches back to back on `stream`, one event pair each."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    flags = _lib.CRC32C_DEVICE | _lib.CRC32C_ASYNC
    for a, b in evs:
        a.record(stream)
        _lib.check(_lib.lib.crc32c_batch(ctypes.byref(spans), flags, ctypes.c_void_p(stream.cuda_stream)))
        b.record(stream)
    return evs


def cpu_baseline(data: torch.Tensor, out: torch.Tensor):
    """Reference crc32c.c on host cores over a bounded sample of the batch."""
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")
    if not os.path.exists(ref):
        return {"value": None, "unit": "GiB/s", "cores": 0, "kind": "reference",
                "sample": "oracle/_ref/libref_crc32c.so missing (build in the container with /root/reference)"}
    lib = ctypes.CDLL(ref)
    lib.ref_crc32c_init()
    lib.ref_crc32c_batch_timed.restype = ctypes.c_double
    lib.ref_crc32c_batch_timed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    n = 1 << 16  # 256 MiB sample: the first 65536 items of rank 0's batch
    host = data[: n * ITEM_BYTES].cpu().numpy()
    import numpy as np
    crc = np.empty(n, np.uint32)
    cores = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))

    def rate(threads, passes):
        best = 0.0
        lib.ref_crc32c_batch_timed(host.ctypes.data, None, None, ITEM_BYTES, ITEM_BYTES, n, threads, crc.ctypes.data)
        for _ in range(passes):
            t = lib.ref_crc32c_batch_timed(host.ctypes.data, None, None, ITEM_BYTES, ITEM_BYTES, n, threads,
                                           crc.ctypes.data)
            best = max(best, n * ITEM_BYTES / t / 2**30)
        return best

    one = rate(1, 5)
    many = rate(cores, 20)
    gpu = out[:n].cpu().numpy().view(np.uint32)
    return {"value": round(many, 2), "unit": "GiB/s", "cores": cores, "kind": "reference",
            "sample": f"first 65536 x 4096 B items of the GPU batch (256 MiB), reference crc32c.c "
                      f"(hw dispatch) per item as storage.c:567, {cores} threads static split, best of 20; "
                      f"1 core: {one:.2f} GiB/s",
            "gpu_match": bool((gpu == crc).all())}


def traffic_per_launch():
    """HBM bytes per K1 launch from the committed rocprofv3 --pmc summary, if any."""
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")))
    if not paths:
        return None
    try:
        rec = json.load(open(paths[-1]))
        if rec.get("items") == ITEMS_PER_GPU and rec.get("item_bytes") == ITEM_BYTES:
            return rec.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--items", type=int, default=ITEMS_PER_GPU, help="items per GPU (default: config 2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank, world, local = dist_setup(args.gpus)
    if _lib.lib.crc32c_gpu_count() < 1:
        raise SystemExit("libmcrc32c.so sees no gfx950 device")
    n = args.items
    data, out, spans = make_batch(n, seed=42 + rank)
    stream = torch.cuda.current_stream()

    # warmup (also initialises the library's device state and tables)
    for a, b in run_steps(spans, max(1, args.warmup), stream):
        pass
    torch.cuda.synchronize()

    elapsed, evs = timed(lambda k: run_steps(spans, k, stream), args.steps, world)

    kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    kernel_ms = max_over_ranks(kernel_ms, world)
    bytes_per_launch = n * ITEM_BYTES
    total_bytes = bytes_per_launch * args.steps * world
    value = total_bytes / elapsed / 2**30
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9

    result = {
        "metric": "CRC32C GiB/s over device-resident item batches; % of HBM roofline",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (torch.randint bytes, seed 42 + rank), device-resident",
        "config": {
            "workload": "BASELINE configs[1]: 1 Mi items x 4096 B per GPU, stride 4096, one 32-lane group per "
                        "item (K1 k_fixed<slice-by-4, 32 lanes, 32 B/lane/row, 4 rows, bitop3 + DPP merge>)",
            "items_per_gpu": n,
            "item_bytes": ITEM_BYTES,
            "parallelism": f"items sharded across {world} rank(s), no collective on the data path",
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
    if rank == 0 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(data, out)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
