#!/usr/bin/env python3
"""ricepp encode+decode benchmark on MI355X.

Workloads (BASELINE.json):
  blocks (default, configs[1]): 4096 independent 64 KiB uint16 blocks per GPU
      (weak scaling: every rank holds its own 4096 blocks);
  mix (configs[3]): one fixed mkdwarfs-style mix of 1 / 4 / 16 MiB blocks,
      32 GiB in all, sharded by block across the ranks with
      parallel.partition_blocks (strong scaling: the total is fixed).
One step = encode every block of the shard on the GPU, all-gather the
per-block encoded sizes over RCCL (N > 1) and scan them into image offsets,
decode every block back.  Inputs are resident in HBM before the timed region;
`value` is uncompressed bytes of all ranks per second (GiB/s), the accounting
of ricepp/ricepp_benchmark.cpp:145-146,155-156 applied to the round trip.

Launch:  python bench.py [--gpus N --steps K --warmup W] [--workload mix]
         (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from dwarfs_amd import codec  # noqa: E402
from dwarfs_amd import parallel  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
WARMUP_FLOOR_S = 0.5  # minimum warm-up time, whatever --warmup says


def make_poisson_blocks(nblocks: int, n: int, lam: float, seed: int, device) -> torch.Tensor:
    """Poisson(lam) sensor samples, stored big endian, generated on the GPU."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty(nblocks * n, dtype=torch.int16, device=device)
    chunk = 1 << 24
    for s in range(0, nblocks * n, chunk):
        e = min(s + chunk, nblocks * n)
        v = torch.poisson(torch.full((e - s,), lam, device=device), generator=g).clamp_(0, 65535).to(torch.int32)
        v = ((v & 0xFF) << 8) | ((v >> 8) & 0xFF)
        out[s:e] = v.to(torch.int16)  # wraps to the same 16 bits
    return out


def mix_block_mib(total_gib: int = 32, seed: int = 2024) -> list:
    """configs[3]'s block list: mkdwarfs cuts each category into blocks of the block size (16 MiB at its
    default -S 24) with a short last block per category, so the mix is mostly 16 MiB blocks with 4 and
    1 MiB ones in between: 3/4 of the bytes in 16 MiB blocks, 3/16 in 4 MiB, 1/16 in 1 MiB, shuffled
    (seeded: every rank derives the same list)."""
    total_mib = total_gib * 1024
    n16, n4, n1 = total_mib * 3 // 4 // 16, total_mib * 3 // 16 // 4, total_mib // 16
    sizes = np.array([16] * n16 + [4] * n4 + [1] * n1, np.int64)
    np.random.default_rng(seed).shuffle(sizes)
    return sizes.tolist()


def make_mix_shard(block_mib: list, lo: int, hi: int, device) -> tuple:
    """This rank's blocks [lo, hi) of the mix, generated on the GPU: block i is Poisson(lambda_i) noise
    (lambda from {300, 1000, 3000} by block), stored big endian, from a generator seeded by the block index
    alone, so the data do not depend on the rank count."""
    n = [m << 19 for m in block_mib[lo:hi]]  # samples per block
    offs = np.zeros(len(n), np.int64)
    if n:
        offs[1:] = np.cumsum(n)[:-1]
    x = torch.empty(max(int(sum(n)), 8), dtype=torch.int16, device=device)
    g = torch.Generator(device=device)
    for j, i in enumerate(range(lo, hi)):
        g.manual_seed(7919 * i + 1)
        lam = (300.0, 1000.0, 3000.0)[i % 3]
        for s0 in range(0, n[j], 1 << 24):
            e0 = min(n[j], s0 + (1 << 24))
            v = torch.poisson(torch.full((e0 - s0,), lam, device=device), generator=g).clamp_(0, 65535).to(torch.int32)
            v = ((v & 0xFF) << 8) | ((v >> 8) & 0xFF)
            x[offs[j] + s0:offs[j] + e0] = v.to(torch.int16)
    return x, offs, np.asarray(n, np.int64)


def device_copy_gbps(dev, nbytes: int = 1 << 30, iters: int = 10) -> float:
    """Measured device-to-device copy rate (read + write bytes / s), the
    'achievable' HBM reference of SURVEY.md §8(d) beside the 8 TB/s spec peak.
    The copy is our own dwordx4 streaming kernel: the PCM transformer with the
    identity format (4-byte little-endian signed 32-bit, dwarfs_amd.pcm), which
    outruns torch's copy_ on this device."""
    from dwarfs_amd.pcm import PcmSampleEndianness as E, PcmSamplePadding as P, PcmSampleSignedness as S
    from dwarfs_amd.pcm import PcmSampleTransformer

    ident = PcmSampleTransformer(E.Little, S.Signed, P.Msb, 4, 32)
    a = torch.ones(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
    ident.unpack(b, a)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        ident.unpack(b, a)
    e1.record(s)
    torch.cuda.synchronize(dev)
    gbps = 2 * nbytes * iters / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    return gbps


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> int:
    """Host threads this job may use: the affinity mask, capped at the GPU box's CPU share (16 per GPU;
    os.cpu_count() there reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return int(os.environ.get("RICEPP_CPU_THREADS", min(16, n)))


def _cpu_roundtrip(O, oc, sample, offs, n, nblocks, cap, threads, min_seconds):
    reps, t0 = 0, time.perf_counter()
    while True:
        out, oo, sz, st = O.encode_batch(oc, sample, offs, [n] * nblocks, cap, nthreads=threads)
        dec, dst = O.decode_batch(oc, out, oo, sz, offs, [n] * nblocks, nblocks * n, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_seconds:
            break
    assert (st == 0).all() and (dst == 0).all() and np.array_equal(dec, sample)
    return reps * sample.nbytes / 2**30 / el, reps, el


def cpu_baseline(sample: np.ndarray, nblocks: int, n: int, cfg: codec.CodecConfig, min_seconds: float):
    """The CPU oracle (C restatement of ricepp, kind "port") on host cores: one thread and the job's whole
    CPU share, over independent blocks."""
    from oracle import oracle as O

    threads = cpu_share()
    oc = O.cfg(cfg.block_size, cfg.component_stream_count, cfg.byteorder == "big", cfg.unused_lsb_count)
    offs = (np.arange(nblocks, dtype=np.uint64) * n)
    cap = O.worst_case_bytes(oc, n)
    nb1 = max(1, nblocks // 8)  # one thread: a smaller sample, same blocks
    v1, r1, e1 = _cpu_roundtrip(O, oc, sample[: nb1 * n], offs[:nb1], n, nb1, cap, 1, min_seconds / 2)
    vn, rn, en = _cpu_roundtrip(O, oc, sample, offs, n, nblocks, cap, threads, min_seconds / 2)
    return {
        "value": round(vn, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "single_thread_value": round(v1, 4),
        "cpu_model": cpu_model(),
        "host_cpus": os.cpu_count(),
        "sample": f"{nblocks} x 64 KiB Poisson(1000) BE bs128 cs1 blocks (first {nblocks} of the GPU workload), "
                  f"encode+decode x{rn}, {en:.1f} s wall, {threads} threads over independent blocks; "
                  f"1 thread: {nb1} blocks x{r1}, {e1:.1f} s",
    }


def kernel_source_sha256() -> str:
    """Identity of the kernels a committed PMC profile was taken of: the HIP sources of the ricepp path
    this bench runs (every .hip but the FLAC codec's, which no bench workload launches)."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted((ROOT / "dwarfs_amd" / "csrc").glob("*.hip")):
        if f.name == "flac_kernels.hip":
            continue
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()


def profiled_counters(kernel: str, profile: str = "pmc_latest.json"):
    """PMC figures of `kernel` per launch from profiles/pmc_latest.json (rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes with the gfx950 corrections of MI355X_MICROARCH.md, GRBM_GUI_ACTIVE), only if they were taken
    of the current kernel sources: (dict or None, provenance).  (profiles/pmc_mix.json: the mix's
    "encode" / "decode" calls, every kernel of a call summed: tools/pmc_mix_summary.py.)"""
    pmc = ROOT / "profiles" / profile
    if not pmc.exists():
        return None, "no PMC profile"
    try:
        j = json.loads(pmc.read_text())
    except ValueError:
        return None, "unreadable PMC profile"
    if j.get("kernel_source_sha256") != kernel_source_sha256():
        return None, "PMC profile of other kernel sources (stale); not reported"
    return j.get(kernel), f"{j.get('source', 'profiles')} (rocprofv3 PMC, kernel sources sha256 " \
                         f"{j['kernel_source_sha256'][:12]} of every dwarfs_amd/csrc/*.hip but flac_kernels.hip, " \
                         f"which no bench workload launches)"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=4096)
    ap.add_argument("--block-bytes", type=int, default=65536)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step as a captured HIP graph (measured no faster than eager launches: "
                         "profiles/r03_graph_ab.jsonl)")
    ap.add_argument("--workload", choices=("blocks", "mix"), default="blocks",
                    help="blocks: configs[1] (default, weak scaling); mix: configs[3] (strong scaling)")
    ap.add_argument("--mix-gib", type=int, default=32, help="total size of the configs[3] mix")
    ap.add_argument("--decode-path", choices=("auto", "fused", "segmented"), default="auto",
                    help="force a decode path (A/B measurements; the default is the library's own choice)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = codec.CodecConfig(block_size=128, component_stream_count=1, byteorder="big", unused_lsb_count=0)
    group = dist.group.WORLD if world > 1 else None
    dopt = codec.DecodeOptions(path=args.decode_path)
    if args.workload == "mix":
        mix = mix_block_mib(args.mix_gib)
        lo, hi = parallel.partition_blocks([m << 20 for m in mix], world)[rank]
        x, in_offsets, ns = make_mix_shard(mix, lo, hi, dev)
        nblocks, n = hi - lo, 0
        pipe = parallel.ShardPipeline(cfg, x, in_offsets, ns, group=group, decode_options=dopt)
        shard_bytes = int(ns.sum()) * 2
    else:
        nblocks, n = args.blocks, args.block_bytes // 2
        x = make_poisson_blocks(nblocks, n, 1000.0, 42 + rank, dev)
        in_offsets = np.arange(nblocks, dtype=np.int64) * n
        pipe = parallel.ShardPipeline(cfg, x, in_offsets, np.full(nblocks, n, np.int64), group=group,
                                      decode_options=dopt)
        shard_bytes = nblocks * n * 2

    # correctness gate before timing: round trip must be exact
    pipe.step()
    torch.cuda.synchronize()
    pipe.check(x)

    # warm-up: the requested steps, then more until the GPU has run for at
    # least WARMUP_FLOOR_S (its clocks settle only after a few ms of load: a
    # count of steps alone made the driver's short command read ~8 % low)
    tw = time.perf_counter()
    warm_steps = 0
    while warm_steps < args.warmup or time.perf_counter() - tw < WARMUP_FLOOR_S:
        pipe.step()
        warm_steps += 1
        if warm_steps % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - tw
    # the step's kernel chain as a HIP graph (one per rank; with several ranks
    # the size all-gather stays eager between two graphs): removes the host
    # launch path and part of the inter-kernel gaps; checked once more below
    graphed = args.graph and args.workload == "blocks"
    if graphed:
        try:
            pipe.capture()
        except RuntimeError as e:  # (a runtime that cannot capture: the eager step, said in the line)
            print(f"bench: graph capture failed, eager steps: {e}", file=sys.stderr)
            graphed = False
        for _ in range(max(1, args.warmup)):
            pipe.step()
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if graphed:
        pipe.check(x)  # (the replayed steps are exact too)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel timing with events on the launch stream (torch's current stream)
    k_enc, k_dec = pipe.kernel_times(iters=max(5, args.steps))
    comp_bytes = int(pipe.enc.sizes.sum().item())
    raw_bytes = shard_bytes
    enc_bytes = raw_bytes + comp_bytes + 8 * nblocks
    dec_bytes = comp_bytes + raw_bytes
    dominant = "decode" if k_dec >= k_enc else "encode"
    kt, kb = (k_dec, dec_bytes) if dominant == "decode" else (k_enc, enc_bytes)
    achieved = kb / kt / 1e9

    if args.workload == "mix":
        t = torch.tensor([raw_bytes, comp_bytes], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t)
        total_raw, total_comp = float(t[0].item()), float(t[1].item())
        value = total_raw * args.steps / elapsed / 2**30
        result = {
            "metric": "ricepp encode+decode GiB/s, device-resident uint16 blocks, 1/2/4/8 GPUs",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": warm_steps,
            "warmup_s": round(warm_s, 3),
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u16",
            "data": "synthetic Poisson(300/1000/3000) sensor samples per block, stored big endian, generated on device",
            "config": {
                "workload": f"mkdwarfs-style mix of 1/4/16 MiB uint16 blocks, {args.mix_gib} GiB in all, sharded by "
                            "block across the ranks (BASELINE.json configs[3]), ricepp bs128 cs1 BE ulsb0, "
                            "encode+decode round trip",
                "blocks_total": len(mix),
                "blocks_rank0": nblocks,
                "bytes_total": int(total_raw),
                "compression_ratio": round(total_comp / total_raw, 5),
                "parallelism": f"shard{world} (byte-balanced contiguous block ranges, RCCL all-gather of encoded sizes)",
                "rank0_encode_ms": round(k_enc * 1e3, 3),
                "rank0_decode_ms": round(k_dec * 1e3, 3),
                "rank0_encode_GiBps": round(raw_bytes / k_enc / 2**30, 2),
                "rank0_decode_GiBps": round(raw_bytes / k_dec / 2**30, 2),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "rpp_decode_batch_ws (segmented: unit parse + extraction + fused short streams)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "traffic_source": "not profiled for the mix",
            },
        }
        # (PMC of a 32 GiB mix: only at that size are the bytes per call this run's)
        mc, msrc = profiled_counters("decode", "pmc_mix.json") if args.mix_gib == 32 and world == 1 else \
            (None, "the PMC profile is of the 32 GiB mix on one GPU")
        if mc and "hbm_bytes_per_call" in mc:
            result["roofline"]["traffic"] = mc["hbm_bytes_per_call"]
            result["roofline"]["traffic_source"] = msrc + ": every kernel of one decode call"
            result["roofline"]["algorithmic_bytes"] = int(dec_bytes)
        else:
            result["roofline"]["traffic_source"] = msrc
        if rank == 0:
            print(json.dumps(result), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    counters, traffic_src = profiled_counters(f"rpp_{dominant}_kernel")
    traffic = counters.get("hbm_bytes_per_launch") if counters else None
    # the launch's length in GPU cycles (GRBM_GUI_ACTIVE per XCD): the kernel's work, whatever the clock
    kcycles = counters.get("cycles_per_launch") if counters else None

    total_bytes = raw_bytes * world * args.steps
    value = total_bytes / elapsed / 2**30
    result = {
        "metric": "ricepp encode+decode GiB/s, device-resident uint16 blocks, 1/2/4/8 GPUs",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_steps_run": warm_steps,
        "warmup_s": round(warm_s, 3),
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic Poisson(1000) sensor samples, stored big endian, generated on device",
        "config": {
            "workload": f"{nblocks} independent {args.block_bytes // 1024} KiB uint16 blocks per GPU, "
                        "ricepp bs128 cs1 BE ulsb0, encode+decode round trip (BASELINE.json configs[1])",
            "blocks_per_gpu": nblocks,
            "block_bytes": args.block_bytes,
            "compression_ratio": round(comp_bytes / raw_bytes, 5),
            "parallelism": f"shard{world} (blocks sharded, RCCL all-gather of encoded sizes)",
            "step_launch": ("HIP graph replay" + (" (encode | eager all-gather | scan + decode)" if world > 1 else "")
                            if graphed else "eager"),
            "encode_kernel_us": round(k_enc * 1e6, 2),
            "decode_kernel_us": round(k_dec * 1e6, 2),
            "encode_GiBps": round(raw_bytes / k_enc / 2**30, 2),
            "decode_GiBps": round(raw_bytes / k_dec / 2**30, 2),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": f"rpp_{dominant}_kernel",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel_cycles_per_launch": kcycles,
            "kernel_clock_GHz": round(kcycles / kt / 1e9, 3) if kcycles else None,
            "device_copy_GBps": round(device_copy_gbps(dev), 1),
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        nb = min(nblocks, 1024)
        sample = x[: nb * n].cpu().numpy().view(np.uint16).copy()
        result["cpu_baseline"] = cpu_baseline(sample, nb, n, cfg, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
