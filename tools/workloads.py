#!/usr/bin/env python3
"""Secondary BASELINE.json workloads on one MI355X (numbers for DESIGN.md;
the headline bench line is bench.py).  Each case prints one JSON line.

  gen      configs[0]'s generator (ricepp_benchmark.cpp:54-71: 6-bit noise +
           exponential-gated full-range outliers), 16 MiB: as one stream and
           as 4096 x 64 KiB blocks, encode + decode
  fits     configs[2]: decode-only, 256 frames of 4096 x 4096 Poisson(1000)
           samples (8 GiB), cut into 1 MiB DwarFS blocks (mkdwarfs -S 20),
           pre-encoded (by the GPU encoder, byte-identical to CPU ricepp per
           the parity tests)
  frames   configs[2] as whole frames: the same 256 frames, one 32 MiB
           stream each (the segmented decode splits them into units)
  mix      configs[3]: the per-GPU share of a 32 GiB 1/4/16 MiB block mix
           (4 GiB: equal bytes per size class), encode + decode
  sweep    configs[4]: bs {16, 32, 128} x component bits {10, 12, 14, 16}
           (ulsb 6/4/2/0), Poisson scaled to the bit depth, 4096 x 64 KiB
  e2e      the headline workload with host buffers: pinned H2D of samples,
           encode, D2H of the compressed image; and pinned H2D of the image,
           decode, D2H of the samples (PCIe included)

Usage: python tools/workloads.py [case ...]   (default: all)
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402

DEV = torch.device("cuda:0")
GIB = 2 ** 30


def gen_benchmark(n: int, seed: int) -> torch.Tensor:
    """ricepp_benchmark.cpp:54-71 generator shape, on the device: 6-bit
    noise, with probability P(Exp(0.1) <= 1) a full 16-bit value; stored BE."""
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    gate = torch.empty(n, device=DEV).exponential_(0.1, generator=g) <= 1.0
    noise = torch.randint(0, 64, (n,), device=DEV, generator=g, dtype=torch.int32)
    full = torch.randint(0, 65536, (n,), device=DEV, generator=g, dtype=torch.int32)
    v = torch.where(gate, full, noise)
    v = ((v & 0xFF) << 8) | ((v >> 8) & 0xFF)
    return v.to(torch.int16)


def poisson_scaled(n: int, lam: float, ulsb: int, seed: int) -> torch.Tensor:
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    out = torch.empty(n, dtype=torch.int16, device=DEV)
    chunk = 1 << 24
    for s in range(0, n, chunk):
        e = min(s + chunk, n)
        v = torch.poisson(torch.full((e - s,), lam, device=DEV), generator=g).clamp_(0, 0xFFFF >> ulsb)
        v = v.to(torch.int32) << ulsb
        v = ((v & 0xFF) << 8) | ((v >> 8) & 0xFF)
        out[s:e] = v.to(torch.int16)
    return out


def pipe_for(cfg, x, block_samples, dec=None):
    nb = len(block_samples)
    offs = np.zeros(nb, np.int64)
    offs[1:] = np.cumsum(block_samples)[:-1]
    p = parallel.ShardPipeline(cfg, x, offs, np.asarray(block_samples, np.int64), decode_options=dec)
    p.step()
    torch.cuda.synchronize()
    p.check(x)
    return p


def timed(fn, iters=5, warm_s=0.05):
    # warm-up of at least warm_s seconds of GPU work: the clocks reach their
    # steady state only after a few milliseconds (bench.py measures 662-677 GiB/s
    # after 3 warm-up steps and 736-740 after 20)
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    while time.perf_counter() - t0 < warm_s:
        fn()
        torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(iters):
        a.record(s)
        fn()
        b.record(s)
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / 1e3)
    return best


def report(case, **kw):
    print(json.dumps({"case": case, **kw}), flush=True)


def case_gen():
    cfg = codec.CodecConfig(128, 1, "big", 0)
    n = 8 * 1024 * 1024
    x = gen_benchmark(n, 42)
    for label, blocks in (("one 16 MiB stream", [n]), ("4096 x 64 KiB blocks", [32768] * 256),
                          ("16 x 1 MiB blocks", [n // 16] * 16)):
        if label.startswith("4096"):
            xx = gen_benchmark(4096 * 32768, 43)
            blocks = [32768] * 4096
        else:
            xx = x
        p = pipe_for(cfg, xx, blocks)
        raw = sum(blocks) * 2
        te, td = timed(p.encode), timed(p.decode)
        report("gen", layout=label, raw_MiB=raw / 2**20, ratio=round(int(p.sizes.sum()) / raw, 4),
               encode_GiBps=round(raw / te / GIB, 2), decode_GiBps=round(raw / td / GIB, 2),
               encode_us=round(te * 1e6, 1), decode_us=round(td * 1e6, 1))
        del p


def case_fits():
    cfg = codec.CodecConfig(128, 1, "big", 0)
    frames, fs = 256, 4096 * 4096
    blk = 1 << 19  # 1 MiB blocks
    n = frames * fs
    x = poisson_scaled(n, 1000.0, 0, 42)
    p = pipe_for(cfg, x, [blk] * (n // blk))
    comp = int(p.sizes.sum())
    raw = n * 2
    td = timed(p.decode, iters=3)
    report("fits", frames=frames, block="1 MiB", raw_GiB=raw / GIB, ratio=round(comp / raw, 4),
           decode_GiBps=round(raw / td / GIB, 2), decode_ms=round(td * 1e3, 2),
           hbm_GBps_algorithmic=round((raw + comp) / td / 1e9, 1),
           roofline_frac=round((raw + comp) / td / 1e9 / 8000.0, 4))


def case_frames():
    """configs[2] with one stream per frame: 256 whole 4096x4096 frames (32 MiB each), decode only
    (the segmented decode splits every frame into units)."""
    cfg = codec.CodecConfig(128, 1, "big", 0)
    frames, fs = 256, 4096 * 4096
    n = frames * fs
    x = poisson_scaled(n, 1000.0, 0, 42)
    p = pipe_for(cfg, x, [fs] * frames)
    comp = int(p.sizes.sum())
    raw = n * 2
    td = timed(p.decode, iters=3)
    report("frames", frames=frames, block="one 32 MiB stream per frame", raw_GiB=raw / GIB,
           ratio=round(comp / raw, 4), decode_GiBps=round(raw / td / GIB, 2), decode_ms=round(td * 1e3, 2),
           hbm_GBps_algorithmic=round((raw + comp) / td / 1e9, 1),
           roofline_frac=round((raw + comp) / td / 1e9 / 8000.0, 4))


def case_mix():
    cfg = codec.CodecConfig(128, 1, "big", 0)
    per_class = 1344 * 2**20 // 2  # samples per size class (4032 MiB per GPU in total)
    blocks = []
    for mib in (1, 4, 16):
        bs = mib * 2**20 // 2
        blocks += [bs] * (per_class // bs)
    rng = np.random.default_rng(5)
    rng.shuffle(blocks)
    n = int(sum(blocks))
    x = poisson_scaled(n, 1000.0, 0, 7)
    p = pipe_for(cfg, x, blocks)
    raw = n * 2
    te, td = timed(p.encode, 3), timed(p.decode, 3)
    report("mix", blocks=len(blocks), raw_GiB=round(raw / GIB, 3), ratio=round(int(p.sizes.sum()) / raw, 4),
           encode_GiBps=round(raw / te / GIB, 2), decode_GiBps=round(raw / td / GIB, 2),
           encode_ms=round(te * 1e3, 2), decode_ms=round(td * 1e3, 2),
           note="per-GPU share of 32 GiB over 8 GPUs; blocks are independent, so N GPUs run N such shares")


def case_sweep():
    for bs in (16, 32, 128):
        for bits in (10, 12, 14, 16):
            ulsb = 16 - bits
            lam = 1000.0 / (1 << (2 * ulsb))  # Poisson scaled to the bit depth
            cfg = codec.CodecConfig(bs, 1, "big", ulsb)
            x = poisson_scaled(4096 * 32768, max(lam, 4.0), ulsb, 11)
            p = pipe_for(cfg, x, [32768] * 4096)
            raw = 4096 * 32768 * 2
            te, td = timed(p.encode), timed(p.decode)
            report("sweep", bs=bs, bits=bits, ulsb=ulsb, ratio=round(int(p.sizes.sum()) / raw, 4),
                   encode_GiBps=round(raw / te / GIB, 2), decode_GiBps=round(raw / td / GIB, 2))
            del p


def case_paths():
    """configs[4] bs 16 / 32 decode by each path: the default (rows kernel), one wave per
    stream (fused) and the segmented decode at three unit sizes."""
    for bs in (16, 32):
        for bits in (10, 16):
            ulsb = 16 - bits
            lam = 1000.0 / (1 << (2 * ulsb))
            cfg = codec.CodecConfig(bs, 1, "big", ulsb)
            x = poisson_scaled(4096 * 32768, max(lam, 4.0), ulsb, 11)
            raw = 4096 * 32768 * 2
            res = {}
            for name, dec in (("auto", None), ("fused", codec.DecodeOptions(path="fused")),
                              ("seg12", codec.DecodeOptions(path="segmented", seg_log2=12)),
                              ("seg13", codec.DecodeOptions(path="segmented", seg_log2=13)),
                              ("seg14", codec.DecodeOptions(path="segmented", seg_log2=14))):
                p = pipe_for(cfg, x, [32768] * 4096, dec)
                res[name] = round(raw / timed(p.decode) / GIB, 2)
                del p
            report("paths", bs=bs, bits=bits, ulsb=ulsb, decode_GiBps=res)


def case_e2e():
    cfg = codec.CodecConfig(128, 1, "big", 0)
    nb, n = 4096, 32768
    x = make_poisson_blocks(nb, n, 1000.0, 42, DEV)
    p = pipe_for(cfg, x, [n] * nb)
    raw = nb * n * 2
    h_in = torch.empty(nb * n, dtype=torch.int16, pin_memory=True)
    h_in.copy_(x)
    h_comp = torch.empty(p.data.numel(), dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(nb * n, dtype=torch.int16, pin_memory=True)

    def enc_e2e():
        p.samples.copy_(h_in, non_blocking=True)
        p.encode()
        h_comp.copy_(p.data, non_blocking=True)  # worst-case strided image; a packed D2H is smaller

    def dec_e2e():
        p.data.copy_(h_comp, non_blocking=True)
        p.decode()
        h_out.copy_(p.decoded[: nb * n], non_blocking=True)

    te, td = timed(enc_e2e, 3), timed(dec_e2e, 3)
    torch.cuda.synchronize()
    assert torch.equal(h_out, h_in)
    tk_e, tk_d = timed(p.encode), timed(p.decode)
    # the copies alone, the same buffers
    t_h2d = timed(lambda: p.samples.copy_(h_in, non_blocking=True), 3)
    t_d2h = timed(lambda: h_out.copy_(p.decoded[: nb * n], non_blocking=True), 3)
    report("e2e", workload="4096 x 64 KiB Poisson(1000), pinned host buffers", raw_MiB=raw / 2**20,
           encode_e2e_GiBps=round(raw / te / GIB, 2), decode_e2e_GiBps=round(raw / td / GIB, 2),
           roundtrip_e2e_GiBps=round(raw / (te + td) / GIB, 2),
           encode_kernel_GiBps=round(raw / tk_e / GIB, 2), decode_kernel_GiBps=round(raw / tk_d / GIB, 2),
           h2d_GiBps=round(raw / t_h2d / GIB, 2), d2h_GiBps=round(raw / t_d2h / GIB, 2),
           samples_contiguous=bool(p.samples.is_contiguous()), samples_dtype=str(p.samples.dtype),
           transfer_bytes_note="encode D2H copies the worst-case-strided image (raw size + framing)")


def case_giant():
    """Streams of 2^27 samples and more (DwarFS -S 28..30 blocks): one stream each, decode by the default
    path (segmented for any stream below 2^32 bytes since round 6; 2^29 bytes before) against the fused
    kernel.  The last one, 2^29 + 3 generator samples, compresses to 7.5 Gbit (past 2^32 bits)."""
    cfg = codec.CodecConfig(128, 1, "big", 0)
    for label, n, make in (("2^27+5 generator (~14 bits/sample)", (1 << 27) + 5, lambda n: gen_benchmark(n, 7)),
                           ("2^28 Poisson(1000) (~7.7 bits/sample)", 1 << 28, lambda n: poisson_scaled(n, 1000.0, 0, 8)),
                           ("2^29 Poisson(1000) (~7.7 bits/sample)", 1 << 29, lambda n: poisson_scaled(n, 1000.0, 0, 9)),
                           ("2^29+3 generator (~14 bits/sample, 7.5 Gbit)", (1 << 29) + 3,
                            lambda n: gen_benchmark(n, 11))):
        x = make(n)
        p = pipe_for(cfg, x, [n])
        raw = n * 2
        te, td = timed(p.encode, iters=3), timed(p.decode, iters=3)
        seg = codec.segmented_decode_stats(reset=True)
        pf = pipe_for(cfg, x, [n], dec=codec.DecodeOptions(path="fused"))
        tf = timed(pf.decode, iters=1, warm_s=0.0)
        report("giant", layout=label, raw_MiB=raw / 2**20, ratio=round(int(p.sizes.sum()) / raw, 4),
               encode_GiBps=round(raw / te / GIB, 2), decode_GiBps=round(raw / td / GIB, 2),
               decode_fused_GiBps=round(raw / tf / GIB, 3), encode_ms=round(te * 1e3, 2), decode_ms=round(td * 1e3, 2),
               decode_fused_ms=round(tf * 1e3, 1), segmented_stats=seg)
        del p, pf, x
        torch.cuda.empty_cache()


CASES = {"gen": case_gen, "giant": case_giant, "fits": case_fits, "frames": case_frames, "mix": case_mix, "sweep": case_sweep,
         "e2e": case_e2e, "paths": case_paths}

if __name__ == "__main__":
    for name in sys.argv[1:] or list(CASES):
        t0 = time.time()
        CASES[name]()
        torch.cuda.empty_cache()
        print(f"# {name} took {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
