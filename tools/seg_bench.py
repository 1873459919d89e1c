"""Encode and decode time of long-stream layouts: the library's default choice (auto), the segmented decode
forced and the fused one-wave-per-stream decode (DecodeOptions.path), with the segmented decode's counters.

usage: python tools/seg_bench.py [--bs=N] [layout ...]   (default: bs 128, all layouts)
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import datagen  # noqa: E402
from dwarfs_amd import codec  # noqa: E402

DEV = torch.device("cuda:0")
MIB = 1 << 20


def layouts():
    rng = np.random.default_rng(5)
    yield "one 16 MiB Poisson stream", [datagen.poisson_data(rng, 8 * MIB)]
    yield "one 16 MiB generator stream", [datagen.benchmark_data(rng, 8 * MIB)]
    yield "16 x 1 MiB Poisson", [datagen.poisson_data(rng, MIB // 2) for _ in range(16)]
    yield "one 32 MiB FITS-like frame", [datagen.poisson_data(rng, 16 * MIB)]
    yield "16 x 1 MiB generator", [datagen.benchmark_data(rng, MIB // 2) for _ in range(16)]
    yield "8 x 4 MiB Poisson", [datagen.poisson_data(rng, 2 * MIB) for _ in range(8)]
    sizes = [1] * 84 + [4] * 21 + [16] * 21  # configs[3] proportions, 1/16 of a GPU's share
    rng.shuffle(sizes)
    yield "mkdwarfs mix (126 blocks of 1/4/16 MiB)", [datagen.poisson_data(rng, m * MIB // 2,
                                                                          lam=float(rng.integers(200, 3000)))
                                                      for m in sizes]


def timed(fn, iters=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return min(ts)


def main():
    want = [a for a in sys.argv[1:] if not a.startswith("--bs=")]
    bs = int(next((a[5:] for a in sys.argv[1:] if a.startswith("--bs=")), 128))
    cfg = codec.CodecConfig(bs, 1, "big", 0)
    for name, blocks in layouts():
        if want and not any(w in name for w in want):
            continue
        ns = [len(b) for b in blocks]
        offs = np.zeros(len(blocks), np.int64)
        offs[1:] = np.cumsum(ns)[:-1]
        x = torch.from_numpy(np.concatenate(blocks).view(np.int16)).to(DEV)
        enc = codec.encode_batch(cfg, x, offs, ns)
        torch.cuda.synchronize()
        res = {"layout": name, "bs": bs, "raw_MiB": round(2 * sum(ns) / MIB, 1)}
        ems = timed(lambda: codec.encode_batch(cfg, x, offs, ns, out=enc.data, out_offsets=enc.offsets))
        res["encode"] = {"ms": round(ems, 3), "GiBps": round(2 * sum(ns) / 2**30 / (ems / 1e3), 2)}
        for mode in ("auto", "segmented", "fused"):
            opt = codec.DecodeOptions(path=mode)
            codec.segmented_decode_stats(reset=True)
            out = {}

            def dec():
                out["r"] = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, ns, options=opt)

            ms = timed(dec, iters=1 if mode == "fused" else 3)
            o, st = out["r"]
            ok = bool((st == 0).all().item()) and torch.equal(o[: sum(ns)], x)
            res[mode] = {"ms": round(ms, 3), "GiBps": round(2 * sum(ns) / 2**30 / (ms / 1e3), 2), "exact": ok}
            if mode != "fused":
                res[mode]["stats"] = codec.segmented_decode_stats(reset=True)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
