"""Where the segmented parse spends its time: s_memtime cycles (shader clock) in the guess and in the unit
chains, sub-blocks parsed, units -- for one 16 MiB Poisson stream and the block mix.

usage: python tools/seg_parse_diag.py            (16 MiB Poisson / generator streams, the 504 MiB mix)
       python tools/seg_parse_diag.py giant      (one 2^29 + 3-sample generator stream, 7.7 Gbit)"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import datagen  # noqa: E402
from dwarfs_amd import _native as N  # noqa: E402
from dwarfs_amd import codec  # noqa: E402

MIB = 1 << 20


def run(name, blocks, x=None):
    cfg = codec.CodecConfig(128, 1, "big", 0)
    ns = [len(b) for b in blocks]
    offs = np.zeros(len(ns), np.int64)
    offs[1:] = np.cumsum(ns)[:-1]
    if x is None:
        x = torch.from_numpy(np.concatenate(blocks).view(np.int16)).cuda()
    enc = codec.encode_batch(cfg, x, offs, ns)
    codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, ns)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 16)()
    N.lib().rpp_parse_diag_read(buf, 1)
    codec.segmented_decode_stats(reset=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    out, st = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, ns)
    ev[1].record()
    torch.cuda.synchronize()
    N.lib().rpp_parse_diag_read(buf, 1)
    g, ch, sb, un, nch, nst, nsl, reg, cser, ctail, ntail = map(int, buf[:11])
    # (s_memtime counts shader-clock cycles on gfx950)
    print(f"{name}: {ev[0].elapsed_time(ev[1]):.3f} ms, units {un}, sub-blocks {sb}, "
          f"guess {g / max(un, 1) / 1e3:.0f} K cycles/unit, chain {ch / max(un, 1) / 1e3:.0f} K cycles/unit = "
          f"{ch / max(sb, 1):.0f} cycles/sub-block; per guess {nch / max(un, 1):.2f} chunks {nst / max(un, 1):.1f} steps "
          f"{nsl / max(un, 1):.1f} slot-steps; lane-serial {cser / max(un, 1) / 1e3:.0f} K cycles/unit, tail "
          f"{ctail / max(un, 1) / 1e3:.0f} K cycles/unit ({ntail / max(un, 1):.1f} sub-blocks, "
          f"{ctail / max(ntail, 1):.0f} cycles each); re-guesses {reg}, exact {torch.equal(out[:sum(ns)], x)}, "
          f"{codec.segmented_decode_stats()}", flush=True)


if sys.argv[1:] == ["giant"]:
    sys.path.insert(0, str(ROOT / "tools"))
    from workloads import gen_benchmark  # noqa: E402

    n = (1 << 29) + 3
    run("one 2^29+3 generator stream", [range(n)], x=gen_benchmark(n, 11))
    sys.exit(0)
rng = np.random.default_rng(3)
run("one 16 MiB Poisson", [datagen.poisson_data(rng, 8 * MIB)])
run("one 16 MiB generator", [datagen.benchmark_data(rng, 8 * MIB)])
sizes = [1] * 84 + [4] * 21 + [16] * 21
rng.shuffle(sizes)
run("mix 504 MiB", [datagen.poisson_data(rng, m * MIB // 2, lam=float(rng.integers(200, 3000))) for m in sizes])
