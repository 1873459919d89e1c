#!/usr/bin/env python3
"""configs[4] bs 16 / 32 decode for a kernel trace: 4096 x 64 KiB Poisson blocks at one bit depth,
encoded once, decoded `reps` times (run under rocprofv3 --kernel-trace --stats).

usage: python tools/rows_prof.py [bs] [bits] [reps]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tools")]
from dwarfs_amd import codec  # noqa: E402
from workloads import poisson_scaled  # noqa: E402


def main() -> None:
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    bits = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    ulsb = 16 - bits
    cfg = codec.CodecConfig(bs, 1, "big", ulsb)
    x = poisson_scaled(4096 * 32768, max(1000.0 / (1 << (2 * ulsb)), 4.0), ulsb, 11)
    offs = np.arange(4096, dtype=np.int64) * 32768
    ns = np.full(4096, 32768, np.int64)
    enc = codec.encode_batch(cfg, x, offs, ns)
    for _ in range(reps):
        out, st = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, ns)
    torch.cuda.synchronize()
    assert torch.equal(out[:x.numel()], x)
    print("ok", bs, bits, reps)


if __name__ == "__main__":
    main()
