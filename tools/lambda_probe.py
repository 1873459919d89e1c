#!/usr/bin/env python3
"""Decode rate by Poisson lambda (the configs[3] mix uses 300 / 1000 / 3000): the fused kernel on
4096 x 64 KiB blocks and the segmented decode on 16 x 16 MiB streams, with the histogram of the
sub-blocks' Rice parameters (read from the encoded streams on the host).

usage: python tools/lambda_probe.py [lambda ...]"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tools")]
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import codec  # noqa: E402
from workloads import timed  # noqa: E402

DEV = torch.device("cuda:0")
GIB = 2 ** 30


def fs_hist(data: np.ndarray, off: int, nbytes: int, n: int, bs: int = 128) -> dict:
    """Walk the sub-block headers of one bs128 cs1 16-bit stream (decode.h's layout: 16-bit first value,
    then per sub-block a 4-bit header fs+1 (0: zero sub-block, 15: raw), codes unary-then-fs-bits, LSB
    first within 64-bit little-endian words)."""
    words = np.frombuffer(data[off:off + ((nbytes + 7) // 8) * 8].tobytes() + b"\0" * 16, dtype="<u8")
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    pos, hist, left = 16, {}, n
    while left > 0:
        m = min(bs, left)
        h = int(bits[pos] | bits[pos + 1] << 1 | bits[pos + 2] << 2 | bits[pos + 3] << 3)
        pos += 4
        hist[h] = hist.get(h, 0) + 1
        if h == 0:
            pass
        elif h == 15:
            pos += 16 * m
        else:
            fs = h - 1
            for _ in range(m):
                while bits[pos] == 0:
                    pos += 1
                pos += 1 + fs
        left -= m
    return {k - 1: v for k, v in sorted(hist.items())}


def main() -> None:
    lams = [float(a) for a in sys.argv[1:]] or [300.0, 1000.0, 3000.0]
    cfg = codec.CodecConfig(128, 1, "big", 0)
    for lam in lams:
        for name, nb, n in (("4096x64KiB", 4096, 32768), ("16x16MiB", 16, 8 << 20)):
            x = make_poisson_blocks(nb, n, lam, 7, DEV)
            offs = np.arange(nb, dtype=np.int64) * n
            ns = np.full(nb, n, np.int64)
            enc = codec.encode_batch(cfg, x, offs, ns)
            torch.cuda.synchronize()
            out, st = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, ns)
            torch.cuda.synchronize()
            assert torch.equal(out[:nb * n], x), "round trip"
            codec.segmented_decode_stats(reset=True)
            t = timed(lambda: codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, ns))
            te = timed(lambda: codec.encode_batch(cfg, x, offs, ns))
            sizes = enc.sizes.cpu().numpy() if torch.is_tensor(enc.sizes) else np.asarray(enc.sizes)
            rec = {"lambda": lam, "layout": name, "decode_us": round(t * 1e6, 1),
                   "decode_GiBps": round(nb * n * 2 / t / GIB, 1), "encode_GiBps": round(nb * n * 2 / te / GIB, 1),
                   "bits_per_sample": round(float(sizes.sum()) * 8 / (nb * n), 3),
                   "seg_stats": codec.segmented_decode_stats(reset=True)}
            if name.startswith("4096"):
                host = enc.data.cpu().numpy()
                eo = enc.offsets.cpu().numpy() if torch.is_tensor(enc.offsets) else np.asarray(enc.offsets)
                rec["fs_hist_block0"] = fs_hist(host, int(eo[0]), int(sizes[0]), n)
            print(json.dumps(rec), flush=True)
            del x, enc, out


if __name__ == "__main__":
    main()
