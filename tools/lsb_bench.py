"""FITS unused-LSB detection throughput on one MI355X.

configs[2] shape: 4096 x 4096 uint16 frames (32 MiB each), 128 of them (4 GiB)
resident in HBM, samples with 4 unused LSBs; rpp_unused_lsb_batch timed with
HIP events on the launch stream.  Algorithmic bytes = 2 bytes per sample
read (+ 8 per image written); one JSON line.

    python tools/lsb_bench.py [n_images] [iters]
"""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from dwarfs_amd import _native as N  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E


def main():
    ni = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda:0")
    n = 4096 * 4096
    g = torch.Generator(device=dev).manual_seed(3)
    x = (torch.randint(0, 1 << 12, (ni * n,), dtype=torch.int32, device=dev, generator=g) << 4)
    x = ((x >> 8) | ((x & 0xFF) << 8)).to(torch.int16)  # stored big endian
    offs = torch.arange(ni, dtype=torch.int64, device=dev) * n
    ns = torch.full((ni,), n, dtype=torch.int64, device=dev)
    work = torch.empty(ni, dtype=torch.int32, device=dev)
    counts = torch.empty(ni, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    L = N.lib()

    def run():
        st = L.rpp_unused_lsb_batch(C.c_void_p(x.data_ptr()), C.c_void_p(offs.data_ptr()),
                                    C.c_void_p(ns.data_ptr()), n, ni, 1, C.c_void_p(work.data_ptr()),
                                    C.c_void_p(counts.data_ptr()), C.c_void_p(s.cuda_stream))
        assert st == 0

    run()
    torch.cuda.synchronize()
    assert (counts == 4).all().item(), counts[:8]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    algo = 2 * ni * n + 8 * ni
    print(json.dumps({"op": "rpp_unused_lsb_batch", "images": ni, "image": "4096x4096 u16", "us": round(us, 1),
                      "GBps": round(algo / us / 1e3, 1), "frac_hbm": round(algo / us / 1e3 / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
