"""Diagnostic: fused-decode time per sub-block vs streams per SIMD.

Decodes the bench workload's Poisson(1000) 64 KiB streams with 1024 / 2048 /
3072 / 4096 / 8192 streams and the workgroup width that puts 1, 2, 3, 4 (and
2 x 4) waves on every SIMD; prints one JSON line per case with the kernel
time (HIP events, steady clocks after a warm-up) and the SIMD cycles per
sub-block at the clock given (default 2.4 GHz).  Usage:
python tools/occupancy_sweep.py [clock_GHz]"""
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

clock = float(sys.argv[1]) if len(sys.argv) > 1 else 2.4
n = 32768
dev = torch.device("cuda:0")
cfg = codec.CodecConfig(128, 1, "big", 0)
CUS = torch.cuda.get_device_properties(dev).multi_processor_count
for nblocks, waves in ((1024, 4), (2048, 8), (3072, 12), (4096, 16), (4096, 8), (8192, 16)):
    x = make_poisson_blocks(nblocks, n, 1000.0, 42, dev)
    pipe = parallel.ShardPipeline(cfg, x, np.arange(nblocks, dtype=np.int64) * n, np.full(nblocks, n, np.int64),
                                  decode_options=codec.DecodeOptions(path="fused", fused_waves=waves))
    pipe.encode()
    pipe.decode()
    torch.cuda.synchronize()
    pipe.check(x)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        pipe.decode()
        torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 20
    e0.record(s)
    for _ in range(iters):
        pipe.decode()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    sb = nblocks * n // 128
    simds = 4 * CUS
    print(json.dumps({"streams": nblocks, "waves_per_wg": waves, "waves_per_simd": nblocks / simds,
                      "decode_us": round(us, 2), "GiBps": round(nblocks * n * 2 / (us * 1e-6) / 2**30, 1),
                      "simd_cycles_per_subblock": round(us * 1e3 * clock / (sb / simds), 1)}), flush=True)
    del pipe, x
    torch.cuda.empty_cache()
