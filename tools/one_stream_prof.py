"""Diagnostic: configs[0]'s shape, one 16 MiB stream (generator data as
ricepp_benchmark.cpp, and Poisson(1000)), encoded then decoded 10 times by
the default path; run under rocprofv3 --kernel-trace --stats to see where a
lone long stream's time goes.  Prints host-timed encode / decode per call."""
import json
import sys
import time

import numpy as np
import torch

sys.path[:0] = [".", "tests"]
import datagen  # noqa: E402
from dwarfs_amd import codec  # noqa: E402

cfg = codec.CodecConfig(128, 1, "big", 0)
n = 8 << 20
rng = np.random.default_rng(7)
for name, x in (("generator", datagen.benchmark_data(rng, n)), ("poisson", datagen.poisson_data(rng, n))):
    d = torch.from_numpy(x.view(np.int16)).to("cuda:0")
    enc = codec.encode_batch(cfg, d, [0], [n])
    out, st = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, [n])
    torch.cuda.synchronize()
    assert torch.equal(out[:n], d)
    te = td = 0.0
    for _ in range(10):
        t0 = time.perf_counter()
        enc = codec.encode_batch(cfg, d, [0], [n])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, [n])
        torch.cuda.synchronize()
        te += t1 - t0
        td += time.perf_counter() - t1
    print(json.dumps({"data": name, "ratio": round(int(enc.sizes.cpu()[0]) / (2 * n), 4),
                      "encode_ms": round(te / 10 * 1e3, 3), "decode_ms": round(td / 10 * 1e3, 3),
                      "stats": codec.segmented_decode_stats(reset=True)}), flush=True)
