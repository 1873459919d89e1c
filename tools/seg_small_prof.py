"""Diagnostic: one 64 KiB stream decoded by the segmented path at small unit
sizes (seg_log2 12..16) under a kernel trace; prints host time per call."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import datagen  # noqa: E402
from dwarfs_amd import codec  # noqa: E402

cfg = codec.CodecConfig(128, 1, "big", 0)
rng = np.random.default_rng(1)
n = 32768
x = datagen.poisson_data(rng, n)
d = torch.from_numpy(x.view(np.int16)).to("cuda:0")
enc = codec.encode_batch(cfg, d, [0], [n])
torch.cuda.synchronize()
for lg in (int(a) for a in sys.argv[1:] or ["13", "14", "15", "16"]):
    opt = codec.DecodeOptions(path="segmented", seg_log2=lg)
    codec.segmented_decode_stats(reset=True)
    out, st = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, [n], options=opt)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint16)[:n], x)
    stats = codec.segmented_decode_stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(20):
        codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, [n], options=opt)
        torch.cuda.synchronize()
    print(json.dumps({"seg_log2": lg, "us": round((time.perf_counter() - t0) / 20 * 1e6, 1), "stats": stats}), flush=True)
