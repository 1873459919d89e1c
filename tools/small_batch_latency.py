"""Diagnostic: latency of one decode call for a small batch of 64 KiB blocks
(the facade's batches at 16 threads hold ~5), fused (one wave per stream)
against the segmented decode forced, and the encode call, on device-resident
data.  One JSON line per (blocks, path)."""
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
for nb in (1, 2, 4, 8, 16):
    x = np.concatenate([datagen.poisson_data(rng, n) for _ in range(nb)])
    d = torch.from_numpy(x.view(np.int16)).to("cuda:0")
    offs, ns = [i * n for i in range(nb)], [n] * nb
    enc = codec.encode_batch(cfg, d, offs, ns)
    torch.cuda.synchronize()

    def timed(fn, reps=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e6

    res = {"blocks": nb, "encode_us": round(timed(lambda: codec.encode_batch(cfg, d, offs, ns)), 1)}
    for path, opt in (("fused", codec.DecodeOptions(path="fused")), ("segmented", codec.DecodeOptions(path="segmented")),
                      ("seg12", codec.DecodeOptions(path="segmented", seg_log2=12)),
                      ("seg14", codec.DecodeOptions(path="segmented", seg_log2=14))):
        out, st = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, ns, options=opt)
        torch.cuda.synchronize()
        assert (st.cpu().numpy() == 0).all() and np.array_equal(out.cpu().numpy().view(np.uint16), x), path
        res[f"decode_{path}_us"] = round(timed(lambda: codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, ns,
                                                                          options=opt)), 1)
    print(json.dumps(res), flush=True)
