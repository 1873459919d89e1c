"""Diagnostic: one 64 KiB Poisson block decoded repeatedly by the fused
kernel and by the segmented decode (for rocprofv3 --kernel-trace: where a lone
stream's decode time goes).  Usage: python tools/lone_stream_trace.py [reps]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import datagen  # noqa: E402
from dwarfs_amd import codec  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = codec.CodecConfig(128, 1, "big", 0)
rng = np.random.default_rng(1)
n = 32768
x = datagen.poisson_data(rng, n)
d = torch.from_numpy(x.view(np.int16)).to("cuda:0")
enc = codec.encode_batch(cfg, d, [0], [n])
torch.cuda.synchronize()
for path in ("fused", "segmented"):
    opt = codec.DecodeOptions(path=path)
    for _ in range(reps):
        out, st = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, [n], options=opt)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all() and np.array_equal(out.cpu().numpy().view(np.uint16), x), path
print("ok")
