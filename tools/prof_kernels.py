"""Runs the bench workload's encode and decode kernels a few times (for
rocprofv3 --kernel-trace / --pmc).  Usage: python tools/prof_kernels.py [iters] [kind]"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
nblocks, n = 4096, 32768
dev = torch.device("cuda:0")
x = make_poisson_blocks(nblocks, n, 1000.0, 42, dev)
cfg = codec.CodecConfig(128, 1, "big", 0)
pipe = parallel.ShardPipeline(cfg, x, np.arange(nblocks, dtype=np.int64) * n, np.full(nblocks, n, np.int64))
for _ in range(iters):
    pipe.encode()
    pipe.decode()
torch.cuda.synchronize()
pipe.check(x)
print("ok", int(pipe.sizes.sum().item()))
