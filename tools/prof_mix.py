"""Runs the configs[3] mix (bench.py --workload mix, one GPU) for rocprofv3:
one encode+decode round trip (checked), then ENC encodes and DEC decodes.
tools/pmc_mix_summary.py attributes the dispatches to calls.
Usage: python tools/prof_mix.py [gib] [enc] [dec]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402

gib = int(sys.argv[1]) if len(sys.argv) > 1 else 32
n_enc = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n_dec = int(sys.argv[3]) if len(sys.argv) > 3 else 2
dev = torch.device("cuda", 0)
mix = bench.mix_block_mib(gib)
x, offs, ns = bench.make_mix_shard(mix, 0, len(mix), dev)
cfg = codec.CodecConfig(128, 1, "big", 0)
pipe = parallel.ShardPipeline(cfg, x, offs, ns)
pipe.step()
torch.cuda.synchronize()
pipe.check(x)
for _ in range(n_enc):
    pipe.encode()
torch.cuda.synchronize()
for _ in range(n_dec):
    pipe.decode()
torch.cuda.synchronize()
print(f"prof_mix: {len(mix)} blocks, {int(np.sum(ns)) * 2 / 2**30:.2f} GiB, {n_enc} encodes, {n_dec} decodes")
