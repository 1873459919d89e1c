#!/usr/bin/env python3
"""Encode-only timing of the configs[3] mix (diagnostics for variant libraries; no output check).
usage: python tools/enc_time.py [gib]"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT)]
import bench  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402

gib = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
mix = bench.mix_block_mib(gib)
x, offs, ns = bench.make_mix_shard(mix, 0, len(mix), dev)
pipe = parallel.ShardPipeline(codec.CodecConfig(128, 1, "big", 0), x, offs, ns)
for _ in range(3):
    pipe.encode()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for _ in range(5):
    a.record()
    pipe.encode()
    b.record()
    torch.cuda.synchronize()
    best = min(best, a.elapsed_time(b))
print(json.dumps({"gib": gib, "encode_ms": round(best, 3), "GiBps": round(gib / best * 1e3, 1)}))
