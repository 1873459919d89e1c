#!/usr/bin/env python3
"""One 2^29 + 3-sample generator stream (~14 bits per sample, 7.5 Gbit compressed: past 2^32 bits), encoded
once and decoded by the segmented decode a few times, for a kernel trace of the decode
(rocprofv3 --kernel-trace --stats -- python tools/giant_prof.py [log2_units] [reps]).  Prints one JSON line:
decode time per call (best of reps) and the segmented-decode counters.  DESIGN.md section 4 "Segmented
decode of long streams"."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
from dwarfs_amd import codec  # noqa: E402
from workloads import gen_benchmark, pipe_for  # noqa: E402

log2 = int(sys.argv[1]) if len(sys.argv) > 1 else 0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = (1 << 29) + 3
cfg = codec.CodecConfig(128, 1, "big", 0)
x = gen_benchmark(n, 11)
dec = codec.DecodeOptions(path="segmented", seg_log2=log2) if log2 else None
p = pipe_for(cfg, x, [n], dec=dec)
codec.segmented_decode_stats(reset=True)
best = float("inf")
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    p.decode()
    torch.cuda.synchronize()
    best = min(best, time.perf_counter() - t0)
st = codec.segmented_decode_stats(reset=True)
print(json.dumps({"case": "giant_prof", "samples": n, "compressed_bits": int(p.sizes.sum()) * 8, "log2_units": log2,
                  "decode_ms": round(best * 1e3, 2), "decode_GiBps": round(2 * n / best / 2**30, 1),
                  "segmented_stats_per_call": {k: v / reps for k, v in st.items()}}), flush=True)
