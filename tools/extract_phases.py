"""Diagnostic: per-phase cycles of the segmented decode's extraction tiles
(RPP_TEST_PHASE_TIMERS: tile hand-out, stage, decode, tile scan + look-back, stores; wave 0
of each workgroup, s_memtime), on 16 x 16 MiB Poisson(1000) blocks.
Usage: python tools/extract_phases.py"""
import ctypes as C
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dwarfs_amd import _native as N, codec, parallel  # noqa: E402
from tools.workloads import poisson_scaled  # noqa: E402

cfg = codec.CodecConfig(128, 1, "big", 0)
nb, n = 16, 8 << 20
x = poisson_scaled(nb * n, 1000.0, 0, 5)
offs = np.arange(nb, dtype=np.int64) * n
for flags, label in ((0, "plain"), (4, "timers")):
    p = parallel.ShardPipeline(cfg, x, offs, np.full(nb, n, np.int64),
                               decode_options=codec.DecodeOptions(path="segmented", test_flags=flags))
    p.step()
    torch.cuda.synchronize()
    p.check(x)
    buf = (C.c_ulonglong * 8)()
    N.lib().rpp_diag_read(buf, 1)
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        p.decode()
    torch.cuda.synchronize()
    N.lib().rpp_diag_read(buf, 1)
    a.record(s)
    p.decode()
    b.record(s)
    torch.cuda.synchronize()
    N.lib().rpp_diag_read(buf, 0)
    tiles = max(1, buf[7])
    ph = {k: round(buf[i] / tiles) for i, k in enumerate(("between_tiles", "stage", "decode", "scan_lookback",
                                                           "stores"))}
    print(json.dumps({"mode": label, "decode_ms": round(a.elapsed_time(b), 3), "tiles": int(buf[7]),
                      "cycles_per_tile": ph}), flush=True)
    del p
