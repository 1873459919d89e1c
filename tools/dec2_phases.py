"""Phase timers of the extraction kernel (RICEPP_DEC2_DBG=4): cycles per tile spent in setup, staging,
decode, scan + look-back, stores, summed over three decode launches.

usage: python tools/dec2_phases.py [bench|long]
  bench  the bench workload (4096 x 64 KiB) through the two-stage decode
  long   64 streams of 16 MiB (the segmented decode)"""
import ctypes as C
import os
import sys
from pathlib import Path

os.environ["RICEPP_DEC2_DBG"] = "4"
import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import _native as N  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402

layout = sys.argv[1] if len(sys.argv) > 1 else "bench"
if layout == "bench":
    os.environ["RICEPP_DECODE"] = "two-stage"
    nblocks, n = 4096, 32768
else:
    nblocks, n = 64, 8 << 20
dev = torch.device("cuda:0")
x = make_poisson_blocks(nblocks, n, 1000.0, 42, dev)
pipe = parallel.ShardPipeline(codec.CodecConfig(128, 1, "big", 0), x, np.arange(nblocks, dtype=np.int64) * n,
                              np.full(nblocks, n, np.int64))
pipe.encode()
torch.cuda.synchronize()
buf = (C.c_ulonglong * 8)()
N.lib().rpp_diag_read(buf, 1)
for _ in range(3):
    pipe.decode()
torch.cuda.synchronize()
N.lib().rpp_diag_read(buf, 1)
tiles = buf[7]
names = ["setup", "stage", "decode", "scan+lookback", "store"]
print({k: round(buf[i] / max(tiles, 1)) for i, k in enumerate(names)}, "tiles", tiles, "(s_memtime units per tile)")
pipe.check(x)
