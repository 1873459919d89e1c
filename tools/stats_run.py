"""Diagnostic: runs the bench workload against the -DRPP_STATS build and
prints the per-slot phase cycles per fast-loop iteration (slot 0 counts the
iterations).  Build: tools/build_stats.sh.  Usage: python tools/stats_run.py [nblocks] [waves]"""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["RICEPP_AMD_LIB"] = str(ROOT / "dwarfs_amd" / "lib" / "libricepp_amd_stats.so")
nblocks = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
waves = int(sys.argv[2]) if len(sys.argv) > 2 else 0
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import _native, codec, parallel  # noqa: E402

L = _native.lib()
L.rpp_stats_fetch.argtypes = [C.c_void_p, C.c_int]
n = 32768
x = make_poisson_blocks(nblocks, n, 1000.0, 42, torch.device("cuda:0"))
pipe = parallel.ShardPipeline(codec.CodecConfig(128, 1, "big", 0), x, np.arange(nblocks) * n, np.full(nblocks, n),
                              decode_options=codec.DecodeOptions(fused_waves=waves))
pipe.encode()
torch.cuda.synchronize()
st = np.zeros(16, np.uint64)
L.rpp_stats_fetch(st.ctypes.data, 1)
pipe.decode()
torch.cuda.synchronize()
pipe.check(x)
L.rpp_stats_fetch(st.ctypes.data, 1)
it = float(st[0])
print(f"nblocks {nblocks} waves {waves or 'auto'}: fast iterations {int(it)}")
for i in range(1, 16):
    if st[i]:
        print(f"slot {i:2d} cycles/iteration {st[i] / it:8.1f}")
