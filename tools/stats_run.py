"""Diagnostic: runs the bench workload against the -DRPP_STATS build and
prints per-sub-block loop trip counts.  Build: tools/build_stats.sh"""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["RICEPP_AMD_LIB"] = str(ROOT / "dwarfs_amd" / "lib" / "libricepp_amd_stats.so")
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import _native, codec, parallel  # noqa: E402

L = _native.lib()
L.rpp_stats_fetch.argtypes = [C.c_void_p, C.c_int]
nblocks, n = 4096, 32768
x = make_poisson_blocks(nblocks, n, 1000.0, 42, torch.device("cuda:0"))
pipe = parallel.ShardPipeline(codec.CodecConfig(128, 1, "big", 0), x, np.arange(nblocks) * n, np.full(nblocks, n))
pipe.encode()
torch.cuda.synchronize()
st = np.zeros(16, np.uint64)
L.rpp_stats_fetch(st.ctypes.data, 1)
pipe.decode()
torch.cuda.synchronize()
pipe.check(x)
L.rpp_stats_fetch(st.ctypes.data, 1)
names = ["windows", "-", "-", "-", "t_looptop", "t_ensure",
         "subblocks", "t_load+header", "-", "t_zero/raw", "t_lookup", "t_maps+terms", "t_count+extract", "-",
         "t_winend", "t_flush+request"]
sb = float(st[6])
for i, nm in enumerate(names):
    print(f"{nm:20s} total={int(st[i]):12d}  per_subblock={st[i] / sb:8.3f}")
