"""Diagnostic: decode time vs streams and waves per workgroup (RICEPP_DEC_WAVES).
Usage: python tools/occ_run.py <nblocks> <waves>"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
nb, w = int(sys.argv[1]), sys.argv[2]
os.environ["RICEPP_DEC_WAVES"] = w
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402

n = 32768
x = make_poisson_blocks(nb, n, 1000.0, 42, torch.device("cuda:0"))
pipe = parallel.ShardPipeline(codec.CodecConfig(128, 1, "big", 0), x, np.arange(nb) * n, np.full(nb, n))
pipe.encode()
torch.cuda.synchronize()
ts = []
for _ in range(5):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    pipe.decode()
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b) * 1000)
pipe.check(x)
t = min(ts)
print(f"nblocks {nb} waves/WG {w}: decode {t:.1f} us, {t * 2400 / 256:.0f} cycles per sub-block iteration")
