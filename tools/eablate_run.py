"""Diagnostic: encode kernel time of an ablation build (tools/eablate.sh).
Usage: python tools/eablate_run.py <mask|base>  (outputs are not checked)"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
m = sys.argv[1]
if m != "base":
    os.environ["RICEPP_AMD_LIB"] = str(ROOT / "dwarfs_amd" / "lib" / f"libricepp_amd_eabl{m}.so")
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402

nblocks, n = 4096, 32768
x = make_poisson_blocks(nblocks, n, 1000.0, 42, torch.device("cuda:0"))
pipe = parallel.ShardPipeline(codec.CodecConfig(128, 1, "big", 0), x, np.arange(nblocks) * n, np.full(nblocks, n))
ts = []
for _ in range(6):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    pipe.encode()
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b) * 1000)
print(f"eablate {m}: encode {min(ts[1:]):.1f} us")
