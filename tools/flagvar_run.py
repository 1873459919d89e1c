"""Diagnostic: encode/decode kernel times of a flag-variant build (tools/flagvar.sh).
Usage: python tools/flagvar_run.py <tag|base>"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
m = sys.argv[1]
if m != "base":
    os.environ["RICEPP_AMD_LIB"] = str(ROOT / "dwarfs_amd" / "lib" / f"libricepp_amd_fv{m}.so")
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402

nblocks, n = 4096, 32768
x = make_poisson_blocks(nblocks, n, 1000.0, 42, torch.device("cuda:0"))
pipe = parallel.ShardPipeline(codec.CodecConfig(128, 1, "big", 0), x, np.arange(nblocks) * n, np.full(nblocks, n))
pipe.step()
torch.cuda.synchronize()
pipe.check(x)
te, td = pipe.kernel_times(10)
print(f"variant {m}: encode {te * 1e6:.1f} us decode {td * 1e6:.1f} us")
