"""Diagnostic: encode kernel time vs number of blocks (waves per SIMD).
Usage: python tools/enc_occ.py <nblocks>..."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import make_poisson_blocks  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402

n = 32768
for nb in map(int, sys.argv[1:]):
    x = make_poisson_blocks(nb, n, 1000.0, 42, torch.device("cuda:0"))
    pipe = parallel.ShardPipeline(codec.CodecConfig(128, 1, "big", 0), x, np.arange(nb) * n, np.full(nb, n))
    pipe.encode()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        pipe.encode()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1000)
    t = min(ts)
    print(f"encode nblocks {nb}: {t:.1f} us, {t * 1e-6 * 2.4e9 / 32:.0f} cycles per 8-sub-block iteration")
