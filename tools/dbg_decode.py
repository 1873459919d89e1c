"""Debug: decode oracle-encoded blocks on the GPU, report the first wrong
sample per block and the sub-block it falls in (test infrastructure)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from dwarfs_amd import codec  # noqa: E402
from oracle import oracle as O  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 128
nblk = int(sys.argv[2]) if len(sys.argv) > 2 else 32
n = 32768
rng = np.random.default_rng(7)
oc = O.cfg(bs, 1, True, 0)
cfg = codec.CodecConfig(bs, 1, "big", 0)
blocks = [rng.poisson(1000, n).astype(np.uint16).byteswap() for _ in range(nblk)]
enc = [O.encode(oc, x) for x in blocks]
offs = np.zeros(nblk, np.int64)
for i in range(1, nblk):
    offs[i] = offs[i - 1] + (len(enc[i - 1]) + 15) // 16 * 16
buf = np.zeros(int(offs[-1]) + len(enc[-1]) + 64, np.uint8)
for o, e in zip(offs, enc):
    buf[o:o + len(e)] = np.frombuffer(e, np.uint8)
out, st = codec.decode_batch(cfg, torch.from_numpy(buf).cuda(), offs, [len(e) for e in enc], [n] * nblk)
torch.cuda.synchronize()
st = st.cpu().numpy()
got = out.cpu().numpy().view(np.uint16)
bad = 0
for i in range(nblk):
    y = got[i * n:(i + 1) * n]
    d = np.flatnonzero(y != blocks[i])
    if st[i] or len(d):
        bad += 1
        if bad <= 8:
            k = int(d[0]) if len(d) else -1
            print(f"block {i}: status {st[i]} mismatches {len(d)} first {k} (sub-block {k // bs}, pos {k % bs}) "
                  f"got {y[k] if k >= 0 else None} want {blocks[i][k] if k >= 0 else None}")
print(f"{bad}/{nblk} blocks wrong")
