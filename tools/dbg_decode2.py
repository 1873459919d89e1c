"""Debug: decode oracle-encoded blocks on the GPU over (cs, ulsb, endianness)
at one block size; reports the first wrong sample per config (test infrastructure)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from dwarfs_amd import codec  # noqa: E402
from oracle import oracle as O  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 128
nblk, n = 8, 32768
for cs in (1, 2):
    for ulsb in (0, 2):
        for be in (True, False):
            rng = np.random.default_rng(7)
            oc = O.cfg(bs, cs, be, ulsb)
            cfg = codec.CodecConfig(bs, cs, "big" if be else "little", ulsb)
            blocks = []
            for _ in range(nblk):
                x = (rng.poisson(1000, n).astype(np.uint16) << ulsb)
                blocks.append(x.byteswap() if be else x)
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
            msg = []
            for i in range(nblk):
                y = got[i * n:(i + 1) * n]
                d = np.flatnonzero(y != blocks[i])
                if st[i] or len(d):
                    k = int(d[0]) if len(d) else -1
                    msg.append(f"blk{i} st{st[i]} n{len(d)} first {k} got {y[k] if k >= 0 else None:#x} "
                               f"want {blocks[i][k] if k >= 0 else 0:#x}")
            print(f"cs{cs} ulsb{ulsb} be{int(be)}: {len(msg)}/{nblk} wrong", *msg[:2])
