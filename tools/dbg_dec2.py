"""Diagnostics for the two-stage decode (rpp_decode_batch_ws): decodes oracle-encoded streams on the GPU,
reports mismatching samples and compares the parse pass's sub-block start positions (read back from the
workspace) with the positions a plain Python parse of the stream gives.

usage: python tools/dbg_dec2.py [bs] [cs] [n]
"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import datagen  # noqa: E402
from dwarfs_amd import _native as N  # noqa: E402
from dwarfs_amd import codec  # noqa: E402
from oracle import oracle as O  # noqa: E402


def positions(data: bytes, n: int, bs: int, cs: int):
    bits = np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")
    pos, out = 16 * cs, []
    nch = (n + cs * bs - 1) // (cs * bs)
    for c in range(nch):
        m = min(n - c * cs * bs, cs * bs) // cs
        for _ in range(cs):
            out.append(pos)
            f = int(bits[pos] | bits[pos + 1] << 1 | bits[pos + 2] << 2 | bits[pos + 3] << 3)
            pos += 4
            if f == 15:
                pos += 16 * m
            elif f:
                for _ in range(m):
                    while bits[pos] == 0:
                        pos += 1
                    pos += f
    out.append(pos)
    return out


def main():
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    cs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    rng = np.random.default_rng(42)
    x = datagen.dwarfs_test_data(rng, n // cs, cs, 2)
    cfg = codec.CodecConfig(bs, cs, "big", 2)
    oc = O.cfg(bs, cs, True, 2)
    data = O.encode(oc, x)
    dev = torch.device("cuda:0")
    d = torch.from_numpy(np.frombuffer(data + bytes(64), np.uint8).copy()).to(dev)
    total = len(x)
    ws = codec.decode_workspace(cfg, total, 1, dev, total)
    ws.zero_()
    out = torch.zeros(total + 8, dtype=torch.int16, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    t = lambda v: torch.as_tensor(np.asarray(v, np.int64), device=dev)  # noqa: E731
    c = codec._check(cfg)
    keep = [t([0]), t([len(data)]), t([0]), t([total])]  # (alive until the kernels ran)
    r = N.lib().rpp_decode_batch_ws(C.byref(c), C.c_void_p(d.data_ptr()), C.c_void_p(keep[0].data_ptr()),
                                    C.c_void_p(keep[1].data_ptr()), 1, C.c_void_p(out.data_ptr()),
                                    C.c_void_p(keep[2].data_ptr()), C.c_void_p(keep[3].data_ptr()),
                                    C.c_void_p(st.data_ptr()), total, total, C.c_void_p(ws.data_ptr()), ws.numel(),
                                    C.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    print("call", r, "status", int(st.item()))
    got = out[:total].cpu().numpy().view(np.uint16)
    bad = np.nonzero(got != x)[0]
    print("mismatches", len(bad), "first", bad[:20])
    for i in bad[:8]:
        where = np.nonzero(x == got[i])[0][:6]
        print(f"  sample {i}: chunk {i // (cs * bs)} comp {i % cs} idx {(i % (cs * bs)) // cs} got {got[i]:04x} "
              f"want {x[i]:04x}; got value found at {where}")
    print("bad chunks", sorted(set((bad // (cs * bs)).tolist())))
    # workspace layout (ricepp_decode2.hip layout()): 4 u64 arrays of B+1, tile_state, tile_map, sb_pos
    B = 1
    al = lambda v: (v + 255) // 256 * 256  # noqa: E731
    max_sb = total // bs + B * cs
    max_tiles = max_sb // 256 + B
    off = 4 * al((B + 1) * 8) + al(max_tiles * 8) + al(max_tiles * 4)
    want = positions(data, total, bs, cs)
    sb = ws[off:off + 4 * len(want)].cpu().numpy().view(np.uint32)
    diff = np.nonzero(sb != np.array(want, np.uint32))[0]
    print("sub-blocks", len(want) - 1, "position mismatches", len(diff), diff[:10])
    for k in diff[:5]:
        print(f"  sb {k}: gpu {sb[k]} want {want[k]}")
    bits = np.unpackbits(np.frombuffer(data, np.uint8), bitorder="little")
    hdrs = [int(bits[p] | bits[p + 1] << 1 | bits[p + 2] << 2 | bits[p + 3] << 3) for p in want[:-1]]
    print("headers", hdrs[:24])


if __name__ == "__main__":
    main()
