"""CPU replay behind profiles/r03_spec_ab.jsonl: for the fs 5-7 sub-blocks of Poisson 64 KiB blocks, how often
the composition of the 2 / 4 lane segments (24 bits each) before a lane is a constant state map for every lane up to
the sub-block end (the condition under which RPP_SPEC could skip the exact map scan).  Uses the CPU oracle to encode."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from oracle import oracle as O
import datagen
rng = np.random.default_rng(1)
oc = O.cfg(128, 1, True, 0)
def table(fs, fix):
    T = []
    for b in range(256):
        m = []
        for s in range(8):
            c = s
            while True:
                rest = b >> c if c < 8 else 0
                if rest == 0: ex = 0; break
                tp = c + ((rest & -rest).bit_length() - 1)
                c = tp + 1 + fs
                if c >= 8: ex = c - 8; break
            m.append(ex)
        if fix:
            r = max(fs, 4)
            for s in range(r + 1, 8): m[s] = m[0]
        T.append(m)
    return T
def comp(g, f): return [g[f[s]] for s in range(8)]   # apply f first
for fix in (False, True):
    tabs = {fs: table(fs, fix) for fs in range(8)}
    tot = fb1 = fb2 = 0
    for blk in range(3):
        x = datagen.poisson_data(rng, 32768)
        data = O.encode(oc, x)
        bits = np.unpackbits(np.frombuffer(data + b'\0'*512, np.uint8), bitorder='little')
        def rd(p, n): return int(sum(int(bits[p+i]) << i for i in range(n)))
        P = 16
        for sb in range(256):
            h = rd(P, 4); fs = h - 1
            # serial parse to the end
            q = P + 4
            for i in range(128):
                while bits[q] == 0: q += 1
                q += 1 + fs
            end = q
            if 5 <= fs <= 7:
                T = tabs[fs]
                M = []
                for l in range(64):
                    st = P + 24 * l
                    mm = list(range(8))
                    for j in range(3):
                        mm = comp(T[rd(st + 8 * j, 8)], mm)
                    M.append(mm)
                const4 = [4] * 8
                X = [const4] + M[:63]
                B = [comp(X[l], X[l - 1] if l else const4) for l in range(64)]
                C = [comp(B[l], B[l - 2] if l >= 2 else const4) for l in range(64)]
                lend = (end - P) // 24
                tot += 1
                if any(len(set(B[l])) > 1 for l in range(min(lend + 1, 64))): fb1 += 1
                if any(len(set(C[l])) > 1 for l in range(min(lend + 1, 64))): fb2 += 1
            P = end
    print(f"fix={fix}: sub-blocks {tot}, fallback spec1 {fb1/tot:.3f}, spec2 {fb2/tot:.3f}")
