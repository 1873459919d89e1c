"""CPU prototype of a cheap unit guess for a low-latency decode of one short
stream (DESIGN.md section 8, round-5 status item 5): not product code, no GPU.

Decoding one stream with several waves needs, for each unit start S_u after
the first, the first true sub-block header at or after S_u (decode.h:42-83:
nothing in the format marks it).  The segmented decode tests every candidate
c = S_u, S_u + 1, ... by parsing its sub-blocks code by code (a lane per
candidate: ~21 K cycles per step of a wave), which is what makes it 395 us
per call on one 64 KiB stream (profiles/r05_seg_small_prof.txt).

The cheaper test measured here: a Rice code is 'zeros, 1, fs bits'
(encode.h:127-145), so two parses of the same bits with the same fs merge
once they meet a common code start, and they meet within a few codes.  With
the parse chain of each fs from a fixed start (the 'canonical chain' C_fs:
a sorted array of code starts), the end of a candidate's sub-block (128
codes from c + 4 at fs = header - 1) is: parse m codes from c + 4 until a
start lies on C_fs (m is small), then C_fs[rank + 128 - m].  A candidate
costs m lane-serial codes instead of 128; its chain of K sub-blocks (the
validation: header values within a range, zero headers only in an all-zero
chain) costs K such lookups.

Reports, per data kind: how many codes it takes to merge (the per-candidate
cost), whether the lowest candidate whose chain passes K steps is the true
header (the guess), and the candidate work per unit.  Run:
    python tools/guess_proto.py [units_per_stream] [K]
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import datagen  # noqa: E402
from oracle import oracle as O  # noqa: E402

BS = 128


def bit_array(enc: bytes) -> np.ndarray:
    return np.unpackbits(np.frombuffer(enc, np.uint8), bitorder="little").astype(np.int8)


class Stream:
    def __init__(self, enc: bytes, n: int):
        self.bits = bit_array(enc)
        self.L = len(self.bits)
        ones = np.nonzero(self.bits)[0]
        i = np.searchsorted(ones, np.arange(self.L + 1))
        self.nxt1 = np.where(i < len(ones), ones[np.minimum(i, len(ones) - 1)], self.L + 10**6)
        self.n = n
        self.chains = {}

    def hdr(self, p):
        if p + 4 > self.L:
            return None
        b = self.bits
        return int(b[p]) | int(b[p + 1]) << 1 | int(b[p + 2]) << 2 | int(b[p + 3]) << 3

    def code_next(self, q, k):
        return int(self.nxt1[q]) + 1 + k if q < self.L else self.L + 10**6

    def sb_end_direct(self, c):
        """decode.h:42-83: the end of the sub-block whose header is at c (None past the stream)."""
        h = self.hdr(c)
        if h is None:
            return None
        q = c + 4
        if h == 0:
            return q
        if h == 15:
            return q + 16 * BS
        for _ in range(BS):
            q = self.code_next(q, h - 1)
            if q > self.L:
                return None
        return q

    def chain(self, k):
        """C_k: code starts of the fs-k parse from bit 0 (sorted) and its position -> rank map."""
        if k not in self.chains:
            pos = []
            q = 0
            while q < self.L:
                pos.append(q)
                q = self.code_next(q, k)
            pos.append(q)  # (the end of the last code: a sub-block may end there)
            pos = np.array(pos, np.int64)
            rank = np.full(self.L + 1, -1, np.int64)
            rank[pos[:-1]] = np.arange(len(pos) - 1)
            if pos[-1] <= self.L:
                rank[pos[-1]] = len(pos) - 1
            self.chains[k] = (pos, rank)
        return self.chains[k]

    def sb_end_merge(self, c, stat):
        """The same end through C_fs: m codes to the merge, then one lookup."""
        h = self.hdr(c)
        if h is None:
            return None
        q = c + 4
        if h == 0:
            return q
        if h == 15:
            return q + 16 * BS
        k = h - 1
        pos, rank = self.chain(k)
        m = 0
        while m < BS and q <= self.L and rank[min(q, self.L)] < 0:
            q = self.code_next(q, k)
            m += 1
        stat.append(m)
        if m == BS or q > self.L:
            return q if q <= self.L else None
        r = int(rank[q]) + BS - m
        return int(pos[r]) if r < len(pos) else None

    def true_headers(self):
        p, out = 16, []
        nsb = self.n // BS
        for _ in range(nsb):
            out.append(p)
            p = self.sb_end_direct(p)
        return np.array(out, np.int64)


def guess(st: Stream, S: int, K: int, rng_max: int, stat, cand_steps):
    """Lowest candidate >= S whose chain of K sub-blocks keeps its header values within rng_max and has zero
    headers only if all are; the chain may run off the stream's end (a unit near the end)."""
    for c in range(S, min(S + 16 * BS + 64, st.L)):
        lo, hi, q, ok = 15, 0, c, True
        for step in range(K):
            h = st.hdr(q)
            if h is None:
                break
            lo, hi = min(lo, h), max(hi, h)
            cand_steps[0] += 1
            if hi - lo > rng_max or (lo == 0 and hi != 0):
                ok = False
                break
            q = st.sb_end_merge(q, stat)
            if q is None:
                break
        if ok:
            return c
    return None


def main():
    units = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rng = np.random.default_rng(3)
    n = 32768
    kinds = {
        "poisson300": lambda: datagen.poisson_data(rng, n, lam=300.0),
        "poisson1000": lambda: datagen.poisson_data(rng, n, lam=1000.0),
        "poisson3000": lambda: datagen.poisson_data(rng, n, lam=3000.0),
        "generator": lambda: datagen.benchmark_data(rng, n),
        "spiky": lambda: datagen.spiky_data(rng, n),
        "dwarfs_test": lambda: datagen.dwarfs_test_data(rng, n),
        "test.fits": lambda: datagen.parse_fits(ROOT / "tests" / "golden" / "test.fits")[1][:n],
        "dark.fits": lambda: datagen.parse_fits(ROOT / "tests" / "golden" / "dark.fits")[1][:n],
    }
    oc = O.cfg(BS, 1, True, 0)
    for name, make in kinds.items():
        x = make()
        nn = len(x) // BS * BS
        x = x[:nn]
        st = Stream(O.encode(oc, x), nn)
        th = st.true_headers()
        # the merge path gives the exact end on every true header
        stat = []
        for p in th:
            assert st.sb_end_merge(int(p), stat) == st.sb_end_direct(int(p)), (name, p)
        merge_true = np.array(stat)
        stat, cand_steps, exact, none = [], [0], 0, 0
        thset = set(int(t) for t in th)
        meet = []  # sub-blocks from the guess until its chain reaches a true header (the stitch's meeting point)
        for u in range(1, units):
            S = st.L * u // units
            want = int(th[np.searchsorted(th, S)]) if S <= th[-1] else None
            got = guess(st, S, K, 3, stat, cand_steps)
            if got is None:
                got = guess(st, S, K, 5, stat, cand_steps)
            if got is None:
                none += 1
                continue
            if got == want:
                exact += 1
            q, j = got, 0
            while q is not None and q not in thset and j < 64:
                q = st.sb_end_direct(q)
                j += 1
            meet.append(j if q in thset else 99)
        m = np.array(stat) if stat else np.zeros(1)
        print(f"{name:12s} bits {st.L:7d} sub-blocks {len(th)}: merge codes at true headers median "
              f"{np.median(merge_true) if len(merge_true) else 0:.0f} max {merge_true.max() if len(merge_true) else 0}; "
              f"guesses exact {exact}/{units - 1} (none {none}), chains meeting the true one after "
              f"{sorted(meet)} sub-blocks; candidate steps per unit "
              f"{cand_steps[0] / (units - 1):.0f}, codes per lookup median {np.median(m):.0f} p99 "
              f"{np.percentile(m, 99):.0f}, lane-serial codes per unit {m.sum() / (units - 1):.0f}", flush=True)


if __name__ == "__main__":
    main()
