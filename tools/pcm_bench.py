"""PCM unpack/pack throughput on one MI355X.

Per format: n samples resident in HBM, rpp_pcm_unpack (bytes*n read, 4n
written) and rpp_pcm_pack (4n read, bytes*n written) timed with HIP events on
the launch stream; achieved = algorithmic bytes / average launch time, against
the 8 TB/s HBM peak.  One JSON line per format and direction.

    python tools/pcm_bench.py [n_samples] [iters]
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from dwarfs_amd.pcm import PcmSampleEndianness as E, PcmSamplePadding as P, PcmSampleSignedness as S  # noqa: E402
from dwarfs_amd.pcm import PcmSampleTransformer  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256 << 20
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    v = torch.randint(-(1 << 15), 1 << 15, (n,), dtype=torch.int32, device=dev)
    w = torch.empty_like(v)
    for nb, bits, end, sig, pad in ((2, 16, E.Little, S.Signed, P.Msb), (3, 24, E.Big, S.Signed, P.Lsb),
                                    (4, 24, E.Little, S.Signed, P.Msb), (1, 8, E.Big, S.Unsigned, P.Msb),
                                    (2, 12, E.Big, S.Unsigned, P.Lsb)):
        t = PcmSampleTransformer(end, sig, pad, nb, bits)
        b = torch.empty(nb * n, dtype=torch.uint8, device=dev)
        t.pack(b, v & ((1 << (bits - 1)) - 1))
        t.unpack(w, b)
        torch.cuda.synchronize()
        for name, fn in (("unpack", lambda: t.unpack(w, b)), ("pack", lambda: t.pack(b, w))):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(iters):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / iters
            algo = (nb + 4) * n
            print(json.dumps({"op": f"pcm_{name}", "format": f"{end} {sig} {pad} {nb}B/{bits}b",
                              "n_samples": n, "us": round(us, 2), "GBps": round(algo / us / 1e3, 1),
                              "frac_hbm": round(algo / us / 1e3 / PEAK, 4)}), flush=True)


if __name__ == "__main__":
    main()
