"""Diagnostic for DESIGN.md §4 "64-bit shifts and the last VGPR": encodes 4096 x 64 KiB
benchmark-generator blocks at bs 128 cs 2 with the library named by
RICEPP_AMD_LIB (a tools/variant.sh build), counts the streams that differ from
the oracle, and -- for a -DRPP_DIAG_BRANCH_CHECK build -- reads the emission
branch counters (ricepp_kernels.hip branch_diag).  One JSON line per repeat.
Usage: RICEPP_AMD_LIB=... python tools/branch_diag.py <label> [repeats] [nblocks]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import datagen  # noqa: E402
from dwarfs_amd import _native, codec  # noqa: E402
from oracle import oracle as O  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else "?"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
nblocks = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
n = 32768
L = _native.lib()
fetch = getattr(L, "rpp_branch_diag_fetch", None)
if fetch is not None:
    fetch.argtypes = [C.c_void_p, C.c_int]
    fetch.restype = C.c_int
rng = np.random.default_rng(42)
x = datagen.benchmark_data(rng, nblocks * n)
cfg = codec.CodecConfig(128, 2, "big", 0)
oc = O.cfg(128, 2, True, 0)
offs = np.arange(nblocks, dtype=np.int64) * n
ob, oo, osz, ost = O.encode_batch(oc, x, offs.astype(np.uint64), [n] * nblocks, O.worst_case_bytes(oc, n), nthreads=16)
d = torch.from_numpy(x.view(np.int16)).to("cuda:0")
fill = int(os.environ["FILL"]) if "FILL" in os.environ else None
first = None  # rep 0's output: later reps report the streams that differ from it (run-to-run nondeterminism)
for rep in range(reps):
    cnt = np.zeros(8, np.uint64)
    if fetch is not None:
        fetch(cnt.ctypes.data, 1)
    if fill is None:
        enc = codec.encode_batch(cfg, d, offs, [n] * nblocks)
    else:  # output buffer pre-filled with one byte value (default: torch.empty, whatever was there)
        cap = (O.worst_case_bytes(oc, n) + 15) // 16 * 16
        outbuf = torch.full((cap * nblocks,), fill, dtype=torch.uint8, device="cuda:0")
        enc = codec.encode_batch(cfg, d, offs, [n] * nblocks, out=outbuf,
                                 out_offsets=np.arange(nblocks, dtype=np.int64) * cap)
    torch.cuda.synchronize()
    if fetch is not None:
        fetch(cnt.ctypes.data, 1)
    sizes = enc.sizes.cpu().numpy()
    data = enc.data.cpu().numpy()
    wrong = 0
    wrong_bytes = 0
    extra_bits = missing_bits = 0
    first_bits, spans = [], []
    for i in range(nblocks):
        a = data[enc.offsets[i]:enc.offsets[i] + sizes[i]]
        b = ob[int(oo[i]):int(oo[i]) + int(osz[i])]
        if a.shape != b.shape or not np.array_equal(a, b):
            wrong += 1
            m = min(a.size, b.size)
            dif = np.nonzero(a[:m] != b[:m])[0]
            wrong_bytes += int(dif.size)
            extra_bits += int(np.unpackbits(a[:m] & ~b[:m]).sum())
            missing_bits += int(np.unpackbits(b[:m] & ~a[:m]).sum())
            if dif.size:
                first_bits.append(int(dif[0]) * 8)
                spans.append(int(dif[-1] - dif[0]) + 1)
    rec = {"label": label, "rep": rep, "streams": nblocks, "wrong_streams": wrong, "wrong_bytes": wrong_bytes,
           "extra_bits": extra_bits, "missing_bits": missing_bits}
    blocks_out = [bytes(data[enc.offsets[i]:enc.offsets[i] + sizes[i]]) for i in range(nblocks)]
    if first is None:
        first = blocks_out
        if os.environ.get("DUMP"):  # the first 64 wrong streams of rep 0, for offline analysis
            bad = [i for i in range(nblocks) if blocks_out[i] != bytes(ob[int(oo[i]):int(oo[i]) + int(osz[i])])][:64]
            np.savez_compressed(os.environ["DUMP"], idx=np.array(bad, np.int64),
                                **{f"s{i}": np.frombuffer(blocks_out[i], np.uint8) for i in bad})
    else:
        rec["differ_from_rep0"] = sum(1 for i in range(nblocks) if blocks_out[i] != first[i])
    if first_bits:
        fb = np.array(first_bits)
        rec.update({"first_diff_bit_pct": [int(np.percentile(fb, q)) for q in (0, 10, 50, 90, 100)],
                    "diff_span_bytes_pct": [int(np.percentile(spans, q)) for q in (0, 10, 50, 90, 100)],
                    "first_diff_bit_mod_32k_pct": [int(np.percentile(fb % 32768, q)) for q in (0, 50, 100)]})
    if fetch is not None:
        rec.update(dict(zip(["fast", "fast_wrong", "slow", "slow_needless", "wrong_exec_hi_empty",
                             "wrong_exec_lo_empty", "wrong_wide_lo", "wrong_wide_hi"], map(int, cnt))))
    print(json.dumps(rec), flush=True)
