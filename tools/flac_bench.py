"""FLAC block codec throughput on one GPU: DwarFS-sized blocks (16 MiB of
stereo 16-bit and 8-channel 24-in-32-bit PCM sines + noise), compress and
decompress through dwarfs_amd.flac (host bytes in and out, so PCIe and host
copies are included) and the kernels alone (device-resident), against the CPU
restatement (oracle/flac_oracle.c, one thread; libFLAC itself is absent).
One JSON line per case.  --gpu-only: the kernels alone, no CPU oracle or
host path (for profiling)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from dwarfs_amd import _native as N  # noqa: E402
from dwarfs_amd import flac as FL  # noqa: E402
from oracle import flac as F  # noqa: E402
from test_flac import sines  # noqa: E402

import ctypes as C  # noqa: E402

dev = torch.device("cuda:0")
gpu_only = "--gpu-only" in sys.argv
for channels, nbytes, bits in ((2, 2, 16), (8, 4, 24)):
    n = (16 << 20) // (channels * nbytes)
    rng = np.random.default_rng(1)
    x = (sines(channels, n, bits).astype(np.int64) + rng.integers(-8, 9, n * channels))
    x = np.clip(x, -(1 << (bits - 1)), (1 << (bits - 1)) - 1).astype(np.int32)
    meta = json.dumps({"endianness": "little", "signedness": "signed", "padding": "msb", "bytes_per_sample": nbytes,
                       "bits_per_sample": bits, "number_of_channels": channels})
    xt = torch.from_numpy(x).to(dev)
    raw = torch.empty(x.size * nbytes, dtype=torch.uint8, device=dev)
    FL._transformer((nbytes - 1) | FL.FLAG_SIGNED, bits).pack(raw, xt)  # (LE, signed, MSB: the meta above)
    data = raw.cpu().numpy().tobytes()
    comp = FL.FlacBlockCompressor().compress(data, meta)
    assert FL.decompress(comp) == data

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    te = td = float("nan")
    if not gpu_only:
        te = timed(lambda: FL.FlacBlockCompressor().compress(data, meta))
        td = timed(lambda: FL.decompress(comp))
    # kernels alone
    L = N.lib()
    frames = (n + 4095) // 4096
    out = torch.empty(frames * int(L.rpp_flac_frame_bound(channels, bits)) + 64, dtype=torch.uint8, device=dev)
    wsb = int(L.rpp_flac_encode_workspace_bytes(n, channels, bits))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    tk_e = timed(lambda: L.rpp_flac_encode(C.c_void_p(xt.data_ptr()), n, channels, bits, C.c_void_p(out.data_ptr()),
                                           C.c_void_p(tot.data_ptr()), C.c_void_p(ws.data_ptr()), wsb,
                                           C.c_void_p(s.cuda_stream)))
    d = FL.FlacBlockDecompressor(comp)
    body = torch.from_numpy(np.frombuffer(d.stream, np.uint8)[d.frames_at:].copy()).to(dev)
    y = torch.empty(n * channels, dtype=torch.int32, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    nc = torch.zeros(1, dtype=torch.int32, device=dev)
    mc = n // 4096 + body.numel() // 4096 + 64
    wdb = int(L.rpp_flac_decode_workspace_bytes(body.numel(), channels, bits, 4096, mc))
    wd = torch.empty(wdb, dtype=torch.uint8, device=dev)
    tk_d = timed(lambda: L.rpp_flac_decode(C.c_void_p(body.data_ptr()), body.numel(), channels, bits, 4096, n,
                                           C.c_void_p(y.data_ptr()), C.c_void_p(st.data_ptr()), mc,
                                           C.c_void_p(wd.data_ptr()), wdb, C.c_void_p(nc.data_ptr()),
                                           C.c_void_p(s.cuda_stream)))
    assert int(st.item()) == 0 and torch.equal(y, xt)
    tc_e = tc_d = float("nan")
    if not gpu_only:
        t0 = time.perf_counter()
        cs = F.encode(x, channels, bits, 4096, F.EncodeOptions(max_lpc_order=0))
        tc_e = time.perf_counter() - t0
        t0 = time.perf_counter()
        F.decode(cs, x.size)
        tc_d = time.perf_counter() - t0
    mib = len(data) / 2**20
    print(json.dumps({"case": "flac", "block_MiB": round(mib, 1), "channels": channels, "bits": bits,
                      "ratio": round(len(comp) / len(data), 4),
                      "compress_MiBps_host": round(mib / te, 1), "decompress_MiBps_host": round(mib / td, 1),
                      "encode_kernels_MiBps": round(mib / tk_e, 1), "decode_kernels_MiBps": round(mib / tk_d, 1),
                      "cpu_oracle_encode_MiBps_1t": round(mib / tc_e, 1),
                      "cpu_oracle_decode_MiBps_1t": round(mib / tc_d, 1)}), flush=True)

# libFLAC-like streams: every subframe LPC of order 8 (libFLAC level 5 codes up to order 8; its
# streams are what a DwarFS image made by the reference holds), written by the CPU restatement;
# the GPU decode kernels alone
channels, bits = 2, 16
n = (16 << 20) // (channels * 2)
rng = np.random.default_rng(1)
x = (sines(channels, n, bits).astype(np.int64) + rng.integers(-8, 9, n * channels))
x = np.clip(x, -(1 << (bits - 1)), (1 << (bits - 1)) - 1).astype(np.int32)
stream = F.encode(x, channels, bits, 4096, F.EncodeOptions(subframe_type="lpc", lpc_order=8, lpc_precision=12))
info, at = FL.parse_stream(stream)
L = N.lib()
body = torch.from_numpy(np.frombuffer(stream, np.uint8)[at:].copy()).to(dev)
y = torch.empty(n * channels, dtype=torch.int32, device=dev)
st = torch.zeros(1, dtype=torch.int32, device=dev)
nc = torch.zeros(1, dtype=torch.int32, device=dev)
mc = n // 4096 + body.numel() // 4096 + 64
wdb = int(L.rpp_flac_decode_workspace_bytes(body.numel(), channels, bits, 4096, mc))
wd = torch.empty(wdb, dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream()
args = (C.c_void_p(body.data_ptr()), body.numel(), channels, bits, 4096, n, C.c_void_p(y.data_ptr()),
        C.c_void_p(st.data_ptr()), mc, C.c_void_p(wd.data_ptr()), wdb, C.c_void_p(nc.data_ptr()), C.c_void_p(s.cuda_stream))
L.rpp_flac_decode(*args)
torch.cuda.synchronize()
assert int(st.item()) == 0 and np.array_equal(y.cpu().numpy(), x)
t0 = time.perf_counter()
for _ in range(5):
    L.rpp_flac_decode(*args)
torch.cuda.synchronize()
tk = (time.perf_counter() - t0) / 5
print(json.dumps({"case": "flac-lpc8-stream", "block_MiB": 16.0, "channels": channels, "bits": bits,
                  "ratio": round(len(stream) / (n * channels * 2), 4),
                  "decode_kernels_MiBps": round(16 / tk, 1)}), flush=True)
