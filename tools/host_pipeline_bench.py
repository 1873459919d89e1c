"""PCIe-inclusive throughput of the host-resident pipelines:
4096 x 64 KiB Poisson(1000) blocks in pinned host memory -> GPU encode + pack
-> pinned host, and back through the chunked decode.  Prints one JSON line per
(direction, chunk) plus the plain pinned copy rates for context."""

import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from dwarfs_amd import codec, host_pipeline as HP  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, r


def main():
    nb, n = 4096, 32768
    g = torch.Generator(device="cuda").manual_seed(42)
    x = torch.poisson(torch.full((nb * n,), 1000.0, device="cuda"), generator=g).clamp(0, 65535).to(torch.int32)
    x = (((x & 0xFF) << 8) | (x >> 8)).to(torch.int16)  # stored big endian
    host = x.cpu().pin_memory()
    raw = nb * n * 2
    gib = float(1 << 30)
    cfg = codec.CodecConfig(block_size=128, component_stream_count=1, byteorder="big", unused_lsb_count=0)
    offs = np.arange(nb, dtype=np.int64) * n
    d = torch.empty_like(x)
    t, _ = timed(lambda: d.copy_(host, non_blocking=True), 5)
    print(json.dumps({"what": "pinned H2D copy", "GiBps": round(raw / t / gib, 2)}), flush=True)
    t, _ = timed(lambda: host.copy_(d, non_blocking=True), 5)
    print(json.dumps({"what": "pinned D2H copy", "GiBps": round(raw / t / gib, 2)}), flush=True)
    for chunk in (256, 512, 1024, 4096):
        ep = HP.HostEncodePipeline(cfg, chunk_blocks=chunk)
        hout = ep.run(host, offs, [n] * nb).data  # pinned output buffer, reused
        t, enc = timed(lambda: ep.run(host, offs, [n] * nb, out=hout), 5)
        comp = int(enc.sizes.sum())
        print(json.dumps({"what": "host encode pipeline", "chunk_blocks": chunk, "ms": round(t * 1e3, 3),
                          "GiBps": round(raw / t / gib, 2), "pcie_bytes": raw + comp}), flush=True)
        dp = HP.HostDecodePipeline(cfg, chunk_blocks=chunk)
        out = torch.empty(nb * n, dtype=torch.int16, pin_memory=True)
        t, _ = timed(lambda: dp.run(enc.data, enc.offsets, enc.sizes, [n] * nb, out=out), 5)
        assert torch.equal(out, host)
        print(json.dumps({"what": "host decode pipeline", "chunk_blocks": chunk, "ms": round(t * 1e3, 3),
                          "GiBps": round(raw / t / gib, 2), "pcie_bytes": raw + comp}), flush=True)


if __name__ == "__main__":
    main()
