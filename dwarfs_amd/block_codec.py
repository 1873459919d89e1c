"""DwarFS block codec for ricepp over the MI355X kernels (Python mirror).

Mirrors src/compression/ricepp.cpp: ``ricepp_block_compressor`` (:57-182),
``ricepp_block_decompressor`` (:184-255) and the factory registered as
``"ricepp"`` with option ``block_size`` (default 128, :272-301; like the
reference's factory the value is not range-checked there: an unsupported
size raises "Unsupported configuration" from the encoder at compress time,
:97-102).  A
compressed DwarFS block is

    varint(uncompressed bytes) + thrift-compact ricepp_block_header + bitstream

(the framing is produced/parsed by the C ABI: rpp_frame_header /
rpp_parse_frame).  Besides the one-block API the reference has, this module
offers ``compress_many`` / ``decompress_many``: the MI355X way to feed the
writer's per-block jobs (src/writer/filesystem_writer.cpp:255-287) and the
reader's block-cache jobs (src/reader/internal/block_cache.cpp:628-706) --
one launch for a whole batch of blocks.
"""

from __future__ import annotations

import ctypes as C
import json
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from .codec import CodecConfig, _check, _raise_status, decode_batch, encode_batch

COMPRESSION_TYPE_RICEPP = 7  # include/dwarfs/compression.h
RICEPP_VERSION = 1  # src/compression/ricepp.cpp:55


def _meta_fields(metadata: str):
    m = json.loads(metadata)
    return (str(m["endianness"]), int(m["component_count"]), int(m["unused_lsb_count"]),
            int(m["bytes_per_sample"]))


def frame_header(uncompressed: int, block_size: int, cs: int, bps: int, ulsb: int, big_endian: bool,
                 version: int = RICEPP_VERSION) -> bytes:
    f = N.RppFrame(uncompressed, block_size, cs, bps, ulsb, 1 if big_endian else 0, version)
    buf = (C.c_uint8 * 64)()
    n = N.lib().rpp_frame_header(C.byref(f), buf)
    return bytes(buf[:n])


def parse_frame(data: bytes):
    buf = np.frombuffer(data, np.uint8)
    f = N.RppFrame()
    n = N.lib().rpp_parse_frame(buf.ctypes.data_as(C.c_void_p), len(buf), C.byref(f))
    if n < 0:
        raise RuntimeError("malformed ricepp block header")
    return f, int(n)


class RiceppBlockCompressor:
    """``ricepp_block_compressor`` (src/compression/ricepp.cpp:57-182)."""

    def __init__(self, block_size: int = 128, device="cuda"):
        self.block_size = int(block_size)
        self.device = torch.device(device)

    def clone(self) -> "RiceppBlockCompressor":
        return RiceppBlockCompressor(self.block_size, self.device)

    def type(self) -> int:
        return COMPRESSION_TYPE_RICEPP

    def describe(self) -> str:
        return f"ricepp [block_size={self.block_size}]"

    def metadata_requirements(self) -> str:
        return json.dumps({
            "bytes_per_sample": ["set", [2]],
            "component_count": ["range", 1, 2],
            "endianness": ["set", ["big", "little"]],
            "unused_lsb_count": ["range", 0, 8],
        }, separators=(",", ":"))

    def get_compression_constraints(self, metadata: str) -> dict:
        _, cs, _, bps = _meta_fields(metadata)
        return {"granularity": cs * bps}

    def estimate_memory_usage(self, data_size: int) -> int:
        return data_size

    def _config(self, metadata: Optional[str], size: int) -> CodecConfig:
        if metadata is None:
            raise RuntimeError("internal error: ricepp compression requires metadata")
        endianness, cs, ulsb, bps = _meta_fields(metadata)
        if size % (cs * bps):
            raise RuntimeError(f"unexpected data configuration: {size} bytes to compress, {cs} components, "
                               f"{bps} bytes per sample")
        cfg = CodecConfig(self.block_size, cs, "big" if endianness == "big" else "little", ulsb)
        _check(cfg)  # create_encoder's "Unsupported configuration" (:97-102)
        return cfg

    def compress(self, data: bytes, metadata: Optional[str]) -> bytes:
        return self.compress_many([data], metadata)[0]

    def compress_many(self, blocks: Sequence[bytes], metadata: Optional[str]) -> List[bytes]:
        """Compresses many blocks of one category in a single launch."""
        cfgs = {self._config(metadata, len(b)) for b in blocks}
        if not blocks:
            return []
        cfg = cfgs.pop()
        n = [len(b) // 2 for b in blocks]
        offs = np.zeros(len(blocks), np.int64)
        for i in range(1, len(blocks)):
            offs[i] = offs[i - 1] + (n[i - 1] + 7) // 8 * 8
        flat = np.zeros(int(offs[-1] + n[-1]) + 8 if blocks else 8, np.uint16)
        for o, b in zip(offs, blocks):
            flat[o:o + len(b) // 2] = np.frombuffer(b, np.uint16)
        d = torch.from_numpy(flat.view(np.int16)).to(self.device)
        res = encode_batch(cfg, d, offs, n)
        torch.cuda.current_stream().synchronize()
        res.check()
        sizes = res.sizes.cpu().numpy()
        data = res.data.cpu().numpy()
        out = []
        for i, b in enumerate(blocks):
            hdr = frame_header(len(b), self.block_size, cfg.component_stream_count, 2, cfg.unused_lsb_count,
                               cfg.byteorder == "big")
            o = int(res.offsets[i])
            out.append(hdr + data[o:o + int(sizes[i])].tobytes())
        return out


class RiceppBlockDecompressor:
    """``ricepp_block_decompressor`` (src/compression/ricepp.cpp:184-255)."""

    def __init__(self, data: bytes, device="cuda"):
        f, n = parse_frame(data)
        if f.ricepp_version > RICEPP_VERSION:
            raise RuntimeError(f"[RICEPP] unsupported version: {f.ricepp_version}")
        self.config = CodecConfig(f.block_size, f.component_count, "big" if f.big_endian else "little",
                                  f.unused_lsb_count)
        _check(self.config)
        if f.bytes_per_sample != 2:
            raise RuntimeError(f"[RICEPP] unsupported bytes per sample: {f.bytes_per_sample}")
        self.frame = f
        self.data = data[n:]
        self.device = torch.device(device)
        self._target: Optional[bytearray] = None
        self._done = False

    def type(self) -> int:
        return COMPRESSION_TYPE_RICEPP

    def uncompressed_size(self) -> int:
        return int(self.frame.uncompressed_bytes)

    def metadata(self) -> str:
        return json.dumps({
            "bytes_per_sample": int(self.frame.bytes_per_sample),
            "component_count": int(self.frame.component_count),
            "endianness": "big" if self.frame.big_endian else "little",
            "unused_lsb_count": int(self.frame.unused_lsb_count),
        }, separators=(",", ":"))

    def start_decompression(self, target: bytearray) -> None:
        self._target = target

    def decompress_frame(self, frame_size: int = 0) -> bool:
        if self._target is None:
            raise RuntimeError("decompression not started")
        if self._done:
            return False
        out = decompress_many([self], self.device)[0]
        self._target[:] = out
        self._done = True
        return True


def decompress(data: bytes, device="cuda") -> bytes:
    """``block_decompressor::decompress`` (src/block_decompressor.cpp:41-49)."""
    return decompress_many([RiceppBlockDecompressor(data, device)], device)[0]


def decompress_many(decs: Sequence[RiceppBlockDecompressor], device="cuda") -> List[bytes]:
    """Decodes many ricepp blocks with one launch per distinct config."""
    dev = torch.device(device)
    out: List[Optional[bytes]] = [None] * len(decs)
    groups = {}
    for i, d in enumerate(decs):
        groups.setdefault(d.config, []).append(i)
    for cfg, idx in groups.items():
        offs = np.zeros(len(idx), np.int64)
        lens = [len(decs[i].data) for i in idx]
        for k in range(1, len(idx)):
            offs[k] = offs[k - 1] + (lens[k - 1] + 15) // 16 * 16
        buf = np.zeros(int(offs[-1] + lens[-1]) + 32, np.uint8)
        for o, i in zip(offs, idx):
            buf[o:o + len(decs[i].data)] = np.frombuffer(decs[i].data, np.uint8)
        ns = [decs[i].uncompressed_size() // 2 for i in idx]
        samples, status = decode_batch(cfg, torch.from_numpy(buf).to(dev), offs, lens, ns)
        torch.cuda.current_stream().synchronize()
        st = status.cpu().numpy()
        host = samples.cpu().numpy().view(np.uint16)
        pos = 0
        for k, i in enumerate(idx):
            _raise_status(int(st[k]))
            out[i] = host[pos:pos + ns[k]].tobytes()
            pos += ns[k]
    return out  # type: ignore[return-value]


def block_compressor(spec: str, device="cuda") -> RiceppBlockCompressor:
    """``block_compressor(spec)`` for ``ricepp[:block_size=N]`` (src/compressor_registry.cpp:50-59)."""
    name, _, opts = spec.partition(":")
    if name != "ricepp":
        raise RuntimeError(f"unknown compression: {name}")
    bs = 128
    for kv in filter(None, opts.split(",")):
        k, eq, v = kv.partition("=")
        if k != "block_size" or not eq:
            raise RuntimeError(f"invalid option(s) for ricepp: {kv}")
        bs = int(v)
    return RiceppBlockCompressor(bs, device)
