"""Host-resident batches through the GPU codec: the batching callers of
SURVEY.md §8(f2), with the PCIe transfers overlapped with the kernels.

Reader side (``HostDecodePipeline``): the block cache decompresses whole
blocks on demand (src/reader/internal/block_cache.cpp:628-706,
src/reader/internal/cached_block.cpp:92-109) into host memory.  Here a batch
of compressed blocks in pinned host memory is decoded in chunks: chunk k+1's
host->device copy and chunk k-1's device->host copy run on their own streams
(the two DMA directions) while chunk k decodes, each device buffer used by two
chunks in turn (double buffering, ordered by events, no host waits until the
end).  Decoded samples land directly in the caller's pinned output.

Writer side (``HostEncodePipeline``): the writer compresses one block per
worker job (src/writer/filesystem_writer.cpp:255-287).  Here host samples are
encoded a chunk at a time; ``rpp_pack_batch`` packs each chunk's streams back
to back on the device so only sum(encoded sizes) crosses PCIe.  The packed
length is read back (a small copy per chunk, on the compute stream) before the
payload copy is issued; the next chunk is already queued behind it, so the GPU
does not idle on that host wait.

Product path only: no CPU fallback; the native library must be present.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from .codec import CodecConfig, _check, _raise_status


def _ptr(t: torch.Tensor) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


def _round_up(x: np.ndarray, a: int) -> np.ndarray:
    return (x + a - 1) // a * a


def _chunks(n: int, chunk: int):
    return [(lo, min(lo + chunk, n)) for lo in range(0, n, chunk)]


def pinned_empty(nbytes: int) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, pin_memory=True)


class HostDecodePipeline:
    """Decodes ricepp streams held in pinned host memory into pinned host
    memory, ``chunk_blocks`` blocks per launch, transfers overlapped."""

    def __init__(self, config: CodecConfig, chunk_blocks: int = 512, device="cuda"):
        self.cfg = _check(config)
        self.config = config
        self.chunk = int(chunk_blocks)
        self.dev = torch.device(device)
        self.h2d = torch.cuda.Stream(device=self.dev)
        self.comp = torch.cuda.Stream(device=self.dev)
        self.d2h = torch.cuda.Stream(device=self.dev)

    @staticmethod
    def output_offsets(n_samples: Sequence[int]) -> np.ndarray:
        """Sample offset of every block in the output (8-sample aligned)."""
        n = np.asarray(n_samples, np.int64)
        off = np.zeros(len(n), np.int64)
        if len(n):
            off[1:] = np.cumsum(_round_up(n, 8))[:-1]
        return off

    def run(self, comp: torch.Tensor, in_offsets: Sequence[int], in_bytes: Sequence[int], n_samples: Sequence[int],
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``comp``: pinned uint8 host tensor; block b's stream at
        ``in_offsets[b]`` (16-aligned), ``in_bytes[b]`` bytes.  Returns a pinned
        int16 host tensor with block b at ``output_offsets(n_samples)[b]``."""
        if comp.device.type != "cpu" or not comp.is_pinned():
            raise ValueError("HostDecodePipeline: compressed input must be a pinned host tensor")
        in_off = np.asarray(in_offsets, np.int64)
        in_len = np.asarray(in_bytes, np.int64)
        n = np.asarray(n_samples, np.int64)
        nb = len(n)
        if len(in_off) != nb or len(in_len) != nb:
            raise ValueError("HostDecodePipeline: ragged per-block arrays")
        if (in_off % 16).any():
            raise ValueError("HostDecodePipeline: input offsets must be 16-aligned")
        if nb and int((in_off + in_len).max()) > comp.numel():
            raise ValueError("HostDecodePipeline: block extends past the input")
        out_off = self.output_offsets(n)
        total = int(out_off[-1] + _round_up(n[-1:], 8)[0]) if nb else 0
        if out is None:
            out = torch.empty(max(total, 8), dtype=torch.int16, pin_memory=True)
        elif out.numel() < total or not out.is_pinned():
            raise ValueError("HostDecodePipeline: output must be pinned and hold every block")
        if nb == 0:
            return out
        chunks = _chunks(nb, self.chunk)
        # per-chunk device-relative offsets, uploaded once
        rel_in = np.empty(nb, np.int64)
        rel_out = np.empty(nb, np.int64)
        cin, cout = [], []
        for lo, hi in chunks:
            a = int(in_off[lo:hi].min())
            rel_in[lo:hi] = in_off[lo:hi] - a
            rel_out[lo:hi] = out_off[lo:hi] - out_off[lo]
            cin.append((a, int((in_off[lo:hi] + in_len[lo:hi]).max())))
            cout.append((int(out_off[lo]), int(out_off[hi - 1] + _round_up(n[hi - 1:hi], 8)[0])))
        cur = torch.cuda.current_stream(self.dev)
        with torch.cuda.stream(cur):
            d_rel_in = torch.as_tensor(rel_in, device=self.dev)
            d_rel_out = torch.as_tensor(rel_out, device=self.dev)
            d_len = torch.as_tensor(in_len, device=self.dev)
            d_n = torch.as_tensor(n, device=self.dev)
            status = torch.zeros(nb, dtype=torch.int32, device=self.dev)
            cap_in = max(b - a for a, b in cin) + 64  # the decoder may fetch past a stream's end
            cap_out = max(b - a for a, b in cout) + 8
            d_in = [torch.empty(cap_in, dtype=torch.uint8, device=self.dev) for _ in range(2)]
            d_out = [torch.empty(cap_out, dtype=torch.int16, device=self.dev) for _ in range(2)]
            # one decode workspace: the chunk decodes are ordered on self.comp
            ws_bytes = max(int(N.lib().rpp_decode_workspace_bytes(
                C.byref(self.cfg), int(n[lo:hi].sum()), int(n[lo:hi].max()), hi - lo)) for lo, hi in chunks)
            ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=self.dev)
        for s in (self.h2d, self.comp, self.d2h):
            s.wait_stream(cur)
        ev_h2d = [torch.cuda.Event() for _ in range(2)]
        ev_dec = [torch.cuda.Event() for _ in range(2)]
        ev_d2h = [torch.cuda.Event() for _ in range(2)]
        used = [False, False]
        for k, (lo, hi) in enumerate(chunks):
            slot = k % 2
            a, b = cin[k]
            with torch.cuda.stream(self.h2d):
                if used[slot]:
                    self.h2d.wait_event(ev_dec[slot])  # d_in[slot] read by chunk k-2's decode
                d_in[slot][: b - a].copy_(comp[a:b], non_blocking=True)
                ev_h2d[slot].record(self.h2d)
            with torch.cuda.stream(self.comp):
                self.comp.wait_event(ev_h2d[slot])
                if used[slot]:
                    self.comp.wait_event(ev_d2h[slot])  # d_out[slot] drained by chunk k-2's copy
                _raise_status(N.lib().rpp_decode_batch_ws(
                    C.byref(self.cfg), _ptr(d_in[slot]), _ptr(d_rel_in[lo:hi]), _ptr(d_len[lo:hi]), hi - lo,
                    _ptr(d_out[slot]), _ptr(d_rel_out[lo:hi]), _ptr(d_n[lo:hi]), _ptr(status[lo:hi]),
                    int(n[lo:hi].sum()), int(n[lo:hi].max()), _ptr(ws), ws.numel(),
                    C.c_void_p(self.comp.cuda_stream)))
                ev_dec[slot].record(self.comp)
            oa, ob = cout[k]
            with torch.cuda.stream(self.d2h):
                self.d2h.wait_event(ev_dec[slot])
                out[oa:ob].copy_(d_out[slot][: ob - oa], non_blocking=True)
                ev_d2h[slot].record(self.d2h)
            used[slot] = True
        for s in (self.h2d, self.comp, self.d2h):
            cur.wait_stream(s)
        cur.synchronize()  # every queued use of the device buffers has finished
        st = status.cpu().numpy()
        bad = np.nonzero(st)[0]
        if len(bad):
            _raise_status(int(st[bad[0]]))
        return out


@dataclass
class PackedBatch:
    """Host result of :class:`HostEncodePipeline`: block b's ricepp stream is
    ``data[offsets[b] : offsets[b] + sizes[b]]``."""

    data: torch.Tensor    # pinned uint8
    offsets: np.ndarray   # int64 [nblocks]
    sizes: np.ndarray     # int64 [nblocks]

    def block(self, b: int) -> bytes:
        o = int(self.offsets[b])
        return self.data[o:o + int(self.sizes[b])].numpy().tobytes()


class HostEncodePipeline:
    """Encodes stored uint16 samples held in pinned host memory, ``chunk_blocks``
    blocks per launch, and returns the packed streams in pinned host memory."""

    def __init__(self, config: CodecConfig, chunk_blocks: int = 512, device="cuda"):
        self.cfg = _check(config)
        self.config = config
        self.chunk = int(chunk_blocks)
        self.dev = torch.device(device)
        self.h2d = torch.cuda.Stream(device=self.dev)
        self.comp = torch.cuda.Stream(device=self.dev)
        self.d2h = torch.cuda.Stream(device=self.dev)

    def run(self, samples: torch.Tensor, in_offsets: Sequence[int], n_samples: Sequence[int],
            out: Optional[torch.Tensor] = None) -> PackedBatch:
        """``samples``: pinned 16-bit host tensor of stored samples; block b is
        ``samples[in_offsets[b] : in_offsets[b] + n_samples[b]]`` (offsets
        8-aligned).  ``out``: optional pinned uint8 buffer of at least the
        summed 16-rounded worst-case sizes (reused across calls)."""
        if samples.device.type != "cpu" or not samples.is_pinned() or samples.element_size() != 2:
            raise ValueError("HostEncodePipeline: samples must be a pinned 16-bit host tensor")
        samples = samples.view(torch.int16)
        in_off = np.asarray(in_offsets, np.int64)
        n = np.asarray(n_samples, np.int64)
        nb = len(n)
        if len(in_off) != nb:
            raise ValueError("HostEncodePipeline: ragged per-block arrays")
        if (in_off % 8).any():
            raise ValueError("HostEncodePipeline: input offsets must be 8-aligned")
        if nb and int((in_off + n).max()) > samples.numel():
            raise ValueError("HostEncodePipeline: block extends past the input")
        uniq, inv = np.unique(n, return_inverse=True)
        caps = np.array([N.lib().rpp_worst_case_bytes(C.byref(self.cfg), int(x)) for x in uniq], np.int64)
        caps = _round_up(caps, 16)[inv.reshape(-1)] if nb else np.zeros(0, np.int64)
        need = int(caps.sum()) if nb else 16
        if out is None:
            out = pinned_empty(need)
        elif out.numel() < need or not out.is_pinned() or out.dtype != torch.uint8:
            raise ValueError("HostEncodePipeline: output must be a pinned uint8 tensor of the summed capacities")
        host = out
        offsets = np.zeros(nb, np.int64)
        sizes = np.zeros(nb, np.int64)
        if nb == 0:
            return PackedBatch(host, offsets, sizes)
        chunks = _chunks(nb, self.chunk)
        rel_in = np.empty(nb, np.int64)
        rel_cap = np.empty(nb, np.int64)
        spans, cap_chunk = [], []
        for lo, hi in chunks:
            rel_in[lo:hi] = in_off[lo:hi] - in_off[lo:hi].min()
            c = caps[lo:hi]
            rel_cap[lo:hi] = np.concatenate([[0], np.cumsum(c)[:-1]])
            spans.append((int(in_off[lo:hi].min()), int((in_off[lo:hi] + n[lo:hi]).max())))
            cap_chunk.append(int(c.sum()))
        cur = torch.cuda.current_stream(self.dev)
        with torch.cuda.stream(cur):
            d_rel_in = torch.as_tensor(rel_in, device=self.dev)
            d_rel_cap = torch.as_tensor(rel_cap, device=self.dev)
            d_n = torch.as_tensor(n, device=self.dev)
            d_sizes = torch.zeros(nb, dtype=torch.int64, device=self.dev)
            status = torch.zeros(nb, dtype=torch.int32, device=self.dev)
            span_max = max(b - a for a, b in spans) + 8
            d_in = [torch.empty(span_max, dtype=torch.int16, device=self.dev) for _ in range(2)]
            d_enc = [torch.empty(max(cap_chunk) + 16, dtype=torch.uint8, device=self.dev) for _ in range(2)]
            d_pack = [torch.empty(max(cap_chunk) + 16, dtype=torch.uint8, device=self.dev) for _ in range(2)]
            # per slot: packed offsets [chunk] followed by the packed total
            d_meta = [torch.empty(self.chunk + 1, dtype=torch.int64, device=self.dev) for _ in range(2)]
        h_meta = [torch.empty(self.chunk + 1, dtype=torch.int64, pin_memory=True) for _ in range(2)]
        h_sizes = torch.empty(nb, dtype=torch.int64, pin_memory=True)
        for s in (self.h2d, self.comp, self.d2h):
            s.wait_stream(cur)
        ev_h2d = [torch.cuda.Event() for _ in range(2)]
        ev_enc = [torch.cuda.Event() for _ in range(2)]
        ev_meta = [torch.cuda.Event() for _ in range(2)]
        ev_d2h = [torch.cuda.Event() for _ in range(2)]
        used = [False, False]
        host_pos = 0

        def issue(k: int) -> None:
            lo, hi = chunks[k]
            slot = k % 2
            a, b = spans[k]
            with torch.cuda.stream(self.h2d):
                if used[slot]:
                    self.h2d.wait_event(ev_enc[slot])
                d_in[slot][: b - a].copy_(samples[a:b], non_blocking=True)
                ev_h2d[slot].record(self.h2d)
            with torch.cuda.stream(self.comp):
                self.comp.wait_event(ev_h2d[slot])
                if used[slot]:
                    self.comp.wait_event(ev_d2h[slot])  # d_pack / d_meta of chunk k-2 drained
                _raise_status(N.lib().rpp_encode_batch(
                    C.byref(self.cfg), _ptr(d_in[slot]), _ptr(d_rel_in[lo:hi]), _ptr(d_n[lo:hi]), hi - lo,
                    _ptr(d_enc[slot]), _ptr(d_rel_cap[lo:hi]), _ptr(d_sizes[lo:hi]), _ptr(status[lo:hi]),
                    C.c_void_p(self.comp.cuda_stream)))
                ev_enc[slot].record(self.comp)
                _raise_status(N.lib().rpp_pack_batch(
                    _ptr(d_enc[slot]), _ptr(d_rel_cap[lo:hi]), _ptr(d_sizes[lo:hi]), hi - lo, _ptr(d_pack[slot]),
                    _ptr(d_meta[slot]), C.c_void_p(d_meta[slot].data_ptr() + 8 * self.chunk),
                    C.c_void_p(self.comp.cuda_stream)))
                # the small read-back rides the compute stream: on the copy stream
                # it would queue chunk k+1's read-back ahead of chunk k's payload
                h_meta[slot].copy_(d_meta[slot], non_blocking=True)
                h_sizes[lo:hi].copy_(d_sizes[lo:hi], non_blocking=True)
                ev_meta[slot].record(self.comp)
            used[slot] = True

        issue(0)
        for k, (lo, hi) in enumerate(chunks):
            if k + 1 < len(chunks):
                # slot (k+1)%2 held chunk k-1, whose payload copy was queued last iteration
                issue(k + 1)
            slot = k % 2
            ev_meta[slot].synchronize()  # packed offsets + total of chunk k
            meta = h_meta[slot].numpy()
            total = int(meta[self.chunk])
            offsets[lo:hi] = meta[: hi - lo] + host_pos
            with torch.cuda.stream(self.d2h):
                self.d2h.wait_event(ev_meta[slot])
                host[host_pos:host_pos + total].copy_(d_pack[slot][:total], non_blocking=True)
                ev_d2h[slot].record(self.d2h)
            host_pos += total
        for s in (self.h2d, self.comp, self.d2h):
            cur.wait_stream(s)
        cur.synchronize()
        st = status.cpu().numpy()
        bad = np.nonzero(st)[0]
        if len(bad):
            _raise_status(int(st[bad[0]]))
        sizes[:] = h_sizes.numpy()
        return PackedBatch(host, offsets, sizes)
