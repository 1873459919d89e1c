"""Block sharding across the GPUs of one node.

ricepp blocks are independent streams (the codec's running state resets per
stream, ricepp/include/ricepp/codec.h:69-74,81-86), so a batch of DwarFS
blocks shards by contiguous block ranges with no data exchange.  The only
collective is an all-gather of the per-block encoded sizes (RCCL over xGMI
with the "nccl" backend; gloo on CPU in tests), from which every rank knows
the global byte offset of each compressed block in the output image.  That is
the multi-GPU analogue of filesystem_writer's per-block jobs
(src/writer/filesystem_writer.cpp:255-287) whose compressed sizes are laid
out one after another.
"""

from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _native as N
from .codec import CodecConfig, DecodeOptions, _check, _raise_status, decode_workspace, encode_workspace


def partition_blocks(block_bytes: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous block ranges [start, end) per rank, balanced by bytes.

    Rank r takes the blocks whose byte midpoint falls in
    [r * total / world, (r + 1) * total / world)."""
    sizes = np.asarray(block_bytes, dtype=np.float64)
    if world <= 1 or len(sizes) == 0:
        return [(0, len(sizes))] + [(len(sizes), len(sizes))] * max(0, world - 1)
    ends = np.cumsum(sizes)
    mids = ends - sizes / 2
    total = ends[-1] if len(ends) else 0.0
    owner = np.minimum((mids * world / max(total, 1e-300)).astype(np.int64), world - 1)
    ranges = []
    for r in range(world):
        idx = np.nonzero(owner == r)[0]
        if len(idx):
            ranges.append((int(idx[0]), int(idx[-1]) + 1))
        else:
            prev = ranges[-1][1] if ranges else 0
            ranges.append((prev, prev))
    return ranges


class SizeGather:
    """All-gather of int64 per-block encoded sizes, rank order, ragged counts
    allowed.  The per-rank block counts are fixed for a shard, so they are
    exchanged once (the only host synchronisation); every later call is one
    collective into preallocated buffers: `all_gather_into_tensor` straight
    from the sizes when every rank holds the same count (RCCL on the GPU
    path), else pad -> gather -> one index_select."""

    def __init__(self, local_count: int, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if group is not None and dist.is_initialized() else 1
        self.device = torch.device(device)
        if self.world == 1:
            self.counts = [local_count]
            return
        cnt = torch.tensor([local_count], dtype=torch.int64, device=self.device)
        counts = [torch.zeros_like(cnt) for _ in range(self.world)]
        dist.all_gather(counts, cnt, group=group)
        self.counts = [int(c.item()) for c in counts]
        self.m = max(self.counts)
        self.uniform = all(c == self.m for c in self.counts)
        self.out = torch.empty(self.world * self.m, dtype=torch.int64, device=self.device)
        self.padded = None if self.uniform else torch.zeros(self.m, dtype=torch.int64, device=self.device)
        if not self.uniform:
            idx = np.concatenate([r * self.m + np.arange(c) for r, c in enumerate(self.counts)]).astype(np.int64)
            self.index = torch.as_tensor(idx, device=self.device)
            self.result = torch.empty(int(sum(self.counts)), dtype=torch.int64, device=self.device)

    def __call__(self, local_sizes: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return local_sizes
        if local_sizes.numel() != self.counts[dist.get_rank(self.group)]:
            raise ValueError("SizeGather: local block count changed")
        src = local_sizes
        if not self.uniform:
            self.padded[: local_sizes.numel()] = local_sizes
            src = self.padded
        if self.device.type == "cuda":
            dist.all_gather_into_tensor(self.out, src, group=self.group)
        else:
            dist.all_gather(list(self.out.view(self.world, self.m)), src, group=self.group)
        if self.uniform:
            return self.out
        return torch.index_select(self.out, 0, self.index, out=self.result)


def gather_sizes(local_sizes: torch.Tensor, group=None) -> torch.Tensor:
    """All-gathers int64 per-block sizes from every rank (ragged counts
    allowed) and returns them concatenated in rank order (one-shot form of
    SizeGather)."""
    if group is None or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return local_sizes
    return SizeGather(local_sizes.numel(), local_sizes.device, group)(local_sizes)


def global_offsets(all_sizes: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Exclusive prefix sum: byte offset of every block in the concatenated
    image.  Device sizes: one launch of the native scan
    (rpp_exclusive_scan_u64) on the current stream; host sizes (the gloo
    path): torch on the CPU."""
    if all_sizes.device.type == "cuda":
        sizes = all_sizes.contiguous()
        if out is None or out.numel() != sizes.numel():
            out = torch.empty_like(sizes)
        _raise_status(N.lib().rpp_exclusive_scan_u64(
            C.c_void_p(sizes.data_ptr()), sizes.numel(), C.c_void_p(out.data_ptr()),
            C.c_void_p(torch.cuda.current_stream().cuda_stream)))
        return out
    off = torch.zeros_like(all_sizes)
    if all_sizes.numel() > 1:
        off[1:] = torch.cumsum(all_sizes[:-1], 0)
    return off


class ShardPipeline:
    """This rank's shard of blocks, resident on its GPU, with every device
    array preallocated so one step is encode, size all-gather + image-offset
    scan, decode, and no host-device synchronisation."""

    def __init__(self, config: CodecConfig, samples: torch.Tensor, in_offsets, n_samples, group=None,
                 decode_options: Optional[DecodeOptions] = None):
        self.cfg = _check(config)
        self.decode_options = decode_options or DecodeOptions()
        self._dopt = self.decode_options.native()
        self.config = config
        self.group = group
        self.samples = samples
        dev = samples.device
        self.nblocks = len(n_samples)
        n_samples = np.asarray(n_samples, np.int64)
        caps = np.array([N.lib().rpp_worst_case_bytes(C.byref(self.cfg), int(n)) for n in n_samples], np.int64)
        caps = (caps + 15) // 16 * 16
        out_off = np.zeros(self.nblocks, np.int64)
        if self.nblocks:
            out_off[1:] = np.cumsum(caps)[:-1]
        self.out_offsets = out_off
        self.d_in_off = torch.as_tensor(np.asarray(in_offsets, np.int64), device=dev)
        self.d_n = torch.as_tensor(n_samples, device=dev)
        self.d_out_off = torch.as_tensor(out_off, device=dev)
        self.data = torch.empty(max(int(caps.sum()), 16), dtype=torch.uint8, device=dev)
        self.sizes = torch.zeros(self.nblocks, dtype=torch.int64, device=dev)
        self.enc_status = torch.zeros(self.nblocks, dtype=torch.int32, device=dev)
        dec_off = np.zeros(self.nblocks, np.int64)
        if self.nblocks:
            dec_off[1:] = np.cumsum(n_samples)[:-1]
        self.d_dec_off = torch.as_tensor(dec_off, device=dev)
        self.decoded = torch.empty(max(int(n_samples.sum()), 8), dtype=torch.int16, device=dev)
        self.dec_status = torch.zeros(self.nblocks, dtype=torch.int32, device=dev)
        self.total_samples = int(n_samples.sum())
        self.max_samples = int(n_samples.max()) if self.nblocks else 0
        self.workspace = decode_workspace(config, self.total_samples, self.nblocks, dev, self.max_samples,
                                          self.decode_options)
        self.enc_workspace = encode_workspace(config, self.total_samples, self.max_samples, self.nblocks, dev)
        self.all_sizes: Optional[torch.Tensor] = None
        self.image_offsets: Optional[torch.Tensor] = None
        self.size_gather = SizeGather(self.nblocks, dev, group)
        self._graphs = None  # (capture)

        class _Enc:
            pass

        self.enc = _Enc()
        self.enc.sizes = self.sizes

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def encode(self) -> None:
        _raise_status(N.lib().rpp_encode_batch_ws(
            C.byref(self.cfg), C.c_void_p(self.samples.data_ptr()), C.c_void_p(self.d_in_off.data_ptr()),
            C.c_void_p(self.d_n.data_ptr()), self.nblocks, C.c_void_p(self.data.data_ptr()),
            C.c_void_p(self.d_out_off.data_ptr()), C.c_void_p(self.sizes.data_ptr()),
            C.c_void_p(self.enc_status.data_ptr()), self.total_samples, self.max_samples,
            C.c_void_p(self.enc_workspace.data_ptr()),
            self.enc_workspace.numel(), self._stream()))

    def decode(self) -> None:
        _raise_status(N.lib().rpp_decode_batch_ex(
            C.byref(self.cfg), C.c_void_p(self.data.data_ptr()), C.c_void_p(self.d_out_off.data_ptr()),
            C.c_void_p(self.sizes.data_ptr()), self.nblocks, C.c_void_p(self.decoded.data_ptr()),
            C.c_void_p(self.d_dec_off.data_ptr()), C.c_void_p(self.d_n.data_ptr()),
            C.c_void_p(self.dec_status.data_ptr()), self.total_samples, self.max_samples,
            C.c_void_p(self.workspace.data_ptr()), self.workspace.numel(), C.byref(self._dopt), self._stream()))

    def gather(self) -> None:
        self.all_sizes = self.size_gather(self.sizes)
        self.image_offsets = global_offsets(self.all_sizes, self.image_offsets)

    def step(self) -> None:
        """encode -> size all-gather + image-offset scan -> decode, in stream
        order.  (A side stream overlapping the gather/scan with the decode
        measured slower at N=1: the cross-stream dependency opened a ~7 us
        gap before the decode, more than the 5 us scan it hid.)"""
        if self._graphs is not None:
            self._replay()
            return
        self.encode()
        self.gather()
        self.decode()

    def capture(self) -> None:
        """Records the step's kernel chains as HIP graphs (every buffer is
        preallocated and every launch is asynchronous, so a step replays
        exactly): one graph for the whole step on one rank; with several ranks
        the encode and the scan + decode, the size all-gather between them
        issued eagerly (a collective is not captured).  Call after one eager
        step (it sizes the gather's buffers)."""
        if self.all_sizes is None:
            raise RuntimeError("ShardPipeline.capture: run one step first")
        world = self.size_gather.world
        graphs = []
        torch.cuda.synchronize()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            parts = [(self.encode, self.gather, self.decode)] if world == 1 else [(self.encode,),
                                                                                   (self._scan, self.decode)]
            for fns in parts:
                g = torch.cuda.CUDAGraph()
                # (thread-local: RCCL's proxy threads keep making HIP calls
                # while this thread captures)
                with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                    for f in fns:
                        f()
                graphs.append(g)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self._graphs = graphs

    def _scan(self) -> None:
        self.image_offsets = global_offsets(self.all_sizes, self.image_offsets)

    def _replay(self) -> None:
        if len(self._graphs) == 1:
            self._graphs[0].replay()
        else:
            self._graphs[0].replay()
            self.all_sizes = self.size_gather(self.sizes)
            self._graphs[1].replay()

    def check(self, reference: torch.Tensor) -> None:
        if int(self.enc_status.abs().sum().item()) or int(self.dec_status.abs().sum().item()):
            raise RuntimeError(f"codec status enc={self.enc_status.unique().tolist()} dec={self.dec_status.unique().tolist()}")
        n = int(self.d_n.sum().item())
        if not torch.equal(self.decoded[:n], reference[:n]):
            raise RuntimeError("round trip mismatch")

    def kernel_times(self, iters: int = 10) -> Tuple[float, float]:
        """Average encode / decode kernel durations (s), HIP events on the
        stream the kernels are launched on."""
        s = torch.cuda.current_stream()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        self.encode()
        self.decode()
        torch.cuda.synchronize()
        te = td = 0.0
        for _ in range(iters):
            e[0].record(s)
            self.encode()
            e[1].record(s)
            self.decode()
            e[2].record(s)
            torch.cuda.synchronize()
            te += e[0].elapsed_time(e[1]) / 1e3
            td += e[1].elapsed_time(e[2]) / 1e3
        return te / iters, td / iters
