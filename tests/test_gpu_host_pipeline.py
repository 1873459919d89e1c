"""GPU tests of the host-resident batching pipelines (dwarfs_amd.host_pipeline,
SURVEY.md §8(f2)): chunked encode with on-device packing and chunked decode,
PCIe copies overlapped.  Bar: every packed stream bit-exact against the
oracle, every decoded block equal to its input."""

import numpy as np
import pytest
import torch

import datagen
from dwarfs_amd import codec, host_pipeline as HP
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _host_blocks(blocks):
    offs, pos = [], 0
    for b in blocks:
        pos = (pos + 7) // 8 * 8
        offs.append(pos)
        pos += len(b)
    flat = torch.zeros(max(pos, 1) + 8, dtype=torch.int16, pin_memory=True)
    fv = flat.numpy().view(np.uint16)
    for o, b in zip(offs, blocks):
        fv[o:o + len(b)] = b
    return flat, offs


@pytest.mark.parametrize("chunk", [1, 3, 8, 64])
@pytest.mark.parametrize("cs,bs", [(1, 128), (2, 64), (1, 16)])
def test_host_encode_decode_pipelines_match_oracle(chunk, cs, bs):
    rng = np.random.default_rng(chunk * 7 + cs + bs)
    cfg = codec.CodecConfig(block_size=bs, component_stream_count=cs, byteorder="big", unused_lsb_count=0)
    oc = O.cfg(bs, cs, True, 0)
    lens = [0, 2, 130, 4096, 32768, 1000, 32768, 254, 65536 // 2, 6] + [int(x) * cs for x in rng.integers(1, 5000, 9)]
    blocks = [datagen.poisson_data(rng, n) if i % 3 else datagen.full_range_data(rng, n) for i, n in enumerate(lens)]
    blocks = [b[: len(b) // cs * cs] for b in blocks]
    flat, offs = _host_blocks(blocks)
    enc = HP.HostEncodePipeline(cfg, chunk_blocks=chunk).run(flat, offs, [len(b) for b in blocks])
    wants = [O.encode(oc, b) for b in blocks]
    for i, w in enumerate(wants):
        assert enc.block(i) == w, f"block {i}"
        assert enc.offsets[i] % 16 == 0
    out = HP.HostDecodePipeline(cfg, chunk_blocks=chunk).run(enc.data, enc.offsets, enc.sizes,
                                                             [len(b) for b in blocks])
    ov = out.numpy().view(np.uint16)
    for i, (o, b) in enumerate(zip(HP.HostDecodePipeline.output_offsets([len(b) for b in blocks]), blocks)):
        assert np.array_equal(ov[o:o + len(b)], b), f"decode block {i}"


def test_host_pipelines_full_size_round_trip():
    """4096 x 64 KiB (the bench workload) through both host pipelines: the
    packed streams equal the device-resident encode, the decode restores the
    input (size-independent properties at full size)."""
    nb, n = 4096, 32768
    x = torch.randint(0, 2000, (nb * n,), dtype=torch.int16)
    host = x.pin_memory()
    cfg = codec.CodecConfig(block_size=128, component_stream_count=1, byteorder="big", unused_lsb_count=0)
    offs = np.arange(nb, dtype=np.int64) * n
    enc = HP.HostEncodePipeline(cfg, chunk_blocks=512).run(host, offs, [n] * nb)
    dev = codec.encode_batch(cfg, host.to("cuda"), offs, [n] * nb)
    torch.cuda.synchronize()
    dsz = dev.sizes.cpu().numpy()
    assert np.array_equal(dsz, enc.sizes)
    ddata = dev.data.cpu().numpy()
    hdata = enc.data.numpy()
    for b in range(0, nb, 97):
        assert ddata[dev.offsets[b]:dev.offsets[b] + dsz[b]].tobytes() == hdata[enc.offsets[b]:enc.offsets[b] + dsz[b]].tobytes()
    out = HP.HostDecodePipeline(cfg, chunk_blocks=512).run(enc.data, enc.offsets, enc.sizes, [n] * nb)
    assert torch.equal(out[: nb * n], host)


def test_pipeline_rejects_unpinned_and_misaligned():
    cfg = codec.CodecConfig(block_size=128, component_stream_count=1, byteorder="big", unused_lsb_count=0)
    with pytest.raises(ValueError):
        HP.HostEncodePipeline(cfg).run(torch.zeros(64, dtype=torch.int16), [0], [64])
    with pytest.raises(ValueError):
        HP.HostDecodePipeline(cfg).run(HP.pinned_empty(64), [8], [16], [8])


def test_pack_batch_empty_and_scan_total():
    """rpp_pack_batch with no blocks writes a zero total."""
    import ctypes as C
    from dwarfs_amd import _native as N
    tot = torch.full((1,), 77, dtype=torch.int64, device="cuda")
    st = N.lib().rpp_pack_batch(None, None, None, 0, None, None, C.c_void_p(tot.data_ptr()),
                                C.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert st == 0 and int(tot.item()) == 0


@pytest.mark.parametrize("kind", ["blocks", "long"])
def test_shard_pipeline_graph_replay_exact(kind):
    """parallel.ShardPipeline.capture (the bench's HIP-graph step): after an eager step, replayed steps give
    the same encoded streams (oracle-exact) and decode every block exactly, for short blocks (one wave each)
    and for a batch with long streams (segmented encode and decode, side-stream fork/join inside the graph)."""
    from dwarfs_amd import parallel

    rng = np.random.default_rng(17 if kind == "blocks" else 18)
    cfg = codec.CodecConfig(128, 1, "big", 0)
    oc = O.cfg(128, 1, True, 0)
    lens = [32768] * 48 if kind == "blocks" else [1 << 19, 3000, 1 << 18, 40000]
    blocks = [datagen.poisson_data(rng, n) for n in lens]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    x = torch.from_numpy(np.concatenate(blocks).view(np.int16)).to("cuda:0")
    pipe = parallel.ShardPipeline(cfg, x, offs, np.asarray(lens, np.int64))
    pipe.step()
    torch.cuda.synchronize()
    pipe.check(x)
    pipe.capture()
    pipe.data.zero_()
    pipe.decoded.zero_()
    for _ in range(3):
        pipe.step()
    torch.cuda.synchronize()
    pipe.check(x)
    data, sizes = pipe.data.cpu().numpy(), pipe.sizes.cpu().numpy()
    for i, b in enumerate(blocks):
        o = int(pipe.out_offsets[i])
        assert data[o:o + int(sizes[i])].tobytes() == O.encode(oc, b), i
