"""Multi-process (world_size 2, gloo on CPU) tests of the block-sharded path:
contiguous byte-balanced block ranges per rank, the all-gather of per-block
encoded sizes (RCCL on the GPU path) and the global image offsets derived
from it.  The per-rank encoder here is the CPU oracle (test infrastructure:
the GPU codec is exercised by the -m gpu tests); what is under test is the
sharding / collective plumbing of dwarfs_amd.parallel."""

import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import datagen
from dwarfs_amd import parallel
from oracle import oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_blocks():
    rng = np.random.default_rng(17)
    sizes = [512 * 1024, 64 * 1024, 2 * 1024 * 1024, 64 * 1024, 0, 1024 * 1024, 4 * 1024, 256 * 1024, 3 * 1024 * 1024]
    return [datagen.poisson_data(rng, s // 2) for s in sizes]


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blocks = make_blocks()
    ranges = parallel.partition_blocks([b.nbytes for b in blocks], world)
    lo, hi = ranges[rank]
    c = O.cfg(128, 1, True, 0)
    mine = [O.encode(c, b) for b in blocks[lo:hi]]
    sizes = torch.tensor([len(m) for m in mine], dtype=torch.int64)
    all_sizes = parallel.gather_sizes(sizes, dist.group.WORLD)
    offs = parallel.global_offsets(all_sizes)
    payloads = [None] * world
    dist.all_gather_object(payloads, mine)
    if rank == 0:
        image = b"".join(p for part in payloads for p in part)
        json.dump({"ranges": ranges, "sizes": all_sizes.tolist(), "offsets": offs.tolist(),
                   "image_len": len(image), "image_hex_head": image[:64].hex(),
                   "image_crc": int(np.frombuffer(image, np.uint8).astype(np.uint64).sum())}, open(out_path, "w"))
    dist.barrier()
    dist.destroy_process_group()


def test_partition_blocks_balanced_and_contiguous():
    sizes = [1, 4, 16, 1, 4, 16, 1, 4, 16, 8]
    for world in (1, 2, 4, 8):
        r = parallel.partition_blocks(sizes, world)
        assert len(r) == world
        assert r[0][0] == 0 and r[-1][1] == len(sizes)
        for a, b in zip(r, r[1:]):
            assert a[1] == b[0]
    r = parallel.partition_blocks([10] * 8, 4)
    assert r == [(0, 2), (2, 4), (4, 6), (6, 8)]


def test_world2_gather_sizes_and_image_offsets(tmp_path):
    out = tmp_path / "r0.json"
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    res = json.loads(out.read_text())
    blocks = make_blocks()
    c = O.cfg(128, 1, True, 0)
    ref = [O.encode(c, b) for b in blocks]
    assert res["sizes"] == [len(r) for r in ref]
    assert res["offsets"] == list(np.concatenate([[0], np.cumsum([len(r) for r in ref])[:-1]]).astype(int))
    image = b"".join(ref)
    assert res["image_len"] == len(image)
    assert res["image_hex_head"] == image[:64].hex()
    assert res["image_crc"] == int(np.frombuffer(image, np.uint8).astype(np.uint64).sum())
    lo0, hi0 = res["ranges"][0]
    lo1, hi1 = res["ranges"][1]
    assert lo0 == 0 and hi0 == lo1 and hi1 == len(blocks)
    b0 = sum(b.nbytes for b in blocks[lo0:hi0])
    total = sum(b.nbytes for b in blocks)
    assert abs(b0 - total / 2) <= max(b.nbytes for b in blocks)


def _size_gather_worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    for name, count in (("uniform", 5), ("ragged", 3 + 4 * rank), ("empty", 0 if rank == 0 else 6)):
        g = parallel.SizeGather(count, "cpu", dist.group.WORLD)
        got = []
        for step in range(3):  # the cached buffers are reused every step
            sizes = torch.arange(count, dtype=torch.int64) + 1000 * rank + 100 * step
            all_sizes = g(sizes)
            got.append([all_sizes.tolist(), parallel.global_offsets(all_sizes).tolist()])
        res[name] = got
    if rank == 0:
        json.dump(res, open(out_path, "w"))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_size_gather_cached_uniform_and_ragged(tmp_path):
    out = tmp_path / "sg.json"
    mp.spawn(_size_gather_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    res = json.loads(out.read_text())
    for name, counts in (("uniform", [5, 5]), ("ragged", [3, 7]), ("empty", [0, 6])):
        for step, (sizes, offs) in enumerate(res[name]):
            want = [v for r, c in enumerate(counts) for v in (np.arange(c) + 1000 * r + 100 * step).tolist()]
            assert sizes == want, name
            assert offs == [0] + np.cumsum(want)[:-1].tolist() if want else offs == [], name


def _mix_worker(rank, world, port, out_path):
    """bench.py --workload mix on one rank, without the codec: its byte-balanced share of the configs[3]
    block list, a stand-in encoded size per block (a function of the block index alone), the all-gather of
    the sizes and the image offsets."""
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mix = bench.mix_block_mib(32)
    ranges = parallel.partition_blocks([m << 20 for m in mix], world)
    lo, hi = ranges[rank]
    sizes = torch.tensor([(mix[i] << 19) + 7 * i for i in range(lo, hi)], dtype=torch.int64)
    gather = parallel.SizeGather(hi - lo, "cpu", dist.group.WORLD)
    all_sizes = gather(sizes)
    offs = parallel.global_offsets(all_sizes)
    if rank == 0:
        json.dump({"ranges": ranges, "sizes": all_sizes.tolist(), "offsets": offs.tolist()}, open(out_path, "w"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_mix_workload_partition_and_offsets(tmp_path, world):
    """configs[3] strong-scaling mode: the ranks' shards cover the 32 GiB mix exactly once, in order,
    balanced by bytes; the gathered sizes and image offsets are those of the whole list."""
    import bench

    out = tmp_path / "mix.json"
    mp.spawn(_mix_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
    res = json.loads(out.read_text())
    mix = bench.mix_block_mib(32)
    assert sum(mix) == 32 * 1024 and len(mix) == 5120
    ranges = res["ranges"]
    assert ranges[0][0] == 0 and ranges[-1][1] == len(mix)
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    share = [sum(mix[a:b]) for a, b in ranges]
    assert max(share) - min(share) <= 32  # MiB: within two 16 MiB blocks
    want = [(m << 19) + 7 * i for i, m in enumerate(mix)]
    assert res["sizes"] == want
    assert res["offsets"] == list(np.concatenate([[0], np.cumsum(want)[:-1]]).astype(int))
