"""GPU tests of the DwarFS block codec (Python mirror and C++ facade) against
the oracle: framing + bitstream byte-identical, round trips, batching."""

import subprocess
from pathlib import Path

import numpy as np
import pytest

import datagen
from dwarfs_amd import block_codec
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("cs,pixels,ulsb,bs", [(1, 1000, 0, 16), (2, 1000, 2, 32), (1, 1000, 4, 64), (2, 3333, 6, 99)])
def test_ricepp_compressor_params(cs, pixels, ulsb, bs):
    # test/ricepp_compressor_test.cpp:124-161
    rng = np.random.default_rng(42)
    x = datagen.dwarfs_test_data(rng, pixels, cs, ulsb)
    data = x.tobytes()
    meta = f'{{"endianness":"big","bytes_per_sample":2,"unused_lsb_count":{ulsb},"component_count":{cs}}}'
    comp = block_codec.block_compressor(f"ricepp:block_size={bs}")
    out = comp.compress(data, meta)
    want = O.frame_header(len(data), bs, cs, 2, ulsb, True) + O.encode(O.cfg(bs, cs, True, ulsb), x)
    assert out == want
    assert len(out) < 7 * len(data) // 10
    assert block_codec.decompress(out) == data
    d = block_codec.RiceppBlockDecompressor(out)
    assert d.uncompressed_size() == len(data)
    assert d.metadata() == (f'{{"bytes_per_sample":2,"component_count":{cs},"endianness":"big",'
                            f'"unused_lsb_count":{ulsb}}}')
    target = bytearray()
    d.start_decompression(target)
    assert d.decompress_frame(len(data)) is True
    assert d.decompress_frame(len(data)) is False
    assert bytes(target) == data


def test_compress_many_decompress_many():
    rng = np.random.default_rng(3)
    meta = '{"endianness":"little","bytes_per_sample":2,"unused_lsb_count":2,"component_count":2}'
    blocks = [datagen.poisson_data(rng, 2 * int(rng.integers(1, 20000)), lam=200, ulsb=2, big_endian=False).tobytes()
              for _ in range(100)]
    comp = block_codec.RiceppBlockCompressor(128)
    outs = comp.compress_many(blocks, meta)
    oc = O.cfg(128, 2, False, 2)
    for b, o in zip(blocks, outs):
        assert o == O.frame_header(len(b), 128, 2, 2, 2, False) + O.encode(oc, np.frombuffer(b, np.uint16))
    decs = [block_codec.RiceppBlockDecompressor(o) for o in outs]
    assert block_codec.decompress_many(decs) == blocks


def _facade_exe():
    exe = ROOT / "tests" / "cpp" / "build" / "facade_test"
    if not exe.exists():
        subprocess.run(["bash", str(ROOT / "tests" / "cpp" / "build.sh")], check=True)
    return exe


def test_cpp_facade():
    r = subprocess.run([str(_facade_exe())], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "facade_test: OK" in r.stdout


def test_cpp_facade_exit_with_batches_in_flight():
    # std::exit() from a worker thread while other workers' batches are queued
    # or on the device: the facade's atexit hook stops its queue threads before
    # the HIP runtime's teardown, so the process exits cleanly (VERDICT r04:
    # the detached driver threads raced the teardown and dumped core)
    r = subprocess.run([str(_facade_exe()), "--exit-in-flight"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout + r.stderr)
    assert "exiting after" in r.stdout
