"""Unused-LSB detection of 16-bit images: the FITS
categorizer's get_unused_lsb_count<uint16_t>
(src/writer/categorizer/fits_categorizer.cpp:118-178), HIP OR-reduction via
the C ABI rpp_unused_lsb_batch against the CPU oracle.

The cases follow the reference's own test
(test/fits_categorizer_test.cpp:119-170): a 16x8 image with one pixel set to
big-endian (1 << u), u = 0..8, at every position and at 32 data alignments,
must report u; plus all-zero / empty images and large random images."""

import numpy as np
import pytest
import torch

import datagen
from dwarfs_amd import codec
from oracle import oracle as O

GOLDEN = __import__("pathlib").Path(__file__).resolve().parent / "golden"


def be(v):
    return ((v >> 8) | (v << 8)) & 0xFFFF


def test_oracle_single_pixel_images():
    # fits_categorizer_test.cpp:129-156 (one alignment is enough on the CPU)
    for pos in range(128):
        for u in range(9):
            img = np.zeros(128, np.uint16)
            img[pos] = be(1 << u)
            assert O.unused_lsb_count(img) == u


def test_oracle_edge_cases():
    assert O.unused_lsb_count(np.zeros(0, np.uint16)) == 16
    assert O.unused_lsb_count(np.zeros(77, np.uint16)) == 16
    assert O.unused_lsb_count(np.array([be(0x8000)], np.uint16)) == 15
    assert O.unused_lsb_count(np.array([0x0001], np.uint16), big_endian=False) == 0
    assert O.unused_lsb_count(np.array([be(5 << 4), be(3 << 6)], np.uint16)) == 4


@pytest.mark.parametrize("name", ["dark.fits", "test.fits"])
def test_oracle_fits_fixtures_are_plausible(name):
    _, x = datagen.parse_fits(GOLDEN / name)
    u = O.unused_lsb_count(x)
    # the stored frames are 16-bit images; every sample must be a multiple of 2^u
    vals = ((x.astype(np.uint32) >> 8) | (x.astype(np.uint32) << 8)) & 0xFFFF
    assert 0 <= u <= 16 and np.all(vals % (1 << min(u, 15)) == 0)


@pytest.mark.gpu
def test_gpu_reference_single_pixel_cases():
    dev = torch.device("cuda:0")
    imgs, offs, ns, want = [], [], [], []
    pos_total = 0
    for align in range(32):  # sample offsets 0..31: every 16-byte alignment
        pos_total += align
        for pos in range(128):
            for u in range(9):
                img = np.zeros(128, np.uint16)
                img[pos] = be(1 << u)
                imgs.append(img)
                offs.append(pos_total)
                ns.append(128)
                want.append(u)
                pos_total += 128
    flat = np.zeros(pos_total + 16, np.uint16)
    for o, img in zip(offs, imgs):
        flat[o:o + 128] = img
    d = torch.from_numpy(flat.view(np.int16)).to(dev)
    got = []
    for s in range(0, len(ns), 30000):  # <= 65535 images per call
        got.append(codec.unused_lsb_count_batch(d, offs[s:s + 30000], ns[s:s + 30000]).cpu().numpy())
    assert np.array_equal(np.concatenate(got), np.array(want))


@pytest.mark.gpu
def test_gpu_random_images_match_oracle():
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(7)
    sizes = [0, 1, 7, 8, 9, 1000, 32768, 32769, 100003, 1 << 20, 3 * (1 << 20) + 5]
    offs, ns, pos = [], [], 0
    parts = []
    for i, n in enumerate(sizes):
        pos += int(rng.integers(0, 9))  # ragged alignment
        u = int(rng.integers(0, 12)) if i % 3 else 16
        vals = (rng.poisson(300, n).astype(np.uint32) << u) & 0xFFFF if u < 16 else np.zeros(n, np.uint32)
        x = be(vals).astype(np.uint16)
        offs.append(pos)
        ns.append(n)
        parts.append((pos, x))
        pos += n
    flat = np.zeros(pos + 16, np.uint16)
    for o, x in parts:
        flat[o:o + len(x)] = x
    d = torch.from_numpy(flat.view(np.int16)).to(dev)
    got = codec.unused_lsb_count_batch(d, offs, ns).cpu().numpy()
    want = [O.unused_lsb_count(x) for _, x in parts]
    assert list(got) == want
    got_le = codec.unused_lsb_count_batch(d, offs, ns, big_endian=False).cpu().numpy()
    assert list(got_le) == [O.unused_lsb_count(x, big_endian=False) for _, x in parts]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["dark.fits", "test.fits"])
def test_gpu_fits_fixtures(name):
    _, x = datagen.parse_fits(GOLDEN / name)
    d = torch.from_numpy(np.ascontiguousarray(x).view(np.int16)).to("cuda:0")
    got = codec.unused_lsb_count_batch(d, [0], [len(x)]).cpu().numpy()
    assert int(got[0]) == O.unused_lsb_count(x)
