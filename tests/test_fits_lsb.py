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


def _one_pixel_batch(n, positions, aligns, us):
    """Images of n samples, each all zero but one sample 1 << u at `pos`, stored at ragged alignments."""
    imgs, offs, want, pos_total = [], [], [], 0
    for a in aligns:
        for p in positions:
            for u in us:
                pos_total += a
                offs.append(pos_total)
                imgs.append((p, u))
                want.append(u)
                pos_total += n
    flat = np.zeros(pos_total + 16, np.uint16)
    for o, (p, u) in zip(offs, imgs):
        flat[o + p] = be(1 << u)
    return flat, offs, want


@pytest.mark.gpu
@pytest.mark.parametrize("n", [131072 + 3, 3 * 131072 + 5])
def test_gpu_single_pixel_in_every_load_slot(n):
    """One set sample in each of the four in-flight 16-byte loads (w0..w3), the remainder loop, the ragged
    head and tail, and the next chunk, for both chunk sizes (64 KiB for small batches, 256 KiB once the
    batch gives the 256 CUs four blocks each)."""
    dev = torch.device("cuda:0")
    T = 256
    pos = {0, 1, 7, 8, 9, n - 1, n - 2, n - 9}
    for chunk in (32768, 131072):
        for j in range(4):  # w0..w3 of the first unrolled trip, lanes 0 and 255
            pos |= {8 * (j * T) + 3, 8 * (j * T + T - 1) + 5}
        pos |= {8 * (4 * T) + 2, chunk - 9, chunk - 1, chunk, chunk + 1, chunk + 8 * (3 * T) + 6}
        pos |= {min(n - 1, 2 * chunk + 17), chunk - 8 * T + 4}  # remainder loop of a chunk
    positions = sorted(p for p in pos if 0 <= p < n)
    flat, offs, want = _one_pixel_batch(n, positions, aligns=(0, 1, 3), us=(0, 7))
    d = torch.from_numpy(flat.view(np.int16)).to(dev)
    ns = [n] * len(offs)
    got = codec.unused_lsb_count_batch(d, offs, ns).cpu().numpy()  # small batch: 64 KiB chunks
    assert list(got) == want
    # the same images padded with aliased all-zero images to a big batch: 256 KiB chunks
    zero_off = len(flat) - 16
    pad = max(0, 1100 - len(offs))
    got2 = codec.unused_lsb_count_batch(d, offs + [zero_off] * pad, ns + [1] * pad).cpu().numpy()
    assert list(got2[:len(offs)]) == want and set(got2[len(offs):]) <= {16}


@pytest.mark.gpu
def test_gpu_images_longer_than_max_samples_are_read_whole():
    """max_samples only sizes the grid: a caller passing a smaller value still gets whole images scanned
    (the blocks stride over the chunks)."""
    import ctypes as C

    from dwarfs_amd import _native as N

    dev = torch.device("cuda:0")
    n = 5 * 32768 + 11
    flat, offs, want = _one_pixel_batch(n, [n - 1, 4 * 32768 + 5, 40000], aligns=(0, 2), us=(3,))
    d = torch.from_numpy(flat.view(np.int16)).to(dev)
    d_off = torch.as_tensor(np.asarray(offs, np.int64), device=dev)
    d_n = torch.as_tensor(np.full(len(offs), n, np.int64), device=dev)
    work = torch.empty(len(offs), dtype=torch.int32, device=dev)
    counts = torch.empty(len(offs), dtype=torch.int32, device=dev)
    st = N.lib().rpp_unused_lsb_batch(C.c_void_p(d.data_ptr()), C.c_void_p(d_off.data_ptr()),
                                      C.c_void_p(d_n.data_ptr()), 1, len(offs), 1, C.c_void_p(work.data_ptr()),
                                      C.c_void_p(counts.data_ptr()), C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert st == 0
    assert list(counts.cpu().numpy()) == want


@pytest.mark.gpu
def test_gpu_more_than_65535_images_are_split():
    dev = torch.device("cuda:0")
    ni = 70001
    x = np.zeros(ni * 4 + 16, np.uint16)
    want = []
    for i in range(ni):
        u = i % 11
        x[4 * i + (i % 4)] = be(1 << u)
        want.append(u)
    d = torch.from_numpy(x.view(np.int16)).to(dev)
    got = codec.unused_lsb_count_batch(d, [4 * i for i in range(ni)], [4] * ni).cpu().numpy()
    assert np.array_equal(got, np.array(want))
