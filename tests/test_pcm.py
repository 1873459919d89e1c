"""PCM sample transformer: DwarFS's
pcm_sample_transformer<int32_t> (include/dwarfs/pcm_sample_transformer.h:36-71,
src/pcm_sample_transformer.cpp:44-228), HIP unpack/pack through the C ABI
rpp_pcm_unpack / rpp_pcm_pack against the CPU oracle (oracle/oracle.py
pcm_unpack / pcm_pack).

The oracle is pinned by the reference's own known-answer tests
(test/pcm_sample_transformer_test.cpp:33-293 -> tests/golden/pcm_kat.json, made
by tests/golden/make_pcm_kat.py) and by a scalar per-sample restatement below.
GPU cases: every endianness x signedness x padding x byte count, several bit
widths, random bytes (padding and above-`bits` garbage included, which the
reference does not mask), ragged lengths and unaligned buffers -- bit-exact."""

import ctypes as C
import itertools
import json
from pathlib import Path

import numpy as np
import pytest
import torch

from dwarfs_amd import _native as N
from dwarfs_amd.pcm import PcmSampleEndianness as E, PcmSamplePadding as P, PcmSampleSignedness as S
from dwarfs_amd.pcm import PcmSampleTransformer
from oracle import oracle as O

KATS = json.loads((Path(__file__).resolve().parent / "golden" / "pcm_kat.json").read_text())
FORMATS = [(be, sg, lp, nb, bits)
           for be, sg, lp in itertools.product((1, 0), (1, 0), (1, 0))
           for nb in (1, 2, 3, 4)
           for bits in sorted({1, 8 * nb - 3 if nb > 1 else 5, 8 * nb, {1: 8, 2: 12, 3: 20, 4: 24}[nb]})]


def scalar_unpack(b, be, sg, lp, nb, bits):
    """Per-sample restatement of basic_pcm_sample_transformer::unpack
    (src/pcm_sample_transformer.cpp:50-93, :141-158), Python ints mod 2^32."""
    out = []
    for i in range(len(b) // nb):
        t = 0
        for k in range(nb):
            t |= b[i * nb + k] << (8 * (nb - 1 - k) if be else 8 * k)
        if lp:
            t >>= 8 * nb - bits
        if sg:
            if bits < 32 and t & (1 << (bits - 1)):
                t |= (0xFFFFFFFF << bits) & 0xFFFFFFFF
        else:
            t = (t - (1 << (bits - 1))) & 0xFFFFFFFF
        out.append(t - (1 << 32) if t & 0x80000000 else t)
    return out


def xfm(be, sg, lp, nb, bits):
    return PcmSampleTransformer(E.Big if be else E.Little, S.Signed if sg else S.Unsigned,
                                P.Lsb if lp else P.Msb, nb, bits)


# ---------------------------------------------------------------- CPU / oracle

@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_oracle_reference_kats(kat):
    args = (kat["big_endian"], kat["is_signed"], kat["lsb_padded"], kat["bytes"], kat["bits"])
    packed = bytes(kat["packed"])
    got = O.pcm_unpack(packed, *args)
    assert got.tolist() == kat["ref"]
    assert O.pcm_pack(got, *args) == packed  # EXPECT_EQ(packed, repacked)


@pytest.mark.parametrize("fmt", FORMATS)
def test_oracle_matches_scalar_restatement(fmt):
    nb = fmt[3]
    b = np.random.default_rng(sum(fmt)).integers(0, 256, nb * 257, dtype=np.uint8).tobytes()
    assert O.pcm_unpack(b, *fmt).tolist() == scalar_unpack(b, *fmt)


@pytest.mark.parametrize("fmt", FORMATS)
def test_oracle_pack_unpack_round_trip_of_valid_samples(fmt):
    be, sg, lp, nb, bits = fmt
    lo, hi = (-(1 << (bits - 1)), (1 << (bits - 1)) - 1)
    v = np.random.default_rng(bits).integers(lo, hi + 1, 1000, dtype=np.int64).astype(np.int32)
    v[:2] = (lo, hi)
    assert np.array_equal(O.pcm_unpack(O.pcm_pack(v, *fmt), *fmt), v)


def test_format_validation_maps_to_reference_errors():
    for nb in (0, 5, 8):
        with pytest.raises(RuntimeError, match=f"unsupported number of bytes per sample: {nb}"):
            xfm(1, 1, 0, nb, 8)
    with pytest.raises(ValueError):
        xfm(1, 1, 0, 2, 17)
    with pytest.raises(ValueError):
        xfm(1, 1, 0, 2, 0)
    f = N.RppPcmFormat(1, 0, 1, 3, 20)
    assert N.lib().rpp_pcm_check_format(C.byref(f)) == N.RPP_OK
    assert str(E.Big) == "big-endian" and str(S.Unsigned) == "unsigned" and str(P.Msb) == "msb-padded"


def test_empty_and_invalid_calls_without_gpu():
    f = N.RppPcmFormat(0, 1, 0, 2, 16)
    assert N.lib().rpp_pcm_unpack(C.byref(f), None, None, 0, None) == N.RPP_OK
    assert N.lib().rpp_pcm_pack(C.byref(f), None, None, 0, None) == N.RPP_OK
    assert N.lib().rpp_pcm_unpack(C.byref(f), None, None, 4, None) == N.RPP_INVALID_ARGUMENT
    bad = N.RppPcmFormat(0, 1, 0, 7, 16)
    assert N.lib().rpp_pcm_pack(C.byref(bad), None, None, 4, None) == N.RPP_UNSUPPORTED_CONFIG


# ---------------------------------------------------------------- GPU parity

@pytest.mark.gpu
@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_gpu_reference_kats(kat):
    dev = torch.device("cuda:0")
    t = xfm(kat["big_endian"], kat["is_signed"], kat["lsb_padded"], kat["bytes"], kat["bits"])
    src = torch.tensor(kat["packed"], dtype=torch.uint8, device=dev)
    dst = torch.empty(len(kat["ref"]), dtype=torch.int32, device=dev)
    t.unpack(dst, src)
    re = torch.empty_like(src)
    t.pack(re, dst)
    torch.cuda.synchronize()
    assert dst.cpu().tolist() == kat["ref"]
    assert re.cpu().tolist() == kat["packed"]


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", FORMATS)
def test_gpu_random_bytes_match_oracle(fmt):
    """Random packed bytes (garbage padding and upper bits included) at ragged
    lengths and every src/dst misalignment, unpack then pack, bit-exact."""
    dev = torch.device("cuda:0")
    nb = fmt[3]
    t = xfm(*fmt)
    rng = np.random.default_rng(1000 + sum(fmt))
    for n in (1, 3, 4, 5, 63, 64, 1023, 65541):
        raw = rng.integers(0, 256, nb * n, dtype=np.uint8)
        want = O.pcm_unpack(raw.tobytes(), *fmt)
        for so, do in ((0, 0), (1, 0), (0, 1), (3, 3)):
            sbuf = torch.zeros(nb * n + 8, dtype=torch.uint8, device=dev)
            sbuf[so:so + nb * n] = torch.from_numpy(raw).to(dev)
            dbuf = torch.full((n + 8,), -7, dtype=torch.int32, device=dev)
            t.unpack(dbuf[do:do + n], sbuf[so:so + nb * n])
            pbuf = torch.zeros(nb * n + 8, dtype=torch.uint8, device=dev)
            t.pack(pbuf[so:so + nb * n], dbuf[do:do + n])
            torch.cuda.synchronize()
            d = dbuf.cpu().numpy()
            assert np.array_equal(d[do:do + n], want), (fmt, n, so, do)
            assert (d[:do] == -7).all() and (d[do + n:] == -7).all()  # no writes outside the span
            p = pbuf.cpu().numpy()
            assert O.pcm_pack(want, *fmt) == p[so:so + nb * n].tobytes(), (fmt, n, so, do)
            assert not p[:so].any() and not p[so + nb * n:].any()


@pytest.mark.gpu
def test_gpu_large_round_trip_of_valid_samples():
    """24-bit big-endian signed LSB-padded in 3 bytes (the FLAC front end's
    common case), 48 Mi samples: pack(unpack(x)) == x; a spot check vs the oracle."""
    dev = torch.device("cuda:0")
    n = 48 << 20
    fmt = (1, 1, 1, 3, 24)
    t = xfm(*fmt)
    g = torch.Generator(device=dev).manual_seed(5)
    v = torch.randint(-(1 << 23), 1 << 23, (n,), dtype=torch.int32, device=dev, generator=g)
    b = torch.empty(3 * n, dtype=torch.uint8, device=dev)
    t.pack(b, v)
    w = torch.empty_like(v)
    t.unpack(w, b)
    torch.cuda.synchronize()
    assert torch.equal(v, w)
    head = b[:3 * 4096].cpu().numpy().tobytes()
    assert O.pcm_unpack(head, *fmt).tolist() == v[:4096].cpu().tolist()
