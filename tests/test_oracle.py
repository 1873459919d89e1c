"""CPU tests: pin the oracle against the reference's own fixtures and KATs.

The oracle (oracle/ricepp_oracle.c) is the parity checker for the GPU path,
so it is checked first against everything the reference's tests hold:
  * bitstream_test.cpp:113-1466 -- 1000-op script -> 4186-byte golden stream
  * codec_test.cpp:164-196      -- worst-case size KATs 29138 / 58275
  * codec_test.cpp:171-172      -- incompressible data encodes to exactly
                                   the worst case
  * codec_test.cpp:198-222      -- unsupported configurations
  * codec_test.cpp:65-152, test/ricepp_compressor_test.cpp:124-131 --
                                   round-trip configurations
  * test/fits/*.fits            -- real sensor frames, round trip
"""

import json
from pathlib import Path

import numpy as np
import pytest

import datagen
from oracle import oracle as O

GOLDEN = Path(__file__).resolve().parent / "golden"


def test_bitstream_kat_matches_reference_golden():
    kat = json.loads((GOLDEN / "bitstream_kat.json").read_text())
    values = [int(v, 16) for v in kat["values"]]
    out, mismatches = O.bitstream_run_ops(kat["ops"], kat["bits"], values)
    assert len(out) == 4186
    assert out.hex() == kat["expected_hex"]
    assert mismatches == 0


def test_worst_case_kats():
    assert O.worst_case_bytes(O.cfg(29, 1, True, 0), 14443) == 29138
    assert O.worst_case_bytes(O.cfg(29, 2, True, 0), 28886) == 58275


def test_incompressible_encodes_to_exact_worst_case():
    rng = np.random.default_rng(42)
    x = datagen.full_range_data(rng, 14443)
    c = O.cfg(29, 1, True, 0)
    enc = O.encode(c, x)
    assert len(enc) == 29138
    assert np.array_equal(O.decode(c, enc, x.size), x)


@pytest.mark.parametrize("bs,cs", [(513, 2), (128, 3), (0, 1), (128, 0)])
def test_unsupported_configuration(bs, cs):
    with pytest.raises(O.OracleError) as e:
        O.encode(O.cfg(bs, cs, True, 0), np.zeros(8, np.uint16))
    assert e.value.status == O.UNSUPPORTED_CONFIG


# codec_test.cpp:65-152 and ricepp_compressor_test.cpp:124-131
REF_CONFIGS = [
    (16, 1, 0, 12345, "codec_test"),
    (13, 1, 4, 4321, "codec_test"),
    (32, 1, 0, 1500, "mixed"),
    (29, 2, 2, 23456, "codec_test"),
    (16, 1, 0, 1000, "codec_test"),
    (32, 2, 2, 2000, "codec_test"),
    (64, 1, 4, 1000, "codec_test"),
    (99, 2, 6, 6666, "codec_test"),
]


@pytest.mark.parametrize("bs,cs,ulsb,n,kind", REF_CONFIGS)
@pytest.mark.parametrize("be", [True, False])
def test_reference_roundtrips(bs, cs, ulsb, n, kind, be):
    rng = np.random.default_rng(bs * 1000 + n)
    x = datagen.KINDS[kind](rng, n, ulsb, be)
    c = O.cfg(bs, cs, be, ulsb)
    enc = O.encode(c, x)
    assert len(enc) <= O.worst_case_bytes(c, n)
    assert np.array_equal(O.decode(c, enc, n), x)


# test/ricepp_compressor_test.cpp:124-131 {components, pixels, ulsb, block}
DWARFS_PARAMS = [(1, 1000, 0, 16), (2, 1000, 2, 32), (1, 1000, 4, 64), (2, 3333, 6, 99)]


@pytest.mark.parametrize("cs,pixels,ulsb,bs", DWARFS_PARAMS)
def test_dwarfs_compressor_params(cs, pixels, ulsb, bs):
    rng = np.random.default_rng(42)
    x = datagen.dwarfs_test_data(rng, pixels, cs, ulsb)
    c = O.cfg(bs, cs, True, ulsb)
    enc = O.encode(c, x)
    assert np.array_equal(O.decode(c, enc, x.size), x)
    assert len(enc) + 16 < 7 * 2 * x.size / 10  # ricepp_compressor_test.cpp:154


@pytest.mark.parametrize("name,cs", [("dark.fits", 1), ("test.fits", 2)])
def test_fits_fixture_roundtrip(name, cs):
    hdr, x = datagen.parse_fits(GOLDEN / name)
    c = O.cfg(128, cs, True, 0)
    enc = O.encode(c, x)
    assert np.array_equal(O.decode(c, enc, x.size), x)
    assert len(enc) < 2 * x.size


def test_truncated_input_is_out_of_range():
    rng = np.random.default_rng(7)
    x = datagen.poisson_data(rng, 4096)
    c = O.cfg(128, 1, True, 0)
    enc = O.encode(c, x)
    # dropping the last full 8-byte packet must fail (bitstream_reader.h:150-152)
    cut = (len(enc) - 1) // 8 * 8
    with pytest.raises(O.OracleError) as e:
        O.decode(c, enc[:cut], x.size)
    assert e.value.status == O.TRUNCATED_INPUT
    with pytest.raises(O.OracleError):
        O.decode(c, b"", 1)


def test_framing_bytes():
    # bytes confirmed by running the reference's thrift-lite codegen + compact
    # writer.
    assert O.frame_header(65536, 128, 1, 2, 0, True).hex() == "808004158002140213021300111402" + "00"
    assert O.frame_header(65536, 128, 1, 2, 0, False).hex() == "808004158002140213021300121402" + "00"
    assert O.frame_header(65536, 16, 1, 2, 0, True)[3:5].hex() == "1520"
    assert O.frame_header(65536, 512, 1, 2, 0, True)[3:6].hex() == "158008"


def test_batch_matches_single():
    rng = np.random.default_rng(3)
    sizes = [0, 1, 7, 128, 129, 1000, 4096]
    x = np.concatenate([datagen.poisson_data(rng, n) for n in sizes])
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    c = O.cfg(128, 1, True, 0)
    caps = [O.worst_case_bytes(c, n) for n in sizes]
    out, oo, sz, st = O.encode_batch(c, x, offs, sizes, caps, nthreads=4)
    assert (st == 0).all()
    for i, n in enumerate(sizes):
        blk = out[int(oo[i]):int(oo[i]) + int(sz[i])].tobytes()
        assert blk == O.encode(c, x[int(offs[i]):int(offs[i]) + n])
