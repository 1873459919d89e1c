"""FLAC block codec, CPU side: the format restatement (oracle/flac_oracle.c)
round-trips every subframe kind and option it writes, and the library's
framing (C ABI, no GPU compute) agrees with it.

Parity unpinned: libFLAC, the reference's FLAC coder
(src/compression/flac.cpp), is absent here and the reference holds no FLAC
fixture; see oracle/flac_oracle.c.  The data shapes follow
test/flac_compressor_test.cpp:97-113 (sines of 599 (c + 1) mod 256 * 3.1
samples period per channel)."""

import ctypes as C
import json

import numpy as np
import pytest

from dwarfs_amd import _native as N
from oracle import flac as F

# test/flac_compressor_test.cpp:97-113: channels, samples, bytes, bits
DATA_PARAMS = [(1, 1000, 2, 16), (3, 1000, 1, 8), (1, 1000, 2, 12), (1, 100000, 3, 20), (8, 10000, 3, 20),
               (4, 10000, 4, 20), (4, 10000, 4, 24), (4, 10000, 3, 24), (7, 799999, 4, 32)]


def sine(bits, n, period):
    """make_sine (flac_compressor_test.cpp:38-47), int64 before the cast."""
    a = (1 << bits) / 2
    v = (a * np.sin(2 * np.pi * np.arange(n) / period) - 0.5).astype(np.int64)
    return np.clip(v, -(1 << (bits - 1)), (1 << (bits - 1)) - 1)


def sines(channels, n, bits):
    return np.stack([sine(bits, n, 3.1 * ((599 * (c + 1)) % 256)) for c in range(channels)], 1).reshape(-1) \
        .astype(np.int32)


def test_sine_generator_matches_reference():
    """TEST(flac_compressor, sine) (flac_compressor_test.cpp:115-136) for the int8/int16 cases."""
    assert sine(8, 5, 4.0).astype(np.int8).tolist() == [0, 127, 0, -128, 0]
    assert sine(5, 5, 4.0).tolist() == [0, 15, 0, -16, 0]
    assert sine(16, 5, 4.0).astype(np.int16).tolist() == [0, 32767, 0, -32768, 0]
    assert sine(12, 5, 4.0).tolist() == [0, 2047, 0, -2048, 0]


@pytest.mark.parametrize("channels,n,nbytes,bits", DATA_PARAMS[:8])
def test_oracle_round_trip_and_ratio(channels, n, nbytes, bits):
    x = sines(channels, n, bits)
    s = F.encode(x, channels, bits)
    st, y, ch, b = F.decode(s, x.size)
    assert st == F.OK and ch == channels and b == bits
    assert np.array_equal(y, x)
    assert len(s) < x.size * nbytes / 2  # EXPECT_LT(compressed.size(), data.size() / 2)


OPTS = {
    "fixed0": F.EncodeOptions(subframe_type="fixed", fixed_order=0),
    "fixed4": F.EncodeOptions(subframe_type="fixed", fixed_order=4),
    "lpc1": F.EncodeOptions(subframe_type="lpc", lpc_order=1, lpc_precision=15),
    "lpc12": F.EncodeOptions(subframe_type="lpc", lpc_order=12, lpc_precision=9),
    "lpc32": F.EncodeOptions(subframe_type="lpc", lpc_order=32, lpc_precision=15),
    "verbatim": F.EncodeOptions(subframe_type="verbatim"),
    "escape": F.EncodeOptions(escape=True),
    "rice2": F.EncodeOptions(rice2=True),
    "po0": F.EncodeOptions(max_partition_order=0),
    "po8": F.EncodeOptions(max_partition_order=8),
    "meta": F.EncodeOptions(padding_block=True),
    "variable": F.EncodeOptions(variable_blocking=True),
    "nowasted": F.EncodeOptions(wasted=False),
    "fixedonly": F.EncodeOptions(max_lpc_order=0),
}


@pytest.mark.parametrize("name", sorted(OPTS))
@pytest.mark.parametrize("channels,bits", [(1, 16), (2, 16), (2, 24), (3, 8), (2, 32)])
def test_oracle_every_option_round_trips(name, channels, bits):
    rng = np.random.default_rng(len(name) * 7 + channels + bits)
    n = 9000
    x = sines(channels, n, bits).astype(np.int64)
    x += rng.integers(-3, 4, x.size)
    x[::997] = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), x[::997].size)  # outliers
    x = np.clip(x, -(1 << (bits - 1)), (1 << (bits - 1)) - 1).astype(np.int32)
    for blocksize in (4096, 1152, 200):
        s = F.encode(x, channels, bits, blocksize, OPTS[name])
        st, y, _, _ = F.decode(s, x.size)
        assert st == F.OK and np.array_equal(y, x), (name, blocksize)


@pytest.mark.parametrize("stereo", [0, 8, 9, 10])
def test_oracle_stereo_assignments(stereo):
    x = sines(2, 5000, 16)
    s = F.encode(x, 2, 16, 4096, F.EncodeOptions(stereo=stereo))
    st, y, _, _ = F.decode(s, x.size)
    assert st == F.OK and np.array_equal(y, x)


def test_oracle_constant_and_wasted_bits():
    x = (np.repeat(np.arange(6000) // 100, 2) << 4).astype(np.int32)  # steps, 4 wasted bits
    x[: 2 * 4096] = 1234 << 4  # first frame constant
    for o in (F.EncodeOptions(), F.EncodeOptions(subframe_type="constant")):
        s = F.encode(x, 2, 20, 4096, o)
        st, y, _, _ = F.decode(s, x.size)
        assert st == F.OK and np.array_equal(y, x)


def test_oracle_rejects_corruption():
    x = sines(2, 10000, 16)
    s = bytearray(F.encode(x, 2, 16))
    s[len(s) // 2] ^= 0x10
    st, _, _, _ = F.decode(bytes(s), x.size)
    assert st != F.OK
    st, _, _, _ = F.decode(bytes(s[: len(s) - 5]), x.size)
    assert st != F.OK


def test_flac_symbols_exported():
    L = N.lib()
    for name in ("rpp_flac_frame_header", "rpp_flac_parse_frame", "rpp_flac_stream_header", "rpp_flac_parse_stream",
                 "rpp_flac_frame_bound", "rpp_flac_encode_workspace_bytes", "rpp_flac_encode",
                 "rpp_flac_encode_ex", "rpp_flac_encode_batch_workspace_bytes", "rpp_flac_encode_batch",
                 "rpp_flac_decode_workspace_bytes", "rpp_flac_decode", "rpp_flac_decode_batch_workspace_bytes",
                 "rpp_flac_decode_batch"):
        assert hasattr(L, name)


@pytest.mark.parametrize("size,channels,bits,flags", [(0, 1, 8, 0), (4000, 2, 16, 0xC1), (10**9, 8, 32, 0x63),
                                                      (123457, 7, 20, 0x22)])
def test_flac_block_header_round_trip(size, channels, bits, flags):
    from dwarfs_amd import flac as FL
    h = FL.frame_header(size, channels, bits, flags)
    f, n = FL.parse_frame(h + b"fLaC")
    assert n == len(h)
    assert (f.uncompressed_bytes, f.num_channels, f.bits_per_sample, f.flags) == (size, channels, bits, flags)
    # varint + field headers of the thrift compact protocol (thrift/compression.thrift:36-40)
    assert h[-1] == 0 and h[-3] == 0x13 and h[-5] == 0x13


@pytest.mark.parametrize("channels,bits,n", [(1, 16, 1000), (2, 24, 2**33 + 5), (8, 32, 12345678), (3, 8, 0)])
def test_stream_header_parses_in_oracle_and_library(channels, bits, n):
    """The library's "fLaC" + STREAMINFO (rpp_flac_stream_header) in front of the oracle's frames decodes
    in the oracle, and rpp_flac_parse_stream reads the oracle's (padding block included) back."""
    from dwarfs_amd import flac as FL
    buf = (C.c_uint8 * 64)()
    size = N.lib().rpp_flac_stream_header(channels, bits, n, buf)
    head = bytes(buf[:size])
    info, at = FL.parse_stream(head)
    assert at == 42 and (info.channels, info.bits_per_sample, info.total_samples) == (channels, bits, n)
    assert (info.min_blocksize, info.max_blocksize, info.sample_rate) == (4096, 4096, 48000)
    if 0 < n < 10**6:
        x = sines(channels, n, bits)
        s = F.encode(x, channels, bits, 4096, F.EncodeOptions(padding_block=True))
        info2, at2 = FL.parse_stream(s)
        assert at2 == 42 + 4 + 13 and info2.total_samples == n
        st, y, _, _ = F.decode(head + s[at2:], x.size)
        assert st == F.OK and np.array_equal(y, x)


def test_flac_factory_options_and_description():
    from dwarfs_amd import flac as FL
    assert FL.block_compressor("flac").describe() == "flac [level=5]"
    assert FL.block_compressor("flac:level=8:exhaustive").describe() == "flac [level=8, exhaustive]"
    with pytest.raises(RuntimeError):
        FL.block_compressor("flac:level=9")
    req = json.loads(FL.FlacBlockCompressor().metadata_requirements())
    assert req["number_of_channels"] == ["range", 1, 8] and req["bits_per_sample"] == ["range", 8, 32]
    with pytest.raises(RuntimeError, match="requires metadata"):
        FL.FlacBlockCompressor().compress(b"\0\0", None)


def test_flac_metadata_json_is_nlohmann_dump():
    # flac.cpp:368-379 / :429-440 build nlohmann::json objects, whose dump() sorts the keys and writes no
    # spaces; the C++ facade (ricepp_facade.cpp) writes the same string
    from dwarfs_amd import flac as FL
    assert FL.FlacBlockCompressor().metadata_requirements() == (
        '{"bits_per_sample":["range",8,32],"bytes_per_sample":["range",1,4],"endianness":["set",["big","little"]],'
        '"number_of_channels":["range",1,8],"padding":["set",["msb","lsb"]],"signedness":["set",["signed","unsigned"]]}')


def _pcmaudio_fixtures():
    from pathlib import Path
    return json.loads((Path(__file__).resolve().parent / "golden" / "pcmaudio_fixtures.json").read_text())


@pytest.mark.parametrize("fx", _pcmaudio_fixtures(), ids=lambda f: f["file"].rsplit("/", 1)[1])
def test_oracle_round_trips_reference_pcm_fixtures(fx):
    """The reference's real PCM fixtures (test/pcmaudio/test{8,12,16,20,24,32}.{wav,aiff}, payload and the metadata
    the pcmaudio categorizer emits: tests/golden/make_golden.py) through the CPU restatement: samples unpacked as
    the FLAC compressor's pcm_sample_transformer would (flac.cpp:211), encoded, decoded back exactly."""
    from oracle import oracle as O
    m = fx["metadata"]
    pcm = bytes.fromhex(fx["pcm_hex"])
    x = O.pcm_unpack(pcm, m["endianness"] == "big", m["signedness"] == "signed", m["padding"] == "lsb",
                     m["bytes_per_sample"], m["bits_per_sample"])
    assert x.size == len(pcm) // m["bytes_per_sample"] == 7 * m["number_of_channels"]
    stream = F.encode(x, m["number_of_channels"], m["bits_per_sample"])
    st, y, ch, bps = F.decode(stream, x.size)
    assert st == F.OK and (ch, bps) == (m["number_of_channels"], m["bits_per_sample"])
    assert np.array_equal(y, x)
    assert O.pcm_pack(y, m["endianness"] == "big", m["signedness"] == "signed", m["padding"] == "lsb",
                      m["bytes_per_sample"], m["bits_per_sample"]) == pcm
