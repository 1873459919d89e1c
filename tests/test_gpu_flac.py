"""FLAC block codec on the GPU (dwarfs_amd.flac over rpp_flac_encode /
rpp_flac_decode).  Parity unpinned (libFLAC absent, no FLAC fixture in the
reference): every GPU stream is decoded by the CPU restatement
(oracle/flac_oracle.c) as well as by the GPU, and the GPU decoder reads the
restatement's streams of every subframe kind.  The matrix is the reference's
own (test/flac_compressor_test.cpp:138-205: endianness x signedness x padding
x data shapes, compressed below half the input, exact round trip)."""

import json

import numpy as np
import pytest
import torch

from dwarfs_amd import flac as FL
from dwarfs_amd.pcm import PcmSampleEndianness as E, PcmSamplePadding as Pd, PcmSampleSignedness as S
from dwarfs_amd.pcm import PcmSampleTransformer
from oracle import flac as F
from test_flac import DATA_PARAMS, OPTS, sines

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def pcm_bytes(x: np.ndarray, end, sig, pad, nbytes, bits) -> bytes:
    """make_test_data (flac_compressor_test.cpp:65-81): the samples packed by pcm_sample_transformer."""
    t = PcmSampleTransformer(end, sig, pad, nbytes, bits)
    out = torch.empty(x.size * nbytes, dtype=torch.uint8, device=DEV)
    t.pack(out, torch.from_numpy(x.astype(np.int32)).to(DEV))
    return out.cpu().numpy().tobytes()


def meta(end, sig, pad, channels, nbytes, bits):
    return json.dumps({"endianness": "big" if end is E.Big else "little",
                       "signedness": "signed" if sig is S.Signed else "unsigned",
                       "padding": "msb" if pad is Pd.Msb else "lsb",
                       "bytes_per_sample": nbytes, "bits_per_sample": bits, "number_of_channels": channels})


def test_basic():
    """TEST(flac_compressor, basic) (flac_compressor_test.cpp:138-158)."""
    x = sines(2, 1000, 16)
    data = pcm_bytes(x, E.Little, S.Signed, Pd.Msb, 2, 16)
    comp = FL.block_compressor("flac").compress(data, meta(E.Little, S.Signed, Pd.Msb, 2, 2, 16))
    assert len(comp) < len(data) / 2
    assert FL.decompress(comp) == data


@pytest.mark.parametrize("channels,n,nbytes,bits", DATA_PARAMS)
@pytest.mark.parametrize("end", [E.Big, E.Little])
@pytest.mark.parametrize("sig", [S.Signed, S.Unsigned])
@pytest.mark.parametrize("pad", [Pd.Lsb, Pd.Msb])
def test_combinations(channels, n, nbytes, bits, end, sig, pad):
    """TEST_P(flac_param, combinations) (flac_compressor_test.cpp:165-196), plus the GPU stream checked by
    the CPU restatement's decoder."""
    x = sines(channels, n, bits)
    data = pcm_bytes(x, end, sig, pad, nbytes, bits)
    comp = FL.FlacBlockCompressor().compress(data, meta(end, sig, pad, channels, nbytes, bits))
    assert len(comp) < len(data) / 2
    d = FL.FlacBlockDecompressor(comp)
    assert json.loads(d.metadata()) == json.loads(meta(end, sig, pad, channels, nbytes, bits))
    assert d.decompress() == data
    # the stream itself, by an independent decoder: the samples as unpacked by the transformer
    t = PcmSampleTransformer(end, sig, pad, nbytes, bits)
    want = torch.empty(x.size, dtype=torch.int32, device=DEV)
    t.unpack(want, torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(DEV))
    st, y, ch, b = F.decode(d.stream, x.size)
    assert st == F.OK and (ch, b) == (channels, bits)
    assert np.array_equal(y, want.cpu().numpy())


@pytest.mark.parametrize("name", sorted(OPTS))
@pytest.mark.parametrize("channels,bits", [(1, 16), (2, 16), (2, 24), (3, 8), (2, 32)])
def test_gpu_decodes_every_oracle_stream(name, channels, bits):
    """The restatement's streams -- LPC up to order 32, escape partitions, 5-bit Rice parameters, partition
    orders 0-8, a PADDING block, variable blocking, verbatim and constant subframes, block sizes that need
    the 8 / 16-bit size field -- decoded by the GPU."""
    rng = np.random.default_rng(len(name) * 11 + channels + bits)
    x = sines(channels, 9000, bits).astype(np.int64)
    x += rng.integers(-3, 4, x.size)
    x[::997] = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), x[::997].size)
    x = np.clip(x, -(1 << (bits - 1)), (1 << (bits - 1)) - 1).astype(np.int32)
    nbytes = (bits + 7) // 8
    for blocksize in (4096, 1152, 200):
        stream = F.encode(x, channels, bits, blocksize, OPTS[name])
        block = FL.frame_header(x.size * nbytes, channels, bits, 0x40 | (nbytes - 1)) + stream
        want = pcm_bytes(x, E.Little, S.Signed, Pd.Msb, nbytes, bits)
        assert FL.decompress(block) == want, (name, blocksize)


def test_gpu_encoder_kinds():
    """Silence (constant subframes), low bits always zero (wasted bits), one channel constant and one not,
    a frame of white noise (verbatim), a ragged last frame -- round trip and the oracle's decode."""
    rng = np.random.default_rng(5)
    n = 3 * 4096 + 77
    x = np.zeros((n, 2), np.int64)
    x[4096:8192, 0] = sines(1, 4096, 13)[:4096].astype(np.int64) << 3  # (16-bit samples, 3 wasted bits)
    x[4096:8192, 1] = 1000
    x[8192:, 0] = rng.integers(-32768, 32768, n - 8192)
    x[8192:, 1] = rng.integers(-32768, 32768, n - 8192) & ~7
    x = x.reshape(-1).astype(np.int32)
    data = pcm_bytes(x, E.Big, S.Signed, Pd.Msb, 2, 16)
    comp = FL.FlacBlockCompressor().compress(data, meta(E.Big, S.Signed, Pd.Msb, 2, 2, 16))
    d = FL.FlacBlockDecompressor(comp)
    assert d.decompress() == data
    st, y, _, _ = F.decode(d.stream, x.size)
    assert st == F.OK
    if not np.array_equal(y, x):
        bad = np.flatnonzero(y != x)
        import os
        import subprocess
        import sys
        open("/tmp/flac_kinds.bin", "wb").write(d.stream)
        trace = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, '.'); from oracle import flac as F; "
                                "F.decode(open('/tmp/flac_kinds.bin','rb').read(), %d)" % x.size],
                               env={**os.environ, "FO_TRACE": "1"}, capture_output=True, text=True).stderr
        raise AssertionError(f"{bad.size} samples differ, first {bad[:8].tolist()}: oracle {y[bad[:8]].tolist()} "
                             f"want {x[bad[:8]].tolist()}\n{trace[:3000]}")


def ar_audio(channels, n, bits, seed=9):
    """Band-limited 'audio' a linear predictor models well and fixed predictors do not: white noise through a
    sixth-order all-pole resonator (poles at radius 0.97), per channel, scaled to `bits`."""
    from scipy.signal import lfilter
    rng = np.random.default_rng(seed)
    poles = [0.97 * np.exp(1j * w) for w in (0.07, 0.31, 0.9)]
    a = np.real(np.poly(poles + [np.conj(p) for p in poles]))
    out = np.empty((n, channels), np.int64)
    lim = (1 << (bits - 1)) - 1
    for c in range(channels):
        y = lfilter([1.0], a, rng.standard_normal(n))
        out[:, c] = np.clip(np.round(y / np.abs(y).max() * 0.8 * lim), -lim, lim)
    return out.reshape(-1).astype(np.int32)


@pytest.mark.parametrize("channels,bits", [(1, 16), (2, 16), (2, 24), (3, 12)])
def test_gpu_lpc_levels(channels, bits):
    """LPC subframes (rpp_flac_encode_ex): every level and the exhaustive search round-trip through the GPU decoder
    and the restatement's decoder; on all-pole audio LPC (level 5) codes smaller than level 2's fixed predictors,
    and the exhaustive search (every order coded) is never larger than the estimated order."""
    n = 5 * 4096 + 123
    x = ar_audio(channels, n, bits)
    nbytes = (bits + 7) // 8
    data = pcm_bytes(x, E.Little, S.Signed, Pd.Msb, nbytes, bits)
    m = meta(E.Little, S.Signed, Pd.Msb, channels, nbytes, bits)
    sizes = {}
    for level, exh in [(0, False), (2, False), (3, False), (5, False), (5, True), (8, False), (8, True)]:
        comp = FL.FlacBlockCompressor(level, exh).compress(data, m)
        d = FL.FlacBlockDecompressor(comp)
        assert d.decompress() == data, (level, exh)
        st, y, ch, b = F.decode(d.stream, x.size)
        assert st == F.OK and (ch, b) == (channels, bits), (level, exh)
        assert np.array_equal(y, x), (level, exh)
        sizes[(level, exh)] = len(comp)
    assert sizes[(5, False)] < 0.97 * sizes[(2, False)], sizes
    assert sizes[(5, True)] <= sizes[(5, False)], sizes
    assert sizes[(8, True)] <= sizes[(8, False)], sizes


@pytest.mark.parametrize("level,exh", [(5, False), (8, True), (1, False)])
def test_gpu_encode_batch_matches_single_blocks(level, exh):
    """rpp_flac_encode_batch: blocks of different shapes (channels 1-3, 8-32 bits, empty, ragged, several frames)
    in one launch give the same bytes as one rpp_flac_encode_ex per block, and decode."""
    shapes = [(2, 3 * 4096 + 5, 2, 16), (1, 100, 1, 8), (3, 4096, 3, 24), (2, 0, 2, 16), (1, 9000, 4, 32),
              (2, 4096 * 2, 2, 16), (1, 1, 2, 12)]
    rng = np.random.default_rng(level)
    comp = FL.FlacBlockCompressor(level, exh)
    items = []
    for k, (channels, n, nbytes, bits) in enumerate(shapes):
        x = ar_audio(channels, n, bits, seed=k) if n else np.zeros(0, np.int32)
        if k == 4:
            x = rng.integers(-(1 << 31), (1 << 31) - 1, n * channels).astype(np.int32)
        items.append((pcm_bytes(x, E.Big, S.Signed, Pd.Msb, nbytes, bits) if n else b"",
                      meta(E.Big, S.Signed, Pd.Msb, channels, nbytes, bits)))
    many = comp.compress_many(items)
    for (data, m), got in zip(items, many):
        assert got == comp.compress(data, m)
        assert FL.decompress(got) == data


@pytest.mark.parametrize("level", [5, 8])
def test_gpu_decode_batch_matches_single_blocks(level):
    """rpp_flac_decode_batch (FL.decompress_many): blocks of different shapes -- channels 1-3, 8-32 bits (the
    32-bit block on the lane decoder's int64 instance, the others on the wave decoder), empty, one sample,
    several frames, trailing bytes after the last frame (the serial chain walk) -- decoded in one sequence
    of launches give the samples each block gives alone."""
    shapes = [(2, 3 * 4096 + 5, 2, 16), (1, 100, 1, 8), (3, 4096, 3, 24), (2, 0, 2, 16), (1, 9000, 4, 32),
              (2, 4096 * 2, 2, 16), (1, 1, 2, 12), (4, 5000, 3, 20)]
    rng = np.random.default_rng(level + 100)
    comp = FL.FlacBlockCompressor(level)
    datas, blocks = [], []
    for k, (channels, n, nbytes, bits) in enumerate(shapes):
        x = ar_audio(channels, n, bits, seed=k + 50) if n else np.zeros(0, np.int32)
        if k == 4:
            x = rng.integers(-(1 << 31), (1 << 31) - 1, n * channels).astype(np.int32)
        data = pcm_bytes(x, E.Little, S.Signed, Pd.Msb, nbytes, bits) if n else b""
        c = comp.compress(data, meta(E.Little, S.Signed, Pd.Msb, channels, nbytes, bits))
        if k == 5:
            c += bytes(9)
        datas.append(data)
        blocks.append(c)
    many = FL.decompress_many(blocks)
    for k, (data, c, got) in enumerate(zip(datas, blocks, many)):
        assert got == data, k
        assert got == FL.decompress(c), k
    # one corrupt block in the batch fails with the single decode's error
    bad = bytearray(blocks[0])
    bad[len(bad) // 2] ^= 0x04
    with pytest.raises(RuntimeError, match="FLAC"):
        FL.decompress_many([blocks[1], bytes(bad), blocks[2]])


def test_empty_block():
    comp = FL.FlacBlockCompressor().compress(b"", meta(E.Big, S.Signed, Pd.Msb, 2, 2, 16))
    assert FL.decompress(comp) == b""


def test_corrupt_frame_is_an_error():
    x = sines(2, 20000, 16)
    data = pcm_bytes(x, E.Little, S.Signed, Pd.Msb, 2, 16)
    comp = bytearray(FL.FlacBlockCompressor().compress(data, meta(E.Little, S.Signed, Pd.Msb, 2, 2, 16)))
    comp[len(comp) // 2] ^= 0x04
    with pytest.raises(RuntimeError, match="FLAC"):
        FL.decompress(bytes(comp))
    with pytest.raises(RuntimeError, match="FLAC"):
        FL.decompress(bytes(comp[: len(comp) - 100]))


def test_trailing_bytes_after_the_last_frame():
    """Bytes after the frame holding the last sample are ignored (the decoder stops at the stream's sample
    count, as the chain walk does): the parallel link check cannot place the last frame, so the serial walk
    runs."""
    x = sines(2, 3 * 4096 + 100, 16)
    data = pcm_bytes(x, E.Little, S.Signed, Pd.Msb, 2, 16)
    comp = FL.FlacBlockCompressor().compress(data, meta(E.Little, S.Signed, Pd.Msb, 2, 2, 16))
    assert FL.decompress(comp + bytes(7)) == data
    assert FL.decompress(comp + b"\xff\xf8" + bytes(30)) == data


def _pcmaudio_fixtures():
    from pathlib import Path
    return json.loads((Path(__file__).resolve().parent / "golden" / "pcmaudio_fixtures.json").read_text())


@pytest.mark.parametrize("fx", _pcmaudio_fixtures(), ids=lambda f: f["file"].rsplit("/", 1)[1])
def test_reference_pcm_fixtures_round_trip(fx):
    """The reference's real PCM fixtures (test/pcmaudio/test{8,12,16,20,24,32}.{wav,aiff}) with the metadata the
    pcmaudio categorizer emits for them (tests/golden/pcmaudio_fixtures.json) through flac_block_compressor /
    flac_block_decompressor on the GPU: exact bytes back, the metadata carried in the block header, and the GPU's
    FLAC stream decoded by the CPU restatement to the samples the transformer unpacks.  Parity unpinned: no
    libFLAC output exists to compare the stream itself with."""
    from oracle import oracle as O
    m = fx["metadata"]
    pcm = bytes.fromhex(fx["pcm_hex"])
    comp = FL.FlacBlockCompressor().compress(pcm, json.dumps(m))
    d = FL.FlacBlockDecompressor(comp)
    assert json.loads(d.metadata()) == m
    assert d.uncompressed_size() == len(pcm)
    assert d.decompress() == pcm
    x = O.pcm_unpack(pcm, m["endianness"] == "big", m["signedness"] == "signed", m["padding"] == "lsb",
                     m["bytes_per_sample"], m["bits_per_sample"])
    st, y, ch, bps = F.decode(d.stream, x.size)
    assert st == F.OK and (ch, bps) == (m["number_of_channels"], m["bits_per_sample"])
    assert np.array_equal(y, x)
    # and the restatement's stream of the same samples decoded by the GPU
    stream = F.encode(x, m["number_of_channels"], m["bits_per_sample"])
    nb = m["bytes_per_sample"]
    flags = (FL.FLAG_BIG_ENDIAN if m["endianness"] == "big" else 0) | (FL.FLAG_SIGNED if m["signedness"] == "signed" else 0) \
        | (FL.FLAG_LSB_PADDING if m["padding"] == "lsb" else 0) | (nb - 1)
    assert FL.decompress(FL.frame_header(len(pcm), m["number_of_channels"], m["bits_per_sample"], flags) + stream) == pcm
