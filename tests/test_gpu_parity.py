"""GPU parity tests: the HIP codec (through the C ABI) against the CPU oracle.

Bar: bit-exact.  Every encoded stream must equal the oracle's bytes, every
decoded block must equal the oracle's decode of the same bytes (including
error status for truncated or corrupt input), on the same seeded inputs.
"""

import numpy as np
import pytest
import torch

import datagen
from dwarfs_amd import codec
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
GOLDEN = __import__("pathlib").Path(__file__).resolve().parent / "golden"


def ocfg(c: codec.CodecConfig):
    return O.cfg(c.block_size, c.component_stream_count, c.byteorder == "big", c.unused_lsb_count)


def seg(log2=0, **kw):
    """Decode options forcing the segmented decode (units of 2**log2 bits; 0: chosen from the batch)."""
    return codec.DecodeOptions(path="segmented", seg_log2=log2, **kw)


FUSED = codec.DecodeOptions(path="fused")


def run_batch(cfg, blocks, in_align=8, dec=None):
    """Encodes the list of stored-sample arrays on the GPU, checks every
    stream against the oracle, decodes on the GPU (decode options `dec`, or
    each of a list of them) and checks the samples."""
    oc = ocfg(cfg)
    offs, pos = [], 0
    for b in blocks:
        pos = (pos + in_align - 1) // in_align * in_align if in_align else pos
        offs.append(pos)
        pos += len(b)
    flat = np.zeros(max(pos, 1) + 8, np.uint16)
    for o, b in zip(offs, blocks):
        flat[o:o + len(b)] = b
    d = torch.from_numpy(flat.view(np.int16)).to(DEV)
    ns = [len(b) for b in blocks]
    enc = codec.encode_batch(cfg, d, offs, ns)
    torch.cuda.synchronize()
    st = enc.status.cpu().numpy()
    assert (st == 0).all(), st
    wants = [O.encode(oc, b) for b in blocks]
    sizes = enc.sizes.cpu().numpy()
    data = enc.data.cpu().numpy()
    for i, w in enumerate(wants):
        got = data[enc.offsets[i]:enc.offsets[i] + sizes[i]].tobytes()
        if got != w:
            diff = next((k for k in range(min(len(got), len(w))) if got[k] != w[k]), None)
            raise AssertionError(f"block {i} (n={ns[i]}): GPU {len(got)} B vs oracle {len(w)} B, first diff at {diff}")
    del data
    for opt in dec if isinstance(dec, list) else [dec]:
        out, dst = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, ns, options=opt)
        torch.cuda.synchronize()
        assert (dst.cpu().numpy() == 0).all(), (opt, dst)
        outn = out.cpu().numpy().view(np.uint16)
        del out
        pos = 0
        for i, b in enumerate(blocks):
            assert np.array_equal(outn[pos:pos + len(b)], b), f"decode mismatch block {i} ({opt})"
            pos += len(b)
    return wants


KIND_ORDER = ["poisson", "benchmark", "codec_test", "constant", "full_range", "ramp", "mixed", "spiky", "zeros"]


@pytest.mark.parametrize("bs", [1, 7, 8, 13, 16, 29, 32, 64, 99, 128, 200, 256, 500, 512])
@pytest.mark.parametrize("cs", [1, 2])
def test_config_matrix(bs, cs):
    rng = np.random.default_rng(1000 * bs + cs)
    for be in (True, False):
        for ulsb in (0, 4):
            blocks = []
            for ki, kind in enumerate(KIND_ORDER):
                n = int(rng.integers(1, 3 * bs * cs + 700)) // cs * cs
                blocks.append(datagen.KINDS[kind](rng, n, ulsb, be))
            blocks.append(datagen.poisson_data(rng, cs * bs * 7, ulsb=ulsb, big_endian=be))
            blocks.append(datagen.poisson_data(rng, cs, ulsb=ulsb, big_endian=be))
            run_batch(codec.CodecConfig(bs, cs, "big" if be else "little", ulsb), blocks)


@pytest.mark.parametrize("bs", [16, 32, 64, 128])
@pytest.mark.parametrize("cs", [1, 2])
@pytest.mark.parametrize("ulsb", [0, 4])
def test_rice_parameter_classes(bs, cs, ulsb):
    """Streams whose sub-blocks take every Rice parameter (fs 0-13), each
    class alone (the decoder's fs 2-4 and 5-7 fast loops, one or two codes
    per lane, and the general path) and switching class from one sub-block
    to the next (Poisson lambda varied per sub-block run)."""
    rng = np.random.default_rng(77 + 10 * cs + ulsb + bs)
    lams = [0.3, 2, 6, 20, 60, 200, 600, 2000, 6000, 20000]
    blocks = [datagen.poisson_data(rng, bs * cs * 40, lam=lam, ulsb=ulsb) for lam in lams]
    runs = [datagen.poisson_data(rng, bs * cs, lam=lams[int(rng.integers(0, len(lams)))], ulsb=ulsb)
            for _ in range(120)]
    blocks.append(np.concatenate(runs))
    run_batch(codec.CodecConfig(bs, cs, "big", ulsb), blocks)


@pytest.mark.parametrize("bs", [16, 32, 64, 128])
@pytest.mark.parametrize("cs", [1, 2])
@pytest.mark.parametrize("ulsb", [0, 3])
def test_high_rice_parameters(bs, cs, ulsb):
    """fs 8-13 (the decoder's 32-bit-segment loop with jacobi entry states):
    uniform noise of 9..14 bits (each class alone, and switching class per
    sub-block), the configs[0] generator (noise + full-range outliers: raw
    sub-blocks between Rice ones), and noisy sub-blocks whose codes overflow
    a 2048-bit window (general path between loop runs)."""
    rng = np.random.default_rng(5 + 100 * bs + 10 * cs + ulsb)
    top = 16 - ulsb

    def noise(count, bits):
        base = int(rng.integers(0, 1 << top))
        v = (base + rng.integers(0, 1 << min(bits, top), count)) & ((1 << top) - 1)
        return datagen.store(v.astype(np.uint64) << ulsb, ulsb, True)

    n = bs * cs * 40
    blocks = [noise(n, b) for b in range(9, 16)]
    blocks.append(np.concatenate([noise(bs * cs, int(rng.integers(8, 16))) for _ in range(150)]))
    blocks.append(datagen.benchmark_data(rng, n + 7 * cs, ulsb, True))
    cfg = codec.CodecConfig(bs, cs, "big", ulsb)
    run_batch(cfg, blocks)
    # the same streams split into 4 Kib / 32 Kib units (the segmented
    # decode's parse runs the same loop per unit)
    for log2 in (12, 15):
        run_batch(cfg, blocks, dec=seg(log2))


@pytest.mark.parametrize("bs", [16, 32, 64, 128])
@pytest.mark.parametrize("cs", [1, 2])
def test_low_bit_depth_fs1_fs2_mix(bs, cs):
    """configs[4]'s 10/12-bit rows: Poisson(4) samples put ~30 % of the sub-blocks at fs 1 and
    the rest at fs 2 (the fs 1-4 loop, 12 terminators per segment, with switches to and from
    the fs 2-4 loop), plus fs 0 runs (the general path) between them; fused and segmented."""
    rng = np.random.default_rng(31 + bs + cs)
    cases = []
    for ulsb in (6, 4):
        v = np.clip(rng.poisson(4.0, bs * cs * 300), 0, 0xFFFF >> ulsb).astype(np.uint64) << ulsb
        cases.append((ulsb, [datagen.store(v, ulsb, True)]))
    runs = [datagen.poisson_data(rng, bs * cs, lam=float(rng.choice([0.2, 1.0, 4.0, 12.0, 40.0])))
            for _ in range(200)]
    cases.append((0, [np.concatenate(runs)]))
    for ulsb, blocks in cases:
        cfg = codec.CodecConfig(bs, cs, "big", ulsb)
        run_batch(cfg, blocks)
        run_batch(cfg, blocks, dec=seg(12))


@pytest.mark.parametrize("ulsb", list(range(0, 16)))
def test_unused_lsb_sweep(ulsb):
    rng = np.random.default_rng(ulsb)
    blocks = [datagen.KINDS[k](rng, 3000, ulsb, True) for k in ("poisson", "benchmark", "codec_test")]
    for bs in (16, 32, 128):
        run_batch(codec.CodecConfig(bs, 1, "big", ulsb), blocks)


def test_reference_configs_and_kats():
    rng = np.random.default_rng(42)
    run_batch(codec.CodecConfig(16, 1, "big", 0), [datagen.codec_test_data(rng, 12345)])
    run_batch(codec.CodecConfig(13, 1, "big", 4), [datagen.codec_test_data(rng, 4321, 4)])
    run_batch(codec.CodecConfig(32, 1, "big", 0), [datagen.mixed_data(rng, 1500)])
    run_batch(codec.CodecConfig(29, 2, "big", 2), [datagen.codec_test_data(rng, 23456, 2)])
    # codec_test.cpp:164-172: incompressible -> exactly the worst case 29138
    wants = run_batch(codec.CodecConfig(29, 1, "big", 0), [datagen.full_range_data(rng, 14443)])
    assert len(wants[0]) == 29138
    assert codec.worst_case_encoded_bytes(codec.CodecConfig(29, 2, "big", 0), 28886) == 58275
    for cs, pixels, ulsb, bs in [(1, 1000, 0, 16), (2, 1000, 2, 32), (1, 1000, 4, 64), (2, 3333, 6, 99)]:
        run_batch(codec.CodecConfig(bs, cs, "big", ulsb), [datagen.dwarfs_test_data(rng, pixels, cs, ulsb)])


def test_unsupported_configuration():
    for bad in (codec.CodecConfig(513, 2), codec.CodecConfig(128, 3), codec.CodecConfig(0, 1)):
        with pytest.raises(RuntimeError, match="Unsupported configuration"):
            codec.create_encoder(bad)
        with pytest.raises(RuntimeError, match="Unsupported configuration"):
            codec.create_decoder(bad)


@pytest.mark.parametrize("name,cs", [("dark.fits", 1), ("test.fits", 2), ("test.fits", 1)])
def test_fits_fixtures(name, cs):
    _, x = datagen.parse_fits(GOLDEN / name)
    for bs in (16, 128, 512):
        run_batch(codec.CodecConfig(bs, cs, "big", 0), [x, x[: len(x) // 2 // cs * cs]])


def test_ragged_and_unaligned_blocks():
    rng = np.random.default_rng(5)
    cfg = codec.CodecConfig(128, 1, "big", 0)
    sizes = [0, 1, 2, 3, 127, 128, 129, 255, 256, 257, 1023, 5000]
    blocks = [datagen.poisson_data(rng, n) for n in sizes]
    run_batch(cfg, blocks, in_align=1)  # odd sample offsets: scalar load path
    run_batch(cfg, blocks, in_align=8)
    cfg2 = codec.CodecConfig(64, 2, "little", 3)
    blocks2 = [datagen.poisson_data(rng, n, lam=500, ulsb=3, big_endian=False) for n in (0, 2, 4, 126, 128, 130, 2222)]
    run_batch(cfg2, blocks2, in_align=1)


def test_api_facade_roundtrip():
    rng = np.random.default_rng(9)
    cfg = codec.CodecConfig(128, 2, "big", 2)
    x = datagen.poisson_data(rng, 10000, lam=250, ulsb=2)
    enc = codec.create_encoder(cfg)
    data = enc.encode(x)
    assert data == O.encode(ocfg(cfg), x)
    assert enc.worst_case_encoded_bytes(x.size) == O.worst_case_bytes(ocfg(cfg), x.size)
    dec = codec.create_decoder(cfg)
    assert np.array_equal(dec.decode(data, x.size), x)


def _oracle_status(oc, data, n):
    try:
        return 0, O.decode(oc, data, n)
    except O.OracleError as e:
        return e.status, None


def test_truncated_input_status_matches_oracle(dec=None):
    rng = np.random.default_rng(11)
    cfg = codec.CodecConfig(128, 1, "big", 0)
    oc = ocfg(cfg)
    x = datagen.poisson_data(rng, 3000)
    full = O.encode(oc, x)
    cuts = sorted(set([0, 1, 2, 3, 4, 8, 9, 100, len(full) // 2] + list(range(len(full) - 20, len(full) + 1))))
    streams = [full[:c] for c in cuts]
    offs = np.zeros(len(streams), np.int64)
    buf = bytearray()
    for i, s in enumerate(streams):
        offs[i] = len(buf)
        buf += s + bytes((-len(s)) % 16 + 16)
    d = torch.from_numpy(np.frombuffer(bytes(buf), np.uint8).copy()).to(DEV)
    out, st = codec.decode_batch(cfg, d, offs, [len(s) for s in streams], [x.size] * len(streams), options=dec)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    outn = out.cpu().numpy().view(np.uint16)
    for i, s in enumerate(streams):
        want_st, want = _oracle_status(oc, s, x.size)
        assert st[i] == want_st, (cuts[i], st[i], want_st)
        if want_st == 0:
            assert np.array_equal(outn[i * x.size:(i + 1) * x.size], want)


@pytest.mark.parametrize("bs,cs", [(128, 1), (16, 2), (29, 1)])
def test_corrupt_streams_match_oracle(bs, cs, dec=None):
    """Random bytes decode to whatever the reference decodes them to (or fail
    the same way): the decoder follows the reference bit for bit."""
    rng = np.random.default_rng(bs + cs)
    cfg = codec.CodecConfig(bs, cs, "big", 1)
    oc = ocfg(cfg)
    nstreams, n = 64, 256 * cs
    streams = []
    for i in range(nstreams):
        ln = int(rng.integers(4, 900))
        raw = rng.integers(0, 256, ln, dtype=np.uint8)
        if i % 3 == 0:  # sparse ones -> long unary runs
            raw &= rng.integers(0, 256, ln, dtype=np.uint8) & rng.integers(0, 256, ln, dtype=np.uint8)
        streams.append(raw.tobytes())
    offs = np.zeros(nstreams, np.int64)
    buf = bytearray()
    for i, s in enumerate(streams):
        offs[i] = len(buf)
        buf += s + bytes((-len(s)) % 16 + 16)
    d = torch.from_numpy(np.frombuffer(bytes(buf), np.uint8).copy()).to(DEV)
    out, st = codec.decode_batch(cfg, d, offs, [len(s) for s in streams], [n] * nstreams, options=dec)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    outn = out.cpu().numpy().view(np.uint16)
    for i, s in enumerate(streams):
        want_st, want = _oracle_status(oc, s, n)
        assert st[i] == want_st, (i, st[i], want_st)
        if want_st == 0:
            assert np.array_equal(outn[i * n:(i + 1) * n], want), i


def _full_size(kind, nblocks=4096, n=32768, bs=128, cs=1, nthreads=8, dec=None, byteorder="big", ulsb=0):
    rng = np.random.default_rng(42)
    if kind == "poisson":
        x = datagen.poisson_data(rng, nblocks * n)
    else:
        x = datagen.benchmark_data(rng, nblocks * n)
    if ulsb:  # unused low bits are zero in the pixel values (ricepp_cpuspecific_traits.h:63-67), else no round trip
        keep = np.uint16((0xFFFF << ulsb) & 0xFFFF)
        x = x & (keep.byteswap() if byteorder == "big" else keep)
    cfg = codec.CodecConfig(bs, cs, byteorder, ulsb)
    oc = ocfg(cfg)
    offs = np.arange(nblocks, dtype=np.int64) * n
    d = torch.from_numpy(x.view(np.int16)).to(DEV)
    enc = codec.encode_batch(cfg, d, offs, [n] * nblocks)
    torch.cuda.synchronize()
    assert (enc.status.cpu().numpy() == 0).all()
    cap = O.worst_case_bytes(oc, n)
    ob, oo, osz, ost = O.encode_batch(oc, x, offs.astype(np.uint64), [n] * nblocks, cap, nthreads=nthreads)
    assert (ost == 0).all()
    sizes = enc.sizes.cpu().numpy()
    assert np.array_equal(sizes, osz.astype(np.int64)), "encoded sizes differ from oracle"
    data = enc.data.cpu().numpy()
    for i in range(nblocks):
        a = data[enc.offsets[i]:enc.offsets[i] + sizes[i]]
        b = ob[int(oo[i]):int(oo[i]) + int(osz[i])]
        assert np.array_equal(a, b), f"block {i} differs"
    out, st = codec.decode_batch(cfg, enc.data, enc.offsets, enc.sizes, [n] * nblocks, options=dec)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert torch.equal(out[: nblocks * n], d), "round trip mismatch"


def test_full_size_4096x64k_poisson_bit_exact():
    _full_size("poisson")


def test_full_size_4096x64k_benchmark_generator_bit_exact():
    _full_size("benchmark")


def test_full_size_4096x64k_generator_two_streams_bit_exact():
    """Two component streams (bs 128 cs 2) on high-entropy data: the launch that runs several encode waves per SIMD
    and takes the emission slow path in almost every group: the round-5 build corrupted most streams here, a 64-bit
    shift taking its amount from the kernel's last allocated VGPR (DESIGN.md section 4 "64-bit shifts and the last
    VGPR")."""
    _full_size("benchmark", cs=2)


@pytest.mark.parametrize("kind", ["poisson", "benchmark"])
@pytest.mark.parametrize("cs", [1, 2])
@pytest.mark.parametrize("bs", [16, 32, 64, 256, 512])
def test_at_scale_block_sizes(bs, cs, kind):
    """2048 x 64 KiB blocks (eight encode waves per CU, the occupancy at which the bs 128 cs 2 emission branch once
    went wrong) for every other block size, both component counts, low and high entropy: bit-exact encode against the
    oracle and decode round trip."""
    _full_size(kind, nblocks=2048, bs=bs, cs=cs)


@pytest.mark.parametrize("kind", ["poisson", "benchmark"])
@pytest.mark.parametrize("cs", [1, 2])
@pytest.mark.parametrize("bs", [16, 64, 256])
def test_at_scale_long_streams(bs, cs, kind):
    """64 x 1 MiB blocks (bs 256: 16 x 4 MiB, the length from which it splits streams): long streams, so the
    segmented encode (units of chunks, concat) and the segmented decode (guess, unit parse, stitch, extraction) run
    at several block sizes and both component counts; the decode is checked to have taken the segmented path."""
    codec.segmented_decode_stats(reset=True)
    if bs > 128:
        _full_size(kind, nblocks=16, n=1 << 21, bs=bs, cs=cs)
    else:
        _full_size(kind, nblocks=64, n=1 << 19, bs=bs, cs=cs)
    assert codec.segmented_decode_stats(reset=True)["met"] > 0


@pytest.mark.parametrize("bs,cs,byteorder,ulsb", [(128, 2, "little", 0), (128, 2, "big", 3), (64, 2, "little", 2)])
def test_at_scale_byteorder_lsb(bs, cs, byteorder, ulsb):
    _full_size("benchmark", nblocks=2048, bs=bs, cs=cs, byteorder=byteorder, ulsb=ulsb)


@pytest.mark.parametrize("mib", [1, 4, 16])
def test_large_blocks(mib):
    rng = np.random.default_rng(mib)
    n = mib * (1 << 20) // 2
    blocks = [datagen.poisson_data(rng, n), datagen.benchmark_data(rng, n // 2)]
    run_batch(codec.CodecConfig(128, 1, "big", 0), blocks)
    run_batch(codec.CodecConfig(128, 2, "big", 0), [blocks[0]])


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 1000, 4096, 4097, 12289, 100000])
def test_image_offsets_scan(n):
    """rpp_exclusive_scan_u64 (image offsets of appended blocks) against numpy,
    across one and several 4096-entry passes and ragged tails."""
    from dwarfs_amd import parallel
    rng = np.random.default_rng(n)
    sizes = rng.integers(0, 1 << 40, n, dtype=np.int64) if n != 1000 else rng.integers(0, 200000, n, dtype=np.int64)
    d = torch.as_tensor(sizes, device=DEV)
    got = parallel.global_offsets(d)
    torch.cuda.synchronize()
    want = np.zeros(n, np.int64)
    if n > 1:
        want[1:] = np.cumsum(sizes)[:-1]
    assert np.array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("cs", [1, 2])
def test_configs3_block_mix_in_one_launch(cs):
    """BASELINE configs[3]: a shuffled mix of 1, 4 and 16 MiB Poisson blocks (the mkdwarfs block sizes)
    encoded in ONE rpp_encode_batch and decoded in ONE rpp_decode_batch, every stream byte-identical to
    the oracle's and every block restored."""
    rng = np.random.default_rng(300 + cs)
    sizes_mib = [1, 16, 1, 4, 1, 4, 1]
    rng.shuffle(sizes_mib)
    blocks = [datagen.poisson_data(rng, m * (1 << 19), lam=float(rng.integers(200, 3000))) for m in sizes_mib]
    run_batch(codec.CodecConfig(128, cs, "big", 0), blocks)


def _decode_oracle_streams(cfg, blocks, ragged=False, dec=None):
    """Decode-only (BASELINE configs[2]): streams produced by the CPU oracle, decoded on the GPU.
    ragged: streams start at arbitrary byte offsets (a DwarFS payload follows a 13-18 byte header)."""
    oc = ocfg(cfg)
    streams = [O.encode(oc, b) for b in blocks]
    offs, pos = [], 0
    for i, s in enumerate(streams):
        if ragged:
            pos += 1 + (7 * i) % 15
        offs.append(pos)
        pos += len(s) if ragged else (len(s) + 15) // 16 * 16
    buf = np.zeros(pos + 16, np.uint8)
    for o, s in zip(offs, streams):
        buf[o:o + len(s)] = np.frombuffer(s, np.uint8)
    d = torch.from_numpy(buf).to(DEV)
    ns = [len(b) for b in blocks]
    out, st = codec.decode_batch(cfg, d, offs, [len(s) for s in streams], ns, options=dec)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    outn = out.cpu().numpy().view(np.uint16)
    p = 0
    for i, b in enumerate(blocks):
        assert np.array_equal(outn[p:p + len(b)], b), f"block {i}"
        p += len(b)


def test_decode_oracle_encoded_1mib_blocks():
    """configs[2] as DwarFS stores frames with -S 20: 4096x4096 uint16 frames cut into 1 MiB blocks, the
    streams encoded by the CPU oracle (per-frame seed 42+i), decoded on the GPU."""
    blocks = []
    for i in range(2):
        frame = datagen.poisson_data(np.random.default_rng(42 + i), 4096 * 4096)
        blocks += [frame[k:k + (1 << 19)] for k in range(0, len(frame), 1 << 19)][:12]
    _decode_oracle_streams(codec.CodecConfig(128, 1, "big", 0), blocks)


def test_decode_oracle_encoded_32mib_frame():
    """configs[2] with one stream per frame: a whole 4096x4096 frame (32 MiB) encoded by the CPU oracle."""
    frame = datagen.poisson_data(np.random.default_rng(42), 4096 * 4096)
    _decode_oracle_streams(codec.CodecConfig(128, 1, "big", 0), [frame])


# ---- the lane-per-sub-block extraction (the second half of the segmented decode) on every stream ----

@pytest.mark.parametrize("bs", [16, 32, 64, 128])
@pytest.mark.parametrize("cs", [1, 2])
@pytest.mark.parametrize("general", [False, True])
def test_extraction_config_matrix(bs, cs, general):
    """Every stream longer than 1 Kib split (segmented, 2**10-bit units), so nearly every sub-block of every
    data kind goes through the extraction kernel; general=True sends every lane down its exact runtime-loop
    path (RPP_TEST_NO_FAST_LANES) instead of the unrolled fast lanes."""
    rng = np.random.default_rng(7000 + bs + cs)
    dec = seg(10, test_flags=codec.N.RPP_TEST_NO_FAST_LANES if general else 0)
    for be, ulsb in ((True, 0), (False, 3)):
        cfg = codec.CodecConfig(bs, cs, "big" if be else "little", ulsb)
        sizes = rng.integers(1, 6000, 7)
        blocks = _kind_blocks(rng, sizes, cs, ulsb, be)
        run_batch(cfg, blocks, dec=dec)
        _decode_oracle_streams(cfg, blocks, dec=dec)


def test_segmented_decode_long_streams_and_mix():
    rng = np.random.default_rng(77)
    blocks = [datagen.poisson_data(rng, m * (1 << 19)) for m in (1, 4, 1)] + [datagen.benchmark_data(rng, 300000)]
    run_batch(codec.CodecConfig(128, 1, "big", 0), blocks, dec=seg(14))
    run_batch(codec.CodecConfig(128, 2, "big", 0), blocks[:2], dec=seg(14))


@pytest.mark.parametrize("path", ["auto", "segmented"])
def test_decode_streams_at_any_byte_offset(path):
    """Decode takes streams at any byte offset (no repack of DwarFS payloads): the fused kernel (auto on
    these short streams) and the segmented decode with 1 Kib units."""
    rng = np.random.default_rng(99)
    dec = seg(10) if path == "segmented" else None
    for bs, cs in ((128, 1), (16, 2), (29, 1), (64, 2)):
        blocks = [datagen.poisson_data(rng, int(n) // cs * cs) for n in rng.integers(0, 40000, 9)]
        blocks += [datagen.benchmark_data(rng, 3000 // cs * cs), datagen.full_range_data(rng, 1000 // cs * cs)]
        _decode_oracle_streams(codec.CodecConfig(bs, cs, "big", 0), blocks, ragged=True, dec=dec)


@pytest.mark.parametrize("bs,cs", [(128, 1), (16, 1), (32, 2), (13, 2), (512, 1)])
def test_segmented_encode_of_long_streams(bs, cs):
    """rpp_encode_batch_ws splits long streams into segments encoded by separate waves and then places
    their bits; the result must be the oracle's stream byte for byte, at every segment count and tail
    shape.  Units are 256 chunks when the batch fills the GPU with them, else smaller powers of two down
    to 16 (these batches: 16), so the sizes below -- multiples of 256 chunks plus a chunk, a sample, a
    ragged chunk -- give one-chunk and one-sample last units, and the data makes raw / zero / Rice
    sub-blocks."""
    rng = np.random.default_rng(bs * 10 + cs)
    seg = 256 * bs * cs
    sizes = [seg, seg + bs * cs, seg + cs, 2 * seg + 5 * cs, 3 * seg - cs, 5 * seg + 7 * cs]
    blocks = []
    for i, n in enumerate(sizes):
        kind = i % 4
        if kind == 0:
            blocks.append(datagen.poisson_data(rng, n))
        elif kind == 1:
            blocks.append(datagen.mixed_data(rng, n))
        elif kind == 2:
            blocks.append(datagen.full_range_data(rng, n))
        else:
            blocks.append(datagen.benchmark_data(rng, n))
    blocks.append(datagen.constant_data(2 * seg + cs))
    run_batch(codec.CodecConfig(bs, cs, "big", 0), blocks)
    run_batch(codec.CodecConfig(bs, cs, "little", 2), [datagen.poisson_data(rng, 2 * seg + 3 * cs, lam=300,
                                                                             ulsb=2, big_endian=False)])


# ---- the segmented decode of long streams (units parsed from guessed headers, stitched exactly) ----

def _kind_blocks(rng, sizes, cs, ulsb=0, be=True):
    kinds = ("poisson", "benchmark", "mixed", "full_range", "constant", "spiky", "codec_test", "zeros")
    blocks = []
    for i, n in enumerate(sizes):
        n = int(n) // cs * cs
        k = kinds[i % len(kinds)]
        if k == "poisson":
            blocks.append(datagen.poisson_data(rng, n, ulsb=ulsb, big_endian=be))
        elif k == "benchmark":
            blocks.append(datagen.benchmark_data(rng, n, ulsb=ulsb, big_endian=be))
        elif k == "mixed":
            blocks.append(datagen.mixed_data(rng, n, ulsb=ulsb, big_endian=be))
        elif k == "full_range":
            blocks.append(datagen.full_range_data(rng, n, ulsb=ulsb, big_endian=be))
        elif k == "constant":
            blocks.append(datagen.constant_data(n, ulsb=ulsb, big_endian=be))
        elif k == "spiky":
            blocks.append(datagen.spiky_data(rng, n, ulsb=ulsb, big_endian=be))
        elif k == "codec_test":
            blocks.append(datagen.codec_test_data(rng, n, ulsb=ulsb, big_endian=be))
        else:
            blocks.append(np.zeros(n, np.uint16))
    return blocks


@pytest.mark.parametrize("bs", [16, 32, 64, 128])
@pytest.mark.parametrize("cs", [1, 2])
@pytest.mark.parametrize("seg_log2", [10, 13, 16])
def test_segmented_decode_config_matrix(bs, cs, seg_log2):
    """Every stream split into units of 2^seg_log2 bits (1 Kib units make most guesses fail and exercise the
    rerun and serial passes; 64 Kib units mostly stitch at once): the decode must be the oracle's, for every
    data kind, byte order, unused-LSB count, ragged last chunk and stream byte offset."""
    rng = np.random.default_rng(9000 + 100 * seg_log2 + bs + cs)
    sizes = [rng.integers(1, 400) * cs, 40000, 70001, 123457, 5000, 31, 65536 + 3, 90000, 200000]
    codec.segmented_decode_stats(reset=True)
    diag = (__import__("ctypes").c_ulonglong * 8)()
    __import__("dwarfs_amd._native", fromlist=["lib"]).lib().rpp_diag_read(diag, 1)  # (clear earlier tests' counts)
    for be, ulsb in ((True, 0), (False, 3)):
        cfg = codec.CodecConfig(bs, cs, "big" if be else "little", ulsb)
        blocks = _kind_blocks(rng, sizes, cs, ulsb, be)
        run_batch(cfg, blocks, dec=seg(seg_log2))
        _decode_oracle_streams(cfg, blocks, ragged=True, dec=seg(seg_log2))
    stats = codec.segmented_decode_stats(reset=True)
    assert stats["met"] > 0, stats  # the units were split and stitched
    __import__("dwarfs_amd._native", fromlist=["lib"]).lib().rpp_diag_read(diag, 1)
    assert diag[6] == 0, "an extraction tile waited for a predecessor that never published"
    if seg_log2 == 10:
        assert stats["reruns"] + stats["serial"] > 0, stats


def test_segmented_decode_errors_match_oracle():
    """Truncated and corrupt streams, split into 1 Kib units: the status and the output are the oracle's
    (a corrupt chain that runs past the region a stream's sample count allows is decoded by the fused kernel)."""
    for log2 in (10, 12):
        test_truncated_input_status_matches_oracle(dec=seg(log2))
        for bs, cs in ((128, 1), (16, 2)):
            test_corrupt_streams_match_oracle(bs, cs, dec=seg(log2))


def test_segmented_decode_is_chosen_for_long_streams():
    """Default mode: a batch whose longest stream dominates (one 16 MiB generator block, a 4 MiB Poisson
    block and small ones) takes the segmented decode; the result is the oracle's, the same as with the fused
    kernel forced."""
    rng = np.random.default_rng(4242)
    blocks = [datagen.benchmark_data(rng, 8 << 20), datagen.poisson_data(rng, 2 << 20)]
    blocks += [datagen.poisson_data(rng, int(n)) for n in rng.integers(1, 40000, 5)]
    cfg = codec.CodecConfig(128, 1, "big", 0)
    codec.segmented_decode_stats(reset=True)
    run_batch(cfg, blocks)
    stats = codec.segmented_decode_stats(reset=True)
    assert stats["met"] > 0 and stats["fallback"] == 0, stats
    _decode_oracle_streams(cfg, blocks[1:3], dec=FUSED)


def test_segmented_decode_of_a_64mib_stream():
    """The longest stream of the suite: 32 Mi samples (64 MiB) in one stream, cs 2, little endian, ulsb 1 --
    segmented encode and decode against the oracle byte for byte."""
    rng = np.random.default_rng(6464)
    x = datagen.poisson_data(rng, 32 << 20, lam=700.0, ulsb=1, big_endian=False)
    codec.segmented_decode_stats(reset=True)
    run_batch(codec.CodecConfig(128, 2, "little", 1), [x])
    assert codec.segmented_decode_stats(reset=True)["met"] > 0


@pytest.mark.parametrize("cs", [1, 2])
def test_segmented_decode_many_tiles(cs):
    """A batch of >= 2048 extraction tiles (8 x 16 MiB streams at bs 128: 2048 tiles of 256 sub-blocks) takes
    the extraction kernel with the 48 KiB stage (three workgroups per CU): Poisson streams of three densities
    (one tile per window) and a generator stream (14 bits per sample: lanes past the stage read the stream
    from memory), with 1 MiB blocks between them -- encoded byte for byte as the oracle and decoded back."""
    rng = np.random.default_rng(4848 + cs)
    n16 = (8 << 20) // cs * cs
    blocks = [datagen.poisson_data(rng, n16, lam=float(lam)) for lam in (300, 1000, 3000, 1000, 300, 3000, 1000)]
    blocks.insert(3, datagen.benchmark_data(rng, n16))
    blocks += [datagen.poisson_data(rng, (1 << 19) // cs * cs) for _ in range(3)]
    codec.segmented_decode_stats(reset=True)
    run_batch(codec.CodecConfig(128, cs, "big", 0), blocks)
    assert codec.segmented_decode_stats(reset=True)["met"] > 0


@pytest.mark.parametrize("cs", [1, 2])
def test_stream_longer_than_2_27_samples(cs):
    """One stream of 2**27 + 5 samples (cs 1; 2**27 + 6 for cs 2) with short blocks beside it: past the
    one-wave encode's 2**27-sample range and, with the generator's ~14 bits per sample, past 2**30 bits, where
    the fused decode rebases its bit positions. Encoded on the GPU byte for byte as the oracle
    (ricepp/ricepp_cpu.cpp encode), decoded back to the input by the default mode, the segmented decode
    (since round 5 it takes any stream compressed below 2**29 bytes: here it does, by units) and the fused
    kernel."""
    rng = np.random.default_rng(2727 + cs)
    n = (1 << 27) + (5 if cs == 1 else 6)
    big = datagen.benchmark_data(rng, n) if cs == 1 else datagen.poisson_data(rng, n, lam=3000.0)
    blocks = [datagen.poisson_data(rng, 4096 * cs), big, datagen.poisson_data(rng, 777 * cs)]
    cfg = codec.CodecConfig(128, cs, "big", 0)
    codec.segmented_decode_stats(reset=True)
    run_batch(cfg, blocks, dec=[None, seg(), FUSED])
    st = codec.segmented_decode_stats(reset=True)
    assert st["met"] > 0 and st["fallback"] == 0, st


def _chunked(gen, rng, n, parts=16, **kw):
    step = (n + parts - 1) // parts
    return np.concatenate([gen(rng, min(step, n - i), **kw) for i in range(0, n, step)])


def test_stream_of_2_29_samples_past_2_32_bits():
    """one stream of 2**29 + 3 samples of the benchmark generator (~14 bits per sample, 7.5e9
    bits: past 2**32, with the segmented encode's 64-bit unit offsets near their largest), encoded byte for
    byte as the oracle and decoded back by the default path -- since round 6 the segmented decode, whose
    units work in frames of their own and whose sub-block positions are 64-bit (checked to have run: units
    met, no stream handed to the fused kernel) -- and by the fused kernel, which rebases its 32-bit
    positions seven times."""
    rng = np.random.default_rng(2929)
    n = (1 << 29) + 3
    big = _chunked(datagen.benchmark_data, rng, n)
    cfg = codec.CodecConfig(128, 1, "big", 0)
    codec.segmented_decode_stats(reset=True)
    wants = run_batch(cfg, [big], dec=[None, FUSED])
    st = codec.segmented_decode_stats(reset=True)
    assert 8 * len(wants[0]) > (1 << 32)
    assert st["met"] > 0 and st["fallback"] == 0, st


@pytest.mark.parametrize("bs", [17, 99, 200, 256, 512])
@pytest.mark.parametrize("cs", [1, 2])
def test_segmented_decode_other_block_sizes(bs, cs):
    """The segmented decode for block sizes without unrolled fast lanes (256, 512 and sizes that are not a
    power of two, all allowed by ricepp:block_size, src/compression/ricepp.cpp:284-286): the units parse
    them, the extraction decodes them with its exact general lanes; every data kind, both byte orders."""
    rng = np.random.default_rng(31000 + bs + cs)
    sizes = [rng.integers(1, 400) * cs, 40000, 70001, 123457, 5000, 65536 + 3, 200000]
    codec.segmented_decode_stats(reset=True)
    for be, ulsb in ((True, 0), (False, 2)):
        cfg = codec.CodecConfig(bs, cs, "big" if be else "little", ulsb)
        blocks = _kind_blocks(rng, sizes, cs, ulsb, be)
        for log2 in (12, 15):
            run_batch(cfg, blocks, dec=seg(log2))
        _decode_oracle_streams(cfg, blocks, ragged=True, dec=seg(13))
    assert codec.segmented_decode_stats(reset=True)["met"] > 0


def test_segmented_decode_default_16mib_bs512_block():
    """A 16 MiB DwarFS block written with ricepp:block_size=512 is decoded segmented by default (not by one
    wave), bit-exact, in a batch with short blocks."""
    rng = np.random.default_rng(512)
    blocks = [datagen.poisson_data(rng, 8 << 20, lam=900.0)] + [datagen.poisson_data(rng, int(n))
                                                               for n in rng.integers(1, 30000, 4)]
    codec.segmented_decode_stats(reset=True)
    run_batch(codec.CodecConfig(512, 1, "big", 0), blocks)
    st = codec.segmented_decode_stats(reset=True)
    assert st["met"] > 0 and st["fallback"] == 0, st


# ---- bs 16 / 32: four streams per wave (rpp_decode_rows_kernel), the rest by the fused kernel ----

@pytest.mark.parametrize("bs", [16, 32])
@pytest.mark.parametrize("cs", [1, 2])
@pytest.mark.parametrize("be,ulsb", [(True, 0), (False, 3), (True, 6)])
def test_rows_decode_matches_oracle(bs, cs, be, ulsb):
    """The default (auto) decode of bs 16 / 32 batches runs the four-streams-per-wave kernel and hands every
    stream it cannot take (raw, fs 0 or >= 8, a sub-block past its 384-bit window, odd arguments) to the
    fused kernel: every stream must decode to the oracle's samples whichever kernel took it, and mixing
    both kinds in one wave (rows of one wave: consecutive streams) must not disturb either.  Sizes: ragged
    last chunks, zero- and one-chunk streams, more than 16 streams (several workgroups), byte offsets."""
    rng = np.random.default_rng(3000 + 10 * bs + cs + ulsb)
    sizes = [0, cs, bs * cs, bs * cs + cs, 3 * bs * cs - cs] + [int(x) * cs for x in rng.integers(1, 6000, 27)]
    cfg = codec.CodecConfig(bs, cs, "big" if be else "little", ulsb)
    blocks = _kind_blocks(rng, sizes, cs, ulsb, be)
    run_batch(cfg, blocks)
    _decode_oracle_streams(cfg, blocks, ragged=True)
    # a wave of four Poisson streams at every bit depth the configs[4] sweep uses (fs 1..7: the rows path)
    for lam in (4.0, 60.0, 250.0, 1000.0):
        run_batch(cfg, [datagen.poisson_data(rng, 32768 // cs * cs, lam=lam, ulsb=ulsb, big_endian=be)
                        for _ in range(20)])


def test_rows_decode_truncated_and_corrupt_streams():
    """Truncated and corrupt bs 16 / 32 streams through the default decode: the status and the samples must be
    the oracle's (the rows kernel hands such streams to the fused kernel, which owns the error contract)."""
    rng = np.random.default_rng(77)
    for bs in (16, 32):
        cfg = codec.CodecConfig(bs, 1, "big", 0)
        oc = ocfg(cfg)
        blocks = [datagen.poisson_data(rng, 5000) for _ in range(12)]
        streams = [O.encode(oc, b) for b in blocks]
        streams = [s[: len(s) * (i % 4 + 1) // 5] if i % 3 == 0 else s for i, s in enumerate(streams)]
        streams[4] = rng.integers(0, 256, len(streams[4]), dtype=np.uint8).tobytes()
        offs, pos = [], 0
        for s in streams:
            offs.append(pos)
            pos += (len(s) + 15) // 16 * 16
        buf = np.zeros(pos + 16, np.uint8)
        for o, s in zip(offs, streams):
            buf[o:o + len(s)] = np.frombuffer(s, np.uint8)
        ns = [len(b) for b in blocks]
        out, st = codec.decode_batch(cfg, torch.from_numpy(buf).to(DEV), offs, [len(s) for s in streams], ns)
        torch.cuda.synchronize()
        st, outn = st.cpu().numpy(), out.cpu().numpy().view(np.uint16)
        p = 0
        for i, s in enumerate(streams):
            want_st, want = _oracle_status(oc, s, ns[i])
            assert int(st[i]) == want_st, (bs, i, st[i], want_st)
            if want_st == 0:
                assert np.array_equal(outn[p:p + ns[i]], want), (bs, i)
            p += ns[i]
