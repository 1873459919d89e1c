"""GPU tests of the C ABI called directly (include/ricepp_amd.h), not through
the Python codec's default ``_ws`` path:

* the plain, workspace-free ``rpp_encode_batch`` / ``rpp_decode_batch``
  (one wave per stream) with real data -- the full 4096 x 64 KiB workload, a
  16 MiB block, streams at any byte offset -- against the CPU oracle;
* the device-side workspace guard of the ``_ws`` forms: a batch larger than
  the caller promised is still coded exactly (one wave per stream), never out
  of the workspace's bounds;
* the error contract of the decode look-back: a predecessor tile that never
  publishes makes the stream ``RPP_INTERNAL_ERROR``, not wrong samples with
  ``RPP_OK`` (fault injected with ``RPP_TEST_LOOKBACK_STALL``).
"""

import ctypes as C

import numpy as np
import pytest
import torch

import datagen
from dwarfs_amd import _native as N
from dwarfs_amd import codec
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _p(t: torch.Tensor) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


def _u64(v) -> torch.Tensor:
    return torch.as_tensor(np.asarray(v, np.int64), device=DEV)


def _stream() -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ocfg(c: codec.CodecConfig):
    return O.cfg(c.block_size, c.component_stream_count, c.byteorder == "big", c.unused_lsb_count)


def plain_encode(cfg: codec.CodecConfig, flat: np.ndarray, offs, ns):
    """rpp_encode_batch (no workspace) over blocks of `flat` (stored uint16 samples)."""
    c = cfg.native()
    caps = np.array([(N.lib().rpp_worst_case_bytes(C.byref(c), int(n)) + 15) // 16 * 16 for n in ns], np.int64)
    oo = np.zeros(len(ns), np.int64)
    oo[1:] = np.cumsum(caps)[:-1]
    d_in = torch.from_numpy(flat.view(np.int16)).to(DEV)
    out = torch.zeros(int(caps.sum()) + 16, dtype=torch.uint8, device=DEV)
    sizes = torch.zeros(len(ns), dtype=torch.int64, device=DEV)
    st = torch.full((len(ns),), 99, dtype=torch.int32, device=DEV)
    d_off, d_n, d_oo = _u64(offs), _u64(ns), _u64(oo)
    r = N.lib().rpp_encode_batch(C.byref(c), _p(d_in), _p(d_off), _p(d_n), len(ns), _p(out), _p(d_oo), _p(sizes),
                                 _p(st), _stream())
    assert r == N.RPP_OK
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    return out, oo, sizes.cpu().numpy()


def plain_decode(cfg: codec.CodecConfig, data: torch.Tensor, in_offs, in_bytes, ns):
    """rpp_decode_batch (no workspace: one wave per stream)."""
    c = cfg.native()
    oo = np.zeros(len(ns), np.int64)
    oo[1:] = np.cumsum(ns)[:-1]
    out = torch.zeros(max(int(np.sum(ns)), 8), dtype=torch.int16, device=DEV)
    st = torch.full((len(ns),), 99, dtype=torch.int32, device=DEV)
    d_off, d_b, d_oo, d_n = _u64(in_offs), _u64(in_bytes), _u64(oo), _u64(ns)
    r = N.lib().rpp_decode_batch(C.byref(c), _p(data), _p(d_off), _p(d_b), len(ns), _p(out), _p(d_oo), _p(d_n),
                                 _p(st), _stream())
    assert r == N.RPP_OK
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint16), st.cpu().numpy()


def test_plain_abi_full_size_4096x64k():
    """BASELINE configs[1] through the plain ABI: 4096 x 64 KiB Poisson blocks, every stream byte-identical to
    the oracle's, decoded back exactly."""
    nb, n = 4096, 32768
    rng = np.random.default_rng(4096)
    x = datagen.poisson_data(rng, nb * n)
    cfg = codec.CodecConfig(128, 1, "big", 0)
    oc = _ocfg(cfg)
    offs = np.arange(nb, dtype=np.int64) * n
    out, oo, sizes = plain_encode(cfg, x, offs, [n] * nb)
    cap = O.worst_case_bytes(oc, n)
    ob, ooo, osz, ost = O.encode_batch(oc, x, offs.astype(np.uint64), [n] * nb, cap, nthreads=16)
    assert (ost == 0).all() and np.array_equal(sizes, osz.astype(np.int64))
    data = out.cpu().numpy()
    for i in range(nb):
        assert np.array_equal(data[oo[i]:oo[i] + sizes[i]], ob[int(ooo[i]):int(ooo[i]) + int(osz[i])]), i
    dec, st = plain_decode(cfg, out, oo, sizes, [n] * nb)
    assert (st == 0).all()
    assert np.array_equal(dec, x)


def test_plain_abi_16mib_block_one_wave():
    """A 16 MiB DwarFS block through the workspace-free forms (one wave each way), plus short blocks."""
    rng = np.random.default_rng(16)
    blocks = [datagen.poisson_data(rng, 8 << 20, lam=700.0), datagen.benchmark_data(rng, 5000),
              datagen.poisson_data(rng, 1)]
    for cs in (1, 2):
        cfg = codec.CodecConfig(128, cs, "big", 0)
        oc = _ocfg(cfg)
        bl = [b[: len(b) // cs * cs] for b in blocks]
        offs, pos = [], 0
        for b in bl:
            offs.append(pos)
            pos += (len(b) + 7) // 8 * 8
        flat = np.zeros(pos + 8, np.uint16)
        for o, b in zip(offs, bl):
            flat[o:o + len(b)] = b
        ns = [len(b) for b in bl]
        out, oo, sizes = plain_encode(cfg, flat, offs, ns)
        data = out.cpu().numpy()
        for i, b in enumerate(bl):
            assert data[oo[i]:oo[i] + sizes[i]].tobytes() == O.encode(oc, b), i
        dec, st = plain_decode(cfg, out, oo, sizes, ns)
        assert (st == 0).all()
        p = 0
        for b in bl:
            assert np.array_equal(dec[p:p + len(b)], b)
            p += len(b)


def test_plain_abi_decode_at_any_byte_offset():
    """rpp_decode_batch takes streams at any byte offset (a DwarFS payload right after its header)."""
    rng = np.random.default_rng(77)
    for bs, cs in ((128, 1), (16, 2), (29, 1), (512, 2)):
        cfg = codec.CodecConfig(bs, cs, "little", 2)
        oc = _ocfg(cfg)
        blocks = [datagen.poisson_data(rng, int(n) // cs * cs, lam=300.0, ulsb=2, big_endian=False)
                  for n in rng.integers(0, 50000, 12)]
        streams = [O.encode(oc, b) for b in blocks]
        offs, pos = [], 0
        for i, s in enumerate(streams):
            pos += 13 + (i * 5) % 6  # a 13-18 byte header before each payload
            offs.append(pos)
            pos += len(s)
        buf = np.zeros(pos + 16, np.uint8)
        for o, s in zip(offs, streams):
            buf[o:o + len(s)] = np.frombuffer(s, np.uint8)
        ns = [len(b) for b in blocks]
        dec, st = plain_decode(cfg, torch.from_numpy(buf).to(DEV), offs, [len(s) for s in streams], ns)
        assert (st == 0).all()
        p = 0
        for b in blocks:
            assert np.array_equal(dec[p:p + len(b)], b)
            p += len(b)


def _ws_decode(cfg, data, in_offs, in_bytes, ns, total_claim, max_claim, opt=None):
    c = cfg.native()
    o = (opt or codec.DecodeOptions()).native()
    oo = np.zeros(len(ns), np.int64)
    oo[1:] = np.cumsum(ns)[:-1]
    wsb = int(N.lib().rpp_decode_workspace_bytes_ex(C.byref(c), total_claim, max_claim, len(ns), C.byref(o)))
    ws = torch.zeros(max(wsb, 256), dtype=torch.uint8, device=DEV)
    out = torch.zeros(int(np.sum(ns)) + 8, dtype=torch.int16, device=DEV)
    st = torch.full((len(ns),), 99, dtype=torch.int32, device=DEV)
    d_off, d_b, d_oo, d_n = _u64(in_offs), _u64(in_bytes), _u64(oo), _u64(ns)
    r = N.lib().rpp_decode_batch_ex(C.byref(c), _p(data), _p(d_off), _p(d_b), len(ns), _p(out), _p(d_oo), _p(d_n),
                                    _p(st), total_claim, max_claim, _p(ws), wsb, C.byref(o), _stream())
    assert r == N.RPP_OK
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint16), st.cpu().numpy()


def test_workspace_guard_decode_batch_larger_than_promised():
    """rpp_decode_batch_ws sized for fewer samples than the batch holds: the device guard sends the whole
    batch to the one-wave-per-stream kernel; the output is still exact."""
    rng = np.random.default_rng(3)
    cfg = codec.CodecConfig(128, 1, "big", 0)
    oc = _ocfg(cfg)
    blocks = [datagen.poisson_data(rng, 1 << 20), datagen.poisson_data(rng, 3 << 18), datagen.poisson_data(rng, 999)]
    streams = [O.encode(oc, b) for b in blocks]
    offs, pos = [], 0
    for s in streams:
        offs.append(pos)
        pos += (len(s) + 15) // 16 * 16
    buf = np.zeros(pos + 16, np.uint8)
    for o, s in zip(offs, streams):
        buf[o:o + len(s)] = np.frombuffer(s, np.uint8)
    data = torch.from_numpy(buf).to(DEV)
    ns = [len(b) for b in blocks]
    want = np.concatenate(blocks)
    # honest claims (segmented), then understated total and understated maximum
    for total, mx in ((sum(ns), max(ns)), (sum(ns) // 3, max(ns)), (sum(ns), max(ns) // 4)):
        dec, st = _ws_decode(cfg, data, offs, [len(s) for s in streams], ns, total, mx,
                             codec.DecodeOptions(path="segmented", seg_log2=14))
        assert (st == 0).all(), (total, mx, st)
        assert np.array_equal(dec[: len(want)], want), (total, mx)


def test_workspace_guard_encode_batch_larger_than_promised():
    """rpp_encode_batch_ws sized for fewer samples than the batch holds: nothing is split, every stream is
    encoded by one wave, byte-identical to the oracle."""
    rng = np.random.default_rng(4)
    cfg = codec.CodecConfig(64, 1, "big", 0)
    c = cfg.native()
    oc = _ocfg(cfg)
    blocks = [datagen.poisson_data(rng, 64 * 256 * 5 + 17), datagen.poisson_data(rng, 64 * 256 * 3)]
    ns = [len(b) for b in blocks]
    offs = [0, (ns[0] + 7) // 8 * 8]
    flat = np.zeros(offs[1] + ns[1] + 8, np.uint16)
    flat[: ns[0]] = blocks[0]
    flat[offs[1]:offs[1] + ns[1]] = blocks[1]
    d_in = torch.from_numpy(flat.view(np.int16)).to(DEV)
    caps = [(N.lib().rpp_worst_case_bytes(C.byref(c), n) + 15) // 16 * 16 for n in ns]
    oo = [0, caps[0]]
    for total in (sum(ns), ns[1]):  # honest, then understated
        wsb = int(N.lib().rpp_encode_workspace_bytes(C.byref(c), total, max(ns), 2))
        ws = torch.zeros(max(wsb, 256), dtype=torch.uint8, device=DEV)
        out = torch.zeros(sum(caps) + 16, dtype=torch.uint8, device=DEV)
        sizes = torch.zeros(2, dtype=torch.int64, device=DEV)
        st = torch.full((2,), 99, dtype=torch.int32, device=DEV)
        d_off, d_n, d_oo = _u64(offs), _u64(ns), _u64(oo)
        r = N.lib().rpp_encode_batch_ws(C.byref(c), _p(d_in), _p(d_off), _p(d_n), 2, _p(out), _p(d_oo), _p(sizes),
                                        _p(st), total, max(ns), _p(ws), wsb, _stream())
        assert r == N.RPP_OK
        torch.cuda.synchronize()
        assert (st.cpu().numpy() == 0).all()
        data, sz = out.cpu().numpy(), sizes.cpu().numpy()
        for i, b in enumerate(blocks):
            assert data[oo[i]:oo[i] + sz[i]].tobytes() == O.encode(oc, b), (total, i)


def test_stalled_lookback_reports_internal_error():
    """RPP_TEST_LOOKBACK_STALL: tile 1 of every split stream never publishes its prefix.  Streams with more
    than two tiles (> 512 sub-blocks) must come back RPP_INTERNAL_ERROR -- not RPP_OK with wrong samples --
    while a stream with at most two tiles decodes exactly."""
    rng = np.random.default_rng(6)
    cfg = codec.CodecConfig(128, 1, "big", 0)
    oc = _ocfg(cfg)
    blocks = [datagen.poisson_data(rng, 128 * 2000), datagen.poisson_data(rng, 128 * 400),
              datagen.poisson_data(rng, 128 * 1500)]
    streams = [O.encode(oc, b) for b in blocks]
    offs, pos = [], 0
    for s in streams:
        offs.append(pos)
        pos += (len(s) + 15) // 16 * 16
    buf = np.zeros(pos + 16, np.uint8)
    for o, s in zip(offs, streams):
        buf[o:o + len(s)] = np.frombuffer(s, np.uint8)
    ns = [len(b) for b in blocks]
    dec, st = _ws_decode(cfg, torch.from_numpy(buf).to(DEV), offs, [len(s) for s in streams], ns, sum(ns), max(ns),
                         codec.DecodeOptions(path="segmented", seg_log2=12, test_flags=N.RPP_TEST_LOOKBACK_STALL))
    assert st[0] == N.RPP_INTERNAL_ERROR and st[2] == N.RPP_INTERNAL_ERROR, st
    assert st[1] == 0, st
    assert np.array_equal(dec[ns[0]:ns[0] + ns[1]], blocks[1])
    with pytest.raises(codec.CodecError, match="INTERNAL_ERROR"):
        codec._raise_status(int(st[0]))
    diag = (C.c_ulonglong * 8)()
    N.lib().rpp_diag_read(diag, 1)  # the stalled look-backs were counted; clear for later tests
    assert diag[6] > 0
    # without the fault the same call is exact
    dec, st = _ws_decode(cfg, torch.from_numpy(buf).to(DEV), offs, [len(s) for s in streams], ns, sum(ns), max(ns),
                         codec.DecodeOptions(path="segmented", seg_log2=12))
    assert (st == 0).all() and np.array_equal(dec[: sum(ns)], np.concatenate(blocks))
