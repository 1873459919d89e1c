"""CPU tests of the C-ABI boundary (no GPU needed): the library loads, exports
every symbol include/ricepp_amd.h declares, and its host-side entry points
(config check, worst-case size, DwarFS framing) agree with the oracle."""

import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from dwarfs_amd import _native as N
from dwarfs_amd import block_codec, codec
from oracle import oracle as O

ROOT = Path(__file__).resolve().parent.parent


def header_functions():
    text = (ROOT / "include" / "ricepp_amd.h").read_text()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(rpp_\w+)\s*\(", text, re.M)))


def test_header_symbols_exported():
    L = N.lib()
    declared = header_functions()
    assert set(declared) == set(N.EXPORTED_SYMBOLS)
    for name in declared:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True).stdout
    for name in declared:
        assert re.search(rf"\bT {name}$", out, re.M), name


def test_abi_version():
    assert N.lib().rpp_abi_version() == 1


@pytest.mark.parametrize("bs", [0, 1, 13, 128, 512, 513])
@pytest.mark.parametrize("cs", [0, 1, 2, 3])
@pytest.mark.parametrize("ulsb", [0, 8, 15, 16])
def test_check_config_and_worst_case_match_oracle(bs, cs, ulsb):
    c = N.RppConfig(bs, cs, 1, ulsb)
    oc = O.cfg(bs, cs, True, ulsb)
    st = N.lib().rpp_check_config(C.byref(c))
    assert st == O.lib().rpo_check_config(C.byref(oc))
    if st == 0:
        for n in (0, cs, 14443 // cs * cs, 32768, 8 * 1024 * 1024):
            assert N.lib().rpp_worst_case_bytes(C.byref(c), n) == O.worst_case_bytes(oc, n)


def test_unsupported_config_maps_to_runtime_error():
    with pytest.raises(RuntimeError, match="^Unsupported configuration$"):
        codec.create_encoder(codec.CodecConfig(513, 2))
    with pytest.raises(RuntimeError, match="^Unsupported configuration$"):
        codec.create_decoder(codec.CodecConfig(128, 3))


def test_empty_batch_is_ok_without_gpu():
    c = N.RppConfig(128, 1, 1, 0)
    null = C.c_void_p(0)
    assert N.lib().rpp_encode_batch(C.byref(c), null, null, null, 0, null, null, null, null, null) == 0
    assert N.lib().rpp_decode_batch(C.byref(c), null, null, null, 0, null, null, null, null, null) == 0
    bad = N.RppConfig(1000, 1, 1, 0)
    assert N.lib().rpp_encode_batch(C.byref(bad), null, null, null, 5, null, null, null, null, null) == -1


def test_decode_options_validated_without_gpu():
    """rpp_decode_batch_ex: a NULL or zeroed options struct is rpp_decode_batch_ws; out-of-range options are
    RPP_INVALID_ARGUMENT before anything is launched; the workspace size follows the forced path."""
    c = N.RppConfig(128, 1, 1, 0)
    null = C.c_void_p(0)
    L = N.lib()

    def call(o):
        return L.rpp_decode_batch_ex(C.byref(c), null, null, null, 0, null, null, null, null, 0, 0, null, 0,
                                     C.byref(o) if o is not None else None, null)

    assert call(None) == N.RPP_OK
    assert call(N.RppDecodeOptions(0, 0, 0, 0)) == N.RPP_OK
    assert call(N.RppDecodeOptions(3, 0, 0, 0)) == N.RPP_INVALID_ARGUMENT
    assert call(N.RppDecodeOptions(2, 9, 0, 0)) == N.RPP_INVALID_ARGUMENT
    assert call(N.RppDecodeOptions(2, 27, 0, 0)) == N.RPP_INVALID_ARGUMENT
    assert call(N.RppDecodeOptions(1, 0, 17, 0)) == N.RPP_INVALID_ARGUMENT

    def ws(o, total, mx, nb):
        return L.rpp_decode_workspace_bytes_ex(C.byref(c), total, mx, nb, C.byref(o) if o is not None else None)

    # 4096 x 64 KiB: one wave per stream by default, no workspace
    assert ws(None, 4096 * 32768, 32768, 4096) == 0 == L.rpp_decode_workspace_bytes(C.byref(c), 4096 * 32768, 32768, 4096)
    assert ws(N.RppDecodeOptions(2, 12, 0, 0), 4096 * 32768, 32768, 4096) > 0
    # one 16 MiB block: segmented by default, never when fused is forced
    assert ws(None, 1 << 23, 1 << 23, 1) > 0
    assert ws(N.RppDecodeOptions(1, 0, 0, 0), 1 << 23, 1 << 23, 1) == 0


@pytest.mark.parametrize("size,bs,cs,ulsb,be", [(65536, 128, 1, 0, True), (65536, 128, 1, 0, False),
                                               (0, 16, 2, 8, True), (2**40 + 3, 512, 2, 6, False)])
def test_frame_header_matches_oracle_and_roundtrips(size, bs, cs, ulsb, be):
    mine = block_codec.frame_header(size, bs, cs, 2, ulsb, be)
    assert mine == O.frame_header(size, bs, cs, 2, ulsb, be)
    f, n = block_codec.parse_frame(mine + b"\xde\xad")
    assert n == len(mine)
    assert (f.uncompressed_bytes, f.block_size, f.component_count, f.bytes_per_sample, f.unused_lsb_count,
            f.big_endian, f.ricepp_version) == (size, bs, cs, 2, ulsb, int(be), 1)


def test_parse_frame_skips_unknown_fields():
    # field 7 (string "x") and field 20 (long-form header, i32) appended before stop
    hdr = block_codec.frame_header(1000, 32, 2, 2, 4, True)
    assert hdr[-1] == 0
    extra = bytes([0x18, 0x01, ord("x")]) + bytes([0x05, 0x28, 0x54])
    f, n = block_codec.parse_frame(hdr[:-1] + extra + b"\x00")
    assert n == len(hdr) + len(extra)
    assert (f.block_size, f.component_count, f.unused_lsb_count) == (32, 2, 4)


def test_block_compressor_host_side_contract():
    comp = block_codec.block_compressor("ricepp:block_size=64")
    assert comp.describe() == "ricepp [block_size=64]"
    assert comp.type() == 7
    meta = '{"endianness":"big","bytes_per_sample":2,"unused_lsb_count":0,"component_count":2}'
    assert comp.get_compression_constraints(meta) == {"granularity": 4}
    assert json_eq(comp.metadata_requirements(), {
        "bytes_per_sample": ["set", [2]], "component_count": ["range", 1, 2],
        "endianness": ["set", ["big", "little"]], "unused_lsb_count": ["range", 0, 8]})
    with pytest.raises(RuntimeError, match="requires metadata"):
        comp.compress(b"\0\0", None)
    with pytest.raises(RuntimeError, match="unexpected data configuration: 6 bytes to compress, 2 components"):
        comp.compress(b"\0" * 6, meta)
    # the factory does not range-check (src/compression/ricepp.cpp:277-281): block_size=8 is a
    # valid ricepp configuration, 513 fails in create_encoder at compress time (:97-102)
    assert block_codec.block_compressor("ricepp:block_size=8").describe() == "ricepp [block_size=8]"
    big = block_codec.block_compressor("ricepp:block_size=513")
    with pytest.raises(RuntimeError, match="Unsupported configuration"):
        big.compress(b"\0" * 4, meta)
    with pytest.raises(RuntimeError, match="unsupported version: 2"):
        block_codec.RiceppBlockDecompressor(block_codec.frame_header(16, 128, 1, 2, 0, True, version=2))
    with pytest.raises(RuntimeError, match="unsupported bytes per sample: 3"):
        block_codec.RiceppBlockDecompressor(block_codec.frame_header(16, 128, 1, 3, 0, True))


def json_eq(s, obj):
    import json

    return json.loads(s) == obj


def test_cpp_facade_test_builds():
    r = subprocess.run(["bash", str(ROOT / "tests" / "cpp" / "build.sh")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (ROOT / "tests" / "cpp" / "build" / "facade_test").exists()


def test_plugin_callsites_compile_against_facade():
    """src/compression/ricepp.cpp's ricepp calls compile against include/ricepp_amd.hpp with only the
    include and the namespace changed (tests/cpp/plugin_callsites.cpp restates the call expressions)."""
    r = subprocess.run(["g++", "-std=c++20", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I", str(ROOT / "include"),
                        str(ROOT / "tests" / "cpp" / "plugin_callsites.cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def test_host_code_under_asan_ubsan():
    """SURVEY.md section 5 (reference CMakeLists.txt:67-69 sanitizer builds): the DwarFS frame parser of the
    product library and the CPU oracle under AddressSanitizer + UBSan, fed hostile headers and streams."""
    r = subprocess.run(["bash", str(ROOT / "tests" / "cpp" / "build_sanitize.sh")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([str(ROOT / "tests" / "cpp" / "build" / "fuzz_host"), "200000"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "fuzz_host: OK" in r.stdout, (r.stdout[-1000:], r.stderr[-3000:])
