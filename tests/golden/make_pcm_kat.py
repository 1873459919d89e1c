#!/usr/bin/env python3
"""Writes tests/golden/pcm_kat.json: the known-answer cases of the reference's
test/pcm_sample_transformer_test.cpp (:33-293), as data.

Each reference test builds `packed` bytes from a value list with
convert<std::endian::...> (for int24_20bit_be_lsb: bytes 1..3 of each
big-endian int32, :266-276), unpacks it with a given transformer, expects
`ref`, and packs it back expecting the original bytes.  The value lists and
transformer arguments below are transcribed from those tests; the packed bytes
are produced by the same byte-order rule.  Run once: python tests/golden/make_pcm_kat.py
"""

import json
import struct
from pathlib import Path

HERE = Path(__file__).resolve().parent


def conv(fmt, vals):
    return b"".join(struct.pack(fmt, v) for v in vals)


def main():
    u12 = [0, 1, 2047, 2048, 2049, 4094, 4095]
    r12 = [-2048, -2047, -1, 0, 1, 2046, 2047]
    s16 = [-32768, -32767, -1, 0, 1, 32766, 32767]
    s14 = [-8192, -8191, -1, 0, 1, 8190, 8191]
    s24 = [-8388608, -8388607, -1, 0, 1, 8388606, 8388607]
    s20 = [-524288, -524287, -1, 0, 1, 524286, 524287]
    cases = [
        # name, big_endian, is_signed, lsb_padded, bytes, bits, packed, ref
        ("uint8_8bit", 1, 0, 0, 1, 8, bytes([0, 1, 42, 254, 255]), [-128, -127, -86, 126, 127]),
        ("uint16_12bit_be_msb", 1, 0, 0, 2, 12, conv(">H", u12), r12),
        ("uint16_12bit_be_lsb", 1, 0, 1, 2, 12, conv(">H", [v * 16 for v in u12]), r12),
        ("int16_16bit_be", 1, 1, 0, 2, 16, conv(">h", s16), s16),
        ("int16_14bit_le_lsb", 0, 1, 1, 2, 14, conv("<h", [v * 4 for v in s14]), s14),
        ("int32_24bit_be_lsb", 1, 1, 1, 4, 24, conv(">i", [v * 256 for v in s24]), s24),
        ("int32_24bit_le_msb", 0, 1, 0, 4, 24, conv("<i", s24), s24),
        ("int24_20bit_be_lsb", 1, 1, 1, 3, 20, b"".join(struct.pack(">i", v * 16)[1:] for v in s20), s20),
    ]
    out = [dict(name=n, big_endian=be, is_signed=sg, lsb_padded=lp, bytes=nb, bits=bt, packed=list(p), ref=r)
           for n, be, sg, lp, nb, bt, p, r in cases]
    (HERE / "pcm_kat.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
