#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the reference tree.

Run once in the build container (the reference is NOT present on the GPU box):

    python tests/golden/make_golden.py /root/reference

Outputs (all are data extracted from the reference's own test fixtures):
  bitstream_kat.json  -- the 1000-op script and the 4186-byte expected
                         bitstream of ricepp/test/bitstream_test.cpp:113-1466
                         (compared at :1491-1494).
  dark.fits, test.fits -- the real FITS fixtures of test/fits/ (ZWO
                         ASI1600MM mono, ASI294MC Bayer RGGB), used as inputs.
"""

import json
import re
import shutil
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent


def extract_bitstream_kat(src: str) -> dict:
    ops_m = re.search(r"testdata\{\{(.*?)\}\};", src, re.S)
    exp_m = re.search(r"expected_bitstream\{\{(.*?)\}\};", src, re.S)
    if not ops_m or not exp_m:
        raise SystemExit("could not find testdata / expected_bitstream")
    opnames = {"single": 0, "sequence": 1, "multi": 2}
    ops, bits, values = [], [], []
    for m in re.finditer(
        r"\{\s*oper::(\w+)\s*,\s*(\d+)\s*,\s*(?:UINT64_C\()?(0x[0-9a-fA-F]+|\d+)\)?\s*\}",
        ops_m.group(1),
    ):
        ops.append(opnames[m.group(1)])
        bits.append(int(m.group(2)))
        values.append(int(m.group(3), 0))
    expected = bytes(int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", exp_m.group(1)))
    return {
        "source": "ricepp/test/bitstream_test.cpp:113-1466",
        "ops": ops,
        "bits": bits,
        "values": [f"{v:#x}" for v in values],
        "expected_hex": expected.hex(),
    }


def main() -> None:
    ref = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
    src = (ref / "ricepp/test/bitstream_test.cpp").read_text()
    kat = extract_bitstream_kat(src)
    assert len(kat["ops"]) == 1000, len(kat["ops"])
    assert len(kat["expected_hex"]) == 2 * 4186
    (HERE / "bitstream_kat.json").write_text(json.dumps(kat, indent=0) + "\n")
    for name in ("dark.fits", "test.fits"):
        shutil.copyfile(ref / "test/fits" / name, HERE / name)
    print("wrote", HERE)


if __name__ == "__main__":
    main()
