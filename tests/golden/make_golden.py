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
  pcmaudio_fixtures.json -- the PCM payload of test/pcmaudio/test{8,12,16,20,
                         24,32}.{wav,aiff} with the metadata the pcmaudio
                         categorizer emits for each file
                         (src/writer/categorizer/pcmaudio_categorizer.cpp:
                         604-697 AIFF, 887-1055 WAV, 444-470 metadata JSON),
                         the FLAC category's real inputs.
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


def _chunks(data: bytes, pos: int, big: bool):
    """IFF chunks from `pos`: (fourcc, payload offset, size); chunks are padded to even sizes."""
    order = "big" if big else "little"
    while pos + 8 <= len(data):
        cid = data[pos:pos + 4].decode("latin-1")
        size = int.from_bytes(data[pos + 4:pos + 8], order)
        yield cid, pos + 8, size
        pos += 8 + size + (size & 1)


def pcm_fixture(name: str, data: bytes) -> dict:
    """The categorizer's reading of a WAV / AIFF file: its metadata and PCM fragment."""
    if data[:4] == b"RIFF" and data[8:12] == b"WAVE":
        meta, pcm = None, None
        for cid, off, size in _chunks(data, 12, False):
            if cid == "fmt ":
                code, chans = int.from_bytes(data[off:off + 2], "little"), int.from_bytes(data[off + 2:off + 4], "little")
                bits = int.from_bytes(data[off + 14:off + 16], "little")
                if size == 40 and code == 0xFFFE:  # WAVE_FORMAT_EXTENSIBLE: the sub-format code decides
                    code = int.from_bytes(data[off + 24:off + 26], "little")
                assert code == 1, (name, code)  # PCM (:1016)
                # :1028-1034
                meta = {"endianness": "little", "signedness": "signed" if bits > 8 else "unsigned", "padding": "lsb",
                        "bytes_per_sample": (bits + 7) // 8, "bits_per_sample": bits, "number_of_channels": chans}
            elif cid == "data":
                frame = meta["number_of_channels"] * meta["bytes_per_sample"]
                pcm = data[off:off + size - size % frame]  # handle_pcm_data (:1089-1100) drops the partial frame
                break
    elif data[:4] == b"FORM" and data[8:12] == b"AIFF":
        meta, pcm, frames = None, None, 0
        for cid, off, size in _chunks(data, 12, True):
            if cid == "COMM":  # :632-659
                chans = int.from_bytes(data[off:off + 2], "big")
                frames = int.from_bytes(data[off + 2:off + 6], "big")
                bits = int.from_bytes(data[off + 6:off + 8], "big")
                meta = {"endianness": "big", "signedness": "signed", "padding": "lsb",
                        "bytes_per_sample": (bits + 7) // 8, "bits_per_sample": bits, "number_of_channels": chans}
            elif cid == "SSND":  # :660-692
                ssnd_off = int.from_bytes(data[off:off + 4], "big")
                start = off + 8 + ssnd_off
                pcm = data[start:start + frames * meta["number_of_channels"] * meta["bytes_per_sample"]]
                break
    else:
        raise SystemExit(f"{name}: not WAV / AIFF")
    assert meta is not None and pcm is not None, name
    return {"file": f"test/pcmaudio/{name}", "metadata": meta, "pcm_hex": pcm.hex()}


def main() -> None:
    ref = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
    src = (ref / "ricepp/test/bitstream_test.cpp").read_text()
    kat = extract_bitstream_kat(src)
    assert len(kat["ops"]) == 1000, len(kat["ops"])
    assert len(kat["expected_hex"]) == 2 * 4186
    (HERE / "bitstream_kat.json").write_text(json.dumps(kat, indent=0) + "\n")
    for name in ("dark.fits", "test.fits"):
        shutil.copyfile(ref / "test/fits" / name, HERE / name)
    fixtures = [pcm_fixture(f"test{b}.{ext}", (ref / "test/pcmaudio" / f"test{b}.{ext}").read_bytes())
                for b in (8, 12, 16, 20, 24, 32) for ext in ("wav", "aiff")]
    (HERE / "pcmaudio_fixtures.json").write_text(json.dumps(fixtures, indent=1) + "\n")
    print("wrote", HERE)


if __name__ == "__main__":
    main()
