"""ctypes wrapper around the CPU FLAC restatement (oracle/flac_oracle.c).

TEST INFRASTRUCTURE ONLY (parity unpinned: libFLAC, the reference's FLAC
coder, is absent -- see the C file's header).  Never imported by the product
package ``dwarfs_amd``.
"""

from __future__ import annotations

import ctypes as C
import subprocess
from dataclasses import dataclass
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "libflac_oracle.so"

OK, TRUNCATED, INVALID, TOO_SMALL, BAD_STREAM = 0, -2, -3, -4, -7


class Opts(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("subframe_type", "fixed_order", "lpc_order", "lpc_precision", "stereo",
                                       "max_partition_order", "rice2", "escape", "padding_block", "wasted",
                                       "variable_blocking", "max_lpc_order")]


@dataclass
class EncodeOptions:
    """subframe_type: "auto", "constant", "verbatim", "fixed", "lpc"."""
    subframe_type: str = "auto"
    fixed_order: int = 2
    lpc_order: int = 8
    lpc_precision: int = 12
    stereo: int = -1  # -1 auto, 0 independent, 8 left/side, 9 side/right, 10 mid/side
    max_partition_order: int = 5
    rice2: bool = False
    escape: bool = False
    padding_block: bool = False
    wasted: bool = True
    variable_blocking: bool = False
    max_lpc_order: int = 8

    def native(self) -> Opts:
        kinds = {"auto": 0, "constant": 1, "verbatim": 2, "fixed": 3, "lpc": 4}
        return Opts(kinds[self.subframe_type], self.fixed_order, self.lpc_order, self.lpc_precision, self.stereo,
                    self.max_partition_order, int(self.rice2), int(self.escape), int(self.padding_block),
                    int(self.wasted), int(self.variable_blocking), self.max_lpc_order)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / "flac_oracle.c").stat().st_mtime:
            subprocess.run(["make", "-C", str(HERE), "-s"], check=True)
        L = C.CDLL(str(LIB_PATH))
        P = C.c_void_p
        L.fo_encode.argtypes = [P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(Opts), P, C.c_size_t]
        L.fo_encode.restype = C.c_size_t
        L.fo_decode.argtypes = [P, C.c_size_t, P, C.c_uint64, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                C.POINTER(C.c_uint64)]
        L.fo_decode.restype = C.c_int
        _lib = L
    return _lib


def encode(samples: np.ndarray, channels: int, bps: int, blocksize: int = 4096,
           opts: EncodeOptions | None = None) -> bytes:
    """A FLAC stream of interleaved int32 samples (len = frames * channels)."""
    x = np.ascontiguousarray(samples, dtype=np.int32)
    n = x.size // channels
    cap = 64 + 42 + 20 + (n // max(blocksize, 1) + 1) * (32 + 8 * channels) + x.size * 5 + 1024
    out = np.zeros(cap, np.uint8)
    size = lib().fo_encode(x.ctypes.data, n, channels, bps, blocksize, C.byref((opts or EncodeOptions()).native()),
                           out.ctypes.data, cap)
    if size == 0:
        raise ValueError("flac oracle: encode failed")
    return out[:size].tobytes()


def decode(stream: bytes, max_values: int) -> tuple:
    """(status, interleaved int32 samples, channels, bps)."""
    buf = np.frombuffer(stream, np.uint8)
    out = np.zeros(max(max_values, 1), np.int32)
    ch, bps, n = C.c_uint32(), C.c_uint32(), C.c_uint64()
    st = lib().fo_decode(buf.ctypes.data, buf.size, out.ctypes.data, max_values, C.byref(ch), C.byref(bps),
                         C.byref(n))
    if st != OK:
        return st, None, 0, 0
    return st, out[: n.value * ch.value], ch.value, bps.value
