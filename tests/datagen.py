"""Synthetic sample generators for parity tests and the benchmark.

They mirror the shapes of the reference's generators (the exact libstdc++
random streams are not reproducible in numpy and are not needed: parity is
checked against the oracle on the same inputs):
  * ricepp/test/codec_test.cpp:43-61 -- noise U[20000,21000], full-range
    outliers with probability 1/(full_chance+1), masked to ulsb, byteswapped;
  * ricepp/ricepp_benchmark.cpp:54-71 -- `noise_bits` uniform noise, with
    full-range values when an exponential(full_freq) draw is <= 1;
  * Poisson(lambda) sensor-like data (BASELINE.json configs).
All return *stored* uint16 samples (byteswapped when big endian).
"""

import numpy as np


def store(values, ulsb=0, big_endian=True):
    v = (np.asarray(values, dtype=np.uint64) & 0xFFFF).astype(np.uint16)
    mask = np.uint16((0xFFFF << ulsb) & 0xFFFF)
    v = v & mask
    return v.byteswap() if big_endian else v


def codec_test_data(rng, count, ulsb=0, big_endian=True, full_chance=50):
    full = rng.integers(0, 65536, count)
    noise = rng.integers(20000, 21001, count)
    pick = rng.integers(0, full_chance + 1, count) == 0
    return store(np.where(pick, full, noise), ulsb, big_endian)


def benchmark_data(rng, count, ulsb=0, big_endian=True, noise_bits=6, full_bits=16, full_freq=0.1):
    gate = rng.exponential(1.0 / full_freq, count) <= 1.0
    noise = rng.integers(0, 1 << (noise_bits + ulsb), count)
    full = rng.integers(0, 1 << min(full_bits + ulsb, 16), count)
    return store(np.where(gate, full, noise), ulsb, big_endian)


def poisson_data(rng, count, lam=1000.0, ulsb=0, big_endian=True):
    v = np.minimum(rng.poisson(lam, count), (0xFFFF >> ulsb)).astype(np.uint64) << ulsb
    return store(v, ulsb, big_endian)


def constant_data(count, value=25000, ulsb=0, big_endian=True):
    return store(np.full(count, value), ulsb, big_endian)


def full_range_data(rng, count, ulsb=0, big_endian=True):
    return store(rng.integers(0, 65536, count), ulsb, big_endian)


def ramp_data(count, ulsb=0, big_endian=True, step=3):
    return store(np.arange(count) * step, ulsb, big_endian)


def mixed_data(rng, count, ulsb=0, big_endian=True):
    """codec_test.cpp:107-131: random + constant + all-full-range thirds."""
    a = count // 3
    return np.concatenate([
        codec_test_data(rng, a, ulsb, big_endian),
        constant_data(a, 25000, ulsb, big_endian),
        full_range_data(rng, count - 2 * a, ulsb, big_endian),
    ])


def dwarfs_test_data(rng, pixels, components=1, ulsb=0):
    """test/ricepp_compressor_test.cpp:66-101: per component a third of
    noise U[30000,31000] (full-range outliers p=1/51), a third of one
    constant, a third of full-range values; components interleaved; stored
    big endian."""
    comps = []
    for _ in range(components):
        a = pixels // 3
        noise = rng.integers(30000, 31001, a)
        pick = rng.integers(0, 51, a) == 0
        d1 = np.where(pick, rng.integers(0, 65536, a), noise)
        d2 = np.full(a, (int(rng.integers(0, 65536)) << ulsb) & 0xFFFF)
        d3 = rng.integers(0, 65536, pixels - 2 * a)
        comps.append(np.concatenate([d1, d2, d3]))
    inter = np.stack(comps, axis=1).reshape(-1)
    return store(inter, ulsb, True)


def spiky_data(rng, count, ulsb=0, big_endian=True):
    """Mostly flat with rare huge spikes: long unary runs at small fs."""
    v = rng.integers(100, 104, count)
    spikes = rng.random(count) < 0.01
    v[spikes] = rng.integers(30000, 65536, int(spikes.sum()))
    return store(v, ulsb, big_endian)


KINDS = {
    "poisson": lambda rng, n, ulsb, be: poisson_data(rng, n, 1000.0 / (1 << ulsb) if ulsb else 1000.0, ulsb, be),
    "benchmark": lambda rng, n, ulsb, be: benchmark_data(rng, n, ulsb, be),
    "codec_test": lambda rng, n, ulsb, be: codec_test_data(rng, n, ulsb, be),
    "constant": lambda rng, n, ulsb, be: constant_data(n, 25000, ulsb, be),
    "full_range": lambda rng, n, ulsb, be: full_range_data(rng, n, ulsb, be),
    "ramp": lambda rng, n, ulsb, be: ramp_data(n, ulsb, be),
    "mixed": lambda rng, n, ulsb, be: mixed_data(rng, n, ulsb, be),
    "spiky": lambda rng, n, ulsb, be: spiky_data(rng, n, ulsb, be),
    "zeros": lambda rng, n, ulsb, be: store(np.zeros(n), ulsb, be),
}


def parse_fits(path):
    """Minimal FITS primary-HDU reader for the 16-bit fixtures in
    tests/golden (test/fits/*.fits of the reference): returns (header dict,
    raw big-endian uint16 image samples as stored)."""
    raw = open(path, "rb").read()
    hdr = {}
    off = 0
    while True:
        block = raw[off:off + 2880]
        off += 2880
        done = False
        for i in range(0, 2880, 80):
            card = block[i:i + 80].decode("ascii", "replace")
            key = card[:8].strip()
            if key == "END":
                done = True
                break
            if card[8:10] == "= ":
                val = card[10:].split("/")[0].strip().strip("'").strip()
                hdr[key] = val
        if done:
            break
    assert int(hdr["BITPIX"]) == 16
    dims = [int(hdr[f"NAXIS{i + 1}"]) for i in range(int(hdr["NAXIS"]))]
    n = int(np.prod(dims))
    data = np.frombuffer(raw[off:off + 2 * n], dtype=np.uint16).copy()  # stored (big endian) bytes
    return hdr, data
