// ricepp_frame.cpp -- DwarFS ricepp block framing (host side of the C ABI).
//
// A DwarFS ricepp block is
//   varint(uncompressed bytes)                 (src/varint.cpp:39-51, LEB128)
//   thrift-compact ricepp_block_header          (thrift/compression.thrift:42-49)
//   ricepp bitstream
// written by ricepp_block_compressor::compress (src/compression/ricepp.cpp:
// 107-127) and parsed by ricepp_block_decompressor's constructor (:186-201,
// :237-249).  Only the compact-protocol subset that header needs is
// implemented; unknown fields are skipped like thrift-lite's reader does.
#include <stdint.h>
#include <string.h>

#include "ricepp_amd.h"

namespace {

size_t put_varint(uint8_t* p, uint64_t v) {
  size_t n = 0;
  while (v >= 0x80) {
    p[n++] = static_cast<uint8_t>(v | 0x80);
    v >>= 7;
  }
  p[n++] = static_cast<uint8_t>(v);
  return n;
}

uint64_t zz(int64_t v) { return (static_cast<uint64_t>(v) << 1) ^ static_cast<uint64_t>(v >> 63); }
int64_t unzz(uint64_t v) { return static_cast<int64_t>(v >> 1) ^ -static_cast<int64_t>(v & 1); }

struct reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;

  uint8_t u8() {
    if (p >= end) {
      ok = false;
      return 0;
    }
    return *p++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      uint8_t b = u8();
      if (!ok) return 0;
      v |= static_cast<uint64_t>(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
};

// compact protocol type ids
enum : uint8_t {
  CT_STOP = 0, CT_TRUE = 1, CT_FALSE = 2, CT_BYTE = 3, CT_I16 = 4, CT_I32 = 5, CT_I64 = 6,
  CT_DOUBLE = 7, CT_BINARY = 8, CT_LIST = 9, CT_SET = 10, CT_MAP = 11, CT_STRUCT = 12
};

bool skip(reader& r, uint8_t t, int depth);

bool skip_struct(reader& r, int depth) {
  if (depth > 16) return false;
  int16_t last = 0;
  for (;;) {
    uint8_t h = r.u8();
    if (!r.ok) return false;
    uint8_t t = h & 0x0f;
    if (t == CT_STOP) return true;
    uint8_t delta = h >> 4;
    last = delta ? static_cast<int16_t>(last + delta) : static_cast<int16_t>(unzz(r.varint()));
    if (t == CT_TRUE || t == CT_FALSE) continue;
    if (!skip(r, t, depth + 1)) return false;
  }
}

bool skip(reader& r, uint8_t t, int depth) {
  switch (t) {
    case CT_TRUE: case CT_FALSE: case CT_BYTE: r.u8(); return r.ok;
    case CT_I16: case CT_I32: case CT_I64: r.varint(); return r.ok;
    case CT_DOUBLE: for (int i = 0; i < 8; ++i) r.u8(); return r.ok;
    case CT_BINARY: {
      uint64_t n = r.varint();
      if (!r.ok || n > static_cast<uint64_t>(r.end - r.p)) return false;
      r.p += n;
      return true;
    }
    case CT_LIST: case CT_SET: {
      uint8_t h = r.u8();
      uint64_t n = h >> 4;
      if (n == 15) n = r.varint();
      for (uint64_t i = 0; r.ok && i < n; ++i)
        if (!skip(r, h & 0x0f, depth + 1)) return false;
      return r.ok;
    }
    case CT_MAP: {
      uint64_t n = r.varint();
      if (n == 0) return r.ok;
      uint8_t kv = r.u8();
      for (uint64_t i = 0; r.ok && i < n; ++i)
        if (!skip(r, kv >> 4, depth + 1) || !skip(r, kv & 0x0f, depth + 1)) return false;
      return r.ok;
    }
    case CT_STRUCT: return skip_struct(r, depth + 1);
    default: return false;
  }
}

}  // namespace

extern "C" {

size_t rpp_frame_header(const rpp_frame* f, uint8_t* out) {
  size_t n = put_varint(out, f->uncompressed_bytes);
  out[n++] = 0x15;  // field 1 block_size: i32
  n += put_varint(out + n, zz(static_cast<int32_t>(f->block_size)));
  out[n++] = 0x14;  // field 2 component_count: i16
  n += put_varint(out + n, zz(static_cast<int16_t>(f->component_count)));
  out[n++] = 0x13;  // field 3 bytes_per_sample: byte
  out[n++] = static_cast<uint8_t>(f->bytes_per_sample);
  out[n++] = 0x13;  // field 4 unused_lsb_count: byte
  out[n++] = static_cast<uint8_t>(f->unused_lsb_count);
  out[n++] = f->big_endian ? 0x11 : 0x12;  // field 5 big_endian: bool
  out[n++] = 0x14;  // field 6 ricepp_version: i16
  n += put_varint(out + n, zz(static_cast<int16_t>(f->ricepp_version)));
  out[n++] = CT_STOP;
  return n;
}

long rpp_parse_frame(const uint8_t* in, size_t in_len, rpp_frame* f) {
  reader r{in, in + in_len};
  memset(f, 0, sizeof *f);
  f->uncompressed_bytes = r.varint();
  int16_t last = 0;
  for (;;) {
    uint8_t h = r.u8();
    if (!r.ok) return RPP_INVALID_ARGUMENT;
    uint8_t t = h & 0x0f;
    if (t == CT_STOP) break;
    uint8_t delta = h >> 4;
    int16_t id = delta ? static_cast<int16_t>(last + delta) : static_cast<int16_t>(unzz(r.varint()));
    last = id;
    uint64_t v = 0;
    if (t == CT_TRUE || t == CT_FALSE) {
      v = t == CT_TRUE;
    } else if (t == CT_BYTE) {
      v = r.u8();
    } else if (t == CT_I16 || t == CT_I32 || t == CT_I64) {
      v = static_cast<uint64_t>(unzz(r.varint()));
    } else {
      if (!skip(r, t, 0)) return RPP_INVALID_ARGUMENT;
      continue;
    }
    if (!r.ok) return RPP_INVALID_ARGUMENT;
    switch (id) {
      case 1: f->block_size = static_cast<uint32_t>(v); break;
      case 2: f->component_count = static_cast<uint16_t>(v); break;
      case 3: f->bytes_per_sample = static_cast<uint8_t>(v); break;
      case 4: f->unused_lsb_count = static_cast<uint8_t>(v); break;
      case 5: f->big_endian = v ? 1 : 0; break;
      case 6: f->ricepp_version = static_cast<uint16_t>(v); break;
      default: break;
    }
  }
  return static_cast<long>(r.p - in);
}

// ---- FLAC blocks (src/compression/flac.cpp:284-304, :477-484) ----
// varint(uncompressed bytes) + thrift-compact flac_block_header
// (thrift/compression.thrift:36-40) + a native FLAC stream.

size_t rpp_flac_frame_header(const rpp_flac_frame* f, uint8_t* out) {
  size_t n = put_varint(out, f->uncompressed_bytes);
  out[n++] = 0x14;  // field 1 num_channels: i16
  n += put_varint(out + n, zz(static_cast<int16_t>(f->num_channels)));
  out[n++] = 0x13;  // field 2 bits_per_sample: byte
  out[n++] = static_cast<uint8_t>(f->bits_per_sample);
  out[n++] = 0x13;  // field 3 flags: byte
  out[n++] = static_cast<uint8_t>(f->flags);
  out[n++] = CT_STOP;
  return n;
}

long rpp_flac_parse_frame(const uint8_t* in, size_t in_len, rpp_flac_frame* f) {
  reader r{in, in + in_len};
  memset(f, 0, sizeof *f);
  f->uncompressed_bytes = r.varint();
  int16_t last = 0;
  for (;;) {
    uint8_t h = r.u8();
    if (!r.ok) return RPP_INVALID_ARGUMENT;
    uint8_t t = h & 0x0f;
    if (t == CT_STOP) break;
    uint8_t delta = h >> 4;
    int16_t id = delta ? static_cast<int16_t>(last + delta) : static_cast<int16_t>(unzz(r.varint()));
    last = id;
    uint64_t v = 0;
    if (t == CT_BYTE) {
      v = r.u8();
    } else if (t == CT_I16 || t == CT_I32 || t == CT_I64) {
      v = static_cast<uint64_t>(unzz(r.varint()));
    } else {
      if (!skip(r, t, 0)) return RPP_INVALID_ARGUMENT;
      continue;
    }
    if (!r.ok) return RPP_INVALID_ARGUMENT;
    switch (id) {
      case 1: f->num_channels = static_cast<uint16_t>(v); break;
      case 2: f->bits_per_sample = static_cast<uint8_t>(v); break;
      case 3: f->flags = static_cast<uint8_t>(v); break;
      default: break;
    }
  }
  return static_cast<long>(r.p - in);
}

// "fLaC" + STREAMINFO (RFC 9639 8.2): block sizes 4096, frame sizes unknown,
// 48 kHz (flac.cpp:311), MD5 unknown (the reference's decoder does not check
// it: flac.cpp:411)
size_t rpp_flac_stream_header(uint32_t channels, uint32_t bps, uint64_t nsamples, uint8_t* out) {
  memset(out, 0, 42);
  memcpy(out, "fLaC", 4);
  out[4] = 0x80;  // last metadata block, STREAMINFO
  out[7] = 34;
  out[8] = 0x10;  // min block size 4096
  out[10] = 0x10;  // max block size 4096
  const uint32_t rate = 48000;
  out[18] = static_cast<uint8_t>(rate >> 12);
  out[19] = static_cast<uint8_t>(rate >> 4);
  out[20] = static_cast<uint8_t>(((rate & 15u) << 4) | (((channels - 1) & 7u) << 1) | (((bps - 1) >> 4) & 1u));
  out[21] = static_cast<uint8_t>((((bps - 1) & 15u) << 4) | ((nsamples >> 32) & 15u));
  out[22] = static_cast<uint8_t>(nsamples >> 24);
  out[23] = static_cast<uint8_t>(nsamples >> 16);
  out[24] = static_cast<uint8_t>(nsamples >> 8);
  out[25] = static_cast<uint8_t>(nsamples);
  return 42;
}

long rpp_flac_parse_stream(const uint8_t* in, size_t len, rpp_flac_stream_info* info) {
  memset(info, 0, sizeof *info);
  if (len < 4 || memcmp(in, "fLaC", 4) != 0) return RPP_INVALID_ARGUMENT;
  size_t p = 4;
  bool have_info = false;
  for (bool last = false; !last;) {
    if (p + 4 > len) return RPP_TRUNCATED_INPUT;
    last = (in[p] & 0x80) != 0;
    const uint32_t type = in[p] & 0x7f;
    const size_t blen = (static_cast<size_t>(in[p + 1]) << 16) | (static_cast<size_t>(in[p + 2]) << 8) | in[p + 3];
    p += 4;
    if (p + blen > len) return RPP_TRUNCATED_INPUT;
    if (type == 0) {
      if (blen < 34) return RPP_INVALID_ARGUMENT;
      const uint8_t* s = in + p;
      info->min_blocksize = (static_cast<uint32_t>(s[0]) << 8) | s[1];
      info->max_blocksize = (static_cast<uint32_t>(s[2]) << 8) | s[3];
      info->sample_rate = (static_cast<uint32_t>(s[10]) << 12) | (static_cast<uint32_t>(s[11]) << 4) | (s[12] >> 4);
      info->channels = ((s[12] >> 1) & 7u) + 1;
      info->bits_per_sample = (((s[12] & 1u) << 4) | (s[13] >> 4)) + 1;
      info->total_samples = (static_cast<uint64_t>(s[13] & 15u) << 32) | (static_cast<uint64_t>(s[14]) << 24) |
                            (static_cast<uint64_t>(s[15]) << 16) | (static_cast<uint64_t>(s[16]) << 8) | s[17];
      have_info = true;
    }
    p += blen;
  }
  if (!have_info) return RPP_INVALID_ARGUMENT;
  return static_cast<long>(p);
}

}  // extern "C"
