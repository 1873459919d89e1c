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

}  // extern "C"
