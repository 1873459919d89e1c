/*
 * ricepp_oracle.c -- CPU restatement of the reference ricepp codec.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the
 * MI355X codec in dwarfs_amd/.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path never links,
 * calls or falls back to it.
 *
 * It restates, in plain C, the algorithm of the reference ricepp library
 * (mhx/dwarfs, /root/reference/ricepp).  Each function cites the reference
 * file:line it follows.  No reference source is copied.
 *
 * Parity pinning (see DESIGN.md "Oracle"): the reference cannot be built in
 * this image (it needs range-v3, which is absent), so this restatement is
 * pinned by the reference's own fixtures:
 *   - the 4186-byte bitstream KAT of ricepp/test/bitstream_test.cpp:113-1466
 *     (writer and reader, via rpo_bitstream_run_ops),
 *   - the worst-case size KATs of ricepp/test/codec_test.cpp:164-196,
 *   - "incompressible data encodes to exactly the worst case"
 *     (codec_test.cpp:171-172),
 *   - the error-config KATs (codec_test.cpp:198-222),
 *   - round trips over the reference's test configurations and the real FITS
 *     fixtures in test/fits/.
 */

#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define RPO_OK 0
#define RPO_UNSUPPORTED_CONFIG (-1)
#define RPO_TRUNCATED_INPUT (-2)
#define RPO_INVALID_ARGUMENT (-3)
#define RPO_OUTPUT_TOO_SMALL (-4)

/* codec_config, ricepp/include/ricepp/codec_config.h:36-41 */
typedef struct rpo_config {
  uint32_t block_size;
  uint32_t component_stream_count;
  uint32_t big_endian; /* byteorder == std::endian::big */
  uint32_t unused_lsb_count;
} rpo_config;

/* Config validation: ricepp_cpuspecific_traits.h:118-151 (block_size <= 512,
 * cs in {1,2}); dynamic traits assert ulsb < 16 (:59).  block_size 0 would
 * make range-v3 chunk(0) loop forever in the reference; rejected here. */
int rpo_check_config(const rpo_config* c) {
  if (c->block_size == 0 || c->block_size > 512) return RPO_UNSUPPORTED_CONFIG;
  if (c->component_stream_count != 1 && c->component_stream_count != 2)
    return RPO_UNSUPPORTED_CONFIG;
  if (c->unused_lsb_count >= 16) return RPO_UNSUPPORTED_CONFIG;
  return RPO_OK;
}

static inline uint16_t bswap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

/* pixel traits read/write, ricepp_cpuspecific_traits.h:63-75 */
static inline uint32_t px_read(const rpo_config* c, uint16_t v) {
  uint16_t t = c->big_endian ? bswap16(v) : v;
  return (uint32_t)(t >> c->unused_lsb_count);
}
static inline uint16_t px_write(const rpo_config* c, uint32_t v) {
  uint16_t t = (uint16_t)((uint16_t)v << c->unused_lsb_count);
  return c->big_endian ? bswap16(t) : t;
}

/* ---------------------------------------------------------------------- */
/* bitstream writer: ricepp/include/ricepp/bitstream_writer.h:58-150       */
/* LSB-first 64-bit accumulator, little-endian 8-byte packets; the final   */
/* packet keeps ceil(bit_pos/8) bytes (write_packet, :139-145).            */
/* ---------------------------------------------------------------------- */
typedef struct bw {
  uint8_t* out;
  size_t pos; /* bytes written */
  size_t cap;
  uint64_t data;
  unsigned bit_pos;
  int overflow;
} bw;

static inline void bw_packet(bw* w, uint64_t bits, size_t nbytes) {
  if (w->pos + nbytes > w->cap) {
    w->overflow = 1;
    return;
  }
  for (size_t i = 0; i < nbytes; ++i) w->out[w->pos + i] = (uint8_t)(bits >> (8 * i));
  w->pos += nbytes;
}

/* write_bits_impl, bitstream_writer.h:125-137 */
static inline void bw_impl(bw* w, uint64_t bits, unsigned n) {
  if (n < 64) bits &= (UINT64_C(1) << n) - 1;
  w->data |= bits << w->bit_pos; /* n>0 implies bit_pos < 64 */
  w->bit_pos += n;
  if (w->bit_pos == 64) {
    bw_packet(w, w->data, 8);
    w->data = 0;
    w->bit_pos = 0;
  }
}

/* write_bits, bitstream_writer.h:91-108 */
static inline void bw_bits(bw* w, uint64_t bits, unsigned n) {
  while (n > 0) {
    unsigned room = 64 - w->bit_pos;
    unsigned k = n < room ? n : room;
    bw_impl(w, bits, k);
    bits = (k == 64) ? 0 : bits >> k;
    n -= k;
  }
}

/* write_bit(bit, repeat), bitstream_writer.h:73-89 */
static inline void bw_repeat(bw* w, int bit, uint64_t repeat) {
  uint64_t bits = bit ? ~UINT64_C(0) : 0;
  if (w->bit_pos != 0) {
    unsigned rem = 64 - w->bit_pos;
    if (repeat > rem) {
      bw_impl(w, bits, rem);
      repeat -= rem;
    }
  }
  while (repeat > 64) {
    bw_packet(w, bits, 8);
    repeat -= 64;
  }
  if (repeat > 0) bw_impl(w, bits, (unsigned)repeat);
}

/* flush, bitstream_writer.h:110-120 */
static inline void bw_flush(bw* w) {
  if (w->bit_pos > 0) {
    bw_packet(w, w->data, (w->bit_pos + 7) / 8);
    w->data = 0;
    w->bit_pos = 0;
  }
}

/* ---------------------------------------------------------------------- */
/* bitstream reader: ricepp/include/ricepp/bitstream_reader.h:44-188       */
/* Reading a packet when none is left is std::out_of_range (:150-152); a   */
/* partial last packet is zero padded (:165-166).                          */
/* ---------------------------------------------------------------------- */
typedef struct br {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t data;
  unsigned bit_pos;
  int err;
} br;

static inline uint64_t br_packet(br* r) {
  if (r->p == r->end) {
    r->err = 1;
    return 0;
  }
  size_t remain = (size_t)(r->end - r->p);
  uint64_t v = 0;
  if (remain >= 8) {
    memcpy(&v, r->p, 8); /* host is little endian */
    r->p += 8;
  } else {
    memcpy(&v, r->p, remain);
    r->p = r->end;
  }
  return v;
}

/* peek_bits + skip_bits, bitstream_reader.h:113-147 */
static inline uint64_t br_impl(br* r, unsigned n) {
  if (r->bit_pos == 0) r->data = br_packet(r);
  uint64_t bits = r->data >> r->bit_pos;
  if (n < 64) bits &= (UINT64_C(1) << n) - 1;
  r->bit_pos = (r->bit_pos + n) & 63;
  return bits;
}

/* read_bits, bitstream_reader.h:59-77 */
static inline uint64_t br_bits(br* r, unsigned n) {
  uint64_t bits = 0;
  unsigned pos = 0;
  while (n > 0) {
    unsigned rem = 64 - r->bit_pos;
    if (n <= rem) {
      bits |= br_impl(r, n) << pos;
      break;
    }
    bits |= br_impl(r, rem) << pos;
    n -= rem;
    pos += rem;
  }
  return bits;
}

/* find_first_set, bitstream_reader.h:79-111 */
static inline uint64_t br_ffs(br* r) {
  uint64_t zeros = 0;
  if (r->bit_pos != 0) {
    if ((r->data >> r->bit_pos) & 1) {
      r->bit_pos = (r->bit_pos + 1) & 63;
      return 0;
    }
    unsigned rem = 64 - r->bit_pos;
    uint64_t bits = r->data >> r->bit_pos;
    if (bits != 0) {
      unsigned f = (unsigned)__builtin_ctzll(bits);
      r->bit_pos = (r->bit_pos + f + 1) & 63;
      return f;
    }
    r->bit_pos = 0;
    zeros += rem;
  }
  for (;;) {
    uint64_t bits = br_packet(r);
    if (r->err) return zeros;
    if (bits != 0) {
      unsigned f = (unsigned)__builtin_ctzll(bits);
      if (f + 1 != 64) {
        r->data = bits;
        r->bit_pos = f + 1;
      } else {
        r->bit_pos = 0;
      }
      return zeros + f;
    }
    zeros += 64;
  }
}

/* ---------------------------------------------------------------------- */
/* codec                                                                   */
/* ---------------------------------------------------------------------- */

/* codec::worst_case_bit_count, ricepp/include/ricepp/codec.h:142-151, and
 * encoder_impl::worst_case_encoded_bytes_impl, ricepp_cpuspecific.cpp:75-77 */
size_t rpo_worst_case_bytes(const rpo_config* c, size_t n) {
  size_t cs = c->component_stream_count, bs = c->block_size;
  size_t per = n / cs;
  size_t num = 16 + 4 * ((per + bs - 1) / bs) + 16 * per;
  return (num * cs + 7) / 8;
}

/* compute_best_split<FsMax=14>, ricepp/include/ricepp/detail/encode.h:43-90 */
static void best_split(const uint16_t* delta, size_t n, uint64_t sum, unsigned* fs_out,
                       size_t* bits_out) {
#define BITS_FOR_FS(fs_, res_)                                   \
  do {                                                           \
    uint32_t mask_ = (uint32_t)(0xFFFFu << (fs_));               \
    uint32_t acc_ = 0;                                           \
    for (size_t i_ = 0; i_ < n; ++i_) acc_ += delta[i_] & mask_; \
    (res_) = n * ((fs_) + 1) + (acc_ >> (fs_));                  \
  } while (0)
  uint64_t avg = sum / n;
  unsigned clz = avg ? (unsigned)__builtin_clzll(avg) : 64;
  unsigned start = 64 - (clz + 2 < 64 ? clz + 2 : 64);
  size_t bits0, bits1;
  BITS_FOR_FS(start, bits0);
  BITS_FOR_FS(start + 1, bits1);
  int cand, dir;
  size_t bits;
  if (bits1 <= bits0) {
    cand = (int)start + 1;
    bits = bits1;
    dir = 1;
  } else {
    cand = (int)start;
    bits = bits0;
    dir = -1;
  }
  if (bits0 != bits1) {
    while (cand > 0 && cand < 14) {
      size_t tmp;
      BITS_FOR_FS((unsigned)(cand + dir), tmp);
      if (tmp > bits) break;
      bits = tmp;
      cand += dir;
    }
  }
  *fs_out = (unsigned)cand;
  *bits_out = bits;
#undef BITS_FOR_FS
}

/* encode_block, ricepp/include/ricepp/detail/encode.h:92-157.
 * `src` points at the first raw sample of the sub-block, `stride` = cs. */
static void encode_block(bw* w, const rpo_config* c, const uint16_t* src, size_t n,
                         size_t stride, uint32_t* last_value) {
  uint16_t delta[512];
  uint32_t last = *last_value;
  uint64_t sum = 0;
  for (size_t i = 0; i < n; ++i) {
    uint32_t px = px_read(c, src[i * stride]);
    uint32_t diff = (px - last) & 0xFFFFu;
    uint16_t d = (uint16_t)((diff & 0x8000u) ? ~(diff << 1) : (diff << 1));
    delta[i] = d;
    sum += d;
    last = px;
  }
  *last_value = last;
  if (sum > 0) {
    unsigned fs;
    size_t bits;
    best_split(delta, n, sum, &fs, &bits);
    if (fs < 14 && bits < 16 * n) {
      bw_bits(w, fs + 1, 4);
      for (size_t i = 0; i < n; ++i) {
        uint32_t top = (uint32_t)delta[i] >> fs;
        if (top > 0) bw_repeat(w, 0, top);
        bw_impl(w, 1, 1);
        if (fs) bw_bits(w, delta[i], fs);
      }
    } else {
      bw_bits(w, 15, 4);
      for (size_t i = 0; i < n; ++i) bw_bits(w, src[i * stride], 16);
    }
  } else {
    bw_bits(w, 0, 4);
  }
}

/* codec::encode, ricepp/include/ricepp/codec.h:62-101.  Empty input is UB in
 * the reference (reads input[0]); here it writes zero initial values. */
int rpo_encode(const rpo_config* c, const uint16_t* in, size_t n, uint8_t* out,
               size_t out_cap, size_t* out_len) {
  int st = rpo_check_config(c);
  if (st) return st;
  size_t cs = c->component_stream_count, bs = c->block_size;
  if (n % cs) return RPO_INVALID_ARGUMENT;
  bw w = {out, 0, out_cap, 0, 0, 0};
  uint32_t last[2] = {0, 0};
  for (size_t i = 0; i < cs; ++i) {
    last[i] = n ? px_read(c, in[i]) : 0;
    bw_bits(&w, last[i], 16);
  }
  for (size_t base = 0; base < n; base += cs * bs) {
    size_t len = n - base < cs * bs ? n - base : cs * bs;
    for (size_t i = 0; i < cs; ++i)
      encode_block(&w, c, in + base + i, len / cs, cs, &last[i]);
  }
  bw_flush(&w);
  if (w.overflow) return RPO_OUTPUT_TOO_SMALL;
  *out_len = w.pos;
  return RPO_OK;
}

/* decode_block, ricepp/include/ricepp/detail/decode.h:42-83 */
static void decode_block(br* r, const rpo_config* c, uint16_t* dst, size_t n,
                         size_t stride, uint32_t* last_value) {
  uint32_t last = *last_value;
  unsigned fsp1 = (unsigned)br_bits(r, 4);
  if (fsp1 > 0) {
    if (fsp1 <= 14) {
      unsigned fs = fsp1 - 1;
      for (size_t i = 0; i < n; ++i) {
        uint32_t diff = (uint32_t)(br_ffs(r) << fs);
        diff |= (uint32_t)br_bits(r, fs);
        last += ((diff & 1) ? ~0u : 0u) ^ (diff >> 1);
        dst[i * stride] = px_write(c, last);
      }
    } else {
      for (size_t i = 0; i < n; ++i) dst[i * stride] = (uint16_t)br_bits(r, 16);
      last = px_read(c, dst[(n - 1) * stride]);
    }
  } else {
    uint16_t v = px_write(c, last);
    for (size_t i = 0; i < n; ++i) dst[i * stride] = v;
  }
  *last_value = last;
}

/* codec::decode, ricepp/include/ricepp/codec.h:103-140 */
int rpo_decode(const rpo_config* c, const uint8_t* in, size_t in_len, uint16_t* out,
               size_t n) {
  int st = rpo_check_config(c);
  if (st) return st;
  size_t cs = c->component_stream_count, bs = c->block_size;
  if (n % cs) return RPO_INVALID_ARGUMENT;
  br r = {in, in + in_len, 0, 0, 0};
  uint32_t last[2] = {0, 0};
  for (size_t i = 0; i < cs; ++i) last[i] = (uint32_t)br_bits(&r, 16);
  for (size_t base = 0; base < n && !r.err; base += cs * bs) {
    size_t len = n - base < cs * bs ? n - base : cs * bs;
    for (size_t i = 0; i < cs; ++i) decode_block(&r, c, out + base + i, len / cs, cs, &last[i]);
  }
  return r.err ? RPO_TRUNCATED_INPUT : RPO_OK;
}

/* ---------------------------------------------------------------------- */
/* Bitstream op-script, driving the KAT of ricepp/test/bitstream_test.cpp  */
/* :1470-1534.  op: 0 single (write_bit(value)), 1 sequence               */
/* (write_bit(false, bits); write_bit(true)), 2 multi (write_bits(value,   */
/* bits)).  Returns bytes written; read-back mismatches go to *mismatch.   */
/* ---------------------------------------------------------------------- */
long rpo_bitstream_run_ops(const uint8_t* ops, const uint32_t* bits, const uint64_t* values,
                           size_t nops, uint8_t* out, size_t cap, long* mismatch) {
  bw w = {out, 0, cap, 0, 0, 0};
  for (size_t i = 0; i < nops; ++i) {
    switch (ops[i]) {
      case 0: bw_impl(&w, values[i] & 1, 1); break;
      case 1:
        bw_repeat(&w, 0, bits[i]);
        bw_impl(&w, 1, 1);
        break;
      default: bw_bits(&w, values[i], bits[i]); break;
    }
  }
  bw_flush(&w);
  if (w.overflow) return -1;
  br r = {out, out + w.pos, 0, 0, 0};
  long bad = 0;
  for (size_t i = 0; i < nops; ++i) {
    uint64_t got, want;
    switch (ops[i]) {
      case 0: got = br_bits(&r, 1); want = values[i] & 1; break;
      case 1: got = br_ffs(&r); want = bits[i]; break;
      default: got = br_bits(&r, bits[i]); want = values[i]; break;
    }
    if (got != want || r.err) ++bad;
  }
  *mismatch = bad;
  return (long)w.pos;
}

/* ---------------------------------------------------------------------- */
/* Batched CPU codec over independent blocks (the CPU baseline leg).       */
/* This is the host-thread analogue of DwarFS's worker_group running one   */
/* compression job per block (src/writer/filesystem_writer.cpp:255-287).   */
/* ---------------------------------------------------------------------- */
typedef struct batch_job {
  const rpo_config* c;
  int encode;
  const uint16_t* in16;
  const uint8_t* in8;
  const uint64_t* in_off;
  const uint64_t* in_len; /* decode: bytes; encode: samples */
  uint16_t* out16;
  uint8_t* out8;
  const uint64_t* out_off;
  const uint64_t* out_len; /* encode: capacity bytes; decode: samples */
  uint64_t* result;        /* encode: bytes written */
  int32_t* status;
  size_t nblocks;
  size_t next;
  pthread_mutex_t mu;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t b = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (b >= j->nblocks) break;
    if (j->encode) {
      size_t len = 0;
      j->status[b] = rpo_encode(j->c, j->in16 + j->in_off[b], j->in_len[b],
                                j->out8 + j->out_off[b], j->out_len[b], &len);
      j->result[b] = len;
    } else {
      j->status[b] = rpo_decode(j->c, j->in8 + j->in_off[b], j->in_len[b],
                                j->out16 + j->out_off[b], j->out_len[b]);
    }
  }
  return NULL;
}

static void run_batch(batch_job* j, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  pthread_mutex_init(&j->mu, NULL);
  j->next = 0;
  for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, batch_worker, j);
  batch_worker(j);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&j->mu);
}

/* in_off/n_samples in samples; out_off/out_cap in bytes. */
void rpo_encode_batch(const rpo_config* c, const uint16_t* in, const uint64_t* in_off,
                      const uint64_t* n_samples, size_t nblocks, uint8_t* out,
                      const uint64_t* out_off, const uint64_t* out_cap, uint64_t* out_bytes,
                      int32_t* status, int nthreads) {
  batch_job j;
  memset(&j, 0, sizeof j);
  j.c = c;
  j.encode = 1;
  j.in16 = in;
  j.in_off = in_off;
  j.in_len = n_samples;
  j.out8 = out;
  j.out_off = out_off;
  j.out_len = out_cap;
  j.result = out_bytes;
  j.status = status;
  j.nblocks = nblocks;
  run_batch(&j, nthreads);
}

/* in_off/in_bytes in bytes; out_off/n_samples in samples. */
void rpo_decode_batch(const rpo_config* c, const uint8_t* in, const uint64_t* in_off,
                      const uint64_t* in_bytes, size_t nblocks, uint16_t* out,
                      const uint64_t* out_off, const uint64_t* n_samples, int32_t* status,
                      int nthreads) {
  batch_job j;
  memset(&j, 0, sizeof j);
  j.c = c;
  j.encode = 0;
  j.in8 = in;
  j.in_off = in_off;
  j.in_len = in_bytes;
  j.out16 = out;
  j.out_off = out_off;
  j.out_len = n_samples;
  j.status = status;
  j.nblocks = nblocks;
  run_batch(&j, nthreads);
}

/* ---------------------------------------------------------------------- */
/* DwarFS ricepp block framing (src/compression/ricepp.cpp:107-127):       */
/* varint(uncompressed bytes) (src/varint.cpp:39-51, LEB128) followed by   */
/* a thrift-compact ricepp_block_header (thrift/compression.thrift:42-49,  */
/* src/thrift_lite/compact_writer.cpp:92-162).                              */
/* ---------------------------------------------------------------------- */
static size_t put_varint(uint8_t* p, uint64_t v) {
  size_t n = 0;
  while (v >= 0x80) {
    p[n++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  p[n++] = (uint8_t)v;
  return n;
}

static uint64_t zigzag(int64_t v) { return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }

/* Writes the framing prefix; returns its length (<= 32 bytes). */
size_t rpo_frame_header(uint8_t* out, uint64_t uncompressed_bytes, uint32_t block_size,
                        uint32_t component_count, uint32_t bytes_per_sample,
                        uint32_t unused_lsb_count, int big_endian, uint32_t version) {
  size_t n = put_varint(out, uncompressed_bytes);
  out[n++] = 0x15; /* field 1, delta 1, i32 */
  n += put_varint(out + n, zigzag((int32_t)block_size));
  out[n++] = 0x14; /* field 2, i16 */
  n += put_varint(out + n, zigzag((int16_t)component_count));
  out[n++] = 0x13; /* field 3, byte */
  out[n++] = (uint8_t)bytes_per_sample;
  out[n++] = 0x13; /* field 4, byte */
  out[n++] = (uint8_t)unused_lsb_count;
  out[n++] = big_endian ? 0x11 : 0x12; /* field 5, bool true/false */
  out[n++] = 0x14;                     /* field 6, i16 */
  n += put_varint(out + n, zigzag((int16_t)version));
  out[n++] = 0x00; /* stop */
  return n;
}
