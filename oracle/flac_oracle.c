/*
 * flac_oracle.c -- CPU restatement of the FLAC bitstream (RFC 9639) for the
 * tests of the GPU FLAC block codec (dwarfs_amd/csrc/flac_kernels.hip).
 *
 * TEST INFRASTRUCTURE ONLY: linked by tests/ (through oracle/flac.py) as the
 * independent encoder and decoder the GPU codec is checked against.  The
 * product path never loads it.
 *
 * PARITY UNPINNED.  The reference compresses FLAC blocks with libFLAC
 * (src/compression/flac.cpp:215-403 via FLAC++ 1.x, "level 5", blocksize
 * 4096 through process_interleaved, :325-345) and decodes them with libFLAC's
 * stream decoder (:107-213, :405-489).  libFLAC is not in this image and the
 * reference holds no FLAC bitstream fixture, so neither this file nor the GPU
 * codec can be compared with libFLAC's bytes.  What is pinned instead: the
 * format itself (RFC 9639 sections 8 and 9, restated below), round trips of
 * every subframe kind both ways (this encoder -> GPU decoder, GPU encoder ->
 * this decoder), and the reference's own round-trip test shapes
 * (test/flac_compressor_test.cpp:97-205).
 *
 * Restated format (MSB-first bit order throughout):
 *   stream   "fLaC", metadata blocks (1 bit last, 7 bits type, 24 bits length),
 *            STREAMINFO first (type 0, 34 bytes), then frames
 *   frame    header: sync 0b11111111111110, reserved 0, blocking strategy (1 bit);
 *            block size code (4), sample rate code (4), channel assignment (4),
 *            sample size code (3), reserved 0; coded frame / sample number
 *            ("UTF-8"); optional 8 / 16-bit block size - 1 and sample rate;
 *            CRC-8 (poly 0x07) of the header.  Subframes, zero padding to a
 *            byte, CRC-16 (poly 0x8005) of the frame.
 *   subframe 0 pad bit, 6-bit type (0 constant, 1 verbatim, 8+o fixed order o
 *            <= 4, 32+o-1 LPC order o <= 32), wasted-bits flag (+ unary k-1);
 *            samples of bps - wasted (+1 for a side channel) bits.
 *   residual 2-bit method (0: 4-bit Rice parameters, 1: 5-bit), 4-bit
 *            partition order; per partition a parameter (all ones: escape,
 *            5-bit raw width then raw signed values) and Rice codes of the
 *            folded residual u = 2r (r >= 0) / -2r-1: u >> k zeros, a one,
 *            the k low bits.
 *   stereo   8 left/side, 9 side/right, 10 mid/side (side = L - R,
 *            mid = (L + R) >> 1).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define FO_OK 0
#define FO_TRUNCATED (-2)
#define FO_INVALID (-3)
#define FO_TOO_SMALL (-4)
#define FO_BAD_STREAM (-7)

typedef struct {
  int subframe_type;     /* 0 auto, 1 constant, 2 verbatim, 3 fixed, 4 lpc */
  int fixed_order;       /* 0..4 (type 3) */
  int lpc_order;         /* 1..32 (type 4; auto tries 1..8) */
  int lpc_precision;     /* 1..15 bits of the quantized coefficients (0: 12) */
  int stereo;            /* -1 auto, 0 independent, 8 / 9 / 10 forced (2 channels) */
  int max_partition_order; /* 0..15 */
  int rice2;             /* 1: method 1 (5-bit parameters) */
  int escape;            /* 1: every partition escaped (raw residuals) */
  int padding_block;     /* 1: a PADDING metadata block after STREAMINFO */
  int wasted;            /* 1: detect wasted low bits */
  int variable_blocking; /* 1: blocking strategy 1 (sample numbers) */
  int max_lpc_order;     /* auto: LPC orders 1..this (0: fixed predictors only) */
} fo_opts;

/* ---- CRCs ---- */
static uint8_t crc8_tab[256];
static uint16_t crc16_tab[256];
static int crc_ready = 0;
static void crc_init(void) {
  if (crc_ready) return;
  for (int i = 0; i < 256; ++i) {
    uint8_t c = (uint8_t)i;
    for (int k = 0; k < 8; ++k) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : c << 1);
    crc8_tab[i] = c;
    uint16_t d = (uint16_t)(i << 8);
    for (int k = 0; k < 8; ++k) d = (uint16_t)((d & 0x8000) ? (d << 1) ^ 0x8005 : d << 1);
    crc16_tab[i] = d;
  }
  crc_ready = 1;
}
static uint8_t crc8(const uint8_t* p, size_t n) {
  uint8_t c = 0;
  for (size_t i = 0; i < n; ++i) c = crc8_tab[c ^ p[i]];
  return c;
}
static uint16_t crc16(const uint8_t* p, size_t n) {
  uint16_t c = 0;
  for (size_t i = 0; i < n; ++i) c = (uint16_t)((c << 8) ^ crc16_tab[(c >> 8) ^ p[i]]);
  return c;
}

/* ---- bit writer (zeroed buffer, MSB first) ---- */
typedef struct {
  uint8_t* buf;
  size_t cap; /* bytes */
  uint64_t pos; /* bits */
  int overflow;
} bw_t;
static void bw_put(bw_t* w, uint64_t v, unsigned n) {
  if (w->pos + n > 8ull * w->cap) {
    w->overflow = 1;
    return;
  }
  for (unsigned i = n; i-- > 0;) {
    if ((v >> i) & 1u) w->buf[w->pos >> 3] |= (uint8_t)(0x80u >> (w->pos & 7));
    ++w->pos;
  }
}
static void bw_signed(bw_t* w, int64_t v, unsigned n) {
  bw_put(w, n == 64 ? (uint64_t)v : ((uint64_t)v & ((1ull << n) - 1)), n);
}
static void bw_unary(bw_t* w, uint64_t q) {
  if (w->pos + q + 1 > 8ull * w->cap) {
    w->overflow = 1;
    return;
  }
  w->pos += q;
  bw_put(w, 1, 1);
}
static void bw_align(bw_t* w) { w->pos = (w->pos + 7) & ~7ull; }
static void bw_utf8(bw_t* w, uint64_t v) {
  if (v < 0x80) {
    bw_put(w, v, 8);
    return;
  }
  int n = v < 0x800 ? 2 : v < 0x10000 ? 3 : v < 0x200000 ? 4 : v < 0x4000000 ? 5 : v < 0x80000000ull ? 6 : 7;
  if (n == 7) {
    bw_put(w, 0xFE, 8);
  } else {
    const unsigned lead = (0xFF00u >> n) & 0xFFu;
    bw_put(w, lead | (v >> (6 * (n - 1))), 8);
  }
  for (int i = n - 2; i >= 0; --i) bw_put(w, 0x80 | ((v >> (6 * i)) & 0x3F), 8);
}

/* ---- bit reader ---- */
typedef struct {
  const uint8_t* buf;
  size_t len; /* bytes */
  uint64_t pos;
  int err;
} br_t;
static uint64_t br_get(br_t* r, unsigned n) {
  if (r->pos + n > 8ull * r->len) {
    r->err = FO_TRUNCATED;
    r->pos = 8ull * r->len;
    return 0;
  }
  uint64_t v = 0;
  for (unsigned i = 0; i < n; ++i) {
    v = (v << 1) | ((r->buf[r->pos >> 3] >> (7 - (r->pos & 7))) & 1u);
    ++r->pos;
  }
  return v;
}
static int64_t br_signed(br_t* r, unsigned n) {
  if (n == 0) return 0;
  uint64_t v = br_get(r, n);
  if (n < 64 && (v >> (n - 1)) & 1u) v |= ~0ull << n;
  return (int64_t)v;
}
static uint64_t br_unary(br_t* r) {
  uint64_t q = 0;
  for (;;) {
    if (r->pos >= 8ull * r->len) {
      r->err = FO_TRUNCATED;
      return q;
    }
    if ((r->buf[r->pos >> 3] >> (7 - (r->pos & 7))) & 1u) {
      ++r->pos;
      return q;
    }
    ++r->pos;
    ++q;
  }
}
static int br_utf8(br_t* r, uint64_t* out) {
  uint64_t b = br_get(r, 8);
  int n;
  if (!(b & 0x80)) {
    *out = b;
    return 0;
  }
  if (b == 0xFE) {
    n = 7;
    b = 0;
  } else if ((b & 0xE0) == 0xC0) {
    n = 2;
    b &= 0x1F;
  } else if ((b & 0xF0) == 0xE0) {
    n = 3;
    b &= 0x0F;
  } else if ((b & 0xF8) == 0xF0) {
    n = 4;
    b &= 0x07;
  } else if ((b & 0xFC) == 0xF8) {
    n = 5;
    b &= 0x03;
  } else if ((b & 0xFE) == 0xFC) {
    n = 6;
    b &= 0x01;
  } else {
    return FO_BAD_STREAM;
  }
  for (int i = 1; i < n; ++i) {
    uint64_t c = br_get(r, 8);
    if ((c & 0xC0) != 0x80) return FO_BAD_STREAM;
    b = (b << 6) | (c & 0x3F);
  }
  *out = b;
  return r->err;
}

/* ---- residual coding ---- */
static uint64_t fold(int64_t r) { return r >= 0 ? (uint64_t)r << 1 : ((uint64_t)(-(r + 1)) << 1) | 1u; }
static unsigned signed_width(int64_t v) { /* bits of the two's complement form */
  unsigned n = 1;
  while (n < 64 && !(v >= -(1ll << (n - 1)) && v < (1ll << (n - 1)))) ++n;
  return n;
}

/* exact bits of a partition at parameter k, or of its escape (k = -1) */
static uint64_t part_bits(const int64_t* r, uint32_t n, int k, unsigned pbits) {
  if (k < 0) {
    unsigned wmax = 0;
    for (uint32_t i = 0; i < n; ++i) {
      unsigned w = r[i] ? signed_width(r[i]) : 0;
      if (w > wmax) wmax = w;
    }
    if (wmax > 31) return ~0ull >> 2; /* the 5-bit width field holds 0..31 */
    return pbits + 5 + (uint64_t)wmax * n;
  }
  uint64_t b = pbits;
  for (uint32_t i = 0; i < n; ++i) b += (fold(r[i]) >> k) + 1 + (unsigned)k;
  return b;
}

/* residual section for samples [order, bs) of res (res[i] for i >= order);
   returns bits (write = 0: cost only).  Method 0 (4-bit parameters) unless
   asked for method 1 or cheaper with it (parameters above 14). */
static uint64_t code_residual_m(bw_t* w, const int64_t* res, uint32_t bs, uint32_t order, const fo_opts* o, int write,
                                int method) {
  const unsigned pbits = method ? 5 : 4;
  const int kmax = method ? 30 : 14;
  uint64_t best = ~0ull;
  int best_po = 0;
  for (int po = 0; po <= o->max_partition_order; ++po) {
    if (bs % (1u << po) || (bs >> po) < order || ((bs >> po) == order && po > 0)) break;
    uint64_t tot = 6;
    for (uint32_t p = 0; p < (1u << po); ++p) {
      const uint32_t lo = p == 0 ? order : p * (bs >> po), hi = (p + 1) * (bs >> po);
      uint64_t pb = part_bits(res + lo, hi - lo, -1, pbits);
      if (!o->escape || pb >= (~0ull >> 2))
        for (int k = 0; k <= kmax; ++k) {
          const uint64_t b = part_bits(res + lo, hi - lo, k, pbits);
          if (b < pb) pb = b;
        }
      tot += pb;
    }
    if (tot < best) {
      best = tot;
      best_po = po;
    }
  }
  if (!write) return best;
  bw_put(w, (uint64_t)method, 2);
  bw_put(w, (uint64_t)best_po, 4);
  for (uint32_t p = 0; p < (1u << best_po); ++p) {
    const uint32_t lo = p == 0 ? order : p * (bs >> best_po), hi = (p + 1) * (bs >> best_po);
    int bk = -1;
    uint64_t pb = part_bits(res + lo, hi - lo, -1, pbits);
    if (!o->escape || pb >= (~0ull >> 2))
      for (int k = 0; k <= kmax; ++k) {
        const uint64_t b = part_bits(res + lo, hi - lo, k, pbits);
        if (b < pb) {
          pb = b;
          bk = k;
        }
      }
    if (bk < 0) {
      unsigned wmax = 0;
      for (uint32_t i = lo; i < hi; ++i) {
        unsigned wd = res[i] ? signed_width(res[i]) : 0;
        if (wd > wmax) wmax = wd;
      }
      bw_put(w, (1u << pbits) - 1, pbits);
      bw_put(w, wmax, 5);
      for (uint32_t i = lo; i < hi; ++i) bw_signed(w, res[i], wmax);
    } else {
      bw_put(w, (uint64_t)bk, pbits);
      for (uint32_t i = lo; i < hi; ++i) {
        const uint64_t u = fold(res[i]);
        bw_unary(w, u >> bk);
        if (bk) bw_put(w, u & ((1ull << bk) - 1), (unsigned)bk);
      }
    }
  }
  return best;
}
static uint64_t code_residual(bw_t* w, const int64_t* res, uint32_t bs, uint32_t order, const fo_opts* o, int write) {
  int method = 1;
  if (!o->rice2) {
    const uint64_t b0 = code_residual_m(NULL, res, bs, order, o, 0, 0);
    const uint64_t b1 = code_residual_m(NULL, res, bs, order, o, 0, 1);
    method = b1 < b0 ? 1 : 0;
  }
  return code_residual_m(w, res, bs, order, o, write, method);
}

static const int64_t fixed_coef[5][4] = {{0, 0, 0, 0}, {1, 0, 0, 0}, {2, -1, 0, 0}, {3, -3, 1, 0}, {4, -6, 4, -1}};
static int fixed_residual(const int64_t* s, uint32_t bs, int order, int64_t* res) {
  for (uint32_t i = (uint32_t)order; i < bs; ++i) {
    int64_t p = 0;
    for (int j = 0; j < order; ++j) p += fixed_coef[order][j] * s[i - 1 - j];
    res[i] = s[i] - p;
    if (res[i] < INT32_MIN || res[i] > INT32_MAX) return 0;
  }
  return 1;
}

/* LPC of `order` by autocorrelation + Levinson-Durbin, quantized to
   `prec` bits; 0 if it cannot code this block */
static int lpc_residual(const int64_t* s, uint32_t bs, int order, int prec, int32_t* q, int* shift, int64_t* res) {
  double ac[33] = {0}, lpc[33] = {0}, tmp[33];
  if ((uint32_t)order >= bs) return 0;
  for (int l = 0; l <= order; ++l)
    for (uint32_t i = (uint32_t)l; i < bs; ++i) ac[l] += (double)s[i] * (double)s[i - l];
  if (ac[0] <= 0) return 0;
  double err = ac[0];
  for (int i = 0; i < order; ++i) {
    double acc = ac[i + 1];
    for (int j = 0; j < i; ++j) acc -= lpc[j] * ac[i - j];
    const double k = err != 0 ? acc / err : 0;
    for (int j = 0; j < i; ++j) tmp[j] = lpc[j] - k * lpc[i - 1 - j];
    for (int j = 0; j < i; ++j) lpc[j] = tmp[j];
    lpc[i] = k;
    err *= 1 - k * k;
  }
  double cmax = 0;
  for (int j = 0; j < order; ++j) cmax = fabs(lpc[j]) > cmax ? fabs(lpc[j]) : cmax;
  if (cmax <= 0) return 0;
  int e;
  frexp(cmax, &e);
  int sh = prec - 1 - e;
  if (sh > 15) sh = 15;
  if (sh < 0) return 0;
  const int32_t qmax = (1 << (prec - 1)) - 1, qmin = -(1 << (prec - 1));
  double carry = 0;
  for (int j = 0; j < order; ++j) {
    double v = lpc[j] * (double)(1 << sh) + carry;
    long r = lround(v);
    if (r > qmax) r = qmax;
    if (r < qmin) r = qmin;
    carry = v - (double)r;
    q[j] = (int32_t)r;
  }
  *shift = sh;
  for (uint32_t i = (uint32_t)order; i < bs; ++i) {
    int64_t p = 0;
    for (int j = 0; j < order; ++j) p += (int64_t)q[j] * s[i - 1 - j];
    res[i] = s[i] - (p >> sh);
    if (res[i] < INT32_MIN || res[i] > INT32_MAX) return 0;
  }
  return 1;
}

/* one subframe of samples s (bits sbps); returns 0 on overflow */
static int code_subframe(bw_t* w, const int64_t* s0, uint32_t bs, unsigned sbps, const fo_opts* o, int64_t* sc,
                         int64_t* res, int64_t* res2) {
  /* wasted bits */
  unsigned wasted = 0;
  if (o->wasted) {
    uint64_t acc = 0;
    for (uint32_t i = 0; i < bs; ++i) acc |= (uint64_t)s0[i];
    if (acc)
      while (!((acc >> wasted) & 1u) && wasted < sbps - 1) ++wasted;
  }
  for (uint32_t i = 0; i < bs; ++i) sc[i] = s0[i] >> wasted;
  const int64_t* s = sc;
  const unsigned bps = sbps - wasted;
  int type = o->subframe_type;
  int order = 0, prec = o->lpc_precision ? o->lpc_precision : 12, shift = 0;
  int32_t q[32];
  if (type == 1) { /* forced constant: only where it is exact */
    for (uint32_t i = 1; i < bs && type == 1; ++i)
      if (s[i] != s[0]) type = 0;
  }
  if (type == 0) {
    int same = 1;
    for (uint32_t i = 1; i < bs && same; ++i) same = s[i] == s[0];
    if (same) {
      type = 1;
    } else {
      uint64_t best = (uint64_t)bps * bs;
      type = 2;
      for (int fo = 0; fo <= 4 && (uint32_t)fo < bs; ++fo) {
        if (!fixed_residual(s, bs, fo, res)) continue;
        const uint64_t b = (uint64_t)fo * bps + code_residual(NULL, res, bs, (uint32_t)fo, o, 0);
        if (b < best) {
          best = b;
          type = 3;
          order = fo;
        }
      }
      for (int lo = 1; lo <= o->max_lpc_order && (uint32_t)lo < bs; ++lo) {
        int32_t qq[32];
        int sh;
        if (!lpc_residual(s, bs, lo, prec, qq, &sh, res)) continue;
        const uint64_t b = (uint64_t)lo * bps + 9 + (uint64_t)lo * prec + code_residual(NULL, res, bs, (uint32_t)lo, o, 0);
        if (b < best) {
          best = b;
          type = 4;
          order = lo;
        }
      }
    }
  } else if (type == 3) {
    order = o->fixed_order;
    if ((uint32_t)order > bs || !fixed_residual(s, bs, order, res)) type = 2;
  } else if (type == 4) {
    order = o->lpc_order;
    if ((uint32_t)order >= bs || !lpc_residual(s, bs, order, prec, q, &shift, res)) type = 2;
  }
  bw_put(w, 0, 1);
  switch (type) {
    case 1: bw_put(w, 0, 6); break;
    case 2: bw_put(w, 1, 6); break;
    case 3: bw_put(w, 8u + (unsigned)order, 6); break;
    default: bw_put(w, 32u + (unsigned)order - 1, 6); break;
  }
  if (wasted) {
    bw_put(w, 1, 1);
    bw_unary(w, wasted - 1);
  } else {
    bw_put(w, 0, 1);
  }
  if (type == 1) {
    bw_signed(w, s[0], bps);
  } else if (type == 2) {
    for (uint32_t i = 0; i < bs; ++i) bw_signed(w, s[i], bps);
  } else if (type == 3) {
    fixed_residual(s, bs, order, res);
    for (int i = 0; i < order; ++i) bw_signed(w, s[i], bps);
    code_residual(w, res, bs, (uint32_t)order, o, 1);
  } else {
    lpc_residual(s, bs, order, prec, q, &shift, res2);
    for (int i = 0; i < order; ++i) bw_signed(w, s[i], bps);
    bw_put(w, (uint64_t)(prec - 1), 4);
    bw_signed(w, shift, 5);
    for (int i = 0; i < order; ++i) bw_signed(w, q[i], (unsigned)prec);
    code_residual(w, res2, bs, (uint32_t)order, o, 1);
  }
  return !w->overflow;
}

static unsigned bs_code(uint32_t bs, int* extra) {
  *extra = 0;
  if (bs == 192) return 1;
  for (unsigned c = 2; c <= 5; ++c)
    if (bs == 576u << (c - 2)) return c;
  for (unsigned c = 8; c <= 15; ++c)
    if (bs == 256u << (c - 8)) return c;
  if (bs <= 256) {
    *extra = 8;
    return 6;
  }
  *extra = 16;
  return 7;
}
static unsigned ss_code(unsigned bps) {
  switch (bps) {
    case 8: return 1;
    case 12: return 2;
    case 16: return 4;
    case 20: return 5;
    case 24: return 6;
    case 32: return 7;
    default: return 0;
  }
}

/* Encodes a whole FLAC stream; returns its size, 0 if `cap` is too small or
   the arguments are invalid. */
size_t fo_encode(const int32_t* x, uint64_t nsamples, uint32_t channels, uint32_t bps, uint32_t blocksize,
                 const fo_opts* opts, uint8_t* out, size_t cap) {
  crc_init();
  fo_opts o = *opts;
  if (channels < 1 || channels > 8 || bps < 4 || bps > 32 || blocksize < 16 || blocksize > 65535) return 0;
  if (o.max_partition_order > 15) o.max_partition_order = 15;
  memset(out, 0, cap);
  bw_t w = {out, cap, 0, 0};
  bw_put(&w, 0x664C6143u, 32); /* "fLaC" */
  bw_put(&w, o.padding_block ? 0 : 1, 1);
  bw_put(&w, 0, 7);
  bw_put(&w, 34, 24);
  bw_put(&w, blocksize, 16);
  bw_put(&w, blocksize, 16);
  bw_put(&w, 0, 24);
  bw_put(&w, 0, 24);
  bw_put(&w, 48000, 20);
  bw_put(&w, channels - 1, 3);
  bw_put(&w, bps - 1, 5);
  bw_put(&w, nsamples >> 32, 4);
  bw_put(&w, nsamples & 0xFFFFFFFFu, 32);
  for (int i = 0; i < 4; ++i) bw_put(&w, 0, 32); /* MD5 unknown */
  if (o.padding_block) {
    bw_put(&w, 1, 1);
    bw_put(&w, 1, 7);
    bw_put(&w, 13, 24);
    w.pos += 13 * 8;
  }
  int64_t* ch = malloc(sizeof(int64_t) * blocksize * (channels + 2));
  int64_t* sc = malloc(sizeof(int64_t) * blocksize);
  int64_t* res = malloc(sizeof(int64_t) * blocksize);
  int64_t* res2 = malloc(sizeof(int64_t) * blocksize);
  uint8_t* tmp = malloc(8 * (size_t)blocksize * (channels + 1) + 64);
  size_t result = 0;
  if (!ch || !sc || !res || !res2 || !tmp) goto done;
  for (uint64_t f0 = 0, fn = 0; f0 < nsamples; f0 += blocksize, ++fn) {
    const uint32_t bs = (uint32_t)(nsamples - f0 < blocksize ? nsamples - f0 : blocksize);
    for (uint32_t c = 0; c < channels; ++c)
      for (uint32_t i = 0; i < bs; ++i) ch[(size_t)c * blocksize + i] = x[(f0 + i) * channels + c];
    /* stereo decorrelation: the smallest of the four (exact costs) */
    int assign = (int)channels - 1;
    if (channels == 2 && o.stereo != 0 && bps < 32) {
      int64_t* side = ch + 2 * (size_t)blocksize;
      int64_t* mid = ch + 3 * (size_t)blocksize;
      for (uint32_t i = 0; i < bs; ++i) {
        side[i] = ch[i] - ch[blocksize + i];
        mid[i] = (ch[i] + ch[blocksize + i]) >> 1;
      }
      if (o.stereo > 0) {
        assign = o.stereo;
      } else {
        uint64_t cost[4];
        const int64_t* src[4] = {ch, ch + blocksize, side, mid};
        const unsigned sb[4] = {bps, bps, bps + 1, bps};
        for (int k = 0; k < 4; ++k) {
          memset(tmp, 0, 8 * (size_t)blocksize + 64);
          bw_t t = {tmp, 8 * (size_t)blocksize + 64, 0, 0};
          code_subframe(&t, src[k], bs, sb[k], &o, sc, res, res2);
          cost[k] = t.overflow ? ~0ull : t.pos;
        }
        const uint64_t c_ind = cost[0] + cost[1], c_ls = cost[0] + cost[2], c_rs = cost[2] + cost[1],
                       c_ms = cost[3] + cost[2];
        uint64_t best = c_ind;
        assign = 1;
        if (c_ls < best) best = c_ls, assign = 8;
        if (c_rs < best) best = c_rs, assign = 9;
        if (c_ms < best) best = c_ms, assign = 10;
      }
    }
    const uint64_t start = w.pos;
    int extra;
    const unsigned bcode = bs_code(bs, &extra);
    bw_put(&w, 0x3FFE, 14);
    bw_put(&w, 0, 1);
    bw_put(&w, o.variable_blocking ? 1 : 0, 1);
    bw_put(&w, bcode, 4);
    bw_put(&w, 10, 4); /* 48 kHz */
    bw_put(&w, (uint64_t)assign, 4);
    bw_put(&w, ss_code(bps), 3);
    bw_put(&w, 0, 1);
    bw_utf8(&w, o.variable_blocking ? f0 : fn);
    if (extra) bw_put(&w, bs - 1, (unsigned)extra);
    if (w.overflow) goto done;
    bw_put(&w, crc8(out + (start >> 3), (size_t)((w.pos - start) >> 3)), 8);
    for (uint32_t c = 0; c < channels; ++c) {
      const int64_t* src = ch + (size_t)c * blocksize;
      unsigned sb = bps;
      if (assign == 8 && c == 1) src = ch + 2 * (size_t)blocksize, sb = bps + 1;
      if (assign == 9 && c == 0) src = ch + 2 * (size_t)blocksize, sb = bps + 1;
      if (assign == 10) src = c == 0 ? ch + 3 * (size_t)blocksize : ch + 2 * (size_t)blocksize, sb = c == 0 ? bps : bps + 1;
      if (!code_subframe(&w, src, bs, sb, &o, sc, res, res2)) goto done;
    }
    bw_align(&w);
    if (w.overflow || w.pos + 16 > 8ull * cap) goto done;
    bw_put(&w, crc16(out + (start >> 3), (size_t)((w.pos - start) >> 3)), 16);
  }
  result = (size_t)(w.pos >> 3);
done:
  free(ch);
  free(sc);
  free(res);
  free(res2);
  free(tmp);
  return result;
}

/* ---- decoder ---- */
static int decode_residual(br_t* r, int64_t* res, uint32_t bs, uint32_t order) {
  const unsigned method = (unsigned)br_get(r, 2);
  if (method > 1) return FO_BAD_STREAM;
  const unsigned pbits = method ? 5 : 4;
  const unsigned po = (unsigned)br_get(r, 4);
  if (bs % (1u << po) || (bs >> po) < order) return FO_BAD_STREAM;
  for (uint32_t p = 0; p < (1u << po); ++p) {
    const uint32_t lo = p == 0 ? order : p * (bs >> po), hi = (p + 1) * (bs >> po);
    const unsigned k = (unsigned)br_get(r, pbits);
    if (k == (1u << pbits) - 1) {
      const unsigned n = (unsigned)br_get(r, 5);
      for (uint32_t i = lo; i < hi; ++i) res[i] = br_signed(r, n);
    } else {
      for (uint32_t i = lo; i < hi; ++i) {
        const uint64_t q = br_unary(r);
        if (r->err) return r->err;
        const uint64_t u = (q << k) | br_get(r, k);
        res[i] = (u & 1u) ? -(int64_t)(u >> 1) - 1 : (int64_t)(u >> 1);
      }
    }
    if (r->err) return r->err;
  }
  return FO_OK;
}

static int fo_trace = 0; /* FO_TRACE=1: one line per subframe on stderr (diagnostics) */
static int decode_subframe(br_t* r, int64_t* s, uint32_t bs, unsigned sbps) {
  const uint64_t at = r->pos;
  if (br_get(r, 1)) return FO_BAD_STREAM;
  const unsigned type = (unsigned)br_get(r, 6);
  unsigned wasted = 0;
  if (br_get(r, 1)) wasted = (unsigned)br_unary(r) + 1;
  if (fo_trace)
    fprintf(stderr, "  subframe at bit %llu: type %u wasted %u bs %u sbps %u\n", (unsigned long long)at, type, wasted,
            bs, sbps);
  if (r->err) return r->err;
  if (wasted >= sbps) return FO_BAD_STREAM;
  const unsigned bps = sbps - wasted;
  if (type == 0) {
    const int64_t v = br_signed(r, bps);
    for (uint32_t i = 0; i < bs; ++i) s[i] = v;
  } else if (type == 1) {
    for (uint32_t i = 0; i < bs; ++i) s[i] = br_signed(r, bps);
  } else if (type >= 8 && type <= 12) {
    const uint32_t order = type - 8;
    if (order > bs) return FO_BAD_STREAM;
    for (uint32_t i = 0; i < order; ++i) s[i] = br_signed(r, bps);
    int e = decode_residual(r, s, bs, order);
    if (e) return e;
    for (uint32_t i = order; i < bs; ++i) {
      int64_t p = 0;
      for (uint32_t j = 0; j < order; ++j) p += fixed_coef[order][j] * s[i - 1 - j];
      s[i] += p;
    }
  } else if (type >= 32) {
    const uint32_t order = type - 31;
    if (order > bs) return FO_BAD_STREAM;
    for (uint32_t i = 0; i < order; ++i) s[i] = br_signed(r, bps);
    const unsigned prec = (unsigned)br_get(r, 4) + 1;
    if (prec == 16) return FO_BAD_STREAM;
    const int shift = (int)br_signed(r, 5);
    if (shift < 0) return FO_BAD_STREAM;
    int64_t q[32];
    for (uint32_t j = 0; j < order; ++j) q[j] = br_signed(r, prec);
    int e = decode_residual(r, s, bs, order);
    if (e) return e;
    for (uint32_t i = order; i < bs; ++i) {
      int64_t p = 0;
      for (uint32_t j = 0; j < order; ++j) p += q[j] * s[i - 1 - j];
      s[i] += p >> shift;
    }
  } else {
    return FO_BAD_STREAM;
  }
  if (r->err) return r->err;
  if (wasted)
    for (uint32_t i = 0; i < bs; ++i) s[i] = (int64_t)((uint64_t)s[i] << wasted);
  return FO_OK;
}

/* Decodes a whole FLAC stream into interleaved samples (at most `cap`
   values); returns FO_OK and the stream's shape, or an error. */
int fo_decode(const uint8_t* in, size_t len, int32_t* out, uint64_t cap, uint32_t* channels_out, uint32_t* bps_out,
              uint64_t* nsamples_out) {
  crc_init();
  fo_trace = getenv("FO_TRACE") != NULL;
  br_t r = {in, len, 0, 0};
  if (br_get(&r, 32) != 0x664C6143u) return r.err ? r.err : FO_BAD_STREAM;
  uint32_t channels = 0, bps = 0, maxbs = 0;
  uint64_t total = 0;
  for (int last = 0; !last;) {
    last = (int)br_get(&r, 1);
    const unsigned type = (unsigned)br_get(&r, 7);
    const uint32_t blen = (uint32_t)br_get(&r, 24);
    if (r.err) return r.err;
    if (type == 0) {
      br_get(&r, 16);
      maxbs = (uint32_t)br_get(&r, 16);
      br_get(&r, 24);
      br_get(&r, 24);
      br_get(&r, 20);
      channels = (uint32_t)br_get(&r, 3) + 1;
      bps = (uint32_t)br_get(&r, 5) + 1;
      total = br_get(&r, 36);
      r.pos += 128;
    } else {
      r.pos += 8ull * blen;
    }
    if (r.pos > 8ull * len) return FO_TRUNCATED;
  }
  if (!channels) return FO_BAD_STREAM;
  int64_t* ch = malloc(sizeof(int64_t) * 65536 * 8);
  if (!ch) return FO_INVALID;
  uint64_t done = 0;
  int err = FO_OK;
  while (done < total) {
    const uint64_t start = r.pos;
    if (start & 7) {
      err = FO_BAD_STREAM;
      break;
    }
    if (br_get(&r, 14) != 0x3FFE || br_get(&r, 1)) {
      err = r.err ? r.err : FO_BAD_STREAM;
      break;
    }
    const unsigned variable = (unsigned)br_get(&r, 1);
    const unsigned bcode = (unsigned)br_get(&r, 4), rcode = (unsigned)br_get(&r, 4);
    const unsigned assign = (unsigned)br_get(&r, 4), scode = (unsigned)br_get(&r, 3);
    if (br_get(&r, 1)) {
      err = FO_BAD_STREAM;
      break;
    }
    uint64_t num;
    if (br_utf8(&r, &num)) {
      err = r.err ? r.err : FO_BAD_STREAM;
      break;
    }
    (void)variable;
    uint32_t bs;
    if (bcode == 0) {
      err = FO_BAD_STREAM;
      break;
    } else if (bcode == 1) {
      bs = 192;
    } else if (bcode <= 5) {
      bs = 576u << (bcode - 2);
    } else if (bcode == 6) {
      bs = (uint32_t)br_get(&r, 8) + 1;
    } else if (bcode == 7) {
      bs = (uint32_t)br_get(&r, 16) + 1;
    } else {
      bs = 256u << (bcode - 8);
    }
    if (rcode == 12) br_get(&r, 8);
    else if (rcode == 13 || rcode == 14) br_get(&r, 16);
    else if (rcode == 15) {
      err = FO_BAD_STREAM;
      break;
    }
    static const unsigned sizes[8] = {0, 8, 12, 0, 16, 20, 24, 32};
    const unsigned fbps = scode == 0 ? bps : sizes[scode];
    const uint32_t fch = assign < 8 ? assign + 1 : 2;
    if (assign > 10 || scode == 3 || fbps != bps || fch != channels) {
      err = FO_BAD_STREAM;
      break;
    }
    if (fo_trace)
      fprintf(stderr, "frame at byte %llu: bs %u assign %u samples %llu..\n", (unsigned long long)(start >> 3), bs,
              assign, (unsigned long long)done);
    const uint8_t hcrc = crc8(in + (start >> 3), (size_t)((r.pos - start) >> 3));
    if ((uint8_t)br_get(&r, 8) != hcrc) {
      err = r.err ? r.err : FO_BAD_STREAM;
      break;
    }
    (void)maxbs;
    if (bs > 65536 || done + bs > total || (done + bs) * channels > cap) {
      err = FO_BAD_STREAM;
      break;
    }
    for (uint32_t c = 0; c < fch && !err; ++c) {
      unsigned sb = bps;
      if ((assign == 8 && c == 1) || (assign == 9 && c == 0) || (assign == 10 && c == 1)) sb = bps + 1;
      err = decode_subframe(&r, ch + (size_t)c * 65536, bs, sb);
    }
    if (err) break;
    r.pos = (r.pos + 7) & ~7ull;
    const uint16_t fcrc = crc16(in + (start >> 3), (size_t)((r.pos - start) >> 3));
    if ((uint16_t)br_get(&r, 16) != fcrc) {
      err = r.err ? r.err : FO_BAD_STREAM;
      break;
    }
    int64_t* a = ch;
    int64_t* b = ch + 65536;
    for (uint32_t i = 0; i < bs; ++i) {
      int64_t L, R;
      if (assign == 8) {
        L = a[i], R = a[i] - b[i];
      } else if (assign == 9) {
        R = b[i], L = a[i] + b[i];
      } else if (assign == 10) {
        const int64_t m = (a[i] * 2) | (b[i] & 1);
        L = (m + b[i]) >> 1, R = (m - b[i]) >> 1;
      } else {
        L = a[i], R = b[i];
      }
      if (assign >= 8) {
        a[i] = L;
        b[i] = R;
      }
    }
    for (uint32_t i = 0; i < bs; ++i)
      for (uint32_t c = 0; c < channels; ++c) out[(done + i) * channels + c] = (int32_t)ch[(size_t)c * 65536 + i];
    done += bs;
  }
  free(ch);
  if (err) return err;
  *channels_out = channels;
  *bps_out = bps;
  *nsamples_out = total;
  return FO_OK;
}
