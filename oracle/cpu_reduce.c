/* cpu_reduce.c — ORACLE / TEST INFRASTRUCTURE ONLY (see cpu_reduce.h).
 *
 * Restates gloo/math.h:15-73 element by element:
 *   sum      c = a + b                       gloo/math.h:15-23
 *   product  c = a * b                       gloo/math.h:30-38
 *   max      c = std::max(a, b) = (a<b)?b:a  gloo/math.h:45-53
 *   min      c = std::min(a, b) = (b<a)?b:a  gloo/math.h:60-68
 * Integers: C++ promotes int8/uint8 to int and converts back modulo 2^8; the
 * 32/64-bit cases wrap as the hardware does — computed here in unsigned.
 * float16: the F16C path of gloo/math.cc:17-97 (vcvtph2ps, op in f32,
 * vcvtps2ph with imm 0 = round-to-nearest-even).  The scalar float16 path is
 * NOT restated: it is defective.
 * bfloat16: c10::BFloat16 (the type gloo/cuda.cu:394-401 instantiates): widen
 * by <<16, op in f32, round_to_nearest_even with NaN -> 0x7FC0.
 */
#include "cpu_reduce.h"

#include <pthread.h>
#include <string.h>

enum { I8, U8, I32, U32, I64, U64, F16, BF16, F32, F64 };
enum { SUM = 1, PRODUCT = 2, MAX = 3, MIN = 4 };

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* vcvtph2ps: exact; a NaN keeps sign and payload, quiet bit set. */
float oracle_f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000) << 16;
  const uint32_t exp = (h >> 10) & 0x1f;
  uint32_t mant = h & 0x3ff;
  if (exp == 0x1f) {
    if (mant) return u2f(sign | 0x7fc00000u | (mant << 13));
    return u2f(sign | 0x7f800000u);
  }
  if (exp == 0) {
    if (mant == 0) return u2f(sign);
    /* subnormal: mant * 2^-24 */
    int e = -14;
    while (!(mant & 0x400)) { mant <<= 1; e--; }
    mant &= 0x3ff;
    return u2f(sign | ((uint32_t)(e + 127) << 23) | (mant << 13));
  }
  return u2f(sign | ((exp - 15 + 127) << 23) | (mant << 13));
}

/* vcvtps2ph imm=0: round to nearest even; NaN -> quiet NaN, upper payload. */
uint16_t oracle_f32_to_f16(float f) {
  const uint32_t x = f2u(f);
  const uint16_t sign = (uint16_t)((x >> 16) & 0x8000);
  const uint32_t ax = x & 0x7fffffffu;
  if (ax > 0x7f800000u) return (uint16_t)(sign | 0x7e00 | ((ax >> 13) & 0x3ff));
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00); /* >= 65520 -> inf */
  if (ax >= 0x38800000u) {                                  /* normal half */
    const uint32_t mant = ax & 0x7fffff;
    uint32_t h = (((ax >> 23) - 112) << 10) | (mant >> 13);
    const uint32_t rem = mant & 0x1fff;
    if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) h++;
    return (uint16_t)(sign | h);
  }
  if (ax <= 0x33000000u) return sign; /* <= 2^-25 rounds to (signed) zero */
  {
    const uint32_t mant = (ax & 0x7fffff) | 0x800000;
    const int e = (int)(ax >> 23) - 127; /* in [-25, -15] */
    const int shift = -(e + 1);          /* value / 2^-24 = mant >> shift */
    uint32_t h = mant >> shift;
    const uint32_t rem = mant & ((1u << shift) - 1);
    const uint32_t half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1))) h++;
    return (uint16_t)(sign | h);
  }
}

float oracle_bf16_to_f32(uint16_t h) { return u2f((uint32_t)h << 16); }

uint16_t oracle_f32_to_bf16(float f) {
  if (f != f) return 0x7FC0;
  const uint32_t u = f2u(f);
  return (uint16_t)((u + (((u >> 16) & 1) + 0x7FFFu)) >> 16);
}

#define DEF_INT(NAME, S, U)                                                     \
  static void NAME(int op, S* c, const S* a, const S* b, size_t n) {           \
    size_t i;                                                                   \
    for (i = 0; i < n; i++) {                                                   \
      const S x = a[i], y = b[i];                                               \
      S r;                                                                      \
      if (op == SUM) r = (S)(U)((U)x + (U)y);                                   \
      else if (op == PRODUCT) r = (S)(U)((U)x * (U)y);                          \
      else if (op == MAX) r = (x < y) ? y : x;                                  \
      else r = (y < x) ? y : x;                                                 \
      c[i] = r;                                                                 \
    }                                                                           \
  }
DEF_INT(red_i8, int8_t, uint32_t)
DEF_INT(red_u8, uint8_t, uint32_t)
DEF_INT(red_i32, int32_t, uint32_t)
DEF_INT(red_u32, uint32_t, uint32_t)
DEF_INT(red_i64, int64_t, uint64_t)
DEF_INT(red_u64, uint64_t, uint64_t)

#define DEF_FLT(NAME, S)                                                        \
  static void NAME(int op, S* c, const S* a, const S* b, size_t n) {           \
    size_t i;                                                                   \
    for (i = 0; i < n; i++) {                                                   \
      const S x = a[i], y = b[i];                                               \
      S r;                                                                      \
      if (op == SUM) r = x + y;                                                 \
      else if (op == PRODUCT) r = x * y;                                        \
      else if (op == MAX) r = (x < y) ? y : x;                                  \
      else r = (y < x) ? y : x;                                                 \
      c[i] = r;                                                                 \
    }                                                                           \
  }
DEF_FLT(red_f32, float)
DEF_FLT(red_f64, double)

/* A NaN result of a 16-bit SUM / PRODUCT, stated explicitly rather than left
 * to the host's SSE NaN propagation:
 *  - fp16, the F16C body as the reference builds it (g++ -O3 -mavx -mf16c,
 *    gloo/math.cc:22-36): the second operand's NaN quietened, else the
 *    first's, else x86's default NaN 0xFE00 (inf - inf, 0 * inf).  Probed on
 *    oracle/_ref over every pair of signed payloads (oracle/gen_golden.py
 *    "f16_nan");
 *  - bf16: c10's round_to_nearest_even returns 0x7FC0 for any NaN. */
static inline int f16_nan(uint16_t x) { return (x & 0x7fff) > 0x7c00; }
static inline uint16_t nan_f16(uint16_t x, uint16_t y) {
  return f16_nan(y) ? (uint16_t)(y | 0x200) : f16_nan(x) ? (uint16_t)(x | 0x200) : 0xFE00;
}
static inline uint16_t nan_bf16(uint16_t x, uint16_t y) { (void)x; (void)y; return 0x7FC0; }

#define DEF_HALF(NAME, WIDEN, NARROW, NANOF)                                    \
  static void NAME(int op, uint16_t* c, const uint16_t* a, const uint16_t* b,   \
                   size_t n) {                                                  \
    size_t i;                                                                   \
    for (i = 0; i < n; i++) {                                                   \
      const uint16_t x = a[i], y = b[i];                                        \
      const float fx = WIDEN(x), fy = WIDEN(y);                                 \
      uint16_t r;                                                               \
      float f;                                                                  \
      if (op == SUM || op == PRODUCT) {                                         \
        f = op == SUM ? fx + fy : fx * fy;                                      \
        r = f != f ? NANOF(x, y) : NARROW(f);                                   \
      } else if (op == MAX) r = (fx < fy) ? y : x;                              \
      else r = (fy < fx) ? y : x;                                               \
      c[i] = r;                                                                 \
    }                                                                           \
  }
DEF_HALF(red_f16, oracle_f16_to_f32, oracle_f32_to_f16, nan_f16)
DEF_HALF(red_bf16, oracle_bf16_to_f32, oracle_f32_to_bf16, nan_bf16)

int oracle_reduce3(int op, int dtype, void* c, const void* a, const void* b, size_t n) {
  if (op < SUM || op > MIN) return -1;
  switch (dtype) {
    case I8: red_i8(op, c, a, b, n); return 0;
    case U8: red_u8(op, c, a, b, n); return 0;
    case I32: red_i32(op, c, a, b, n); return 0;
    case U32: red_u32(op, c, a, b, n); return 0;
    case I64: red_i64(op, c, a, b, n); return 0;
    case U64: red_u64(op, c, a, b, n); return 0;
    case F16: red_f16(op, c, a, b, n); return 0;
    case BF16: red_bf16(op, c, a, b, n); return 0;
    case F32: red_f32(op, c, a, b, n); return 0;
    case F64: red_f64(op, c, a, b, n); return 0;
  }
  return -2;
}

static const size_t kSizes[] = {1, 1, 4, 4, 8, 8, 2, 2, 4, 8};

int oracle_reduce_multi(int op, int dtype, void* dst, const void* const* srcs, int k,
                        size_t n) {
  int j, rc;
  if (dtype < 0 || dtype > F64) return -2;
  if (k < 1) return -4;
  if (dst != srcs[0]) memmove(dst, srcs[0], n * kSizes[dtype]);
  for (j = 1; j < k; j++) {
    rc = oracle_reduce3(op, dtype, dst, dst, srcs[j], n);
    if (rc) return rc;
  }
  return 0;
}

struct mt_arg {
  float* c;
  const float* a;
  const float* b;
  size_t n;
};

static void* mt_body(void* p) {
  struct mt_arg* m = (struct mt_arg*)p;
  red_f32(SUM, m->c, m->a, m->b, m->n);
  return NULL;
}

void oracle_sum_f32_mt(float* c, const float* a, const float* b, size_t n, int nthreads) {
  pthread_t th[256];
  struct mt_arg args[256];
  int t, used = 0;
  size_t per;
  if (nthreads <= 1) {
    red_f32(SUM, c, a, b, n);
    return;
  }
  if (nthreads > 256) nthreads = 256;
  per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
  for (t = 0; t < nthreads; t++) {
    const size_t lo = per * (size_t)t;
    if (lo >= n) break;
    args[t].c = c + lo;
    args[t].a = a + lo;
    args[t].b = b + lo;
    args[t].n = (lo + per > n) ? n - lo : per;
    pthread_create(&th[t], NULL, mt_body, &args[t]);
    used++;
  }
  for (t = 0; t < used; t++) pthread_join(th[t], NULL);
}
