/* ORACLE (test infrastructure only -- never linked into the product path).
 *
 * Prime field in Montgomery form, R = 2^(64*N), 64-bit little-endian limbs,
 * values canonical in [0, p).  "Template" header: include once per field with
 *   FF      -- name prefix (e.g. bn254_fr)
 *   FF_N    -- number of 64-bit limbs
 *   FF_P / FF_R / FF_R2 / FF_INV -- modulus, R mod p, R^2 mod p, -p^-1 mod 2^64
 *
 * Restates tachyon/math/finite_fields/prime_field_fallback.h:
 *   Add        :199-214 (add + Clamp)          Sub    :234-251
 *   Negate     :253-260                        Mul    :273-290 -> DoFastMul :331-355 (CIOS, no-carry)
 *   Square     :292-300 -> DoSquareImpl :364-394 + BigInt::MontgomeryReduce64 (big_int.h:300-305)
 *   ToBigInt   :166-169 (BigInt::FromMontgomery64)
 *   Inverse    :310-317 uses a Bernstein-Yang inverter; the oracle uses Fermat
 *              (a^(p-2)), which returns the same unique canonical inverse.
 */
#include <stdint.h>
#include <string.h>

#define FF_CAT2(a, b) a##_##b
#define FF_CAT(a, b) FF_CAT2(a, b)
#define FF_T FF_CAT(FF, t)
#define FF_FN(name) FF_CAT(FF, name)

typedef struct { uint64_t l[FF_N]; } FF_T;

static inline int FF_FN(geq_p)(const uint64_t* a) {
  for (int i = FF_N - 1; i >= 0; --i) {
    if (a[i] > FF_P[i]) return 1;
    if (a[i] < FF_P[i]) return 0;
  }
  return 1;
}

static inline void FF_FN(sub_p)(uint64_t* a) {
  unsigned __int128 borrow = 0;
  for (int i = 0; i < FF_N; ++i) {
    unsigned __int128 d = (unsigned __int128)a[i] - FF_P[i] - (uint64_t)borrow;
    a[i] = (uint64_t)d;
    borrow = (d >> 64) ? 1 : 0;
  }
}

/* BigInt::Clamp (big_int.h:279-291): conditional subtraction of p. */
static inline void FF_FN(clamp)(uint64_t* a, uint64_t carry) {
  if (carry || FF_FN(geq_p)(a)) FF_FN(sub_p)(a);
}

static inline FF_T FF_FN(zero)(void) { FF_T r; memset(&r, 0, sizeof r); return r; }
static inline FF_T FF_FN(one)(void) { FF_T r; memcpy(r.l, FF_R, sizeof r.l); return r; }
static inline int FF_FN(is_zero)(const FF_T* a) {
  for (int i = 0; i < FF_N; ++i) if (a->l[i]) return 0;
  return 1;
}
static inline int FF_FN(eq)(const FF_T* a, const FF_T* b) { return memcmp(a, b, sizeof *a) == 0; }
static inline int FF_FN(is_one)(const FF_T* a) { FF_T o = FF_FN(one)(); return FF_FN(eq)(a, &o); }

static inline FF_T FF_FN(add)(FF_T a, FF_T b) {
  unsigned __int128 c = 0;
  for (int i = 0; i < FF_N; ++i) {
    c += (unsigned __int128)a.l[i] + b.l[i];
    a.l[i] = (uint64_t)c;
    c >>= 64;
  }
  FF_FN(clamp)(a.l, (uint64_t)c);
  return a;
}

static inline FF_T FF_FN(dbl)(FF_T a) { return FF_FN(add)(a, a); }

static inline FF_T FF_FN(sub)(FF_T a, FF_T b) {
  /* if b > a: a += p first (prime_field_fallback.h:234-241) */
  int b_gt_a = 0;
  for (int i = FF_N - 1; i >= 0; --i) {
    if (b.l[i] > a.l[i]) { b_gt_a = 1; break; }
    if (b.l[i] < a.l[i]) break;
  }
  unsigned __int128 c = 0;
  if (b_gt_a) {
    for (int i = 0; i < FF_N; ++i) {
      c += (unsigned __int128)a.l[i] + FF_P[i];
      a.l[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  unsigned __int128 borrow = 0;
  for (int i = 0; i < FF_N; ++i) {
    unsigned __int128 d = (unsigned __int128)a.l[i] - b.l[i] - (uint64_t)borrow;
    a.l[i] = (uint64_t)d;
    borrow = (d >> 64) ? 1 : 0;
  }
  return a;
}

static inline FF_T FF_FN(neg)(FF_T a) {
  if (FF_FN(is_zero)(&a)) return a;
  FF_T p;
  memcpy(p.l, FF_P, sizeof p.l);
  return FF_FN(sub)(p, a);
}

/* DoFastMul, prime_field_fallback.h:331-355 (CIOS with the no-carry trick;
 * valid because every modulus here leaves the top bit of its top limb clear). */
static inline FF_T FF_FN(mul)(FF_T a, FF_T b) {
  uint64_t r[FF_N];
  memset(r, 0, sizeof r);
  for (int i = 0; i < FF_N; ++i) {
    unsigned __int128 t = (unsigned __int128)a.l[0] * b.l[i] + r[0];
    r[0] = (uint64_t)t;
    uint64_t hi1 = (uint64_t)(t >> 64);
    uint64_t k = r[0] * FF_INV;
    unsigned __int128 t2 = (unsigned __int128)k * FF_P[0] + r[0];
    uint64_t hi2 = (uint64_t)(t2 >> 64);
    for (int j = 1; j < FF_N; ++j) {
      t = (unsigned __int128)a.l[j] * b.l[i] + r[j] + hi1;
      r[j] = (uint64_t)t;
      hi1 = (uint64_t)(t >> 64);
      t2 = (unsigned __int128)k * FF_P[j] + r[j] + hi2;
      r[j - 1] = (uint64_t)t2;
      hi2 = (uint64_t)(t2 >> 64);
    }
    r[FF_N - 1] = hi1 + hi2;
  }
  FF_T c;
  memcpy(c.l, r, sizeof r);
  FF_FN(clamp)(c.l, 0);
  return c;
}

/* BigInt<N>::MontgomeryReduce64 (big_int.h:300-305 -> :560-590 region). */
static inline FF_T FF_FN(mont_reduce)(uint64_t* r /* 2N limbs, clobbered */) {
  uint64_t carry2 = 0;
  for (int i = 0; i < FF_N; ++i) {
    uint64_t k = r[i] * FF_INV;
    unsigned __int128 t = (unsigned __int128)k * FF_P[0] + r[i];
    uint64_t carry = (uint64_t)(t >> 64);
    for (int j = 1; j < FF_N; ++j) {
      t = (unsigned __int128)k * FF_P[j] + r[i + j] + carry;
      r[i + j] = (uint64_t)t;
      carry = (uint64_t)(t >> 64);
    }
    unsigned __int128 s = (unsigned __int128)r[i + FF_N] + carry + carry2;
    r[i + FF_N] = (uint64_t)s;
    carry2 = (uint64_t)(s >> 64);
  }
  FF_T c;
  memcpy(c.l, r + FF_N, sizeof c.l);
  FF_FN(clamp)(c.l, carry2);
  return c;
}

/* DoSquareImpl, prime_field_fallback.h:364-394. */
static inline FF_T FF_FN(sqr)(FF_T a) {
  uint64_t r[2 * FF_N];
  memset(r, 0, sizeof r);
  for (int i = 0; i < FF_N - 1; ++i) {
    uint64_t hi = 0;
    for (int j = i + 1; j < FF_N; ++j) {
      unsigned __int128 t = (unsigned __int128)a.l[i] * a.l[j] + r[i + j] + hi;
      r[i + j] = (uint64_t)t;
      hi = (uint64_t)(t >> 64);
    }
    r[i + FF_N] = hi;
  }
  r[2 * FF_N - 1] = r[2 * FF_N - 2] >> 63;
  for (int i = 2; i < 2 * FF_N - 1; ++i)
    r[2 * FF_N - i] = (r[2 * FF_N - i] << 1) | (r[2 * FF_N - (i + 1)] >> 63);
  r[1] <<= 1;
  uint64_t hi = 0;
  for (int i = 0; i < FF_N; ++i) {
    unsigned __int128 t = (unsigned __int128)a.l[i] * a.l[i] + r[2 * i] + hi;
    r[2 * i] = (uint64_t)t;
    unsigned __int128 s = (unsigned __int128)r[2 * i + 1] + (uint64_t)(t >> 64);
    r[2 * i + 1] = (uint64_t)s;
    hi = (uint64_t)(s >> 64);
  }
  return FF_FN(mont_reduce)(r);
}

/* ToBigInt / FromMontgomery64: multiply by 1 (Montgomery reduce of a||0). */
static inline void FF_FN(to_bigint)(const FF_T* a, uint64_t* out) {
  uint64_t r[2 * FF_N];
  memset(r, 0, sizeof r);
  memcpy(r, a->l, sizeof a->l);
  FF_T c = FF_FN(mont_reduce)(r);
  memcpy(out, c.l, sizeof c.l);
}

/* FromBigInt: x*R mod p = MontMul(x, R^2). Input must be < p. */
static inline FF_T FF_FN(from_bigint)(const uint64_t* x) {
  FF_T a, r2;
  memcpy(a.l, x, sizeof a.l);
  memcpy(r2.l, FF_R2, sizeof r2.l);
  return FF_FN(mul)(a, r2);
}

static inline FF_T FF_FN(from_u64)(uint64_t v) {
  uint64_t x[FF_N];
  memset(x, 0, sizeof x);
  x[0] = v;
  return FF_FN(from_bigint)(x);
}

/* Pow by a little-endian exponent of `nlimbs` limbs. */
static inline FF_T FF_FN(pow)(FF_T a, const uint64_t* e, int nlimbs) {
  FF_T r = FF_FN(one)();
  for (int i = nlimbs - 1; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      r = FF_FN(sqr)(r);
      if ((e[i] >> b) & 1) r = FF_FN(mul)(r, a);
    }
  return r;
}

static inline FF_T FF_FN(inv)(FF_T a) {
  uint64_t e[FF_N];
  memcpy(e, FF_P, sizeof e);
  /* p - 2 (p is odd and > 2, so no borrow past limb 0) */
  e[0] -= 2;
  return FF_FN(pow)(a, e, FF_N);
}

#undef FF_T
#undef FF_FN
#undef FF_CAT
#undef FF_CAT2
