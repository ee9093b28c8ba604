/* ORACLE (test infrastructure only -- never linked into the product path).
 *
 * Short-Weierstrass points with a = 0 over base field EF (Fq or Fq2).
 * "Template" header; define before including:
 *   EC       -- point prefix (e.g. bn254_g1)
 *   EF       -- base-field prefix providing EF_t, EF_add/sub/dbl/neg/mul/sqr/inv/eq/is_zero/is_one/one/zero
 *
 * Restates tachyon/math/elliptic_curves/short_weierstrass/:
 *   affine_point.h:39,125   identity = (0,0), no infinity flag
 *   point_xyzz.h:38,193     zero = (1,1,0,0), IsZero <=> zz == 0
 *   point_xyzz_impl.h:44-97   add-2008-s      (XYZZ + XYZZ)
 *   point_xyzz_impl.h:99-176  madd-2008-s     (XYZZ + affine, with identity handling)
 *   point_xyzz_impl.h:199-236 dbl-2008-s-1
 *   point_xyzz.h:199-212      ToAffine        point_xyzz.h:228-237 ToJacobian
 *   jacobian_point.h:195-215  IsZero / ToAffine
 */
#define EC_CAT2(a, b) a##_##b
#define EC_CAT(a, b) EC_CAT2(a, b)
#define EC_FN(name) EC_CAT(EC, name)
#define EF_FN(name) EC_CAT(EF, name)
#define EF_T EC_CAT(EF, t)
#define EC_AFF EC_CAT(EC, affine_t)
#define EC_XYZZ EC_CAT(EC, xyzz_t)
#define EC_JAC EC_CAT(EC, jacobian_t)

typedef struct { EF_T x, y; } EC_AFF;
typedef struct { EF_T x, y, zz, zzz; } EC_XYZZ;
typedef struct { EF_T x, y, z; } EC_JAC;

static inline int EC_FN(affine_is_zero)(const EC_AFF* p) {
  return EF_FN(is_zero)(&p->x) && EF_FN(is_zero)(&p->y);
}

static inline EC_XYZZ EC_FN(xyzz_zero)(void) {
  EC_XYZZ r;
  r.x = EF_FN(one)(); r.y = EF_FN(one)(); r.zz = EF_FN(zero)(); r.zzz = EF_FN(zero)();
  return r;
}

static inline int EC_FN(xyzz_is_zero)(const EC_XYZZ* p) { return EF_FN(is_zero)(&p->zz); }

static inline EC_XYZZ EC_FN(affine_to_xyzz)(const EC_AFF* a) {
  if (EC_FN(affine_is_zero)(a)) return EC_FN(xyzz_zero)();
  EC_XYZZ r;
  r.x = a->x; r.y = a->y; r.zz = EF_FN(one)(); r.zzz = EF_FN(one)();
  return r;
}

/* dbl-2008-s-1, point_xyzz_impl.h:199-236 (a = 0). */
static inline EC_XYZZ EC_FN(xyzz_dbl)(const EC_XYZZ* a) {
  if (EC_FN(xyzz_is_zero)(a)) return *a;
  EF_T u = EF_FN(dbl)(a->y);
  EF_T v = EF_FN(sqr)(u);
  EF_T w = EF_FN(mul)(u, v);
  EF_T s = EF_FN(mul)(a->x, v);
  EF_T m = EF_FN(sqr)(a->x);
  m = EF_FN(add)(m, EF_FN(dbl)(m));
  EC_XYZZ b;
  b.x = EF_FN(sub)(EF_FN(sqr)(m), EF_FN(dbl)(s));
  b.y = EF_FN(sub)(EF_FN(mul)(m, EF_FN(sub)(s, b.x)), EF_FN(mul)(w, a->y));
  b.zz = EF_FN(mul)(v, a->zz);
  b.zzz = EF_FN(mul)(w, a->zzz);
  return b;
}

/* madd-2008-s with the zero handling of AddInPlace(affine), point_xyzz_impl.h:99-176. */
static inline EC_XYZZ EC_FN(xyzz_madd)(const EC_XYZZ* a, const EC_AFF* b) {
  if (EC_FN(xyzz_is_zero)(a)) return EC_FN(affine_to_xyzz)(b);
  if (EC_FN(affine_is_zero)(b)) return *a;
  EF_T p = EF_FN(sub)(EF_FN(mul)(b->x, a->zz), a->x);
  EF_T r = EF_FN(sub)(EF_FN(mul)(b->y, a->zzz), a->y);
  if (EF_FN(is_zero)(&p) && EF_FN(is_zero)(&r)) return EC_FN(xyzz_dbl)(a);
  EF_T pp = EF_FN(sqr)(p);
  EF_T ppp = EF_FN(mul)(p, pp);
  EF_T q = EF_FN(mul)(a->x, pp);
  EC_XYZZ c;
  c.x = EF_FN(sub)(EF_FN(sub)(EF_FN(sqr)(r), ppp), EF_FN(dbl)(q));
  c.y = EF_FN(sub)(EF_FN(mul)(r, EF_FN(sub)(q, c.x)), EF_FN(mul)(a->y, ppp));
  c.zz = EF_FN(mul)(a->zz, pp);
  c.zzz = EF_FN(mul)(a->zzz, ppp);
  return c;
}

/* add-2008-s, point_xyzz_impl.h:44-97, plus the IsZero short-cuts of operator+. */
static inline EC_XYZZ EC_FN(xyzz_add)(const EC_XYZZ* a, const EC_XYZZ* b) {
  if (EC_FN(xyzz_is_zero)(a)) return *b;
  if (EC_FN(xyzz_is_zero)(b)) return *a;
  EF_T u1 = EF_FN(mul)(a->x, b->zz);
  EF_T s1 = EF_FN(mul)(a->y, b->zzz);
  EF_T p = EF_FN(sub)(EF_FN(mul)(b->x, a->zz), u1);
  EF_T r = EF_FN(sub)(EF_FN(mul)(b->y, a->zzz), s1);
  if (EF_FN(is_zero)(&p) && EF_FN(is_zero)(&r)) return EC_FN(xyzz_dbl)(a);
  EF_T pp = EF_FN(sqr)(p);
  EF_T ppp = EF_FN(mul)(p, pp);
  EF_T q = EF_FN(mul)(u1, pp);
  EC_XYZZ c;
  c.x = EF_FN(sub)(EF_FN(sub)(EF_FN(sqr)(r), ppp), EF_FN(dbl)(q));
  c.y = EF_FN(sub)(EF_FN(mul)(r, EF_FN(sub)(q, c.x)), EF_FN(mul)(s1, ppp));
  c.zz = EF_FN(mul)(EF_FN(mul)(a->zz, b->zz), pp);
  c.zzz = EF_FN(mul)(EF_FN(mul)(a->zzz, b->zzz), ppp);
  return c;
}

static inline EC_AFF EC_FN(affine_neg)(const EC_AFF* a) {
  EC_AFF r = *a;
  r.y = EF_FN(neg)(a->y);
  return r;
}

static inline EC_XYZZ EC_FN(xyzz_neg)(const EC_XYZZ* a) {
  EC_XYZZ r = *a;
  r.y = EF_FN(neg)(a->y);
  return r;
}

/* point_xyzz.h:199-212 */
static inline EC_AFF EC_FN(xyzz_to_affine)(const EC_XYZZ* a) {
  EC_AFF r;
  if (EC_FN(xyzz_is_zero)(a)) { r.x = EF_FN(zero)(); r.y = EF_FN(zero)(); return r; }
  if (EF_FN(is_one)(&a->zz)) { r.x = a->x; r.y = a->y; return r; }
  EF_T zinv3 = EF_FN(inv)(a->zzz);
  EF_T zinv2 = EF_FN(sqr)(EF_FN(mul)(zinv3, a->zz));
  r.x = EF_FN(mul)(a->x, zinv2);
  r.y = EF_FN(mul)(a->y, zinv3);
  return r;
}

/* point_xyzz.h:228-237 */
static inline EC_JAC EC_FN(xyzz_to_jacobian)(const EC_XYZZ* a) {
  EC_JAC r;
  if (EC_FN(xyzz_is_zero)(a)) { r.x = EF_FN(one)(); r.y = EF_FN(one)(); r.z = EF_FN(zero)(); return r; }
  if (EF_FN(is_one)(&a->zz)) { r.x = a->x; r.y = a->y; r.z = EF_FN(one)(); return r; }
  EF_T z = EF_FN(mul)(a->zz, a->zzz);
  r.x = EF_FN(mul)(EF_FN(mul)(a->x, a->zzz), z);
  r.y = EF_FN(mul)(EF_FN(mul)(a->y, a->zz), EF_FN(sqr)(z));
  r.z = z;
  return r;
}

/* jacobian_point.h:201-215 */
static inline EC_AFF EC_FN(jacobian_to_affine)(const EC_JAC* a) {
  EC_AFF r;
  if (EF_FN(is_zero)(&a->z)) { r.x = EF_FN(zero)(); r.y = EF_FN(zero)(); return r; }
  if (EF_FN(is_one)(&a->z)) { r.x = a->x; r.y = a->y; return r; }
  EF_T zi = EF_FN(inv)(a->z);
  EF_T zi2 = EF_FN(sqr)(zi);
  r.x = EF_FN(mul)(a->x, zi2);
  r.y = EF_FN(mul)(EF_FN(mul)(a->y, zi2), zi);
  return r;
}

/* Curve equation y^2 = x^3 + b (a = 0); identity counts as on-curve. */
static inline int EC_FN(affine_is_on_curve)(const EC_AFF* a, const EF_T* b) {
  if (EC_FN(affine_is_zero)(a)) return 1;
  EF_T lhs = EF_FN(sqr)(a->y);
  EF_T rhs = EF_FN(add)(EF_FN(mul)(EF_FN(sqr)(a->x), a->x), *b);
  return EF_FN(eq)(&lhs, &rhs);
}

/* Double-and-add scalar multiplication by a canonical little-endian scalar
 * (used by the naive MSM of variable_base_msm_unittest.cc and by the random
 * base generator of test/random.h:12-28). */
static inline EC_XYZZ EC_FN(scalar_mul)(const EC_AFF* p, const uint64_t* k, int nlimbs) {
  EC_XYZZ acc = EC_FN(xyzz_zero)();
  for (int i = nlimbs - 1; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      acc = EC_FN(xyzz_dbl)(&acc);
      if ((k[i] >> b) & 1) acc = EC_FN(xyzz_madd)(&acc, p);
    }
  return acc;
}

/* Batch normalisation XYZZ -> affine with one inversion (Montgomery's trick);
 * yields the same canonical affine coordinates as xyzz_to_affine. */
static inline void EC_FN(batch_to_affine)(const EC_XYZZ* in, EC_AFF* out, size_t n, EF_T* scratch) {
  EF_T acc = EF_FN(one)();
  for (size_t i = 0; i < n; ++i) {
    scratch[i] = acc;
    if (!EC_FN(xyzz_is_zero)(&in[i])) acc = EF_FN(mul)(acc, in[i].zzz);
  }
  EF_T inv = EF_FN(inv)(acc);
  for (size_t i = n; i-- > 0;) {
    if (EC_FN(xyzz_is_zero)(&in[i])) {
      out[i].x = EF_FN(zero)(); out[i].y = EF_FN(zero)();
      continue;
    }
    EF_T zinv3 = EF_FN(mul)(inv, scratch[i]);
    inv = EF_FN(mul)(inv, in[i].zzz);
    EF_T zinv2 = EF_FN(sqr)(EF_FN(mul)(zinv3, in[i].zz));
    out[i].x = EF_FN(mul)(in[i].x, zinv2);
    out[i].y = EF_FN(mul)(in[i].y, zinv3);
  }
}

#undef EC_CAT2
#undef EC_CAT
#undef EC_FN
#undef EF_FN
#undef EF_T
#undef EC_AFF
#undef EC_XYZZ
#undef EC_JAC
