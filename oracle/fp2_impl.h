/* ORACLE (test infrastructure only -- never linked into the product path).
 *
 * Quadratic extension Fq2 = Fq[u]/(u^2 - beta) with beta = -1 (the non-residue of
 * both BN254 and BLS12-381: bn/bn254/BUILD.bazel:62-71, bls12/bls12_381/BUILD.bazel:73-81).
 * Restates tachyon/math/finite_fields/quadratic_extension_field.h:
 *   DoMul (Karatsuba) :315-360, DoSquare, Inverse (norm-based).
 * Define F2 (prefix of the extension) and F1 (base-field prefix) before including.
 */
#define F2_CAT2(a, b) a##_##b
#define F2_CAT(a, b) F2_CAT2(a, b)
#define F2_FN(name) F2_CAT(F2, name)
#define F1_FN(name) F2_CAT(F1, name)
#define F2_T F2_CAT(F2, t)
#define F1_T F2_CAT(F1, t)

typedef struct { F1_T c0, c1; } F2_T;

static inline F2_T F2_FN(zero)(void) { F2_T r; r.c0 = F1_FN(zero)(); r.c1 = F1_FN(zero)(); return r; }
static inline F2_T F2_FN(one)(void) { F2_T r; r.c0 = F1_FN(one)(); r.c1 = F1_FN(zero)(); return r; }
static inline int F2_FN(is_zero)(const F2_T* a) { return F1_FN(is_zero)(&a->c0) && F1_FN(is_zero)(&a->c1); }
static inline int F2_FN(is_one)(const F2_T* a) { return F1_FN(is_one)(&a->c0) && F1_FN(is_zero)(&a->c1); }
static inline int F2_FN(eq)(const F2_T* a, const F2_T* b) { return F1_FN(eq)(&a->c0, &b->c0) && F1_FN(eq)(&a->c1, &b->c1); }
static inline F2_T F2_FN(add)(F2_T a, F2_T b) { a.c0 = F1_FN(add)(a.c0, b.c0); a.c1 = F1_FN(add)(a.c1, b.c1); return a; }
static inline F2_T F2_FN(sub)(F2_T a, F2_T b) { a.c0 = F1_FN(sub)(a.c0, b.c0); a.c1 = F1_FN(sub)(a.c1, b.c1); return a; }
static inline F2_T F2_FN(dbl)(F2_T a) { return F2_FN(add)(a, a); }
static inline F2_T F2_FN(neg)(F2_T a) { a.c0 = F1_FN(neg)(a.c0); a.c1 = F1_FN(neg)(a.c1); return a; }

/* (a0 + a1 u)(b0 + b1 u) = (a0 b0 - a1 b1) + ((a0 + a1)(b0 + b1) - a0 b0 - a1 b1) u */
static inline F2_T F2_FN(mul)(F2_T a, F2_T b) {
  F1_T v0 = F1_FN(mul)(a.c0, b.c0);
  F1_T v1 = F1_FN(mul)(a.c1, b.c1);
  F2_T r;
  r.c1 = F1_FN(sub)(F1_FN(sub)(F1_FN(mul)(F1_FN(add)(a.c0, a.c1), F1_FN(add)(b.c0, b.c1)), v0), v1);
  r.c0 = F1_FN(sub)(v0, v1);
  return r;
}

/* (a0 + a1 u)^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u  (beta = -1) */
static inline F2_T F2_FN(sqr)(F2_T a) {
  F2_T r;
  r.c1 = F1_FN(dbl)(F1_FN(mul)(a.c0, a.c1));
  r.c0 = F1_FN(mul)(F1_FN(add)(a.c0, a.c1), F1_FN(sub)(a.c0, a.c1));
  return r;
}

/* 1/(a0 + a1 u) = (a0 - a1 u) / (a0^2 + a1^2) */
static inline F2_T F2_FN(inv)(F2_T a) {
  F1_T t = F1_FN(inv)(F1_FN(add)(F1_FN(sqr)(a.c0), F1_FN(sqr)(a.c1)));
  F2_T r;
  r.c0 = F1_FN(mul)(a.c0, t);
  r.c1 = F1_FN(neg)(F1_FN(mul)(a.c1, t));
  return r;
}

#undef F2_CAT2
#undef F2_CAT
#undef F2_FN
#undef F1_FN
#undef F2_T
#undef F1_T
