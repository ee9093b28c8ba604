// Short-Weierstrass (a = 0) point arithmetic for the MSM hot path.
//
// Layouts match the reference (tachyon/math/elliptic_curves/short_weierstrass):
//   Affine {x, y}, identity = (0, 0), no infinity flag    affine_point.h:39,125
//   XYZZ   {x, y, zz, zzz}, zero <=> zz == 0               point_xyzz.h:38,193
//   Jacobian {x, y, z}, zero <=> z == 0                     jacobian_point.h:40,195
// Formulas (EFD, as in point_xyzz_impl.h; the y coordinates' a b - c d as
// one fused product, Fp::mul_sub):
//   madd-2008-s (:129-176), add-2008-s (:44-97), dbl-2008-s-1 (:199-236).
#pragma once
#include "../field/ff.h"

namespace tachyon_amd {

template <class F>
struct Affine {
  F x, y;
  TA_HD bool is_zero() const { return x.is_zero() && y.is_zero(); }
  // identity test of an input point (canonical coordinates)
  TA_HD bool is_zero_canonical() const { return x.is_zero_canonical() && y.is_zero_canonical(); }
  TA_HD static Affine zero() { return {F::zero(), F::zero()}; }
  TA_HD Affine neg() const { return is_zero() ? *this : Affine{x, -y}; }
  TA_HD Affine canonical() const { return {x.canonical(), y.canonical()}; }
};

template <class F>
struct Jacobian {
  F x, y, z;
  TA_HD bool is_zero() const { return z.is_zero(); }
  TA_HD static Jacobian zero() { return {F::one(), F::one(), F::zero()}; }
  TA_HD Jacobian canonical() const { return {x.canonical(), y.canonical(), z.canonical()}; }
};

template <class F>
struct XYZZ {
  F x, y, zz, zzz;

  TA_HD static XYZZ zero() { return {F::one(), F::one(), F::zero(), F::zero()}; }
  TA_HD bool is_zero() const { return zz.is_zero(); }
  TA_HD static XYZZ from_affine(const Affine<F>& a) {
    if (a.is_zero()) return zero();
    return {a.x, a.y, F::one(), F::one()};
  }
  TA_HD XYZZ neg() const { return {x, -y, zz, zzz}; }
  TA_HD XYZZ canonical() const { return {x.canonical(), y.canonical(), zz.canonical(), zzz.canonical()}; }

  // Doubling for the exceptional P == Q branch of the adds.  For one-word
  // (32-byte) fields it stays inline: an out-of-line call there makes the
  // compiler keep the accumulator in scratch (the sret / `this` slots are
  // addressable), which cost a 272-byte scratch round trip per madd on
  // MI355X.  Wider fields (Fq2, BLS12-381 Fq) take the call to bound code size.
  TA_HD XYZZ dbl_slowpath() const {
    if constexpr (sizeof(F) <= 32) return dbl();
    else return dbl_outline();
  }
  TA_HD_NOINLINE XYZZ dbl_outline() const { return dbl(); }

  // dbl-2008-s-1 (a = 0)
  TA_HD XYZZ dbl() const {
    if (is_zero()) return *this;
    F u = y.dbl();
    F v = u.sqr();
    F w = u * v;
    F s = x * v;
    F m = x.sqr();
    m = m + m.dbl();
    XYZZ r;
    r.x = m.sqr() - s.dbl();
    r.y = m.mul_sub(s - r.x, w, y);
    r.zz = v * zz;
    r.zzz = w * zzz;
    return r;
  }

  // madd-2008-s: *this + affine (identity-aware, like AddInPlace(affine)).
  TA_HD XYZZ madd(const Affine<F>& b) const {
    if (b.is_zero()) return *this;
    if (is_zero()) return from_affine(b);
    F p = b.x * zz - x;
    F r = b.y * zzz - y;
    if (p.is_zero() && r.is_zero()) return dbl_slowpath();
    F pp = p.sqr();
    F ppp = p * pp;
    F q = x * pp;
    XYZZ c;
    c.x = r.sqr() - ppp - q.dbl();
    c.y = r.mul_sub(q - c.x, y, ppp);
    c.zz = zz * pp;
    c.zzz = zzz * ppp;
    return c;
  }

  // madd-2008-s for the bucket accumulation's common case: neither *this nor
  // b is the identity (the caller tracks an identity accumulator itself), so
  // the only test left is P == +-this; *now_zero is set when b == -this.
  TA_HD XYZZ madd_nz(const Affine<F>& b, bool* now_zero) const {
    F p = b.x * zz - x;
    F r = b.y * zzz - y;
    if (p.is_zero()) {
      if (r.is_zero()) return dbl_slowpath();
      *now_zero = true;
      return zero();
    }
    F pp = p.sqr();
    F ppp = p * pp;
    F q = x * pp;
    XYZZ c;
    c.x = r.sqr() - ppp - q.dbl();
    c.y = r.mul_sub(q - c.x, y, ppp);
    c.zz = zz * pp;
    c.zzz = zzz * ppp;
    return c;
  }

  // add-2008-s
  TA_HD XYZZ operator+(const XYZZ& b) const {
    if (is_zero()) return b;
    if (b.is_zero()) return *this;
    F u1 = x * b.zz;
    F s1 = y * b.zzz;
    F p = b.x * zz - u1;
    F r = b.y * zzz - s1;
    if (p.is_zero() && r.is_zero()) return dbl_slowpath();
    F pp = p.sqr();
    F ppp = p * pp;
    F q = u1 * pp;
    XYZZ c;
    c.x = r.sqr() - ppp - q.dbl();
    c.y = r.mul_sub(q - c.x, s1, ppp);
    c.zz = zz * b.zz * pp;
    c.zzz = zzz * b.zzz * ppp;
    return c;
  }

  // point_xyzz.h:199-212
  TA_HD_NOINLINE Affine<F> to_affine() const {
    if (is_zero()) return Affine<F>::zero();
    if (zz.is_one()) return Affine<F>{x, y}.canonical();
    F zinv3 = zzz.inverse();
    F zinv2 = (zinv3 * zz).sqr();
    return Affine<F>{x * zinv2, y * zinv3}.canonical();
  }

  // point_xyzz.h:228-237
  TA_HD_NOINLINE Jacobian<F> to_jacobian() const {
    if (is_zero()) return Jacobian<F>::zero();
    if (zz.is_one()) return {x, y, F::one()};
    F z = zz * zzz;
    return {x * zzz * z, y * zz * z.sqr(), z};
  }

  TA_HD static XYZZ from_jacobian(const Jacobian<F>& j) {
    if (j.is_zero()) return zero();
    F z2 = j.z.sqr();
    return {j.x, j.y, z2, z2 * j.z};
  }
};

// Curve descriptors: base field, scalar field, coefficient b (Montgomery).
struct Bn254G1 {
  using F = Bn254Fq;
  using Fr = Bn254Fr;
  static constexpr const char* kName = "bn254_g1";
};
struct Bn254G2 {
  using F = Bn254Fq2;
  using Fr = Bn254Fr;
  static constexpr const char* kName = "bn254_g2";
};
struct Bls381G1 {
  using F = Bls381Fq;
  using Fr = Bls381Fr;
  static constexpr const char* kName = "bls12_381_g1";
};
struct Bls381G2 {
  using F = Bls381Fq2;
  using Fr = Bls381Fr;
  static constexpr const char* kName = "bls12_381_g2";
};

}  // namespace tachyon_amd
