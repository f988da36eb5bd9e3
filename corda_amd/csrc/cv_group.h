// cv_group.h — edwards25519 group operations (a = -1 twisted Edwards, extended coordinates).
//
// Representations (HWCD'08 extended coordinates):
//   p2     (X:Y:Z)            x = X/Z, y = Y/Z
//   p3     (X:Y:Z:T)          + T = XY/Z
//   p1p1   ((X:Z),(Y:T))      "completed": x = X/Z, y = Y/T — output of add/dbl before conversion
//   cached (Y+X, Y-X, Z, 2dT) right operand of a variable-point add
//   precomp(y+x, y-x, 2dxy)   affine right operand (Z = 1) of a fixed-point add (basepoint table)
// The unified addition is complete for d non-square, so every routine below is exact group
// arithmetic on ALL curve points, torsion included — which is what makes the GPU's fixed-window
// schedule produce the same point (hence the same verdict) as eddsa-0.1.0's slide()-based one.
//
// Limb bounds (units of M, cv_field.h): every p2/p3 coordinate is tight (T) at rest.  p1p1 from
// add/madd: X=E<=3.01, Y=H<=2.02, Z=G<=3.03, T=F<=4.02; from dbl: E<=3.01, H'=T, G<=3.01, F'<=5.01.
// Conversions therefore always pass p1p1.T as the unrestricted `f` operand of fe_mul (<= 8) and the
// other coordinate as `g` (<= 3.3).
#pragma once
#include "cv_field.h"

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YplusX, YminusX, Z, T2d; };
struct ge_precomp { fe yplusx, yminusx, xy2d; };

// curve constants, canonical limbs (< M_i), generated and checked by the host tests
#define CV_FE_D   {56195235, 13857412, 51736253, 6949390, 114729, 24766616, 60832955, 30306712, 48412415, 21499315}
#define CV_FE_D2  {45281625, 27714825, 36363642, 13898781, 229458, 15978800, 54557047, 27058993, 29715967, 9444199}
#define CV_FE_SQRTM1 {34513072, 25610706, 9377949, 3500415, 12389472, 33281959, 41962654, 31548777, 326685, 11406482}

CV_HD void fe_const_d(fe &h) { const fe c = {CV_FE_D}; h = c; }
CV_HD void fe_const_d2(fe &h) { const fe c = {CV_FE_D2}; h = c; }
CV_HD void fe_const_sqrtm1(fe &h) { const fe c = {CV_FE_SQRTM1}; h = c; }

CV_HD void ge_p3_identity(ge_p3 &r) { fe_zero(r.X); fe_one(r.Y); fe_one(r.Z); fe_zero(r.T); }
CV_HD void ge_p2_identity(ge_p2 &r) { fe_zero(r.X); fe_one(r.Y); fe_one(r.Z); }
CV_HD void ge_cached_identity(ge_cached &r) { fe_one(r.YplusX); fe_one(r.YminusX); fe_one(r.Z); fe_zero(r.T2d); }
CV_HD void ge_precomp_identity(ge_precomp &r) { fe_one(r.yplusx); fe_one(r.yminusx); fe_zero(r.xy2d); }

// Independent multiplications of one formula run interleaved (fe_mul_n, cv_field.h).
CV_HD void ge_p1p1_to_p2(ge_p2 &r, const ge_p1p1 &p) {
    fe h[3];
    const fe f[3] = {p.T, p.Y, p.T}, g[3] = {p.X, p.Z, p.Z};
    fe_mul_n<3>(h, f, g);
    r.X = h[0]; r.Y = h[1]; r.Z = h[2];
}
// T3 = X*Y takes Y as f and X as g, so the four products need the 19*g operand of only two
// elements (X and Z) — 9 fewer v_mul_lo_u32 per conversion than {.., X} x {.., Y}.
CV_HD void ge_p1p1_to_p3(ge_p3 &r, const ge_p1p1 &p) {
    fe h[4];
    const fe f[4] = {p.T, p.Y, p.T, p.Y}, g[4] = {p.X, p.Z, p.Z, p.X};
    fe_mul_n<4>(h, f, g);
    r.X = h[0]; r.Y = h[1]; r.Z = h[2]; r.T = h[3];
}
CV_HD void ge_p3_to_p2(ge_p2 &r, const ge_p3 &p) { r.X = p.X; r.Y = p.Y; r.Z = p.Z; }
CV_HD void ge_p3_to_cached(ge_cached &r, const ge_p3 &p) {
    fe d2;
    fe_const_d2(d2);
    fe_add(r.YplusX, p.Y, p.X);
    fe_sub<2>(r.YminusX, p.Y, p.X);
    r.Z = p.Z;
    fe_mul(r.T2d, p.T, d2);
}

// r = 2p: 4 squarings.  p1p1 = (E, H', G, F') with E = 2XY, H' = X^2+Y^2, G = Y^2-X^2,
// F' = 2Z^2-G: the negated (E, -H, G, -F) form of HWCD's doubling, which names the same point.
CV_HD void ge_p2_dbl(ge_p1p1 &r, const ge_p2 &p) {
    fe a, sq[4];
    fe_add(a, p.X, p.Y);
    const fe in[4] = {p.X, p.Y, p.Z, a};
    fe_sq_n<4, 0x4>(sq, in);      // X^2, Y^2, 2 Z^2, (X+Y)^2
    const fe &xx = sq[0], &yy = sq[1], &zz2 = sq[2], &aa = sq[3];
    fe_add(r.Y, yy, xx);          // H' <= 2.02 (an f operand: not carried)
    fe_sub<2>(r.Z, yy, xx);       // G  <= 3.01
    fe_sub_carry_even<3>(r.X, aa, r.Y);   // E <= 4.01, a g operand: its even limbs carried (<= 1.0, odd <= 4.01)
    fe_sub<4>(r.T, zz2, r.Z);     // F' <= 5.01
}
CV_HD void ge_p3_dbl(ge_p1p1 &r, const ge_p3 &p) {
    ge_p2 q;
    ge_p3_to_p2(q, p);
    ge_p2_dbl(r, q);
}

// r = p + q (q cached, possibly conditionally negated)
CV_HD void ge_add(ge_p1p1 &r, const ge_p3 &p, const ge_cached &q) {
    fe s, d, m[4];
    fe_add(s, p.Y, p.X);          // <= 2.02
    fe_sub<2>(d, p.Y, p.X);       // <= 3.01
    const fe f[4] = {q.YplusX, q.YminusX, q.T2d, p.Z}, g[4] = {s, d, p.T, q.Z};
    fe_mul_n<4>(m, f, g);
    const fe &a = m[0], &b = m[1], &c = m[2];
    fe dd;
    fe_add(dd, m[3], m[3]);
    fe_sub<2>(r.X, a, b);         // E <= 3.01
    fe_add(r.Y, a, b);            // H <= 2.02
    fe_add(r.Z, dd, c);           // G <= 3.03
    fe_sub<2>(r.T, dd, c);        // F <= 4.02
}
// r = p + q (q affine precomp)
CV_HD void ge_madd(ge_p1p1 &r, const ge_p3 &p, const ge_precomp &q) {
    fe s, d, m[3], dd;
    fe_add(s, p.Y, p.X);
    fe_sub<2>(d, p.Y, p.X);
    const fe f[3] = {q.yplusx, q.yminusx, q.xy2d}, g[3] = {s, d, p.T};
    fe_mul_n<3>(m, f, g);
    const fe &a = m[0], &b = m[1], &c = m[2];
    fe_add(dd, p.Z, p.Z);
    fe_sub<2>(r.X, a, b);
    fe_add(r.Y, a, b);
    fe_add(r.Z, dd, c);
    fe_sub<2>(r.T, dd, c);
}

// Conditional negation of a table entry, branch-free: -(x,y) = (-x, y) swaps Y+X <-> Y-X and
// negates T (2p - T, still within the g <= 3.3 budget).
// -2dT = 2p - 2dT as (x XOR m) + (m AND (2p + 1)) with m all ones or zero: one v_xad_u32 per limb instead of a
// subtraction and a select (the mask is opaque, or LLVM turns the xor-add back into a select).
CV_HD void ge_cached_cneg(ge_cached &r, bool neg) {
    fe a = r.YplusX, b = r.YminusX;
    fe_sel(r.YplusX, a, b, neg);
    fe_sel(r.YminusX, b, a, neg);
    uint32_t m = neg ? 0xffffffffu : 0u;
#ifdef __HIP_DEVICE_COMPILE__
    asm("" : "+v"(m));
#endif
#pragma unroll
    for (int i = 0; i < 10; i++) {
        CV_ASSERT(r.T2d.v[i] <= cv_kp(2, i), "ge_cached_cneg: 2dT limb exceeds 2p");
        r.T2d.v[i] = (r.T2d.v[i] ^ m) + (m & (cv_kp(2, i) + 1u));
    }
}
CV_HD void ge_precomp_cneg(ge_precomp &r, bool neg) {
    fe a = r.yplusx, b = r.yminusx, t;
    fe_sel(r.yplusx, a, b, neg);
    fe_sel(r.yminusx, b, a, neg);
    fe_neg(t, r.xy2d);
    fe_sel(r.xy2d, r.xy2d, t, neg);
}

// GroupElement.toByteArray(): affine y (canonical) with the sign of x in bit 255, as 8 LE words.
__host__ __device__ __forceinline__ void ge_p2_encode(uint32_t w[8], const ge_p2 &p) {
    fe zi, x, y;
    fe_invert(zi, p.Z);
    fe_mul(x, p.X, zi);
    fe_mul(y, p.Y, zi);
    uint32_t xw[8];
    fe_to_words(w, y);
    fe_to_words(xw, x);
    w[7] |= (xw[0] & 1u) << 31;
}

// EdDSAPublicKey.getAbyte() (= A.toByteArray() after decoding) WITHOUT the square root: the decoded
// y is the key's 255-bit value mod p, and the decoded x has isNegative(x) == bit 255 unless x = 0,
// which happens exactly when y = +-1.  (For keys that fail to decode the value is irrelevant: the
// verdict is forced false.)
CV_HD void ge_abyte_from_key(uint32_t abyte[8], const uint32_t w[8]) {
    fe y;
    fe_from_words(y, w);
    fe_to_words(abyte, y);
    uint32_t one_or = abyte[0] ^ 1u, m1_or = abyte[0] ^ 0xffffffecu;     // y == 1, y == p - 1
#pragma unroll
    for (int q = 1; q < 7; q++) { one_or |= abyte[q]; m1_or |= abyte[q] ^ 0xffffffffu; }
    one_or |= abyte[7];
    m1_or |= abyte[7] ^ 0x7fffffffu;
    const bool x_zero = (one_or == 0) | (m1_or == 0);
    abyte[7] |= (x_zero ? 0u : (w[7] & 0x80000000u));
}

// eddsa-0.1.0 GroupElement(curve, bytes) decode of a public key given as 8 LE words.
// Returns false where the reference throws IllegalArgumentException("not a valid GroupElement").
// y keeps its non-reduced value; x is negated when isNegative(x) != bit 255 (x = 0 with the sign
// bit set is therefore accepted as x = 0).  All output coordinates are tight.
template <bool LAT = false> __host__ __device__ __forceinline__ bool ge_decode_0_1_0(ge_p3 &A, const uint32_t w[8]) {
    fe y, yy, u, v, v3, x, vxx, chk, one, d;
    fe_from_words(y, w);
    fe_one(one);
    fe_const_d(d);
    fe_sq_m<LAT>(yy, y);
    fe_sub<2>(u, yy, one);       // u = y^2 - 1         (<= 3.01)
    fe_mul_m<LAT>(v, yy, d);
    fe_add(v, v, one);           // v = d y^2 + 1       (<= 1.02)
    fe_sq_m<LAT>(v3, v);
    fe_mul_m<LAT>(v3, v3, v);           // v^3
    fe_sq_m<LAT>(x, v3);
    fe_mul_m<LAT>(x, x, v);
    fe_mul_m<LAT>(x, x, u);             // u v^7
    fe_pow22523<LAT>(x, x);           // (u v^7)^((p-5)/8)
    fe_mul_m<LAT>(x, x, v3);
    fe_mul_m<LAT>(x, x, u);             // u v^3 (u v^7)^((p-5)/8)
    fe_sq_m<LAT>(vxx, x);
    fe_mul_m<LAT>(vxx, vxx, v);
    fe_sub<4>(chk, vxx, u);
    bool ok = true;
    if (!fe_is_zero(chk)) {
        fe_add(chk, vxx, u);
        if (!fe_is_zero(chk)) ok = false;
        fe sqm1, xi;
        fe_const_sqrtm1(sqm1);
        fe_mul_m<LAT>(xi, x, sqm1);
        x = xi;
    }
    const int sign = (int)(w[7] >> 31);
    fe nx;
    fe_neg(nx, x);
    fe_carry(nx, nx);
    fe_sel(x, x, nx, fe_is_negative(x) != sign);
    A.X = x;
    A.Y = y;
    fe_one(A.Z);
    fe_mul_m<LAT>(A.T, x, y);
    return ok;
}

// ---------------------------------------------------------------- two decodes, interleaved
// The eddsa-0.1.0 decode above for two encodings at once (the key A and the signature's R in the
// fused half-size prep): every field operation of the two square-root chains runs as a 2-way
// interleaved pair (fe_mul_n<2> / fe_sq_n<2>), which doubles the independent work per instruction
// window of a lane at the same instruction count.
// LAT = true: each element by the latency (ILP) forms instead (small batches, lone waves).
template <bool LAT = false> CV_HD void fe_sq2(fe (&h)[2], const fe (&f)[2]) {
    if constexpr (LAT) {
        fe_sq_ilp(h[0], f[0], false);
        fe_sq_ilp(h[1], f[1], false);
    } else {
        fe_sq_n<2, 0>(h, f);
    }
}
template <bool LAT = false> __host__ __device__ __forceinline__ void fe_sqn2(fe (&h)[2], const fe (&f)[2], int n) {
#ifdef __HIP_DEVICE_COMPILE__
    asm volatile("" : "+s"(n));
#endif
    fe_sq2<LAT>(h, f);
#pragma nounroll
    for (int i = 1; i < n; i++) fe_sq2<LAT>(h, h);
}
template <bool LAT = false> CV_HD void fe_mul2(fe (&h)[2], const fe &f0, const fe &g0, const fe &f1, const fe &g1) {
    if constexpr (LAT) {
        fe a, b;
        fe_mul_ilp(a, f0, g0);
        fe_mul_ilp(b, f1, g1);
        h[0] = a;
        h[1] = b;
    } else {
        const fe f[2] = {f0, f1}, g[2] = {g0, g1};
        fe_mul_n<2>(h, f, g);
    }
}
// z^(2^252 - 3) for two elements
template <bool LAT = false> __host__ __device__ __forceinline__ void fe_pow22523_2(fe (&out)[2], const fe (&z)[2]) {
    fe t0[2], t1[2], t2[2];
    fe_sq2<LAT>(t0, z);                                  // z^2
    fe_sqn2<LAT>(t1, t0, 2);                                    // z^8
    fe_mul2<LAT>(t1, z[0], t1[0], z[1], t1[1]);                 // z^9
    fe_mul2<LAT>(t0, t0[0], t1[0], t0[1], t1[1]);               // z^11
    fe_sq2<LAT>(t0, t0);                                 // z^22
    fe_mul2<LAT>(t0, t1[0], t0[0], t1[1], t0[1]);               // z^31
    fe_sqn2<LAT>(t1, t0, 5);
    fe_mul2<LAT>(t0, t1[0], t0[0], t1[1], t0[1]);               // 2^10 - 1
    fe_sqn2<LAT>(t1, t0, 10);
    fe_mul2<LAT>(t1, t1[0], t0[0], t1[1], t0[1]);               // 2^20 - 1
    fe_sqn2<LAT>(t2, t1, 20);
    fe_mul2<LAT>(t1, t2[0], t1[0], t2[1], t1[1]);               // 2^40 - 1
    fe_sqn2<LAT>(t1, t1, 10);
    fe_mul2<LAT>(t0, t1[0], t0[0], t1[1], t0[1]);               // 2^50 - 1
    fe_sqn2<LAT>(t1, t0, 50);
    fe_mul2<LAT>(t1, t1[0], t0[0], t1[1], t0[1]);               // 2^100 - 1
    fe_sqn2<LAT>(t2, t1, 100);
    fe_mul2<LAT>(t1, t2[0], t1[0], t2[1], t1[1]);               // 2^200 - 1
    fe_sqn2<LAT>(t1, t1, 50);
    fe_mul2<LAT>(t0, t1[0], t0[0], t1[1], t0[1]);               // 2^250 - 1
    fe_sqn2<LAT>(t0, t0, 2);                                    // 2^252 - 4
    fe_mul2<LAT>(out, t0[0], z[0], t0[1], z[1]);                // 2^252 - 3
}
// ge_decode_0_1_0 of w[0] and w[1] together; ok[k] as ge_decode_0_1_0's return value.
template <bool LAT = false>
__host__ __device__ __forceinline__ void ge_decode2_0_1_0(ge_p3 (&P)[2], bool (&ok)[2], const uint32_t *w0,
                                                          const uint32_t *w1) {
    fe y[2], yy[2], u[2], v[2], v3[2], x[2], vxx[2], one, d;
    fe_from_words(y[0], w0);
    fe_from_words(y[1], w1);
    fe_one(one);
    fe_const_d(d);
    fe_sq2<LAT>(yy, y);
    fe_mul2<LAT>(v, yy[0], d, yy[1], d);
#pragma unroll
    for (int k = 0; k < 2; k++) {
        fe_sub<2>(u[k], yy[k], one);       // u = y^2 - 1
        fe_add(v[k], v[k], one);           // v = d y^2 + 1
    }
    fe_sq2<LAT>(v3, v);
    fe_mul2<LAT>(v3, v3[0], v[0], v3[1], v[1]);                 // v^3
    fe_sq2<LAT>(x, v3);
    fe_mul2<LAT>(x, x[0], v[0], x[1], v[1]);
    fe_mul2<LAT>(x, x[0], u[0], x[1], u[1]);                    // u v^7
    fe_pow22523_2<LAT>(x, x);
    fe_mul2<LAT>(x, x[0], v3[0], x[1], v3[1]);
    fe_mul2<LAT>(x, x[0], u[0], x[1], u[1]);                    // u v^3 (u v^7)^((p-5)/8)
    fe_sq2<LAT>(vxx, x);
    fe_mul2<LAT>(vxx, vxx[0], v[0], vxx[1], v[1]);
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint32_t *w = k ? w1 : w0;
        fe chk;
        fe_sub<4>(chk, vxx[k], u[k]);
        ok[k] = true;
        if (!fe_is_zero(chk)) {
            fe_add(chk, vxx[k], u[k]);
            if (!fe_is_zero(chk)) ok[k] = false;
            fe sqm1, xi;
            fe_const_sqrtm1(sqm1);
            fe_mul(xi, x[k], sqm1);
            x[k] = xi;
        }
        const int sign = (int)(w[7] >> 31);
        fe nx;
        fe_neg(nx, x[k]);
        fe_carry(nx, nx);
        fe_sel(x[k], x[k], nx, fe_is_negative(x[k]) != sign);
        P[k].X = x[k];
        P[k].Y = y[k];
        fe_one(P[k].Z);
    }
    fe T[2];
    fe_mul2<LAT>(T, x[0], y[0], x[1], y[1]);
    P[0].T = T[0];
    P[1].T = T[1];
}
