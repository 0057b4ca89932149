// trig.h -- f64 sincos for the env step's Euler angles.
//
// The device library's sincos(double) spends ~95 VALU instructions per call
// on a double-double range reduction (plus a Payne-Hanek path for huge
// arguments).  The env step evaluates three of them per env on a
// latency-bound critical path (one wave per SIMD at 65,536 envs), so this
// version does the medium-range reduction with three FMAs (|x| < 2^19 rad;
// k*P1 is exact there, so r carries <= 0.5 ulp of rounding) and evaluates
// one shared pair of minimax polynomials on [-pi/4, pi/4] (the classic
// fdlibm k_sin/k_cos coefficient sets, with k_cos's compensated 1 - z/2).
// Error <= 1 ulp vs a correctly rounded sin/cos (checked against numpy on
// the host by tests/test_trig_host.py).  Arguments outside the fast range,
// infinities and NaN go to the library sincos.
#pragma once

#include <cmath>
#include <cstdint>

#ifndef __HIP__
#define DR_HD
#else
#define DR_HD __host__ __device__
#endif

namespace dr {

struct SinCos {
    double s, c;
};

// x with its sign bit XORed by bit 31 of m (m's other bits zero).
DR_HD inline double flip_sign_hi(double x, uint32_t m) {
    return __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, x) ^ ((uint64_t)m << 32));
}

// r in [-pi/4, pi/4] (slightly beyond by rounding of k): sin(r), cos(r).
DR_HD inline SinCos sincos_kernel(double r) {
    const double z = r * r;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    // sin: r + r^3 (S1 + z (S2 + ... ))
    double ps = fma(z, S6, S5);
    ps = fma(z, ps, S4);
    ps = fma(z, ps, S3);
    ps = fma(z, ps, S2);
    const double rz = r * z;
    const double s = fma(rz, fma(z, ps, S1), r);
    // cos: (1 - z/2) + z^2 (C1 + z (C2 + ...)), 1 - z/2 compensated
    double pc = fma(z, C6, C5);
    pc = fma(z, pc, C4);
    pc = fma(z, pc, C3);
    pc = fma(z, pc, C2);
    pc = fma(z, pc, C1);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double corr = (1.0 - w) - hz;  // exact rounding error of w
    const double c = w + fma(z * z, pc, corr);
    return {s, c};
}

DR_HD inline bool sincos_fast_range(double x) { return fabs(x) < 524288.0; }

// Precondition: sincos_fast_range(x).
DR_HD inline SinCos sincos_medium(double x) {
    const double kInvPio2 = 6.36619772367581382433e-01;
    const double P1 = 1.57079632679489655800e+00;   // RN(pi/2)
    const double P2 = 6.12323399573676603587e-17;   // RN(pi/2 - P1)
    const double P3 = -1.49738490485916983053e-33;  // RN(pi/2 - P1 - P2)
    const double k = rint(x * kInvPio2);
    double r = fma(-k, P1, x);  // exact: |k| < 2^19
    r = fma(-k, P2, r);
    r = fma(-k, P3, r);
    const SinCos t = sincos_kernel(r);
    const int q = (int)k;
    const double s0 = (q & 1) ? t.c : t.s;
    const double c0 = (q & 1) ? t.s : t.c;
    // the quadrant's sign flips as a sign-bit XOR of the high word: bit 1 of
    // q (of q + 1 for cos) moved to bit 31 -- the same bits as negating, in
    // two integer ops per result (round 5: the compiler's select form of
    // `(q & 2) ? -s0 : s0` took five)
    const uint32_t sgn_s = ((uint32_t)q << 30) & 0x80000000u;
    const uint32_t sgn_c = ((uint32_t)(q + 1) << 30) & 0x80000000u;
    return {flip_sign_hi(s0, sgn_s), flip_sign_hi(c0, sgn_c)};
}

// ---------------------------------------------------------------------------
// f32 state mode: the same shared-reduction scheme in single precision.  The
// reduction runs in f64 (k = rint(x 2/pi), r = x - k pi/2 with a two-part
// pi/2: the f32 argument is exact in f64 and r is far more accurate than one
// f32 ulp for |x| < 2^19), the polynomials in f32 on [-pi/4, pi/4] (the
// cephes sinf / cosf minimax sets).  <= 2 ulp from the correctly rounded
// f32 sin / cos (tests/test_trig_host.py); replaces ~3x the instructions of
// the library sincosf, whose large-argument path it keeps for |x| >= 2^19,
// infinities and NaN.
struct SinCosF {
    float s, c;
};

DR_HD inline bool sincosf_fast_range(float x) { return fabsf(x) < 524288.0f; }

// Precondition: sincosf_fast_range(x).
DR_HD inline SinCosF sincosf_medium(float xf) {
    const double kInvPio2 = 6.36619772367581382433e-01;
    const double P1 = 1.57079632679489655800e+00;   // RN(pi/2)
    const double P2 = 6.12323399573676603587e-17;   // RN(pi/2 - P1)
    const double x = (double)xf;
    const double k = rint(x * kInvPio2);
    const float r = (float)fma(-k, P2, fma(-k, P1, x));
    const float z = r * r;
    float ps = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
    ps = fmaf(z, ps, -1.6666654611e-1f);
    const float sr = fmaf(r * z, ps, r);
    float pc = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    pc = fmaf(z, pc, 4.166664568298827e-2f);
    const float cr = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
    const int q = (int)k & 3;
    const float s0 = (q & 1) ? cr : sr;
    const float c0 = (q & 1) ? sr : cr;
    return {(q & 2) ? -s0 : s0, ((q + 1) & 2) ? -c0 : c0};
}

}  // namespace dr
