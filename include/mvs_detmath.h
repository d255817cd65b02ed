/* mvs_detmath.h -- the numerical definition of the reference's OpenCL builtins.
 *
 * clcode.cl calls exp/powr/distance/normalize/round/sqrt whose accuracy OpenCL
 * leaves implementation-defined, and the reference build passes no options, so
 * FP contraction is also implementation-defined.  This build
 * pins them ONCE, here, from IEEE-754 +,-,*,/,sqrt,fma and exact scalings only,
 * so that the CPU oracle (oracle/mvs_oracle.c) and the HIP kernels
 * (cl_multiview_stereo_amd/csrc/ HIP sources) evaluate bit-identically:
 *
 *   exp(float)  -> mvs_expf   (single-precision Cody-Waite + degree-7 Taylor)
 *   exp(double) -> mvs_exp    (Cody-Waite + degree-13 Taylor, fma Horner)
 *   powr(x,y)   -> mvs_powrf  = (float) mvs_exp(y * mvs_log(x))
 *   distance    -> mvs_distance3 = sqrtf((dx*dx + dy*dy) + dz*dz)
 *   normalize   -> mvs_normalize4: v / sqrtf(dot(v,v)), v unchanged if 0
 *   round       -> roundf (half away from zero, exact everywhere)
 *
 * Every translation unit that includes this header must be compiled with
 * -ffp-contract=off and IEEE division/sqrt (HIP's default
 * -fhip-fp32-correctly-rounded-divide-sqrt), no fast-math.
 */
#ifndef MVS_DETMATH_H
#define MVS_DETMATH_H

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MVS_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define MVS_HD static inline
#endif

MVS_HD double mvs_exp(double x) {
  if (x != x) return x;
  if (x > 709.782712893384) return 1.0 / 0.0;
  if (x < -745.1332191019412) return 0.0;
  const double log2e = 1.4426950408889634;
  const double ln2_hi = 6.93147180369123816490e-01; /* 32 significant bits */
  const double ln2_lo = 1.90821492927058770002e-10;
  double k = rint(x * log2e);
  double r = (x - k * ln2_hi) - k * ln2_lo;
  double p = 1.0 / 6227020800.0;          /* 1/13! */
  p = fma(p, r, 1.0 / 479001600.0);       /* 1/12! */
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)k);
}

MVS_HD double mvs_log(double x) {
  if (x != x || x < 0.0) return 0.0 / 0.0;
  if (x == 0.0) return -1.0 / 0.0;
  if (x == 1.0 / 0.0) return x;
  int e;
  double m = frexp(x, &e); /* m in [0.5, 1) */
  if (m < 0.70710678118654752440) {
    m = m * 2.0;
    e = e - 1;
  }
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  double f = m - 1.0;
  double s = f / (2.0 + f); /* |s| <= 0.1716 */
  double s2 = s * s;
  double q = 2.0 / 23.0;
  q = fma(q, s2, 2.0 / 21.0);
  q = fma(q, s2, 2.0 / 19.0);
  q = fma(q, s2, 2.0 / 17.0);
  q = fma(q, s2, 2.0 / 15.0);
  q = fma(q, s2, 2.0 / 13.0);
  q = fma(q, s2, 2.0 / 11.0);
  q = fma(q, s2, 2.0 / 9.0);
  q = fma(q, s2, 2.0 / 7.0);
  q = fma(q, s2, 2.0 / 5.0);
  q = fma(q, s2, 2.0 / 3.0);
  double logm = fma(s * s2, q, 2.0 * s);
  double de = (double)e;
  return de * ln2_hi + (logm + de * ln2_lo);
}

/* exp(float): a single-precision kernel (FP32 issues at twice the FP64 rate
 * on gfx950 and the refinement evaluates ~10^4 of these per superpixel):
 * Cody-Waite with fma, degree-7 Taylor by fma Horner, exact scaling.  Results
 * stay normal: x < -86.5 gives 0, x > ln(FLT_MAX) gives +inf.  <= 2 ulp. */
MVS_HD float mvs_expf(float x) {
  /* one range test on the common path (a NaN fails it); the rare cases after */
  if (!(x >= -86.5f && x <= 88.72283935546875f)) return x != x ? x : (x > 0.0f ? 1.0f / 0.0f : 0.0f);
  const float log2e = 1.44269502162933349609375f;
  const float ln2_hi = 0.693147182464599609375f;   /* (float) ln 2 */
  const float ln2_lo = -1.904654323148236e-09f;    /* ln 2 - ln2_hi */
  float k = rintf(x * log2e);
  float r = fmaf(-k, ln2_hi, x);
  r = fmaf(-k, ln2_lo, r);
  float p = 1.0f / 5040.0f;
  p = fmaf(p, r, 1.0f / 720.0f);
  p = fmaf(p, r, 1.0f / 120.0f);
  p = fmaf(p, r, 1.0f / 24.0f);
  p = fmaf(p, r, 1.0f / 6.0f);
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  return ldexpf(p, (int)k);
}

/* OpenCL powr(x, y), defined for x >= 0 */
MVS_HD float mvs_powrf(float x, float y) {
  if (x != x || y != y || x < 0.0f) return 0.0f / 0.0f;
  if (x == 0.0f) return y > 0.0f ? 0.0f : (y < 0.0f ? 1.0f / 0.0f : 0.0f / 0.0f);
  return (float)mvs_exp((double)y * mvs_log((double)x));
}

MVS_HD float mvs_distance3(float ax, float ay, float az, float bx, float by, float bz) {
  float dx = ax - bx, dy = ay - by, dz = az - bz;
  float s = dx * dx;
  s = s + dy * dy;
  s = s + dz * dz;
  return sqrtf(s);
}

#endif /* MVS_DETMATH_H */
