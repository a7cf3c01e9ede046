// Device pieces of the Metropolis walker update shared by mcmc.hip (propose / accept kernels)
// and det.hip (det_value_kernel's fused accept + next proposal, round 5).
#pragma once
#include "dh_internal.h"
#include "device_common.h"

namespace dh {

constexpr int kPurposeMcmc = 0, kPurposeInit = 1;

// One electron's move: (th, ph) -> x2[e] (and its geometry sin/cos of the stored f32
// angles into geo[e], as input_kernel computes it, when geo is given).
__device__ __forceinline__ void propose_one(float th_f, float ph_f, float* __restrict__ x2, float* __restrict__ geo,
                                            int e, int b, int i, int N, float width, uint64_t seed, uint64_t step,
                                            int64_t woff, const float* __restrict__ noise) {
  float xi, up;
  if (noise) {
    xi = noise[(size_t)b * (2 * N + 1) + i];
    up = noise[(size_t)b * (2 * N + 1) + N + i];
  } else {
    u32x4 r = dh_random(seed, kPurposeMcmc, (uint32_t)i, (uint64_t)(woff + b), step);
    xi = box_muller(r.x, r.y);
    up = u01(r.z);
  }
  // The move is evaluated in double (the same formulas as mcmc.py:71-101, then rounded to
  // f32): phi = sign(y) arccos(x / sin theta) loses ~eps / |sin phi| near phi = 0, pi in
  // f32 (the reference's own f32 result is off by up to ~3e-4 rad there); in double the
  // stored walker is the correctly rounded exact move.  ~20 double ops per electron.
  const double th = th_f, ph = ph_f;
  const double thp = atan((double)xi * (double)width);
  const double php = (double)up * 2.0 * M_PI;
  double stp, ctp, spp, cpp, st, ct, sp, cp;
  sincos(thp, &stp, &ctp);
  sincos(php, &spp, &cpp);
  sincos(th, &st, &ct);
  sincos(ph, &sp, &cp);
  const double X = stp * cpp, Y = stp * spp, Z = ctp;
  // R_y(theta) then R_z(phi)
  const double ax = ct * X + st * Z, ay = Y, az = -st * X + ct * Z;
  const double x2x = cp * ax - sp * ay, x2y = sp * ax + cp * ay, x2z = az;
  const double thd = acos(fmin(fmax(x2z, -1.0), 1.0));
  const double sgn = (x2y > 0.0) ? 1.0 : ((x2y < 0.0) ? -1.0 : 0.0);
  const double q = x2x / sin(thd);
  // clip(q) with NaN propagation as jnp.clip (NaN in -> NaN out)
  const double qc = (q != q) ? q : fmin(fmax(q, -1.0), 1.0);
  const float thn = (float)thd;
  const float phn = (float)(sgn * acos(qc));
  x2[2 * e] = thn;
  x2[2 * e + 1] = phn;
  if (geo) {
    float gst, gct, gsp, gcp;
    sincosf(thn, &gst, &gct);
    sincosf(phn, &gsp, &gcp);
    *reinterpret_cast<float4*>(geo + 4 * (size_t)e) = make_float4(gst, gct, gsp, gcp);
  }
}


// accept of walker b at `step` (mcmc.py:55-62): u from the injected noise or the walker's
// Philox stream; true when 2 Re log psi(x') - lp > log u
__device__ __forceinline__ bool accept_one(float lp2, float lp_old, int b, int N, uint64_t seed, uint64_t step,
                                           int64_t woff, const float* __restrict__ noise) {
  float u;
  if (noise) {
    u = noise[(size_t)b * (2 * N + 1) + 2 * N];
  } else {
    u32x4 r = dh_random(seed, kPurposeMcmc, (uint32_t)N, (uint64_t)(woff + b), step);
    u = u01(r.x);
  }
  return (lp2 - lp_old) > logf(u);
}

}  // namespace dh
