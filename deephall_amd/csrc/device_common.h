// Device-side helpers: complex float, Philox4x32-10 counter RNG, wave reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dh {

constexpr float kPi = 3.14159265358979323846f;

// ---------------------------------------------------------------- complex
struct cf {
  float re, im;
};
__device__ __forceinline__ cf cmk(float r, float i) { return cf{r, i}; }
__device__ __forceinline__ cf operator+(cf a, cf b) { return cf{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cf operator-(cf a, cf b) { return cf{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cf operator*(cf a, cf b) {
  return cf{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ cf operator*(float s, cf a) { return cf{s * a.re, s * a.im}; }
__device__ __forceinline__ cf& operator+=(cf& a, cf b) {
  a.re += b.re;
  a.im += b.im;
  return a;
}
__device__ __forceinline__ cf& operator-=(cf& a, cf b) {
  a.re -= b.re;
  a.im -= b.im;
  return a;
}
// a += b * c
__device__ __forceinline__ void cfma(cf& a, cf b, cf c) {
  a.re = fmaf(b.re, c.re, fmaf(-b.im, c.im, a.re));
  a.im = fmaf(b.re, c.im, fmaf(b.im, c.re, a.im));
}
__device__ __forceinline__ cf cdiv(cf a, cf b) {
  // Smith's algorithm
  if (fabsf(b.re) >= fabsf(b.im)) {
    float r = b.im / b.re, den = b.re + b.im * r;
    return cf{(a.re + a.im * r) / den, (a.im - a.re * r) / den};
  } else {
    float r = b.re / b.im, den = b.re * r + b.im;
    return cf{(a.re * r + a.im) / den, (a.im * r - a.re) / den};
  }
}
__device__ __forceinline__ float cabs1(cf a) { return fabsf(a.re) + fabsf(a.im); }

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += W0;
      k1 += W1;
    }
    uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
  }
  return c;
}
// Counter layout shared with oracle/philox.py:
//   ctr = (lane_id | purpose << 24, walker (low 32 bits), step low, step high)
//   key = (seed low, seed high)
__device__ __forceinline__ u32x4 dh_random(uint64_t seed, int purpose, uint32_t lane_id, uint64_t walker,
                                           uint64_t step) {
  u32x4 c{lane_id | (uint32_t(purpose) << 24), uint32_t(walker), uint32_t(step), uint32_t(step >> 32)};
  return philox4x32_10(c, uint32_t(seed), uint32_t(seed >> 32));
}
// [0,1) with 24 random bits
__device__ __forceinline__ float u01(uint32_t b) { return float(b >> 8) * (1.0f / 16777216.0f); }
// (0,1]
__device__ __forceinline__ float u01_open0(uint32_t b) { return float((b >> 8) + 1u) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float box_muller(uint32_t b0, uint32_t b1) {
  float u1 = u01_open0(b0), u2 = u01(b1);
  return sqrtf(-2.0f * logf(u1)) * cosf(2.0f * kPi * u2);
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Sum over each 16-lane row (DPP: quad swaps, then the half-row and row mirrors); every
// lane of the row receives the sum.  VALU only: no LDS permute round trips.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

// tanh by the odd rational form XLA / Eigen evaluate for f32 (argument clamped to
// +-7.90531, x itself below 4e-4; the quotient by reciprocal + one Newton step): a few ulp
// against float64 tanh (tests/test_gpu_kernels.py), ~16 VALU operations against libm's ~40
__device__ __forceinline__ float tanh_rat(float x) {
  const float c = fminf(fmaxf(x, -7.90531110763549805f), 7.90531110763549805f);
  const float x2 = c * c;
  float p = fmaf(x2, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = fmaf(p, x2, -8.60467152213735e-11f);
  p = fmaf(p, x2, 5.12229709037114e-08f);
  p = fmaf(p, x2, 1.48572235717979e-05f);
  p = fmaf(p, x2, 6.37261928875436e-04f);
  p = fmaf(p, x2, 4.89352455891786e-03f);
  float q = fmaf(x2, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = fmaf(q, x2, 2.26843463243900e-03f);
  q = fmaf(q, x2, 4.89352518554385e-03f);
  float rq = __builtin_amdgcn_rcpf(q);  // q in [4.9e-3, 2.1e-2]: one Newton step
  rq = rq * fmaf(-q, rq, 2.f);
  return fabsf(x) < 4e-4f ? x : (c * p) * rq;
}

// tanhf with the device library's exact operation sequence (ROCm 7 ocml, gfx950 ISA of
// tanhf: |x| < 0.625 odd polynomial in x^2, else 1 - 2 / (exp(2|x|) + 1) with exp from
// v_exp_f32 + split log2(e) + ldexp), but both branches evaluated and selected: no
// divergent control flow, so a register-heavy caller (gemm_lnch MODE 1) does not spill
// around it.  Bit-identical to tanhf for every f32 (tools/tanh_exact.hip, exhaustive).
__device__ __forceinline__ float tanh_ocml(float x) {
#pragma clang fp contract(off)
  const float y = fabsf(x);
  // |x| >= 0.625
  const float t = y + y;
  const float p = t * 0x1.715476p+0f;  // log2(e) hi
  const float r = __builtin_rintf(p);
  const float f = p - r;
  float e = __builtin_fmaf(t, 0x1.715476p+0f, -p);
  e = __builtin_fmaf(t, 0x1.4ae0bep-26f, e);  // log2(e) lo
  float v = __builtin_amdgcn_ldexpf(__builtin_amdgcn_exp2f(f + e), (int)r);
  v = (t < -0x1.9d1da0p+6f) ? 0.f : v;
  v = (t > 0x1.62e430p+6f) ? __builtin_inff() : v;
  const float big = __builtin_fmaf(__builtin_amdgcn_rcpf(v + 1.f), -2.f, 1.f);
  // |x| < 0.625
  const float x2 = x * x;
  float s = __builtin_fmaf(-0x1.758e7ap-8f, x2, 0x1.521192p-6f);
  s = __builtin_fmaf(x2, s, -0x1.b8389cp-5f);
  s = __builtin_fmaf(x2, s, 0x1.110704p-3f);
  s = __builtin_fmaf(x2, s, -0x1.555532p-2f);
  const float small = __builtin_fmaf(x2, y * s, y);
  const float m = (y < 0.625f) ? small : big;
  return __builtin_bit_cast(float, (__builtin_bit_cast(uint32_t, m) & 0x7fffffffu) |
                                       (__builtin_bit_cast(uint32_t, x) & 0x80000000u));
}

}  // namespace dh
