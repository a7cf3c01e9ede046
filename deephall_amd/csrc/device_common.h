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

}  // namespace dh
