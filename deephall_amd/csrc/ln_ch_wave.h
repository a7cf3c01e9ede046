// Channel LayerNorm of ONE electron's C = 2N+5 rows by one wave (D = 256; lane l owns
// columns 4l..4l+3 of every row, in registers): layernorm.hip's algebra (header there),
// shared by layernorm_ch_wave_kernel (rows in HBM) and the channel chain kernel (rows in
// LDS).  src(c): row c of X (mode 0) or of Z (mode 1); res(c): row c of h (mode 1);
// dst(c, v): the normalised row c.  b: the walker (flow coefficients from geo).
#pragma once
#include "device_common.h"

namespace dh {

template <int N, class Src, class Res, class Dst>
__device__ __forceinline__ void ln_ch_wave(int mode, Src src, Res res, Dst dst, const float* __restrict__ ln,
                                           const float* __restrict__ geo, int b, int lane) {
  constexpr int T = 2 * N, C = 2 * N + 5, D = 256;
  // flow coefficients alpha[k][t] (uniform over the wave)
  float al[3][T];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));  // st ct sp cp
    al[0][2 * i] = -g.z;
    al[1][2 * i] = g.w;
    al[2][2 * i] = 0.f;
    al[0][2 * i + 1] = -(g.y * g.w);
    al[1][2 * i + 1] = -(g.y * g.z);
    al[2][2 * i + 1] = g.x;
  }
  float4 z[C];
  if (mode == 0) {
#pragma unroll
    for (int c = 0; c < C; ++c) z[c] = src(c);
  } else {
    // y = h + tanh_ch(Z), componentwise; Z streamed channel by channel
    const float4 z0 = src(0);
    float4 y0, d1, d2;
#define DH_TANH_D(F)          \
  y0.F = tanhf(z0.F);         \
  d1.F = 1.f - y0.F * y0.F;   \
  d2.F = -2.f * y0.F * d1.F;
    DH_TANH_D(x) DH_TANH_D(y) DH_TANH_D(z) DH_TANH_D(w)
#undef DH_TANH_D
    float4 sq = make_float4(0.f, 0.f, 0.f, 0.f), uz[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) uz[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    z[0] = res(0);
    z[0].x += y0.x;
    z[0].y += y0.y;
    z[0].z += y0.z;
    z[0].w += y0.w;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float4 zt = src(1 + t);
      z[1 + t] = res(1 + t);
#define DH_TANH_T(F)                        \
  sq.F = fmaf(zt.F, zt.F, sq.F);            \
  uz[0].F = fmaf(al[0][t], zt.F, uz[0].F);  \
  uz[1].F = fmaf(al[1][t], zt.F, uz[1].F);  \
  uz[2].F = fmaf(al[2][t], zt.F, uz[2].F);  \
  z[1 + t].F = fmaf(d1.F, zt.F, z[1 + t].F);
      DH_TANH_T(x) DH_TANH_T(y) DH_TANH_T(z) DH_TANH_T(w)
#undef DH_TANH_T
    }
#pragma unroll
    for (int c = 1 + T; c < C; ++c) {
      const float4 zc = src(c);
      z[c] = res(c);
      const float4 w = (c == 1 + T) ? sq : uz[c - 2 - T];
      const bool L = c == 1 + T;
#define DH_TANH_O(F) z[c].F += d1.F * zc.F + d2.F * (L ? w.F : w.F * w.F);
      DH_TANH_O(x) DH_TANH_O(y) DH_TANH_O(z) DH_TANH_O(w)
#undef DH_TANH_O
    }
  }
  // channel means, centre
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float mu = wave_sum((z[c].x + z[c].y) + (z[c].z + z[c].w)) * (1.f / D);
    z[c].x -= mu;
    z[c].y -= mu;
    z[c].z -= mu;
    z[c].w -= mu;
  }
  float4 u[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    u[k] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      u[k].x = fmaf(al[k][t], z[1 + t].x, u[k].x);
      u[k].y = fmaf(al[k][t], z[1 + t].y, u[k].y);
      u[k].z = fmaf(al[k][t], z[1 + t].z, u[k].z);
      u[k].w = fmaf(al[k][t], z[1 + t].w, u[k].w);
    }
  }
  auto dot4 = [](const float4& a, const float4& b) { return (a.x * b.x + a.y * b.y) + (a.z * b.z + a.w * b.w); };
  float p[C], q[T], uu[3];
#pragma unroll
  for (int c = 0; c < C; ++c) p[c] = wave_sum(dot4(z[0], z[c])) * (1.f / D);
#pragma unroll
  for (int t = 0; t < T; ++t) q[t] = wave_sum(dot4(z[1 + t], z[1 + t])) * (1.f / D);
#pragma unroll
  for (int k = 0; k < 3; ++k) uu[k] = wave_sum(dot4(u[k], u[k])) * (1.f / D);
  const float s = 1.f / sqrtf(p[0] + 1e-5f), s2 = s * s;
  float at[T], cl = 0.f;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    at[t] = s2 * p[1 + t];
    cl += 3.f * at[t] * at[t] - s2 * q[t];
  }
  float au[3], cs[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    au[k] = 0.f;
#pragma unroll
    for (int t = 0; t < T; ++t) au[k] = fmaf(al[k][t], at[t], au[k]);
    cs[k] = 3.f * au[k] * au[k] - s2 * uu[k];
  }
  const float4 g = reinterpret_cast<const float4*>(ln)[lane];
  const float4 bb = reinterpret_cast<const float4*>(ln + D)[lane];
  const float aL = s2 * p[1 + T];
  // each output row is written as soon as it is formed (no arrays of outputs held: the
  // chain kernel runs this at a 256-VGPR budget); the arithmetic per element is unchanged
  const float4 gs = make_float4(g.x * s, g.y * s, g.z * s, g.w * s);
  dst(0, make_float4(g.x * (s * z[0].x) + bb.x, g.y * (s * z[0].y) + bb.y, g.z * (s * z[0].z) + bb.z,
                     g.w * (s * z[0].w) + bb.w));
#pragma unroll
  for (int t = 0; t < T; ++t)
    dst(1 + t, make_float4(gs.x * (z[1 + t].x - at[t] * z[0].x), gs.y * (z[1 + t].y - at[t] * z[0].y),
                           gs.z * (z[1 + t].z - at[t] * z[0].z), gs.w * (z[1 + t].w - at[t] * z[0].w)));
  float4 sat = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int t = 0; t < T; ++t) {
    sat.x = fmaf(at[t], z[1 + t].x, sat.x);
    sat.y = fmaf(at[t], z[1 + t].y, sat.y);
    sat.z = fmaf(at[t], z[1 + t].z, sat.z);
    sat.w = fmaf(at[t], z[1 + t].w, sat.w);
  }
#define DH_LN_L(F) gs.F*(z[1 + T].F - aL * z[0].F - 2.f * sat.F + cl * z[0].F)
  dst(1 + T, make_float4(DH_LN_L(x), DH_LN_L(y), DH_LN_L(z), DH_LN_L(w)));
#undef DH_LN_L
#pragma unroll
  for (int k = 0; k < 3; ++k) {
#define DH_LN_S(F) gs.F*(z[2 + T + k].F - s2 * p[2 + T + k] * z[0].F - 2.f * au[k] * u[k].F + cs[k] * z[0].F)
    dst(2 + T + k, make_float4(DH_LN_S(x), DH_LN_S(y), DH_LN_S(z), DH_LN_S(w)));
#undef DH_LN_S
  }
}

}  // namespace dh
