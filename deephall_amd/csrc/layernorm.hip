// Channel LayerNorm (flax LayerNorm(epsilon=1e-5), psiformer.py:46,48), optionally
// fused with the tanh MLP branch and its residual (psiformer.py:47):
//
//   mode 0:  h = LN_ch(X)
//   mode 1:  h = LN_ch(h + tanh_ch(Z))
//
// One workgroup per (walker, electron); the [C][D] channel tile lives in LDS.
// With z = x - mean_D(x) per channel, s = (mean(z0^2) + eps)^-1/2 and
// a_c = s^2 mean(z0 z_c):
//   n0   = s z0
//   n_t  = s (z_t - a_t z0)
//   n_L  = s (z_L - a_L z0 - 2 sum_t a_t z_t + z0 sum_t (3 a_t^2 - s^2 mean(z_t^2)))
//   n_Sk = s (z_Sk - a_Sk z0 - 2 a_uk u_k + z0 (3 a_uk^2 - s^2 mean(u_k^2))),
//          u_k = sum_t alpha_kt z_t,  a_uk = sum_t alpha_kt a_t
//   y    = scale * n  (+ bias on the value channel)
// tanh_ch: y0 = tanh z0, y_t = tanh' z_t, y_L = tanh' z_L + tanh'' sum_t z_t^2,
//          y_Sk = tanh' z_Sk + tanh'' (sum_t alpha_kt z_t)^2.
#include "dh_internal.h"
#include "device_common.h"

namespace dh {
namespace {

__global__ void layernorm_kernel(const float* X, const float* __restrict__ Z, const float* __restrict__ ln,
                                 const float* __restrict__ geo, float* h, int N, int C, int D, int mode) {
  extern __shared__ float sm[];
  const int T = 2 * N;
  const bool ch = C > 1;
  float* tile = sm;                       // [C][D]
  float* u = tile + (size_t)C * D;        // [3][D]       (ch only)
  float* al = u + (ch ? 3 * D : 0);       // [3][T]
  float* red = al + (ch ? 3 * T : 0);     // reductions: mu[C], p[C], q[T], uu[3]
  float* coef = red + 2 * C + T + 4;      // s, coefL, au[3], coefS[3]
  const int e = blockIdx.x;               // walker*N + electron
  const int b = e / N;
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wid = tid >> 6, nwav = nt >> 6;
  const size_t row0 = (size_t)e * C;

  if (ch) {
    for (int t = tid; t < T; t += nt) {
      const int i = t >> 1;
      const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));
      for (int k = 0; k < 3; ++k) {
        float a;
        if ((t & 1) == 0)
          a = (k == 0) ? -g.z : (k == 1 ? g.w : 0.f);
        else
          a = (k == 0) ? -(g.y * g.w) : (k == 1 ? -(g.y * g.z) : g.x);
        al[k * T + t] = a;
      }
    }
    __syncthreads();
  }

  // ---- load (and optionally apply residual + tanh channel rule)
  for (int d = tid; d < D; d += nt) {
    if (mode == 0) {
      for (int c = 0; c < C; ++c) tile[c * D + d] = X[(row0 + c) * D + d];
    } else {
      const float z0 = Z[row0 * D + d];
      const float y0 = tanhf(z0);
      const float d1 = 1.f - y0 * y0;
      const float d2 = -2.f * y0 * d1;
      tile[d] = h[row0 * D + d] + y0;
      if (ch) {
        float sq = 0.f, u0 = 0.f, u1 = 0.f, u2 = 0.f;
        for (int t = 0; t < T; ++t) {
          const float zt = Z[(row0 + 1 + t) * D + d];
          sq = fmaf(zt, zt, sq);
          u0 = fmaf(al[t], zt, u0);
          u1 = fmaf(al[T + t], zt, u1);
          u2 = fmaf(al[2 * T + t], zt, u2);
          tile[(1 + t) * D + d] = h[(row0 + 1 + t) * D + d] + d1 * zt;
        }
        const float zl = Z[(row0 + 1 + T) * D + d];
        tile[(1 + T) * D + d] = h[(row0 + 1 + T) * D + d] + d1 * zl + d2 * sq;
        const float uu[3] = {u0, u1, u2};
        for (int k = 0; k < 3; ++k) {
          const int c = 2 + T + k;
          const float zs = Z[(row0 + c) * D + d];
          tile[c * D + d] = h[(row0 + c) * D + d] + d1 * zs + d2 * uu[k] * uu[k];
        }
      }
    }
  }
  __syncthreads();

  // ---- channel means
  float* mu = red;
  for (int c = wid; c < C; c += nwav) {
    float s = 0.f;
    for (int d = lane; d < D; d += 64) s += tile[c * D + d];
    s = wave_sum(s);
    if (lane == 0) mu[c] = s / D;
  }
  __syncthreads();
  for (int d = tid; d < D; d += nt) {
    for (int c = 0; c < C; ++c) tile[c * D + d] -= mu[c];
    if (ch) {
      float u0 = 0.f, u1 = 0.f, u2 = 0.f;
      for (int t = 0; t < T; ++t) {
        const float zt = tile[(1 + t) * D + d];
        u0 = fmaf(al[t], zt, u0);
        u1 = fmaf(al[T + t], zt, u1);
        u2 = fmaf(al[2 * T + t], zt, u2);
      }
      u[d] = u0;
      u[D + d] = u1;
      u[2 * D + d] = u2;
    }
  }
  __syncthreads();

  // ---- reductions: p_c = mean(z0 z_c), q_t = mean(z_t^2), uu_k = mean(u_k^2)
  float* p = red + C;
  float* q = p + C;
  float* uu = q + T;
  const int nred = ch ? (C + T + 3) : 1;
  for (int r = wid; r < nred; r += nwav) {
    float s = 0.f;
    if (r < C) {
      for (int d = lane; d < D; d += 64) s = fmaf(tile[d], tile[r * D + d], s);
    } else if (r < C + T) {
      const int t = r - C;
      for (int d = lane; d < D; d += 64) {
        const float v = tile[(1 + t) * D + d];
        s = fmaf(v, v, s);
      }
    } else {
      const int k = r - C - T;
      for (int d = lane; d < D; d += 64) {
        const float v = u[k * D + d];
        s = fmaf(v, v, s);
      }
    }
    s = wave_sum(s);
    if (lane == 0) {
      if (r < C)
        p[r] = s / D;
      else if (r < C + T)
        q[r - C] = s / D;
      else
        uu[r - C - T] = s / D;
    }
  }
  __syncthreads();
  if (tid == 0) {
    const float s = 1.f / sqrtf(p[0] + 1e-5f);
    coef[0] = s;
    if (ch) {
      const float s2 = s * s;
      float cl = 0.f;
      for (int t = 0; t < T; ++t) {
        const float at = s2 * p[1 + t];
        cl += 3.f * at * at - s2 * q[t];
      }
      coef[1] = cl;
      for (int k = 0; k < 3; ++k) {
        float au = 0.f;
        for (int t = 0; t < T; ++t) au = fmaf(al[k * T + t], s2 * p[1 + t], au);
        coef[2 + k] = au;
        coef[5 + k] = 3.f * au * au - s2 * uu[k];
      }
    }
  }
  __syncthreads();

  // ---- outputs
  const float s = coef[0];
  const float* gam = ln;
  const float* bet = ln + D;
  for (int d = tid; d < D; d += nt) {
    const float g = gam[d];
    const float z0 = tile[d];
    h[row0 * D + d] = g * (s * z0) + bet[d];
    if (ch) {
      const float s2 = s * s;
      float sum_at_zt = 0.f;
      for (int t = 0; t < T; ++t) {
        const float at = s2 * p[1 + t];
        const float zt = tile[(1 + t) * D + d];
        sum_at_zt = fmaf(at, zt, sum_at_zt);
        h[(row0 + 1 + t) * D + d] = g * s * (zt - at * z0);
      }
      const float aL = s2 * p[1 + T];
      const float nL = tile[(1 + T) * D + d] - aL * z0 - 2.f * sum_at_zt + coef[1] * z0;
      h[(row0 + 1 + T) * D + d] = g * s * nL;
      for (int k = 0; k < 3; ++k) {
        const int c = 2 + T + k;
        const float aS = s2 * p[c];
        const float nS = tile[c * D + d] - aS * z0 - 2.f * coef[2 + k] * u[k * D + d] + coef[5 + k] * z0;
        h[(row0 + c) * D + d] = g * s * nS;
      }
    }
  }
}

// Value-only rows (log psi / MCMC, C == 1): one wave per row, D = 256 * V floats,
// float4 per lane, two-pass mean/variance in registers.  Pure HBM streaming.
template <int V>
__global__ __launch_bounds__(256) void layernorm_value_kernel(const float* X, const float* __restrict__ Z,
                                                              const float* __restrict__ ln, float* h, int rows,
                                                              int mode) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  constexpr int D = 256 * V;
  const size_t b4 = (size_t)row * (D / 4);
  float4 v[V];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const size_t q = b4 + lane + 64 * j;
    if (mode == 0) {
      v[j] = reinterpret_cast<const float4*>(X)[q];
    } else {
      const float4 z = reinterpret_cast<const float4*>(Z)[q];
      const float4 r = reinterpret_cast<const float4*>(h)[q];
      v[j] = make_float4(r.x + tanhf(z.x), r.y + tanhf(z.y), r.z + tanhf(z.z), r.w + tanhf(z.w));
    }
    sum += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  }
  const float mean = wave_sum(sum) * (1.f / D);
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    v[j].x -= mean;
    v[j].y -= mean;
    v[j].z -= mean;
    v[j].w -= mean;
    sq += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
  }
  const float s = 1.f / sqrtf(wave_sum(sq) * (1.f / D) + 1e-5f);
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c4 = lane + 64 * j;
    const float4 g = reinterpret_cast<const float4*>(ln)[c4];
    const float4 bb = reinterpret_cast<const float4*>(ln + D)[c4];
    reinterpret_cast<float4*>(h)[b4 + c4] =
        make_float4(g.x * (s * v[j].x) + bb.x, g.y * (s * v[j].y) + bb.y, g.z * (s * v[j].z) + bb.z,
                    g.w * (s * v[j].w) + bb.w);
  }
}

// Channel rows, N <= 8, D = 256: ONE WAVE per (walker, electron).  Lane l owns columns
// 4l..4l+3 of all C = 2N+5 channel rows in registers; every mean over D is a wave
// reduction — no LDS, no barriers.  Same algebra as layernorm_kernel.
template <int N>
__global__ __launch_bounds__(256) void layernorm_ch_wave_kernel(const float* X, const float* __restrict__ Z,
                                                                const float* __restrict__ ln,
                                                                const float* __restrict__ geo, float* h, int ne,
                                                                int mode) {
  constexpr int T = 2 * N, C = 2 * N + 5, D = 256;
  const int e = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));  // walker*N + electron
  if (e >= ne) return;
  const int lane = threadIdx.x & 63;
  const int b = e / N;
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
  const size_t r4 = (size_t)e * C * (D / 4) + lane;  // float4 index of (row e*C, column quad lane)
  float4 z[C];
  if (mode == 0) {
#pragma unroll
    for (int c = 0; c < C; ++c) z[c] = reinterpret_cast<const float4*>(X)[r4 + c * (D / 4)];
  } else {
    float4 zz[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      zz[c] = reinterpret_cast<const float4*>(Z)[r4 + c * (D / 4)];
      z[c] = reinterpret_cast<const float4*>(h)[r4 + c * (D / 4)];
    }
    // y = h + tanh_ch(Z), componentwise
#define DH_TANH_COMP(F)                                                         \
  {                                                                             \
    const float y0 = tanhf(zz[0].F);                                            \
    const float d1 = 1.f - y0 * y0, d2 = -2.f * y0 * d1;                        \
    float sq = 0.f, u0 = 0.f, u1 = 0.f, u2 = 0.f;                               \
    _Pragma("unroll") for (int t = 0; t < T; ++t) {                             \
      const float zt = zz[1 + t].F;                                             \
      sq = fmaf(zt, zt, sq);                                                    \
      u0 = fmaf(al[0][t], zt, u0);                                              \
      u1 = fmaf(al[1][t], zt, u1);                                              \
      u2 = fmaf(al[2][t], zt, u2);                                              \
      z[1 + t].F += d1 * zt;                                                    \
    }                                                                           \
    z[0].F += y0;                                                               \
    z[1 + T].F += d1 * zz[1 + T].F + d2 * sq;                                   \
    z[2 + T].F += d1 * zz[2 + T].F + d2 * u0 * u0;                              \
    z[3 + T].F += d1 * zz[3 + T].F + d2 * u1 * u1;                              \
    z[4 + T].F += d1 * zz[4 + T].F + d2 * u2 * u2;                              \
  }
    DH_TANH_COMP(x) DH_TANH_COMP(y) DH_TANH_COMP(z) DH_TANH_COMP(w)
#undef DH_TANH_COMP
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
  float4* out = reinterpret_cast<float4*>(h) + r4;
  const float aL = s2 * p[1 + T];
#define DH_LN_OUT(F)                                                                             \
  {                                                                                              \
    const float z0 = z[0].F, gs = g.F * s;                                                       \
    float sat = 0.f;                                                                             \
    _Pragma("unroll") for (int t = 0; t < T; ++t) sat = fmaf(at[t], z[1 + t].F, sat);            \
    o0.F = g.F * (s * z0) + bb.F;                                                                \
    _Pragma("unroll") for (int t = 0; t < T; ++t) ot[t].F = gs * (z[1 + t].F - at[t] * z0);      \
    oL.F = gs * (z[1 + T].F - aL * z0 - 2.f * sat + cl * z0);                                    \
    _Pragma("unroll") for (int k = 0; k < 3; ++k) oS[k].F =                                      \
        gs * (z[2 + T + k].F - s2 * p[2 + T + k] * z0 - 2.f * au[k] * u[k].F + cs[k] * z0);     \
  }
  float4 o0, ot[T], oL, oS[3];
  DH_LN_OUT(x) DH_LN_OUT(y) DH_LN_OUT(z) DH_LN_OUT(w)
#undef DH_LN_OUT
  out[0] = o0;
#pragma unroll
  for (int t = 0; t < T; ++t) out[(1 + t) * (D / 4)] = ot[t];
  out[(1 + T) * (D / 4)] = oL;
#pragma unroll
  for (int k = 0; k < 3; ++k) out[(2 + T + k) * (D / 4)] = oS[k];
}

template <int N>
void launch_ln_wave(const float* X, const float* Z, const float* ln, const float* geo, float* h, int ne, int mode,
                    hipStream_t s) {
  hipLaunchKernelGGL(layernorm_ch_wave_kernel<N>, dim3((ne + 3) / 4), dim3(256), 0, s, X, Z, ln, geo, h, ne, mode);
}

}  // namespace

void launch_layernorm(const Dims& d, const float* X, const float* Z, const float* ln, const float* geo, float* h,
                      int nw, int C, int mode, hipStream_t s) {
  if (C > 1 && d.D == 256 && d.N <= 8) {
    const int ne = nw * d.N;
    switch (d.N) {
      case 1: launch_ln_wave<1>(X, Z, ln, geo, h, ne, mode, s); return;
      case 2: launch_ln_wave<2>(X, Z, ln, geo, h, ne, mode, s); return;
      case 3: launch_ln_wave<3>(X, Z, ln, geo, h, ne, mode, s); return;
      case 4: launch_ln_wave<4>(X, Z, ln, geo, h, ne, mode, s); return;
      case 5: launch_ln_wave<5>(X, Z, ln, geo, h, ne, mode, s); return;
      case 6: launch_ln_wave<6>(X, Z, ln, geo, h, ne, mode, s); return;
      case 7: launch_ln_wave<7>(X, Z, ln, geo, h, ne, mode, s); return;
      default: launch_ln_wave<8>(X, Z, ln, geo, h, ne, mode, s); return;
    }
  }
  if (C == 1 && (d.D == 256 || d.D == 512)) {
    const int rows = nw * d.N;
    if (d.D == 256)
      hipLaunchKernelGGL(layernorm_value_kernel<1>, dim3((rows + 3) / 4), dim3(256), 0, s, X, Z, ln, h, rows, mode);
    else
      hipLaunchKernelGGL(layernorm_value_kernel<2>, dim3((rows + 3) / 4), dim3(256), 0, s, X, Z, ln, h, rows, mode);
    return;
  }
  const bool ch = C > 1;
  const size_t floats = (size_t)C * d.D + (ch ? 3 * d.D + 3 * d.T : 0) + 2 * C + d.T + 4 + 8;
  const int threads = 256;
  ensure_smem(layernorm_kernel, floats * sizeof(float));
  hipLaunchKernelGGL(layernorm_kernel, dim3(nw * d.N), dim3(threads), floats * sizeof(float), s, X, Z, ln, geo, h,
                     d.N, C, d.D, mode);
}

}  // namespace dh
