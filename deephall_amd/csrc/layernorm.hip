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
#include <type_traits>

#include "dh_internal.h"
#include "device_common.h"
#include "ln_ch_wave.h"

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

// Channel rows, D = 256: ONE WAVE per (walker, electron).  Lane l owns columns
// 4l..4l+3 of all C = 2N+5 channel rows in registers; every mean over D is a wave
// reduction — no LDS, no barriers.  Same algebra as layernorm_kernel.  The tanh branch
// (mode 1) streams Z one channel at a time, so only the C pre-LN rows are held
// (4C VGPRs: 180 at N = 20, one wave per SIMD there).
template <int N>
__global__ __launch_bounds__(256) void layernorm_ch_wave_kernel(const float* X, const float* __restrict__ Z,
                                                                const float* __restrict__ ln,
                                                                const float* __restrict__ geo, float* h, int ne,
                                                                int mode) {
  constexpr int C = 2 * N + 5, D = 256;
  const int e = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));  // walker*N + electron
  if (e >= ne) return;
  const int lane = threadIdx.x & 63;
  const size_t r4 = (size_t)e * C * (D / 4) + lane;  // float4 index of (row e*C, column quad lane)
  const float4* src = reinterpret_cast<const float4*>(mode == 0 ? X : Z);
  float4* hv = reinterpret_cast<float4*>(h);
  ln_ch_wave<N>(
      mode, [&](int c) { return src[r4 + c * (D / 4)]; }, [&](int c) { return hv[r4 + c * (D / 4)]; },
      [&](int c, const float4& v) { hv[r4 + c * (D / 4)] = v; }, ln, geo, e / N, lane);
}

// Channel rows for large N (C = 2N+5 up to 45), D = 256: FOUR WAVES per (walker,
// electron), wave w owning columns 64w..64w+63 (one float per lane per channel row, C
// VGPRs instead of 4C), so several electrons share a SIMD.  The C + (C + T + 3) sums over
// D are transposed through a per-wave LDS scratch 16 rows at a time (16 writes, 16 reads
// and 2 shuffles per 16 sums instead of 6 shuffles per sum), then the four waves'
// partials are combined through LDS (two barriers in all).
template <int N>
__global__ __launch_bounds__(256) void layernorm_ch_quad_kernel(const float* X, const float* __restrict__ Z,
                                                                const float* __restrict__ ln,
                                                                const float* __restrict__ geo, float* h, int ne,
                                                                int mode, const float* __restrict__ W0f, int n_up) {
  constexpr int T = 2 * N, C = 2 * N + 5, D = 256, NR = C + T + 3;
  __shared__ float red[4][C + NR];
  __shared__ float al[3][T];       // flow coefficients (broadcast reads)
  __shared__ float tb[4][16 * 65];  // per-wave transpose scratch
  const int e = blockIdx.x;         // walker*N + electron
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = e / N;
  if (threadIdx.x < N) {
    const int i = threadIdx.x;
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));  // st ct sp cp
    al[0][2 * i] = -g.z;
    al[1][2 * i] = g.w;
    al[2][2 * i] = 0.f;
    al[0][2 * i + 1] = -(g.y * g.w);
    al[1][2 * i + 1] = -(g.y * g.z);
    al[2][2 * i + 1] = g.x;
  }
  __syncthreads();
  float* tw = tb[w];
  // sums over this wave's 64 columns of R per-lane values getv(r) -> dst[r]
  auto rows_sum = [&](auto getv, auto R_, float* dst) {
    constexpr int R = decltype(R_)::value;
#pragma unroll
    for (int r0 = 0; r0 < R; r0 += 16) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (r0 + j < R) tw[j * 65 + lane] = getv(r0 + j);
      __builtin_amdgcn_wave_barrier();
      const int j = lane >> 2, q = lane & 3;
      float v = 0.f;
#pragma unroll
      for (int m = 0; m < 16; ++m) v += tw[j * 65 + 16 * q + m];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      if (q == 0 && r0 + j < R) dst[r0 + j] = v;
      __builtin_amdgcn_wave_barrier();
    }
  };
  const size_t r0 = (size_t)e * C * D + 64 * w + lane;  // (row e*C, this lane's column)
  float z[C];
  if (mode == 0 && W0f) {
    // layer 1 (round 5): the residual h0 = f W0 of input.hip formed here from the geometry
    // (the GEMM wrote t without it): z_c = t_c + f_c . W0[:, col], the GEMM epilogue's sum order
    const int col = 64 * w + lane, i = e - b * N;
    const float w0 = W0f[col], w1 = W0f[D + col], w2 = W0f[2 * D + col], w3 = W0f[3 * D + col];
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)e);  // st ct sp cp
    const float st = g.x, ct = g.y, sp = g.z, cp = g.w;
    const float rx = st * cp, ry = st * sp, rz = ct;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c == 0) {
        f = make_float4(rz, rx, ry, (i < n_up) ? 1.f : -1.f);
      } else if (c <= T) {
        const int t = c - 1;
        if ((t >> 1) == i) f = ((t & 1) == 0) ? make_float4(-st, ct * cp, ct * sp, 0.f) : make_float4(0.f, -sp, cp, 0.f);
      } else if (c == T + 1) {
        f = make_float4(-2.f * rz, -2.f * rx, -2.f * ry, 0.f);
      } else {
        const int k = c - T - 2;  // 0:x 1:y 2:z
        f = make_float4((k == 2) ? 0.f : -rz, (k == 0) ? 0.f : -rx, (k == 1) ? 0.f : -ry, 0.f);
      }
      z[c] = X[r0 + (size_t)c * D] + (f.x * w0 + f.y * w1 + f.z * w2 + f.w * w3);
    }
  } else if (mode == 0) {
#pragma unroll
    for (int c = 0; c < C; ++c) z[c] = X[r0 + (size_t)c * D];
  } else {
    const float zz0 = Z[r0];
    const float y0 = tanhf(zz0), d1 = 1.f - y0 * y0, d2 = -2.f * y0 * d1;
    float sq = 0.f, u0 = 0.f, u1 = 0.f, u2 = 0.f;
    z[0] = h[r0] + y0;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float zt = Z[r0 + (size_t)(1 + t) * D];
      sq = fmaf(zt, zt, sq);
      u0 = fmaf(al[0][t], zt, u0);
      u1 = fmaf(al[1][t], zt, u1);
      u2 = fmaf(al[2][t], zt, u2);
      z[1 + t] = fmaf(d1, zt, h[r0 + (size_t)(1 + t) * D]);
    }
    z[1 + T] = h[r0 + (size_t)(1 + T) * D] + d1 * Z[r0 + (size_t)(1 + T) * D] + d2 * sq;
    const float uu[3] = {u0, u1, u2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const size_t rc = r0 + (size_t)(2 + T + k) * D;
      z[2 + T + k] = h[rc] + d1 * Z[rc] + d2 * uu[k] * uu[k];
    }
  }
  // channel means
  __shared__ float mu[C];
  rows_sum([&](int c) { return z[c]; }, std::integral_constant<int, C>{}, red[w]);
  __syncthreads();
  if (threadIdx.x < C) {
    const int c = threadIdx.x;
    mu[c] = ((red[0][c] + red[1][c]) + (red[2][c] + red[3][c])) * (1.f / D);
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < C; ++c) z[c] -= mu[c];
  float u[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    u[k] = 0.f;
#pragma unroll
    for (int t = 0; t < T; ++t) u[k] = fmaf(al[k][t], z[1 + t], u[k]);
  }
  // p_c = mean(z0 z_c), q_t = mean(z_t^2), uu_k = mean(u_k^2)
  rows_sum(
      [&](int r) {
        if (r < C) return z[0] * z[r];
        if (r < C + T) return z[1 + r - C] * z[1 + r - C];
        return u[r - C - T] * u[r - C - T];
      },
      std::integral_constant<int, NR>{}, red[w] + C);
  __syncthreads();
  // coefficients, once per electron (wave 0): fin = the D-means, at_t, cl, au_k, cs_k
  __shared__ float fin[NR], cf[T + 12];
  for (int r = threadIdx.x; r < NR; r += 256)
    fin[r] = ((red[0][C + r] + red[1][C + r]) + (red[2][C + r] + red[3][C + r])) * (1.f / D);
  __syncthreads();
  const float s = 1.f / sqrtf(fin[0] + 1e-5f), s2 = s * s;
  if (w == 0) {
    float clv = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
    if (lane < T) {
      const float at = s2 * fin[1 + lane];
      cf[lane] = at;
      clv = 3.f * at * at - s2 * fin[C + lane];
      a0 = al[0][lane] * at;
      a1 = al[1][lane] * at;
      a2 = al[2][lane] * at;
    }
    clv = wave_sum(clv);
    a0 = wave_sum(a0);
    a1 = wave_sum(a1);
    a2 = wave_sum(a2);
    if (lane == 0) {
      cf[T] = clv;
      cf[T + 1] = s2 * fin[1 + T];  // aL
      const float au[3] = {a0, a1, a2};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        cf[T + 2 + k] = au[k];
        cf[T + 5 + k] = 3.f * au[k] * au[k] - s2 * fin[C + T + k];
        cf[T + 8 + k] = s2 * fin[2 + T + k];  // aS_k
      }
    }
  }
  __syncthreads();
  const int col = 64 * w + lane;
  const float g = ln[col], bb = ln[D + col], gs = g * s, z0 = z[0];
  float sat = 0.f;
  h[r0] = g * (s * z0) + bb;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const float at = cf[t];
    sat = fmaf(at, z[1 + t], sat);
    h[r0 + (size_t)(1 + t) * D] = gs * (z[1 + t] - at * z0);
  }
  h[r0 + (size_t)(1 + T) * D] = gs * (z[1 + T] - cf[T + 1] * z0 - 2.f * sat + cf[T] * z0);
#pragma unroll
  for (int k = 0; k < 3; ++k)
    h[r0 + (size_t)(2 + T + k) * D] =
        gs * (z[2 + T + k] - cf[T + 8 + k] * z0 - 2.f * cf[T + 2 + k] * u[k] + cf[T + 5 + k] * z0);
}

// Layer 1 of the local energy at N = 10, 20 in ONE launch (round 6), from the o~ rows of
// attention_feat2_kernel (psiformer.py:44-48 on the 2N+5 channel rows):
//   h = LN_ch2(h1 + tanh_ch(h1 Wm + bm)),  h1 = LN_ch1(f W0 + o~ U + bol).
// Four waves per electron as layernorm_ch_quad_kernel (lane = one feature column, all C channel
// rows in registers, the same transposed sums):
//   x_c = f_c . W0[:, col] + o~_c . U[:, col] (+ bol on the value row): 4 + 20 FMAs per row from
//     the lane's columns of W0 / U and the electron's o~ rows (LDS, broadcast reads);
//   LN_ch1 -> h1 (the quad kernel's statistics and output algebra);
//   h1 Wm + bm in coefficient space (gemm_lnch.hip MODE 2): h1_c = r_c B with r_c LN_ch1's
//     combination of the rows zh_c = (f_c, o~_c, [c = 0], -mean_c) and B = [E diag(gamma); beta],
//     so h1_c Wm + bm = r_c V, V = B Wm (+ bm on the beta row; launch_l1_basis, f64 sums):
//     27 FMAs per row from the lane's column of V instead of a 256-deep GEMM;
//   tanh_ch, + h1, LN_ch2, h stored once.
// It replaces the o~ U GEMM, two layernorm_ch_quad passes and the Wm GEMM: the o~ rows are read
// (128 B per row) and h written (1 KB per row), nothing else goes through HBM.
#ifndef L1CH_WPE  // A/B knobs of layer1_ch_kernel: waves per SIMD targeted, rows of LDS reads in flight
#define L1CH_WPE 2
#endif
#ifndef L1CH_XDEP
#define L1CH_XDEP 2
#endif
#ifndef L1CH_YDEP
#define L1CH_YDEP 1
#endif
#ifndef L1CH_MFMA  // A/B knob: layer1_ch_kernel's r V product on the matrix cores (else VALU FMAs on broadcast reads)
#define L1CH_MFMA 1
#endif
#ifndef L1CH_ABL  // ablation builds (tools only, wrong results): bit 0 no x, 1 no LN_ch1, 2 no r rows / y, 3 no LN_ch2
#define L1CH_ABL 0
#endif
template <int N>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(L1CH_WPE))) void layer1_ch_kernel(const float* __restrict__ O, int KO,
                                                        const float* __restrict__ UT, const float* __restrict__ VT,
                                                        const float* __restrict__ W0f, const float* __restrict__ bol,
                                                        const float* __restrict__ ln1, const float* __restrict__ ln2,
                                                        const float* __restrict__ geo, float* __restrict__ h, int n_up) {
  constexpr int T = 2 * N, C = 2 * N + 5, D = 256, NR = C + T + 3, NO = 20, NB = 27;
  __shared__ float red[4][C + NR];
  __shared__ float al[3][T];       // flow coefficients (broadcast reads)
  __shared__ float mu[C], fin[NR], cf[T + 12];
  __shared__ float4 rr4[C * 7];    // LN_ch1's coefficient rows r_c (112-B rows, 27 used + 0 pad)
  float* const rr = reinterpret_cast<float*>(rr4);
  // one pool: the per-wave transpose scratch tb [4][16 * 65], the zh rows zt [C][28] (f_c, o~_c,
  // [c = 0], -mean_c, 0), the o~ rows os [C][20]; overlaid by ys [C][256] (the MFMA form's y,
  // between the r rows and LN_ch2, barriers on both sides)
  constexpr int TBF = 4 * 16 * 65, POOL = (C * D > TBF + C * 28 + C * NO) ? C * D : TBF + C * 28 + C * NO;
  __shared__ float4 pool4[POOL / 4];
  float* const pool = reinterpret_cast<float*>(pool4);
  float* const zt = pool + TBF;
  float* const os = zt + C * 28;
  const float4* const os4 = reinterpret_cast<const float4*>(os);
  const int e = blockIdx.x;    // walker*N + electron
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = e / N, i = e - b * N, col = 64 * w + lane;
  if (tid < N) {
    const int q = tid;
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + q));  // st ct sp cp
    al[0][2 * q] = -g.z;
    al[1][2 * q] = g.w;
    al[2][2 * q] = 0.f;
    al[0][2 * q + 1] = -(g.y * g.w);
    al[1][2 * q + 1] = -(g.y * g.z);
    al[2][2 * q + 1] = g.x;
  }
  for (int q = tid; q < C * NO; q += 256) {
    const int c = q / NO, k = q - (q / NO) * NO;
    os[q] = O[((size_t)e * C + c) * KO + 8 * (k / 5) + k % 5];
  }
  float w0[4], uc[NO];
#pragma unroll
  for (int k = 0; k < 4; ++k) w0[k] = W0f[k * D + col];
#pragma unroll
  for (int k = 0; k < NO; ++k) uc[k] = UT[(size_t)col * KO + 8 * (k / 5) + k % 5];
  const float bo = bol[col];
  const float4 g4 = *reinterpret_cast<const float4*>(geo + 4 * (size_t)e);  // st ct sp cp
  // input.hip's channel seed f_c of this electron
  auto feat = [&](int c) __attribute__((always_inline)) {
    const float st = g4.x, ct = g4.y, sp = g4.z, cp = g4.w;
    const float rx = st * cp, ry = st * sp, rz = ct;
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c == 0) {
      f = make_float4(rz, rx, ry, (i < n_up) ? 1.f : -1.f);
    } else if (c <= T) {
      const int t = c - 1;
      if ((t >> 1) == i) f = ((t & 1) == 0) ? make_float4(-st, ct * cp, ct * sp, 0.f) : make_float4(0.f, -sp, cp, 0.f);
    } else if (c == T + 1) {
      f = make_float4(-2.f * rz, -2.f * rx, -2.f * ry, 0.f);
    } else {
      const int k = c - T - 2;  // 0:x 1:y 2:z
      f = make_float4((k == 2) ? 0.f : -rz, (k == 0) ? 0.f : -rx, (k == 1) ? 0.f : -ry, 0.f);
    }
    return f;
  };
  __syncthreads();
#if L1CH_ABL & 1
  float z[C];
#pragma unroll
  for (int c = 0; c < C; ++c) z[c] = uc[c % NO] * (float)(c + 1);
#else
  // ---- x_c = (o~_c U + [c = 0] bol) + f_c W0 (the GEMM-then-residual order of the two-kernel form)
  // (each row's offset passes through an opaque asm that also takes the row two back: left free,
  // the scheduler issues every row's LDS reads ahead of the first use and spills)
  float z[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    int off = c * (NO / 4);
    if (c >= L1CH_XDEP)
      asm volatile("" : "+s"(off) : "v"(z[c - L1CH_XDEP]));
    else
      asm volatile("" : "+s"(off));
    float x = 0.f;
#pragma unroll
    for (int k4 = 0; k4 < NO / 4; ++k4) {  // broadcast ds_read_b128
      const float4 o4 = os4[off + k4];
      x = fmaf(o4.x, uc[4 * k4], x);
      x = fmaf(o4.y, uc[4 * k4 + 1], x);
      x = fmaf(o4.z, uc[4 * k4 + 2], x);
      x = fmaf(o4.w, uc[4 * k4 + 3], x);
    }
    if (c == 0) x += bo;
    const float4 f = feat(c);
    z[c] = x + (f.x * w0[0] + f.y * w0[1] + f.z * w0[2] + f.w * w0[3]);
  }
#endif
  float* tw = pool + w * 16 * 65;
  // sums over this wave's 64 columns of R per-lane values getv(r) -> dst[r] (layernorm_ch_quad's)
  auto rows_sum = [&](auto getv, auto R_, float* dst) {
    constexpr int R = decltype(R_)::value;
#pragma unroll
    for (int r0 = 0; r0 < R; r0 += 16) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (r0 + j < R) tw[j * 65 + lane] = getv(r0 + j);
      __builtin_amdgcn_wave_barrier();
      const int j = lane >> 2, q = lane & 3;
      float v = 0.f;
#pragma unroll
      for (int m = 0; m < 16; ++m) v += tw[j * 65 + 16 * q + m];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      if (q == 0 && r0 + j < R) dst[r0 + j] = v;
      __builtin_amdgcn_wave_barrier();
    }
  };
  // channel LayerNorm statistics of z (layernorm_ch_quad_kernel's): centres z, forms u, leaves the
  // means in mu, the per-electron coefficients in cf; returns s
  float u[3];
  auto ln_stats = [&]() __attribute__((always_inline)) {
    rows_sum([&](int c) { return z[c]; }, std::integral_constant<int, C>{}, red[w]);
    __syncthreads();
    if (tid < C) mu[tid] = ((red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid])) * (1.f / D);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < C; ++c) z[c] -= mu[c];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      u[k] = 0.f;
#pragma unroll
      for (int t = 0; t < T; ++t) u[k] = fmaf(al[k][t], z[1 + t], u[k]);
    }
    rows_sum(
        [&](int r) {
          if (r < C) return z[0] * z[r];
          if (r < C + T) return z[1 + r - C] * z[1 + r - C];
          return u[r - C - T] * u[r - C - T];
        },
        std::integral_constant<int, NR>{}, red[w] + C);
    __syncthreads();
    for (int r = tid; r < NR; r += 256)
      fin[r] = ((red[0][C + r] + red[1][C + r]) + (red[2][C + r] + red[3][C + r])) * (1.f / D);
    __syncthreads();
    const float s = 1.f / sqrtf(fin[0] + 1e-5f), s2 = s * s;
    if (w == 0) {
      float clv = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
      if (lane < T) {
        const float at = s2 * fin[1 + lane];
        cf[lane] = at;
        clv = 3.f * at * at - s2 * fin[C + lane];
        a0 = al[0][lane] * at;
        a1 = al[1][lane] * at;
        a2 = al[2][lane] * at;
      }
      clv = wave_sum(clv);
      a0 = wave_sum(a0);
      a1 = wave_sum(a1);
      a2 = wave_sum(a2);
      if (lane == 0) {
        cf[T] = clv;
        cf[T + 1] = s2 * fin[1 + T];  // aL
        const float au[3] = {a0, a1, a2};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          cf[T + 2 + k] = au[k];
          cf[T + 5 + k] = 3.f * au[k] * au[k] - s2 * fin[C + T + k];
          cf[T + 8 + k] = s2 * fin[2 + T + k];  // aS_k
        }
      }
    }
    __syncthreads();
    return s;
  };
  // ---- LN_ch1 -> h1 (in z)
#if L1CH_ABL & 2  // (ablation builds only: wrong results)
  float s = 1.f;
  u[0] = u[1] = u[2] = 0.f;
#else
  float s = ln_stats();
#endif
  {
    const float g = ln1[col], bb = ln1[D + col], gs = g * s, z0 = z[0];
    float sat = 0.f;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float at = cf[t];
      sat = fmaf(at, z[1 + t], sat);
      z[1 + t] = gs * (z[1 + t] - at * z0);
    }
    z[1 + T] = gs * (z[1 + T] - cf[T + 1] * z0 - 2.f * sat + cf[T] * z0);
#pragma unroll
    for (int k = 0; k < 3; ++k) z[2 + T + k] = gs * (z[2 + T + k] - cf[T + 8 + k] * z0 - 2.f * cf[T + 2 + k] * u[k] + cf[T + 5 + k] * z0);
    z[0] = g * (s * z0) + bb;
  }
#if L1CH_MFMA
  // V^T fragments of this wave's 4 feature tiles (the MFMA A operand, requested ahead of the r
  // rows): lane (i, kq) holds V[4 ks + kq][64 w + 16 ft + i]
  const int li = lane & 15, kq = lane >> 4;
  const float* vt = VT + (size_t)(64 * w + li) * 32 + kq;
  asm volatile("" : "+v"(vt));
  float va[4][7];
#pragma unroll
  for (int ft = 0; ft < 4; ++ft)
#pragma unroll
    for (int ks = 0; ks < 7; ++ks) va[ft][ks] = vt[ft * 16 * 32 + 4 * ks];
#else
  // V's column, requested here, ahead of the r rows (an opaque base: hoisted to the kernel start,
  // its 27 registers would be live through LN_ch1)
  const float* vt = VT + (size_t)col * 32;
  asm volatile("" : "+v"(vt));
  float v[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) v[j] = vt[j];
#endif
#if !(L1CH_ABL & 4)
  // ---- r rows: LN_ch1's combinations of the zh rows (zh staged in LDS first, one element per
  // task; then the tangent rows one element per task, the L / flow rows below)
#pragma unroll 1
  for (int q = tid; q < C * 28; q += 256) {
    const int c = q / 28, j = q - (q / 28) * 28;
    float v = 0.f;
    if (j < 4) {
      const float4 f = feat(c);
      v = j == 0 ? f.x : (j == 1 ? f.y : (j == 2 ? f.z : f.w));
    } else if (j < 24) {
      v = os[c * NO + j - 4];
    } else if (j == 24) {
      v = c == 0 ? 1.f : 0.f;
    } else if (j == 25) {
      v = -mu[c];
    }
    zt[q] = v;  // j = 26: the beta row (zh has 0 there), j = 27: padding
  }
  __syncthreads();
#pragma unroll 1
  for (int q = tid; q < T * 28; q += 256) {
    const int t = q / 28, j = q - (q / 28) * 28;
    rr[(1 + t) * 28 + j] = s * (zt[(1 + t) * 28 + j] - cf[t] * zt[j]);
  }
  // the L / flow rows: their sums over t split over the four waves (lanes j < 27 of wave w take
  // t = w T / 4 ..), the partials combined in a fixed order
  {
    __shared__ float part4[4][4][28];
    constexpr int TQ = T / 4;
    static_assert(T % 4 == 0, "t split over four waves");
    if (lane < NB) {
      const int j = lane;
      float sat = 0.f, u0 = 0.f, u1 = 0.f, u2 = 0.f;
#pragma unroll
      for (int tt = 0; tt < TQ; ++tt) {
        const int t = w * TQ + tt;
        const float zv = zt[(1 + t) * 28 + j];
        sat = fmaf(cf[t], zv, sat);
        u0 = fmaf(al[0][t], zv, u0);
        u1 = fmaf(al[1][t], zv, u1);
        u2 = fmaf(al[2][t], zv, u2);
      }
      part4[w][0][j] = sat;
      part4[w][1][j] = u0;
      part4[w][2][j] = u1;
      part4[w][3][j] = u2;
    }
    __syncthreads();
    if (tid == NB) {  // the pad column (k = 27 of the MFMA form) of the rows written below
      rr[NB] = 0.f;
      rr[(1 + T) * 28 + NB] = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) rr[(2 + T + k) * 28 + NB] = 0.f;
    }
    if (tid < NB) {
      const int j = tid;
      const float zh0 = zt[j];
      rr[j] = j == 26 ? 1.f : s * zh0;
      float a4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) a4[q] = (part4[0][q][j] + part4[1][q][j]) + (part4[2][q][j] + part4[3][q][j]);
      rr[(1 + T) * 28 + j] = s * (zt[(1 + T) * 28 + j] - cf[T + 1] * zh0 - 2.f * a4[0] + cf[T] * zh0);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        rr[(2 + T + k) * 28 + j] =
            s * (zt[(2 + T + k) * 28 + j] - cf[T + 8 + k] * zh0 - 2.f * cf[T + 2 + k] * a4[1 + k] + cf[T + 5 + k] * zh0);
    }
  }
  __syncthreads();
#endif
#if !(L1CH_ABL & 4)
  // ---- y = h1 Wm + bm = r V, tanh_ch, + h1 (layernorm_ch_quad mode 1's order)
#if L1CH_MFMA
  // y^T = V^T r^T on the matrix cores (v_mfma_f32_16x16x4_f32, exact f32): wave w takes features
  // 64 w .. 64 w + 63 (4 tiles of 16) x all channels (CT tiles of 16), K = 28 (r's 27 terms and
  // the zero pad); the result goes through LDS (ys [C][256]) into the lane-per-feature layout
  float* const ys = pool;
  {
    constexpr int CT = (C + 15) / 16;
    typedef float f4v __attribute__((ext_vector_type(4)));
    f4v acc[4][CT];
#pragma unroll
    for (int ft = 0; ft < 4; ++ft)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[ft][ct] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 7; ++ks) {
      float rb[CT];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int ch = 16 * ct + li;
        rb[ct] = ch < C ? rr[ch * 28 + 4 * ks + kq] : 0.f;
      }
#pragma unroll
      for (int ft = 0; ft < 4; ++ft)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[ft][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[ft][ks], rb[ct], acc[ft][ct], 0, 0, 0);
    }
#pragma unroll
    for (int ft = 0; ft < 4; ++ft)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int ch = 16 * ct + li;
        if (ch < C)
          *reinterpret_cast<float4*>(&ys[ch * D + 64 * w + 16 * ft + 4 * kq]) =
              make_float4(acc[ft][ct][0], acc[ft][ct][1], acc[ft][ct][2], acc[ft][ct][3]);
      }
  }
  __syncthreads();
  {
    auto yrow = [&](int c) __attribute__((always_inline)) { return ys[c * D + col]; };
#else
  {
    float prev = 0.f, prev2 = 0.f;  // the previous rows' results (order the rows' LDS reads, as above)
    auto yrow = [&](int c) __attribute__((always_inline)) {
      int off = c * 7;
      asm volatile("" : "+s"(off) : "v"(L1CH_YDEP == 1 ? prev : prev2));
      float a = 0.f;
#pragma unroll
      for (int j4 = 0; j4 < 7; ++j4) {  // broadcast ds_read_b128 (r[27] = 0 pads the last)
        const float4 r4 = rr4[off + j4];
        a = fmaf(r4.x, v[4 * j4], a);
        a = fmaf(r4.y, v[4 * j4 + 1], a);
        a = fmaf(r4.z, v[4 * j4 + 2], a);
        if (4 * j4 + 3 < NB) a = fmaf(r4.w, v[4 * j4 + 3], a);
      }
      prev2 = prev;
      prev = a;
      return a;
    };
#endif
    const float y0 = tanhf(yrow(0)), d1 = 1.f - y0 * y0, d2 = -2.f * y0 * d1;
    float sq = 0.f, u0 = 0.f, u1 = 0.f, u2 = 0.f;
    z[0] = z[0] + y0;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float yt = yrow(1 + t);
      sq = fmaf(yt, yt, sq);
      u0 = fmaf(al[0][t], yt, u0);
      u1 = fmaf(al[1][t], yt, u1);
      u2 = fmaf(al[2][t], yt, u2);
      z[1 + t] = fmaf(d1, yt, z[1 + t]);
    }
    z[1 + T] = z[1 + T] + d1 * yrow(1 + T) + d2 * sq;
    const float uu[3] = {u0, u1, u2};
#pragma unroll
    for (int k = 0; k < 3; ++k) z[2 + T + k] = z[2 + T + k] + d1 * yrow(2 + T + k) + d2 * uu[k] * uu[k];
  }
#if L1CH_MFMA
  __syncthreads();  // every ys read done: LN_ch2's transposes reuse the pool
#endif
#endif
  // ---- LN_ch2 -> h
#if !(L1CH_ABL & 8)
  s = ln_stats();
#endif
  const size_t r0 = (size_t)e * C * D + col;
  const float g = ln2[col], bb = ln2[D + col], gs = g * s, z0 = z[0];
  float sat = 0.f;
  h[r0] = g * (s * z0) + bb;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const float at = cf[t];
    sat = fmaf(at, z[1 + t], sat);
    h[r0 + (size_t)(1 + t) * D] = gs * (z[1 + t] - at * z0);
  }
  h[r0 + (size_t)(1 + T) * D] = gs * (z[1 + T] - cf[T + 1] * z0 - 2.f * sat + cf[T] * z0);
#pragma unroll
  for (int k = 0; k < 3; ++k)
    h[r0 + (size_t)(2 + T + k) * D] =
        gs * (z[2 + T + k] - cf[T + 8 + k] * z0 - 2.f * cf[T + 2 + k] * u[k] + cf[T + 5 + k] * z0);
}

template <int N>
void launch_ln_wave(const float* X, const float* Z, const float* ln, const float* geo, float* h, int ne, int mode,
                    hipStream_t s) {
  hipLaunchKernelGGL(layernorm_ch_wave_kernel<N>, dim3((ne + 3) / 4), dim3(256), 0, s, X, Z, ln, geo, h, ne, mode);
}

}  // namespace

bool layer1_ch_supported(const Dims& d) { return d.D == 256 && d.H == 4 && ofeat_k(d) == 32 && (d.N == 10 || d.N == 20); }

void launch_layer1_ch(const Dims& d, const float* O, const float* UT, const float* VT, const float* W0f,
                      const float* bol, const float* ln1, const float* ln2, const float* geo, float* h, int nw,
                      hipStream_t s) {
  const int ne = nw * d.N, KO = ofeat_k(d);
  if (d.N == 10)
    hipLaunchKernelGGL(layer1_ch_kernel<10>, dim3(ne), dim3(256), 0, s, O, KO, UT, VT, W0f, bol, ln1, ln2, geo, h,
                       d.n_up);
  else  // layer1_ch_supported: N = 10 or 20
    hipLaunchKernelGGL(layer1_ch_kernel<20>, dim3(ne), dim3(256), 0, s, O, KO, UT, VT, W0f, bol, ln1, ln2, geo, h,
                       d.n_up);
}

void launch_layernorm(const Dims& d, const float* X, const float* Z, const float* ln, const float* geo, float* h,
                      int nw, int C, int mode, hipStream_t s, const float* W0f) {
  if (W0f && !(C > 1 && d.D == 256 && (d.N == 10 || d.N == 20) && mode == 0)) W0f = nullptr;  // quad kernel only
  if (C > 1 && d.D == 256 && (d.N <= 8 || d.N == 10 || d.N == 20)) {
    const int ne = nw * d.N;
    switch (d.N) {
      case 10:
        hipLaunchKernelGGL(layernorm_ch_quad_kernel<10>, dim3(ne), dim3(256), 0, s, X, Z, ln, geo, h, ne, mode, W0f,
                           d.n_up);
        return;
      case 20:
        hipLaunchKernelGGL(layernorm_ch_quad_kernel<20>, dim3(ne), dim3(256), 0, s, X, Z, ln, geo, h, ne, mode, W0f,
                           d.n_up);
        return;
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
