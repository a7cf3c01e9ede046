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

template <int N>
void launch_ln_wave(const float* X, const float* Z, const float* ln, const float* geo, float* h, int ne, int mode,
                    hipStream_t s) {
  hipLaunchKernelGGL(layernorm_ch_wave_kernel<N>, dim3((ne + 3) / 4), dim3(256), 0, s, X, Z, ln, geo, h, ne, mode);
}

}  // namespace

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
