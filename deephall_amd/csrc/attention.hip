// Channel self-attention (flax MultiHeadAttention inside psiformer.py:44), one
// workgroup per (walker, head).  Forward-mode rules:
//
//   scores   S0 = s q0 k0^T,  S_t = s (q_t k0^T + q0 k_t^T)          (s = 1/sqrt(dh))
//            S_L = s (q_L k0^T + q0 k_L^T + 2 sum_t q_t k_t^T)
//            S_Sk = s (q_Sk k0^T + q0 k_Sk^T + 2 qu_k ku_k^T),  qu_k = sum_t alpha_kt q_t
//   softmax  A0 = softmax(S0);  Sbar_t = S_t - <S_t>_A0 (row-wise);  A_t = A0 * Sbar_t
//            A_L  = A0 * [(S_L - <S_L>) + (T2 - <T2>)],      T2 = sum_t Sbar_t^2
//            A_Sk = A0 * [(S_Sk - <S_Sk>) + (U2 - <U2>)],    U2 = (sum_t alpha_kt Sbar_t)^2
//   output   o0 = A0 v0,  o_t = A_t v0 + A0 v_t,  o_L = A_L v0 + A0 v_L + 2 sum_t A_t v_t
//            o_Sk = A_Sk v0 + A0 v_Sk + 2 (sum_t alpha_kt A_t)(sum_t alpha_kt v_t)
//
// qkv rows are (walker, electron, channel); columns [q | k | v], head h at h*dh.
#include <type_traits>

#include "dh_internal.h"
#include "device_common.h"
#include "attn_val.h"

namespace dh {
namespace {

struct AttnSmem {
  // offsets (floats) into dynamic shared memory
  int alpha, q0, k0, v0, qc, kc, vc, A0, S, P, accS, T2, SuB, Au, accOL, qu, ku, vu, total;
};

__host__ __device__ inline AttnSmem attn_layout(int N, int dh, int T, int C) {
  AttnSmem L;
  const int ld = dh + 1;
  const int nd = N * ld, nn = N * N;
  int o = 0;
  L.alpha = o;
  o += 3 * T + 4;
  L.q0 = o;
  o += nd;
  L.k0 = o;
  o += nd;
  L.v0 = o;
  o += nd;
  L.A0 = o;
  o += nn;
  if (C > 1) {
    L.qc = o;
    o += nd;
    L.kc = o;
    o += nd;
    L.vc = o;
    o += nd;
    L.S = o;
    o += nn;
    L.P = o;
    o += nn;
    L.accS = o;
    o += nn;
    L.T2 = o;
    o += nn;
    L.SuB = o;
    o += 3 * nn;
    L.Au = o;
    o += 3 * nn;
    L.accOL = o;
    o += nd;
    L.qu = o;
    o += 3 * nd;
    L.ku = o;
    o += 3 * nd;
    L.vu = o;
    o += 3 * nd;
  } else {
    L.qc = L.kc = L.vc = L.S = L.P = L.accS = L.T2 = L.SuB = L.Au = L.accOL = L.qu = L.ku = L.vu = 0;
  }
  L.total = o;
  return L;
}

// load one channel's q/k/v of head h for all electrons into LDS (row stride dh+1)
__device__ inline void load_qkv(const float* __restrict__ qkv, int b, int c, int h, int N, int C, int D, int dh,
                                float* q, float* k, float* v) {
  const int ld = dh + 1;
  const int tot = N * dh;
  for (int idx = threadIdx.x; idx < tot; idx += blockDim.x) {
    const int i = idx / dh, d = idx % dh;
    const float* row = qkv + ((size_t)(b * N + i) * C + c) * (3 * D) + h * dh + d;
    q[i * ld + d] = row[0];
    k[i * ld + d] = row[D];
    v[i * ld + d] = row[2 * D];
  }
}

__device__ inline void store_o(float* __restrict__ o, int b, int c, int h, int N, int C, int D, int dh, int i, int d,
                               float val) {
  o[((size_t)(b * N + i) * C + c) * D + h * dh + d] = val;
}

// S[i][j] = s * (qa_i . kb_j + qb_i . ka_j) [+ 2 s qx_i . kx_j] ; optional P = qa . ka
__global__ void attention_kernel(const float* __restrict__ qkv, const float* __restrict__ geo, float* __restrict__ o,
                                 int N, int C, int H, int dh) {
  extern __shared__ float sm[];
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int D = H * dh, T = 2 * N, ld = dh + 1, nn = N * N;
  const AttnSmem L = attn_layout(N, dh, T, C);
  const float scale = 1.0f / sqrtf((float)dh);
  const int tid = threadIdx.x, nt = blockDim.x;
  float *q0 = sm + L.q0, *k0 = sm + L.k0, *v0 = sm + L.v0, *A0 = sm + L.A0;

  load_qkv(qkv, b, 0, h, N, C, D, dh, q0, k0, v0);
  if (C > 1) {
    float* al = sm + L.alpha;
    for (int t = tid; t < T; t += nt) {
      const int i = t >> 1;
      const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));  // st ct sp cp
      for (int k = 0; k < 3; ++k) {
        float a;
        if ((t & 1) == 0) {  // phi_hat_k
          a = (k == 0) ? -g.z : (k == 1 ? g.w : 0.f);
        } else {  // -theta_hat_k
          a = (k == 0) ? -(g.y * g.w) : (k == 1 ? -(g.y * g.z) : g.x);
        }
        al[k * T + t] = a;
      }
    }
  }
  __syncthreads();
  // value scores + softmax
  for (int p = tid; p < nn; p += nt) {
    const int i = p / N, j = p % N;
    float acc = 0.f;
    for (int d = 0; d < dh; ++d) acc = fmaf(q0[i * ld + d], k0[j * ld + d], acc);
    A0[p] = acc * scale;
  }
  __syncthreads();
  for (int i = tid; i < N; i += nt) {
    float m = -INFINITY;
    for (int j = 0; j < N; ++j) m = fmaxf(m, A0[i * N + j]);
    float ssum = 0.f;
    for (int j = 0; j < N; ++j) {
      const float e = expf(A0[i * N + j] - m);
      A0[i * N + j] = e;
      ssum += e;
    }
    const float inv = 1.f / ssum;
    for (int j = 0; j < N; ++j) A0[i * N + j] *= inv;
  }
  __syncthreads();
  for (int p = tid; p < N * dh; p += nt) {
    const int i = p / dh, d = p % dh;
    float acc = 0.f;
    for (int j = 0; j < N; ++j) acc = fmaf(A0[i * N + j], v0[j * ld + d], acc);
    store_o(o, b, 0, h, N, C, D, dh, i, d, acc);
  }
  if (C == 1) return;

  const float* al = sm + L.alpha;
  float *qc = sm + L.qc, *kc = sm + L.kc, *vc = sm + L.vc, *S = sm + L.S, *P = sm + L.P;
  float *accS = sm + L.accS, *T2 = sm + L.T2, *SuB = sm + L.SuB, *Au = sm + L.Au;
  float *accOL = sm + L.accOL, *qu = sm + L.qu, *ku = sm + L.ku, *vu = sm + L.vu;
  for (int p = tid; p < nn; p += nt) {
    accS[p] = 0.f;
    T2[p] = 0.f;
    for (int k = 0; k < 3; ++k) {
      SuB[k * nn + p] = 0.f;
      Au[k * nn + p] = 0.f;
    }
  }
  for (int p = tid; p < N * ld; p += nt) {
    accOL[p] = 0.f;
    for (int k = 0; k < 3; ++k) {
      qu[k * N * ld + p] = 0.f;
      ku[k * N * ld + p] = 0.f;
      vu[k * N * ld + p] = 0.f;
    }
  }
  __syncthreads();

  // ---------------- tangent channels
  for (int t = 0; t < T; ++t) {
    load_qkv(qkv, b, 1 + t, h, N, C, D, dh, qc, kc, vc);
    __syncthreads();
    for (int p = tid; p < nn; p += nt) {
      const int i = p / N, j = p % N;
      float s1 = 0.f, s2 = 0.f;
      for (int d = 0; d < dh; ++d) {
        s1 = fmaf(qc[i * ld + d], k0[j * ld + d], s1);
        s1 = fmaf(q0[i * ld + d], kc[j * ld + d], s1);
        s2 = fmaf(qc[i * ld + d], kc[j * ld + d], s2);
      }
      S[p] = s1 * scale;
      P[p] = s2;
    }
    __syncthreads();
    for (int p = tid; p < nn; p += nt) {
      const int i = p / N;
      float m = 0.f;
      for (int j = 0; j < N; ++j) m = fmaf(A0[i * N + j], S[i * N + j], m);
      const float sb = S[p] - m;
      const float at = A0[p] * sb;
      accS[p] = fmaf(2.f * scale, P[p], accS[p]);
      T2[p] = fmaf(sb, sb, T2[p]);
      for (int k = 0; k < 3; ++k) {
        const float a = al[k * T + t];
        SuB[k * nn + p] = fmaf(a, sb, SuB[k * nn + p]);
        Au[k * nn + p] = fmaf(a, at, Au[k * nn + p]);
      }
      P[p] = at;  // A_t (S still needed by other threads this phase)
    }
    __syncthreads();
    for (int p = tid; p < N * dh; p += nt) {
      const int i = p / dh, d = p % dh;
      float acc = 0.f, acc2 = 0.f;
      for (int j = 0; j < N; ++j) {
        acc = fmaf(P[i * N + j], v0[j * ld + d], acc);
        acc = fmaf(A0[i * N + j], vc[j * ld + d], acc);
        acc2 = fmaf(P[i * N + j], vc[j * ld + d], acc2);
      }
      store_o(o, b, 1 + t, h, N, C, D, dh, i, d, acc);
      const int q = i * ld + d;
      accOL[q] = fmaf(2.f, acc2, accOL[q]);
      for (int k = 0; k < 3; ++k) {
        const float a = al[k * T + t];
        qu[k * N * ld + q] = fmaf(a, qc[q], qu[k * N * ld + q]);
        ku[k * N * ld + q] = fmaf(a, kc[q], ku[k * N * ld + q]);
        vu[k * N * ld + q] = fmaf(a, vc[q], vu[k * N * ld + q]);
      }
    }
    __syncthreads();
  }

  // ---------------- Laplace-Beltrami channel and the three flow channels
  for (int c2 = 0; c2 < 4; ++c2) {
    const int c = 1 + T + c2;
    load_qkv(qkv, b, c, h, N, C, D, dh, qc, kc, vc);
    __syncthreads();
    const int k = c2 - 1;
    for (int p = tid; p < nn; p += nt) {
      const int i = p / N, j = p % N;
      float s1 = 0.f, s2 = 0.f;
      for (int d = 0; d < dh; ++d) {
        s1 = fmaf(qc[i * ld + d], k0[j * ld + d], s1);
        s1 = fmaf(q0[i * ld + d], kc[j * ld + d], s1);
      }
      if (k >= 0) {
        const float* qk = qu + k * N * ld;
        const float* kk = ku + k * N * ld;
        for (int d = 0; d < dh; ++d) s2 = fmaf(qk[i * ld + d], kk[j * ld + d], s2);
        S[p] = scale * (s1 + 2.f * s2);
        const float u = SuB[k * nn + p];
        P[p] = u * u;
      } else {
        S[p] = scale * s1 + accS[p];
        P[p] = T2[p];
      }
    }
    __syncthreads();
    // A2 = A0 * [(S - <S>) + (P - <P>)]  -> stored into S after all reads (use registers)
    float vals[4];
    int cnt = 0;
    for (int p = tid; p < nn; p += nt, ++cnt) {
      const int i = p / N;
      float m1 = 0.f, m2 = 0.f;
      for (int j = 0; j < N; ++j) {
        m1 = fmaf(A0[i * N + j], S[i * N + j], m1);
        m2 = fmaf(A0[i * N + j], P[i * N + j], m2);
      }
      const float v = A0[p] * ((S[p] - m1) + (P[p] - m2));
      if (cnt < 4) vals[cnt] = v;
    }
    __syncthreads();
    cnt = 0;
    for (int p = tid; p < nn; p += nt, ++cnt)
      if (cnt < 4) S[p] = vals[cnt];
    __syncthreads();
    for (int p = tid; p < N * dh; p += nt) {
      const int i = p / dh, d = p % dh;
      float acc = 0.f;
      for (int j = 0; j < N; ++j) {
        acc = fmaf(S[i * N + j], v0[j * ld + d], acc);
        acc = fmaf(A0[i * N + j], vc[j * ld + d], acc);
      }
      if (k >= 0) {
        const float* Auk = Au + k * nn;
        const float* vuk = vu + k * N * ld;
        float a2 = 0.f;
        for (int j = 0; j < N; ++j) a2 = fmaf(Auk[i * N + j], vuk[j * ld + d], a2);
        acc = fmaf(2.f, a2, acc);
      } else {
        acc += accOL[i * ld + d];
      }
      store_o(o, b, c, h, N, C, D, dh, i, d, acc);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Channel kernel v2: one 256-thread workgroup per (walker, head); channel c+1's q/k/v are
// prefetched into registers (PF float4 per thread) while channel c is computed, then
// committed to the other half of a double-buffered LDS image: 3 barriers per channel,
// 4 lanes per score pair.
struct AttnSmem2 {
  int alpha, q0, k0, v0, qc, kc, vc, A0, S, P, R, accS, T2, SuB, Au, accOL, qu, ku, vu, total;
};
__host__ __device__ inline AttnSmem2 attn_layout2(int N, int dh) {
  AttnSmem2 L;
  const int ld = dh + 1, nd = N * ld, nn = N * N, T = 2 * N;
  int o = 0;
  L.alpha = o;
  o += 3 * T + 4;
  L.q0 = o;
  o += nd;
  L.k0 = o;
  o += nd;
  L.v0 = o;
  o += nd;
  L.qc = o;
  o += 2 * nd;
  L.kc = o;
  o += 2 * nd;
  L.vc = o;
  o += 2 * nd;
  L.A0 = o;
  o += nn;
  L.S = o;
  o += nn;
  L.P = o;
  o += nn;
  L.R = o;
  o += nn;
  L.accS = o;
  o += nn;
  L.T2 = o;
  o += nn;
  L.SuB = o;
  o += 3 * nn;
  L.Au = o;
  o += 3 * nn;
  L.accOL = o;
  o += nd;
  L.qu = o;
  o += 3 * nd;
  L.ku = o;
  o += 3 * nd;
  L.vu = o;
  o += 3 * nd;
  L.total = o;
  return L;
}

template <int PF, int RPT>
__global__ __launch_bounds__(256) void attention_ch_kernel(const float* __restrict__ qkv,
                                                           const float* __restrict__ geo, float* __restrict__ o,
                                                           int N, int H, int dh) {
  extern __shared__ float sm[];
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int C = 2 * N + 5, T = 2 * N, D = H * dh, ld = dh + 1, nd = N * ld, nn = N * N;
  const AttnSmem2 L = attn_layout2(N, dh);
  const float scale = 1.0f / sqrtf((float)dh);
  const int tid = threadIdx.x, nt = blockDim.x;
  float *al = sm + L.alpha, *q0 = sm + L.q0, *k0 = sm + L.k0, *v0 = sm + L.v0;
  float *A0 = sm + L.A0, *S = sm + L.S, *P = sm + L.P, *Rm = sm + L.R;
  float *accS = sm + L.accS, *T2 = sm + L.T2, *SuB = sm + L.SuB, *Au = sm + L.Au;
  float *accOL = sm + L.accOL, *qu = sm + L.qu, *ku = sm + L.ku, *vu = sm + L.vu;
  const int dq = dh >> 2, nf4 = N * dq, tot4 = 3 * nf4;

  float4 pf[PF];
  auto prefetch = [&](int c) {
#pragma unroll
    for (int s = 0; s < PF; ++s) {
      const int f = tid + s * 256;
      if (f < tot4) {
        const int mat = f / nf4, g = f - mat * nf4, i = g / dq, d4 = g - i * dq;
        pf[s] = *reinterpret_cast<const float4*>(qkv + ((size_t)(b * N + i) * C + c) * (3 * D) + mat * D + h * dh +
                                                 4 * d4);
      }
    }
  };
  auto commit = [&](float* qd, float* kd, float* vd) {
#pragma unroll
    for (int s = 0; s < PF; ++s) {
      const int f = tid + s * 256;
      if (f < tot4) {
        const int mat = f / nf4, g = f - mat * nf4, i = g / dq, d4 = g - i * dq;
        float* dst = (mat == 0 ? qd : (mat == 1 ? kd : vd)) + i * ld + 4 * d4;
        dst[0] = pf[s].x;
        dst[1] = pf[s].y;
        dst[2] = pf[s].z;
        dst[3] = pf[s].w;
      }
    }
  };
  auto store_o = [&](int c, int i, int d, float val) { o[((size_t)(b * N + i) * C + c) * D + h * dh + d] = val; };
  // 4 lanes per (i, j) pair: partial dot products over quarters of dh, reduced by shuffles
  auto dots = [&](const float* qa, const float* kb, const float* qb, const float* ka, const float* qx,
                  const float* kx, int p, float& s1, float& s2) {
    const int pair = p >> 2, qt = p & 3;
    const int i = pair / N, j = pair - (pair / N) * N;
    const int d0 = qt * dq;
    s1 = 0.f;
    s2 = 0.f;
    for (int d = d0; d < d0 + dq; ++d) {
      s1 = fmaf(qa[i * ld + d], kb[j * ld + d], s1);
      if (qb) s1 = fmaf(qb[i * ld + d], ka[j * ld + d], s1);
      if (qx) s2 = fmaf(qx[i * ld + d], kx[j * ld + d], s2);
    }
    s1 += __shfl_xor(s1, 1, 64);
    s1 += __shfl_xor(s1, 2, 64);
    s2 += __shfl_xor(s2, 1, 64);
    s2 += __shfl_xor(s2, 2, 64);
  };

  for (int t = tid; t < T; t += nt) {
    const int i = t >> 1;
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));  // st ct sp cp
    for (int k = 0; k < 3; ++k) {
      float a;
      if ((t & 1) == 0)
        a = (k == 0) ? -g.z : (k == 1 ? g.w : 0.f);
      else
        a = (k == 0) ? -(g.y * g.w) : (k == 1 ? -(g.y * g.z) : g.x);
      al[k * T + t] = a;
    }
  }
  prefetch(0);
  commit(q0, k0, v0);
  prefetch(1);
  for (int p = tid; p < nn; p += nt) {
    accS[p] = 0.f;
    T2[p] = 0.f;
    for (int k = 0; k < 3; ++k) {
      SuB[k * nn + p] = 0.f;
      Au[k * nn + p] = 0.f;
    }
  }
  const int d_own = tid & 63, g_own = tid >> 6;
  float rOL[RPT], rQu[3][RPT], rKu[3][RPT], rVu[3][RPT];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    rOL[r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) rQu[kk][r] = rKu[kk][r] = rVu[kk][r] = 0.f;
  }
  __syncthreads();
  // ---- value channel
  for (int p = tid; p < 4 * nn; p += nt) {
    float s1, s2;
    dots(q0, k0, nullptr, nullptr, nullptr, nullptr, p, s1, s2);
    if ((p & 3) == 0) A0[p >> 2] = s1 * scale;
  }
  __syncthreads();
  for (int i = tid; i < N; i += nt) {
    float m = -INFINITY;
    for (int j = 0; j < N; ++j) m = fmaxf(m, A0[i * N + j]);
    float ssum = 0.f;
    for (int j = 0; j < N; ++j) {
      const float e = expf(A0[i * N + j] - m);
      A0[i * N + j] = e;
      ssum += e;
    }
    const float inv = 1.f / ssum;
    for (int j = 0; j < N; ++j) A0[i * N + j] *= inv;
  }
  commit(sm + L.qc + nd, sm + L.kc + nd, sm + L.vc + nd);  // channel 1 -> buffer 1
  __syncthreads();
  for (int p = tid; p < N * dh; p += nt) {
    const int i = p / dh, d = p - i * dh;
    float acc = 0.f;
    for (int j = 0; j < N; ++j) acc = fmaf(A0[i * N + j], v0[j * ld + d], acc);
    store_o(0, i, d, acc);
  }

  // ---- channels 1 .. C-1
  for (int c = 1; c < C; ++c) {
    const int buf = c & 1;
    const float* qc = sm + L.qc + buf * nd;
    const float* kc = sm + L.kc + buf * nd;
    const float* vc = sm + L.vc + buf * nd;
    if (c + 1 < C) prefetch(c + 1);
    const bool tang = c <= T;
    const int k = c - T - 2;  // flow index (>= 0 for flow channels)
    // phase A: scores
    for (int p = tid; p < 4 * nn; p += nt) {
      float s1, s2;
      if (tang) {
        dots(qc, k0, q0, kc, qc, kc, p, s1, s2);
      } else if (k < 0) {
        dots(qc, k0, q0, kc, nullptr, nullptr, p, s1, s2);
      } else {
        dots(qc, k0, q0, kc, qu + k * nd, ku + k * nd, p, s1, s2);
      }
      if ((p & 3) == 0) {
        const int pair = p >> 2;
        if (tang) {
          S[pair] = s1 * scale;
          P[pair] = s2;
        } else if (k < 0) {
          S[pair] = s1 * scale + accS[pair];
          P[pair] = T2[pair];
        } else {
          S[pair] = scale * (s1 + 2.f * s2);
          const float u = SuB[k * nn + pair];
          P[pair] = u * u;
        }
      }
    }
    __syncthreads();
    // phase B: softmax derivatives
    for (int p = tid; p < nn; p += nt) {
      const int i = p / N;
      if (tang) {
        const int t = c - 1;
        float m = 0.f;
        for (int j = 0; j < N; ++j) m = fmaf(A0[i * N + j], S[i * N + j], m);
        const float sb = S[p] - m;
        const float at = A0[p] * sb;
        accS[p] = fmaf(2.f * scale, P[p], accS[p]);
        T2[p] = fmaf(sb, sb, T2[p]);
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) {
          const float a = al[kk * T + t];
          SuB[kk * nn + p] = fmaf(a, sb, SuB[kk * nn + p]);
          Au[kk * nn + p] = fmaf(a, at, Au[kk * nn + p]);
        }
        Rm[p] = at;
      } else {
        float m1 = 0.f, m2 = 0.f;
        for (int j = 0; j < N; ++j) {
          m1 = fmaf(A0[i * N + j], S[i * N + j], m1);
          m2 = fmaf(A0[i * N + j], P[i * N + j], m2);
        }
        Rm[p] = A0[p] * ((S[p] - m1) + (P[p] - m2));
      }
    }
    __syncthreads();
    // phase C: outputs.  Thread (d = lane, g = wave) owns rows i = g + 4r (r < RPT): the
    // v loads are shared by its rows and the running sums of the flow first-order parts
    // (qu, ku, vu) and of 2 sum_t A_t v_t stay in registers through the tangent loop.
    if (d_own < dh) {
      float acc[RPT], acc2[RPT];
#pragma unroll
      for (int r = 0; r < RPT; ++r) acc[r] = acc2[r] = 0.f;
      for (int j = 0; j < N; ++j) {
        const float v0j = v0[j * ld + d_own], vcj = vc[j * ld + d_own];
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
          const int i = g_own + 4 * r;
          if (i < N) {
            const float at = Rm[i * N + j];
            acc[r] = fmaf(at, v0j, fmaf(A0[i * N + j], vcj, acc[r]));
            acc2[r] = fmaf(at, vcj, acc2[r]);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const int i = g_own + 4 * r;
        if (i >= N) continue;
        const int q = i * ld + d_own;
        float out = acc[r];
        if (tang) {
          const int t = c - 1;
          rOL[r] = fmaf(2.f, acc2[r], rOL[r]);
          const float qv = qc[q], kv = kc[q], vv = vc[q];
#pragma unroll
          for (int kk = 0; kk < 3; ++kk) {
            const float a = al[kk * T + t];
            rQu[kk][r] = fmaf(a, qv, rQu[kk][r]);
            rKu[kk][r] = fmaf(a, kv, rKu[kk][r]);
            rVu[kk][r] = fmaf(a, vv, rVu[kk][r]);
          }
          if (c == T) {  // last tangent: publish the accumulated first-order parts
            accOL[q] = rOL[r];
#pragma unroll
            for (int kk = 0; kk < 3; ++kk) {
              qu[kk * nd + q] = rQu[kk][r];
              ku[kk * nd + q] = rKu[kk][r];
              vu[kk * nd + q] = rVu[kk][r];
            }
          }
        } else if (k < 0) {
          out += rOL[r];
        } else {
          float a2 = 0.f;
          for (int j = 0; j < N; ++j) a2 = fmaf(Au[k * nn + i * N + j], vu[k * nd + j * ld + d_own], a2);
          out = fmaf(2.f, a2, out);
        }
        store_o(c, i, d_own, out);
      }
    }
    if (c + 1 < C) {
      const int nb = (c + 1) & 1;
      commit(sm + L.qc + nb * nd, sm + L.kc + nb * nd, sm + L.vc + nb * nd);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Channel kernel v3 (N <= 8, dh = 64): ONE WAVE per (walker, head), no block barriers.
// Lane = feature column d for loads / outputs (the running first-order flow sums live in
// registers), lane = (score pair, quarter of d) for the scores (16-byte LDS reads).
// LDS is private to the wave; LDS ops of one wave execute in order, so a
// __builtin_amdgcn_wave_barrier() (compiler ordering) separates the phases.
//
// FEAT (layer 1 only): q|k|v are not read from memory but formed in registers from the
// input-feature channels of every electron (see input.hip for the channel seeds) times
// the folded W0 Wqkv (+ bias on the value channel) — the K=4 input map fused into the
// attention, so the 3D-wide q|k|v rows of all channels never touch HBM.

// Input-feature channel c of electron i from its geometry g = (st, ct, sp, cp):
// [z, x, y, spin] order of psiformer.py:51-60, derivative seeds as in input.hip.
template <int T>
__device__ __forceinline__ float4 feature_channel(int c, int i, float4 g, float spin) {
  const float st = g.x, ct = g.y, sp = g.z, cp = g.w;
  if (c == 0) return make_float4(ct, st * cp, st * sp, spin);
  if (c <= T) {
    const int t = c - 1;
    if ((t >> 1) != i) return make_float4(0.f, 0.f, 0.f, 0.f);
    return ((t & 1) == 0) ? make_float4(-st, ct * cp, ct * sp, 0.f) : make_float4(0.f, -sp, cp, 0.f);
  }
  const float rz = ct, rx = st * cp, ry = st * sp;
  if (c == T + 1) return make_float4(-2.f * rz, -2.f * rx, -2.f * ry, 0.f);
  const int k = c - T - 2;  // rotation flow about axis k (0:x 1:y 2:z)
  return make_float4((k == 2) ? 0.f : -rz, (k == 0) ? 0.f : -rx, (k == 1) ? 0.f : -ry, 0.f);
}

template <int N, bool FEAT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(N <= 8 ? 3 : (N <= 12 ? 2 : 1)))) void attention_wave_kernel(const float* __restrict__ qkv,
                                                            const float* __restrict__ geo, float* __restrict__ o,
                                                            int H, const float* __restrict__ W0qkv,
                                                            const float* __restrict__ bqkv, int n_up) {
  constexpr int dh = 64, ld = 68, T = 2 * N, C = 2 * N + 5, nn = N * N;
  extern __shared__ float sm[];
  // VR (N > 8): v of the value channel and of the current channel live in registers
  // (lane = column), which frees 2 N x 68 floats of LDS per wave (C5: 61 vs 88 ms per
  // step); for N <= 8 the LDS copy keeps the register count down (C2: 1.0 vs 1.27 ms)
  constexpr bool VR = N > 8;
  constexpr int NV = VR ? 0 : N * ld;
  float *q0 = sm, *k0 = q0 + N * ld, *v0 = k0 + N * ld, *qc = v0 + NV, *kc = qc + N * ld, *vc = kc + N * ld;
  float *A0 = vc + NV, *S = A0 + nn, *P = S + nn, *Rm = P + nn, *accS = Rm + nn, *T2 = accS + nn;
  float *SuB = T2 + nn, *Au = SuB + 3 * nn, *QK = Au + 3 * nn, *al = QK + 3 * nn;
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H, lane = threadIdx.x;
  const int D = H * dh;
  const float scale = 0.125f;  // 1 / sqrt(64)
  const float* base = qkv + (size_t)b * N * C * (3 * D) + h * dh + lane;
  // channel c's q|k|v rows: prefetched from memory into registers one channel ahead, or
  // (FEAT) formed from the features only when committed to LDS
  constexpr int NP = FEAT ? 1 : N;
  float pq[NP], pk[NP], pv[NP];
  FeatW fw;
  if constexpr (FEAT) fw.load(W0qkv, bqkv, D, h * dh + lane);
  int pending = 0;  // channel held by the prefetch registers / to be formed (FEAT)
  auto prefetch = [&](int c) {
    pending = c;
    if constexpr (!FEAT) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const float* r = base + (size_t)(i * C + c) * (3 * D);
        pq[i] = r[0];
        pk[i] = r[D];
        pv[i] = r[2 * D];
      }
    }
  };
  float v0reg[VR ? N : 1], vcreg[VR ? N : 1];
  auto commit = [&](float* qd, float* kd, float* vl, float* vr) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if constexpr (FEAT) {
        const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));
        const float4 f = feature_channel<T>(pending, i, g, (i < n_up) ? 1.f : -1.f);
        const bool v = pending == 0;
        qd[i * ld + lane] = FeatW::dot(f, fw.wq) + (v ? fw.bq : 0.f);
        kd[i * ld + lane] = FeatW::dot(f, fw.wk) + (v ? fw.bk : 0.f);
        const float vv = FeatW::dot(f, fw.wv) + (v ? fw.bv : 0.f);
        if constexpr (VR)
          vr[i] = vv;
        else
          vl[i * ld + lane] = vv;
      } else {
        qd[i * ld + lane] = pq[i];
        kd[i * ld + lane] = pk[i];
        if constexpr (VR)
          vr[i] = pv[i];
        else
          vl[i * ld + lane] = pv[i];
      }
    }
  };
  float* obase = o + (size_t)b * N * C * D + h * dh + lane;
  auto wsync = [] { __builtin_amdgcn_wave_barrier(); };
  // 4 lanes per pair; dots over 16 columns with float4 LDS reads
  auto dot16 = [&](const float* x, const float* y) {
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float4 a = *reinterpret_cast<const float4*>(x + 4 * m);
      const float4 c = *reinterpret_cast<const float4*>(y + 4 * m);
      s = fmaf(a.x, c.x, fmaf(a.y, c.y, fmaf(a.z, c.z, fmaf(a.w, c.w, s))));
    }
    return s;
  };

  if (lane < T) {
    const int i = lane >> 1;
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));  // st ct sp cp
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float a;
      if ((lane & 1) == 0)
        a = (k == 0) ? -g.z : (k == 1 ? g.w : 0.f);
      else
        a = (k == 0) ? -(g.y * g.w) : (k == 1 ? -(g.y * g.z) : g.x);
      al[k * T + lane] = a;
    }
  }
  prefetch(0);
  commit(q0, k0, v0, v0reg);
  prefetch(1);
  for (int p = lane; p < nn; p += 64) {
    accS[p] = 0.f;
    T2[p] = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) SuB[k * nn + p] = Au[k * nn + p] = 0.f;
  }
  wsync();
  // ---- value channel
  for (int p = lane; p < 4 * nn; p += 64) {
    const int pair = p >> 2, qt = p & 3, i = pair / N, j = pair - (pair / N) * N;
    float s = dot16(q0 + i * ld + 16 * qt, k0 + j * ld + 16 * qt);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (qt == 0) A0[pair] = s * scale;
  }
  wsync();
  if (lane < N) {
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < N; ++j) m = fmaxf(m, A0[lane * N + j]);
    float e[N], ssum = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      e[j] = expf(A0[lane * N + j] - m);
      ssum += e[j];
    }
    const float inv = 1.f / ssum;
#pragma unroll
    for (int j = 0; j < N; ++j) A0[lane * N + j] = e[j] * inv;
  }
  wsync();
  {
    float v0r[N];
#pragma unroll
    for (int j = 0; j < N; ++j) v0r[j] = VR ? v0reg[VR ? j : 0] : v0[j * ld + lane];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fmaf(A0[i * N + j], v0r[j], acc);
      obase[(size_t)(i * C) * D] = acc;
    }
  }
  // running flow sums Qu_k = sum_t alpha_kt q_t (and Ku, Vu), one column per lane.  In the
  // FEAT form they are not accumulated: tangent t moves only electron t/2's features, so
  // Qu_k[i] = g_k(i) . Wq with g_k(i) = sum_{t of i} alpha_kt f_t(i) (4-vectors), and
  // Qu_k[i] . Ku_k[j] = g_k(i)^T (Wq Wk^T) g_k(j) with a 4 x 4 Wq Wk^T per head.
  constexpr int NU = FEAT ? 1 : N;
  float rOL[N], rQu[3][NU], rKu[3][NU], rVu[3][NU];
#pragma unroll
  for (int i = 0; i < N; ++i) rOL[i] = 0.f;
#pragma unroll
  for (int i = 0; i < NU; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k) rQu[k][i] = rKu[k][i] = rVu[k][i] = 0.f;
  // g_k(i) of the FEAT form: alpha-weighted tangent features of electron i
  auto gflow = [&](int k, int i) -> float4 {
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));  // st ct sp cp
    const float st = g.x, ct = g.y, sp = g.z, cp = g.w;
    const float ae = (k == 0) ? -sp : (k == 1 ? cp : 0.f);                  // alpha[k][2i]
    const float ao = (k == 0) ? -(ct * cp) : (k == 1 ? -(ct * sp) : st);  // alpha[k][2i+1]
    // ae * (-st, ct cp, ct sp, 0) + ao * (0, -sp, cp, 0)
    return make_float4(-ae * st, ae * ct * cp - ao * sp, ae * ct * sp + ao * cp, 0.f);
  };

  // one channel c >= 1 (the loops below run the tangents, then the Laplacian and flow
  // channels, with the flow products in between: each loop sees a fixed channel kind)
  auto chan = [&](const int c) __attribute__((always_inline)) {
    wsync();
    commit(qc, kc, vc, vcreg);
    if (c + 1 < C) prefetch(c + 1);
    wsync();
    const bool tang = c <= T;
    const int k = c - T - 2;
    // phase A: scores.  FEAT tangents: channel t moves only electron e = t / 2, so q_t, k_t,
    // v_t are zero off row e and S_t = s (q_t k0^T + q0 k_t^T) lives on row e and column e
    // only, P_t = q_t k_t^T on (e, e): 2N dots instead of 3 N^2
    if (FEAT && tang) {
      const int e = (c - 1) >> 1;
      for (int p = lane; p < nn; p += 64) S[p] = P[p] = 0.f;
      if (lane < 8 * N) {  // task = lane / 4: j < N row e; N + i (i != e) column e; 2N - 1 + ... P
        const int task = lane >> 2, qt = lane & 3;
        int i, j;
        float s1;
        if (task < N) {  // S[e][j] = qc[e] . k0[j] (+ q0[e] . kc[e] at j = e)
          i = e;
          j = task;
          s1 = dot16(qc + e * ld + 16 * qt, k0 + j * ld + 16 * qt);
          if (j == e) s1 += dot16(q0 + e * ld + 16 * qt, kc + e * ld + 16 * qt);
        } else if (task < 2 * N - 1) {  // S[i][e] = q0[i] . kc[e], i != e
          i = task - N;
          if (i >= e) ++i;
          j = e;
          s1 = dot16(q0 + i * ld + 16 * qt, kc + e * ld + 16 * qt);
        } else {  // P[e][e]
          i = j = e;
          s1 = dot16(qc + e * ld + 16 * qt, kc + e * ld + 16 * qt);
        }
        s1 += __shfl_xor(s1, 1, 64);
        s1 += __shfl_xor(s1, 2, 64);
        if (qt == 0 && task < 2 * N) {
          if (task < 2 * N - 1)
            S[i * N + j] = s1 * scale;
          else
            P[i * N + j] = s1;
        }
      }
    }
    // dense channels: lane = (row i, group of JB columns j, quarter of d): the q rows of i
    // are read once per JB pairs (N = 6: one pass of 48 lanes, 32 b128 reads per lane where
    // one pair per lane took three passes of 24)
    constexpr int JB = 3, NG = (N + JB - 1) / JB;
    for (int p = lane; p < ((FEAT && tang) ? 0 : 4 * N * NG); p += 64) {
      const int qt = p & 3, ig = p >> 2, i = ig / NG, j0 = (ig - (ig / NG) * NG) * JB;
      const float* qci = qc + i * ld + 16 * qt;
      const float* q0i = q0 + i * ld + 16 * qt;
      float s1[JB], s2[JB];
#pragma unroll
      for (int jj = 0; jj < JB; ++jj) s1[jj] = s2[jj] = 0.f;
#pragma unroll 1
      for (int m = 0; m < 4; ++m) {  // rolled: the live running sums leave few registers
        const float4 a = *reinterpret_cast<const float4*>(qci + 4 * m);
        const float4 a0 = *reinterpret_cast<const float4*>(q0i + 4 * m);
#pragma unroll
        for (int jj = 0; jj < JB; ++jj) {
          if (N % JB != 0 && j0 + jj >= N) continue;
          const int oj = (j0 + jj) * ld + 16 * qt + 4 * m;
          const float4 b0 = *reinterpret_cast<const float4*>(k0 + oj);
          const float4 bc = *reinterpret_cast<const float4*>(kc + oj);
          s1[jj] = fmaf(a.x, b0.x, fmaf(a.y, b0.y, fmaf(a.z, b0.z, fmaf(a.w, b0.w, s1[jj]))));
          s1[jj] = fmaf(a0.x, bc.x, fmaf(a0.y, bc.y, fmaf(a0.z, bc.z, fmaf(a0.w, bc.w, s1[jj]))));
          if (tang) s2[jj] = fmaf(a.x, bc.x, fmaf(a.y, bc.y, fmaf(a.z, bc.z, fmaf(a.w, bc.w, s2[jj]))));
        }
      }
#pragma unroll
      for (int jj = 0; jj < JB; ++jj) {
        s1[jj] += __shfl_xor(s1[jj], 1, 64);
        s1[jj] += __shfl_xor(s1[jj], 2, 64);
        if (tang) {
          s2[jj] += __shfl_xor(s2[jj], 1, 64);
          s2[jj] += __shfl_xor(s2[jj], 2, 64);
        }
      }
      if (qt == 0) {
#pragma unroll
        for (int jj = 0; jj < JB; ++jj) {
          if (N % JB != 0 && j0 + jj >= N) continue;
          const int pair = i * N + j0 + jj;
          if (tang) {
            S[pair] = s1[jj] * scale;
            P[pair] = s2[jj];
          } else if (k < 0) {
            S[pair] = s1[jj] * scale + accS[pair];
            P[pair] = T2[pair];
          } else {
            S[pair] = scale * (s1[jj] + 2.f * QK[k * nn + pair]);
            const float u = SuB[k * nn + pair];
            P[pair] = u * u;
          }
        }
      }
    }
    wsync();
    // phase B: softmax derivatives (lane = pair)
    for (int p = lane; p < nn; p += 64) {
      const int i = p / N;
      float m1 = 0.f, m2 = 0.f;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        m1 = fmaf(A0[i * N + j], S[i * N + j], m1);
        m2 = fmaf(A0[i * N + j], P[i * N + j], m2);
      }
      if (tang) {
        const int t = c - 1;
        const float sb = S[p] - m1;
        const float at = A0[p] * sb;
        accS[p] = fmaf(2.f * scale, P[p], accS[p]);
        T2[p] = fmaf(sb, sb, T2[p]);
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) {
          const float a = al[kk * T + t];
          SuB[kk * nn + p] = fmaf(a, sb, SuB[kk * nn + p]);
          Au[kk * nn + p] = fmaf(a, at, Au[kk * nn + p]);
        }
        Rm[p] = at;
      } else {
        Rm[p] = A0[p] * ((S[p] - m1) + (P[p] - m2));
      }
    }
    wsync();
    // phase C: outputs (lane = d)
    {
      float v0r[N], vcr[N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        v0r[j] = VR ? v0reg[VR ? j : 0] : v0[j * ld + lane];
        vcr[j] = VR ? vcreg[VR ? j : 0] : vc[j * ld + lane];
      }
      // flow channels: Vu_k[j] (this lane's column) once per channel, not once per (i, j)
      // (FEAT: g_k(j) . Wv from the geometry; else the running sums, k selected once)
      float vuj[N];
      if (!tang && k >= 0) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
          if constexpr (FEAT)
            vuj[j] = FeatW::dot(gflow(k, j), fw.wv);
          else
            vuj[j] = (k == 0) ? rVu[0][j] : (k == 1 ? rVu[1][j] : rVu[2][j]);
        }
      }
      // FEAT tangents: v_t lives on row e only, so A0 v_t and sum_j A_t v_t are one term each
      const int e_t = (c - 1) >> 1;
      const float vce = (FEAT && tang) ? (VR ? vcreg[VR ? e_t : 0] : vc[e_t * ld + lane]) : 0.f;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        float acc = 0.f, acc2 = 0.f;
        if (FEAT && tang) {
#pragma unroll
          for (int j = 0; j < N; ++j) acc = fmaf(Rm[i * N + j], v0r[j], acc);
          acc = fmaf(A0[i * N + e_t], vce, acc);
          acc2 = Rm[i * N + e_t] * vce;
        } else {
#pragma unroll
          for (int j = 0; j < N; ++j) {
            const float r = Rm[i * N + j];
            acc = fmaf(r, v0r[j], fmaf(A0[i * N + j], vcr[j], acc));
            if (tang) acc2 = fmaf(r, vcr[j], acc2);
          }
        }
        if (tang) {
          rOL[i] = fmaf(2.f, acc2, rOL[i]);
          if constexpr (!FEAT) {
            const int t = c - 1;
            const float qv = qc[i * ld + lane], kv = kc[i * ld + lane];
#pragma unroll
            for (int kk = 0; kk < 3; ++kk) {
              const float a = al[kk * T + t];
              rQu[kk][i] = fmaf(a, qv, rQu[kk][i]);
              rKu[kk][i] = fmaf(a, kv, rKu[kk][i]);
              rVu[kk][i] = fmaf(a, vcr[i], rVu[kk][i]);
            }
          }
        } else if (k < 0) {
          acc += rOL[i];
        } else {
          float a2 = 0.f;
#pragma unroll
          for (int j = 0; j < N; ++j) a2 = fmaf(Au[k * nn + i * N + j], vuj[j], a2);
          acc = fmaf(2.f, a2, acc);
        }
        obase[(size_t)(i * C + c) * D] = acc;
      }
    }
  };
  for (int c = 1; c <= T; ++c) chan(c);
  {  // after the last tangent: qu_k . ku_k^T for the flow channels
      // sums over the 64 lanes of R per-lane values, 8 at a time transposed through the
      // current channel's q|k|v rows (free until the next commit): 8 writes, 2 b128 reads
      // and 3 swaps per 8 sums, where a butterfly costs 6 ds_bpermute per sum.  TSUM: those
      // rows hold the [8][68] scratch
      constexpr bool TSUM = (VR ? 2 : 3) * N * ld >= 8 * 68;
      float* tw = qc;  // [8][68]
      auto lane_sums = [&](auto getv, auto R_, float* dst) __attribute__((always_inline)) {
        constexpr int R = decltype(R_)::value, HS = 8;  // rows per pass (8 lanes per row)
        wsync();
#pragma unroll
        for (int r0 = 0; r0 < R; r0 += HS) {
#pragma unroll
          for (int j = 0; j < HS; ++j)
            if (r0 + j < R) tw[j * 68 + lane] = getv(r0 + j);
          wsync();
          const int jr = lane >> 3, q = lane & 7;
          const float4 t0 = *reinterpret_cast<const float4*>(tw + jr * 68 + 8 * q);
          const float4 t1 = *reinterpret_cast<const float4*>(tw + jr * 68 + 8 * q + 4);
          float v = ((t0.x + t0.y) + (t0.z + t0.w)) + ((t1.x + t1.y) + (t1.z + t1.w));
          v += __shfl_xor(v, 1, 64);
          v += __shfl_xor(v, 2, 64);
          v += __shfl_xor(v, 4, 64);
          if (q == 0 && r0 + jr < R) dst[r0 + jr] = v;
          wsync();
        }
      };
      if constexpr (FEAT) {
        // 4 x 4 Wq Wk^T of this head (sums over the head's 64 columns), through QK's slots
        const float wq[4] = {fw.wq.x, fw.wq.y, fw.wq.z, fw.wq.w};
        const float wk[4] = {fw.wk.x, fw.wk.y, fw.wk.z, fw.wk.w};
        float Mqk[4][4];
        if constexpr (TSUM) {
          lane_sums([&](int r) { return wq[r >> 2] * wk[r & 3]; }, std::integral_constant<int, 16>{}, QK);
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int e = 0; e < 4; ++e) Mqk[a][e] = QK[4 * a + e];
          wsync();
        } else {
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int e = 0; e < 4; ++e) Mqk[a][e] = wave_sum(wq[a] * wk[e]);
        }
        for (int p = lane; p < 3 * nn; p += 64) {
          const int kk = p / nn, pair = p - kk * nn, i = pair / N, j = pair - (pair / N) * N;
          const float4 gi_ = gflow(kk, i), gj = gflow(kk, j);
          const float gia[4] = {gi_.x, gi_.y, gi_.z, gi_.w}, gja[4] = {gj.x, gj.y, gj.z, gj.w};
          float v = 0.f;
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int e = 0; e < 4; ++e) v = fmaf(gia[a] * Mqk[a][e], gja[e], v);
          QK[p] = v;
        }
      } else if constexpr (TSUM) {
        // one pass per (k, i): the N products qu_k[i] ku_k[j] (compile-time register indices)
#pragma unroll
        for (int kk = 0; kk < 3; ++kk)
#pragma unroll
          for (int i = 0; i < N; ++i)
            lane_sums([&](int j) { return rQu[kk][i] * rKu[kk][j]; }, std::integral_constant<int, N>{},
                      QK + kk * nn + i * N);
      } else {
#pragma unroll
        for (int kk = 0; kk < 3; ++kk)
#pragma unroll
          for (int i = 0; i < N; ++i)
#pragma unroll
            for (int j = 0; j < N; ++j) {
              const float v = wave_sum(rQu[kk][i] * rKu[kk][j]);
              if (lane == 0) QK[kk * nn + i * N + j] = v;
            }
      }
  }
#pragma unroll
  for (int c = T + 1; c < C; ++c) chan(c);  // unrolled: the flow index k is a constant
}

// ---------------------------------------------------------------------------------------
// Value-only kernel (log psi, N <= 8, dh = 64): one wave per (walker, head), four waves
// per workgroup, no block barriers.  Lane = feature column; q|k staged in the wave's LDS
// for the N x N scores (4 lanes per pair, 16-byte reads); v stays in registers.
template <int N, bool FEAT>
__global__ __launch_bounds__(256) void attention_val_kernel(const float* __restrict__ qkv,
                                                            const float* __restrict__ geo, float* __restrict__ o,
                                                            int H, int ntask, const float* __restrict__ W0qkv,
                                                            const float* __restrict__ bqkv, const float* __restrict__ Mqk,
                                                            int n_up) {
  constexpr int dh = 64, PER = attn_val_floats<N>();
  extern __shared__ float sm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int task = blockIdx.x * 4 + w;
  if (task >= ntask) return;  // the whole wave leaves; nothing below synchronises waves
  float* qs = sm + w * PER;  // q, k rows and the weights (attn_val_core)
  const int b = task / H, h = task - (task / H) * H;
  const int D = H * dh;
  float pq[1][N], pk[1][N], pv[1][N];
  float out[1][N];
  if constexpr (FEAT) {  // scores from the features (attn_feat_core), v formed in registers
    FeatW fw;
    fw.load(W0qkv, bqkv, D, h * dh + lane);
    feat_v<N>(fw, geo, b, n_up, pv[0]);
    attn_feat_core<N, 1>(Mqk + h * kMqkStride, geo, b, n_up, pv, qs, lane, out);
  } else {
    const float* base = qkv + (size_t)b * N * (3 * D) + h * dh + lane;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      pq[0][i] = base[(size_t)i * 3 * D];
      pk[0][i] = base[(size_t)i * 3 * D + D];
      pv[0][i] = base[(size_t)i * 3 * D + 2 * D];
    }
    attn_val_core<N, 1>(pq, pk, pv, qs, lane, out);
  }
  float* ob = o + (size_t)b * N * D + h * dh + lane;
#pragma unroll
  for (int i = 0; i < N; ++i) ob[(size_t)i * D] = out[0][i];
}

// ---------------------------------------------------------------------------------------
// Layer 1's CHANNEL attention in feature space (round 5; local energy, C = 2N + 5, dh = 64).
// Every q|k|v row of layer 1 is a feature-channel vector times the folded map: with
// f~_c,i = (f_c,i, [c == 0]) (the 4 input features of psiformer.py:51-60 or their channel
// seeds, input.hip; the bias only on the value channel),
//   q_c,i = f~_c,i Wq~,  k_c,j = f~_c,j Wk~,  v_c,j = f~_c,j Wv~   (Wx~ = 5 x 64 per head),
// so every score of the channel rules (header of this file) is a 5 x 5 form with the head's
// Mqk = s Wq~ Wk~^T (launch_lowrank_qk): s q_a,i . k_b,j = f~_a,i^T Mqk f~_b,j, and every output
// is a 5-vector o^_c,i (the same combinations applied to f~ instead of v) times Wv~:
//   o_c,i = o^_c,i Wv~,   o^_0 = A0 f~0,  o^_t = A_t f~0 + A0 f~t,
//   o^_L = A_L f~0 + A0 f~L + 2 sum_t A_t f~t,  o^_Sk = A_Sk f~0 + A0 f~Sk + 2 Au_k g_k
// (g_k,j = sum_{t of j} alpha_kt f~t,j: the flow sums of the tangent seeds).  Tangent t moves
// only electron e = t / 2, so S_t lives on row e and column e and sum_t A_t f~t is one term per
// tangent.  One wave per (walker, head): the N x N algebra on lanes = pairs (LDS-staged,
// wave barriers only), the 5-vectors on lanes = (electron, component), then lane = feature
// column d for o_c,i[d] = o^_c,i . (Wv~[:, d]) and the store: no q|k|v row is ever formed,
// the 64-wide dots of attention_wave_kernel<N, true> become 30-FMA forms per pair.
// ---------------------------------------------------------------------------------------
// attention_feat_kernel restructured (round 5, "feat2"): the same rules in the same feature
// space, with the tangent channels in O(N) per channel instead of O(N^2) LDS passes and O(N^3)
// row sums.  S_t lives on row e and column e only (Srow_j = s f~e^T M f~0_j, Scol_i = s f~0_i^T
// M f~e), so
//   m1_i = <S_t>_A0,i = A0_ie Scol_i (i != e),  sum_j A0_ej S_t,ej (i = e);
//   o^_t,i = sum_j A_t,ij f~0_j + A0_ie f~e = m1_i (f~0_e - o^_0,i) + A0_ie f~e  (i != e; o^_0 = A0 f~0),
//   row e directly (N terms);  oL += 2 A_t,ie f~e.
// The dense accumulators T2 = sum_t Sbar_t^2 and SuB_k = sum_t alpha_kt Sbar_t stay in registers
// on the pairs each lane owns (p = lane + 64 u), and Au_k = sum_t alpha_kt A_t = A0 * SuB_k is
// formed once for the flow channels.  The four dense channels (L, S_0..2) keep the pairwise
// form.  LDS: A0 and three N x N scratch arrays, the rest small (C5: 10 KB per wave).
// Output (round 6): the 5-vectors o^_c,i themselves (ofeat_k columns per row, dh_internal.h),
// not o = o^ Wv~: the next map folds Wv~ into its weights (o Wol = o^ U), so each (row, head)
// writes 8 floats instead of 64.
template <int N>
struct Feat2Smem {
  static constexpr int nn = N * N, T = 2 * N;
  static constexpr int G = 0, F0 = G + 4 * N, OH0 = F0 + 5 * N, GK = OH0 + 5 * N, AL = GK + 15 * N, ACC = AL + 3 * T,
                       SR = ACC + N, SC = SR + N, M1 = SC + N, M2 = M1 + N, OH = M2 + N, FC = OH + 5 * N,
                       A0 = FC + 5 * N, S = A0 + nn, P = S + nn, RM = P + nn, TOTAL = RM + nn;
};

template <int N>
__global__ __launch_bounds__(64) void attention_feat2_kernel(const float* __restrict__ geo, float* __restrict__ o,
                                                             int H, int KO, const float* __restrict__ Mqk, int n_up) {
  constexpr int dh = 64, T = 2 * N, C = 2 * N + 5, nn = N * N;
  constexpr int PP = (nn + 63) / 64, QQ = (5 * N + 63) / 64;  // pairs / (electron, component) per lane
  using L = Feat2Smem<N>;
  extern __shared__ float sm[];
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H, lane = threadIdx.x;
  const int D = H * dh;
  auto wsync = [] { __builtin_amdgcn_wave_barrier(); };
  float *g = sm + L::G, *f0 = sm + L::F0, *oh0 = sm + L::OH0, *gk = sm + L::GK, *al = sm + L::AL, *accS = sm + L::ACC;
  float *SR = sm + L::SR, *SC = sm + L::SC, *M1 = sm + L::M1, *M2 = sm + L::M2, *oh = sm + L::OH, *fc = sm + L::FC;
  float *A0 = sm + L::A0, *Ss = sm + L::S, *Ps = sm + L::P, *Rm = sm + L::RM;
  float Mr[25];
#pragma unroll
  for (int q = 0; q < 25; ++q) Mr[q] = Mqk[h * kMqkStride + q];
  for (int i = lane; i < N; i += 64) {
    const float4 gi = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));  // st ct sp cp
    g[4 * i] = gi.x;
    g[4 * i + 1] = gi.y;
    g[4 * i + 2] = gi.z;
    g[4 * i + 3] = gi.w;
    const float4 f = feature_channel<T>(0, i, gi, (i < n_up) ? 1.f : -1.f);
    f0[5 * i] = f.x;
    f0[5 * i + 1] = f.y;
    f0[5 * i + 2] = f.z;
    f0[5 * i + 3] = f.w;
    f0[5 * i + 4] = 1.f;
    accS[i] = 0.f;
  }
  for (int t = lane; t < T; t += 64) {
    const int i = t >> 1;
    const float4 gi = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));
    const float st = gi.x, ct = gi.y, sp = gi.z, cp = gi.w;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float a;
      if ((t & 1) == 0)
        a = (k == 0) ? -sp : (k == 1 ? cp : 0.f);
      else
        a = (k == 0) ? -(ct * cp) : (k == 1 ? -(ct * sp) : st);
      al[k * T + t] = a;
    }
  }
  for (int q = lane; q < 3 * N; q += 64) {  // g_k,i: alpha-weighted tangent seeds of electron i
    const int k = q / N, i = q - k * N;
    const float4 gi = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));
    const float st = gi.x, ct = gi.y, sp = gi.z, cp = gi.w;
    const float ae = (k == 0) ? -sp : (k == 1 ? cp : 0.f);
    const float ao = (k == 0) ? -(ct * cp) : (k == 1 ? -(ct * sp) : st);
    float* d = gk + (k * N + i) * 5;
    d[0] = -ae * st;
    d[1] = ae * ct * cp - ao * sp;
    d[2] = ae * ct * sp + ao * cp;
    d[3] = 0.f;
    d[4] = 0.f;
  }
  wsync();
  auto form = [&](const float* x, const float* y) __attribute__((always_inline)) {
    float sres = 0.f;
#pragma unroll
    for (int a = 0; a < 5; ++a) {
      float u = 0.f;
#pragma unroll
      for (int c2 = 0; c2 < 5; ++c2) u = fmaf(Mr[5 * a + c2], y[c2], u);
      sres = fmaf(x[a], u, sres);
    }
    return sres;
  };
  // channel c's o~ rows: this head's 8-column segment (the five sums, three zeros) of every
  // electron, lane = (electron, slot); the last head also zeroes the columns past 8 H
  float* obase = o + (size_t)b * N * C * KO;
  const int tail = h == H - 1 ? KO - 8 * H : 0;
  auto expand = [&](int c) __attribute__((always_inline)) {
    wsync();
    for (int q = lane; q < 8 * N; q += 64) {
      const int i = q >> 3, a = q & 7;
      obase[(size_t)(i * C + c) * KO + 8 * h + a] = a < 5 ? oh[5 * i + a] : 0.f;
    }
    for (int q = lane; q < tail * N; q += 64) {
      const int i = q / tail;
      obase[(size_t)(i * C + c) * KO + 8 * H + (q - i * tail)] = 0.f;
    }
  };

  // ---- value channel: A0 = softmax(f~0 Mqk f~0^T), o^_0 = A0 f~0
  float a0r[PP];
#pragma unroll
  for (int u = 0; u < PP; ++u) {
    const int p = lane + 64 * u;
    if (p < nn) {
      const int i = p / N, j = p - (p / N) * N;
      A0[p] = form(f0 + 5 * i, f0 + 5 * j);
    }
  }
  wsync();
  for (int i = lane; i < N; i += 64) {
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < N; ++j) m = fmaxf(m, A0[i * N + j]);
    float e[N], ssum = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      e[j] = expf(A0[i * N + j] - m);
      ssum += e[j];
    }
    const float inv = 1.f / ssum;
#pragma unroll
    for (int j = 0; j < N; ++j) A0[i * N + j] = e[j] * inv;
  }
  wsync();
#pragma unroll
  for (int u = 0; u < PP; ++u) {
    const int p = lane + 64 * u;
    a0r[u] = p < nn ? A0[p] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < QQ; ++u) {
    const int q = lane + 64 * u;
    if (q < 5 * N) {
      const int i = q / 5, a = q - (q / 5) * 5;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fmaf(A0[i * N + j], f0[5 * j + a], acc);
      oh0[q] = acc;
      oh[q] = acc;
    }
  }
  expand(0);

  // ---- tangents
  float T2r[PP], SuBr[3][PP], oLr[QQ];
#pragma unroll
  for (int u = 0; u < PP; ++u) {
    T2r[u] = 0.f;
    SuBr[0][u] = SuBr[1][u] = SuBr[2][u] = 0.f;
  }
#pragma unroll
  for (int u = 0; u < QQ; ++u) oLr[u] = 0.f;
#pragma unroll 1
  for (int t = 0; t < T; ++t) {
    const int c = 1 + t, e = t >> 1;
    float fe[5];
    {
      const float4 ge = make_float4(g[4 * e], g[4 * e + 1], g[4 * e + 2], g[4 * e + 3]);
      const float4 f = feature_channel<T>(c, e, ge, (e < n_up) ? 1.f : -1.f);
      fe[0] = f.x;
      fe[1] = f.y;
      fe[2] = f.z;
      fe[3] = f.w;
      fe[4] = 0.f;
    }
    for (int j = lane; j < N; j += 64) {
      SR[j] = form(fe, f0 + 5 * j);
      SC[j] = form(f0 + 5 * j, fe);
    }
    if (lane == 0) accS[e] += 2.f * form(fe, fe);  // s q_t . k_t, twice (S_L)
    wsync();
    for (int i = lane; i < N; i += 64) {
      float m1;
      if (i != e) {
        m1 = A0[i * N + e] * SC[i];
      } else {
        m1 = 0.f;
#pragma unroll
        for (int j = 0; j < N; ++j) m1 = fmaf(A0[e * N + j], SR[j] + (j == e ? SC[e] : 0.f), m1);
      }
      M1[i] = m1;
    }
    wsync();
    const float a_0 = al[t], a_1 = al[T + t], a_2 = al[2 * T + t];
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int p = lane + 64 * u;
      if (p < nn) {
        const int i = p / N, j = p - (p / N) * N;
        const float sv = (i == e ? SR[j] : 0.f) + (j == e ? SC[i] : 0.f);
        const float sb = sv - M1[i];
        T2r[u] = fmaf(sb, sb, T2r[u]);
        SuBr[0][u] = fmaf(a_0, sb, SuBr[0][u]);
        SuBr[1][u] = fmaf(a_1, sb, SuBr[1][u]);
        SuBr[2][u] = fmaf(a_2, sb, SuBr[2][u]);
      }
    }
#pragma unroll
    for (int u = 0; u < QQ; ++u) {
      const int q = lane + 64 * u;
      if (q < 5 * N) {
        const int i = q / 5, a = q - (q / 5) * 5;
        const float m1 = M1[i], a0ie = A0[i * N + e];
        float acc, atie;
        if (i != e) {
          acc = m1 * (f0[5 * e + a] - oh0[q]);
          atie = a0ie * (SC[i] - m1);
        } else {
          acc = 0.f;
#pragma unroll
          for (int j = 0; j < N; ++j) {
            const float at = A0[e * N + j] * ((SR[j] + (j == e ? SC[e] : 0.f)) - m1);
            acc = fmaf(at, f0[5 * j + a], acc);
          }
          atie = a0ie * ((SR[e] + SC[e]) - m1);
        }
        acc = fmaf(a0ie, fe[a], acc);
        oLr[u] = fmaf(2.f * atie, fe[a], oLr[u]);
        oh[q] = acc;
      }
    }
    expand(c);
  }
  // ---- Laplace-Beltrami and flow channels (dense seeds on every electron)
#pragma unroll 1
  for (int c = T + 1; c < C; ++c) {
    const int k = c - T - 2;  // flow axis (k < 0: the Laplace-Beltrami channel)
    wsync();
    for (int i = lane; i < N; i += 64) {
      const float4 gi = make_float4(g[4 * i], g[4 * i + 1], g[4 * i + 2], g[4 * i + 3]);
      const float4 f = feature_channel<T>(c, i, gi, (i < n_up) ? 1.f : -1.f);
      fc[5 * i] = f.x;
      fc[5 * i + 1] = f.y;
      fc[5 * i + 2] = f.z;
      fc[5 * i + 3] = f.w;
      fc[5 * i + 4] = 0.f;
    }
    wsync();
    float sr[PP], pr[PP];
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int p = lane + 64 * u;
      sr[u] = pr[u] = 0.f;
      if (p < nn) {
        const int i = p / N, j = p - (p / N) * N;
        float sv = form(fc + 5 * i, f0 + 5 * j) + form(f0 + 5 * i, fc + 5 * j);
        float pv;
        if (k < 0) {
          if (i == j) sv += accS[i];
          pv = T2r[u];
        } else {
          sv += 2.f * form(gk + (k * N + i) * 5, gk + (k * N + j) * 5);
          const float sbk = k == 0 ? SuBr[0][u] : (k == 1 ? SuBr[1][u] : SuBr[2][u]);
          pv = sbk * sbk;
        }
        sr[u] = sv;
        pr[u] = pv;
        Ss[p] = sv;
        Ps[p] = pv;
      }
    }
    wsync();
    for (int i = lane; i < N; i += 64) {
      float m1 = 0.f, m2 = 0.f;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        m1 = fmaf(A0[i * N + j], Ss[i * N + j], m1);
        m2 = fmaf(A0[i * N + j], Ps[i * N + j], m2);
      }
      M1[i] = m1;
      M2[i] = m2;
    }
    wsync();
#pragma unroll
    for (int u = 0; u < PP; ++u) {
      const int p = lane + 64 * u;
      if (p < nn) {
        const int i = p / N;
        Rm[p] = a0r[u] * ((sr[u] - M1[i]) + (pr[u] - M2[i]));
        if (k >= 0) {  // Au_k = A0 * SuB_k, over the scores (read above)
          const float sbk = k == 0 ? SuBr[0][u] : (k == 1 ? SuBr[1][u] : SuBr[2][u]);
          Ss[p] = a0r[u] * sbk;
        }
      }
    }
    wsync();
#pragma unroll
    for (int u = 0; u < QQ; ++u) {
      const int q = lane + 64 * u;
      if (q < 5 * N) {
        const int i = q / 5, a = q - (q / 5) * 5;
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < N; ++j) acc = fmaf(Rm[i * N + j], f0[5 * j + a], fmaf(A0[i * N + j], fc[5 * j + a], acc));
        if (k < 0) {
          acc += oLr[u];
        } else {
          float a2 = 0.f;
#pragma unroll
          for (int j = 0; j < N; ++j) a2 = fmaf(Ss[i * N + j], gk[(k * N + j) * 5 + a], a2);
          acc = fmaf(2.f, a2, acc);
        }
        oh[q] = acc;
      }
    }
    expand(c);
  }
}

template <int N>
void launch_feat(const Dims& d, const float* geo, float* o, int nw, const float* Mqk, hipStream_t s) {
  const size_t smem2 = (size_t)Feat2Smem<N>::TOTAL * sizeof(float);
  ensure_smem(attention_feat2_kernel<N>, smem2);
  hipLaunchKernelGGL(attention_feat2_kernel<N>, dim3(nw * d.H), dim3(64), smem2, s, geo, o, d.H, ofeat_k(d), Mqk,
                     d.n_up);
}

__global__ void lowrank_qk_kernel(const float* __restrict__ W0qkv, const float* __restrict__ bqkv, int D, int H,
                                  float* __restrict__ Mqk) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= H * 25) return;
  const int h = t / 25, a = (t % 25) / 5, c = t % 5, ld = 3 * D;
  double s = 0.0;
  for (int e = 0; e < 64; ++e) {
    const int col = h * 64 + e;
    const double q = a < 4 ? (double)W0qkv[a * ld + col] : (double)bqkv[col];
    const double k = c < 4 ? (double)W0qkv[c * ld + D + col] : (double)bqkv[D + col];
    s += q * k;
  }
  Mqk[h * kMqkStride + 5 * a + c] = (float)(0.125 * s);
}

// U^T[n][8 h + a] = sum_d Wv~[a][h 64 + d] Wol[h 64 + d][n] (a < 5: Wv~ = the folded W0 Wv
// rows and bv), f64 sums; padding columns stay as the caller's memset left them (zero)
__global__ void ofeat_weight_kernel(const float* __restrict__ W0qkv, const float* __restrict__ bqkv,
                                    const float* __restrict__ Wol, int D, int H, int KO, float* __restrict__ UT) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= D * 8 * H) return;
  const int n = t / (8 * H), k = t - n * (8 * H), h = k >> 3, a = k & 7, ld = 3 * D;
  if (a >= 5) return;
  double s = 0.0;
  for (int e = 0; e < 64; ++e) {
    const int col = h * 64 + e;
    const double v = a < 4 ? (double)W0qkv[a * ld + 2 * D + col] : (double)bqkv[2 * D + col];
    s += v * (double)Wol[(size_t)col * D + n];
  }
  UT[(size_t)n * KO + k] = (float)s;
}

// layer 1's coefficient-space maps (gemm_lnch.hip MODE 2): thread (n, j), j < 32
__global__ void l1_basis_kernel(const float* __restrict__ W0, const float* __restrict__ UT, int KO,
                                const float* __restrict__ bol, const float* __restrict__ ln1,
                                const float* __restrict__ Wm, const float* __restrict__ bm, int D,
                                float* __restrict__ BT, float* __restrict__ VT) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= D * 32) return;
  const int n = t >> 5, j = t & 31;
  auto basis = [&](int k) -> double {  // B[j][k]
    double e;
    if (j < 4)
      e = W0[j * D + k];
    else if (j < 24)
      e = UT[(size_t)k * KO + 8 * ((j - 4) / 5) + (j - 4) % 5];
    else if (j == 24)
      e = bol[k];
    else if (j == 25)
      e = 1.0;
    else
      return j == 26 ? (double)ln1[D + k] : 0.0;
    return (double)ln1[k] * e;
  };
  double v = j == 26 ? (double)bm[n] : 0.0;
  if (j <= 26)
    for (int k = 0; k < D; ++k) v += basis(k) * (double)Wm[(size_t)k * D + n];
  BT[(size_t)n * 32 + j] = (float)basis(n);
  VT[(size_t)n * 32 + j] = (float)v;
}

template <int N>
void launch_wave(const Dims& d, const float* qkv, const float* W0qkv, const float* bqkv, const float* Mqk,
                 const float* geo, float* o, int nw, int C, hipStream_t s) {
  const int nn = N * N;
  if (C == 1) {
    const int ntask = nw * d.H;
    const size_t smem = (size_t)4 * (2 * N * 68 + nn) * sizeof(float);
    if (W0qkv)
      hipLaunchKernelGGL((attention_val_kernel<N, true>), dim3((ntask + 3) / 4), dim3(256), smem, s, qkv, geo, o,
                         d.H, ntask, W0qkv, bqkv, Mqk, d.n_up);
    else
      hipLaunchKernelGGL((attention_val_kernel<N, false>), dim3((ntask + 3) / 4), dim3(256), smem, s, qkv, geo, o,
                         d.H, ntask, W0qkv, bqkv, Mqk, d.n_up);
    return;
  }
  const size_t smem = (size_t)((N > 8 ? 4 : 6) * N * 68 + 15 * nn + 6 * N) * sizeof(float);  // VR above
  if (W0qkv)
    hipLaunchKernelGGL((attention_wave_kernel<N, true>), dim3(nw * d.H), dim3(64), smem, s, qkv, geo, o, d.H, W0qkv,
                       bqkv, d.n_up);
  else
    hipLaunchKernelGGL((attention_wave_kernel<N, false>), dim3(nw * d.H), dim3(64), smem, s, qkv, geo, o, d.H, W0qkv,
                       bqkv, d.n_up);
}

template <int PF, int RPT>
void launch_ch(const Dims& d, const float* qkv, const float* geo, float* o, int nw, hipStream_t s) {
  const size_t smem = (size_t)attn_layout2(d.N, d.dh).total * sizeof(float);
  ensure_smem(attention_ch_kernel<PF, RPT>, smem);
  hipLaunchKernelGGL((attention_ch_kernel<PF, RPT>), dim3(nw * d.H), dim3(256), smem, s, qkv, geo, o, d.N, d.H,
                     d.dh);
}

}  // namespace

// wave kernels: every N <= 8, plus the N = 10 and N = 20 instances of BASELINE.json's
// C4 / C5 configs (one wave per (walker, head) there too: 2x / 10x faster than the
// 256-thread channel kernel v2, whose three barriers per channel dominate)
bool attention_takes_features(const Dims& d, int C) {
  (void)C;  // the wave kernels and the MFMA kernel both form layer 1's q|k|v from the features
  return d.dh == 64 && (d.N <= 8 || d.N == 10 || d.N == 20);
}

void launch_lowrank_qk(const Dims& d, const float* W0qkv, const float* bqkv, float* Mqk, hipStream_t s) {
  hipLaunchKernelGGL(lowrank_qk_kernel, dim3((d.H * 25 + 127) / 128), dim3(128), 0, s, W0qkv, bqkv, d.D, d.H, Mqk);
}

void launch_ofeat_weight(const Dims& d, const float* W0qkv, const float* bqkv, const float* Wol, float* UT,
                         hipStream_t s) {
  const int n = d.D * 8 * d.H;
  hipLaunchKernelGGL(ofeat_weight_kernel, dim3((n + 255) / 256), dim3(256), 0, s, W0qkv, bqkv, Wol, d.D, d.H,
                     ofeat_k(d), UT);
}

void launch_l1_basis(const Dims& d, const float* W0, const float* UT, const float* bol, const float* ln1,
                     const float* Wm, const float* bm, float* BT, float* VT, hipStream_t s) {
  hipLaunchKernelGGL(l1_basis_kernel, dim3((d.D * 32 + 255) / 256), dim3(256), 0, s, W0, UT, ofeat_k(d), bol, ln1, Wm,
                     bm, d.D, BT, VT);
}

void launch_attention(const Dims& d, const float* qkv, const float* geo, float* o, int nw, int C, hipStream_t s,
                      const float* W0qkv, const float* bqkv, const float* Mqk) {
  // wave kernels (value and channel) for dh = 64, N <= 8; W0qkv != nullptr selects the
  // fused layer-1 form (q|k|v from the input features), valid only for those kernels.
  if (C > 1 && W0qkv && Mqk && d.dh == 64 && attention_takes_features(d, C)) {
    switch (d.N) {  // layer 1, feature space (attention_feat2_kernel): o holds the o~ rows
      case 1: launch_feat<1>(d, geo, o, nw, Mqk, s); return;
      case 2: launch_feat<2>(d, geo, o, nw, Mqk, s); return;
      case 3: launch_feat<3>(d, geo, o, nw, Mqk, s); return;
      case 4: launch_feat<4>(d, geo, o, nw, Mqk, s); return;
      case 5: launch_feat<5>(d, geo, o, nw, Mqk, s); return;
      case 6: launch_feat<6>(d, geo, o, nw, Mqk, s); return;
      case 7: launch_feat<7>(d, geo, o, nw, Mqk, s); return;
      case 8: launch_feat<8>(d, geo, o, nw, Mqk, s); return;
      case 10: launch_feat<10>(d, geo, o, nw, Mqk, s); return;
      default: launch_feat<20>(d, geo, o, nw, Mqk, s); return;
    }
  }
  if (C > 1 && attention_mfma_supported(d)) {
    launch_attention_mfma(d, qkv, geo, o, nw, s, W0qkv, bqkv);
    return;
  }
  if (attention_takes_features(d, C)) {
    switch (d.N) {
      case 1: launch_wave<1>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
      case 2: launch_wave<2>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
      case 3: launch_wave<3>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
      case 4: launch_wave<4>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
      case 5: launch_wave<5>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
      case 6: launch_wave<6>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
      case 7: launch_wave<7>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
      case 8: launch_wave<8>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
      case 10: launch_wave<10>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
      default: launch_wave<20>(d, qkv, W0qkv, bqkv, Mqk, geo, o, nw, C, s); return;
    }
  }
  // channel kernel v2 needs dh <= 64 (one feature column per lane) and dh % 4 == 0;
  // PF = float4 prefetch slots >= 3 N dh / 1024, RPT = rows per thread >= N / 4
  if (C > 1 && d.dh % 4 == 0 && d.dh <= 64 && d.N <= 32) {
    const int N = d.N;
    if (N <= 4)
      launch_ch<1, 1>(d, qkv, geo, o, nw, s);
    else if (N <= 8)
      launch_ch<2, 2>(d, qkv, geo, o, nw, s);
    else if (N <= 12)
      launch_ch<3, 3>(d, qkv, geo, o, nw, s);
    else if (N <= 16)
      launch_ch<3, 4>(d, qkv, geo, o, nw, s);
    else if (N <= 20)
      launch_ch<4, 5>(d, qkv, geo, o, nw, s);
    else if (N <= 24)
      launch_ch<5, 6>(d, qkv, geo, o, nw, s);
    else
      launch_ch<6, 8>(d, qkv, geo, o, nw, s);
    return;
  }
  const AttnSmem L = attn_layout(d.N, d.dh, d.T, C);
  const size_t smem = (size_t)L.total * sizeof(float);
  const int threads = (C == 1) ? 64 : 256;
  // nn <= 4 * threads is required by the register staging of the second-order pass
  ensure_smem(attention_kernel, smem);
  hipLaunchKernelGGL(attention_kernel, dim3(nw * d.H), dim3(threads), smem, s, qkv, geo, o, d.N, C, d.H, d.dh);
}

}  // namespace dh
