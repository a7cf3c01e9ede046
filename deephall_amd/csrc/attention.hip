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
#include "dh_internal.h"
#include "device_common.h"

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

}  // namespace

void launch_attention(const Dims& d, const float* qkv, const float* geo, float* o, int nw, int C, hipStream_t s) {
  const AttnSmem L = attn_layout(d.N, d.dh, d.T, C);
  const size_t smem = (size_t)L.total * sizeof(float);
  const int threads = (C == 1) ? 64 : 256;
  // nn <= 4 * threads is required by the register staging of the second-order pass
  ensure_smem(attention_kernel, smem);
  hipLaunchKernelGGL(attention_kernel, dim3(nw * d.H), dim3(threads), smem, s, qkv, geo, o, d.N, C, d.H, d.dh);
}

}  // namespace dh
