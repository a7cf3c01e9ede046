// Channel self-attention on the matrix cores (exact f32: v_mfma_f32_16x16x4_f32), for
// the large-N systems (BASELINE.json C4 / C5: N = 10, 20).  Same forward-mode rules as
// attention.hip (header there), psiformer.py:44:
//
//   S_t  = s (q_t k0^T + q0 k_t^T)      Sbar_t = S_t - <S_t>_A0     A_t = A0 * Sbar_t
//   o_t  = A_t v0 + A0 v_t,  o_L = A_L v0 + A0 v_L + 2 sum_t A_t v_t,
//   o_Sk = A_Sk v0 + A0 v_Sk + 2 Au_k Vu_k, ...
//
// One 256-thread workgroup per (walker, head); every channel's N x N score matrix and
// N x 64 output are 16 x 16 MFMA tiles (N padded to NP = 16 NB):
//   scores:  NB = 2: one tile per wave (K = 64 per product);  NB = 1: one tile, the K
//            range split over the 4 waves (partials summed in the elementwise phase);
//   outputs: wave w owns feature columns 16w..16w+15 of every row tile;
//   [A_t | A0] x [v0 ; v_t] is ONE accumulation (K = 2 round_up(N, 4)), and the running
//   sums sum_t q_t k_t^T (accS) and sum_t A_t v_t (OL) stay in MFMA accumulators.
// K-permuted fragments: for a 64-wide product lane (row, kq = lane >> 4) takes
// k = 16 kq + ks at k-step ks, so its 16 operands are contiguous (4 ds_read_b128, rows of
// stride 68 floats: the 16 lanes of a read pass hit distinct banks); the outputs' K = j
// is permuted the same way (k = KQ kq + ks).
// Per channel: the q|k|v rows arrive through registers (prefetched one channel ahead) into
// a double-buffered LDS set; three barriers (scores -> elementwise -> outputs).  The flow
// sums Qu_k, Ku_k, Vu_k (N x 64 each) and the elementwise accumulators (T2, SuB_k, Au_k)
// are spread over the threads' registers and written to LDS for the three flow channels.
#include <cstdlib>

#include "dh_internal.h"
#include "device_common.h"

namespace dh {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int N>
struct MAttn {
  static constexpr int NB = (N + 15) / 16, NP = 16 * NB, LD = 68, LDA = NP + 4;
  static constexpr int T = 2 * N, C = 2 * N + 5, dh = 64;
  static constexpr int KP = (N + 3) & ~3, KQ = KP / 4;  // output K (= j) padded to 4, per lane quarter
  static constexpr int JU = (N + 7) / 8;                // elementwise: 8 threads per row, JU columns each
  static constexpr int NU = (N * dh + 255) / 256;       // flow sums: elements per thread and matrix
  static constexpr int NSLOT = (3 * N * 16 + 255) / 256;  // float4 prefetch slots per thread
  // q | k | v rows of one channel: N, N and KP rows (v's rows N..KP-1 zero).  MFMA tiles of q
  // and k read rows up to NP - 1, i.e. into the next array: finite or not, those rows only
  // reach score entries (i or j >= N) that are never used.
  static constexpr int SET = (2 * N + KP) * LD;
  static constexpr int SPW = 16 * 17;                   // NB = 1: per-wave partial tile
  static constexpr int SPSZ = NB == 1 ? 4 * SPW : NP * (NP + 1);
  // LDS offsets (floats); A0 / AT / AU are N x LDA (columns N..KP-1 zero; tile rows past N
  // read the next array, like q / k above)
  static constexpr int oS0 = 0, oB1 = SET, oB2 = 2 * SET, oA0 = 3 * SET, oAT = oA0 + N * LDA, oAU = oAT + N * LDA;
  static constexpr int oSP = oAU + N * LDA, oAL = oSP + SPSZ, TOTAL = oAL + 3 * T;
};

// Input-feature channel c of electron i (layer 1, FEAT): [z, x, y, spin] of psiformer.py:51-60
// and their channel seeds (input.hip), from the geometry g = (st, ct, sp, cp).
template <int T>
__device__ __forceinline__ f4v feat_channel(int c, int i, float4 g, float spin) {
  const float st = g.x, ct = g.y, sp = g.z, cp = g.w;
  if (c == 0) return f4v{ct, st * cp, st * sp, spin};
  if (c <= T) {
    const int t = c - 1;
    if ((t >> 1) != i) return f4v{0.f, 0.f, 0.f, 0.f};
    return ((t & 1) == 0) ? f4v{-st, ct * cp, ct * sp, 0.f} : f4v{0.f, -sp, cp, 0.f};
  }
  const float rz = ct, rx = st * cp, ry = st * sp;
  if (c == T + 1) return f4v{-2.f * rz, -2.f * rx, -2.f * ry, 0.f};
  const int k = c - T - 2;  // rotation flow about axis k (0:x 1:y 2:z)
  return f4v{(k == 2) ? 0.f : -rz, (k == 0) ? 0.f : -rx, (k == 1) ? 0.f : -ry, 0.f};
}

// FEAT (layer 1): the q|k|v rows are formed from the K = 4 input features and the folded
// W0 Wqkv (+ the bias on the value channel) in the prefetch, instead of read from memory.
#ifndef ATTN_MFMA_LBAR  // A/B knob: the barriers wait for LDS only (1); __syncthreads' vmcnt(0) drained the
#define ATTN_MFMA_LBAR 1  // next channels' q|k|v prefetch at every one of them (0)
#endif
__device__ __forceinline__ void mbar() {
#if ATTN_MFMA_LBAR
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#else
  __syncthreads();
#endif
}

#ifndef AMF_WPE10  // waves per SIMD targeted at N <= 10 / N = 20 (0 = the compiler's choice; 4 at N = 10: 128 VGPRs, no spill, r06 v30)
#define AMF_WPE10 4
#endif
#ifndef AMF_WPE20
#define AMF_WPE20 0
#endif
template <int N, bool FEAT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(N <= 10 ? (AMF_WPE10 ? AMF_WPE10 : 1) : (AMF_WPE20 ? AMF_WPE20 : 1)))) void attention_mfma_kernel(const float* __restrict__ qkv,
                                                             const float* __restrict__ geo, float* __restrict__ o,
                                                             int H, const float* __restrict__ W0qkv,
                                                             const float* __restrict__ bqkv, int n_up) {
  using L = MAttn<N>;
  constexpr int NB = L::NB, NP = L::NP, LD = L::LD, LDA = L::LDA, T = L::T, C = L::C, KQ = L::KQ, JU = L::JU,
                NU = L::NU, NSLOT = L::NSLOT;
  extern __shared__ float sm[];
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, kq = lane >> 4;
  const int D = H * 64;
  const float scale = 0.125f;  // 1 / sqrt(64)
  float* A0 = sm + L::oA0;
  float* AT = sm + L::oAT;
  float* AU = sm + L::oAU;
  float* SP = sm + L::oSP;
  float* al = sm + L::oAL;

  // ---- setup: zero V pad rows of every set and the N x N arrays (pads must be 0, not stale)
  for (int e = tid; e < 3 * N * LDA; e += 256) A0[e] = 0.f;  // A0, AT, AU are contiguous
  for (int e = tid; e < 3 * (L::KP - N) * LD; e += 256) {
    const int s = e / ((L::KP - N) * LD), r = e - s * ((L::KP - N) * LD);
    sm[s * L::SET + 3 * N * LD + r] = 0.f;
  }
  if (tid < T) {
    const int i = tid >> 1;
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));  // st ct sp cp
    al[tid] = (tid & 1) ? -(g.y * g.w) : -g.z;
    al[T + tid] = (tid & 1) ? -(g.y * g.z) : g.w;
    al[2 * T + tid] = (tid & 1) ? g.x : 0.f;
  }

  // ---- q|k|v rows of channel c: prefetch into registers, commit into an LDS set
  const f4v* src = reinterpret_cast<const f4v*>(qkv);
  f4v pf[NSLOT];  // native vectors (a HIP float4 array copy would stay in scratch)
  auto prefetch = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NSLOT; ++u) {
      const int idx = tid + 256 * u;
      if (idx < 3 * N * 16) {
        const int m = idx / (N * 16), rem = idx - m * (N * 16), i = rem >> 4, q4 = rem & 15;
        if constexpr (FEAT) {
          const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));
          const f4v f = feat_channel<T>(c, i, g, i < n_up ? 1.f : -1.f);
          const int col = m * D + h * 64 + 4 * q4;
          f4v v = {0.f, 0.f, 0.f, 0.f};
          if (f[0] != 0.f || f[1] != 0.f || f[2] != 0.f || f[3] != 0.f) {
            const f4v* W = reinterpret_cast<const f4v*>(W0qkv + col);
            const f4v w0 = W[0], w1 = W[3 * D / 4], w2 = W[6 * D / 4], w3 = W[9 * D / 4];
#pragma unroll
            for (int e = 0; e < 4; ++e)  // the wave kernels' order: f.x w.x + (f.y w.y + (f.z w.z + f.w w.w))
              v[e] = fmaf(f[0], w0[e], fmaf(f[1], w1[e], fmaf(f[2], w2[e], f[3] * w3[e])));
          }
          if (c == 0) v += *reinterpret_cast<const f4v*>(bqkv + col);
          pf[u] = v;
        } else {
          pf[u] = src[((((size_t)(b * N + i) * C + c) * 3 * D) + m * D + h * 64) / 4 + q4];
        }
      }
    }
  };
  auto commit = [&](float* set) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NSLOT; ++u) {
      const int idx = tid + 256 * u;
      if (idx < 3 * N * 16) {
        const int m = idx / (N * 16), rem = idx - m * (N * 16), i = rem >> 4, q4 = rem & 15;
        *reinterpret_cast<f4v*>(set + m * N * LD + i * LD + 4 * q4) = pf[u];
      }
    }
  };
  auto bufof = [&](int c) __attribute__((always_inline)) { return sm + ((c & 1) ? L::oB1 : L::oB2); };

  // ---- MFMA building blocks
  // 64-wide product rows A[arow] . B[brow] over this wave's k-steps
  auto dot64 = [&](const float* Am, const float* Bm, int arow, int brow, f4v acc) __attribute__((always_inline)) {
    const float* a = Am + arow * LD + 16 * kq;
    const float* bb = Bm + brow * LD + 16 * kq;
    if constexpr (NB == 1) {  // k-steps 4w .. 4w+3
      const float4 av = *reinterpret_cast<const float4*>(a + 4 * w);
      const float4 bv = *reinterpret_cast<const float4*>(bb + 4 * w);
      acc = mfma4(av.x, bv.x, acc);
      acc = mfma4(av.y, bv.y, acc);
      acc = mfma4(av.z, bv.z, acc);
      acc = mfma4(av.w, bv.w, acc);
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float4 av = *reinterpret_cast<const float4*>(a + 4 * m);
        const float4 bv = *reinterpret_cast<const float4*>(bb + 4 * m);
        acc = mfma4(av.x, bv.x, acc);
        acc = mfma4(av.y, bv.y, acc);
        acc = mfma4(av.z, bv.z, acc);
        acc = mfma4(av.w, bv.w, acc);
      }
    }
    return acc;
  };
  const int tI = NB == 1 ? 0 : (w >> 1), tJ = NB == 1 ? 0 : (w & 1);  // this wave's score tile
  const int arow = 16 * tI + r16, brow = 16 * tJ + r16;
  auto store_scores = [&](f4v acc) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * kq + r;
      if constexpr (NB == 1)
        SP[w * L::SPW + i * 17 + r16] = scale * acc[r];
      else
        SP[(16 * tI + i) * (NP + 1) + 16 * tJ + r16] = scale * acc[r];
    }
  };
  // out tile (I, w) += X[NP x KP] (row stride LDA) . V[KP x 64] (row stride LD)
  auto outmm = [&](const float* X, const float* V, int I, f4v acc) __attribute__((always_inline)) {
    const float* a = X + (16 * I + r16) * LDA + KQ * kq;
    const float* bb = V + (KQ * kq) * LD + 16 * w + r16;
#pragma unroll
    for (int ks = 0; ks < KQ; ++ks) acc = mfma4(a[ks], bb[ks * LD], acc);
    return acc;
  };

  // elementwise phase: thread -> row i = tid >> 3, columns j = (tid & 7) + 8u
  const int ei = tid >> 3, ej = tid & 7;
  const bool erow = ei < N;
  auto score = [&](int i, int j) __attribute__((always_inline)) -> float {
    if constexpr (NB == 1)
      return (SP[i * 17 + j] + SP[L::SPW + i * 17 + j]) + (SP[2 * L::SPW + i * 17 + j] + SP[3 * L::SPW + i * 17 + j]);
    else
      return SP[i * (NP + 1) + j];
  };
  auto rowsum8 = [](float v) __attribute__((always_inline)) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    return v;
  };

  // ---- value channel: S0, softmax -> A0, o0 = A0 v0
  float* S0 = sm + L::oS0;
  prefetch(0);
  commit(S0);
  prefetch(1);
  mbar();
  {
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    acc = dot64(S0, S0 + N * LD, arow, brow, acc);
    store_scores(acc);
  }
  mbar();
  if (erow) {
    float sv[JU], mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < JU; ++u) {
      const int j = ej + 8 * u;
      sv[u] = j < N ? score(ei, j) : -INFINITY;
      mx = fmaxf(mx, sv[u]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
    float sum = 0.f;
#pragma unroll
    for (int u = 0; u < JU; ++u) {
      sv[u] = (ej + 8 * u < N) ? expf(sv[u] - mx) : 0.f;
      sum += sv[u];
    }
    const float inv = 1.f / rowsum8(sum);
#pragma unroll
    for (int u = 0; u < JU; ++u)
      if (ej + 8 * u < N) A0[ei * LDA + ej + 8 * u] = sv[u] * inv;
  }
  commit(bufof(1));  // channel 1 (its buffer is untouched so far)
  prefetch(2);
  mbar();
  float* obase = o + (size_t)b * N * C * D + h * 64 + 16 * w + r16;
  auto store_out = [&](int c, int I, f4v acc) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * I + 4 * kq + r;
      if (i < N) obase[(size_t)(i * C + c) * D] = acc[r];
    }
  };
#pragma unroll
  for (int I = 0; I < NB; ++I) {
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    acc = outmm(A0, S0 + 2 * N * LD, I, acc);
    store_out(0, I, acc);
  }

  // ---- accumulators carried over the tangent channels
  f4v accS = {0.f, 0.f, 0.f, 0.f};  // sum_t q_t k_t^T on this wave's score tile (partial K for NB = 1)
  f4v OL[NB];                        // sum_t A_t v_t on this wave's output tiles
#pragma unroll
  for (int I = 0; I < NB; ++I) OL[I] = f4v{0.f, 0.f, 0.f, 0.f};
  float T2[JU], SuB[3][JU], Au[3][JU];
#pragma unroll
  for (int u = 0; u < JU; ++u) {
    T2[u] = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) SuB[k][u] = Au[k][u] = 0.f;
  }
  float Qu[3][NU], Ku[3][NU], Vu[3][NU];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int u = 0; u < NU; ++u) Qu[k][u] = Ku[k][u] = Vu[k][u] = 0.f;

  const float* Q0 = S0;
  const float* K0 = S0 + N * LD;
  const float* V0 = S0 + 2 * N * LD;
  for (int c = 1; c < C; ++c) {
    const bool tang = c <= T, lap = c == T + 1;
    const int kf = c - T - 2;  // flow axis for c >= T + 2
    float* buf = kf >= 0 ? sm + L::oB1 : bufof(c);
    const float* QC = buf;
    const float* KC = buf + N * LD;
    const float* VC = buf + 2 * N * LD;
    float* FS = sm + L::oB2;  // flow set (Qu_k | Ku_k | Vu_k) for c >= T + 2
    mbar();  // B1: channel c committed (and, for a flow channel, its flow set)
    // phase 1: scores
    {
      f4v acc = {0.f, 0.f, 0.f, 0.f};
      acc = dot64(QC, K0, arow, brow, acc);
      acc = dot64(Q0, KC, arow, brow, acc);
      if (tang) {
        accS = dot64(QC, KC, arow, brow, accS);
      } else if (lap) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] += 2.f * accS[r];
      } else {
        f4v a2 = {0.f, 0.f, 0.f, 0.f};
        a2 = dot64(FS, FS + N * LD, arow, brow, a2);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] += 2.f * a2[r];
      }
      store_scores(acc);
    }
    mbar();  // B2
    // phase 2: softmax derivative -> AT; accumulators
    if (erow) {
      float sv[JU], pv[JU], a0[JU], m1 = 0.f, m2 = 0.f;
#pragma unroll
      for (int u = 0; u < JU; ++u) {
        const int j = ej + 8 * u;
        const bool ok = j < N;
        sv[u] = ok ? score(ei, j) : 0.f;
        a0[u] = ok ? A0[ei * LDA + j] : 0.f;
        const float sbk = kf == 0 ? SuB[0][u] : (kf == 1 ? SuB[1][u] : SuB[2][u]);  // no dynamic register index
        pv[u] = tang ? 0.f : (lap ? T2[u] : sbk * sbk);
        m1 = fmaf(a0[u], sv[u], m1);
        m2 = fmaf(a0[u], pv[u], m2);
      }
      m1 = rowsum8(m1);
      if (!tang) m2 = rowsum8(m2);
      const int t = c - 1;
      const float a_0 = tang ? al[t] : 0.f, a_1 = tang ? al[T + t] : 0.f, a_2 = tang ? al[2 * T + t] : 0.f;
#pragma unroll
      for (int u = 0; u < JU; ++u) {
        const int j = ej + 8 * u;
        if (j >= N) continue;
        float at;
        if (tang) {
          const float sb = sv[u] - m1;
          at = a0[u] * sb;
          T2[u] = fmaf(sb, sb, T2[u]);
          SuB[0][u] = fmaf(a_0, sb, SuB[0][u]);
          SuB[1][u] = fmaf(a_1, sb, SuB[1][u]);
          SuB[2][u] = fmaf(a_2, sb, SuB[2][u]);
          Au[0][u] = fmaf(a_0, at, Au[0][u]);
          Au[1][u] = fmaf(a_1, at, Au[1][u]);
          Au[2][u] = fmaf(a_2, at, Au[2][u]);
        } else {
          at = a0[u] * ((sv[u] - m1) + (pv[u] - m2));
        }
        AT[ei * LDA + j] = at;
      }
    }
    if (tang) {  // flow sums Qu_k += alpha_kt q_t (and k, v), thread-owned elements
      const int t = c - 1;
      const float a_0 = al[t], a_1 = al[T + t], a_2 = al[2 * T + t];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int e = tid + 256 * u, i = e >> 6, d = e & 63;
        if (i < N) {
          const float q = QC[i * LD + d], k = KC[i * LD + d], v = VC[i * LD + d];
          Qu[0][u] = fmaf(a_0, q, Qu[0][u]);
          Qu[1][u] = fmaf(a_1, q, Qu[1][u]);
          Qu[2][u] = fmaf(a_2, q, Qu[2][u]);
          Ku[0][u] = fmaf(a_0, k, Ku[0][u]);
          Ku[1][u] = fmaf(a_1, k, Ku[1][u]);
          Ku[2][u] = fmaf(a_2, k, Ku[2][u]);
          Vu[0][u] = fmaf(a_0, v, Vu[0][u]);
          Vu[1][u] = fmaf(a_1, v, Vu[1][u]);
          Vu[2][u] = fmaf(a_2, v, Vu[2][u]);
        }
      }
    }
    mbar();  // B3: AT complete
    // the next channel's rows into the other buffer (its last readers finished before B1)
    const bool next_flow = c + 1 >= T + 2;
    if (c + 1 < C && !next_flow) {
      commit(bufof(c + 1));
      if (c + 2 < C) prefetch(c + 2);
    }
    // phase 3: outputs
#pragma unroll
    for (int I = 0; I < NB; ++I) {
      f4v acc = {0.f, 0.f, 0.f, 0.f};
      acc = outmm(AT, V0, I, acc);
      acc = outmm(A0, VC, I, acc);
      if (tang) {
        OL[I] = outmm(AT, VC, I, OL[I]);
      } else if (lap) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] += 2.f * OL[I][r];
      } else {
        f4v a2 = {0.f, 0.f, 0.f, 0.f};
        a2 = outmm(AU, FS + 2 * N * LD, I, a2);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] += 2.f * a2[r];
      }
      store_out(c, I, acc);
    }
    if (c + 1 < C && next_flow) {
      // flow channel k = c + 1 - T - 2: single-buffered (B1 <- its rows, B2 <- the flow set)
      const int k = c + 1 - T - 2;
      mbar();  // B4: every reader of B1 / B2 / AU is done
      commit(sm + L::oB1);
      if (c + 2 < C) prefetch(c + 2);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int e = tid + 256 * u, i = e >> 6, d = e & 63;
        if (i < N) {
          const float q = k == 0 ? Qu[0][u] : (k == 1 ? Qu[1][u] : Qu[2][u]);
          const float kk = k == 0 ? Ku[0][u] : (k == 1 ? Ku[1][u] : Ku[2][u]);
          const float v = k == 0 ? Vu[0][u] : (k == 1 ? Vu[1][u] : Vu[2][u]);
          FS[i * LD + d] = q;
          FS[N * LD + i * LD + d] = kk;
          FS[2 * N * LD + i * LD + d] = v;
        }
      }
      if (erow) {
#pragma unroll
        for (int u = 0; u < JU; ++u) {
          const int j = ej + 8 * u;
          if (j < N) AU[ei * LDA + j] = k == 0 ? Au[0][u] : (k == 1 ? Au[1][u] : Au[2][u]);
        }
      }
    }
  }
}

template <int N>
void launch_mfma(const Dims& d, const float* qkv, const float* geo, float* o, int nw, hipStream_t s,
                 const float* W0qkv, const float* bqkv) {
  const size_t smem = (size_t)MAttn<N>::TOTAL * sizeof(float);
  auto go = [&](auto kern) {
    ensure_smem(kern, smem);
    hipLaunchKernelGGL(kern, dim3(nw * d.H), dim3(256), smem, s, qkv, geo, o, d.H, W0qkv, bqkv, d.n_up);
  };
  if (W0qkv)
    go(attention_mfma_kernel<N, true>);
  else
    go(attention_mfma_kernel<N, false>);
}

}  // namespace

bool attention_mfma_supported(const Dims& d) { return d.dh == 64 && (d.N == 10 || d.N == 20); }

void launch_attention_mfma(const Dims& d, const float* qkv, const float* geo, float* o, int nw, hipStream_t s,
                           const float* W0qkv, const float* bqkv) {
  switch (d.N) {
    case 10: launch_mfma<10>(d, qkv, geo, o, nw, s, W0qkv, bqkv); return;
    default: launch_mfma<20>(d, qkv, geo, o, nw, s, W0qkv, bqkv); return;
  }
}

}  // namespace dh
