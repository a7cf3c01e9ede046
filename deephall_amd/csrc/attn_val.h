// Self-attention of ONE (walker, head) on value rows (log psi, dh = 64; psiformer.py:44),
// with layer 1's q|k|v formed from the K = 4 input features through the folded W0 Wqkv
// (psiformer.py:51-60).  Shared by attention_val_kernel (attention.hip, o to HBM) and the
// chained layer tail's prologue (gemm_x6.hip chain_x6s_kernel: layer 1's o straight into
// its LDS planes), so both compute bit-identical outputs.
#pragma once
#include "device_common.h"

namespace dh {

// Per-lane slice of the folded layer-1 projection: column (h, lane) of q, k and v.
struct FeatW {
  float4 wq, wk, wv;
  float bq, bk, bv;
  __device__ void load(const float* W0qkv, const float* bqkv, int D, int col) {
    const int ld = 3 * D;
    wq = make_float4(W0qkv[col], W0qkv[ld + col], W0qkv[2 * ld + col], W0qkv[3 * ld + col]);
    wk = make_float4(W0qkv[D + col], W0qkv[ld + D + col], W0qkv[2 * ld + D + col], W0qkv[3 * ld + D + col]);
    wv = make_float4(W0qkv[2 * D + col], W0qkv[ld + 2 * D + col], W0qkv[2 * ld + 2 * D + col],
                     W0qkv[3 * ld + 2 * D + col]);
    bq = bqkv[col];
    bk = bqkv[D + col];
    bv = bqkv[2 * D + col];
  }
  __device__ __forceinline__ static float dot(float4 f, float4 w) {
    return fmaf(f.x, w.x, fmaf(f.y, w.y, fmaf(f.z, w.z, f.w * w.w)));
  }
};

// q|k|v rows of the N electrons of walker b at this lane's column of head h (fw)
template <int N>
__device__ __forceinline__ void feat_qkv(const FeatW& fw, const float* __restrict__ geo, int b, int n_up,
                                         float (&pq)[N], float (&pk)[N], float (&pv)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + i));
    const float4 f = make_float4(g.y, g.x * g.w, g.x * g.z, (i < n_up) ? 1.f : -1.f);
    pq[i] = FeatW::dot(f, fw.wq) + fw.bq;
    pk[i] = FeatW::dot(f, fw.wk) + fw.bk;
    pv[i] = FeatW::dot(f, fw.wv) + fw.bv;
  }
}

// One wave, lane = feature column d of the head: softmax(q k^T / 8) v for the N electrons
// of NT independent (walker, head) tasks, phase by phase so that their LDS round trips
// overlap (each task's arithmetic is the NT = 1 one).  st: NT x attn_val_floats(N) floats
// of wave-private LDS (per task q and k rows at stride 68, then the N x N weights).
// out[t][i] = o of task t, electron i, column d.
template <int N>
__host__ __device__ constexpr int attn_val_floats() { return 2 * N * 68 + N * N; }

template <int N, int NT>
__device__ __forceinline__ void attn_val_core(const float (&pq)[NT][N], const float (&pk)[NT][N],
                                              const float (&pv)[NT][N], float* st, int lane, float (&out)[NT][N]) {
  constexpr int ld = 68, nn = N * N, PER = attn_val_floats<N>();
  __builtin_amdgcn_wave_barrier();  // a previous call's readers of st (LDS ops of a wave run in order)
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < N; ++i) {
      st[t * PER + i * ld + lane] = pq[t][i];
      st[t * PER + N * ld + i * ld + lane] = pk[t][i];
    }
  __builtin_amdgcn_wave_barrier();
  for (int p = lane; p < NT * 4 * nn; p += 64) {
    const int t = p / (4 * nn), pp = p - t * (4 * nn);
    const int pair = pp >> 2, qt = pp & 3, i = pair / N, j = pair - (pair / N) * N;
    const float* x = st + t * PER + i * ld + 16 * qt;
    const float* y = st + t * PER + N * ld + j * ld + 16 * qt;
    float sdot = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float4 a = *reinterpret_cast<const float4*>(x + 4 * m);
      const float4 c = *reinterpret_cast<const float4*>(y + 4 * m);
      sdot = fmaf(a.x, c.x, fmaf(a.y, c.y, fmaf(a.z, c.z, fmaf(a.w, c.w, sdot))));
    }
    sdot += __shfl_xor(sdot, 1, 64);
    sdot += __shfl_xor(sdot, 2, 64);
    if (qt == 0) st[t * PER + 2 * N * ld + pair] = sdot * 0.125f;  // 1 / sqrt(64)
  }
  __builtin_amdgcn_wave_barrier();
  if (lane < NT * N) {  // lane = (task, row)
    const int t = lane / N, r = lane - t * N;
    float* A = st + t * PER + 2 * N * ld + r * N;
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < N; ++j) m = fmaxf(m, A[j]);
    float e[N], ssum = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      e[j] = expf(A[j] - m);
      ssum += e[j];
    }
    const float inv = 1.f / ssum;
#pragma unroll
    for (int j = 0; j < N; ++j) A[j] = e[j] * inv;
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float* A = st + t * PER + 2 * N * ld;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fmaf(A[i * N + j], pv[t][j], acc);
      out[t][i] = acc;
    }
  }
}

// Layer 1's scores straight from the input features (round 5).  With f~ = (z, x, y, spin, 1)
// and the q / k biases as the fifth rows of the folded maps, q_i = f~_i Wq~, k_j = f~_j Wk~, so
//   S_ij = q_i . k_j / sqrt(64) = f~_i^T Mqk f~_j,   Mqk = Wq~ Wk~^T / 8   (5 x 5 per head)
// — 30 FMAs per score pair from the electrons' geometry instead of staging the 64-wide q, k
// rows in LDS and forming the dots.  Mqk is formed once per parameter upload (attention.hip
// lowrank_qk_kernel, f64 sums); attn_val_core's softmax and value sums follow unchanged.
__device__ __forceinline__ void feat5(const float* __restrict__ geo, int row, bool up, float (&f)[5]) {
  const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)row);  // st ct sp cp
  f[0] = g.y;
  f[1] = g.x * g.w;
  f[2] = g.x * g.z;
  f[3] = up ? 1.f : -1.f;
  f[4] = 1.f;
}
template <int N>
__host__ __device__ constexpr int attn_feat_floats() { return N * N; }

// NT walkers b0 .. b0 + NT - 1 of one head (Mh: its 25 Mqk entries, row-major); pv: this lane's
// column of v per task and electron (feat_qkv); st: NT x attn_feat_floats(N) floats of
// wave-private LDS; out[t][i] = o of task t, electron i, column d = lane.
// geo_at(row): the (st, ct, sp cp) float4 of electron row (global memory or a staged copy)
// The softmax weights of NT walkers b0 .. b0 + NT - 1 of one head (Mh: its 25 Mqk entries,
// row-major) into st: NT x attn_feat_floats(N) floats of wave-private LDS, A[t][i][j] at
// t N^2 + i N + j.  geo_at(row): the (st, ct, sp cp) float4 of electron row (global memory
// or a staged copy)
template <int N, int NT, class GeoAt>
__device__ __forceinline__ void attn_feat_weights_g(const float (&M)[25], GeoAt geo_at, int b0, int n_up, float* st,
                                                    int lane) {
  constexpr int nn = N * N, PER = attn_feat_floats<N>();
  auto feat5g = [&](int row, bool up, float (&f)[5]) __attribute__((always_inline)) {
    const float4 g = geo_at(row);  // st ct sp cp
    f[0] = g.y;
    f[1] = g.x * g.w;
    f[2] = g.x * g.z;
    f[3] = up ? 1.f : -1.f;
    f[4] = 1.f;
  };
  __builtin_amdgcn_wave_barrier();  // a previous call's readers of st (LDS ops of a wave run in order)
  for (int p = lane; p < NT * nn; p += 64) {
    const int t = p / nn, pair = p - t * nn, i = pair / N, j = pair - (pair / N) * N;
    float fi[5], fj[5];
    feat5g((b0 + t) * N + i, i < n_up, fi);
    feat5g((b0 + t) * N + j, j < n_up, fj);
    float s = 0.f;
#pragma unroll
    for (int a = 0; a < 5; ++a) {
      float u = 0.f;
#pragma unroll
      for (int c = 0; c < 5; ++c) u = fmaf(M[5 * a + c], fj[c], u);
      s = fmaf(fi[a], u, s);
    }
    st[t * PER + pair] = s;
  }
  __builtin_amdgcn_wave_barrier();
  if (lane < NT * N) {  // lane = (task, row): softmax over j (as attn_val_core)
    const int t = lane / N, r = lane - t * N;
    float* A = st + t * PER + r * N;
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < N; ++j) m = fmaxf(m, A[j]);
    float e[N], ssum = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      e[j] = expf(A[j] - m);
      ssum += e[j];
    }
    const float inv = 1.f / ssum;
#pragma unroll
    for (int j = 0; j < N; ++j) A[j] = e[j] * inv;
  }
  __builtin_amdgcn_wave_barrier();
}

// NT walkers of one head; pv: this lane's column of v per task and electron (feat_qkv);
// out[t][i] = o of task t, electron i, column d = lane.
template <int N, int NT, class GeoAt>
__device__ __forceinline__ void attn_feat_core_g(const float (&M)[25], GeoAt geo_at, int b0, int n_up,
                                                 const float (&pv)[NT][N], float* st, int lane, float (&out)[NT][N]) {
  constexpr int PER = attn_feat_floats<N>();
  attn_feat_weights_g<N, NT>(M, geo_at, b0, n_up, st, lane);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const float* A = st + t * PER;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < N; ++j) acc = fmaf(A[i * N + j], pv[t][j], acc);
      out[t][i] = acc;
    }
  }
}

// Layer 1's attention output in feature space (round 6).  v_j = f~_j Wv~ (Wv~ = [W0 Wv; bv],
// 5 x 64 per head), so o_i = sum_j A_ij v_j = o~_i Wv~ with o~_i = sum_j A_ij f~_j: five
// numbers per (walker, electron, head) instead of 64, and o Wol = o~ (Wv~ Wol) = o~ U (the
// chain kernel's first map contracts over 32 instead of 256).  Outputs in the 8-slot per-head
// segment of an o~ row (dh_internal.h ofeat_k; slots 5..7 zero): value u of lane p = lane +
// 64 u is task t = p / (8 N), electron i = p / 8 % N, slot a = p % 8 (p < 8 N NT).
template <int N, int NT>
__host__ __device__ constexpr int attn_ofeat_regs() { return (8 * N * NT + 63) / 64; }
template <int N, int NT, class GeoAt>
__device__ __forceinline__ void attn_ofeat_core_g(const float (&M)[25], GeoAt geo_at, int b0, int n_up, float* st,
                                                  int lane, float (&out)[attn_ofeat_regs<N, NT>()]) {
  constexpr int PER = attn_feat_floats<N>();
  attn_feat_weights_g<N, NT>(M, geo_at, b0, n_up, st, lane);
#pragma unroll
  for (int u = 0; u < attn_ofeat_regs<N, NT>(); ++u) {
    const int p = lane + 64 * u, t = p / (8 * N), i = (p >> 3) % N, a = p & 7;
    float acc = 0.f;
    if (p < 8 * N * NT && a < 5) {
      const float* A = st + t * PER + i * N;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const float4 g = geo_at((b0 + t) * N + j);  // st ct sp cp
        const float f = a == 0 ? g.y : (a == 1 ? g.x * g.w : (a == 2 ? g.x * g.z : (a == 3 ? (j < n_up ? 1.f : -1.f) : 1.f)));
        acc = fmaf(A[j], f, acc);
      }
    }
    out[u] = acc;
  }
}

template <int N, int NT>
__device__ __forceinline__ void attn_feat_core(const float* __restrict__ Mh, const float* __restrict__ geo, int b0,
                                               int n_up, const float (&pv)[NT][N], float* st, int lane,
                                               float (&out)[NT][N]) {
  float M[25];
#pragma unroll
  for (int q = 0; q < 25; ++q) M[q] = Mh[q];
  attn_feat_core_g<N, NT>(
      M, [&](int row) { return *reinterpret_cast<const float4*>(geo + 4 * (size_t)row); }, b0, n_up, pv, st, lane,
      out);
}

// this lane's column of v only (feat_qkv without q and k: the scores come from Mqk)
template <int N, class GeoAt>
__device__ __forceinline__ void feat_v_g(const FeatW& fw, GeoAt geo_at, int b, int n_up, float (&pv)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float4 g = geo_at(b * N + i);
    const float4 f = make_float4(g.y, g.x * g.w, g.x * g.z, (i < n_up) ? 1.f : -1.f);
    pv[i] = FeatW::dot(f, fw.wv) + fw.bv;
  }
}
template <int N>
__device__ __forceinline__ void feat_v(const FeatW& fw, const float* __restrict__ geo, int b, int n_up, float (&pv)[N]) {
  feat_v_g<N>(fw, [&](int row) { return *reinterpret_cast<const float4*>(geo + 4 * (size_t)row); }, b, n_up, pv);
}

}  // namespace dh
