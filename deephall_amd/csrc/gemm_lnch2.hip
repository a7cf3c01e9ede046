// The fused channel layer tail (gemm_lnch.hip: psiformer.py:44-48 on the 2N + 5 channel rows)
// with TWO tiles in flight per CU, for every N.
//
//   MODE 0:  h = LN_ch(h + X W + b)            (X = o, W = Wo Wl folded)
//   MODE 1:  h = LN_ch(h + tanh_ch(h W + b))   (X = h)
//
// Why.  gemm_lnch_kernel holds a 16-electron tile's pre-LayerNorm rows in registers (16 C x 256
// f32 = 53 % of a CU's register file at N = 6), so one tile runs per CU and its epilogue (the
// residual rows, two statistics rounds, the LayerNorm stores) leaves the matrix cores idle, and
// N > 6 (C4, C5) did not fit at all.  Here a workgroup is 4 waves (one per SIMD, 64 output
// features each) and a tile EPT = 16 / S electrons, S = 2, 4, 8 "channel classes" by N, so the
// accumulators stay at 96-144 VGPRs and TWO independent workgroups share a CU: one's epilogue
// runs beside the other's k loop.
//
// MFMA layout.  v_mfma_f32_16x16x32_bf16 with the weights as the A operand (16 features) and the
// activations as B: column j = EPT s + e is electron e (0 .. EPT - 1) in channel class s, so
// MFMA m covers channels c = S m + s (m = 0 .. MH - 1, MH = ceil(C / S); columns with c >= C are
// padding whose results are discarded).  Lane (j, g) ends the k loop holding, for electron e,
// features 64 w + 16 cb + 4 g .. + 3 (cb = 0..3) of its MH channels of class s.  The channel
// algebra needs every class of a feature: the other classes of the same electron are the lanes
// j + EPT k of the 16-lane row, so a sum over classes is log2(S) DPP row_ror adds (csum) and
// the value row (class 0) reaches every class the same way.
//
// The k loop is gemm_lnch_kernel's (split-bf16 weight planes streamed L2 -> registers one column
// block ahead; the activation k-step loaded one step ahead into registers, split once into three
// bf16 planes in LDS, the image [p][16 m + j][64 B] with lnch_sw's conflict-free slot swizzle),
// the epilogue its algebra (layernorm.hip's channel rules) on the parity-split lanes, with the
// residual rows through LDS by DMA (gemm_lnch.hip LNCH_RDMA).  Same products in the same order;
// the statistics are summed in a different order (f32 rounding, not bitwise).
#include <cstdlib>

#include "dh_internal.h"
#include "device_common.h"

namespace dh {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int L2_D = 256;    // features (= K)
constexpr int L2_BK = 32;    // k per step
constexpr int L2_NWV = 4;    // waves per workgroup (one per SIMD), two workgroups per CU
constexpr int L2_RROWS = 32;  // residual chunk: 32 rows of 1 KB (2 S channels x EPT electrons)
constexpr int L2_RBUF = L2_RROWS * L2_D * 4;

// channel classes by N (accumulators MH * 16 VGPRs: N <= 6 -> 144, <= 12 -> 128, <= 24 -> 112)
__host__ __device__ constexpr int l2_classes(int N) { return N <= 6 ? 2 : N <= 12 ? 4 : 8; }
__host__ __device__ constexpr int l2_mh(int N, int S) { return (2 * N + 5 + S - 1) / S; }
__host__ __device__ constexpr int l2_stage(int N, int S) { return 3 * 16 * l2_mh(N, S) * 64; }
__host__ __device__ constexpr int l2_geo_off(int N, int S) {
  return 2 * l2_stage(N, S) > 2 * L2_RBUF ? 2 * l2_stage(N, S) : 2 * L2_RBUF;
}
__host__ __device__ constexpr int l2_gw(int N, int S) { return (16 / S + N - 1) / N + 1; }  // walkers a tile touches
__host__ __device__ constexpr int l2_smem(int N, int S) { return l2_geo_off(N, S) + l2_gw(N, S) * N * 16; }

__device__ __forceinline__ uint32_t pkbf2(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){x, y}, bf16x2));
}
__device__ __forceinline__ float lof(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hif(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ int l2_sw(int j) { return (0x78 >> (2 * ((j >> 2) & 3))) & 3; }
// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E - 1
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}
// the value of lane (j + R) mod 16 of this lane's 16-lane row (DPP row_ror:R)
template <int R>
__device__ __forceinline__ float ror(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x120 + R, 0xf, 0xf, false));
}
// sum over the S classes of an electron (lanes e + EPT k of the row), in every class's lane
template <int S>
__device__ __forceinline__ float csum(float v) {
  if constexpr (S >= 8) v += ror<2>(v);
  if constexpr (S >= 4) v += ror<4>(v);
  v += ror<8>(v);
  return v;
}

template <int N, int MODE, int S>
__global__ __launch_bounds__(L2_NWV * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_lnch2_kernel(
    const float* X, const uint16_t* __restrict__ Wp, int ldp, const float* __restrict__ bias,
    const float* __restrict__ ln, const float* __restrict__ geo, float* h, int ne) {
  constexpr int C = 2 * N + 5, T = 2 * N, EPT = 16 / S, D = L2_D, K = L2_D, BK = L2_BK, NK = K / BK;
  constexpr int MH = l2_mh(N, S), NWV = L2_NWV, NT = NWV * 64, CB = D / (16 * NWV);
  constexpr int ROWS = EPT * C;                  // activation rows per tile
  constexpr int PLANE = 16 * MH * 64;            // bytes of one bf16 plane per step
  constexpr int STAGE = 3 * PLANE;
  constexpr int NQ = (ROWS * 8 + NT - 1) / NT;   // 16-B activation pieces per thread per step
  constexpr int NR = C + T + 3;                  // second-moment statistics per electron
  constexpr int TS = NR | 1;                     // odd row stride of the totals
  static_assert(STAGE == l2_stage(N, S) && l2_smem(N, S) <= 81920, "two workgroups per CU");
  static_assert(NWV * NR * 4 * EPT * 4 + EPT * TS * 4 <= l2_geo_off(N, S), "reduction scratch");
  static_assert(CB == 4 && MH * 16 <= 144, "64 features per wave, accumulators");
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kg = lane >> 4;
  const int e0 = blockIdx.x * EPT;  // first electron of the tile
  const size_t row0 = (size_t)e0 * C;
  const int rows_valid = min(ROWS, (ne - e0) * C);

  constexpr int GW = l2_gw(N, S);
  float4* gl = reinterpret_cast<float4*>(smem + l2_geo_off(N, S));
  if (tid < GW * N) {
    const int ge = (e0 / N) * N + tid;
    gl[tid] = ge < ne ? reinterpret_cast<const float4*>(geo)[ge] : make_float4(0.f, 1.f, 0.f, 1.f);
  }
  // ---- activation pieces: piece i = tid + NT q -> tile row r = e C + c (global order), quad
  // i & 7; LDS row 16 (c / S) + EPT (c % S) + e (the MFMA column j = EPT (c % S) + e)
  const uint32_t tbytes = (uint32_t)rows_valid * D * 4;
  const auto rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X) + row0 * D, (short)0, tbytes, 0x00020000);
  int goff[NQ], loff[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int i = tid + NT * q;
    const int r = i >> 3, qq = i & 7;
    const int e = r / C, c = r - e * C;
    const int j = EPT * (c % S) + e;
    goff[q] = i < ROWS * 8 ? (r * D + 4 * qq) * 4 : 0x7fffffff;
    loff[q] = i < ROWS * 8 ? (16 * (c / S) + j) * 64 + (((qq >> 1) ^ l2_sw(j)) * 16) + (qq & 1) * 8 : -1;
  }
  auto load_a = [&](int kt, float4 (&ra)[NQ]) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      ra[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsX, goff[q], kt * BK * 4, 0));
  };
  auto split_store = [&](const float4 (&ra)[NQ], int buf) {
    char* P = smem + buf * STAGE;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (loff[q] < 0) continue;
      const float4 u = ra[q];
      const uint32_t h0 = pkbf2(u.x, u.y), h1 = pkbf2(u.z, u.w);
      const float rx = u.x - lof(h0), ry = u.y - hif(h0), rz = u.z - lof(h1), rw = u.w - hif(h1);
      const uint32_t m0 = pkbf2(rx, ry), m1 = pkbf2(rz, rw);
      const uint32_t s0 = pkbf2(rx - lof(m0), ry - hif(m0)), s1 = pkbf2(rz - lof(m1), rw - hif(m1));
      *reinterpret_cast<uint2*>(P + loff[q]) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(P + PLANE + loff[q]) = make_uint2(m0, m1);
      *reinterpret_cast<uint2*>(P + 2 * PLANE + loff[q]) = make_uint2(s0, s1);
    }
  };
  // ---- weight fragments: feature n = 16 (CB wid + cb) + l16, k = 32 kt + 8 kg
  const uint16_t* wbase = Wp + (size_t)(16 * CB * wid + l16) * K + 8 * kg;
  const size_t wplane = (size_t)ldp * K;
  auto load_w = [&](int kt, int cb, bf16x8 (&wf)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
      wf[p] = *reinterpret_cast<const bf16x8*>(wbase + p * wplane + (size_t)cb * 16 * K + kt * BK);
  };
  const int xoff = l16 * 64 + ((kg ^ l2_sw(l16)) * 16);  // + m * 16 * 64 within a plane

  f32x4 acc[MH][CB];
#pragma unroll
  for (int m = 0; m < MH; ++m)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc[m][cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  {
    float4 ra[NQ];
    bf16x8 wf[3], wn[3];
    load_a(0, ra);
    load_w(0, 0, wf);
    split_store(ra, 0);
    load_a(1, ra);
#pragma unroll 1
    for (int kt = 0; kt < NK; ++kt) {
      __syncthreads();  // planes of step kt complete; step kt - 1's buffer is free
      const char* P = smem + (kt & 1) * STAGE + xoff;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        asm volatile("" ::: "memory");  // fragments re-read per block, not held across blocks
        if (cb + 1 < CB)
          load_w(kt, cb + 1, wn);
        else if (kt + 1 < NK)
          load_w(kt + 1, 0, wn);
        bf16x8 xf[2][3];
        auto ldx = [&](int m, bf16x8 (&x)[3]) {
          x[0] = *reinterpret_cast<const bf16x8*>(P + m * 16 * 64);
          x[1] = *reinterpret_cast<const bf16x8*>(P + PLANE + m * 16 * 64);
          x[2] = *reinterpret_cast<const bf16x8*>(P + 2 * PLANE + m * 16 * 64);
        };
        ldx(0, xf[0]);
#pragma unroll
        for (int m = 0; m < MH; ++m) {
          if (m + 1 < MH) ldx(m + 1, xf[(m + 1) & 1]);  // one channel group ahead
          const bf16x8 x0 = xf[m & 1][0], x1 = xf[m & 1][1], x2 = xf[m & 1][2];
          f32x4 a = acc[m][cb];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0], x2, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[2], x0, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1], x1, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0], x1, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1], x0, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0], x0, a, 0, 0, 0);
          acc[m][cb] = a;
          if (cb == 0 && m == MH / 2 && kt + 1 < NK) {
            split_store(ra, (kt + 1) & 1);
            if (kt + 2 < NK) load_a(kt + 2, ra);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) wf[p] = wn[p];
      }
    }
  }
  __syncthreads();  // every wave is past its last plane read: the stage buffers become scratch
  const int lane_e = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));

  // ---- residual rows h by LDS-DMA (as gemm_lnch.hip LNCH_RDMA): chunk k = channel rows
  // RCH k .. RCH k + RCH - 1 (RCH = 2 S: 32 rows), chunk row q = (c - RCH k) EPT + e, 16-B
  // slot z of a row = the row's quad z ^ j (j = EPT (c % S) + e, the lane column that reads it)
  constexpr int RCH = 2 * S, NCHK = (C + RCH - 1) / RCH;
  auto rows_of = [](int k) { return EPT * (C - RCH * k < RCH ? C - RCH * k : RCH); };
  static_assert(RCH * EPT == L2_RROWS && L2_RROWS % NWV == 0 && EPT * S % NWV == 0, "DMA rows per wave");
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);
  auto rdma = [&](int k) {
    const int nrow = rows_of(k);
#pragma unroll
    for (int jj = 0; jj < L2_RROWS / NWV; ++jj) {
      const int q = wid + NWV * jj;  // wave-uniform
      if (q < nrow) {
        const int c = RCH * k + q / EPT, e = q % EPT;
        const int er = e0 + e < ne ? e : 0;
        const float* rowp = h + (row0 + (size_t)(er * C + c)) * D;
        uint32_t voff = (uint32_t)(lane_e ^ (EPT * (c % S) + e)) << 4;
        asm volatile("" : "+v"(voff));
        const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)((k & 1) * L2_RBUF + q * D * 4));
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(rowp), "s"(dst)
                     : "memory");
      }
    }
  };

  const int l16e = lane_e & 15, kge = lane_e >> 4, tide = wid * 64 + lane_e;
  const int s = l16e / EPT, el = l16e % EPT;  // channel class, tile electron
  const int E = e0 + el;
  const bool valid = E < ne;
  const int b = (valid ? E : e0) / N;
  const int nf = 16 * CB * wid + 4 * kge;  // + 16 cb
  const float4* gw = gl + (b - e0 / N) * N;
  // flow coefficient alpha_kt (layernorm.hip) of tangent t (q: electron t / 2's geometry)
  auto alpha = [](const float4& q, int t, int k) -> float {
    if ((t & 1) == 0) return k == 0 ? -q.z : (k == 1 ? q.w : 0.f);
    return k == 0 ? -(q.y * q.w) : (k == 1 ? -(q.y * q.z) : q.x);
  };
  // the value row (channel 0: class 0, m 0) in every class's lane
  auto bcast0 = [&](float v) { return csum<S>(s == 0 ? v : 0.f); };

  // pre-LN rows x_c: bias (value row), MODE 1's tanh_ch, then + h
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + nf + 16 * cb) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (s == 0) {
      acc[0][cb][0] += bv.x;
      acc[0][cb][1] += bv.y;
      acc[0][cb][2] += bv.z;
      acc[0][cb][3] += bv.w;
    }
  }
  if (MODE == 1) {
    float chain = 0.f;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float z0 = bcast0(acc[0][cb][v]);
        const float y0 = tanh_ocml(z0), d1 = 1.f - y0 * y0, d2 = -2.f * y0 * d1;
        // partial sums over this lane's tangent channels t = c - 1 (1 <= c <= T)
        float sq = 0.f, u0 = 0.f, u1 = 0.f, u2 = 0.f;
        int gi = 0;
        asm volatile("" : "+v"(gi) : "v"(y0), "v"(chain));  // geometry re-read per value (registers)
#pragma unroll
        for (int m = 0; m < MH; ++m) {
          const int t = S * m + s - 1;
          const bool tan = t >= 0 && t < T;
          const float4 q = gw[gi + (tan ? t >> 1 : 0)];
          const float zt = tan ? acc[m][cb][v] : 0.f;
          sq = fmaf(zt, zt, sq);
          u0 = fmaf(alpha(q, t, 0), zt, u0);
          u1 = fmaf(alpha(q, t, 1), zt, u1);
          u2 = fmaf(alpha(q, t, 2), zt, u2);
        }
        sq = csum<S>(sq);
        u0 = csum<S>(u0);
        u1 = csum<S>(u1);
        u2 = csum<S>(u2);
        // value row: y0; tangents: d1 z; c = T + 1 (LB): d1 x + d2 sq; T + 2 .. T + 4: d1 x + d2 u_k^2
#pragma unroll
        for (int m = 0; m < MH; ++m) {
          const int c = S * m + s;
          const float x = acc[m][cb][v];
          float y = d1 * x;
          y = c == 0 ? y0 : y;
          y = c == T + 1 ? d1 * x + d2 * sq : y;
          y = c == T + 2 ? d1 * x + d2 * (u0 * u0) : y;
          y = c == T + 3 ? d1 * x + d2 * (u1 * u1) : y;
          y = c == T + 4 ? d1 * x + d2 * (u2 * u2) : y;
          acc[m][cb][v] = y;
        }
        chain = acc[MH - 1][cb][v];
        __builtin_amdgcn_sched_barrier(0);
      }
    // materialised before the DMA blocks (gemm_lnch.hip: otherwise sunk past them, spills)
#pragma unroll
    for (int m = 0; m < MH; ++m)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) asm volatile("" : "+v"(acc[m][cb]));
  }
  rdma(0);
  if (NCHK > 1) rdma(1);
  {
    // this lane's rows in a chunk buffer: channel S (2 k + mm) + s -> chunk row (S mm + s) EPT + e
    const char* const rb0 = smem + (s * EPT + el) * D * 4;
    int rsl[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) rsl[cb] = 16 * ((4 * CB * wid + 4 * cb + kge) ^ l16e);
#pragma unroll
    for (int k = 0; k < NCHK; ++k) {
      // chunk k landed = at most chunk k + 1's DMAs outstanding; the last chunk is short
      // (rows_of), and a wave may issue one more than NWV-th of it: the floor is safe for all
      if (k + 1 < NCHK)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(rows_of(k + 1) / NWV) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#pragma unroll
      for (int mm = 0; mm < 2; ++mm) {
        const int m = 2 * k + mm;
        if (m < MH) {
          const bool ok = S * m + s < C;
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) {
            const float4 r = ok ? *reinterpret_cast<const float4*>(rb0 + (k & 1) * L2_RBUF + mm * S * EPT * D * 4 +
                                                                   rsl[cb])
                                : make_float4(0.f, 0.f, 0.f, 0.f);
            f32x4& a = acc[m][cb];
            a[0] = r.x + a[0];
            a[1] = r.y + a[1];
            a[2] = r.z + a[2];
            a[3] = r.w + a[3];
            asm volatile("" : "+v"(a));
          }
        }
      }
      if (k + 2 < NCHK) {
        __syncthreads();  // every wave is done with buffer k & 1
        rdma(k + 2);
      }
    }
    __syncthreads();  // the chunk buffers become the statistics scratch
  }

  // statistics: each holder lane writes its partial sum (16 features) of a statistic into
  // red[wave][stat][lane row g][electron e]; the total sums the 4 waves x 4 lane rows
  float* red = reinterpret_cast<float*>(smem);  // [NWV][NR][4][EPT] partial sums
  float* tot = red + NWV * NR * 4 * EPT;         // [EPT][TS] totals
  auto cb_sum = [&](const f32x4 (&a)[CB]) {
    float r = 0.f;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) r += (a[cb][0] + a[cb][1]) + (a[cb][2] + a[cb][3]);
    return r;
  };
  auto put = [&](int NS, int j, float v) {
    red[((wid * NS + j) * 4 + kge) * EPT + el] = v;
    __builtin_amdgcn_sched_barrier(0);
  };
  auto total = [&](int NS) {
    __syncthreads();
    for (int i = tide; i < NS * EPT; i += NT) {
      const int j = i / EPT, e = i - j * EPT;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w)
#pragma unroll
        for (int g = 0; g < 4; ++g) t += red[((w * NS + j) * 4 + g) * EPT + e];
      tot[e * TS + j] = t * (1.f / D);
    }
    __syncthreads();
  };
  const float* mt = tot + el * TS;
  // channel means: stat c, held by class c % S at m = c / S
  static_for<0, MH>([&](auto M_) {
    constexpr int m = decltype(M_)::value;
    if (S * m + s < C) put(C, S * m + s, cb_sum(acc[m]));
  });
  total(C);
  static_for<0, MH>([&](auto M_) {
    constexpr int m = decltype(M_)::value;
    const float mu = S * m + s < C ? mt[S * m + s] : 0.f;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[m][cb][v] -= mu;
    __builtin_amdgcn_sched_barrier(0);
  });
  // flow vector u_k of block cb: this lane's tangents, summed over the classes
  auto flow = [&](int k, int cb) {
    f32x4 r = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < MH; ++m) {
      const int t = S * m + s - 1;
      const bool tan = t >= 0 && t < T;
      const float a = tan ? alpha(gw[tan ? t >> 1 : 0], t, k) : 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) r[v] = fmaf(a, acc[m][cb][v], r[v]);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) r[v] = csum<S>(r[v]);
    return r;
  };
  auto dot4 = [](const f32x4& x, const f32x4& y) { return (x[0] * y[0] + x[1] * y[1]) + (x[2] * y[2] + x[3] * y[3]); };
  auto z0of = [&](int cb) {  // the (centred) value row of block cb
    f32x4 r;
#pragma unroll
    for (int v = 0; v < 4; ++v) r[v] = bcast0(acc[0][cb][v]);
    return r;
  };
  // p_c = <z0 z_c> (stat c), q_t = <z_t^2> (stat C + t, channel 1 + t), uu_k = <u_k^2> (stat
  // C + T + k, written by the class-0 lanes)
  {
    f32x4 z0[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) z0[cb] = z0of(cb);
    static_for<0, MH>([&](auto M_) {
      constexpr int m = decltype(M_)::value;
      const int c = S * m + s;
      float p = 0.f, q = 0.f;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        p += dot4(z0[cb], acc[m][cb]);
        q += dot4(acc[m][cb], acc[m][cb]);
      }
      if (c < C) put(NR, c, p);
      if (c >= 1 && c <= T) put(NR, C + c - 1, q);
    });
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float uu = 0.f;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const f32x4 u = flow(k, cb);
      uu += dot4(u, u);
    }
    if (s == 0) put(NR, C + T + k, uu);
  }
  total(NR);
  const float sc = 1.f / sqrtf(mt[0] + 1e-5f), s2 = sc * sc;
  float cl = 0.f, au0 = 0.f, au1 = 0.f, au2 = 0.f;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const float a = s2 * mt[1 + t];
    cl += 3.f * a * a - s2 * mt[C + t];
    const float4 q = gw[t >> 1];
    au0 = fmaf(alpha(q, t, 0), a, au0);
    au1 = fmaf(alpha(q, t, 1), a, au1);
    au2 = fmaf(alpha(q, t, 2), a, au2);
  }
  const float cs0 = 3.f * au0 * au0 - s2 * mt[C + T], cs1 = 3.f * au1 * au1 - s2 * mt[C + T + 1],
              cs2 = 3.f * au2 * au2 - s2 * mt[C + T + 2];
  const float aL = s2 * mt[1 + T];
  char* const htile = reinterpret_cast<char*>(h + row0 * D);
  const uint32_t hv = (uint32_t)(((valid ? el : 0) * C * D + nf) * 4);
  auto sth = [&](int c, int cb, float4 val) {
    uint32_t o = hv + (uint32_t)((c * D + 16 * cb) * 4);
    asm volatile("" : "+v"(o));
    if (valid) *reinterpret_cast<float4*>(htile + o) = val;
  };
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const float4 gv = *reinterpret_cast<const float4*>(ln + nf + 16 * cb);
    const float4 bb = *reinterpret_cast<const float4*>(ln + D + nf + 16 * cb);
    const float gg[4] = {gv.x, gv.y, gv.z, gv.w}, bq[4] = {bb.x, bb.y, bb.z, bb.w};
    const f32x4 z0 = z0of(cb);
    float gs[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) gs[v] = gg[v] * sc;
    // sat = sum_t a_t z_t over every class
    f32x4 sat = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < MH; ++m) {
      const int c = S * m + s;
      const float at = (c >= 1 && c <= T) ? s2 * mt[c] : 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) sat[v] = fmaf(at, acc[m][cb][v], sat[v]);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) sat[v] = csum<S>(sat[v]);
    const f32x4 uk0 = flow(0, cb), uk1 = flow(1, cb), uk2 = flow(2, cb);
#pragma unroll
    for (int m = 0; m < MH; ++m) {
      const int c = S * m + s;
      const int cc = c < C ? c : 0;
      const float at = s2 * mt[cc];
      const int k = c - T - 2;  // flow index of c = T + 2 + k
      const float auk = k == 0 ? au0 : k == 1 ? au1 : au2, csk = k == 0 ? cs0 : k == 1 ? cs1 : cs2;
      float y[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float x = acc[m][cb][v];
        const float ukv = k == 0 ? uk0[v] : k == 1 ? uk1[v] : uk2[v];
        float o = gs[v] * (x - at * z0[v]);  // tangents
        o = c == 0 ? gg[v] * (sc * z0[v]) + bq[v] : o;
        o = c == T + 1 ? gs[v] * (x - aL * z0[v] - 2.f * sat[v] + cl * z0[v]) : o;
        o = (k >= 0 && k < 3) ? gs[v] * (x - at * z0[v] - 2.f * auk * ukv + csk * z0[v]) : o;
        y[v] = o;
      }
      if (c < C) sth(c, cb, make_float4(y[0], y[1], y[2], y[3]));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

template <int N>
void launch_lnch2_n(const float* X, const uint16_t* Wp, int ldp, const float* bias, const float* ln, const float* geo,
                    float* h, int ne, int mode, hipStream_t s) {
  constexpr int S = l2_classes(N), EPT = 16 / S;
  const size_t smem = l2_smem(N, S);
  const int grid = (ne + EPT - 1) / EPT;
  if (mode == 0) {
    ensure_smem(gemm_lnch2_kernel<N, 0, S>, smem);
    hipLaunchKernelGGL((gemm_lnch2_kernel<N, 0, S>), dim3(grid), dim3(L2_NWV * 64), smem, s, X, Wp, ldp, bias, ln, geo,
                       h, ne);
  } else {
    ensure_smem(gemm_lnch2_kernel<N, 1, S>, smem);
    hipLaunchKernelGGL((gemm_lnch2_kernel<N, 1, S>), dim3(grid), dim3(L2_NWV * 64), smem, s, X, Wp, ldp, bias, ln, geo,
                       h, ne);
  }
}

}  // namespace

// instantiated for N <= 12 and N = 16, 20, 24 (C4: 10, C5: 20); other N keep the two-kernel form
bool gemm_lnch2_supported(int N) { return (N >= 1 && N <= 12) || N == 16 || N == 20 || N == 24; }

void launch_gemm_lnch2(int N, const float* X, const uint16_t* Wp, int ldp, const float* bias, const float* ln,
                       const float* geo, float* h, int ne, int mode, hipStream_t s) {
  switch (N) {
#define L2CASE(n) \
  case n: launch_lnch2_n<n>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s); return;
    L2CASE(1) L2CASE(2) L2CASE(3) L2CASE(4) L2CASE(5) L2CASE(6) L2CASE(7) L2CASE(8) L2CASE(9) L2CASE(10)
    L2CASE(11) L2CASE(12) L2CASE(16) L2CASE(20) L2CASE(24)
#undef L2CASE
    default: return;
  }
}

}  // namespace dh
