// Split-bf16 GEMM ("x6") on CDNA4 matrix cores: f32-accurate products at bf16 MFMA rate.
//
//   Y[r][n] = sum_k X[r][k] W[k][n]  + (r % C == 0 ? bias[n] : 0)  + (R ? R[r][n] : 0)
//
// Same contract as gemm_nt_kernel (gemm.hip); used for the channel rows of the local
// energy (all 2N+5 channels of every linear map, psiformer.py:42-47, blocks.py:29-35).
//
// Numerics.  Every f32 operand is split exactly into three bf16 terms, a = a0 + a1 + a2
// (round-to-nearest at each step: a0 = bf16(a), a1 = bf16(a - a0), a2 = a - a0 - a1,
// which has at most 8 significant bits and is therefore exact in bf16), with
// |a1| <= 2^-8 |a|, |a2| <= 2^-16 |a|.  The product is formed from the six terms
// larger than 2^-24 |a b|:
//     a b ~= a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0)
// The three dropped terms (a1 b2, a2 b1, a2 b2) are <= 2^-24 |a b| together, i.e. at
// the f32 unit roundoff; v_mfma_f32_32x32x16_bf16 multiplies bf16 exactly and
// accumulates in f32, so the result carries the error of an f32 GEMM (measured in
// tests/test_gpu_kernels.py against float64 next to the f32-MFMA kernel).  Cost: 6 bf16
// MFMAs (6 x 32 cycles) per 32x32x16 block against 8 f32 MFMAs (8 x 64 cycles):
// 2.67x the f32 matrix rate at equal accuracy.
//
// Operands.  The weight is split once per dh_set_params into three bf16 planes
// Wp[p][n][k] (n padded; launch_split_planes).  The activation tile is staged as f32
// by LDS-DMA (as gemm_nt_kernel: 128-B rows, 16-B slots XOR-swizzled by (row>>1)&7) and
// split in registers by the one wave that consumes it: wave w owns rows 32w..32w+31 of
// the tile and all BN = 32*TN columns, so every activation element is split exactly
// once.  B planes are staged by LDS-DMA into [plane][BN][64 B] images, 16-B slots
// swizzled by (row>>2)&3 (16 lanes of a ds_read_b128 pass hit 16 distinct bank groups).
#include <cstdlib>
#include <type_traits>

#include "attn_val.h"
#include "dh_internal.h"
#include "device_common.h"

#ifndef X6M_BIAS1  // A/B knob: gemm_x6m's epilogue bias loads ahead of its stores (1) or between them (0)
#define X6M_BIAS1 1
#endif
#ifndef CHAIN_P3B  // A/B knob: P3 bias loads hoisted ahead of the stores (1) or between them (0)
#define CHAIN_P3B 1
#endif
#ifndef CHAIN_TANH_EXP  // A/B knob: the chain kernel's tanh as 1 - 2 / (exp(2x) + 1) (2 transcendentals + 3 VALU)
#define CHAIN_TANH_EXP 0
#endif
#ifndef CHAIN_LN1P  // A/B knob: the chain kernel's LayerNorms in one statistics round (fast variance)
#define CHAIN_LN1P 1
#endif
#ifndef CHAIN_P3T  // A/B knob: P3 MFMAs with the operands swapped (accumulator = tile row x 32 columns,
#define CHAIN_P3T 1  // one register = two 128-B row segments: full-rate dword stores) instead of float4
#endif               // stores of 32 rows x 32 B per instruction (round 5)
#ifndef CHAIN_LBAR  // A/B knob: the chain kernel's barriers wait for LDS only (lgkmcnt(0) + s_barrier) instead
#define CHAIN_LBAR 1  // of __syncthreads' vmcnt(0), which also waited for the next GEMM's weight prefetch (round 5)
#endif
#ifndef X6M_NT  // A/B knob: gemm_x6m's output tiles stored nontemporal (streaming) instead of plain stores
#define X6M_NT 0
#endif
#ifndef CHAIN_STAMP  // diagnostic builds only (tools/chain_stamp.py): per-tile phase stamps of chain_x6s
#define CHAIN_STAMP 0
#endif

namespace dh {

#if CHAIN_STAMP
// [2][CHAIN_STAMP_WG][CHAIN_NSTAMP]: slot 1 = layer 1 with its attention (NA > 0), slot 0 = the rest
constexpr int CHAIN_STAMP_WG = 512, CHAIN_NSTAMP = 16;
__device__ unsigned long long g_chain_stamp[2 * CHAIN_STAMP_WG * CHAIN_NSTAMP];
#define CHAIN_T(i)                                                                                  \
  do {                                                                                              \
    if (threadIdx.x == 0 && blockIdx.x < CHAIN_STAMP_WG)                                            \
      g_chain_stamp[((NA > 0) * CHAIN_STAMP_WG + blockIdx.x) * CHAIN_NSTAMP + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
extern "C" int dh_debug_chain_stamps(unsigned long long* out, int n) {
  n = n < 2 * CHAIN_STAMP_WG * CHAIN_NSTAMP ? n : 2 * CHAIN_STAMP_WG * CHAIN_NSTAMP;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chain_stamp), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#else
#define CHAIN_T(i)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int X6_BK = 32;  // k per LDS stage (two 16-k MFMA chunks)

int cu_count_x6() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

// two f32 -> packed bf16 pair (one v_cvt_pk_bf16_f32, round to nearest even)
__device__ __forceinline__ uint32_t pk_bf16(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){x, y}, bf16x2));
}
__device__ __forceinline__ float lo_f(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// 8 f32 -> three bf16x8 terms (per pair: 3 v_cvt_pk_bf16_f32, 4 unpacks, 4 v_sub_f32)
__device__ __forceinline__ void split3(const float4& u, const float4& v, bf16x8& h, bf16x8& m, bf16x8& l) {
  const float a[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
  u32x4v H, Mv, Lv;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float x = a[2 * p], y = a[2 * p + 1];
    const uint32_t h2 = pk_bf16(x, y);
    const float rx = x - lo_f(h2), ry = y - hi_f(h2);
    const uint32_t m2 = pk_bf16(rx, ry);
    const float sx = rx - lo_f(m2), sy = ry - hi_f(m2);
    H[p] = h2;
    Mv[p] = m2;
    Lv[p] = pk_bf16(sx, sy);
  }
  h = __builtin_bit_cast(bf16x8, H);
  m = __builtin_bit_cast(bf16x8, Mv);
  l = __builtin_bit_cast(bf16x8, Lv);
}

// One k-tile of split-bf16 products over TN column blocks with the B fragments of block
// j + 1 read from LDS while block j's six MFMAs issue, and in the last block the NEXT
// k-tile's block-0 fragments (from Bn: that stage has landed, the barrier at the top of
// the k-tile saw to it), carried in nb.  sched_barrier keeps the reads ahead: left to
// itself the compiler sinks each block's reads to just before its MFMAs and the first
// MFMA of every block waits out the LDS latency.  The next k-tile's A split runs after
// block TN / 2 (on zeros past the last k-tile).
template <int TN, int B_PLANE>
__device__ __forceinline__ void ktile_pipelined(const char* Bs, const char* Bn, f32x16 (&acc)[TN], bf16x8 (&nb)[3],
                                                const bf16x8& c0, const bf16x8& c1, const bf16x8& c2,
                                                const float4& u, const float4& v, bf16x8& n0, bf16x8& n1,
                                                bf16x8& n2) {
  bf16x8 fb[2][3];
  auto ld = [&](const char* base, int j, bf16x8(&d)[3]) __attribute__((always_inline)) {
    d[0] = *reinterpret_cast<const bf16x8*>(base + j * 1024);
    d[1] = *reinterpret_cast<const bf16x8*>(base + B_PLANE + j * 1024);
    d[2] = *reinterpret_cast<const bf16x8*>(base + 2 * B_PLANE + j * 1024);
  };
  fb[0][0] = nb[0];
  fb[0][1] = nb[1];
  fb[0][2] = nb[2];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    if (j + 1 < TN)
      ld(Bs, j + 1, fb[(j + 1) & 1]);
    else
      ld(Bn, 0, nb);
    __builtin_amdgcn_sched_barrier(0);  // the reads stay ahead of this block's MFMAs
    const bf16x8 b0 = fb[j & 1][0], b1 = fb[j & 1][1], b2 = fb[j & 1][2];
    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c2, acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, c0, acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, c1, acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c1, acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, c0, acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c0, acc[j], 0, 0, 0);
    if (j == TN / 2) split3(u, v, n0, n1, n2);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One wave = 32 rows x (32*TN) columns; NW waves stacked along rows (BM = 32*NW).
template <int NW, int TN, bool HAS_R>
__global__ __launch_bounds__(NW * 64) void gemm_x6_kernel(const float* __restrict__ X, int ldx,
                                                          const uint16_t* __restrict__ Wp, int ldp,
                                                          const float* __restrict__ bias, const float* R, int ldr,
                                                          float* Y, int ldy, int rows, int ncols, int K, int C,
                                                          int ntm, int ntn) {
  constexpr int BM = 32 * NW, BN = 32 * TN, BK = X6_BK;
  constexpr int A_BYTES = BM * BK * 4, B_PLANE = BN * BK * 2, STAGE = A_BYTES + 3 * B_PLANE;
  constexpr int IA = BM / 8, IBP = BN / 16, IB = 3 * IBP;  // DMA wave-instructions (1 KiB each)
  constexpr int PER = (IA + IB + NW - 1) / NW;
  constexpr bool PREF = HAS_R && TN <= 4;  // residual prefetched into registers (wider tiles would spill)
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;

  // XCD-aware tile order (as gemm_nt_kernel): consecutive tiles of a row panel share an XCD
  const int nblk = ntm * ntn;
  int bid = blockIdx.x;
  {
    const int q = nblk / 8, r8 = nblk % 8, xcd = bid % 8, slot = bid / 8;
    bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
  }
  const int tm = bid / ntn, tn = bid % ntn;
  const int row0 = tm * BM, col0 = tn * BN;
  const size_t plane = (size_t)ldp * K;  // elements per weight plane

  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);
  auto stage = [&](int k0, int buf) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int j = wid + t * NW;  // wave-uniform
      if ((IA + IB) % NW != 0 && j >= IA + IB) break;
      const void* src;
      uint32_t dst;
      if (j < IA) {  // 8 rows x 128 B of f32 activations
        const int r = j * 8 + (lane >> 3);
        const int sl = ((lane & 7) ^ ((r >> 1) & 7)) * 4;
        src = X + (size_t)(row0 + r) * ldx + k0 + sl;
        dst = lds0 + (uint32_t)(buf * STAGE + j * 8 * BK * 4);
      } else {  // 16 rows x 64 B of one bf16 weight plane
        const int jb = j - IA, p = jb / IBP, rg = (jb % IBP) * 16;
        const int r = rg + (lane >> 2);
        const int sl = ((lane & 3) ^ ((r >> 2) & 3)) * 8;
        src = Wp + p * plane + (size_t)(col0 + r) * K + k0 + sl;
        dst = lds0 + (uint32_t)(buf * STAGE + A_BYTES + p * B_PLANE + rg * BK * 2);
      }
      dst = __builtin_amdgcn_readfirstlane(dst);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(dst)
                   : "memory");
    }
  };

  f32x16 acc[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[b][e] = 0.f;
  float rres[PREF ? TN : 1][16];

  const int nk = K / BK;
  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) stage((kt + 1) * BK, cur ^ 1);
    if (PREF && kt + 1 == nk) {  // residual loads overlap the last k-tile's MFMAs
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int c = col0 + ni * 32 + l32;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = row0 + wid * 32 + 4 * lh + (e & 3) + 8 * (e >> 2);
          rres[ni][e] = (c < ncols && r < rows) ? R[(size_t)r * ldr + c] : 0.f;
        }
      }
    }
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int ch = 0; ch < BK / 16; ++ch) {
      // A fragment: row m, k = 16 ch + 8 lh + (0..7) = logical slots 4ch + 2lh, +1
      const int m = wid * 32 + l32;
      const int s0 = 4 * ch + 2 * lh;
      const float* arow = reinterpret_cast<const float*>(As) + m * BK;
      const float4 u = *reinterpret_cast<const float4*>(arow + ((s0 ^ ((m >> 1) & 7)) * 4));
      const float4 v = *reinterpret_cast<const float4*>(arow + (((s0 + 1) ^ ((m >> 1) & 7)) * 4));
      bf16x8 a0, a1, a2;
      split3(u, v, a0, a1, a2);
      const int sb = 2 * ch + lh;  // B fragment: k = 16 ch + 8 lh + (0..7) = slot sb of a 64-B row
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = j * 32 + l32;
        const int off = n * BK * 2 + ((sb ^ ((n >> 2) & 3)) * 16);
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bs + off);
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bs + B_PLANE + off);
        const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(Bs + 2 * B_PLANE + off);
        // smallest terms first
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[j], 0, 0, 0);
      }
    }
  }

  // Epilogue. C/D map of 32x32 MFMA: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
  const int rbase = row0 + wid * 32 + 4 * lh;
  const int rm0 = (C == 1) ? 0 : rbase % C;
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) {
    const int c = col0 + ni * 32 + l32;
    if (c >= ncols) continue;
    const float bv = bias ? bias[c] : 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int off = (e & 3) + 8 * (e >> 2);
      const int r = rbase + off;
      if (r >= rows) continue;
      float v = acc[ni][e];
      if (bias) {
        bool val = true;
        if (C > 1) {
          int t = rm0 + off;
          while (t >= C) t -= C;
          val = (t == 0);
        }
        if (val) v += bv;
      }
      if (PREF) v += rres[PREF ? ni : 0][e];
      else if (HAS_R) v += R[(size_t)r * ldr + c];
      Y[(size_t)r * ldy + c] = v;
    }
  }
}

template <int NW, int TN>
void launch_x6_t(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* R, int ldr,
                 float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  constexpr int BM = 32 * NW, BN = 32 * TN;
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  const size_t smem = 2ull * (BM * X6_BK * 4 + 3 * BN * X6_BK * 2);
  if (R) {
    ensure_smem(gemm_x6_kernel<NW, TN, true>, smem);
    hipLaunchKernelGGL((gemm_x6_kernel<NW, TN, true>), dim3(ntm * ntn), dim3(NW * 64), smem, s, X, ldx, Wp, ldp, bias,
                       R, ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
  } else {
    ensure_smem(gemm_x6_kernel<NW, TN, false>, smem);
    hipLaunchKernelGGL((gemm_x6_kernel<NW, TN, false>), dim3(ntm * ntn), dim3(NW * 64), smem, s, X, ldx, Wp, ldp,
                       bias, R, ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
  }
}

// ---- big-tile form: 256 x (64*TN) tiles, 4 x 2 waves of 64 x 32*TN, BK = 16, DMA ring ----
// Intensity: per 16-k step a workgroup moves 256 x 64 B of A (f32) + BN x 96 B of B (three
// planes) for 2 x 256 x BN x 16 flops: 51 flop/B at BN = 256 (the 64-row tiles above move
// 2x the bytes per flop, which the L2 -> CU path cannot feed at bf16 MFMA rate).
// LDS images per stage: A [256][64 B], 16-B slot s of row m at s ^ ((m >> 2) & 3);
// B [plane][BN][32 B], slot h of row n at h ^ ((n >> 3) & 1)  (conflict-free b128 reads).
// Every wave issues exactly PER DMA instructions per stage (surplus slots repeat the last
// piece, an identical write), so the counted vmcnt waits are exact.
template <int TN, int STAGES>
__global__ __launch_bounds__(512) void gemm_x6b_kernel(const float* __restrict__ X, int ldx,
                                                       const uint16_t* __restrict__ Wp, int ldp,
                                                       const float* __restrict__ bias, const float* R, int ldr,
                                                       float* Y, int ldy, int rows, int ncols, int K, int C, int ntm,
                                                       int ntn) {
  constexpr int NW = 8, BM = 256, WN = 32 * TN, BN = 2 * WN, BK = 16;
  constexpr int A_BYTES = BM * BK * 4, B_PLANE = BN * BK * 2, STAGE = A_BYTES + 3 * B_PLANE;
  constexpr int IA = A_BYTES / 1024, IB = 3 * B_PLANE / 1024, PER = (IA + IB + NW - 1) / NW;
  static_assert(A_BYTES % 1024 == 0 && B_PLANE % 1024 == 0, "DMA pieces");
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int l32 = lane & 31, lh = lane >> 5;

  const int nblk = ntm * ntn;
  int bid = blockIdx.x;
  {
    const int q = nblk / 8, r8 = nblk % 8, xcd = bid % 8, slot = bid / 8;
    bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
  }
  const int tm = bid / ntn, tn = bid % ntn;
  const int row0 = tm * BM, col0 = tn * BN;
  const size_t plane = (size_t)ldp * K;
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);

  auto stage = [&](int k0, int buf) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      int j = wid + t * NW;
      if (j >= IA + IB) j = IA + IB - 1;  // wave-uniform: repeat the last piece
      const void* src;
      uint32_t dst;
      if (j < IA) {  // 16 rows x 64 B of f32 activations
        const int r = j * 16 + (lane >> 2);
        const int sl = ((lane & 3) ^ ((r >> 2) & 3)) * 4;
        src = X + (size_t)(row0 + r) * ldx + k0 + sl;
        dst = lds0 + (uint32_t)(buf * STAGE + j * 1024);
      } else {  // 32 rows x 32 B of one weight plane
        const int jb = j - IA, p = jb / (B_PLANE / 1024), rg = (jb % (B_PLANE / 1024)) * 32;
        const int r = rg + (lane >> 1);
        const int sl = ((lane & 1) ^ ((r >> 3) & 1)) * 8;
        src = Wp + p * plane + (size_t)(col0 + r) * K + k0 + sl;
        dst = lds0 + (uint32_t)(buf * STAGE + A_BYTES + p * B_PLANE + rg * 32);
      }
      dst = __builtin_amdgcn_readfirstlane(dst);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(dst)
                   : "memory");
    }
  };

  f32x16 acc[2][TN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = K / BK;
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < nk) stage(t * BK, t);
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (STAGES == 3 && kt + 1 < nk)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + STAGES - 1 < nk) {
      int nb = cur + STAGES - 1;
      if (nb >= STAGES) nb -= STAGES;
      stage((kt + STAGES - 1) * BK, nb);
    }
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
    if (++cur == STAGES) cur = 0;
    bf16x8 a0[2], a1[2], a2[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // A fragment: row m, k = 8 lh + (0..7) = slots 2lh, 2lh+1
      const int m = wm * 64 + i * 32 + l32;
      const float* arow = reinterpret_cast<const float*>(As) + m * BK;
      const float4 u = *reinterpret_cast<const float4*>(arow + (((2 * lh) ^ ((m >> 2) & 3)) * 4));
      const float4 v = *reinterpret_cast<const float4*>(arow + (((2 * lh + 1) ^ ((m >> 2) & 3)) * 4));
      split3(u, v, a0[i], a1[i], a2[i]);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = wn * WN + j * 32 + l32;
      const int off = n * 32 + ((lh ^ ((n >> 3) & 1)) * 16);
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bs + off);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bs + B_PLANE + off);
      const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(Bs + 2 * B_PLANE + off);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2[i], b0, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[i], b2, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[i], b1, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[i], b0, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[i], b1, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[i], b0, acc[i][j], 0, 0, 0);
      }
    }
  }

#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rbase = row0 + wm * 64 + i * 32 + 4 * lh;
    const int rm0 = (C == 1) ? 0 : rbase % C;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int c = col0 + wn * WN + j * 32 + l32;
      if (c >= ncols) continue;
      const float bv = bias ? bias[c] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int off = (e & 3) + 8 * (e >> 2);
        const int r = rbase + off;
        if (r >= rows) continue;
        float v = acc[i][j][e];
        if (bias) {
          int t = rm0 + off;
          while (t >= C) t -= C;
          if (t == 0) v += bv;
        }
        if (R) v += R[(size_t)r * ldr + c];
        Y[(size_t)r * ldy + c] = v;
      }
    }
  }
}

template <int TN, int STAGES>
void launch_x6b_t(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* R, int ldr,
                  float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  constexpr int BM = 256, BN = 64 * TN;
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  const size_t smem = (size_t)STAGES * (BM * 16 * 4 + 3 * BN * 16 * 2);
  ensure_smem(gemm_x6b_kernel<TN, STAGES>, smem);
  hipLaunchKernelGGL((gemm_x6b_kernel<TN, STAGES>), dim3(ntm * ntn), dim3(512), smem, s, X, ldx, Wp, ldp, bias, R,
                     ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
}

// ---- pipelined form: 256 x 32*TN tiles, 8 waves of 32 x 32*TN, BK = 16, 3-buffer ring ----
// The split of the NEXT k-tile's activations runs between the MFMAs of the current one
// (its f32 fragment is read from LDS one k-tile ahead), so the matrix cores do not idle
// through a VALU-only phase after every barrier.  Ring: at iteration kt the DMA fills
// buffer (kt+2)%3 (last read in iteration kt-1, retired by this iteration's barrier), A of
// kt+1 is read from buffer (kt+1)%3 (landed: vmcnt(0) + barrier), B of kt from kt%3.
// Every activation element is split by exactly one wave (wave w owns rows 32w..32w+31).
template <int TN>
__global__ __launch_bounds__(512) void gemm_x6c_kernel(const float* __restrict__ X, int ldx,
                                                       const uint16_t* __restrict__ Wp, int ldp,
                                                       const float* __restrict__ bias, const float* R, int ldr,
                                                       float* Y, int ldy, int rows, int ncols, int K, int C, int ntm,
                                                       int ntn) {
  constexpr int NW = 8, BM = 256, BN = 32 * TN, BK = 16;
  constexpr int A_BYTES = BM * BK * 4, B_PLANE = BN * BK * 2, STAGE = A_BYTES + 3 * B_PLANE;
  constexpr int IA = A_BYTES / 1024, IB = (3 * B_PLANE + 1023) / 1024, PER = (IA + IB + NW - 1) / NW;
  static_assert(A_BYTES % 1024 == 0 && (3 * B_PLANE) % 1024 == 0, "DMA pieces");
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;

  const int nblk = ntm * ntn;
  int bid = blockIdx.x;
  {
    const int q = nblk / 8, r8 = nblk % 8, xcd = bid % 8, slot = bid / 8;
    bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
  }
  const int tm = bid / ntn, tn = bid % ntn;
  const int row0 = tm * BM, col0 = tn * BN;
  const size_t plane = (size_t)ldp * K;
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);

  auto stage = [&](int k0, int buf) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      int j = wid + t * NW;
      if (j >= IA + IB) j = IA + IB - 1;  // wave-uniform: repeat the last piece
      const void* src;
      uint32_t dst;
      if (j < IA) {  // 16 rows x 64 B of f32 activations
        const int r = j * 16 + (lane >> 2);
        const int sl = ((lane & 3) ^ ((r >> 2) & 3)) * 4;
        src = X + (size_t)(row0 + r) * ldx + k0 + sl;
        dst = lds0 + (uint32_t)(buf * STAGE + j * 1024);
      } else {  // 32 rows x 32 B of the weight planes, rows (plane, n) contiguous
        const int q = (j - IA) * 32 + (lane >> 1);  // global row of the [3][BN] image
        const int p = q / BN, n = q % BN;
        const int sl = ((lane & 1) ^ ((n >> 3) & 1)) * 8;
        src = Wp + p * plane + (size_t)(col0 + n) * K + k0 + sl;
        dst = lds0 + (uint32_t)(buf * STAGE + A_BYTES + (j - IA) * 1024);
      }
      dst = __builtin_amdgcn_readfirstlane(dst);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(dst)
                   : "memory");
    }
  };
  const int m = wid * 32 + l32;  // this lane's A row within the tile
  auto read_a = [&](int buf, float4& u, float4& v) {
    const float* arow = reinterpret_cast<const float*>(smem + buf * STAGE) + m * BK;
    u = *reinterpret_cast<const float4*>(arow + (((2 * lh) ^ ((m >> 2) & 3)) * 4));
    v = *reinterpret_cast<const float4*>(arow + (((2 * lh + 1) ^ ((m >> 2) & 3)) * 4));
  };

  f32x16 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;

  const int nk = K / BK;
  stage(0, 0);
  if (nk > 1) stage(BK, 1);
  if (nk > 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bf16x8 c0, c1, c2;  // split fragments of the current k-tile
  {
    float4 u, v;
    read_a(0, u, v);
    split3(u, v, c0, c1, c2);
  }
  int bcur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage kt+1 (issued one iteration ago)
    __syncthreads();
    int bn1 = bcur + 1, bn2 = bcur + 2;
    if (bn1 >= 3) bn1 -= 3;
    if (bn2 >= 3) bn2 -= 3;
    if (kt + 2 < nk) stage((kt + 2) * BK, bn2);
    const bool more = kt + 1 < nk;
    float4 u, v;
    if (more) read_a(bn1, u, v);
    const char* Bs = smem + bcur * STAGE + A_BYTES;
    bf16x8 n0, n1, n2;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = j * 32 + l32;
      const int off = n * 32 + ((lh ^ ((n >> 3) & 1)) * 16);
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bs + off);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bs + B_PLANE + off);
      const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(Bs + 2 * B_PLANE + off);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c2, b0, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c0, b2, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c1, b1, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c1, b0, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c0, b1, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c0, b0, acc[j], 0, 0, 0);
      if (j == TN / 2 && more) split3(u, v, n0, n1, n2);
    }
    __builtin_amdgcn_s_setprio(0);
    if (more) {
      c0 = n0;
      c1 = n1;
      c2 = n2;
    }
    bcur = bn1;
  }

  const int rbase = row0 + wid * 32 + 4 * lh;
  const int rm0 = (C == 1) ? 0 : rbase % C;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int c = col0 + j * 32 + l32;
    if (c >= ncols) continue;
    const float bv = bias ? bias[c] : 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int off = (e & 3) + 8 * (e >> 2);
      const int r = rbase + off;
      if (r >= rows) continue;
      float val = acc[j][e];
      if (bias) {
        int t = rm0 + off;
        while (t >= C) t -= C;
        if (t == 0) val += bv;
      }
      if (R) val += R[(size_t)r * ldr + c];
      Y[(size_t)r * ldy + c] = val;
    }
  }
}

template <int TN>
void launch_x6c_t(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* R, int ldr,
                  float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  constexpr int BM = 256, BN = 32 * TN;
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  const size_t smem = 3ull * (BM * 16 * 4 + 3 * BN * 16 * 2);
  ensure_smem(gemm_x6c_kernel<TN>, smem);
  hipLaunchKernelGGL((gemm_x6c_kernel<TN>), dim3(ntm * ntn), dim3(512), smem, s, X, ldx, Wp, ldp, bias, R, ldr, Y,
                     ldy, rows, ncols, K, C, ntm, ntn);
}

// ---- lean pipelined form (the production kernel) -------------------------------------------
// As gemm_x6c_kernel (256 x 32*TN tiles, 8 waves of 32 rows, BK = 16, 3-buffer ring, next
// k-tile's split between the current MFMAs), with the issue budget of a bf16 MFMA in mind
// (an MFMA gap of 32 cycles holds ~6 VALU issues, MI355X_MICROARCH.md cycle table):
//  * DMA sources are a per-lane 32-bit offset fixed for the whole tile plus a scalar base
//    advanced per k-tile (global_load_lds saddr form: no VALU address math in the loop);
//  * B fragment addresses are lane-constant + immediate offsets (the slot swizzle depends on
//    l32 only), A fragment addresses lane-constant + the buffer base;
//  * interior tiles store without row / column guards; the channel-bias rows of a lane's 32
//    rows are a bit mask computed once per tile.
// ABL (ablation, tools only): 0 full; 1 no DMA / barriers (LDS contents stale); 2 also no
// split (fragments reinterpreted); 3 also no LDS reads (MFMAs on register operands only).
// NW waves (BM = 32 NW).  ST = 3: the ring above (one workgroup per CU at NW = 8).  ST = 2:
// two buffers, the k-tile's own split at its top and one barrier per k-tile; at NW = 4,
// TN = 8 a workgroup takes 64 KiB of LDS, so two share a CU and one's epilogue stores
// overlap the other's MFMAs.
// LNM != 0 (log-psi rows, BN = ncols = 256, C = 1): the LayerNorm that follows the GEMM
// runs in the epilogue, in place over h = R = Y (as gemm_ln_kernel, gemm.hip):
//   LNM 1:  h = LN(h + X W + b)          (psiformer.py:44-45)
//   LNM 2:  h = LN(h + tanh(X W + b))    (psiformer.py:46-47; X = h)
// A workgroup owns whole rows, so the row statistics are wave-local: each wave transposes
// its 32 x 256 block into LDS once, then sweeps it three times (pre-LN value + mean,
// centred variance, normalise + store) with 16 lanes per row.  X (= h in LNM 2) is only
// read by the DMA of this workgroup's own rows, all landed before the epilogue barrier.
template <int TN, int ABL = 0, int NW = 8, int ST = 3, int LNM = 0, int WN = 1>
__global__ __launch_bounds__(NW * WN * 64) __attribute__((amdgpu_waves_per_eu(NW * WN >= 8 ? 1 : 8 / (NW * WN)))) void gemm_x6d_kernel(const float* X, int ldx,
                                                       const uint16_t* __restrict__ Wp, int ldp,
                                                       const float* __restrict__ bias, const float* R, int ldr,
                                                       float* Y, int ldy, int rows, int ncols, int K, int C, int ntm,
                                                       int ntn, const float* __restrict__ ln, X6Feat feat) {
  // NW x WN waves: wave (wm, wn) computes rows 32 wm.. and columns 32 TN wn.. of the tile
  constexpr int NWT = NW * WN;
  // ablation switches (ABL 5: the full main loop, no epilogue)
  constexpr bool A_DMA = ABL == 0 || ABL >= 5, A_SPLIT = ABL < 2 || ABL >= 5, A_LDS = ABL < 3 || ABL >= 5;
  constexpr int BM = 32 * NW, BN = 32 * TN * WN, BK = 16;
  static_assert(LNM == 0 || BN == 256, "LayerNorm epilogue needs whole 256-column rows");
  static_assert(WN == 1 || BN == 256, "shared-tile epilogue: 64 lanes x 4 columns");
  constexpr int A_BYTES = BM * BK * 4, B_PLANE = BN * BK * 2, STAGE = A_BYTES + 3 * B_PLANE;
  constexpr int IA = A_BYTES / 1024, IB = (3 * B_PLANE) / 1024, PER = (IA + IB + NWT - 1) / NWT;
  static_assert(A_BYTES % 1024 == 0 && (3 * B_PLANE) % 1024 == 0, "DMA pieces");
  static_assert(ST >= 2 && ST <= 6, "ring depth");
  static_assert(ST <= 3 || (ST - 3) * PER <= 63, "vmcnt range");
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int l32 = lane & 31, lh = lane >> 5;

  const int nblk = ntm * ntn;
  int bid = blockIdx.x;
  {
    const int q = nblk / 8, r8 = nblk % 8, xcd = bid % 8, slot = bid / 8;
    bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
  }
  const int tm = bid / ntn, tn = bid % ntn;
  const int row0 = tm * BM, col0 = tn * BN;
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);

  // per-lane DMA source offsets (bytes) relative to the scalar bases xa / wb, and LDS targets
  uint32_t voff[PER], ldst[PER];
  bool isA[PER];
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    int j = wid + t * NWT;
    if (j >= IA + IB) j = IA + IB - 1;  // wave-uniform: repeat the last piece
    isA[t] = j < IA;
    if (j < IA) {  // 16 rows x 64 B of f32 activations
      const int r = j * 16 + (lane >> 2);
      const int sl = ((lane & 3) ^ ((r >> 2) & 3)) * 4;
      voff[t] = (uint32_t)((size_t)r * ldx + sl) * 4u;
      ldst[t] = j * 1024;
    } else {  // 32 rows x 32 B of the weight planes, rows (plane, n) contiguous in LDS
      const int q = (j - IA) * 32 + (lane >> 1);
      const int p = q / BN, n = q % BN;
      const int sl = ((lane & 1) ^ ((n >> 3) & 1)) * 8;
      voff[t] = (uint32_t)(((size_t)p * ldp + n) * K + sl) * 2u;
      ldst[t] = A_BYTES + (j - IA) * 1024;
    }
  }
  const char* xa = reinterpret_cast<const char*>(X + (size_t)row0 * ldx);
  const char* wb = reinterpret_cast<const char*>(Wp + (size_t)col0 * K);
  auto stage = [&](int kt, int buf) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const char* base = isA[t] ? xa + kt * (BK * 4) : wb + kt * (BK * 2);
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(buf * STAGE) + ldst[t]);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(voff[t]), "s"(base), "s"(dst)
                   : "memory");
    }
  };
  // A fragment: row m, k = 8 lh + (0..7) = logical 16-B slots 2lh, 2lh+1 of a 64-B row
  const int m = wm * 32 + l32;
  const int aoff0 = m * 64 + (((2 * lh) ^ ((m >> 2) & 3)) * 16);
  const int aoff1 = m * 64 + (((2 * lh + 1) ^ ((m >> 2) & 3)) * 16);
  // B fragment of column block j: row n = 32j + l32, slot lh ^ ((n >> 3) & 1) = lh ^ ((l32 >> 3) & 1)
  const int boff = A_BYTES + wn * TN * 1024 + l32 * 32 + ((lh ^ ((l32 >> 3) & 1)) * 16);

  f32x16 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;

  const int nk = K / BK;
  if (ST == 2) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const char* Bs = smem + boff;
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) stage(kt + 1, cur ^ 1);  // buffer last read in iteration kt-1
      const char* As = smem + cur * STAGE;
      bf16x8 c0, c1, c2;
      {
        const float4 u = *reinterpret_cast<const float4*>(As + aoff0);
        const float4 v = *reinterpret_cast<const float4*>(As + aoff1);
        split3(u, v, c0, c1, c2);
      }
      const char* Bc = Bs + cur * STAGE;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bc + j * 1024);
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bc + B_PLANE + j * 1024);
        const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(Bc + 2 * B_PLANE + j * 1024);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c2, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, c0, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, c1, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c1, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, c0, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c0, acc[j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage kt+1 landed
      __syncthreads();                                  // ... and buffer cur is free
    }
  } else {
  // ring of ST buffers, ST - 2 stages in flight while a k-tile computes: stages 0 .. ST-2
  // issued up front; at k-tile kt, wait for stage kt + 1 (the younger ST - 3 may stay in
  // flight: VMEM ops of a wave complete in order), barrier, issue stage kt + ST - 1 into the
  // buffer k-tile kt - 1 used
  for (int t = 0; t < ST - 1 && t < nk; ++t) stage(t, t);
  if (nk > ST - 2)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"((ST - 2) * PER) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bf16x8 c0, c1, c2;
  {
    const float4 u = *reinterpret_cast<const float4*>(smem + aoff0);
    const float4 v = *reinterpret_cast<const float4*>(smem + aoff1);
    split3(u, v, c0, c1, c2);
  }
  int bcur = 0;
  bf16x8 rb0 = c0, rb1 = c1, rb2 = c2;  // ABL 3 operands
  constexpr bool PB = A_LDS && A_SPLIT;  // B reads pipelined one column block ahead
  bf16x8 nb[3];
  if constexpr (PB) {
    nb[0] = *reinterpret_cast<const bf16x8*>(smem + boff);
    nb[1] = *reinterpret_cast<const bf16x8*>(smem + boff + B_PLANE);
    nb[2] = *reinterpret_cast<const bf16x8*>(smem + boff + 2 * B_PLANE);
  }
  for (int kt = 0; kt < nk; ++kt) {
    if (A_DMA) {
      if (ST > 3 && kt + ST - 2 < nk)  // stages kt + 2 .. kt + ST - 2 issued: they may stay in flight
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"((ST > 3 ? ST - 3 : 0) * PER) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage kt+1 (issued earlier)
      __syncthreads();
    }
    int bn1 = bcur + 1, bnl = bcur + ST - 1;
    if (bn1 >= ST) bn1 -= ST;
    if (bnl >= ST) bnl -= ST;
    if (A_DMA && kt + ST - 1 < nk) stage(kt + ST - 1, bnl);
    const bool more = kt + 1 < nk;
    float4 u, v;
    if (PB) {  // the next stage's A (stale past the last k-tile: split but never used)
      const char* An = smem + bn1 * STAGE;
      u = *reinterpret_cast<const float4*>(An + aoff0);
      v = *reinterpret_cast<const float4*>(An + aoff1);
    } else if (more) {
      if (A_LDS) {
        const char* An = smem + bn1 * STAGE;  // ABL 3, 4: no LDS reads
        u = *reinterpret_cast<const float4*>(An + aoff0);
        v = *reinterpret_cast<const float4*>(An + aoff1);
      } else {
        u = make_float4(kt, 1.f, 2.f, 3.f);
        v = u;
      }
    }
    const char* Bs = smem + bcur * STAGE + boff;
    bf16x8 n0, n1, n2;
    __builtin_amdgcn_s_setprio(1);
    if constexpr (PB) {
      ktile_pipelined<TN, B_PLANE>(Bs, smem + bn1 * STAGE + boff, acc, nb, c0, c1, c2, u, v, n0, n1, n2);
    } else {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bf16x8 b0, b1, b2;
      if (A_LDS) {
        b0 = *reinterpret_cast<const bf16x8*>(Bs + j * 1024);
        b1 = *reinterpret_cast<const bf16x8*>(Bs + B_PLANE + j * 1024);
        b2 = *reinterpret_cast<const bf16x8*>(Bs + 2 * B_PLANE + j * 1024);
      } else {
        b0 = rb0;
        b1 = rb1;
        b2 = rb2;
      }
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c2, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, c0, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, c1, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c1, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, c0, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c0, acc[j], 0, 0, 0);
      if (j == TN / 2 && more) {
        if (A_SPLIT) {
          split3(u, v, n0, n1, n2);
        } else {
          n0 = __builtin_bit_cast(bf16x8, u);
          n1 = __builtin_bit_cast(bf16x8, v);
          n2 = n0;
        }
      }
    }
    }
    __builtin_amdgcn_s_setprio(0);
    if (more) {
      c0 = n0;
      c1 = n1;
      c2 = n2;
    }
    bcur = bn1;
  }
  }  // ST == 3

  if (ABL == 4 || ABL == 5) {  // ablation: no stores unless the impossible happens (keeps the MFMAs live)
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) t += acc[j][e];
    if (t == 1234.5f) Y[tid] = t;
    return;
  }
  // epilogue.  The MFMA operands are swapped (weight fragment as A), so register e of
  // acc[j] holds output row rw0 + l32, column 32j + 8(e >> 2) + 4lh + (e & 3): four
  // consecutive columns per register group.  Each wave transposes 32 x 64-column panels
  // through a private LDS region (row stride 68 floats: conflict-free ds_write_b128) and
  // writes whole 256-B row pieces with global_store_dwordx4 (4 rows per instruction; the
  // residual is read the same way).  dword stores of the MFMA layout were store-issue bound.
  if constexpr (LNM != 0) {
    // 16 lanes per row, 4 rows per pass: lane (rq = lane >> 4, sub = lane & 15) owns columns
    // c_k = 4 sub + 64 k (k < 4) of tile row 4 (wid + NWT p) + rq, so one store instruction
    // writes four 256-B row pieces and the row statistics are 16-lane DPP sums (two-pass
    // mean / centred variance, eps 1e-5, as gemm_ln_kernel).  The residual (h, or geo for
    // the feature residual) of PC passes is loaded before the tile exchange, so the passes
    // wait on no global load (R aliases Y: the compiler may not hoist the loads itself).
    constexpr int NP = BM / (4 * NWT), PC = NP < 2 ? NP : 2;
    static_assert(BM % (4 * NWT) == 0 && NP % PC == 0, "rows per wave");
    const int sub = lane & 15, rq = lane >> 4;
    float4 rpre[PC][4];
    auto load_res = [&](int p0) {
#pragma unroll
      for (int pc = 0; pc < PC; ++pc) {
        const int r = row0 + 4 * (wid + NWT * (p0 + pc)) + rq;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          rpre[pc][k] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (r < rows) {
            if (feat.W0) {
              if (k == 0) rpre[pc][0] = *reinterpret_cast<const float4*>(feat.geo + 4 * (size_t)r);
            } else {
              rpre[pc][k] = *reinterpret_cast<const float4*>(R + (size_t)r * ldr + 4 * sub + 64 * k);
            }
          }
        }
      }
    };
    load_res(0);
    __syncthreads();  // every wave is done with the ring buffers
    // every wave puts its 32 x 32TN block into the shared [BM][LS] tile (row stride 260:
    // conflict-free ds_write_b128, as 68 below)
    constexpr int LS = 260;
    float* blk = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(blk + (32 * wm + l32) * LS + 32 * (wn * TN + j) + 8 * g + 4 * lh) =
            make_float4(acc[j][4 * g], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]);
    __syncthreads();
    float4 bv[4], gm[4], bt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 4 * sub + 64 * k;
      bv[k] = *reinterpret_cast<const float4*>(bias + c);
      gm[k] = *reinterpret_cast<const float4*>(ln + c);
      bt[k] = *reinterpret_cast<const float4*>(ln + 256 + c);
    }
    for (int p0 = 0; p0 < NP; p0 += PC) {
      if (p0 > 0) load_res(p0);
#pragma unroll
      for (int pc = 0; pc < PC; ++pc) {
        const int rr = 4 * (wid + NWT * (p0 + pc)) + rq;
        const int r = row0 + rr;
        float4 v[4];
        float f[4];
        if (feat.W0) {  // input.hip's h = f W0, same order
          const float4 g = rpre[pc][0];  // st ct sp cp
          f[0] = g.y;
          f[1] = g.x * g.w;
          f[2] = g.x * g.z;
          f[3] = (r % feat.N < feat.n_up) ? 1.f : -1.f;
        }
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int c = 4 * sub + 64 * k;
          float4 t = *reinterpret_cast<const float4*>(blk + rr * LS + c);
          t.x += bv[k].x;
          t.y += bv[k].y;
          t.z += bv[k].z;
          t.w += bv[k].w;
          if (LNM == 2 && ABL != 7) {  // ABL 7: ablation, no tanh
            t.x = tanh_rat(t.x);
            t.y = tanh_rat(t.y);
            t.z = tanh_rat(t.z);
            t.w = tanh_rat(t.w);
          }
          if (r < rows) {
            float4 rv;
            if (feat.W0) {
              float4 w0[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) w0[q] = *reinterpret_cast<const float4*>(feat.W0 + q * 256 + c);
              rv.x = f[0] * w0[0].x + f[1] * w0[1].x + f[2] * w0[2].x + f[3] * w0[3].x;
              rv.y = f[0] * w0[0].y + f[1] * w0[1].y + f[2] * w0[2].y + f[3] * w0[3].y;
              rv.z = f[0] * w0[0].z + f[1] * w0[1].z + f[2] * w0[2].z + f[3] * w0[3].z;
              rv.w = f[0] * w0[0].w + f[1] * w0[1].w + f[2] * w0[2].w + f[3] * w0[3].w;
            } else {
              rv = rpre[pc][k];
            }
            t.x += rv.x;
            t.y += rv.y;
            t.z += rv.z;
            t.w += rv.w;
          }
          v[k] = t;
          sum += (t.x + t.y) + (t.z + t.w);
        }
        const float mean = (ABL == 6 ? sum : row16_sum(sum)) * (1.f / 256.f);
        float ss = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k].x -= mean;
          v[k].y -= mean;
          v[k].z -= mean;
          v[k].w -= mean;
          ss += (v[k].x * v[k].x + v[k].y * v[k].y) + (v[k].z * v[k].z + v[k].w * v[k].w);
        }
        const float var = (ABL == 6 ? ss : row16_sum(ss)) * (1.f / 256.f);
        const float rs = __builtin_amdgcn_rsqf(var + 1e-5f);
        if (r < rows) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float4 o;
            o.x = gm[k].x * (rs * v[k].x) + bt[k].x;
            o.y = gm[k].y * (rs * v[k].y) + bt[k].y;
            o.z = gm[k].z * (rs * v[k].z) + bt[k].z;
            o.w = gm[k].w * (rs * v[k].w) + bt[k].w;
            *reinterpret_cast<float4*>(Y + (size_t)r * ldy + 4 * sub + 64 * k) = o;
          }
        }
      }
    }
    return;
  }
  __syncthreads();  // every wave is done with the ring buffers
  if constexpr (WN > 1) {
    // plain epilogue of the 2-D wave grid: the same shared tile, then whole 1-KB row
    // pieces per wave instruction (ncols % 4 == 0: a float4 is in or out as a whole)
    constexpr int LS = 260;
    float* blk = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(blk + (32 * wm + l32) * LS + 32 * (wn * TN + j) + 8 * g + 4 * lh) =
            make_float4(acc[j][4 * g], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]);
    __syncthreads();
    const int c = col0 + 4 * lane;
    if (c >= ncols) return;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bias) bv = *reinterpret_cast<const float4*>(bias + c);
    for (int rr = wid; rr < BM; rr += NWT) {
      const int r = row0 + rr;
      if (r >= rows) break;
      float4 v = *reinterpret_cast<const float4*>(blk + rr * LS + 4 * lane);
      if (bias && (C == 1 || r % C == 0)) {
        v.x += bv.x;
        v.y += bv.y;
        v.z += bv.z;
        v.w += bv.w;
      }
      if (R) {
        const float4 rv = *reinterpret_cast<const float4*>(R + (size_t)r * ldr + c);
        v.x += rv.x;
        v.y += rv.y;
        v.z += rv.z;
        v.w += rv.w;
      }
      *reinterpret_cast<float4*>(Y + (size_t)r * ldy + c) = v;
    }
    return;
  }
  const int rw0 = row0 + wid * 32;
  float* red = reinterpret_cast<float*>(smem) + wid * (32 * 68);
  const bool full = rw0 + 32 <= rows && col0 + BN <= ncols;
  const int lr = lane >> 4, lc = (lane & 15) * 4;  // read-back: rows 4q + lr, columns lc..lc+3
  uint32_t vq = 0;  // bit q: row rw0 + lr + 4q carries the bias (channel 0)
  if (bias) {
    if (C == 1) {
      vq = 0xffu;
    } else {
      int t = (rw0 + lr) % C;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (t == 0) vq |= 1u << q;
        t += 4;
        while (t >= C) t -= C;
      }
    }
  }
#pragma unroll
  for (int pnl = 0; pnl < TN / 2; ++pnl) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x16& a = acc[2 * pnl + jj];
        *reinterpret_cast<float4*>(red + l32 * 68 + 32 * jj + 8 * g + 4 * lh) =
            make_float4(a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]);
      }
    const int c = col0 + 64 * pnl + lc;
    float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bias && (full || c + 3 < ncols)) bv = *reinterpret_cast<const float4*>(bias + c);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int rr = 4 * q + lr, r = rw0 + rr;
      float4 v = *reinterpret_cast<const float4*>(red + rr * 68 + lc);
      if (full || (r < rows && c + 3 < ncols)) {
        if (vq & (1u << q)) {
          v.x += bv.x;
          v.y += bv.y;
          v.z += bv.z;
          v.w += bv.w;
        }
        if (R) {
          const float4 rv = *reinterpret_cast<const float4*>(R + (size_t)r * ldr + c);
          v.x += rv.x;
          v.y += rv.y;
          v.z += rv.z;
          v.w += rv.w;
        }
        *reinterpret_cast<float4*>(Y + (size_t)r * ldy + c) = v;
      } else if (r < rows) {  // ragged edge: element by element
        const float e4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (c + t >= ncols) break;
          float val = e4[t];
          if (vq & (1u << q)) val += bias[c + t];
          if (R) val += R[(size_t)r * ldr + c + t];
          Y[(size_t)r * ldy + c + t] = val;
        }
      }
    }
  }
}

template <int TN, int ABL = 0, int NW = 8, int ST = 3, int LNM = 0, int WN = 1>
void launch_x6d_t(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* R, int ldr,
                  float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s, const float* ln = nullptr,
                  X6Feat feat = X6Feat{}) {
  constexpr int BM = 32 * NW, BN = 32 * TN * WN;
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  // LDS: the DMA ring, reused by the epilogue's per-wave 32 x 68-float transpose regions
  // (a shared BM x 260-float tile of whole rows with the LayerNorm epilogue or WN > 1)
  const size_t smem =
      std::max((size_t)ST * (BM * 16 * 4 + 3 * BN * 16 * 2), (size_t)(LNM || WN > 1 ? BM * 260 : NW * 32 * 68) * 4);
  ensure_smem(gemm_x6d_kernel<TN, ABL, NW, ST, LNM, WN>, smem);
  hipLaunchKernelGGL((gemm_x6d_kernel<TN, ABL, NW, ST, LNM, WN>), dim3(ntm * ntn), dim3(NW * WN * 64), smem, s, X,
                     ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, ntm, ntn, ln, feat);
}

// ---- persistent lean form: one DMA ring across all of a workgroup's tiles --------------------
// gemm_x6d_kernel (ST = 3) run persistently: the workgroup walks tiles blockIdx.x, +G, ...
// and the (tile, k-tile) steps form one stream, so the next tile's first k-tiles are in
// flight (and its first split done) while the current tile's epilogue runs; the epilogue
// transposes through its own LDS region (not the ring) and its 4*TN dwordx4 stores stay
// in flight under the next steps (counted: vmcnt(4*TN) at the next step's wait; VMEM ops of
// a wave complete in order).  LDS: ring 3 x 40 KiB + 8 x 4.5 KiB transpose = 156 KiB.
// R4: a 4-stage ring (160 KiB, two stages in flight instead of one: the DMA latency cover
// doubles).  No LDS is left for a transpose region, so a tile's last step does not issue
// its step + 3 DMA: the epilogue transposes through that free stage buffer, and the next
// step issues two stages (its wait then counts the epilogue's stores instead).
template <int TN, bool HAS_R, bool R4 = false, int ABLQ = 0, bool PB = false>  // ABLQ 1: no epilogue stores (tools only)
__global__ __launch_bounds__(512) void gemm_x6q_kernel(const float* __restrict__ X, int ldx,
                                                       const uint16_t* __restrict__ Wp, int ldp,
                                                       const float* __restrict__ bias, const float* R, int ldr,
                                                       float* Y, int ldy, int rows, int ncols, int K, int C, int ntm,
                                                       int ntn) {
  constexpr int NW = 8, BM = 256, BN = 32 * TN, BK = 16;
  constexpr int A_BYTES = BM * BK * 4, B_PLANE = BN * BK * 2, STAGE = A_BYTES + 3 * B_PLANE;
  constexpr int IA = A_BYTES / 1024, IB = (3 * B_PLANE) / 1024, PER = (IA + IB + NW - 1) / NW;
  constexpr int NST = 4 * TN, TS = 36;  // stores per wave per tile; transpose row stride (floats)
  static_assert(A_BYTES % 1024 == 0 && (3 * B_PLANE) % 1024 == 0, "DMA pieces");
  static_assert(PER + NST <= 63, "vmcnt range");
  constexpr int NS = R4 ? 4 : 3;  // ring stages
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int nblk = ntm * ntn, G = gridDim.x;
  const int my_tiles = ((int)blockIdx.x < nblk) ? (nblk - 1 - (int)blockIdx.x) / G + 1 : 0;
  const int nk = K / BK, F = my_tiles * nk;
  if (F == 0) return;
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);
  auto tile_of = [&](int i, int& row0, int& col0) {  // XCD-aware order (G is a multiple of 8)
    const int idx = blockIdx.x + i * G;
    const int q = nblk / 8, r8 = nblk % 8, xcd = idx % 8, slot = idx / 8;
    const int bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
    row0 = (bid / ntn) * BM;
    col0 = (bid % ntn) * BN;
  };

  uint32_t voff[PER], ldst[PER];
  bool isA[PER];
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    int j = wid + t * NW;
    if (j >= IA + IB) j = IA + IB - 1;
    isA[t] = j < IA;
    if (j < IA) {
      const int r = j * 16 + (lane >> 2);
      const int sl = ((lane & 3) ^ ((r >> 2) & 3)) * 4;
      voff[t] = (uint32_t)((size_t)r * ldx + sl) * 4u;
      ldst[t] = j * 1024;
    } else {
      const int q = (j - IA) * 32 + (lane >> 1);
      const int p = q / BN, n = q % BN;
      const int sl = ((lane & 1) ^ ((n >> 3) & 1)) * 8;
      voff[t] = (uint32_t)(((size_t)p * ldp + n) * K + sl) * 2u;
      ldst[t] = A_BYTES + (j - IA) * 1024;
    }
  }
  auto stage = [&](int f, int buf) {
    int row0, col0;
    tile_of(f / nk, row0, col0);
    const int kt = f % nk;
    const char* xa = reinterpret_cast<const char*>(X + (size_t)row0 * ldx) + kt * (BK * 4);
    const char* wb = reinterpret_cast<const char*>(Wp + (size_t)col0 * K) + kt * (BK * 2);
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const char* base = isA[t] ? xa : wb;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(buf * STAGE) + ldst[t]);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(voff[t]), "s"(base), "s"(dst)
                   : "memory");
    }
  };
  const int m = wid * 32 + l32;
  const int aoff0 = m * 64 + (((2 * lh) ^ ((m >> 2) & 3)) * 16);
  const int aoff1 = m * 64 + (((2 * lh + 1) ^ ((m >> 2) & 3)) * 16);
  const int boff = A_BYTES + l32 * 32 + ((lh ^ ((l32 >> 3) & 1)) * 16);
  float* red = reinterpret_cast<float*>(smem + 3 * STAGE) + wid * (32 * TS);  // R4: set per tile
  const int lr = lane >> 3, lc = (lane & 7) * 4;  // read-back: rows 8q + lr, columns lc..lc+3

  f32x16 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;

  stage(0, 0);
  if (F > 1) stage(1, 1);
  if (R4 && F > 2) stage(2, 2);
  if (R4 && F > 2)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PER) : "memory");
  else if (F > 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bf16x8 c0, c1, c2;
  {
    const float4 u = *reinterpret_cast<const float4*>(smem + aoff0);
    const float4 v = *reinterpret_cast<const float4*>(smem + aoff1);
    split3(u, v, c0, c1, c2);
  }
  bf16x8 nb[3];  // PB: block-0 B fragments of the current k-tile
  if constexpr (PB) {
    nb[0] = *reinterpret_cast<const bf16x8*>(smem + boff);
    nb[1] = *reinterpret_cast<const bf16x8*>(smem + boff + B_PLANE);
    nb[2] = *reinterpret_cast<const bf16x8*>(smem + boff + 2 * B_PLANE);
  }
  int bcur = 0, kt = 0, tile = 0;
  bool stored = false;  // epilogue stores issued in the previous step
  bool deferred = false;  // R4: the previous (tile-end) step left its step + 3 DMA to this one
  for (int f = 0; f < F; ++f) {
    // wait for step f+1's DMA; younger: (ST 3) the previous epilogue's stores, (R4) step
    // f+2's DMA, or, after a tile end, the epilogue's stores
    if constexpr (R4) {
      if (deferred && stored)  // exactly NST stores behind step f+1's DMA
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NST) : "memory");
      else if (deferred)  // a partial tile's guarded stores: drain
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (f + 2 < F)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (stored)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NST) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    stored = false;
    int bn1 = bcur + 1, bn2 = bcur + 2, bn3 = bcur + 3;
    if (bn1 >= NS) bn1 -= NS;
    if (bn2 >= NS) bn2 -= NS;
    if (bn3 >= NS) bn3 -= NS;
    const bool tile_end = kt + 1 == nk;
    if constexpr (R4) {
      if (deferred && f + 2 < F) stage(f + 2, bn2);  // the transpose buffer of the last epilogue
      if (!tile_end && f + 3 < F) stage(f + 3, bn3);  // the buffer step f-1 read
      deferred = tile_end;
      if (tile_end) red = reinterpret_cast<float*>(smem + bn3 * STAGE) + wid * (32 * TS);
    } else {
      if (f + 2 < F) stage(f + 2, bn2);
    }
    const bool more = f + 1 < F;
    float4 u, v;
    if (PB) {  // the next stage's A (stale past the last k-tile: split but never used)
      const char* An = smem + bn1 * STAGE;
      u = *reinterpret_cast<const float4*>(An + aoff0);
      v = *reinterpret_cast<const float4*>(An + aoff1);
    } else if (more) {
      const char* An = smem + bn1 * STAGE;
      u = *reinterpret_cast<const float4*>(An + aoff0);
      v = *reinterpret_cast<const float4*>(An + aoff1);
    }
    const char* Bs = smem + bcur * STAGE + boff;
    bf16x8 n0, n1, n2;
    __builtin_amdgcn_s_setprio(1);
    if constexpr (PB) {
      ktile_pipelined<TN, B_PLANE>(Bs, smem + bn1 * STAGE + boff, acc, nb, c0, c1, c2, u, v, n0, n1, n2);
    } else {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bs + j * 1024);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bs + B_PLANE + j * 1024);
      const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(Bs + 2 * B_PLANE + j * 1024);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c2, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, c0, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, c1, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c1, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, c0, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, c0, acc[j], 0, 0, 0);
      if (j == TN / 2 && more) split3(u, v, n0, n1, n2);
    }
    }
    __builtin_amdgcn_s_setprio(0);
    if (more) {
      c0 = n0;
      c1 = n1;
      c2 = n2;
    }
    bcur = bn1;
    if (++kt < nk) continue;
    // ---- tile done: epilogue (MFMA layout: acc[j] reg e = row rw0 + l32, column
    // 32j + 8(e>>2) + 4lh + (e&3)); transpose 32 x 32 blocks through `red`, dwordx4 stores
    int row0, col0;
    tile_of(tile, row0, col0);
    kt = 0;
    ++tile;
    const int rw0 = row0 + wid * 32;
    const bool full = rw0 + 32 <= rows && col0 + BN <= ncols;
    uint32_t vq = 0;  // bit q: row rw0 + lr + 8q carries the bias
    if (bias) {
      if (C == 1) {
        vq = 0xfu;
      } else {
        int t = (rw0 + lr) % C;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (t == 0) vq |= 1u << q;
          t += 8;
          while (t >= C) t -= C;
        }
      }
    }
    // Loads first: every load issued after a store would make its wait drain that store
    // (vmcnt counts loads and stores in one in-order queue).  Bias slices of all column
    // blocks up front; the residual of block j+1 before the stores of block j.  Interior
    // tiles run branch-free (bias required; HAS_R a template flag), so the compiler's waits
    // stay counted; partial tiles take a guarded element-wise path.
    if (full) {
      float4 bvv[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j)  // vq == 0 without a bias: the zeros are never added
        bvv[j] = bias ? *reinterpret_cast<const float4*>(bias + col0 + 32 * j + lc) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 rcur[4], rnext[4];
      auto load_r = [&](int j, float4(&dst)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          dst[q] = *reinterpret_cast<const float4*>(R + (size_t)(rw0 + 8 * q + lr) * ldr + col0 + 32 * j + lc);
      };
      if (HAS_R) load_r(0, rcur);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (HAS_R && j + 1 < TN) load_r(j + 1, rnext);
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(red + l32 * TS + 8 * g + 4 * lh) =
              make_float4(acc[j][4 * g], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]);
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = 8 * q + lr;
          float4 val = *reinterpret_cast<const float4*>(red + rr * TS + lc);
          if (vq & (1u << q)) {
            val.x += bvv[j].x;
            val.y += bvv[j].y;
            val.z += bvv[j].z;
            val.w += bvv[j].w;
          }
          if (HAS_R) {
            val.x += rcur[q].x;
            val.y += rcur[q].y;
            val.z += rcur[q].z;
            val.w += rcur[q].w;
          }
          if (ABLQ == 0 || val.x == 1.2345e-30f)
            *reinterpret_cast<float4*>(Y + (size_t)(rw0 + rr) * ldy + col0 + 32 * j + lc) = val;
        }
        if (HAS_R) {
#pragma unroll
          for (int q = 0; q < 4; ++q) rcur[q] = rnext[q];
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(red + l32 * TS + 8 * g + 4 * lh) =
              make_float4(acc[j][4 * g], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]);
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
        const int c = col0 + 32 * j + lc;
        for (int q = 0; q < 4; ++q) {
          const int rr = 8 * q + lr, r = rw0 + rr;
          if (r >= rows) continue;
          const float* x4 = red + rr * TS + lc;
          for (int t2 = 0; t2 < 4 && c + t2 < ncols; ++t2) {
            float x = x4[t2];
            if (vq & (1u << q)) x += bias[c + t2];
            if (HAS_R) x += R[(size_t)r * ldr + c + t2];
            Y[(size_t)r * ldy + c + t2] = x;
          }
        }
      }
    }
    // full tiles issue exactly NST stores per wave (the count the next wait assumes);
    // partial tiles drain everything at the next wait
    stored = full && ABLQ == 0;
  }
}

template <int TN, bool R4 = false, int ABLQ = 0, bool PB = false>
void launch_x6q_t(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* R, int ldr,
                  float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  constexpr int BM = 256, BN = 32 * TN;
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  const size_t st = BM * 16 * 4 + 3 * BN * 16 * 2;
  const size_t smem = R4 ? 4ull * st : 3ull * st + 8ull * 32 * 36 * 4;
  static_assert(!R4 || BM * 16 * 4 + 3 * BN * 16 * 2 >= 8 * 32 * 36 * 4, "transpose fits a stage");
  int grid = std::min(ntm * ntn, cu_count_x6());
  grid = std::max(8, grid / 8 * 8);
  if (R) {
    ensure_smem(gemm_x6q_kernel<TN, true, R4, ABLQ, PB>, smem);
    hipLaunchKernelGGL((gemm_x6q_kernel<TN, true, R4, ABLQ, PB>), dim3(grid), dim3(512), smem, s, X, ldx, Wp, ldp, bias, R,
                       ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
  } else {
    ensure_smem(gemm_x6q_kernel<TN, false, R4, ABLQ, PB>, smem);
    hipLaunchKernelGGL((gemm_x6q_kernel<TN, false, R4, ABLQ, PB>), dim3(grid), dim3(512), smem, s, X, ldx, Wp, ldp, bias,
                       R, ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
  }
}

// ---- persistent form: weight panel resident in LDS, activations straight to registers ----
// A workgroup owns one 64-column panel of the output for its whole life: the three bf16
// planes of that weight panel (64 x K x 3 x 2 B = 96 KiB at K = 256) are loaded into LDS
// once, then every wave walks its own 32-row tiles with NO barrier: it loads its A rows
// from global memory straight into registers (lane (r, h) holds row r, k = 32t + 16h ..
// +15 of k-tile t: 64 contiguous bytes, the two lane halves covering a 128-B line), one
// k-tile ahead, splits them and runs 2 x 6 MFMAs per 16-k chunk against B fragments read
// from LDS.  B k labelling matches: chunk c of k-tile t takes k = 32t + 16h + 8c + j.
// LDS image: [plane][64 rows][K] bf16, 16-B slot s of row n stored at s ^ (n & 15).
// Groups of P workgroups (one per panel, adjacent logical ids, i.e. one XCD) walk the
// same row tiles, so each A row is fetched from HBM once and re-read from L2.
constexpr int XP_BN = 64;

template <int NW, bool HAS_R>
__global__ __launch_bounds__(NW * 64) void gemm_x6p_kernel(const float* __restrict__ X, int ldx,
                                                           const uint16_t* __restrict__ Wp, int ldp,
                                                           const float* __restrict__ bias, const float* R, int ldr,
                                                           float* Y, int ldy, int rows, int ncols, int K, int C,
                                                           int P, int ngroups) {
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  // logical id: consecutive ids share an XCD (gridDim.x is a multiple of 8)
  const int g = blockIdx.x, per_xcd = gridDim.x / 8;
  const int L = (g % 8) * per_xcd + g / 8;
  const int group = L / P, panel = L % P;
  if (group >= ngroups) return;  // whole workgroup exits (no barrier reached)
  const int col0 = panel * XP_BN;
  const int row_bytes = K * 2, slots = K / 8;  // one B row: K bf16 = K/8 slots of 16 B
  const int plane_bytes = XP_BN * row_bytes;
  // ---- load the weight panel (three planes) into LDS, swizzled
  {
    const int total = 3 * XP_BN * slots;  // 16-B pieces
    for (int q = tid; q < total; q += NW * 64) {
      const int p = q / (XP_BN * slots), rem = q % (XP_BN * slots);
      const int n = rem / slots, s = rem % slots;
      const uint4 v =
          *reinterpret_cast<const uint4*>(Wp + ((size_t)p * ldp + col0 + n) * K + (size_t)s * 8);
      *reinterpret_cast<uint4*>(smem + p * plane_bytes + n * row_bytes + ((s ^ (n & 15)) * 16)) = v;
    }
  }
  __syncthreads();

  const int ntiles = (rows + 31) / 32, nk = K / 32;
  // this wave's tiles: group + ngroups * (wid + NW * i)
  const int first = group + ngroups * wid, stride = ngroups * NW;
  const int my_tiles = first < ntiles ? (ntiles - 1 - first) / stride + 1 : 0;
  const int F = my_tiles * nk;
  if (F == 0) return;

  auto load_a = [&](int f, float4 (&a)[4]) {
    const int t = first + (f / nk) * stride, kt = f % nk;
    const float* src = X + (size_t)(t * 32 + l32) * ldx + kt * 32 + lh * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = *reinterpret_cast<const float4*>(src + 4 * q);
  };

  f32x16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;

  float4 an[4], ac[4];
  load_a(0, an);
  int kt = 0, tcount = 0;
  for (int f = 0; f < F; ++f) {
#pragma unroll
    for (int q = 0; q < 4; ++q) ac[q] = an[q];
    if (f + 1 < F) load_a(f + 1, an);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      bf16x8 a0, a1, a2;
      split3(ac[2 * c], ac[2 * c + 1], a0, a1, a2);
      const int s = 4 * kt + 2 * lh + c;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = j * 32 + l32;
        const char* bp = smem + n * row_bytes + ((s ^ (n & 15)) * 16);
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(bp);
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(bp + plane_bytes);
        const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(bp + 2 * plane_bytes);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[j], 0, 0, 0);
      }
    }
    if (++kt == nk) {  // tile done: epilogue
      const int t = first + tcount * stride;
      const int rbase = t * 32 + 4 * lh;
      const int rm0 = (C == 1) ? 0 : rbase % C;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = col0 + j * 32 + l32;
        const bool cok = c < ncols;
        const float bv = (bias && cok) ? bias[c] : 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int off = (e & 3) + 8 * (e >> 2);
          const int r = rbase + off;
          float v = acc[j][e];
          acc[j][e] = 0.f;
          if (!cok || r >= rows) continue;
          if (bias) {
            int tt = rm0 + off;
            while (tt >= C) tt -= C;
            if (tt == 0) v += bv;
          }
          if (HAS_R) v += R[(size_t)r * ldr + c];
          Y[(size_t)r * ldy + c] = v;
        }
      }
      kt = 0;
      ++tcount;
    }
  }
}

template <int NW>
void launch_x6p_t(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* R, int ldr,
                  float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  const int P = (ncols + XP_BN - 1) / XP_BN;
  const int slots = std::max(8, cu_count_x6() / 8 * 8);  // workgroups resident at once (1 per CU)
  int ngroups = std::max(1, slots / P);
  const int ntiles = (rows + 31) / 32;
  ngroups = std::min(ngroups, std::max(1, (ntiles + NW - 1) / NW));
  const int grid = round_up(ngroups * P, 8);
  const size_t smem = 3ull * XP_BN * K * 2;
  ensure_smem(gemm_x6p_kernel<NW, true>, smem);
  ensure_smem(gemm_x6p_kernel<NW, false>, smem);
  if (R)
    hipLaunchKernelGGL((gemm_x6p_kernel<NW, true>), dim3(grid), dim3(NW * 64), smem, s, X, ldx, Wp, ldp, bias, R,
                       ldr, Y, ldy, rows, ncols, K, C, P, ngroups);
  else
    hipLaunchKernelGGL((gemm_x6p_kernel<NW, false>), dim3(grid), dim3(NW * 64), smem, s, X, ldx, Wp, ldp, bias, R,
                       ldr, Y, ldy, rows, ncols, K, C, P, ngroups);
}

// ---- persistent 16x16x32 form (round 3): 2-D wave grid, direct-from-accumulator stores -------
// The channel-row GEMM on v_mfma_f32_16x16x32_bf16 (the shape that holds the higher clock
// under load on MI355X: ≈1.13x the FLOP/s of 32x32x16 with operands re-read from LDS,
// MI355X_MICROARCH.md, DVFS item 7).  Tile 256 x 32*TNC, BK = 32 per step (one barrier
// per 32 k, half the 16-k form's), two 80 KiB stage buffers (LDS-DMA of step f+1 in flight
// while step f computes).  8 waves as 4 (rows) x 2 (columns): a wave owns 64 rows x 16*TNC
// columns = 4 x TNC accumulator blocks of 16 x 16 — its four activation fragments are split
// ONCE per step and reused across the TNC column blocks, the weight fragments stream from
// LDS one column block ahead (LDS reads per step and wave: 8 + 3 TNC b128, against 52 in
// gemm_x6q at the same MFMA count).  With the weights as the MFMA's A operand the C/D layout
// (col = lane & 15 = activation row, row = 4 (lane >> 4) + reg = weight column) hands every
// lane 4 consecutive output columns of one row: the epilogue stores float4 straight from
// the accumulators (no LDS transpose).  LDS images (conflict-free ds_read_b128 for the
// 16x16x32 lane groups, swizzles found by exhaustive search): activations [256][32 f32]
// (128 B rows, 16-B slot s at s ^ fA(r), fA(r) = ((r >> 1) & 1) | ((r >> 3) & 1) << 2);
// weights [plane][BN][32 bf16] (64 B rows, slot s at s ^ fB(n), fB(n) = 2 ((n >> 2) & 1)).
__device__ __forceinline__ int x6m_fa(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int x6m_fb(int n) { return ((n >> 2) & 1) << 1; }

// SPREAD: the next step's DMA pieces are issued between the first column blocks' MFMAs
// instead of all at once after the barrier (LDS-DMA issue costs ~60 cycles a piece), and
// the activation fragments are split just ahead of their first MFMAs.
// ABL (tools/gemm_bench.py ablations only, wrong results): bit 0 no DMA after the first
// stage, bit 1 no barrier, bit 2 no epilogue stores, bit 3 no activation split (hi term only)
template <int TNC, bool HAS_R, bool SPREAD = false, int ABL = 0, bool DMA4 = false>
__global__ __launch_bounds__(512, 1) void gemm_x6m_kernel(const float* __restrict__ X, int ldx,
                                                          const uint16_t* __restrict__ Wp, int ldp,
                                                          const float* __restrict__ bias, const float* R, int ldr,
                                                          float* Y, int ldy, int rows, int ncols, int K, int C, int ntm,
                                                          int ntn) {
  constexpr int NW = 8, BM = 256, BN = 32 * TNC, BK = 32, WC = 16 * TNC;
  constexpr int A_BYTES = BM * BK * 4, B_PLANE = BN * BK * 2, STAGE = A_BYTES + 3 * B_PLANE;
  // DMA4: only the four column-half-0 waves issue the LDS-DMA (twice the pieces each), so on
  // every SIMD one wave issues it while its partner (same rows, other column half) keeps the
  // MFMA pipe busy, instead of both stalling on the issue at the same moment
  constexpr int NDW = DMA4 ? 4 : NW;
  constexpr int IA = A_BYTES / 1024, IB = (3 * B_PLANE) / 1024, PER = (IA + IB + NDW - 1) / NDW;
  constexpr int NST = 4 * TNC;  // float4 stores per wave per tile
  static_assert(A_BYTES % 1024 == 0 && (3 * B_PLANE) % 1024 == 0, "DMA pieces");
  static_assert(PER + NST <= 63, "vmcnt range");
  static_assert(2 * STAGE <= 163840, "LDS");
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid & 3, wc = wid >> 2;  // 64-row group, column half
  const int l16 = lane & 15, kg = lane >> 4;
  const int nblk = ntm * ntn, G = gridDim.x;
  const int my_tiles = ((int)blockIdx.x < nblk) ? (nblk - 1 - (int)blockIdx.x) / G + 1 : 0;
  const int nk = K / BK, F = my_tiles * nk;
  if (F == 0) return;
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);
  auto tile_of = [&](int i, int& row0, int& col0) {  // XCD-aware order (G is a multiple of 8)
    const int idx = blockIdx.x + i * G;
    const int q = nblk / 8, r8 = nblk % 8, xcd = idx % 8, slot = idx / 8;
    const int bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
    row0 = (bid / ntn) * BM;
    col0 = (bid % ntn) * BN;
  };
  // DMA pieces of this wave: activation rows (8 rows x 128 B per KiB) or weight rows
  // (16 rows x 64 B per KiB), the global 16-B slot chosen so the LDS image is swizzled
  uint32_t voff[PER], ldst[PER];
  bool isA[PER];
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    int j = (DMA4 ? wr : wid) + t * NDW;
    if (j >= IA + IB) j = IA + IB - 1;  // a duplicate piece (same bytes, same place)
    isA[t] = j < IA;
    if (j < IA) {
      const int r = j * 8 + (lane >> 3);
      const int s = (lane & 7) ^ x6m_fa(r);
      voff[t] = (uint32_t)((size_t)r * ldx * 4 + s * 16);
      ldst[t] = j * 1024;
    } else {
      const int q = (j - IA) * 16 + (lane >> 2);  // plane-major row index
      const int p = q / BN, n = q % BN;
      const int s = (lane & 3) ^ x6m_fb(n);
      voff[t] = (uint32_t)((((size_t)p * ldp + n) * K) * 2 + s * 16);
      ldst[t] = A_BYTES + (j - IA) * 1024;
    }
  }
  const bool dma_wave = !DMA4 || wc == 0;
  auto stage = [&](int f, int buf) {
    if (!dma_wave) return;
    int row0, col0;
    tile_of(f / nk, row0, col0);
    const int kt = f % nk;
    const char* xa = reinterpret_cast<const char*>(X + (size_t)row0 * ldx) + kt * (BK * 4);
    const char* wb = reinterpret_cast<const char*>(Wp + (size_t)col0 * K) + kt * (BK * 2);
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const char* base = isA[t] ? xa : wb;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(buf * STAGE) + ldst[t]);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(voff[t]), "s"(base), "s"(dst)
                   : "memory");
    }
  };
  // fragment addresses (bytes within a stage)
  int aoff[4][2];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int r = wr * 64 + rb * 16 + l16;
    aoff[rb][0] = r * 128 + (((2 * kg) ^ x6m_fa(r)) * 16);
    aoff[rb][1] = r * 128 + (((2 * kg + 1) ^ x6m_fa(r)) * 16);
  }
  auto boff = [&](int cb) {
    const int n = wc * WC + cb * 16 + l16;
    return A_BYTES + n * 64 + ((kg ^ x6m_fb(n)) * 16);
  };
  f32x4 acc[4][TNC];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int cb = 0; cb < TNC; ++cb) acc[rb][cb] = (f32x4){0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  int kt = 0, tile = 0;
  bool stored = false;  // the previous step ended a tile: NST stores younger than the DMA
  for (int f = 0; f < F; ++f) {
    const int buf = f & 1;
    if (stored)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NST) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(ABL & 2)) __builtin_amdgcn_s_barrier();  // step f landed everywhere; step f-1's buffer is free
    asm volatile("" ::: "memory");
    stored = false;
    const bool more = f + 1 < F && !(ABL & 1);
    if (!SPREAD && more) stage(f + 1, buf ^ 1);
    const char* S = smem + buf * STAGE;
    // activation fragments: 4 row blocks, split once
    bf16x8 a0[4], a1[4], a2[4];
    float4 au[4], av[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      au[rb] = *reinterpret_cast<const float4*>(S + aoff[rb][0]);
      av[rb] = *reinterpret_cast<const float4*>(S + aoff[rb][1]);
      if (ABL & 8) {
        a0[rb] = __builtin_bit_cast(bf16x8, (u32x4v){pk_bf16(au[rb].x, au[rb].y), pk_bf16(au[rb].z, au[rb].w),
                                                       pk_bf16(av[rb].x, av[rb].y), pk_bf16(av[rb].z, av[rb].w)});
        a1[rb] = a0[rb];
        a2[rb] = a0[rb];
      } else if (!SPREAD) {
        split3(au[rb], av[rb], a0[rb], a1[rb], a2[rb]);
      }
    }
    bf16x8 wf[2][3];
    {
      const int o = boff(0);
      wf[0][0] = *reinterpret_cast<const bf16x8*>(S + o);
      wf[0][1] = *reinterpret_cast<const bf16x8*>(S + o + B_PLANE);
      wf[0][2] = *reinterpret_cast<const bf16x8*>(S + o + 2 * B_PLANE);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int cb = 0; cb < TNC; ++cb) {
      if (cb + 1 < TNC) {
        const int o = boff(cb + 1);
        wf[(cb + 1) & 1][0] = *reinterpret_cast<const bf16x8*>(S + o);
        wf[(cb + 1) & 1][1] = *reinterpret_cast<const bf16x8*>(S + o + B_PLANE);
        wf[(cb + 1) & 1][2] = *reinterpret_cast<const bf16x8*>(S + o + 2 * B_PLANE);
      }
      const bf16x8 b0 = wf[cb & 1][0], b1 = wf[cb & 1][1], b2 = wf[cb & 1][2];
      if (SPREAD && more && dma_wave) {  // pieces [cb PER / HALF, (cb + 1) PER / HALF) over the first HALF blocks
        constexpr int HALF = TNC / 2 > 0 ? TNC / 2 : 1;
        if (cb < HALF) {
          int row0n, col0n;
          tile_of((f + 1) / nk, row0n, col0n);
          const int ktn = (f + 1) % nk;
          const char* xa = reinterpret_cast<const char*>(X + (size_t)row0n * ldx) + ktn * (BK * 4);
          const char* wb = reinterpret_cast<const char*>(Wp + (size_t)col0n * K) + ktn * (BK * 2);
#pragma unroll
          for (int t = 0; t < PER; ++t) {
            if (t * HALF / PER != cb) continue;
            const char* base = isA[t] ? xa : wb;
            const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)((buf ^ 1) * STAGE) + ldst[t]);
            unsigned keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(voff[t]), "s"(base), "s"(dst)
                         : "memory");
          }
        }
      }
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        if (SPREAD && !(ABL & 8) && cb == 0) split3(au[rb], av[rb], a0[rb], a1[rb], a2[rb]);
        f32x4 c = acc[rb][cb];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0, a2[rb], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2, a0[rb], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, a1[rb], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0, a1[rb], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, a0[rb], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0, a0[rb], c, 0, 0, 0);
        acc[rb][cb] = c;
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (++kt < nk) continue;
    // ---- tile done: lane holds row r = .. + l16, columns n .. n+3 of every block
    int row0, col0;
    tile_of(tile, row0, col0);
    kt = 0;
    ++tile;
    const int rw0 = row0 + wr * 64, cw0 = col0 + wc * WC;
    const bool full = rw0 + 64 <= rows && cw0 + WC <= ncols;
    float bfl[4];  // 1 on the rows that carry the bias (r % C == 0), else 0: branch-free adds
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) bfl[rb] = (bias && (rw0 + rb * 16 + l16) % C == 0) ? 1.f : 0.f;
    if (full) {
      // (no drain: the compiler's waits on the bias / residual loads also cover the older DMA).
      // The bias values of every column block are loaded before the first store (X6M_BIAS1):
      // a load between two stores would wait for every earlier store (vmcnt counts in order)
#if X6M_BIAS1
      float4 bvs[TNC];
#pragma unroll
      for (int cb = 0; cb < TNC; ++cb)
        bvs[cb] = bias ? *reinterpret_cast<const float4*>(bias + cw0 + cb * 16 + 4 * kg) : make_float4(0.f, 0.f, 0.f, 0.f);
#endif
#pragma unroll
      for (int cb = 0; cb < TNC; ++cb) {
        const int n = cw0 + cb * 16 + 4 * kg;
#if X6M_BIAS1
        const float4 bv = bvs[cb];
#else
        const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#endif
        float4 rv[4];
        if (HAS_R) {
#pragma unroll
          for (int rb = 0; rb < 4; ++rb)
            rv[rb] = *reinterpret_cast<const float4*>(R + (size_t)(rw0 + rb * 16 + l16) * ldr + n);
        }
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          f32x4 c = acc[rb][cb];
          c[0] = fmaf(bfl[rb], bv.x, c[0]);
          c[1] = fmaf(bfl[rb], bv.y, c[1]);
          c[2] = fmaf(bfl[rb], bv.z, c[2]);
          c[3] = fmaf(bfl[rb], bv.w, c[3]);
          if (HAS_R) {
            c[0] += rv[rb].x;
            c[1] += rv[rb].y;
            c[2] += rv[rb].z;
            c[3] += rv[rb].w;
          }
          if (!(ABL & 4) || c[0] == 1.2345e-30f) {
            f32x4* yp = reinterpret_cast<f32x4*>(Y + (size_t)(rw0 + rb * 16 + l16) * ldy + n);
            if constexpr (X6M_NT)
              __builtin_nontemporal_store(c, yp);  // streaming: the weights stay resident in L2
            else
              *yp = c;
          }
        }
      }
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int cb = 0; cb < TNC; ++cb) acc[rb][cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
      stored = !(ABL & 4);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int cb = 0; cb < TNC; ++cb) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int r = rw0 + rb * 16 + l16, n = cw0 + cb * 16 + 4 * kg;
          const f32x4 c = acc[rb][cb];
          acc[rb][cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
          if (r >= rows) continue;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (n + e >= ncols) continue;
            float x = c[e];
            if (bfl[rb] != 0.f) x += bias[n + e];
            if (HAS_R) x += R[(size_t)r * ldr + n + e];
            Y[(size_t)r * ldy + n + e] = x;
          }
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // guarded stores: an uncounted number
    }
  }
}

template <int TNC, bool SPREAD = false, int ABL = 0, bool DMA4 = false>
void launch_x6m_t(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* R, int ldr,
                  float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  constexpr int BM = 256, BN = 32 * TNC;
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  const size_t smem = 2ull * (BM * 32 * 4 + 3 * BN * 32 * 2);
  int grid = std::min(ntm * ntn, cu_count_x6());
  grid = std::max(8, grid / 8 * 8);
  if (R) {
    ensure_smem(gemm_x6m_kernel<TNC, true, SPREAD, ABL, DMA4>, smem);
    hipLaunchKernelGGL((gemm_x6m_kernel<TNC, true, SPREAD, ABL, DMA4>), dim3(grid), dim3(512), smem, s, X, ldx, Wp, ldp, bias, R,
                       ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
  } else {
    ensure_smem(gemm_x6m_kernel<TNC, false, SPREAD, ABL, DMA4>, smem);
    hipLaunchKernelGGL((gemm_x6m_kernel<TNC, false, SPREAD, ABL, DMA4>), dim3(grid), dim3(512), smem, s, X, ldx, Wp, ldp, bias,
                       R, ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
  }
}

// Wt[n][k] f32 (row stride ldw) -> three bf16 planes Wp[p][n][k], p = 0, 1, 2 (rows n >= ncols zero).
__global__ void split_planes_kernel(const float* __restrict__ Wt, int ldw, int ncols, int K, int ldp, uint16_t* Wp) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t plane = (size_t)ldp * K;
  if (i >= plane) return;
  const int n = (int)(i / K), k = (int)(i % K);
  const float a = n < ncols ? Wt[(size_t)n * ldw + k] : 0.f;
  const __bf16 a0 = (__bf16)a;
  const float r1 = a - (float)a0;
  const __bf16 a1 = (__bf16)r1;
  const __bf16 a2 = (__bf16)(r1 - (float)a1);
  Wp[i] = __builtin_bit_cast(uint16_t, a0);
  Wp[plane + i] = __builtin_bit_cast(uint16_t, a1);
  Wp[2 * plane + i] = __builtin_bit_cast(uint16_t, a2);
}


// ---- chained log-psi layer tail ------------------------------------------------------------
// One launch per layer for the walker rows (C = 1) of the split-bf16 log-psi path:
//   P1  h1 = LN1(h + o Wol + bol)                (psiformer.py:44-46; Wol = Wo Wl folded)
//   P2  h2 = LN2(h1 + tanh(h1 Wm + bm))           (psiformer.py:47-48)  -> h (global)
//   P3  Y3 = h2 W3 + b3   (optional)              the next layer's q|k|v, or the orbitals
// 96-row tiles; h1 and h2 stay in the CU (chain_x6s_kernel below).
constexpr int CH_BM = 96, CH_BN = 256, CH_K = 256;
constexpr int CH_KO = 32;  // layer 1's o~ rows (H = 4 heads x 8 slots, dh_internal.h ofeat_k)

struct ChainArgs {
  const float* X1;  // o [rows][256]
  const uint16_t *Wp1, *Wp2, *Wp3;
  int ldp1, ldp2, ldp3;
  const float *b1, *ln1, *b2, *ln2, *b3;
  int n3, ldy3;
  float* Y3;
  float* h;  // residual of P1 (unless feat.W0), output of P2
  int rows;
  X6Feat feat;
  int store_h;  // 0: P2's h is not written back (the last layer: only P3's orbitals are consumed)
};

// ---- chained layer tail, pre-split activations ------------------------------------------------
// Every activation element is split into its three bf16 terms ONCE, by the thread that
// writes it, into LDS planes [3][96][264] (an LDS-ring form that re-split the A tile in every
// wave reading it cost 4-8x the VALU work, round 2), and the weight fragments stream
// from L2 straight into registers PD k-tiles ahead (no LDS ring, no barrier in a pass).
// 8 waves; wave w owns output columns 32 w .. 32 w + 31 of a 256-column pass and all 96
// rows (three 32-row MFMA blocks).  The LayerNorms run on the MFMA layout in registers:
// row sums = 16 values per lane + the lane-half shuffle + 8 wave partials through LDS.
// Same products in the same order as the other x6 kernels; the LayerNorm statistics are
// summed in a different order (f32 rounding, not bitwise).
constexpr int CS_NW = 8, CS_RB = CH_BM / 32, CS_PD = 4, CS_LSP = 264;  // plane row: 528 B
#ifndef CHAIN_PRM  // A/B knob: LN1 / LN2 scale-shift and the P2 bias staged in LDS once per tile
#define CHAIN_PRM 1
#endif
// CS_PRMF: [ln1 gamma | beta][b2][ln2 gamma | beta] floats after the partials (CHAIN_PRM)
constexpr int CS_PRMF = CHAIN_PRM ? 5 * 256 : 0;
constexpr size_t CS_PLANE = (size_t)CH_BM * CS_LSP * 2, CS_SMEM = 3 * CS_PLANE + 2 * CS_NW * CH_BM * 4 + CS_PRMF * 4;
static_assert(CS_SMEM <= 163840, "chain LDS");

// 4 f32 -> three packed bf16 pairs per term (as split3)
__device__ __forceinline__ void split4(const float4& x, uint2& h, uint2& m, uint2& l) {
  const float a[4] = {x.x, x.y, x.z, x.w};
  uint32_t H[2], Mv[2], Lv[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float u = a[2 * p], v = a[2 * p + 1];
    const uint32_t h2 = pk_bf16(u, v);
    const float ru = u - lo_f(h2), rv = v - hi_f(h2);
    const uint32_t m2 = pk_bf16(ru, rv);
    H[p] = h2;
    Mv[p] = m2;
    Lv[p] = pk_bf16(ru - lo_f(m2), rv - hi_f(m2));
  }
  h = make_uint2(H[0], H[1]);
  m = make_uint2(Mv[0], Mv[1]);
  l = make_uint2(Lv[0], Lv[1]);
}

// NA > 0: layer 1 with its attention fused (X1 unused): the prologue forms o of the tile's
// 96 / NA walkers itself (attn_val.h, bit-identical to attention_val_kernel<NA, true>): wave
// w takes head w % 4 for walkers 48 / NA * (w / 4) .., two walkers per attn_feat_core call
// so their LDS round trips overlap (round 5: the scores from the features through the head's
// 5 x 5 form Mqk, no q / k rows), staging the weights in LDS that the planes overwrite
// afterwards, the o values held in registers (48 per lane) until every wave is done.
template <int NA = 0>
__global__ __launch_bounds__(512) void chain_x6s_kernel(ChainArgs a) {
  constexpr int RB = CS_RB, PD = CS_PD, LSP = CS_LSP;
  using K16 = std::integral_constant<int, CH_K / 16>;                     // a 256-deep pass
  using KP1 = std::integral_constant<int, (NA > 0 ? CH_KO / 16 : CH_K / 16)>;  // P1: o~ (layer 1) or o
  using K2 = std::integral_constant<int, 2>;  // layer 1's coefficient-space passes (32 deep)
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  float* part = reinterpret_cast<float*>(smem + 3 * CS_PLANE);  // [2][8 waves][96 rows]
  float* prm = part + 2 * CS_NW * CH_BM;                         // CHAIN_PRM: [ln1 | b2 | ln2]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  int bid = blockIdx.x;
  {
    const int nblk = gridDim.x, q = nblk / 8, r8 = nblk % 8, xcd = bid % 8, slot = bid / 8;
    bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
  }
  // rows per tile: 96, or with the attention in the prologue the whole walkers in 96 (N = 10:
  // 9 walkers = 90 rows; the last 96 - TRW rows of the tile are computed and never stored)
  constexpr int TRW = NA > 0 ? (CH_BM / NA) * NA : CH_BM;
  const int row0 = bid * TRW, rows = min(a.rows, row0 + TRW);
  // every barrier of this kernel orders LDS only (planes, partial sums, staging); no wave reads
  // global memory another wave of the launch wrote, so the VMEM queue (weight prefetch, h / Y3
  // stores) may stay in flight across it
  auto lbar = []() __attribute__((always_inline)) {
#if CHAIN_LBAR
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#else
    __syncthreads();
#endif
  };
  CHAIN_T(0);
  if (CHAIN_PRM) {  // read before the prologue's barrier
    for (int q = tid; q < 5 * 256; q += 512)
      prm[q] = q < 512 ? a.ln1[q] : (q < 768 ? a.b2[q - 512] : a.ln2[q - 768]);
  }
  // plane p, tile row r, column c (bf16 units)
  auto pl = [&](int p, int r, int c) __attribute__((always_inline)) {
    return smem + (size_t)p * CS_PLANE + (size_t)r * (LSP * 2) + c * 2;
  };
  // write 4 consecutive f32 of row r, columns c..c+3 as their three bf16 terms
  auto put4 = [&](int r, int c, const float4& x) __attribute__((always_inline)) {
    uint2 h, m, l;
    split4(x, h, m, l);
    *reinterpret_cast<uint2*>(pl(0, r, c)) = h;
    *reinterpret_cast<uint2*>(pl(1, r, c)) = m;
    *reinterpret_cast<uint2*>(pl(2, r, c)) = l;
  };
  // the f32 value back from the planes (exact: a = a0 + a1 + a2 with no rounding)
  auto get4 = [&](int r, int c) __attribute__((always_inline)) {
    const uint2 h = *reinterpret_cast<const uint2*>(pl(0, r, c));
    const uint2 m = *reinterpret_cast<const uint2*>(pl(1, r, c));
    const uint2 l = *reinterpret_cast<const uint2*>(pl(2, r, c));
    return make_float4((lo_f(h.x) + lo_f(m.x)) + lo_f(l.x), (hi_f(h.x) + hi_f(m.x)) + hi_f(l.x),
                       (lo_f(h.y) + lo_f(m.y)) + lo_f(l.y), (hi_f(h.y) + hi_f(m.y)) + hi_f(l.y));
  };

  // ---- one GEMM pass: acc[rb] = rows 32 rb + l32 x columns col0 + 32 wid + ..  The weight
  // fragments of its first PD k-tiles are requested by prefetch() beforehand, ahead of the
  // previous pass's epilogue: its stores then do not sit in front of them in vmcnt's queue
  f32x16 acc[RB];
  bf16x8 bq[PD][3];
  const uint16_t* wr = nullptr;
  size_t plane = 0;
  // nkt_: 16-wide k-tiles of the pass's contraction (16 = 256; layer 1's P1 from the o~ planes: 2)
  auto prefetch = [&](const uint16_t* Wp, int ldp, int col0, auto nkt_) __attribute__((always_inline)) {
    constexpr int NKT = decltype(nkt_)::value, KK = 16 * NKT;
    plane = (size_t)ldp * KK;
    wr = Wp + (size_t)(col0 + 32 * wid + l32) * KK + 8 * lh;
#pragma unroll
    for (int d = 0; d < (PD < NKT ? PD : NKT); ++d)
#pragma unroll
      for (int p = 0; p < 3; ++p) bq[d][p] = *reinterpret_cast<const bf16x8*>(wr + p * plane + 16 * d);
  };
  // TR: the operands swapped, D[tile row][output column] (P3's store layout, CHAIN_P3T)
  // accumulate_: keep acc's contents (layer 1's residual pass, NA > 0) instead of starting from 0
  auto gemm = [&](auto tr_, auto nkt_, auto accumulate_) __attribute__((always_inline)) {
    constexpr bool TR = decltype(tr_)::value;
    constexpr int nk = decltype(nkt_)::value;
    auto mf = [](const bf16x8& w, const bf16x8& x, const f32x16& c) __attribute__((always_inline)) {
      if constexpr (TR)
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w, c, 0, 0, 0);
      else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(w, x, c, 0, 0, 0);
    };
    if constexpr (!decltype(accumulate_)::value) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[rb][e] = 0.f;
    }
    // A fragments of k-tile kt (rows 32 rb + l32, k = 16 kt + 8 lh ..), read one k-tile ahead
    bf16x8 ca[RB][3];
    auto lda = [&](int kt, bf16x8(&d)[RB][3]) __attribute__((always_inline)) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          d[rb][p] = *reinterpret_cast<const bf16x8*>(pl(p, 32 * rb + l32, 16 * kt + 8 * lh));
    };
    lda(0, ca);
#pragma unroll
    for (int kt = 0; kt < nk; ++kt) {
      const bf16x8 b0 = bq[kt % PD][0], b1 = bq[kt % PD][1], b2 = bq[kt % PD][2];
      if (kt + PD < nk) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bq[kt % PD][p] = *reinterpret_cast<const bf16x8*>(wr + p * plane + 16 * (kt + PD));
      }
      bf16x8 cn[RB][3];
      if (kt + 1 < nk) lda(kt + 1, cn);
      // keep the prefetches where they are: the scheduler would sink each load to just
      // before its first use and expose the L2 / LDS latency
      __builtin_amdgcn_sched_barrier(0);
      // product-major over the three row blocks: consecutive MFMAs are independent
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[rb] = mf(b0, ca[rb][2], acc[rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[rb] = mf(b2, ca[rb][0], acc[rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[rb] = mf(b1, ca[rb][1], acc[rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[rb] = mf(b0, ca[rb][1], acc[rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[rb] = mf(b1, ca[rb][0], acc[rb]);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[rb] = mf(b0, ca[rb][0], acc[rb]);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int p = 0; p < 3; ++p) ca[rb][p] = cn[rb][p];
      }
    }
  };
  using NoTr = std::integral_constant<bool, false>;
  using Zero = std::integral_constant<bool, false>;
  using Accum = std::integral_constant<bool, true>;
  // MFMA layout: reg 4 g + e of acc[rb] = tile row 32 rb + l32, column 32 wid + 8 g + 4 lh + e
  auto colof = [&](int g) __attribute__((always_inline)) { return 32 * wid + 8 * g + 4 * lh; };
  // LayerNorm of the values x (MFMA layout, 16 per lane and row block) in registers:
  // two-pass mean / centred variance (eps 1e-5); the 8 wave partials of a row meet in LDS
  float x[RB][16];
  auto layernorm = [&](const float* ln) __attribute__((always_inline)) {
#if CHAIN_LN1P
    // ONE statistics round: sum x and sum x^2 together (flax's fast variance, the reference's
    // own arithmetic: var = max(E[x^2] - E[x]^2, 0), oracle/reference.py:134-137), one barrier
    // and one LDS exchange per LayerNorm instead of the two of the centred two-pass form
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      float t = 0.f, q = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        t += (x[rb][4 * g] + x[rb][4 * g + 1]) + (x[rb][4 * g + 2] + x[rb][4 * g + 3]);
        q += (x[rb][4 * g] * x[rb][4 * g] + x[rb][4 * g + 1] * x[rb][4 * g + 1]) +
             (x[rb][4 * g + 2] * x[rb][4 * g + 2] + x[rb][4 * g + 3] * x[rb][4 * g + 3]);
      }
      t += __shfl_xor(t, 32, 64);
      q += __shfl_xor(q, 32, 64);
      if (lh == 0) {
        part[wid * CH_BM + 32 * rb + l32] = t;
        part[(CS_NW + wid) * CH_BM + 32 * rb + l32] = q;
      }
    }
    lbar();
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      float t = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < CS_NW; ++w) {
        t += part[w * CH_BM + 32 * rb + l32];
        q += part[(CS_NW + w) * CH_BM + 32 * rb + l32];
      }
      const float mean = t * (1.f / 256.f);
      const float var = fmaxf(q * (1.f / 256.f) - mean * mean, 0.f);
      const float rs = __builtin_amdgcn_rsqf(var + 1e-5f);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 gm = *reinterpret_cast<const float4*>(ln + colof(g));
        const float4 bt = *reinterpret_cast<const float4*>(ln + CH_BN + colof(g));
        x[rb][4 * g] = gm.x * (rs * (x[rb][4 * g] - mean)) + bt.x;
        x[rb][4 * g + 1] = gm.y * (rs * (x[rb][4 * g + 1] - mean)) + bt.y;
        x[rb][4 * g + 2] = gm.z * (rs * (x[rb][4 * g + 2] - mean)) + bt.z;
        x[rb][4 * g + 3] = gm.w * (rs * (x[rb][4 * g + 3] - mean)) + bt.w;
      }
    }
#else
    float s[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) t += (x[rb][4 * g] + x[rb][4 * g + 1]) + (x[rb][4 * g + 2] + x[rb][4 * g + 3]);
      t += __shfl_xor(t, 32, 64);
      if (lh == 0) part[wid * CH_BM + 32 * rb + l32] = t;
    }
    lbar();
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < CS_NW; ++w) t += part[w * CH_BM + 32 * rb + l32];
      s[rb] = t * (1.f / 256.f);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        x[rb][e] -= s[rb];
        q += x[rb][e] * x[rb][e];
      }
      q += __shfl_xor(q, 32, 64);
      if (lh == 0) part[(CS_NW + wid) * CH_BM + 32 * rb + l32] = q;
    }
    lbar();
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < CS_NW; ++w) t += part[(CS_NW + w) * CH_BM + 32 * rb + l32];
      const float rs = __builtin_amdgcn_rsqf(t * (1.f / 256.f) + 1e-5f);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 gm = *reinterpret_cast<const float4*>(ln + colof(g));
        const float4 bt = *reinterpret_cast<const float4*>(ln + CH_BN + colof(g));
        x[rb][4 * g] = gm.x * (rs * x[rb][4 * g]) + bt.x;
        x[rb][4 * g + 1] = gm.y * (rs * x[rb][4 * g + 1]) + bt.y;
        x[rb][4 * g + 2] = gm.z * (rs * x[rb][4 * g + 2]) + bt.z;
        x[rb][4 * g + 3] = gm.w * (rs * x[rb][4 * g + 3]) + bt.w;
      }
    }
#endif
  };

  // ---- P1 prologue: o rows -> planes (each element split once)
  if constexpr (NA > 0) {
    // layer 1's attention in feature space for the tile's TRW / NA walkers and 4 heads, every
    // phase spread over the whole workgroup (round 6; attn_val.h's arithmetic, operation for
    // operation): (1) u_h,r = Mqk_h f~_r per (row, head), (2) per (walker, head, electron i)
    // the scores f~_i . u_h,j and their softmax, (3) o~_h,i = sum_j A_ij f~_j into the planes'
    // first 32 columns (head h at 8 h + a, slots 5..7 zero).  Staging lives in plane 0's
    // columns 32.. (bytes 64.. of each 528-B row: 112 floats per row), which P1 never reads.
    static_assert(CS_NW == 8 && CH_KO == 32, "4 heads of 8 slots");
    constexpr int WT = CH_BM / NA, NH = 4;  // walkers per tile, heads
    static_assert(CH_BM * NH <= 512 && WT * NH * NA <= 512, "one thread per (row, head) and per (walker, head, electron)");
    prefetch(a.Wp1, a.ldp1, 0, KP1{});
    auto stg = [&](int k) __attribute__((always_inline)) {  // staging float k
      return reinterpret_cast<float*>(smem + (size_t)(k / 112) * (LSP * 2) + 64 + (k % 112) * 4);
    };
    constexpr int F_ = 0, M_ = F_ + CH_BM * 5, U_ = M_ + NH * 25, A_ = U_ + CH_BM * NH * 5;  // staging layout
    static_assert(A_ + WT * NH * NA * NA <= CH_BM * 112, "staging fits plane 0's free columns");
    if (tid < CH_BM) {  // f~ of the tile's rows (rows past the batch: a valid dummy geometry)
      const int gr = row0 + tid;
      const float4 g = gr < rows ? *reinterpret_cast<const float4*>(a.feat.geo + 4 * (size_t)gr) : make_float4(0.f, 1.f, 0.f, 1.f);
      *stg(F_ + 5 * tid) = g.y;
      *stg(F_ + 5 * tid + 1) = g.x * g.w;
      *stg(F_ + 5 * tid + 2) = g.x * g.z;
      *stg(F_ + 5 * tid + 3) = (tid % NA < a.feat.n_up) ? 1.f : -1.f;
      *stg(F_ + 5 * tid + 4) = 1.f;
    } else if (tid < CH_BM + NH * 25) {
      const int q = tid - CH_BM;
      *stg(M_ + q) = a.feat.Mqk[(q / 25) * kMqkStride + q % 25];
    }
    lbar();
    if (tid < CH_BM * NH) {  // (1) u_h,r = M_h f~_r
      const int r = tid >> 2, hh = tid & 3;
      float f[5];
#pragma unroll
      for (int c = 0; c < 5; ++c) f[c] = *stg(F_ + 5 * r + c);
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        float u = 0.f;
#pragma unroll
        for (int c = 0; c < 5; ++c) u = fmaf(*stg(M_ + 25 * hh + 5 * q + c), f[c], u);
        *stg(U_ + 5 * (NH * r + hh) + q) = u;
      }
    }
    lbar();
    const int w = tid / (NH * NA), hh = (tid / NA) % NH, i = tid % NA;  // (walker, head, electron)
    const bool act = tid < WT * NH * NA;
    if (act) {  // (2) scores and softmax of row i
      float fi[5], e[NA], m = -INFINITY;
#pragma unroll
      for (int c = 0; c < 5; ++c) fi[c] = *stg(F_ + 5 * (w * NA + i) + c);
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        float sc = 0.f;
#pragma unroll
        for (int q = 0; q < 5; ++q) sc = fmaf(fi[q], *stg(U_ + 5 * (NH * (w * NA + j) + hh) + q), sc);
        e[j] = sc;
        m = fmaxf(m, sc);
      }
      float ssum = 0.f;
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        e[j] = expf(e[j] - m);
        ssum += e[j];
      }
      const float inv = 1.f / ssum;
#pragma unroll
      for (int j = 0; j < NA; ++j) *stg(A_ + NA * tid + j) = e[j] * inv;
    }
    lbar();
    float ov[5];
    if (act) {  // (3) o~ of row (w, i), head hh
      float A[NA];
#pragma unroll
      for (int j = 0; j < NA; ++j) A[j] = *stg(A_ + NA * tid + j);
      const bool live = row0 + w * NA + i < rows;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        float acc1 = 0.f;
#pragma unroll
        for (int j = 0; j < NA; ++j) acc1 = fmaf(A[j], *stg(F_ + 5 * (w * NA + j) + q), acc1);
        ov[q] = live ? acc1 : 0.f;
      }
    }
    lbar();  // every staging read done: the o~ columns of the rows are written below
    if (act) {
      const int r = w * NA + i;
#pragma unroll
      for (int q = 0; q < 8; ++q) {  // one element: the three bf16 terms of split4
        const float x = q < 5 ? ov[q] : 0.f;
        const uint32_t h2 = pk_bf16(x, 0.f);
        const float rx = x - lo_f(h2);
        const uint32_t m2 = pk_bf16(rx, 0.f);
        const uint32_t l2 = pk_bf16(rx - lo_f(m2), 0.f);
        const int c = 8 * hh + q;
        *reinterpret_cast<uint16_t*>(pl(0, r, c)) = (uint16_t)h2;
        *reinterpret_cast<uint16_t*>(pl(1, r, c)) = (uint16_t)m2;
        *reinterpret_cast<uint16_t*>(pl(2, r, c)) = (uint16_t)l2;
      }
    }
    lbar();
  } else {
    prefetch(a.Wp1, a.ldp1, 0, KP1{});
    const float4* src = reinterpret_cast<const float4*>(a.X1 + (size_t)row0 * CH_K);
#pragma unroll 4
    for (int i = tid; i < CH_BM * (CH_K / 4); i += 512) {
      const int r = i / (CH_K / 4), c = 4 * (i % (CH_K / 4));
      put4(r, c, src[i]);
    }
    lbar();
  }
  // ---- P1: h1 = LN1(h + o Wol + bol) -> planes
  CHAIN_T(1);
  gemm(NoTr{}, KP1{}, Zero{});
  CHAIN_T(2);
  {
    // every load of this phase issued before the first use, and P2's weight prefetch after
    // them (round 5): left to the compiler the bias / geometry loads went out one or two at a
    // time, each behind a vmcnt(0) that also waited for the weight prefetch (14 serialised
    // round trips per tile)
    float4 bvv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) bvv[g] = *reinterpret_cast<const float4*>(a.b1 + colof(g));
    if (a.feat.W0) {
      float4 w0[4][4];  // feature residual: W0 rows at this lane's columns
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q) w0[g][q] = *reinterpret_cast<const float4*>(a.feat.W0 + q * CH_BN + colof(g));
      float4 gq[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {  // geo holds exactly rows entries: clamped, masked below
        const int r = min(row0 + 32 * rb + l32, rows - 1);
        gq[rb] = *reinterpret_cast<const float4*>(a.feat.geo + 4 * (size_t)r);  // st ct sp cp
      }
      __builtin_amdgcn_sched_barrier(0);  // the residual loads ahead of the prefetch in vmcnt's queue
      if constexpr (NA > 0)
        prefetch(a.feat.L1V, a.ldp2, 0, K2{});
      else
        prefetch(a.Wp2, a.ldp2, 0, K16{});
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int r = row0 + 32 * rb + l32;
        float f[4] = {0.f, 0.f, 0.f, 0.f};
        if (r < rows) {
          f[0] = gq[rb].y;
          f[1] = gq[rb].x * gq[rb].w;
          f[2] = gq[rb].x * gq[rb].z;
          f[3] = (r % a.feat.N < a.feat.n_up) ? 1.f : -1.f;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 bv = bvv[g];
          float4 rv;
          rv.x = f[0] * w0[g][0].x + f[1] * w0[g][1].x + f[2] * w0[g][2].x + f[3] * w0[g][3].x;
          rv.y = f[0] * w0[g][0].y + f[1] * w0[g][1].y + f[2] * w0[g][2].y + f[3] * w0[g][3].y;
          rv.z = f[0] * w0[g][0].z + f[1] * w0[g][1].z + f[2] * w0[g][2].z + f[3] * w0[g][3].z;
          rv.w = f[0] * w0[g][0].w + f[1] * w0[g][1].w + f[2] * w0[g][2].w + f[3] * w0[g][3].w;
          x[rb][4 * g] = (acc[rb][4 * g] + bv.x) + rv.x;
          x[rb][4 * g + 1] = (acc[rb][4 * g + 1] + bv.y) + rv.y;
          x[rb][4 * g + 2] = (acc[rb][4 * g + 2] + bv.z) + rv.z;
          x[rb][4 * g + 3] = (acc[rb][4 * g + 3] + bv.w) + rv.w;
        }
      }
    } else {
      // the residual rows of h straight into x, then x = (acc + b) + h (the same sum)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int r = row0 + 32 * rb + l32;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 rv = *reinterpret_cast<const float4*>(a.h + (size_t)r * CH_BN + colof(g));  // h padded to 768 rows
          x[rb][4 * g] = rv.x;
          x[rb][4 * g + 1] = rv.y;
          x[rb][4 * g + 2] = rv.z;
          x[rb][4 * g + 3] = rv.w;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      prefetch(a.Wp2, a.ldp2, 0, K16{});
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 bv = bvv[g];
          x[rb][4 * g] = (acc[rb][4 * g] + bv.x) + x[rb][4 * g];
          x[rb][4 * g + 1] = (acc[rb][4 * g + 1] + bv.y) + x[rb][4 * g + 1];
          x[rb][4 * g + 2] = (acc[rb][4 * g + 2] + bv.z) + x[rb][4 * g + 2];
          x[rb][4 * g + 3] = (acc[rb][4 * g + 3] + bv.w) + x[rb][4 * g + 3];
        }
    }
  }
  CHAIN_T(3);
  if constexpr (NA > 0) {
    // ---- layer 1 in coefficient space (gemm_lnch.hip MODE 2's header with C = 1): the row
    // x = f W0 + o~ U + bol is (f, o~, 1) E, so LN1(x) = gamma * rs ((f, o~, 1, -mean) E) + beta
    // = r B with r = rs (f, o~, 1, -mean) and the beta row, and h1 Wm + bm = r V: P2's 256-deep
    // pass becomes two 32-deep ones over r (V, then B accumulated onto tanh: the residual h1),
    // and neither h1 nor its planes are formed.  LN1's statistics as layernorm() (one round).
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      float t = 0.f, q = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        t += (x[rb][4 * g] + x[rb][4 * g + 1]) + (x[rb][4 * g + 2] + x[rb][4 * g + 3]);
        q += (x[rb][4 * g] * x[rb][4 * g] + x[rb][4 * g + 1] * x[rb][4 * g + 1]) +
             (x[rb][4 * g + 2] * x[rb][4 * g + 2] + x[rb][4 * g + 3] * x[rb][4 * g + 3]);
      }
      t += __shfl_xor(t, 32, 64);
      q += __shfl_xor(q, 32, 64);
      if (lh == 0) {
        part[wid * CH_BM + 32 * rb + l32] = t;
        part[(CS_NW + wid) * CH_BM + 32 * rb + l32] = q;
      }
    }
    lbar();
    // row table (mean, rs) in plane 0's columns 32.. of each row (past the o~ columns)
    if (wid == 0 && lh == 0) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        float t = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < CS_NW; ++w) {
          t += part[w * CH_BM + 32 * rb + l32];
          q += part[(CS_NW + w) * CH_BM + 32 * rb + l32];
        }
        const float mean = t * (1.f / 256.f);
        const float var = fmaxf(q * (1.f / 256.f) - mean * mean, 0.f);
        *reinterpret_cast<float2*>(pl(0, 32 * rb + l32, 32)) = make_float2(mean, __builtin_amdgcn_rsqf(var + 1e-5f));
      }
    }
    lbar();
    // thread (row, j): r[j] for rows tid / 32 + 16 p; every read before any plane write
    constexpr int RP = CH_BM / 16;
    const int j = tid & 31;
    float rv[RP];
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const int r = (tid >> 5) + 16 * p, grow = min(row0 + r, rows - 1);
      const float2 st = *reinterpret_cast<const float2*>(pl(0, r, 32));  // mean, rs
      float z = 0.f;
      if (j < 4) {
        const float4 g = *reinterpret_cast<const float4*>(a.feat.geo + 4 * (size_t)grow);  // st ct sp cp
        z = j == 0 ? g.y : (j == 1 ? g.x * g.w : (j == 2 ? g.x * g.z : ((grow % a.feat.N < a.feat.n_up) ? 1.f : -1.f)));
      } else if (j < 24) {
        const int c = 8 * ((j - 4) / 5) + (j - 4) % 5;  // o~ column of (head, slot)
        const uint32_t h = *reinterpret_cast<const uint16_t*>(pl(0, r, c));
        const uint32_t m = *reinterpret_cast<const uint16_t*>(pl(1, r, c));
        const uint32_t l = *reinterpret_cast<const uint16_t*>(pl(2, r, c));
        z = (lo_f(h) + lo_f(m)) + lo_f(l);
      } else if (j == 24) {
        z = 1.f;
      } else if (j == 25) {
        z = -st.x;
      }
      rv[p] = j == 26 ? 1.f : st.y * z;  // row 26: the beta row (unscaled)
    }
    lbar();
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      const int r = (tid >> 5) + 16 * p;
      const float v = rv[p];
      const uint32_t h2 = pk_bf16(v, 0.f);
      const float rx = v - lo_f(h2);
      const uint32_t m2 = pk_bf16(rx, 0.f);
      const uint32_t l2 = pk_bf16(rx - lo_f(m2), 0.f);
      *reinterpret_cast<uint16_t*>(pl(0, r, j)) = (uint16_t)h2;
      *reinterpret_cast<uint16_t*>(pl(1, r, j)) = (uint16_t)m2;
      *reinterpret_cast<uint16_t*>(pl(2, r, j)) = (uint16_t)l2;
    }
    lbar();
    CHAIN_T(4);
    // ---- P2: h2 = LN2(h1 + tanh(h1 Wm + bm)) with h1 Wm + bm = r V, h1 = r B
    CHAIN_T(5);
    gemm(NoTr{}, K2{}, Zero{});
    prefetch(a.feat.L1B, a.ldp2, 0, K2{});
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[rb][e] = tanh_rat(acc[rb][e]);
    gemm(NoTr{}, K2{}, Accum{});
    CHAIN_T(6);
    if (a.Wp3 && 32 * wid < a.n3) prefetch(a.Wp3, a.ldp3, 0, K16{});
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int e = 0; e < 16; ++e) x[rb][e] = acc[rb][e];
  } else {
  layernorm(CHAIN_PRM ? prm : a.ln1);  // its barriers: every wave is past its GEMM reads of the planes
  CHAIN_T(4);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      put4(32 * rb + l32, colof(g), make_float4(x[rb][4 * g], x[rb][4 * g + 1], x[rb][4 * g + 2], x[rb][4 * g + 3]));
  lbar();
  // ---- P2: h2 = LN2(h1 + tanh(h1 Wm + bm)) -> planes and h
  CHAIN_T(5);
  gemm(NoTr{}, K16{}, Zero{});
  CHAIN_T(6);
  if (a.Wp3 && 32 * wid < a.n3) prefetch(a.Wp3, a.ldp3, 0, K16{});
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 bv = *reinterpret_cast<const float4*>((CHAIN_PRM ? prm + 512 : a.b2) + colof(g));
      const float4 h1 = get4(32 * rb + l32, colof(g));
#if CHAIN_TANH_EXP
      auto th = [](float z) { return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * z) + 1.f); };
#else
      auto th = [](float z) { return tanh_rat(z); };
#endif
      x[rb][4 * g] = h1.x + th(acc[rb][4 * g] + bv.x);
      x[rb][4 * g + 1] = h1.y + th(acc[rb][4 * g + 1] + bv.y);
      x[rb][4 * g + 2] = h1.z + th(acc[rb][4 * g + 2] + bv.z);
      x[rb][4 * g + 3] = h1.w + th(acc[rb][4 * g + 3] + bv.w);
    }
  }
  CHAIN_T(7);
  layernorm(CHAIN_PRM ? prm + 768 : a.ln2);
  CHAIN_T(8);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int r = row0 + 32 * rb + l32;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 y = make_float4(x[rb][4 * g], x[rb][4 * g + 1], x[rb][4 * g + 2], x[rb][4 * g + 3]);
      if (a.Wp3) put4(32 * rb + l32, colof(g), y);
      if (a.store_h && r < rows) *reinterpret_cast<float4*>(a.h + (size_t)r * CH_BN + colof(g)) = y;
    }
  }
  if (!a.Wp3) return;
  lbar();
  CHAIN_T(9);
  // ---- P3: Y3 = h2 W3 + b3, 256-column passes (a wave past n3 idles), MFMA-layout stores
  for (int col0 = 0; col0 < a.n3; col0 += CH_BN) {
    if (col0 + 32 * wid >= a.n3) continue;  // wave-uniform
    gemm(std::integral_constant<bool, CHAIN_P3T != 0>{}, K16{}, Zero{});
    if (col0 < 3 * CH_BN) CHAIN_T(10 + 2 * (col0 / CH_BN));
#if CHAIN_P3T
    {  // D[tile row][column]: reg q of acc[rb] = row 32 rb + (q & 3) + 8 (q >> 2) + 4 lh, column l32.
      // Buffer stores: the tile's rows as the resource, one 32-bit lane offset (past the range off
      // n3); full tiles put the row offset in soffset, the partial last tile in voffset
      const int c = col0 + 32 * wid + l32;
      const bool cok = c < a.n3;
      const float bv = cok ? a.b3[c] : 0.f;
      if (col0 + CH_BN + 32 * wid < a.n3) prefetch(a.Wp3, a.ldp3, col0 + CH_BN, K16{});
      const int nrow = min(CH_BM, rows - row0), ldb = a.ldy3 * 4;
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.Y3 + (size_t)row0 * a.ldy3, (short)0, nrow * ldb, 0x00020000);
      const int vo = cok ? 4 * lh * ldb + 4 * c : 0x7fffffff;
      if (nrow == CH_BM) {  // full tile: the row offset in soffset (every row inside the resource)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
          for (int q = 0; q < 16; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc[rb][q] + bv), rs, vo,
                                                  (32 * rb + (q & 3) + 8 * (q >> 2)) * ldb, 0);
        }
      } else {  // the last, partial tile: the raw-buffer range check covers voffset only (not
        // soffset), so the row goes into voffset and rows past the batch are out of range
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int r = 32 * rb + (q & 3) + 8 * (q >> 2) + 4 * lh;
            const int v = (cok && r < nrow) ? 4 * c + r * ldb : 0x7fffffff;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc[rb][q] + bv), rs, v, 0, 0);
          }
        }
      }
      if (col0 < 3 * CH_BN) CHAIN_T(11 + 2 * (col0 / CH_BN));
      continue;
    }
#endif
    // this lane's 16 bias values first (one wait), THEN the prefetch and the stores: a bias load
    // between two stores waits for every earlier store (vmcnt counts in order)
    float4 b3v[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = col0 + colof(g);
      b3v[g] = CHAIN_P3B && c + 3 < a.n3 ? *reinterpret_cast<const float4*>(a.b3 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (col0 + CH_BN + 32 * wid < a.n3) prefetch(a.Wp3, a.ldp3, col0 + CH_BN, K16{});
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int r = row0 + 32 * rb + l32;
      if (r >= rows) continue;
      float* yr = a.Y3 + (size_t)r * a.ldy3;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = col0 + colof(g);
        if (c + 3 < a.n3) {
          const float4 bv = CHAIN_P3B ? b3v[g] : *reinterpret_cast<const float4*>(a.b3 + c);
          *reinterpret_cast<float4*>(yr + c) = make_float4(acc[rb][4 * g] + bv.x, acc[rb][4 * g + 1] + bv.y,
                                                           acc[rb][4 * g + 2] + bv.z, acc[rb][4 * g + 3] + bv.w);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (c + e < a.n3) yr[c + e] = acc[rb][4 * g + e] + a.b3[c + e];
        }
      }
    }
    if (col0 < 3 * CH_BN) CHAIN_T(11 + 2 * (col0 / CH_BN));
  }
}


}  // namespace

int x6_plane_rows(int ncols) { return round_up(ncols, kRowPad) + kRowPad; }

void launch_split_planes(const float* Wt, int ldw, int ncols, int K, uint16_t* Wp, hipStream_t s) {
  const int ldp = x6_plane_rows(ncols);
  const size_t n = (size_t)ldp * K;
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, Wt, ldw, ncols, K, ldp,
                     Wp);
}

bool gemm_x6_supported(int K) { return K % X6_BK == 0; }

void launch_gemm_x6_variant(int v, const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias,
                            const float* R, int ldr, float* Y, int ldy, int rows, int ncols, int K, int C,
                            hipStream_t s) {
  switch (v) {
    case 1:
      launch_x6_t<4, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 2:
      launch_x6_t<4, 8>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 3:
      launch_x6_t<8, 6>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 4:
      launch_x6_t<4, 6>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 5:
      launch_x6_t<2, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 6:
      launch_x6_t<2, 8>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 7:
      launch_x6_t<8, 2>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // persistent, weight panel resident in LDS (K <= 256)
    case 10:
      launch_x6p_t<8>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 11:
      launch_x6p_t<12>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 12:
      launch_x6p_t<16>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 13:
      launch_x6p_t<4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // big tiles 256 x 64*TN, BK = 16
    case 20:
      launch_x6b_t<4, 3>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 21:
      launch_x6b_t<4, 2>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 22:
      launch_x6b_t<3, 3>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 23:
      launch_x6b_t<2, 3>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // pipelined 256 x 32*TN
    case 30:
      launch_x6c_t<8>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 31:
      launch_x6c_t<6>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 32:
      launch_x6c_t<4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // lean pipelined 256 x 32*TN
    case 40:
      launch_x6d_t<8>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 41:
      launch_x6d_t<6>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 42:
      launch_x6d_t<4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // two workgroups per CU: 128 x 32*TN tiles, two buffers
    case 43:
      launch_x6d_t<8, 0, 4, 2>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 44:
      launch_x6d_t<6, 0, 4, 2>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 45:
      launch_x6d_t<4, 0, 4, 2>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 46:
      launch_x6d_t<4, 0, 8, 2>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // 2-D wave grids, 256-column tiles (ncols % 4 == 0): 96 x 256 of 3 x 4 waves (when
    // round_up(rows, 96) stays inside round_up(rows, 256), else 64 x 256), 64 x 256 of
    // 2 x 4 waves, 128 x 256 of 4 x 4 waves
    case 60:
      if (round_up(rows, 96) <= round_up(rows, 256)) {
        launch_x6d_t<2, 0, 3, 3, 0, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
        break;
      }
      [[fallthrough]];
    case 61:
      launch_x6d_t<2, 0, 2, 3, 0, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 62:
      launch_x6d_t<2, 0, 4, 3, 0, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // deeper rings (ST - 2 stages in flight): 96 x 256 of 3 x 4 waves, 128 x 192 / 256 x 128
    case 70:
      if (round_up(rows, 96) <= round_up(rows, 256)) {
        launch_x6d_t<2, 0, 3, 5, 0, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
        break;
      }
      [[fallthrough]];
    case 71:
      launch_x6d_t<6, 0, 4, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 72:
      launch_x6d_t<6, 0, 4, 5>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 73:
      launch_x6d_t<4, 0, 8, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 74:
      launch_x6d_t<8, 0, 4, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 75:
      launch_x6d_t<4, 0, 4, 5>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // persistent lean
    case 50:
      launch_x6q_t<8>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 51:
      launch_x6q_t<6>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 52:
      launch_x6q_t<4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // persistent lean, 4-stage ring (two stages in flight)
    case 53:
      launch_x6q_t<8, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 55:
      launch_x6q_t<5>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // persistent lean with the B fragment reads pipelined one column block ahead
    case 56:
      launch_x6q_t<8, false, 0, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 57:
      launch_x6q_t<6, false, 0, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 58:
      launch_x6q_t<5, false, 0, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // persistent 16x16x32 form, 2-D wave grid (round 3)
    case 80:
      launch_x6m_t<8>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 81:
      launch_x6m_t<6>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 82:
      launch_x6m_t<5>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 83:
      launch_x6m_t<4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 84:
      launch_x6m_t<8, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 85:
      launch_x6m_t<6, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 76:  // DMA from the column-half-0 waves only
      launch_x6m_t<8, false, 0, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 77:
      launch_x6m_t<6, false, 0, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 78:  // DMA4 + spread issue
      launch_x6m_t<8, true, 0, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 79:
      launch_x6m_t<4, false, 0, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 90:
      launch_x6m_t<5, false, 0, true>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // ablations of 80 (wrong results; tools/gemm_bench.py only): cumulative
    case 86:
      launch_x6m_t<8, false, 1>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 87:
      launch_x6m_t<8, false, 3>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 88:
      launch_x6m_t<8, false, 7>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 89:
      launch_x6m_t<8, false, 15>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 95:  // ablation of 50: no epilogue stores (wrong results; tools/gemm_bench.py only)
      launch_x6q_t<8, false, 1>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;

    // ablations of variant 40 (wrong results; tools/gemm_bench.py only)
    case 91:
      launch_x6d_t<8, 1>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 92:
      launch_x6d_t<8, 2>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 93:
      launch_x6d_t<8, 3>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 94:
      launch_x6d_t<8, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    default:
      launch_x6_t<8, 4>(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
  }
}

void launch_gemm_x6(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* R, int ldr,
                    float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  // measured on MI355X (tools/gemm_bench.py, K = 256): channel rows take the persistent lean
  // kernel with 256 x 256 tiles (256 x 192 when ncols is a multiple of 192 only); short
  // (log-psi) row counts take 256 x 128 tiles, two workgroups per CU (128 x 192 when ncols
  // is a multiple of 192: q|k|v 24576 x 768 in 64 vs 68 us).  The 2-D wave grids (60-62)
  // were no faster at these shapes (tools/ln_gemm_bench.py).
  // Channel rows: below 1024 columns the width with the least padding (C4's orbital map,
  // 480 columns: 256-wide 2125 us, 192-wide 1816 us, 160-wide 1628 us; tools/gemm_orb_bench.py),
  // else 256 (C5's 2320 columns: 12.9 ms against 13.8 ms 160-wide); the B fragment reads
  // pipelined one column block ahead (56-58: el_qkv 968 -> 932 us, tools/gemm_bench.py)
  // Round 3: the 16x16x32 two-dimensional wave-grid form (gemm_x6m, DMA from the
  // column-half-0 waves) for the wide maps — C2 q|k|v 417792 x 768: 950 -> 877 us, the
  // 192-column orbital map 361 -> 252 us; the single 256-column tile row (Wol, Wm: 1632
  // tiles over 256 CUs) stays on gemm_x6q (394 vs 404 us).
  int v;
  if (rows >= 65536 && ncols % 256 == 0 && ncols >= 512) {
    v = 76;
  } else if (rows >= 65536 && ncols == 192) {
    v = 77;
  } else if (rows >= 65536) {
    v = 56;
    if (ncols < 1024) {
      const int tns[4] = {8, 6, 5, 4}, vs[4] = {56, 57, 58, 52};
      int best = round_up(ncols, 256);
      for (int q = 1; q < 4; ++q) {
        const int padded = round_up(ncols, 32 * tns[q]);
        if (padded < best) {
          best = padded;
          v = vs[q];
        }
      }
    }
  } else {
    v = (ncols % 192 == 0) ? 44 : 46;
  }
  launch_gemm_x6_variant(v, X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
}


// log-psi GEMM + LayerNorm (LNM 1 / 2 above), in place over h [rows][256].  Form nw:
//   0 = choose; 3 / 4 = 96 / 128-row tiles of 32 x 256 wave blocks (3 / 4 waves);
//   1 = 96-row tiles of 3 x 4 waves with 32 x 64 blocks (12 waves, all four SIMDs busy);
//   2 = 64-row tiles of 2 x 4 waves; 8 = 128-row tiles of 4 x 4 waves.
// One workgroup per CU (LDS).  Callers pad X and h to kWalkerRowPad (768 = lcm(96, 256))
// rows, so no tile reads past them.
void launch_gemm_x6_ln(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* ln,
                       float* h, int rows, int K, int mode, int nw, hipStream_t s, X6Feat feat) {
  if (mode != 0) feat = X6Feat{};
  if (nw >= 32) {  // tools/ln_gemm_bench.py only: ablations / forced forms (caller pads rows to 768)
    switch (nw) {
#define DH_X6LN_A(TNV, NWV, WNV, ABLV)                                                                      \
  launch_x6d_t<TNV, ABLV, NWV, 3, 2, WNV>(X, ldx, Wp, ldp, bias, h, 256, h, 256, rows, 256, K, 1, s, ln)
      case 32: DH_X6LN_A(2, 2, 4, 1); break;
      case 33: DH_X6LN_A(2, 2, 4, 2); break;
      case 34: DH_X6LN_A(2, 2, 4, 3); break;
      case 35: DH_X6LN_A(2, 2, 4, 4); break;
      case 36: DH_X6LN_A(2, 3, 4, 0); break;
      case 37: DH_X6LN_A(2, 3, 4, 4); break;
      case 38: DH_X6LN_A(2, 4, 4, 0); break;
      case 39: DH_X6LN_A(2, 4, 4, 4); break;
      case 40: DH_X6LN_A(2, 2, 4, 5); break;
      case 41: DH_X6LN_A(2, 3, 4, 5); break;
      case 42: DH_X6LN_A(2, 3, 4, 6); break;
      case 43: DH_X6LN_A(2, 3, 4, 7); break;
#undef DH_X6LN_A
    }
    return;
  }
  if (nw == 0) {
    // one workgroup per CU: the launch runs in rounds of cu_count tiles, so take the tile
    // height with the least rounds x per-round time (MI355X, tools/ln_gemm_ablate.py:
    // 64 / 96 / 128-row tiles ~23 / 28 / 30.5 us a round at K = 256; C2 24576 rows -> 96,
    // C4 40960 -> 96, C5 81920 -> 128)
    const int cus = cu_count_x6();
    const int bm[3] = {96, 128, 64}, cost[3] = {280, 305, 230}, form[3] = {1, 8, 2};
    long best = -1;
    for (int q = 0; q < 3; ++q) {
      const long t = (long)(((rows + bm[q] - 1) / bm[q] + cus - 1) / cus) * cost[q];
      if (best < 0 || t < best) {
        best = t;
        nw = form[q];
      }
    }
  }
  if (nw < 1 || nw > 8) nw = 1;
#define DH_X6LN_ST(TNV, NWV, WNV, STV)                                                                      \
  do {                                                                                                      \
    if (mode == 0)                                                                                          \
      launch_x6d_t<TNV, 0, NWV, STV, 1, WNV>(X, ldx, Wp, ldp, bias, h, 256, h, 256, rows, 256, K, 1, s, ln, feat); \
    else                                                                                                    \
      launch_x6d_t<TNV, 0, NWV, STV, 2, WNV>(X, ldx, Wp, ldp, bias, h, 256, h, 256, rows, 256, K, 1, s, ln); \
  } while (0)
#define DH_X6LN(TNV, NWV, WNV)                                                                              \
  do {                                                                                                      \
    if (mode == 0)                                                                                          \
      launch_x6d_t<TNV, 0, NWV, 3, 1, WNV>(X, ldx, Wp, ldp, bias, h, 256, h, 256, rows, 256, K, 1, s, ln, feat); \
    else                                                                                                    \
      launch_x6d_t<TNV, 0, NWV, 3, 2, WNV>(X, ldx, Wp, ldp, bias, h, 256, h, 256, rows, 256, K, 1, s, ln); \
  } while (0)
  switch (nw) {
    case 1: DH_X6LN(2, 3, 4); break;
    case 2: DH_X6LN(2, 2, 4); break;
    case 3: DH_X6LN(8, 3, 1); break;
    case 5: DH_X6LN_ST(2, 3, 4, 5); break;
    case 6: DH_X6LN_ST(2, 3, 4, 4); break;
    case 7: DH_X6LN_ST(2, 2, 4, 5); break;
    case 8: DH_X6LN(2, 4, 4); break;
    default: DH_X6LN(8, 4, 1);
  }
#undef DH_X6LN
#undef DH_X6LN_ST
}

// Chained log-psi layer tail (chain_x6s_kernel above).  X1 and h padded to kWalkerRowPad
// rows; Wp3 may be null (no P3); Y3 rows 16-B aligned (ldy3 % 4 == 0).  feat.W0qkv (layer 1,
// chain_attn_supported): the attention runs in the prologue and Wp1 holds the planes of U^T
// (K = CH_KO), else Wp1 contracts X1 = o over 256.
void launch_chain_x6(const float* X1, const uint16_t* Wp1, int ldp1, const float* b1, const float* ln1,
                     const uint16_t* Wp2, int ldp2, const float* b2, const float* ln2, const uint16_t* Wp3, int ldp3,
                     const float* b3, int n3, float* Y3, int ldy3, float* h, int rows, X6Feat feat, hipStream_t s,
                     bool store_h) {
  ChainArgs a{X1, Wp1, Wp2, Wp3, ldp1, ldp2, ldp3, b1, ln1, b2, ln2, b3, n3, ldy3, Y3, h, rows, feat, store_h ? 1 : 0};
  auto k = chain_x6s_kernel<0>;
  if (feat.W0qkv) {  // chain_attn_supported(feat.N, 4, 64) checked by the caller
    switch (feat.N) {
      case 2: k = chain_x6s_kernel<2>; break;
      case 3: k = chain_x6s_kernel<3>; break;
      case 4: k = chain_x6s_kernel<4>; break;
      case 6: k = chain_x6s_kernel<6>; break;
      case 8: k = chain_x6s_kernel<8>; break;
      case 10: k = chain_x6s_kernel<10>; break;
      default: k = chain_x6s_kernel<20>; break;
    }
  }
  const int trw = feat.W0qkv ? (CH_BM / feat.N) * feat.N : CH_BM;  // the kernel's TRW
  ensure_smem(k, CS_SMEM);
  hipLaunchKernelGGL(k, dim3((rows + trw - 1) / trw), dim3(512), CS_SMEM, s, a);
}

// Layer 1's attention inside the chain prologue (chain_x6s_kernel<N>): walker-aligned 96-row
// tiles, 4 heads of 64 (one per wave pair)
bool chain_attn_supported(int N, int H, int dh) {
  return H == 4 && dh == 64 && (N == 2 || N == 3 || N == 4 || N == 6 || N == 8 || N == 10 || N == 20);
}

}  // namespace dh
