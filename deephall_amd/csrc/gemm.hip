// f32 GEMM on CDNA4 matrix cores (v_mfma_f32_32x32x2_f32: exact f32, 256 FLOP/clk/CU).
//
//   Y[r][n] = sum_k X[r][k] W[k][n]  + (r % C == 0 ? bias[n] : 0)  + (R ? R[r][n] : 0)
//
// Used for every linear map of the Psiformer (psiformer.py:42-47 Dense /
// MultiHeadAttention projections, blocks.py:29-35 orbital DenseGeneral) applied to
// all channel rows at once: rows are (walker, electron, channel) triples, so the
// bias only goes to channel-0 (value) rows — tangents and second-order channels
// of an affine map carry no bias.
//
// Tile BM x BN per workgroup of (BM/WM) x (BN/WN) waves; each wave owns WM x WN =
// (WM/32) x (WN/32) MFMA 32x32 accumulators.  K is staged in BK slices through a
// register-staged LDS double buffer.  A is stored transposed in LDS (As[k][m]) so the
// MFMA A operand (lane l holds A[l&31][l>>5]) is a conflict-free ds_read_b32 row read.
#include "dh_internal.h"
#include "device_common.h"

namespace dh {

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {
constexpr int PAD = 4;

template <int BM, int BN, int BK, int WM, int WN>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64) void gemm_f32_kernel(
    const float* __restrict__ X, int ldx, const float* __restrict__ W, int ldw, const float* __restrict__ bias,
    const float* R, int ldr, float* Y, int ldy, int rows, int ncols, int K, int C, int ntm, int ntn) {
  constexpr int NWN = BN / WN, NT = (BM / WM) * NWN * 64;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int NA4 = BM * BK / 4, NB4 = BK * BN / 4;  // float4 per tile
  constexpr int A4 = (NA4 + NT - 1) / NT, B4 = (NB4 + NT - 1) / NT;
  __shared__ float As[2][BK][BM + PAD];
  __shared__ float Bs[2][BK][BN + PAD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / NWN, wn = wid % NWN;

  // XCD-aware tile order: blocks b and b+8 share an XCD (round-robin dispatch),
  // so give consecutive tiles of one row panel (same A rows) to one XCD.
  const int nblk = ntm * ntn;
  int bid = blockIdx.x;
  {
    const int q = nblk / 8, r8 = nblk % 8, xcd = bid % 8, slot = bid / 8;
    bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
  }
  const int tm = bid / ntn, tn = bid % ntn;
  const int row0 = tm * BM, col0 = tn * BN;

  float4 ra[A4], rb[B4];
  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int q = tid + i * NT;
      if (NA4 % NT != 0 && q >= NA4) break;
      const int r = q / (BK / 4);
      const int k = k0 + (q % (BK / 4)) * 4;
      const float* src = X + (size_t)(row0 + r) * ldx + k;
      if (k + 4 <= K) {
        ra[i] = *reinterpret_cast<const float4*>(src);
      } else {
        ra[i].x = (k + 0 < K) ? src[0] : 0.f;
        ra[i].y = (k + 1 < K) ? src[1] : 0.f;
        ra[i].z = (k + 2 < K) ? src[2] : 0.f;
        ra[i].w = (k + 3 < K) ? src[3] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < B4; ++i) {
      const int q = tid + i * NT;
      if (NB4 % NT != 0 && q >= NB4) break;
      const int kb = k0 + q / (BN / 4);
      const int n = col0 + (q % (BN / 4)) * 4;
      const float* wsrc = W + (size_t)kb * ldw + n;
      if (kb < K && n + 4 <= ncols) {
        rb[i] = *reinterpret_cast<const float4*>(wsrc);
      } else {
        rb[i].x = (kb < K && n + 0 < ncols) ? wsrc[0] : 0.f;
        rb[i].y = (kb < K && n + 1 < ncols) ? wsrc[1] : 0.f;
        rb[i].z = (kb < K && n + 2 < ncols) ? wsrc[2] : 0.f;
        rb[i].w = (kb < K && n + 3 < ncols) ? wsrc[3] : 0.f;
      }
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int q = tid + i * NT;
      if (NA4 % NT != 0 && q >= NA4) break;
      const int r = q / (BK / 4);
      const int kk = (q % (BK / 4)) * 4;
      As[buf][kk + 0][r] = ra[i].x;
      As[buf][kk + 1][r] = ra[i].y;
      As[buf][kk + 2][r] = ra[i].z;
      As[buf][kk + 3][r] = ra[i].w;
    }
#pragma unroll
    for (int i = 0; i < B4; ++i) {
      const int q = tid + i * NT;
      if (NB4 % NT != 0 && q >= NB4) break;
      *reinterpret_cast<float4*>(&Bs[buf][q / (BN / 4)][(q % (BN / 4)) * 4]) = rb[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int nk = (K + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int l32 = lane & 31, lh = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int ka = kk + lh;
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[cur][ka][wm * WM + i * 32 + l32];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[cur][ka][wn * WN + j * 32 + l32];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // Epilogue. C/D map of 32x32 MFMA: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int rbase = row0 + wm * WM + mi * 32 + 4 * lh;
    const int rm0 = (C == 1) ? 0 : rbase % C;
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int c = col0 + wn * WN + ni * 32 + l32;
      if (c >= ncols) continue;
      const float bv = bias ? bias[c] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int off = (e & 3) + 8 * (e >> 2);
        const int r = rbase + off;
        if (r >= rows) continue;
        float v = acc[mi][ni][e];
        if (bias) {
          bool val = true;
          if (C > 1) {
            int t = rm0 + off;
            while (t >= C) t -= C;
            val = (t == 0);
          }
          if (val) v += bv;
        }
        if (R) v += R[(size_t)r * ldr + c];
        Y[(size_t)r * ldy + c] = v;
      }
    }
  }
}

// ---- NT form: Y = X Wt^T with the weight stored transposed, Wt[n][k] --------------------
// Both operands are row-major with k contiguous, so both tiles are staged by
// global_load_lds_dwordx4 (LDS-DMA: no staging VGPRs, no ds_write) into one LDS image of
// BK = 32 floats (128 B) per row, 16-B slots XOR-swizzled by (row >> 1) & 7 on the SOURCE
// address (the DMA destination is lane-linear).  Fragments are read with ds_read_b128:
// lane (l32, lh) of a 32-row sub-tile takes k = 8g + 4lh + j, j = 0..3, for four
// consecutive MFMA k-steps (the same bijective k labelling on A and B, so the contraction
// is exact; only the f32 summation order differs from a k-ordered chain).  Conflict-free:
// each ds_read_b128 lane group reads 16 distinct rows mod 16 -> 16 distinct slots.
// Requirements (checked by the launcher): K % 32 == 0; X has round_up(rows, BM) readable
// rows; Wt has round_up(ncols, BN) readable rows.
constexpr int NT_BK = 32;

template <int BM, int BN, int WM, int WN, bool HAS_R, int STAGES>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64) void gemm_nt_kernel(
    const float* __restrict__ X, int ldx, const float* __restrict__ Wt, int ldw, const float* __restrict__ bias,
    const float* R, int ldr, float* Y, int ldy, int rows, int ncols, int K, int C, int ntm, int ntn) {
  constexpr int NWN = BN / WN, NW = (BM / WM) * NWN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int BK = NT_BK, STAGE = (BM + BN) * BK;  // floats per LDS stage
  constexpr int IA = BM / 8, IB = BN / 8;            // DMA wave-instructions per tile (8 rows each)
  static_assert(BK == 32, "slot swizzle assumes 8 slots of 16 B per row");
  extern __shared__ float4 smem4[];
  float* smem = reinterpret_cast<float*>(smem4);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NWN, wn = wid % NWN;

  const int nblk = ntm * ntn;
  int bid = blockIdx.x;
  {
    const int q = nblk / 8, r8 = nblk % 8, xcd = bid % 8, slot = bid / 8;
    bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
  }
  const int tm = bid / ntn, tn = bid % ntn;
  const int row0 = tm * BM, col0 = tn * BN;

  // per-lane DMA source for an 8-row group: row = L / 8, logical slot = (L % 8) ^ ((row >> 1) & 7)
  const int lr = lane >> 3;
  auto src_slot = [&](int r) { return ((lane & 7) ^ ((r >> 1) & 7)) * 4; };
  static_assert((IA + IB) % NW == 0, "DMA instructions must divide evenly over the waves");
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) float*)smem);
  auto stage = [&](int k0, int buf) {
#pragma unroll
    for (int t = 0; t < (IA + IB) / NW; ++t) {
      const int j = wid + t * NW;  // wave-uniform
      const bool isA = j < IA;
      const int rg = (isA ? j : j - IA) * 8;  // first row of the 8-row group
      const int r = rg + lr;
      const float* src = isA ? X + (size_t)(row0 + r) * ldx + k0 + src_slot(r)
                             : Wt + (size_t)(col0 + r) * ldw + k0 + src_slot(r);
      const uint32_t dst = __builtin_amdgcn_readfirstlane(
          lds0 + 4u * (uint32_t)(buf * STAGE + (isA ? 0 : BM * BK) + rg * BK));
      // LDS-DMA in inline asm: hipcc neither counts it nor inserts a vmcnt(0) before the
      // next ds_read of the OTHER buffer; completion is waited for explicitly below.
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(dst)
                   : "memory");
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int l32 = lane & 31, lh = lane >> 5;
  const int nk = K / BK;
  float rres[TM][TN][16];
  // STAGES-deep ring: tile kt+STAGES-1 is issued while tile kt is consumed.  Each wave
  // issues PER DMA instructions per tile; VMEM completes in order, so "tile kt landed"
  // is vmcnt(PER * tiles issued after it).  The barrier then publishes the whole tile.
  constexpr int PER = (IA + IB) / NW;
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
    if (HAS_R && kt + 1 == nk) {  // residual loads overlap the last k-tile's MFMAs
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int c = col0 + wn * WN + ni * 32 + l32;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int r = row0 + wm * WM + mi * 32 + 4 * lh + (e & 3) + 8 * (e >> 2);
            rres[mi][ni][e] = (c < ncols && r < rows) ? R[(size_t)r * ldr + c] : 0.f;
          }
        }
    }
    const float* As = smem + cur * STAGE;
    const float* Bs = As + BM * BK;
    if (++cur == STAGES) cur = 0;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      const int s = 2 * g + lh;
      float4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = wm * WM + i * 32 + l32;
        a[i] = *reinterpret_cast<const float4*>(As + m * BK + ((s ^ ((m >> 1) & 7)) * 4));
      }
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int n = wn * WN + i * 32 + l32;
        b[i] = *reinterpret_cast<const float4*>(Bs + n * BK + ((s ^ ((n >> 1) & 7)) * 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
        }
    }
  }

#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int rbase = row0 + wm * WM + mi * 32 + 4 * lh;
    const int rm0 = (C == 1) ? 0 : rbase % C;
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int c = col0 + wn * WN + ni * 32 + l32;
      if (c >= ncols) continue;
      const float bv = bias ? bias[c] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int off = (e & 3) + 8 * (e >> 2);
        const int r = rbase + off;
        if (r >= rows) continue;
        float v = acc[mi][ni][e];
        if (bias) {
          bool val = true;
          if (C > 1) {
            int t = rm0 + off;
            while (t >= C) t -= C;
            val = (t == 0);
          }
          if (val) v += bv;
        }
        if (HAS_R) v += rres[mi][ni][e];
        Y[(size_t)r * ldy + c] = v;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int STAGES = 2>
void launch_nt(const float* X, int ldx, const float* Wt, int ldw, const float* bias, const float* R, int ldr,
               float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const size_t smem = (size_t)STAGES * (BM + BN) * NT_BK * sizeof(float);
  if (R) {
    ensure_smem(gemm_nt_kernel<BM, BN, WM, WN, true, STAGES>, smem);
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, true, STAGES>), dim3(ntm * ntn), dim3(NT), smem, s, X, ldx, Wt, ldw,
                       bias, R, ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
  } else {
    ensure_smem(gemm_nt_kernel<BM, BN, WM, WN, false, STAGES>, smem);
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, false, STAGES>), dim3(ntm * ntn), dim3(NT), smem, s, X, ldx, Wt, ldw,
                       bias, R, ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
  }
}

// ---- persistent NT GEMM: one continuous LDS-DMA ring across all of a workgroup's tiles ----
// gemm_nt_kernel idles the matrix cores at every tile boundary (prologue load, epilogue
// stores) and the co-resident workgroups of a CU start in step, so the idle periods line
// up.  Here each workgroup walks tiles blockIdx.x, +gridDim.x, ... and the (tile, k-tile)
// steps form ONE stream: the next tile's first k-tiles are in flight while the current
// tile finishes and its accumulators are stored.
// Stores are unconditional (no row / column guards), so that every wave issues exactly
// NST = TM*TN*16 of them per tile and the counted vmcnt waits stay exact (VMEM ops of a
// wave complete in order): Y must have round_up(rows, BM) rows and ldy >= round_up(ncols,
// BN); rows and columns past (rows, ncols) receive padding garbage.  The bias is read
// only for c < ncols.
template <int BM, int BN, int WM, int WN, bool HAS_R, int STAGES>
__global__ __launch_bounds__((BM / WM) * (BN / WN) * 64) void gemm_ntp_kernel(
    const float* __restrict__ X, int ldx, const float* __restrict__ Wt, int ldw, const float* __restrict__ bias,
    const float* R, int ldr, float* Y, int ldy, int ncols, int K, int C, int ntm, int ntn) {
  constexpr int NWN = BN / WN, NW = (BM / WM) * NWN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int BK = NT_BK, STAGE = (BM + BN) * BK;
  constexpr int IA = BM / 8, IB = BN / 8, PER = (IA + IB) / NW, NST = TM * TN * 16;
  static_assert((IA + IB) % NW == 0, "DMA instructions must divide evenly over the waves");
  static_assert(STAGES == 2 || STAGES == 3, "ring depth");
  static_assert(PER + NST <= 63, "vmcnt range");
  extern __shared__ float4 smem4[];
  float* smem = reinterpret_cast<float*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NWN, wn = wid % NWN;
  const int l32 = lane & 31, lh = lane >> 5, lr = lane >> 3;
  const int nblk = ntm * ntn, G = gridDim.x;
  const int my_tiles = (nblk - (int)blockIdx.x + G - 1) / G;
  const int nk = K / BK, F = my_tiles * nk;
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) float*)smem);
  // XCD-aware order (as gemm_nt_kernel; G is a multiple of 8 so a workgroup keeps its XCD)
  auto tile_of = [&](int i, int& row0, int& col0) {
    const int idx = blockIdx.x + i * G;
    const int q = nblk / 8, r8 = nblk % 8, xcd = idx % 8, slot = idx / 8;
    const int bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + slot;
    row0 = (bid / ntn) * BM;
    col0 = (bid % ntn) * BN;
  };
  auto stage = [&](int f, int buf) {
    int row0, col0;
    tile_of(f / nk, row0, col0);
    const int k0 = (f % nk) * BK;
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int j = wid + t * NW;
      const bool isA = j < IA;
      const int rg = (isA ? j : j - IA) * 8;
      const int r = rg + lr;
      const int sl = ((lane & 7) ^ ((r >> 1) & 7)) * 4;
      const float* src = isA ? X + (size_t)(row0 + r) * ldx + k0 + sl : Wt + (size_t)(col0 + r) * ldw + k0 + sl;
      const uint32_t dst =
          __builtin_amdgcn_readfirstlane(lds0 + 4u * (uint32_t)(buf * STAGE + (isA ? 0 : BM * BK) + rg * BK));
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(dst)
                   : "memory");
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  float rres[TM][TN][16];

#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < F) stage(t, t);
  int cur = 0, kt = 0, tile = 0;
  bool stored = false;  // stores issued in the previous iteration (younger than this step's DMA)
  for (int f = 0; f < F; ++f) {
    // wait for step f: younger VMEM ops = DMA of steps f+1 .. f+STAGES-2 (if any) + the
    // previous iteration's epilogue stores
    const bool dma_after = STAGES == 3 && f + 1 < F;
    if (dma_after && stored)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER + NST) : "memory");
    else if (dma_after)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
    else if (stored)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NST) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the step's LDS image is complete; the buffer being refilled is free
    asm volatile("" ::: "memory");
    if (f + STAGES - 1 < F) {
      int nb = cur + STAGES - 1;
      if (nb >= STAGES) nb -= STAGES;
      stage(f + STAGES - 1, nb);
    }
    int row0, col0;
    tile_of(tile, row0, col0);
    if (HAS_R && kt + 1 == nk) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int c = col0 + wn * WN + ni * 32 + l32;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int r = row0 + wm * WM + mi * 32 + 4 * lh + (e & 3) + 8 * (e >> 2);
            rres[mi][ni][e] = R[(size_t)r * ldr + c];
          }
        }
    }
    const float* As = smem + cur * STAGE;
    const float* Bs = As + BM * BK;
    if (++cur == STAGES) cur = 0;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      const int s = 2 * g + lh;
      float4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = wm * WM + i * 32 + l32;
        a[i] = *reinterpret_cast<const float4*>(As + m * BK + ((s ^ ((m >> 1) & 7)) * 4));
      }
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int n = wn * WN + i * 32 + l32;
        b[i] = *reinterpret_cast<const float4*>(Bs + n * BK + ((s ^ ((n >> 1) & 7)) * 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
        }
    }
    stored = false;
    if (++kt == nk) {  // tile done: epilogue (all NST stores issued by every wave)
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int rbase = row0 + wm * WM + mi * 32 + 4 * lh;
        const int rm0 = (C == 1) ? 0 : rbase % C;
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int c = col0 + wn * WN + ni * 32 + l32;
          const float bv = (bias && c < ncols) ? bias[c] : 0.f;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int off = (e & 3) + 8 * (e >> 2);
            float v = acc[mi][ni][e];
            if (C > 1) {
              int t = rm0 + off;
              while (t >= C) t -= C;
              if (t == 0) v += bv;
            } else {
              v += bv;
            }
            if (HAS_R) v += rres[mi][ni][e];
            Y[(size_t)(rbase + off) * ldy + c] = v;
            acc[mi][ni][e] = 0.f;
          }
        }
      }
      stored = true;
      kt = 0;
      ++tile;
    }
  }
}

int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <int BM, int BN, int WM, int WN, int STAGES, int PER_CU>
void launch_ntp(const float* X, int ldx, const float* Wt, int ldw, const float* bias, const float* R, int ldr,
                float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  const size_t smem = (size_t)STAGES * (BM + BN) * NT_BK * sizeof(float);
  int grid = std::min(ntm * ntn, PER_CU * cu_count());
  grid = std::max(8, grid / 8 * 8);  // a multiple of 8: each workgroup keeps one XCD
  if (R) {
    ensure_smem(gemm_ntp_kernel<BM, BN, WM, WN, true, STAGES>, smem);
    hipLaunchKernelGGL((gemm_ntp_kernel<BM, BN, WM, WN, true, STAGES>), dim3(grid), dim3(NT), smem, s, X, ldx, Wt,
                       ldw, bias, R, ldr, Y, ldy, ncols, K, C, ntm, ntn);
  } else {
    ensure_smem(gemm_ntp_kernel<BM, BN, WM, WN, false, STAGES>, smem);
    hipLaunchKernelGGL((gemm_ntp_kernel<BM, BN, WM, WN, false, STAGES>), dim3(grid), dim3(NT), smem, s, X, ldx, Wt,
                       ldw, bias, R, ldr, Y, ldy, ncols, K, C, ntm, ntn);
  }
}

// ---- log-psi rows: GEMM with the LayerNorm fused into the epilogue --------------------
// One workgroup owns BM whole rows (all D = 256 output columns), so the row statistics of
// the LayerNorm that follows the GEMM are workgroup-local:
//   MODE 0:  h = LN(h + X Wt^T + b)          (psiformer.py:44-45, residual + LN)
//   MODE 1:  h = LN(h + tanh(X Wt^T + b))    (psiformer.py:46-47, MLP + residual + LN)
// written in place over h (R == Y): each workgroup reads only its own rows of h (as the
// residual, and as X in MODE 1), all before the first barrier of the epilogue.
// Waves: (BM/32) x 4, each a 32 x 64 sub-tile.  Staging as gemm_nt_kernel (two stages).
// LayerNorm numerics as layernorm_value_kernel: two-pass mean / centred variance, eps 1e-5.
template <int BM, int MODE>
__global__ __launch_bounds__(BM * 8) void gemm_ln_kernel(const float* X, int ldx, const float* __restrict__ Wt, int ldw,
                                                         const float* __restrict__ bias, const float* __restrict__ ln,
                                                         float* h, int rows, int K) {
  constexpr int BN = 256, WM = 32, WN = 64, NWN = 4, NW = (BM / 32) * NWN, TN = 2;
  constexpr int BK = NT_BK, STAGE = (BM + BN) * BK;
  constexpr int IA = BM / 8, IB = BN / 8, PERW = (IA + IB + NW - 1) / NW;
  extern __shared__ float4 smem4[];
  float* smem = reinterpret_cast<float*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NWN, wn = wid % NWN;
  const int row0 = blockIdx.x * BM;
  const int lr = lane >> 3;
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) float*)smem);
  auto stage = [&](int k0, int buf) {
#pragma unroll
    for (int t = 0; t < PERW; ++t) {
      const int j = wid + t * NW;
      if (j >= IA + IB) break;  // wave-uniform
      const bool isA = j < IA;
      const int rg = (isA ? j : j - IA) * 8;
      const int r = rg + lr;
      const int sl = ((lane & 7) ^ ((r >> 1) & 7)) * 4;
      const float* src = isA ? X + (size_t)(row0 + r) * ldx + k0 + sl : Wt + (size_t)r * ldw + k0 + sl;
      const uint32_t dst =
          __builtin_amdgcn_readfirstlane(lds0 + 4u * (uint32_t)(buf * STAGE + (isA ? 0 : BM * BK) + rg * BK));
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
  const int l32 = lane & 31, lh = lane >> 5;
  const int nk = K / BK;
  float rres[TN][16];
  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) stage((kt + 1) * BK, cur ^ 1);
    if (kt + 1 == nk) {  // residual rows of h, overlapping the last k-tile
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int c = wn * WN + ni * 32 + l32;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = row0 + wm * WM + 4 * lh + (e & 3) + 8 * (e >> 2);
          rres[ni][e] = (r < rows) ? h[(size_t)r * BN + c] : 0.f;
        }
      }
    }
    const float* As = smem + cur * STAGE;
    const float* Bs = As + BM * BK;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      const int s = 2 * g + lh;
      const int m = wm * WM + l32;
      const float4 a = *reinterpret_cast<const float4*>(As + m * BK + ((s ^ ((m >> 1) & 7)) * 4));
      float4 b[TN];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int n = wn * WN + i * 32 + l32;
        b[i] = *reinterpret_cast<const float4*>(Bs + n * BK + ((s ^ ((n >> 1) & 7)) * 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b[j].x, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b[j].y, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b[j].z, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b[j].w, acc[j], 0, 0, 0);
      }
    }
  }
  // ---- epilogue: pre-LN values, then row mean / variance across the 4 column waves
  float v[TN][16];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) {
    const float bv = bias[wn * WN + ni * 32 + l32];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float z = acc[ni][e] + bv;
      v[ni][e] = (MODE == 0) ? rres[ni][e] + z : rres[ni][e] + tanhf(z);
    }
  }
  // the stage buffer not read by the last k-tile is free (all waves passed its barrier)
  float* red = smem + (nk & 1) * STAGE;  // [NWN][BM] partial sums, then [BM] results
  float* res = red + NWN * BM;
  auto row_reduce = [&](bool squares, float* out) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      float p = squares ? v[0][e] * v[0][e] + v[1][e] * v[1][e] : v[0][e] + v[1][e];
      p += __shfl_xor(p, 1, 64);
      p += __shfl_xor(p, 2, 64);
      p += __shfl_xor(p, 4, 64);
      p += __shfl_xor(p, 8, 64);
      p += __shfl_xor(p, 16, 64);
      if (l32 == 0) red[wn * BM + wm * WM + 4 * lh + (e & 3) + 8 * (e >> 2)] = p;
    }
    __syncthreads();
    if (tid < BM) res[tid] = ((red[tid] + red[BM + tid]) + (red[2 * BM + tid] + red[3 * BM + tid])) * (1.f / BN);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 16; ++e) out[e] = res[wm * WM + 4 * lh + (e & 3) + 8 * (e >> 2)];
    __syncthreads();  // red/res are reused by the next reduction
  };
  float mean[16], rstd[16];
  row_reduce(false, mean);
#pragma unroll
  for (int ni = 0; ni < TN; ++ni)
#pragma unroll
    for (int e = 0; e < 16; ++e) v[ni][e] -= mean[e];
  row_reduce(true, rstd);
#pragma unroll
  for (int e = 0; e < 16; ++e) rstd[e] = 1.f / sqrtf(rstd[e] + 1e-5f);
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) {
    const int c = wn * WN + ni * 32 + l32;
    const float g = ln[c], bb = ln[BN + c];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int r = row0 + wm * WM + 4 * lh + (e & 3) + 8 * (e >> 2);
      if (r < rows) h[(size_t)r * BN + c] = g * (rstd[e] * v[ni][e]) + bb;
    }
  }
}

template <int BM, int MODE>
void launch_ln_t(const float* X, int ldx, const float* Wt, int ldw, const float* bias, const float* ln, float* h,
                 int rows, int K, hipStream_t s) {
  const size_t smem = 2ull * (BM + 256) * NT_BK * sizeof(float);
  ensure_smem(gemm_ln_kernel<BM, MODE>, smem);
  hipLaunchKernelGGL((gemm_ln_kernel<BM, MODE>), dim3((rows + BM - 1) / BM), dim3(BM * 8), smem, s, X, ldx, Wt, ldw,
                     bias, ln, h, rows, K);
}

template <int BM, int BN, int BK, int WM, int WN>
void launch_t(const float* X, int ldx, const float* W, int ldw, const float* bias, const float* R, int ldr, float* Y,
              int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  constexpr int NT = (BM / WM) * (BN / WN) * 64;
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, BK, WM, WN>), dim3(ntm * ntn), dim3(NT), 0, s, X, ldx, W, ldw, bias, R,
                     ldr, Y, ldy, rows, ncols, K, C, ntm, ntn);
}

int g_variant = -1;  // -1: automatic
}  // namespace

// X must have round_up(rows, 256) readable rows (workspace rows are padded).
void launch_gemm_variant(int v, const float* X, int ldx, const float* W, int ldw, const float* bias, const float* R,
                         int ldr, float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  switch (v) {
    case 1:
      launch_t<128, 128, 32, 64, 64>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 2:
      launch_t<128, 256, 16, 64, 128>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 3:
      launch_t<256, 128, 16, 128, 64>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 4:
      launch_t<64, 128, 16, 32, 64>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 5:
      launch_t<128, 64, 16, 64, 32>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 6:
      launch_t<64, 64, 16, 32, 32>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 7:
      launch_t<128, 64, 32, 64, 32>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 8:
      launch_t<128, 32, 16, 32, 32>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 9:
      launch_t<256, 64, 16, 64, 32>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 10:
      launch_t<128, 64, 16, 32, 64>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 11:
      launch_t<256, 64, 16, 128, 32>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    default:
      launch_t<128, 128, 16, 64, 64>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
  }
}

// NT variants (Wt[n][k]); K % 32 == 0, Wt rows padded to a multiple of 256.
void launch_gemm_nt_variant(int v, const float* X, int ldx, const float* Wt, int ldw, const float* bias,
                            const float* R, int ldr, float* Y, int ldy, int rows, int ncols, int K, int C,
                            hipStream_t s) {
  switch (v) {
    case 1:
      launch_nt<128, 64, 64, 32>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 2:
      launch_nt<256, 128, 64, 64>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 3:
      launch_nt<128, 256, 64, 64>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 4:
      launch_nt<64, 128, 32, 64>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 5:
      launch_nt<256, 64, 64, 32>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 6:
      launch_nt<128, 128, 32, 64>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 7:
      launch_nt<64, 64, 32, 32>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // persistent (one DMA ring across the workgroup's tiles; Y padded, see gemm_ntp_kernel)
    case 20:
      launch_ntp<128, 128, 32, 64, 2, 2>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 21:
      launch_ntp<128, 128, 32, 64, 3, 1>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 22:
      launch_ntp<128, 64, 64, 32, 3, 2>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 23:
      launch_ntp<64, 64, 32, 32, 2, 4>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 24:
      launch_ntp<256, 64, 64, 32, 2, 2>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 25:
      launch_ntp<64, 128, 32, 64, 2, 3>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 26:
      launch_ntp<128, 64, 64, 32, 2, 3>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    // three-stage rings
    case 10:
      launch_nt<128, 128, 64, 64, 3>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 11:
      launch_nt<128, 64, 64, 32, 3>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 14:
      launch_nt<64, 128, 32, 64, 3>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 15:
      launch_nt<256, 64, 64, 32, 3>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 16:
      launch_nt<128, 128, 32, 64, 3>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 17:
      launch_nt<64, 64, 32, 32, 3>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    case 18:
      launch_nt<256, 128, 64, 64, 3>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
      break;
    default:
      launch_nt<128, 128, 64, 64>(X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
  }
}

void set_gemm_variant(int v) { g_variant = v; }

void launch_gemm_nt(const float* X, int ldx, const float* Wt, int ldw, const float* bias, const float* R, int ldr,
                    float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  // measured on MI355X (tools/gemm_bench.py, K = 256): channel rows (>= 64K) take
  // 128x128 tiles of 32x64 waves when N is a multiple of 256 (persistent with a
  // residual), else 64x64 tiles; log-psi rows take persistent 64x128 tiles for the wide
  // q|k|v map, 64x128 tiles at N = 256 and 64x64 tiles otherwise.
  // Persistent variants write whole tiles (rows padded to 256 by every caller; columns
  // need ldy >= round_up(ncols, 128)).
  int v;
  const bool pad_ok = ldy >= round_up(ncols, 128);
  if (g_variant >= 100) {
    v = g_variant - 100;
  } else if (rows >= 65536) {
    v = (ncols % 256 == 0) ? ((R && pad_ok) ? 20 : 6) : 7;
  } else {
    v = (ncols >= 512 && pad_ok) ? 25 : (ncols == 256 ? 4 : 7);
  }
  launch_gemm_nt_variant(v, X, ldx, Wt, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
}

bool gemm_ln_supported(int D, int K) { return D == 256 && K % NT_BK == 0; }

void launch_gemm_ln(const float* X, int ldx, const float* Wt, int ldw, const float* bias, const float* ln, float* h,
                    int rows, int K, int mode, int bm, hipStream_t s) {
  // bm = rows per workgroup (32..128); default: ~one workgroup per CU
  if (bm <= 0) {
    bm = std::min(96, std::max(32, (rows / 256 + 31) / 32 * 32));
    // callers pad rows to 256: never let the last tile read past round_up(rows, 256)
    while (round_up(rows, bm) > round_up(rows, 256)) bm -= 32;
  }
#define DH_LN_CASE(B)                                                       \
  case B:                                                                   \
    if (mode == 0)                                                          \
      launch_ln_t<B, 0>(X, ldx, Wt, ldw, bias, ln, h, rows, K, s);          \
    else                                                                    \
      launch_ln_t<B, 1>(X, ldx, Wt, ldw, bias, ln, h, rows, K, s);          \
    break;
  switch (bm) {
    DH_LN_CASE(32)
    DH_LN_CASE(64)
    default:
      DH_LN_CASE(96)
  }
#undef DH_LN_CASE
}

namespace {
__global__ void transpose_kernel(const float* __restrict__ src, int ld_src, int rows, int cols, float* dst,
                                 int ld_dst) {
  __shared__ float t[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < rows && c < cols) ? src[(size_t)r * ld_src + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[(size_t)c * ld_dst + r] = t[tx][i];
  }
}
}  // namespace

void launch_transpose(const float* src, int ld_src, int rows, int cols, float* dst, int ld_dst, hipStream_t s) {
  hipLaunchKernelGGL(transpose_kernel, dim3((cols + 31) / 32, (rows + 31) / 32), dim3(256), 0, s, src, ld_src, rows,
                     cols, dst, ld_dst);
}

void launch_gemm(const float* X, int ldx, const float* W, int ldw, const float* bias, const float* R, int ldr,
                 float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  // measured on MI355X (tools/gemm_bench.py): 256x64 tiles (8 waves of 64x32) win on the
  // channel GEMMs and wide outputs; 128x64 tiles of 32x64 waves on short N=256 log-psi GEMMs
  int v = g_variant;
  if (v < 0) v = (rows < 65536 && ncols <= 256) ? 10 : 9;
  launch_gemm_variant(v, X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
}

}  // namespace dh
