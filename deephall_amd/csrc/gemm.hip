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
// Tile: 128x128 per 256-thread workgroup, 4 waves as 2x2, each wave 64x64 =
// 2x2 MFMA 32x32 tiles; BK = 16, register-staged double buffer in LDS.
// A is stored transposed in LDS (As[k][m]) so that the MFMA A operand
// (lane l holds A[l&31][l>>5]) is a conflict-free ds_read_b32 row read.
#include "dh_internal.h"
#include "device_common.h"

namespace dh {

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {
constexpr int BM = 128, BN = 128, BK = 16, NT = 256, PAD = 4;

__global__ __launch_bounds__(NT) void gemm_f32_kernel(const float* __restrict__ X, int ldx,
                                                       const float* __restrict__ W, int ldw,
                                                       const float* __restrict__ bias, const float* R, int ldr,
                                                       float* Y, int ldy, int rows, int ncols, int K, int C,
                                                       int ntm, int ntn) {
  __shared__ float As[2][BK][BM + PAD];
  __shared__ float Bs[2][BK][BN + PAD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

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

  float4 ra[2], rb[2];
  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (tid >> 2) + 64 * i;
      const int k = k0 + (tid & 3) * 4;
      const float* src = X + (size_t)(row0 + r) * ldx + k;
      if (k + 4 <= K) {
        ra[i] = *reinterpret_cast<const float4*>(src);
      } else {
        ra[i].x = (k + 0 < K) ? src[0] : 0.f;
        ra[i].y = (k + 1 < K) ? src[1] : 0.f;
        ra[i].z = (k + 2 < K) ? src[2] : 0.f;
        ra[i].w = (k + 3 < K) ? src[3] : 0.f;
      }
      const int kb = k0 + (tid >> 5) + 8 * i;
      const int n = col0 + (tid & 31) * 4;
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
    for (int i = 0; i < 2; ++i) {
      const int r = (tid >> 2) + 64 * i;
      const int kk = (tid & 3) * 4;
      As[buf][kk + 0][r] = ra[i].x;
      As[buf][kk + 1][r] = ra[i].y;
      As[buf][kk + 2][r] = ra[i].z;
      As[buf][kk + 3][r] = ra[i].w;
      const int kb = (tid >> 5) + 8 * i;
      const int n = (tid & 31) * 4;
      *reinterpret_cast<float4*>(&Bs[buf][kb][n]) = rb[i];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
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
      const float a0 = As[cur][ka][wm * 64 + l32];
      const float a1 = As[cur][ka][wm * 64 + 32 + l32];
      const float b0 = Bs[cur][ka][wn * 64 + l32];
      const float b1 = Bs[cur][ka][wn * 64 + 32 + l32];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // Epilogue. C/D map of 32x32 MFMA: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int c = col0 + wn * 64 + ni * 32 + l32;
      if (c >= ncols) continue;
      const float bv = bias ? bias[c] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = row0 + wm * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (r >= rows) continue;
        float v = acc[mi][ni][e];
        if (bias && (r % C) == 0) v += bv;
        if (R) v += R[(size_t)r * ldr + c];
        Y[(size_t)r * ldy + c] = v;
      }
    }
  }
}
}  // namespace

void launch_gemm(const float* X, int ldx, const float* W, int ldw, const float* bias, const float* R, int ldr,
                 float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  // X must have round_up(rows, 128) readable rows (workspace rows are padded).
  const int ntm = (rows + BM - 1) / BM, ntn = (ncols + BN - 1) / BN;
  hipLaunchKernelGGL(gemm_f32_kernel, dim3(ntm * ntn), dim3(NT), 0, s, X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows,
                     ncols, K, C, ntm, ntn);
}

}  // namespace dh
