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

void set_gemm_variant(int v) { g_variant = v; }

void launch_gemm(const float* X, int ldx, const float* W, int ldw, const float* bias, const float* R, int ldr,
                 float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s) {
  // measured on MI355X (tools/gemm_bench.py): 256x64 tiles (8 waves of 64x32) win on the
  // channel GEMMs and wide outputs; 128x64 tiles of 32x64 waves on short N=256 log-psi GEMMs
  int v = g_variant;
  if (v < 0) v = (rows < 65536 && ncols <= 256) ? 10 : 9;
  launch_gemm_variant(v, X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C, s);
}

}  // namespace dh
