// Reverse mode of log psi with respect to the parameters (the parameter-gradient
// estimator of deephall/loss.py:53-64, 93-108) and the parameter maintenance it needs:
//
//   grad_p = sum_b [ ct_b.re * d Re log psi_b / dp + ct_b.im * d Im log psi_b / dp ]
//
// with the per-walker cotangent ct_b = 2 diff_b / n (ENERGY_GRAD: the real part of
// 2 nanmean(conj(d log psi) diff), loss.py:59-64, 106) or 2 (Im diff, -Re diff) / n (the
// imaginary half of SR_F_VECTOR).  One forward pass stores the layer activations; the
// backward pass runs the chain rule layer by layer on the same row layout (rows = walker x
// electron, features contiguous):
//
//   ln_fwd / ln_bwd   value LayerNorm (flax fast variance, eps 1e-5) with the tanh
//                     residual of the MLP fused; the LN scale/bias gradients are per-block
//                     partial sums
//   attn_bwd          softmax attention, one wave per (walker, head): scores and dA from
//                     LDS, dS = A (dA - <A, dA>), dq, dk, dv
//   tn_partial        weight gradients dW = X^T dY (exact f32 MFMA, v_mfma_f32_32x32x2_f32),
//                     split over row chunks; reduce_partials sums the chunks in double
//   colsum / w0       bias gradients and the K = 4 input map
//   small_gemm        double-accumulated D x D products: the host-side folds of the packed
//                     layout (Wo Wl, bo Wl, W0 Wqkv) and their transposes for the gradient
//   copy2d            packing of the reference parameter tree into the kernel layout
//   adam              optax.adam (b1 0.9, b2 0.999, eps 1e-8) with the reference's
//                     learning-rate schedule (config.py:125-137), optimizers/adam.py:24-43
#include "dh_internal.h"
#include "device_common.h"

namespace dh {

typedef float f32x16_g __attribute__((ext_vector_type(16)));

namespace {

constexpr int kMaxPerLane = 16;  // D <= 1024

// ------------------------------------------------------------------ LayerNorm
// out = LN(a + (z ? tanh(z) : 0)) * gamma + beta; one wave per row
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ a, const float* __restrict__ z,
                                                     const float* __restrict__ ln, float* __restrict__ out, int rows,
                                                     int D) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const size_t base = (size_t)row * D;
  float v[kMaxPerLane];
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int q = 0; q < kMaxPerLane; ++q) {
    const int c = lane + 64 * q;
    v[q] = 0.f;
    if (c < D) {
      float u = a[base + c];
      if (z) u += tanhf(z[base + c]);
      v[q] = u;
      s += u;
      s2 += u * u;
    }
  }
  s = wave_sum(s);
  s2 = wave_sum(s2);
  const float mean = s / D;
  const float var = fmaxf(s2 / D - mean * mean, 0.f);
  const float rstd = rsqrtf(var + 1e-5f);
#pragma unroll
  for (int q = 0; q < kMaxPerLane; ++q) {
    const int c = lane + 64 * q;
    if (c < D) out[base + c] = (v[q] - mean) * rstd * ln[c] + ln[D + c];
  }
}

// Backward of y = LN(u) * gamma + beta with u = a + (z ? tanh(z) : 0):
//   du = rstd (g - mean(g) - xhat mean(g xhat)),  g = dy gamma
//   da = du (+ dres),  dz = du (1 - tanh(z)^2)  (when z != null)
// plus per-block partial sums pg[blk][0][c] = sum dy xhat, pg[blk][1][c] = sum dy.
// One wave per row, RPB rows per 4-wave block.
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ a, const float* __restrict__ z,
                                                     const float* __restrict__ ln, const float* __restrict__ dy,
                                                     const float* dres, float* da, float* __restrict__ dz,
                                                     float* __restrict__ pg, int rows, int D, int rpb) {
  __shared__ float red[4][2][256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float gs[kMaxPerLane], bs[kMaxPerLane];
#pragma unroll
  for (int q = 0; q < kMaxPerLane; ++q) gs[q] = bs[q] = 0.f;
  const int r0 = blockIdx.x * rpb;
  for (int rr = w; rr < rpb; rr += 4) {
    const int row = r0 + rr;
    if (row >= rows) break;
    const size_t base = (size_t)row * D;
    float u[kMaxPerLane], t[kMaxPerLane], g[kMaxPerLane];
    float s = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < kMaxPerLane; ++q) {
      const int c = lane + 64 * q;
      u[q] = t[q] = g[q] = 0.f;
      if (c < D) {
        float x = a[base + c];
        if (z) {
          t[q] = tanhf(z[base + c]);
          x += t[q];
        }
        u[q] = x;
        s += x;
        s2 += x * x;
      }
    }
    s = wave_sum(s);
    s2 = wave_sum(s2);
    const float mean = s / D;
    const float var = fmaxf(s2 / D - mean * mean, 0.f);
    const float rstd = rsqrtf(var + 1e-5f);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int q = 0; q < kMaxPerLane; ++q) {
      const int c = lane + 64 * q;
      if (c < D) {
        const float xh = (u[q] - mean) * rstd;
        const float d = dy[base + c];
        g[q] = d * ln[c];
        sg += g[q];
        sgx += g[q] * xh;
        gs[q] += d * xh;
        bs[q] += d;
        u[q] = xh;
      }
    }
    sg = wave_sum(sg) / D;
    sgx = wave_sum(sgx) / D;
#pragma unroll
    for (int q = 0; q < kMaxPerLane; ++q) {
      const int c = lane + 64 * q;
      if (c < D) {
        const float du = rstd * (g[q] - sg - u[q] * sgx);
        if (da) da[base + c] = du + (dres ? dres[base + c] : 0.f);
        if (dz) dz[base + c] = du * (1.f - t[q] * t[q]);
      }
    }
  }
  // combine the four waves' partial sums, 256 columns at a time
  for (int c0 = 0; c0 < D; c0 += 256) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int qq = c0 / 64 + q;
      if (qq < kMaxPerLane) {
        red[w][0][64 * q + lane] = gs[qq];
        red[w][1][64 * q + lane] = bs[qq];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 256 && c0 + c < D; c += 256) {
      float sg2 = 0.f, sb2 = 0.f;
      for (int j = 0; j < 4; ++j) {
        sg2 += red[j][0][c];
        sb2 += red[j][1][c];
      }
      pg[((size_t)blockIdx.x * 2 + 0) * D + c0 + c] = sg2;
      pg[((size_t)blockIdx.x * 2 + 1) * D + c0 + c] = sb2;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ attention backward
// o_i = sum_j A_ij v_j, A = softmax_j(q_i . k_j * scale) per (walker, head); given dO:
//   dA_ij = dO_i . v_j ; dS = A (dA - sum_j A dA) ; dq_i = scale sum_j dS_ij k_j ;
//   dk_j = scale sum_i dS_ij q_i ; dv_j = sum_i A_ij dO_i
// One 64-lane wave per (walker, head); lane = feature column.
__global__ __launch_bounds__(64) void attn_bwd_kernel(const float* __restrict__ qkv, const float* __restrict__ dO,
                                                      float* __restrict__ dqkv, int N, int H, int dh, float scale) {
  extern __shared__ float sm[];
  const int ld = dh + 1, nn = N * N;
  float* q = sm;
  float* k = q + N * ld;
  float* v = k + N * ld;
  float* g = v + N * ld;
  float* A = g + N * ld;
  float* dS = A + nn;
  const int lane = threadIdx.x;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int D = H * dh;
  for (int i = 0; i < N; ++i) {
    const size_t r = (size_t)b * N + i;
    for (int c = lane; c < dh; c += 64) {
      q[i * ld + c] = qkv[r * 3 * D + h * dh + c];
      k[i * ld + c] = qkv[r * 3 * D + D + h * dh + c];
      v[i * ld + c] = qkv[r * 3 * D + 2 * D + h * dh + c];
      g[i * ld + c] = dO[r * D + h * dh + c];
    }
  }
  __syncthreads();
  for (int p = lane; p < nn; p += 64) {
    const int i = p / N, j = p % N;
    float s = 0.f, da = 0.f;
    for (int c = 0; c < dh; ++c) {
      s = fmaf(q[i * ld + c], k[j * ld + c], s);
      da = fmaf(g[i * ld + c], v[j * ld + c], da);
    }
    A[p] = s * scale;
    dS[p] = da;
  }
  __syncthreads();
  for (int i = lane; i < N; i += 64) {
    float m = -INFINITY;
    for (int j = 0; j < N; ++j) m = fmaxf(m, A[i * N + j]);
    float ssum = 0.f;
    for (int j = 0; j < N; ++j) {
      const float e = expf(A[i * N + j] - m);
      A[i * N + j] = e;
      ssum += e;
    }
    const float inv = 1.f / ssum;
    float dot = 0.f;
    for (int j = 0; j < N; ++j) {
      A[i * N + j] *= inv;
      dot = fmaf(A[i * N + j], dS[i * N + j], dot);
    }
    for (int j = 0; j < N; ++j) dS[i * N + j] = A[i * N + j] * (dS[i * N + j] - dot);
  }
  __syncthreads();
  for (int c = lane; c < dh; c += 64) {
    for (int i = 0; i < N; ++i) {
      float dq = 0.f, dk = 0.f, dv = 0.f;
      for (int j = 0; j < N; ++j) {
        dq = fmaf(dS[i * N + j], k[j * ld + c], dq);
        dk = fmaf(dS[j * N + i], q[j * ld + c], dk);
        dv = fmaf(A[j * N + i], g[j * ld + c], dv);
      }
      const size_t r = (size_t)b * N + i;
      dqkv[r * 3 * D + h * dh + c] = dq * scale;
      dqkv[r * 3 * D + D + h * dh + c] = dk * scale;
      dqkv[r * 3 * D + 2 * D + h * dh + c] = dv;
    }
  }
}

// ------------------------------------------------------------------ weight gradients
// P[chunk][m][n] = sum_{r in chunk} X[r][m] Y[r][n]  (m < M, n < Nc), exact f32 MFMA
// 32x32x2: lane l holds A[l & 31][l >> 5] = X[r + (l >> 5)][m], B[l >> 5][l & 31] =
// Y[r + (l >> 5)][n] — two coalesced 128-B row segments per operand, no LDS.  128 x 128
// tile per 4-wave block (2 x 2 waves of 64 x 64), rows [chunk * cl, +cl).
constexpr int kTnTile = 128;
__global__ __launch_bounds__(256) void tn_partial_kernel(const float* __restrict__ X, int ldx,
                                                         const float* __restrict__ Y, int ldy, int rows, int M,
                                                         int Nc, int cl, int ntn, float* __restrict__ P) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tm = blockIdx.x / ntn, tn = blockIdx.x % ntn;
  const int m0 = tm * kTnTile + (w >> 1) * 64, n0 = tn * kTnTile + (w & 1) * 64;
  const int l32 = lane & 31, lh = lane >> 5;
  const int rbeg = blockIdx.y * cl, rend = min(rows, rbeg + cl);
  f32x16_g acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  const bool am0 = m0 + l32 < M, am1 = m0 + 32 + l32 < M, bn0 = n0 + l32 < Nc, bn1 = n0 + 32 + l32 < Nc;
  for (int r = rbeg; r < rend; r += 8) {
    float xa[4][2], yb[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int rr = r + 2 * u + lh;
      const bool ok = rr < rend;
      const float* xr = X + (size_t)rr * ldx + m0 + l32;
      const float* yr = Y + (size_t)rr * ldy + n0 + l32;
      xa[u][0] = (ok && am0) ? xr[0] : 0.f;
      xa[u][1] = (ok && am1) ? xr[32] : 0.f;
      yb[u][0] = (ok && bn0) ? yr[0] : 0.f;
      yb[u][1] = (ok && bn1) ? yr[32] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[u][a], yb[u][b], acc[a][b], 0, 0, 0);
  }
  // C/D map: col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
  float* Pc = P + (size_t)blockIdx.y * M * Nc;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + 32 * b + l32;
      if (n >= Nc) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (m < M) Pc[(size_t)m * Nc + n] = acc[a][b][e];
      }
    }
}

// P[chunk][n] = sum_{r in chunk} Y[r][n]
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ Y, int ldy, int rows, int Nc,
                                                             int cl, float* __restrict__ P) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= Nc) return;
  const int rbeg = blockIdx.y * cl, rend = min(rows, rbeg + cl);
  float s = 0.f;
  for (int r = rbeg; r < rend; ++r) s += Y[(size_t)r * ldy + n];
  P[(size_t)blockIdx.y * Nc + n] = s;
}

// input map K = 4: P[chunk][a][n] = sum_r feat_r[a] Y[r][n], feat = [cos th, sin th cos ph,
// sin th sin ph, s] (psiformer.py:51-60) from geo = (sin th, cos th, sin ph, cos ph)
__global__ __launch_bounds__(256) void w0_partial_kernel(const float* __restrict__ geo, const float* __restrict__ Y,
                                                         int ldy, int rows, int Nc, int N, int n_up, int cl,
                                                         float* __restrict__ P) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= Nc) return;
  const int rbeg = blockIdx.y * cl, rend = min(rows, rbeg + cl);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int r = rbeg; r < rend; ++r) {
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)r);
    const float y = Y[(size_t)r * ldy + n];
    s0 = fmaf(g.y, y, s0);
    s1 = fmaf(g.x * g.w, y, s1);
    s2 = fmaf(g.x * g.z, y, s2);
    s3 += ((r % N) < n_up) ? y : -y;
  }
  float* p = P + (size_t)blockIdx.y * 4 * Nc;
  p[n] = s0;
  p[Nc + n] = s1;
  p[2 * Nc + n] = s2;
  p[3 * Nc + n] = s3;
}

// out[r][c] (ldo) = scale * sum_ch P[ch * stride + r * ldp + c] (+ out if acc), double
// accumulation over the chunks
__global__ __launch_bounds__(256) void reduce2d_kernel(const float* __restrict__ P, int nchunk, size_t stride, int ldp,
                                                       int nr, int nc, float* __restrict__ out, int ldo, float scale,
                                                       int acc) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)nr * nc) return;
  const int r = (int)(i / nc), c = (int)(i % nc);
  const float* p = P + (size_t)r * ldp + c;
  double s = 0.0;
  for (int ch = 0; ch < nchunk; ++ch) s += p[(size_t)ch * stride];
  const float v = (float)(s * scale);
  float* o = out + (size_t)r * ldo + c;
  *o = acc ? *o + v : v;
}

// ------------------------------------------------------------------ small products
// C[m][n] (ldc) = sum_k op(A)[m][k] op(B)[k][n] (+ C if acc); op(A)[m][k] = ta ? A[k][m] : A[m][k]
__global__ __launch_bounds__(256) void small_gemm_kernel(int Mr, int Nc, int K, const float* __restrict__ A, int lda,
                                                         int ta, const float* __restrict__ B, int ldb, int tb,
                                                         float* __restrict__ C, int ldc, int acc) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int m = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (m >= Mr || n >= Nc) return;
  double s = 0.0;
  for (int k = 0; k < K; ++k) {
    const float a = ta ? A[(size_t)k * lda + m] : A[(size_t)m * lda + k];
    const float b = tb ? B[(size_t)n * ldb + k] : B[(size_t)k * ldb + n];
    s += (double)a * (double)b;
  }
  float* c = C + (size_t)m * ldc + n;
  *c = acc ? *c + (float)s : (float)s;
}

// dst[r][c] (ldd) = src[r][c] (lds), r < nr, c < nc; src == null writes zeros
__global__ __launch_bounds__(256) void copy2d_kernel(const float* __restrict__ src, int lds, float* __restrict__ dst,
                                                     int ldd, int nr, int nc) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)nr * nc) return;
  const int r = (int)(i / nc), c = (int)(i % nc);
  dst[(size_t)r * ldd + c] = src ? src[(size_t)r * lds + c] : 0.f;
}

// ------------------------------------------------------------------ loss weights, Adam
// ct[b] = (2 / n) (d.re, d.im) (part 0) or (2 / n) (d.im, -d.re) (part 1); 0 for NaN d / n = 0
__global__ __launch_bounds__(256) void cotangent_kernel(const float* __restrict__ diff, const float* __restrict__ nv,
                                                        int B, int part, float* __restrict__ ct) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const float n = nv[0];
  const float dr = diff[2 * b], di = diff[2 * b + 1];
  const bool ok = n > 0.f && !(isnan(dr) || isnan(di));
  const float s = ok ? 2.f / n : 0.f;
  ct[2 * b] = ok ? s * (part ? di : dr) : 0.f;
  ct[2 * b + 1] = ok ? s * (part ? -dr : di) : 0.f;
}

// optax.adam: mu = b1 mu + (1 - b1) g ; nu = b2 nu + (1 - b2) g^2 ;
// p -= lr * (mu / (1 - b1^t)) / (sqrt(nu / (1 - b2^t)) + eps), t = step + 1; NaN gradients
// become 0 first (loss_prod's nan_to_num, loss.py:64)
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ mu, float* __restrict__ nu, size_t n, float lr,
                                                   float b1, float b2, float eps, float bc1, float bc2) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float gi = g[i];
  if (isnan(gi)) gi = 0.f;
  if (isinf(gi)) gi = gi > 0.f ? 3.402823466e38f : -3.402823466e38f;
  const float m = (1.f - b1) * gi + b1 * mu[i];
  const float v = (1.f - b2) * (gi * gi) + b2 * nu[i];
  mu[i] = m;
  nu[i] = v;
  const float mh = m / bc1, vh = v / bc2;
  p[i] -= lr * (mh / (sqrtf(vh) + eps));
}

// ------------------------------------------------------------------ "sparse" orbitals
__global__ __launch_bounds__(256) void sparse_fold_kernel(const float* __restrict__ W8, const float* __restrict__ b8,
                                                          const float* __restrict__ Wl, const float* __restrict__ bl,
                                                          int real_part, int D, int NK, int M, float* Wfull, int ldw,
                                                          float* bfull) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t per = (size_t)M * NK;
  if (i >= (size_t)(D + 1) * per) return;
  const int d = (int)(i / per), rem = (int)(i % per), m = rem / NK, jk = rem % NK;
  const float* src = d < D ? W8 + (size_t)d * kSparseFeatures * NK : b8;
  double s = 0.0;
#pragma unroll
  for (int a = 0; a < kSparseFeatures; ++a) s += (double)src[a * NK + jk] * Wl[a * M + m];
  if (d < D)
    Wfull[(size_t)d * ldw + rem] = (float)s;
  else
    bfull[rem] = (float)(s + (real_part ? (double)bl[m] : 0.0));
}

__global__ __launch_bounds__(256) void sparse_unfold_kernel(const float* __restrict__ dWfull, int ldw,
                                                            const float* __restrict__ dbfull,
                                                            const float* __restrict__ Wl, int D, int NK, int M,
                                                            float* dW8, float* db8, int acc) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t per = (size_t)kSparseFeatures * NK;
  if (i >= (size_t)(D + 1) * per) return;
  const int d = (int)(i / per), rem = (int)(i % per), a = rem / NK, jk = rem % NK;
  const float* src = d < D ? dWfull + (size_t)d * ldw : dbfull;
  double s = 0.0;
  for (int m = 0; m < M; ++m) s += (double)src[m * NK + jk] * Wl[a * M + m];
  float* o = d < D ? dW8 + (size_t)d * per + rem : db8 + rem;
  *o = acc ? *o + (float)s : (float)s;
}

// one 256-thread block per (a, m) of lll_weight (+ M blocks for its bias)
__global__ __launch_bounds__(256) void sparse_lll_grad_kernel(SparseBlocks blk, const float* __restrict__ dWfull,
                                                              int ldw, const float* __restrict__ dbfull, int D, int NK,
                                                              int M, float* dWl, float* dbl, int acc) {
  __shared__ double red[4];
  const int o = blockIdx.x, tid = threadIdx.x;
  const int MNK = M * NK;
  double s = 0.0;
  if (o < kSparseFeatures * M) {
    const int a = o / M, m = o % M;
    for (int i = 0; i < blk.n; ++i)
      for (int q = tid; q < (D + 1) * NK; q += 256) {
        const int d = q / NK, jk = q % NK;
        const float w8 = d < D ? blk.W8[i][(size_t)d * kSparseFeatures * NK + a * NK + jk] : blk.b8[i][a * NK + jk];
        const float g = d < D ? dWfull[(size_t)d * ldw + i * MNK + m * NK + jk] : dbfull[i * MNK + m * NK + jk];
        s += (double)w8 * g;
      }
  } else {
    const int m = o - kSparseFeatures * M;
    for (int i = 0; i < blk.n; i += 2)  // real-part blocks: (blk, part 0)
      for (int jk = tid; jk < NK; jk += 256) s += dbfull[i * MNK + m * NK + jk];
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    const float v = (float)(red[0] + red[1] + red[2] + red[3]);
    float* out = o < kSparseFeatures * M ? dWl + o : dbl + (o - kSparseFeatures * M);
    *out = acc ? *out + v : v;
  }
}

unsigned blocks_for(size_t n, int per = 256) { return (unsigned)((n + per - 1) / per); }

}  // namespace

void launch_ln_fwd(const float* a, const float* z, const float* ln, float* out, int rows, int D, hipStream_t s) {
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, a, z, ln, out, rows, D);
}

int ln_bwd_blocks(int rows) { return (rows + kLnRowsPerBlock - 1) / kLnRowsPerBlock; }

void launch_ln_bwd(const float* a, const float* z, const float* ln, const float* dy, const float* dres, float* da,
                   float* dz, float* pg, int rows, int D, hipStream_t s) {
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(ln_bwd_blocks(rows)), dim3(256), 0, s, a, z, ln, dy, dres, da, dz, pg, rows,
                     D, kLnRowsPerBlock);
}

void launch_attn_bwd(const Dims& d, const float* qkv, const float* dO, float* dqkv, int nw, hipStream_t s) {
  const size_t smem = (size_t)(4 * d.N * (d.dh + 1) + 2 * d.N * d.N) * sizeof(float);
  ensure_smem(attn_bwd_kernel, smem);
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(nw * d.H), dim3(64), smem, s, qkv, dO, dqkv, d.N, d.H, d.dh,
                     1.f / sqrtf((float)d.dh));
}

int grad_chunks(int rows) { return (rows + kGradChunk - 1) / kGradChunk; }

void launch_tn_partial(const float* X, int ldx, const float* Y, int ldy, int rows, int M, int Nc, float* P,
                       hipStream_t s) {
  const int ntm = (M + kTnTile - 1) / kTnTile, ntn = (Nc + kTnTile - 1) / kTnTile;
  hipLaunchKernelGGL(tn_partial_kernel, dim3(ntm * ntn, grad_chunks(rows)), dim3(256), 0, s, X, ldx, Y, ldy, rows, M,
                     Nc, kGradChunk, ntn, P);
}

void launch_colsum_partial(const float* Y, int ldy, int rows, int Nc, float* P, hipStream_t s) {
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((Nc + 255) / 256, grad_chunks(rows)), dim3(256), 0, s, Y, ldy, rows,
                     Nc, kGradChunk, P);
}

void launch_w0_partial(const Dims& d, const float* geo, const float* Y, int ldy, int rows, float* P, hipStream_t s) {
  hipLaunchKernelGGL(w0_partial_kernel, dim3((d.D + 255) / 256, grad_chunks(rows)), dim3(256), 0, s, geo, Y, ldy, rows,
                     d.D, d.N, d.n_up, kGradChunk, P);
}

void launch_reduce2d(const float* P, int nchunk, size_t stride, int ldp, int nr, int nc, float* out, int ldo,
                     float scale, int acc, hipStream_t s) {
  const size_t n = (size_t)nr * nc;
  if (n == 0) return;
  hipLaunchKernelGGL(reduce2d_kernel, dim3(blocks_for(n)), dim3(256), 0, s, P, nchunk, stride, ldp, nr, nc, out, ldo,
                     scale, acc);
}

void launch_small_gemm(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb, float* C,
                       int ldc, int acc, hipStream_t s) {
  hipLaunchKernelGGL(small_gemm_kernel, dim3((N + 63) / 64, (M + 3) / 4), dim3(256), 0, s, M, N, K, A, lda, ta, B, ldb,
                     tb, C, ldc, acc);
}

void launch_copy2d(const float* src, int lds, float* dst, int ldd, int nr, int nc, hipStream_t s) {
  if ((size_t)nr * nc == 0) return;
  hipLaunchKernelGGL(copy2d_kernel, dim3(blocks_for((size_t)nr * nc)), dim3(256), 0, s, src, lds, dst, ldd, nr, nc);
}

void launch_cotangent(const float* diff, const float* nvalid, int B, int part, float* ct, hipStream_t s) {
  hipLaunchKernelGGL(cotangent_kernel, dim3(blocks_for(B)), dim3(256), 0, s, diff, nvalid, B, part, ct);
}

void launch_adam(float* p, const float* g, float* mu, float* nu, size_t n, float lr, float b1, float b2, float eps,
                 int step, hipStream_t s) {
  const float bc1 = 1.f - powf(b1, (float)(step + 1)), bc2 = 1.f - powf(b2, (float)(step + 1));
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n)), dim3(256), 0, s, p, g, mu, nu, n, lr, b1, b2, eps, bc1, bc2);
}

void launch_sparse_fold(const float* W8, const float* b8, const float* Wl, const float* bl, int real_part, int D,
                        int NK, int M, float* Wfull, int ldw, float* bfull, hipStream_t s) {
  hipLaunchKernelGGL(sparse_fold_kernel, dim3(blocks_for((size_t)(D + 1) * M * NK)), dim3(256), 0, s, W8, b8, Wl, bl,
                     real_part, D, NK, M, Wfull, ldw, bfull);
}

void launch_sparse_unfold(const float* dWfull, int ldw, const float* dbfull, const float* Wl, int D, int NK, int M,
                          float* dW8, float* db8, int acc, hipStream_t s) {
  hipLaunchKernelGGL(sparse_unfold_kernel, dim3(blocks_for((size_t)(D + 1) * kSparseFeatures * NK)), dim3(256), 0, s,
                     dWfull, ldw, dbfull, Wl, D, NK, M, dW8, db8, acc);
}

void launch_sparse_lll_grad(SparseBlocks blk, const float* dWfull, int ldw, const float* dbfull, int D, int NK, int M,
                            float* dWl, float* dbl, int acc, hipStream_t s) {
  hipLaunchKernelGGL(sparse_lll_grad_kernel, dim3(kSparseFeatures * M + M), dim3(256), 0, s, blk, dWfull, ldw, dbfull,
                     D, NK, M, dWl, dbl, acc);
}

}  // namespace dh
