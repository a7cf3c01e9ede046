// KFAC on MI355X: the curvature statistics, damped inverses and preconditioned update of
// the reference's default optimizer (deephall/optimizers/kfac.py:195-241 on kfac_jax; the
// algorithm restated in oracle/kfac.py and DESIGN.md §3d).
//
// Per iteration (api.cpp dh_kfac_vjp / dh_kfac_step):
//   statistics   A = x~^T x~ / rows and G = dy^T dy / rows of every dense layer from the
//                saved forward activations and a second reverse pass with the Fisher
//                cotangent sqrt(2) on Re log psi (tn_partial X^T X, exact-f32 MFMA, chunk
//                sums in double; the bias row / column from column sums: kfac_aug_kernel;
//                the K = 4 input features: kfac_feat_gram_kernel); generic parameters
//                (LayerNorm, Jastrow) from the squared batch tangent (kfac_generic_kernel)
//   EMA          raw <- 0.95 raw + stats (kfac_ema_kernel)
//   inverses     pi-adjusted damped factors in f64 (kfac_trace_kernel, kfac_damp_kernel),
//                inverted together by the blocked sweep (Gauss-Jordan) operator, 32-wide
//                panels: gj_panel_kernel inverts the diagonal block in LDS and forms the
//                panel row, gj_update_kernel applies the rank-32 update to the rest, one
//                launch pair per panel for ALL matrices of the step
//   update       P V = A_d^-1 V G_d^-1 per block (kfac_gemm_kernel, f64, batched jobs),
//                generic g / (diag + lambda), <P g, g>, the norm constraint and
//                p -= lr c P g (kfac_dot_kernel, kfac_update_kernel) — no host sync
#include "dh_internal.h"

namespace dh {

namespace {

unsigned nblk(size_t n, int per = 256) { return (unsigned)((n + per - 1) / per); }

// bias row / column / corner of an augmented Gram matrix out[(n+1) x (n+1)] (ld):
// column sums of the chunk partials P[ch][n] (double), scaled
__global__ __launch_bounds__(256) void kfac_aug_kernel(const float* __restrict__ P, int nch, int n,
                                                       float* __restrict__ out, int ld, float scale, float corner,
                                                       int acc) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < n) {
    double s = 0.0;
    for (int ch = 0; ch < nch; ++ch) s += P[(size_t)ch * n + c];
    const float v = (float)(s * scale);
    float* a = out + (size_t)c * ld + n;
    float* b = out + (size_t)n * ld + c;
    *a = acc ? *a + v : v;
    *b = acc ? *b + v : v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float* o = out + (size_t)n * ld + n;
    *o = acc ? *o + corner : corner;
  }
}

// Gram matrix of the input features f = [cos th, sin th cos ph, sin th sin ph, s]
// (psiformer.py:51-60) from geo = (sin th, cos th, sin ph, cos ph): P[chunk][4][4]
__global__ __launch_bounds__(256) void kfac_feat_gram_kernel(const float* __restrict__ geo, int rows, int N, int n_up,
                                                             int cl, float* __restrict__ P) {
  __shared__ double red[256][10];
  const int rbeg = blockIdx.x * cl, rend = min(rows, rbeg + cl);
  double s[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = rbeg + threadIdx.x; r < rend; r += 256) {
    const float4 g = *reinterpret_cast<const float4*>(geo + 4 * (size_t)r);
    const double f[4] = {g.y, (double)(g.x * g.w), (double)(g.x * g.z), (r % N) < n_up ? 1.0 : -1.0};
    int k = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = a; b < 4; ++b) s[k++] += f[a] * f[b];
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) red[threadIdx.x][k] = s[k];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st)
#pragma unroll
      for (int k = 0; k < 10; ++k) red[threadIdx.x][k] += red[threadIdx.x + st][k];
    __syncthreads();
  }
  if (threadIdx.x < 16) {
    const int a = threadIdx.x >> 2, b = threadIdx.x & 3;
    const int lo = min(a, b), hi = max(a, b);
    const int k = lo * 4 - lo * (lo - 1) / 2 + (hi - lo);
    P[(size_t)blockIdx.x * 16 + threadIdx.x] = (float)red[0][k];
  }
}

// Fisher cotangent: sqrt(2) on Re log psi (the normal predictive distribution of
// variance 1/2, loss.py:98); 0 for a walker whose log psi is not finite (psi = 0)
__global__ __launch_bounds__(256) void kfac_fisher_ct_kernel(const float* __restrict__ logpsi, int nw,
                                                             float* __restrict__ ct) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nw) return;
  const bool ok = isfinite(logpsi[2 * b]) && isfinite(logpsi[2 * b + 1]);
  ct[2 * b] = ok ? 1.41421356237309515f : 0.f;
  ct[2 * b + 1] = 0.f;
}

// generic (NaiveDiagonal) statistics: diag[c] = fgrad[ref]^2 * scale over the segment table
__global__ __launch_bounds__(256) void kfac_generic_kernel(const float* __restrict__ fgrad, KfacGenTable tab,
                                                           float* __restrict__ diag, float scale) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= tab.total) return;
  int s = 0;
  while (s + 1 < tab.n && tab.cmp[s + 1] <= c) ++s;
  const float g = fgrad[tab.ref[s] + (c - tab.cmp[s])];
  diag[c] = (float)((double)g * g * scale);
}

__global__ __launch_bounds__(256) void kfac_ema_kernel(float* __restrict__ raw, const float* __restrict__ st,
                                                       size_t n, float ema) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) raw[i] = ema * raw[i] + st[i];
}

// trace / n of every factor slot (double): tr[slot]
__global__ __launch_bounds__(256) void kfac_trace_kernel(const float* __restrict__ raw, const KfacSlot* __restrict__ slots,
                                                         double* __restrict__ tr) {
  __shared__ double red[256];
  const KfacSlot sl = slots[blockIdx.x];
  double s = 0.0;
  for (int i = threadIdx.x; i < sl.n; i += 256) s += raw[sl.off + (size_t)i * sl.n + i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) tr[blockIdx.x] = red[0] / sl.n;
}

// damped f64 factor of job j: M = sqrt(s) raw / weight + d I, d = sqrt(lambda) pi (A) or
// sqrt(lambda) / pi (G), pi = sqrt((tr A / dim A) / (tr G / dim G)) (1 if a trace is <= 0)
__global__ __launch_bounds__(256) void kfac_damp_kernel(const float* __restrict__ raw, const KfacSlot* __restrict__ slots,
                                                        const KfacInvJob* __restrict__ jobs, const double* __restrict__ tr,
                                                        double* __restrict__ gj, double inv_weight, double sqrt_lambda) {
  const KfacInvJob jb = jobs[blockIdx.y];
  const KfacSlot sl = slots[jb.slot];
  const size_t nn = (size_t)sl.n * sl.n;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nn) return;
  const double ta = tr[jb.is_a ? jb.slot : jb.partner], tg = tr[jb.is_a ? jb.partner : jb.slot];
  const double pi = (ta > 0.0 && tg > 0.0) ? sqrt(ta / tg) : 1.0;
  const double d = jb.is_a ? sqrt_lambda * pi : sqrt_lambda / pi;
  const int r = (int)(i / sl.n), c = (int)(i % sl.n);
  double v = (double)jb.sqrt_scale * (double)raw[sl.off + i] * inv_weight;
  if (r == c) v += d;
  gj[jb.gj_off + i] = v;
}

// ---- blocked sweep (Gauss-Jordan) inverse of SPD matrices, panel width 32
constexpr int kGJ = 32;

// one workgroup per job: T0 = A11^-1 (LDS Gauss-Jordan, no pivoting: the pivots of a
// positive-definite matrix's Schur complements are positive), T1 = T0 A[K][j not in K]
__global__ __launch_bounds__(256) void gj_panel_kernel(const KfacInvJob* __restrict__ jobs, double* __restrict__ gj,
                                                       int k0, double* __restrict__ tmp, size_t tmp_stride) {
  const KfacInvJob jb = jobs[blockIdx.x];
  const int n = jb.n;
  if (k0 >= n) return;
  const int b = min(kGJ, n - k0);
  const double* A = gj + jb.gj_off;
  double* T0 = tmp + (size_t)blockIdx.x * tmp_stride;
  double* T1 = T0 + kGJ * kGJ;
  __shared__ double S[kGJ][kGJ + 1];
  for (int e = threadIdx.x; e < kGJ * kGJ; e += 256) {
    const int r = e / kGJ, c = e % kGJ;
    S[r][c] = (r < b && c < b) ? A[(size_t)(k0 + r) * n + k0 + c] : (r == c ? 1.0 : 0.0);
  }
  __syncthreads();
  for (int k = 0; k < b; ++k) {
    double old[4], fik[4], rkj[4];
    const double pkk = S[k][k];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = threadIdx.x + 256 * u, r = e / kGJ, c = e % kGJ;
      old[u] = S[r][c];
      fik[u] = S[r][k];
      rkj[u] = S[k][c];
    }
    __syncthreads();
    const double p = 1.0 / pkk;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = threadIdx.x + 256 * u, r = e / kGJ, c = e % kGJ;
      const double nr = (c == k ? 1.0 : rkj[u]) * p;
      S[r][c] = (r == k) ? nr : (c == k ? 0.0 : old[u]) - fik[u] * nr;
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < kGJ * kGJ; e += 256) T0[e] = S[e / kGJ][e % kGJ];
  for (int e = threadIdx.x; e < b * n; e += 256) {
    const int r = e / n, j = e % n;
    if (j >= k0 && j < k0 + b) continue;
    double acc = 0.0;
    for (int l = 0; l < b; ++l) acc = fma(S[r][l], A[(size_t)(k0 + l) * n + j], acc);
    T1[(size_t)r * n + j] = acc;
  }
}

// rows [16 blockIdx.x, +16) of every job: A22 -= A21 T1, A21 <- -A21 T0, A12 <- T1, A11 <- T0
constexpr int kGJRows = 16;
__global__ __launch_bounds__(256) void gj_update_kernel(const KfacInvJob* __restrict__ jobs, double* __restrict__ gj,
                                                        int k0, const double* __restrict__ tmp, size_t tmp_stride) {
  const KfacInvJob jb = jobs[blockIdx.y];
  const int n = jb.n;
  const int r0 = blockIdx.x * kGJRows;
  if (k0 >= n || r0 >= n) return;
  const int b = min(kGJ, n - k0);
  double* A = gj + jb.gj_off;
  const double* T0 = tmp + (size_t)blockIdx.y * tmp_stride;
  const double* T1 = T0 + kGJ * kGJ;
  __shared__ double Aik[kGJRows][kGJ + 1];
  const int nr = min(kGJRows, n - r0);
  for (int e = threadIdx.x; e < kGJRows * kGJ; e += 256) {
    const int ii = e / kGJ, c = e % kGJ;
    Aik[ii][c] = (ii < nr && c < b) ? A[(size_t)(r0 + ii) * n + k0 + c] : 0.0;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nr * n; e += 256) {
    const int ii = e / n, j = e % n, i = r0 + ii;
    const bool iK = i >= k0 && i < k0 + b, jK = j >= k0 && j < k0 + b;
    double* a = A + (size_t)i * n + j;
    if (iK) {
      *a = jK ? T0[(i - k0) * kGJ + (j - k0)] : T1[(size_t)(i - k0) * n + j];
    } else if (jK) {
      double acc = 0.0;
      for (int c = 0; c < b; ++c) acc = fma(Aik[ii][c], T0[c * kGJ + (j - k0)], acc);
      *a = -acc;
    } else {
      double acc = *a;
      for (int c = 0; c < b; ++c) acc = fma(-Aik[ii][c], T1[(size_t)c * n + j], acc);
      *a = acc;
    }
  }
}

// V[dA][dout] (f64) of block j from the gradient's kernel rows and bias row
__global__ __launch_bounds__(256) void kfac_gather_kernel(const float* __restrict__ grad, const KfacBlockJob* __restrict__ jobs,
                                                          double* __restrict__ buf) {
  const KfacBlockJob jb = jobs[blockIdx.y];
  const int dA = jb.din + (jb.bias_off >= 0 ? 1 : 0);
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)dA * jb.dout) return;
  const int r = (int)(i / jb.dout), c = (int)(i % jb.dout);
  const float g = r < jb.din ? grad[jb.kernel_off + i] : grad[jb.bias_off + c];
  buf[jb.v_off + i] = g;
}

// batched f64 GEMM C = A B (row-major), 32 x 32 tiles, 256 threads x 4 outputs
__global__ __launch_bounds__(256) void kfac_gemm_kernel(const KfacGemmJob* __restrict__ jobs, double* __restrict__ buf) {
  const KfacGemmJob jb = jobs[blockIdx.z];
  const int tm = blockIdx.y * 32, tn = blockIdx.x * 32;
  if (tm >= jb.M || tn >= jb.N) return;
  const double* A = buf + jb.a_off;
  const double* B = buf + jb.b_off;
  double* C = buf + jb.c_off;
  __shared__ double As[32][17], Bs[16][33];
  const int tr = threadIdx.x / 32, tc = threadIdx.x % 32;  // rows tr, tr + 8, tr + 16, tr + 24
  double acc[4] = {0, 0, 0, 0};
  for (int k0 = 0; k0 < jb.K; k0 += 16) {
    for (int e = threadIdx.x; e < 32 * 16; e += 256) {
      const int r = e / 16, k = e % 16;
      As[r][k] = (tm + r < jb.M && k0 + k < jb.K) ? A[(size_t)(tm + r) * jb.K + k0 + k] : 0.0;
      const int kb = e / 32, c = e % 32;
      Bs[kb][c] = (k0 + kb < jb.K && tn + c < jb.N) ? B[(size_t)(k0 + kb) * jb.N + tn + c] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const double bv = Bs[k][tc];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = fma(As[tr + 8 * u][k], bv, acc[u]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = tm + tr + 8 * u, c = tn + tc;
    if (r < jb.M && c < jb.N) C[(size_t)r * jb.N + c] = acc[u];
  }
}

// P V of block j back into the reference layout (f32)
__global__ __launch_bounds__(256) void kfac_scatter_kernel(const double* __restrict__ buf,
                                                           const KfacBlockJob* __restrict__ jobs, float* __restrict__ pg) {
  const KfacBlockJob jb = jobs[blockIdx.y];
  const int dA = jb.din + (jb.bias_off >= 0 ? 1 : 0);
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)dA * jb.dout) return;
  const int r = (int)(i / jb.dout), c = (int)(i % jb.dout);
  const float v = (float)buf[jb.pv_off + i];
  if (r < jb.din)
    pg[jb.kernel_off + i] = v;
  else
    pg[jb.bias_off + c] = v;
}

// generic blocks: pg = g / (raw_diag / weight + lambda)
__global__ __launch_bounds__(256) void kfac_generic_pc_kernel(const float* __restrict__ grad,
                                                              const float* __restrict__ raw_diag, KfacGenTable tab,
                                                              float* __restrict__ pg, double inv_weight, double lambda) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= tab.total) return;
  int s = 0;
  while (s + 1 < tab.n && tab.cmp[s + 1] <= c) ++s;
  const size_t ref = tab.ref[s] + (c - tab.cmp[s]);
  pg[ref] = (float)((double)grad[ref] / ((double)raw_diag[c] * inv_weight + lambda));
}

// info[0] += sum pg * g (double; info zeroed by the caller)
__global__ __launch_bounds__(256) void kfac_dot_kernel(const float* __restrict__ pg, const float* __restrict__ g,
                                                       size_t n, double* __restrict__ info) {
  __shared__ double red[256];
  double s = 0.0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    s += (double)pg[i] * (double)g[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(info, red[0]);
}

// p -= lr c pg, c = min(1, sqrt(nc / (lr^2 <pg, g>))) (kfac_jax norm constraint);
// info = [<pg, g>, c, lr c]
__global__ __launch_bounds__(256) void kfac_update_kernel(float* __restrict__ p, const float* __restrict__ pg, size_t n,
                                                          double* __restrict__ info, double lr, double norm_constraint) {
  const double sq = info[0];
  const double c = (sq > 0.0 && norm_constraint > 0.0) ? fmin(1.0, sqrt(norm_constraint / (lr * lr * sq))) : 1.0;
  const float step = (float)(lr * c);
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] -= step * pg[i];
  if (i == 0) {
    info[1] = c;
    info[2] = lr * c;
  }
}

// ---- "sparse" orbitals (oracle/kfac.py header): the rows of spin block
// [lo, lo + na) of every walker, r = w * na + i -> full row w * N + lo + i.
__device__ __forceinline__ size_t sparse_row(int r, int na, int N, int lo) {
  return (size_t)(r / na) * N + lo + (r % na);
}

// tangent of the featured orbitals (the lll_weight input): out[r][a NK + jk] =
// sum_m lll[a][m] dF[row(r)][(seg M + m) NK + jk]   (seg = 2 blk + part of the full layout)
__global__ __launch_bounds__(256) void kfac_sparse_dphi_kernel(const float* __restrict__ dF, int ld,
                                                               const float* __restrict__ lll, int M, int NK, int seg,
                                                               int nr, int na, int N, int lo, float* __restrict__ out) {
  const size_t n = (size_t)nr * 8 * NK;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const int r = (int)(i / (8 * NK)), c = (int)(i % (8 * NK));
    const int a = c / NK, jk = c % NK;
    const float* src = dF + sparse_row(r, na, N, lo) * ld + (size_t)seg * M * NK + jk;
    double acc = 0.0;
    for (int m = 0; m < M; ++m) acc += (double)lll[a * M + m] * (double)src[(size_t)m * NK];
    out[i] = (float)acc;
  }
}

// the lll_weight output tangent (real part = the real feature segment seg) as rows of M:
// out[(r NK + jk) M + m] = dF[row(r)][(seg M + m) NK + jk]
__global__ __launch_bounds__(256) void kfac_sparse_regroup_kernel(const float* __restrict__ dF, int ld, int M, int NK,
                                                                  int seg, int nr, int na, int N, int lo,
                                                                  float* __restrict__ out) {
  const size_t n = (size_t)nr * NK * M;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const int m = (int)(i % M);
    const size_t q = i / M;
    const int r = (int)(q / NK), jk = (int)(q % NK);
    out[i] = dF[sparse_row(r, na, N, lo) * ld + ((size_t)seg * M + m) * NK + jk];
  }
}

}  // namespace

void launch_kfac_sparse_dphi(const float* dF, int ld, const float* lll, int M, int NK, int seg, int nr, int na, int N,
                             int lo, float* out, hipStream_t s) {
  const size_t n = (size_t)nr * 8 * NK;
  hipLaunchKernelGGL(kfac_sparse_dphi_kernel, dim3((unsigned)std::min<size_t>(4096, (n + 255) / 256)), dim3(256), 0, s,
                     dF, ld, lll, M, NK, seg, nr, na, N, lo, out);
}

void launch_kfac_sparse_regroup(const float* dF, int ld, int M, int NK, int seg, int nr, int na, int N, int lo,
                                float* out, hipStream_t s) {
  const size_t n = (size_t)nr * NK * M;
  hipLaunchKernelGGL(kfac_sparse_regroup_kernel, dim3((unsigned)std::min<size_t>(4096, (n + 255) / 256)), dim3(256), 0,
                     s, dF, ld, M, NK, seg, nr, na, N, lo, out);
}

void launch_kfac_aug(const float* P, int nch, int n, float* out, int ld, float scale, float corner, int acc,
                     hipStream_t s) {
  hipLaunchKernelGGL(kfac_aug_kernel, dim3(nblk(n)), dim3(256), 0, s, P, nch, n, out, ld, scale, corner, acc);
}

void launch_kfac_feat_gram(const Dims& d, const float* geo, int rows, float* P, hipStream_t s) {
  hipLaunchKernelGGL(kfac_feat_gram_kernel, dim3(grad_chunks(rows)), dim3(256), 0, s, geo, rows, d.N, d.n_up,
                     kGradChunk, P);
}

void launch_kfac_fisher_ct(const float* logpsi, int nw, float* ct, hipStream_t s) {
  hipLaunchKernelGGL(kfac_fisher_ct_kernel, dim3(nblk(nw)), dim3(256), 0, s, logpsi, nw, ct);
}

void launch_kfac_generic(const float* fgrad, const KfacGenTable& tab, float* diag, float scale, hipStream_t s) {
  if (tab.total > 0)
    hipLaunchKernelGGL(kfac_generic_kernel, dim3(nblk(tab.total)), dim3(256), 0, s, fgrad, tab, diag, scale);
}

void launch_kfac_ema(float* raw, const float* st, size_t n, float ema, hipStream_t s) {
  hipLaunchKernelGGL(kfac_ema_kernel, dim3(nblk(n)), dim3(256), 0, s, raw, st, n, ema);
}

void launch_kfac_invert(const KfacDevPlan& p, const float* raw, double inv_weight, double sqrt_lambda, double* tr,
                        double* gj, double* tmp, hipStream_t s) {
  hipLaunchKernelGGL(kfac_trace_kernel, dim3(p.nslots), dim3(256), 0, s, raw, p.slots, tr);
  hipLaunchKernelGGL(kfac_damp_kernel, dim3(nblk((size_t)p.nmax * p.nmax), p.njobs), dim3(256), 0, s, raw, p.slots,
                     p.inv_jobs, tr, gj, inv_weight, sqrt_lambda);
  const size_t tstride = (size_t)kGJ * kGJ + (size_t)kGJ * p.nmax;
  for (int k0 = 0; k0 < p.nmax; k0 += kGJ) {
    hipLaunchKernelGGL(gj_panel_kernel, dim3(p.njobs), dim3(256), 0, s, p.inv_jobs, gj, k0, tmp, tstride);
    hipLaunchKernelGGL(gj_update_kernel, dim3((p.nmax + kGJRows - 1) / kGJRows, p.njobs), dim3(256), 0, s, p.inv_jobs,
                       gj, k0, tmp, tstride);
  }
}

size_t kfac_gj_tmp_doubles(int njobs, int nmax) { return (size_t)njobs * ((size_t)kGJ * kGJ + (size_t)kGJ * nmax); }

void launch_kfac_precondition(const KfacDevPlan& p, const float* grad, const float* raw_diag, double inv_weight,
                              double lambda, double* buf, float* pg, size_t nref, double* info, hipStream_t s) {
  (void)hipMemsetAsync(pg, 0, nref * sizeof(float), s);
  (void)hipMemsetAsync(info, 0, 4 * sizeof(double), s);
  const unsigned g1 = nblk((size_t)p.max_v);
  hipLaunchKernelGGL(kfac_gather_kernel, dim3(g1, p.nblocks), dim3(256), 0, s, grad, p.block_jobs, buf);
  hipLaunchKernelGGL(kfac_gemm_kernel, dim3((p.max_n + 31) / 32, (p.max_m + 31) / 32, p.nblocks), dim3(256), 0, s,
                     p.gemm1, buf);
  hipLaunchKernelGGL(kfac_gemm_kernel, dim3((p.max_n + 31) / 32, (p.max_m + 31) / 32, p.nblocks), dim3(256), 0, s,
                     p.gemm2, buf);
  hipLaunchKernelGGL(kfac_scatter_kernel, dim3(g1, p.nblocks), dim3(256), 0, s, buf, p.block_jobs, pg);
  if (p.gen.total > 0)
    hipLaunchKernelGGL(kfac_generic_pc_kernel, dim3(nblk(p.gen.total)), dim3(256), 0, s, grad, raw_diag, p.gen, pg,
                       inv_weight, lambda);
  hipLaunchKernelGGL(kfac_dot_kernel, dim3(std::min<unsigned>(1024, nblk(nref))), dim3(256), 0, s, pg, grad, nref,
                     info);
}

void launch_kfac_update(float* params, const float* pg, size_t n, double* info, double lr, double norm_constraint,
                        hipStream_t s) {
  hipLaunchKernelGGL(kfac_update_kernel, dim3(nblk(n)), dim3(256), 0, s, params, pg, n, info, lr, norm_constraint);
}

}  // namespace dh
