// Envelope contraction + batched complex slogdet + local-energy assembly.
//
// Orbital features F (output of the orbital GEMM, blocks.py:27-35) have rows
// (walker, electron i, channel c) and columns ((blk*2+part)*M + m)*N*K + j*K + k.
//   Phi_k[i][j] = sum_m F[i,m,j,k] env[i,m],  env = c_m u^(Q+m) v^(Q-m)   (blocks.py:64-68)
//   log psi     = J + log sum_k exp(log det Phi_k)                       (psiformer.py:74-76, 91)
// (exp(J/N) * Phi inside the determinant, psiformer.py:91, is added as J outside.)
//
// value kernel  (one 64-thread workgroup per walker): log psi only, LU with partial
//               pivoting (|re|+|im| pivot choice, as LAPACK getrf).
// energy kernel (one 256-thread workgroup per walker): channel determinants
//   l_t  = tr(B Phi_t),  B = Phi0^-1 (Gauss-Jordan, partial pivoting)
//   l_L  = tr(B Phi_L) - sum_t tr((B Phi_t)^2)
//   l_Sk = tr(B Phi_Sk) - tr((B Phi_uk)^2),  Phi_uk = sum_t alpha_kt Phi_t
// with Phi channels from the product rule of F and the envelope leaves, then
// Jastrow, potential and the KE / Lz / Lz^2 / L^2 assembly (DESIGN.md §3.4,
// equivalent to hamiltonian.py:115-169).
#include <cstdlib>
#include <type_traits>

#include "dh_internal.h"
#include "device_common.h"
#include "mcmc_common.h"

#ifndef DET_LU_REG  // A/B knob: det_value's LU with one column per lane in registers (1) or eliminate (0):
#define DET_LU_REG 0  // bitwise equal, measured 0.3-0.7 us per call slower at C2 (profiles/r05_v17_det_ab.txt)
#endif
#ifndef DET_WAVE_SQ  // A/B knob: det_energy_wave's envelope leaves with integer powers by squaring (1) or powf (0):
#define DET_WAVE_SQ 1  // det_energy 185 -> 170 us at C2, GPU suite green (profiles/r05_v28_det_sq_ab.txt)
#endif
#ifndef DET_LEAF_SQ  // A/B knob: the envelope leaves of env_contract / env_stream / det_energy_kernel (N > 8) by powers
#define DET_LEAF_SQ 1   // by squaring (1) or powf (0): C5 det class 8.41 -> 8.11 ms (profiles/r05_v32_leaf_sq_ab.txt)
#endif
#ifndef DET_GJ_REG  // A/B knob: det_energy_wave's B = Phi0^-1 by register Gauss-Jordan (1) or eliminate (0)
#define DET_GJ_REG 1
#endif
#ifndef DET_STAMP  // diagnostic builds only (tools/det_stamp.py): phase stamps of det_value / det_energy_wave
#define DET_STAMP 0
#endif
#if DET_STAMP
// [2][DET_STAMP_WG][DET_NSTAMP]: slot 0 = det_value_kernel, slot 1 = det_energy_wave_kernel
constexpr int DET_STAMP_WG = 1024, DET_NSTAMP = 12;
__device__ unsigned long long g_det_stamp[2 * DET_STAMP_WG * DET_NSTAMP];
#define DET_T(slot, i)                                                                                       \
  do {                                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < DET_STAMP_WG)                                                       \
      g_det_stamp[((slot) * DET_STAMP_WG + blockIdx.x) * DET_NSTAMP + (i)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
extern "C" int dh_debug_det_stamps(unsigned long long* out, int n) {
  n = n < 2 * DET_STAMP_WG * DET_NSTAMP ? n : 2 * DET_STAMP_WG * DET_NSTAMP;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_det_stamp), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#else
#define DET_T(slot, i)
#endif

namespace dh {
namespace {

__device__ inline float ipow(float b, int e) { return e < 0 ? 0.f : (e == 0 ? 1.f : powf(b, (float)e)); }
// integer power by squaring (the envelope values and leaves: a few multiplies per power instead
// of powf's log / exp).  Not powf's 1-ulp result: squaring doubles the relative error it
// carries, so b^e is within about (e + popcount(e)) * 2^-24 relative (< 4e-6 at e = 57, C5's
// largest exponent) against powf's ~6e-8; tests/test_gpu_kernels.py::test_env_leaf_powers
// bounds both forms against float64 at M = 58 near the poles (dh_debug_env_leaf)
__device__ inline float ipow_sq(float b, int e) {
  float r = 1.f;
  for (; e > 0; e >>= 1, b *= b)
    if (e & 1) r *= b;
  return r;
}

// F element (complex) of row `row` at (blk, m, j, k)
struct FView {
  const float* F;
  int ld, M, N, K;
  __device__ inline cf at(size_t row, int blk, int m, int j, int k) const {
    const size_t base = row * ld;
    const int MNK = M * N * K;
    const int off = m * N * K + j * K + k;
    return cf{F[base + (size_t)(blk * 2) * MNK + off], F[base + (size_t)(blk * 2 + 1) * MNK + off]};
  }
};

// envelope value (and optionally leaves) for electron angle (th, ph), harmonic index p
struct EnvLeaf {
  cf e0, dth, dph, lb, d2th;
};
// `gauge` = kappa removes the per-electron phase exp(i kappa phi) from the envelope (0 =
// reference gauge); the removed term i sum_i kappa_i phi_i is added back analytically (in
// double) by the energy assembly.  kappa_i = env_gauge(cos theta_i): the envelope's dominant
// harmonic m* = Q cos theta (|u|^2 = cos^2 theta/2 weights Q + m binomially), so the phi
// derivatives i (m - kappa) of the contracted orbitals stay small for every electron.  At the
// poles this is the north / south patch (kappa = +-Q: regular channels where the reference's
// 1 / sin theta terms blow up); near the equator it stays ~0 where the patch choice put up to
// 2Q into every phi channel and the f32 contractions below lost the digits.
// Quantised to 1/64 of Q so that m - kappa is exact in f32.
__device__ __forceinline__ float env_gauge(float ct, int M) {
  return (float)(M - 1) * __builtin_rintf(64.f * ct) * (1.f / 128.f);
}
__device__ inline EnvLeaf env_leaf(float th, float ph, int p, int M, float norm, bool leaves, float gauge = 0.f,
                                   bool sq = false) {
  const int a = p, b = M - 1 - p;
  const float m = 0.5f * (float)(a - b) - gauge;
  float c, s;
  sincosf(0.5f * th, &s, &c);
  float sph, cph;
  sincosf(m * ph, &sph, &cph);
  const float R = sq ? ipow_sq(c, a) * ipow_sq(s, b) : ipow(c, a) * ipow(s, b);
  EnvLeaf L;
  L.e0 = cf{norm * R * cph, norm * R * sph};
  if (leaves) {
    const float fa = (float)a, fb = (float)b;
    // sq: the powers by squaring here too (negative exponents 0, as ipow)
    auto pw = [sq](float x, int e) { return sq ? (e < 0 ? 0.f : ipow_sq(x, e)) : ipow(x, e); };
    const float R1 = 0.5f * (fb * pw(c, a + 1) * pw(s, b - 1) - fa * pw(c, a - 1) * pw(s, b + 1));
    const float R2 = 0.25f * (fb * (fb - 1.f) * pw(c, a + 2) * pw(s, b - 2) - fb * (fa + 1.f) * R -
                              fa * (fb + 1.f) * R + fa * (fa - 1.f) * pw(c, a - 2) * pw(s, b + 2));
    float st, ct;
    sincosf(th, &st, &ct);
    L.dth = cf{norm * R1 * cph, norm * R1 * sph};
    L.d2th = cf{norm * R2 * cph, norm * R2 * sph};
    // d/dphi / sin th = i m e0 / st
    L.dph = cf{-m * L.e0.im / st, m * L.e0.re / st};
    // LB = d2th - m^2 e0 / st^2 + cot th * dth
    const float cot = ct / st;
    const float k2 = m * m / (st * st);
    L.lb = cf{L.d2th.re - k2 * L.e0.re + cot * L.dth.re, L.d2th.im - k2 * L.e0.im + cot * L.dth.im};
  }
  return L;
}

// second derivative of the envelope along the rotation flow about axis k
__device__ inline cf env_flow2(const cf& e0, const cf& dth, const cf& d2th, float m, float st, float ct, float sp,
                               float cp, int k) {
  const float cot = ct / st;
  const float ph_hat[3] = {-sp, cp, 0.f};
  const float th_hat[3] = {ct * cp, ct * sp, -st};
  const float thp[3] = {cp * cot, sp * cot, -1.f};
  const float dthp_dth[3] = {-cp / (st * st), -sp / (st * st), 0.f};
  const float dthp_dph[3] = {-sp * cot, cp * cot, 0.f};
  const float cs[3] = {cp, sp, 0.f};
  const float td = ph_hat[k];
  const float pd = -th_hat[k] / st;
  const float tdd = cs[k] * thp[k];
  const float pdd = -(dthp_dth[k] * td - dthp_dph[k] * thp[k]);
  // d_thph = i m dth ; d_phph = -m^2 e0 ; d_ph = i m e0
  cf r;
  r.re = d2th.re * td * td + 2.f * (-m * dth.im) * td * pd + (-m * m * e0.re) * pd * pd + dth.re * tdd +
         (-m * e0.im) * pdd;
  r.im = d2th.im * td * td + 2.f * (m * dth.re) * td * pd + (-m * m * e0.im) * pd * pd + dth.im * tdd +
         (m * e0.re) * pdd;
  return r;
}

// the first `width` threads (a wave, or a half-wave per walker) find the pivot row (first
// max of |re|+|im| in column p, rows >= p)
__device__ inline void find_pivot(const cf* A, int lda, int N, int p, int* piv, int tid, int width) {
  if (tid < width) {
    const int lane = tid;
    float best = -1.f;
    int bi = N;
    for (int r = p + lane; r < N; r += width) {
      const float v = cabs1(A[r * lda + p]);
      if (v > best) {
        best = v;
        bi = r;
      }
    }
    for (int o = width >> 1; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, width);
      const int oi = __shfl_xor(bi, o, width);
      if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    if (lane == 0) *piv = (bi < N) ? bi : p;
  }
}

// In-place elimination on A [N][ncol] (lda) with partial pivoting.
//   gj = true : Gauss-Jordan on an augmented [A | I] (ncol = 2N): right block -> A^-1
//   gj = false: LU (rows below the pivot only) — determinant only
// Accumulates log det into logdet (complex, phase unwrapped).  Uses __syncthreads.
// tid / nt: this walker's threads (default the whole block; det_value's half-wave form
// passes its 32 lanes and width 32 for the pivot search).
__device__ __forceinline__ void eliminate(cf* A, int lda, int N, int ncol, bool gj, cf* fac, int* piv, cf* logdet,
                          int tid = threadIdx.x, int nt = blockDim.x, int width = 64) {
  if (tid == 0) *logdet = cf{0.f, 0.f};
  __syncthreads();
  for (int p = 0; p < N; ++p) {
    find_pivot(A, lda, N, p, piv, tid, width);
    __syncthreads();
    const int pr = *piv;
    if (pr != p) {
      for (int c = tid; c < ncol; c += nt) {
        const cf t = A[p * lda + c];
        A[p * lda + c] = A[pr * lda + c];
        A[pr * lda + c] = t;
      }
    }
    __syncthreads();
    const cf P = A[p * lda + p];
    if (tid == 0) {
      const float mag = sqrtf(P.re * P.re + P.im * P.im);
      logdet->re += logf(mag);
      logdet->im += atan2f(P.im, P.re) + (pr != p ? kPi : 0.f);
    }
    const cf Pinv = cdiv(cf{1.f, 0.f}, P);
    __syncthreads();
    if (gj) {
      for (int r = tid; r < N; r += nt) fac[r] = (r == p) ? cf{0.f, 0.f} : A[r * lda + p];
      for (int c = tid; c < ncol; c += nt) A[p * lda + c] = A[p * lda + c] * Pinv;
    } else {
      for (int r = tid; r < N; r += nt) fac[r] = (r > p) ? A[r * lda + p] * Pinv : cf{0.f, 0.f};
    }
    __syncthreads();
    const int r0 = gj ? 0 : p + 1;
    const int c0 = gj ? 0 : p;
    const int nr = N - r0, nc = ncol - c0;
    for (int idx = tid; idx < nr * nc; idx += nt) {
      const int r = r0 + idx / nc, c = c0 + idx % nc;
      if (r == p) continue;
      const cf f = fac[r];
      cf v = A[r * lda + c];
      const cf a = A[p * lda + c];
      v.re -= f.re * a.re - f.im * a.im;
      v.im -= f.re * a.im + f.im * a.re;
      A[r * lda + c] = v;
    }
    __syncthreads();
  }
}

// eliminate(Aug, 2N, N, 2N, gj = true) for N <= NMAX, column c of the augmented [A | I] in
// registers of lane c < 2 N (round 5, det_energy_wave_kernel): the same pivots and log det
// terms; pivot row scaled by 1 / P, every other row r minus A[r][p] times it.  The factors reach
// the lanes by shuffles, no LDS round trips.  Not bitwise the LDS form (the compiler fuses the
// complex products differently); B = A^-1 ends in lanes N .. 2 N - 1.
template <int NMAX>
__device__ __forceinline__ cf gj_inverse_cols(cf (&col)[NMAX], int N) {
  auto is = [](int r, int q) __attribute__((always_inline)) {
    int m = r == q;
    asm volatile("" : "+v"(m));
    return m != 0;
  };
  auto pick = [&](int q) __attribute__((always_inline)) {
    cf v = col[0];
#pragma unroll
    for (int r = 1; r < NMAX; ++r)
      if (is(r, q)) v = col[r];
    return v;
  };
  float lre = 0.f, lim = 0.f;
  for (int p = 0; p < N; ++p) {
    float best = -1.f;
    int bi = N;
#pragma unroll
    for (int r = 0; r < NMAX; ++r) {
      if (r >= p && r < N) {
        const float v = cabs1(col[r]);
        if (v > best) {
          best = v;
          bi = r;
        }
      }
    }
    int pr = __shfl(bi, p, 64);
    pr = pr < N ? pr : p;
    if (pr != p) {
      const cf a = pick(p), b = pick(pr);
#pragma unroll
      for (int r = 0; r < NMAX; ++r) {
        if (is(r, p)) col[r] = b;
        if (is(r, pr)) col[r] = a;
      }
    }
    const cf mine = pick(p);
    const cf P{__shfl(mine.re, p, 64), __shfl(mine.im, p, 64)};
    const float mag = sqrtf(P.re * P.re + P.im * P.im);
    lre += logf(mag);
    lim += atan2f(P.im, P.re) + (pr != p ? kPi : 0.f);
    const cf rowp = mine * cdiv(cf{1.f, 0.f}, P);
#pragma unroll
    for (int r = 0; r < NMAX; ++r) {
      if (r < N) {
        const cf f{__shfl(col[r].re, p, 64), __shfl(col[r].im, p, 64)};  // A[r][p]
        cf v = col[r];
        v.re -= f.re * rowp.re - f.im * rowp.im;
        v.im -= f.re * rowp.im + f.im * rowp.re;
        col[r] = is(r, p) ? rowp : v;
      }
    }
  }
  return cf{lre, lim};
}

// eliminate(A, N, N, N, gj = false) for N <= NMAX with column c of A in registers of lane c
// of the (half-)wave (round 5): the same pivots (first maximum of cabs1 at or below the
// diagonal), the same factors f = A[r][p] / P and updates of columns c >= p, the same log det
// terms — without LDS round trips or barriers (the pivot search is lane p's own column, the
// pivot and factors reach the other lanes by shuffles).  Register arrays are indexed only by
// compile-time constants (selects), or they would go to scratch.
template <int NMAX>
__device__ __forceinline__ cf lu_logdet_cols(cf (&col)[NMAX], int N, int lane, int width) {
  // r == q through an opaque value: left visible, the compiler turns the select chain into a
  // run-time index of col (and col into scratch)
  auto is = [](int r, int q) __attribute__((always_inline)) {
    int m = r == q;
    asm volatile("" : "+v"(m));
    return m != 0;
  };
  auto pick = [&](int q) __attribute__((always_inline)) {
    cf v = col[0];
#pragma unroll
    for (int r = 1; r < NMAX; ++r)
      if (is(r, q)) v = col[r];
    return v;
  };
  float lre = 0.f, lim = 0.f;
  for (int p = 0; p < N; ++p) {
    float best = -1.f;
    int bi = N;
#pragma unroll
    for (int r = 0; r < NMAX; ++r) {
      if (r >= p && r < N) {
        const float v = cabs1(col[r]);
        if (v > best) {
          best = v;
          bi = r;
        }
      }
    }
    int pr = __shfl(bi, p, width);
    pr = pr < N ? pr : p;
    if (pr != p) {  // swap rows p and pr (every column)
      const cf a = pick(p), b = pick(pr);
#pragma unroll
      for (int r = 0; r < NMAX; ++r) {
        if (is(r, p)) col[r] = b;
        if (is(r, pr)) col[r] = a;
      }
    }
    const cf mine = pick(p);  // A[p][lane]
    const cf P{__shfl(mine.re, p, width), __shfl(mine.im, p, width)};
    const float mag = sqrtf(P.re * P.re + P.im * P.im);
    lre += logf(mag);
    lim += atan2f(P.im, P.re) + (pr != p ? kPi : 0.f);
    const cf Pinv = cdiv(cf{1.f, 0.f}, P);
#pragma unroll
    for (int r = 0; r < NMAX; ++r) {
      if (r > p && r < N) {
        // the roundings of eliminate's code (its factor and update as the compiler emits them:
        // one product of each pair fused), so that equal rows cancel exactly as there and a
        // singular matrix keeps its zero pivot (psi = 0, tests/test_gpu_grad.py)
#pragma clang fp contract(off)
        const cf c = col[r];
        const cf fl{c.re * Pinv.re - c.im * Pinv.im, __builtin_fmaf(c.im, Pinv.re, c.re * Pinv.im)};
        const cf f{__shfl(fl.re, p, width), __shfl(fl.im, p, width)};  // lane p's: row r's factor
        if (lane >= p) {
          const float tre = __builtin_fmaf(f.re, mine.re, -(f.im * mine.im));
          const float tim = __builtin_fmaf(f.im, mine.re, f.re * mine.im);
          col[r] = cf{c.re - tre, c.im - tim};
        }
      }
    }
  }
  return cf{lre, lim};
}

__device__ inline double jastrow_pair(double r, double al, double cst, double* f1, double* f2) {
  const double ar = al + r;
  *f1 = (cst * al * al) / (ar * ar);
  *f2 = -2.0 * (cst * al * al) / (ar * ar * ar);
  return -(cst * al * al) / ar;
}

// ------------------------------------------------------------------ value kernel
// The orbital matrix is contracted row by row: lane (j, g) sums harmonics m = g + G u
// (G = 64 / N lane groups, u < MGV, all loads of a row in flight at once, one wave load
// instruction covering G consecutive harmonics = 4 G N contiguous bytes), groups combined
// with shuffles.
// HW (MGV = 0 only): two walkers per wave, one per 32-lane half (per-walker LDS regions of
// `per` floats): the serial parts (pivot search, log det, Jastrow reduction) then serve two
// walkers per instruction.
template <int MGV, bool HW = false>
// x is not __restrict__: with the MCMC epilogue it is the same buffer as epi.x2, which the
// epilogue writes (each thread reads its own walker's angles before that, behind a barrier)
__global__ __launch_bounds__(64) void det_value_kernel(const float* __restrict__ Fp, int ldF, const float* x,
                                 const float* __restrict__ jas, const float* __restrict__ norm, float* __restrict__ logpsi,
                                 int N, int n_up, int M, int K, int nw, int per, McmcEpi epi) {
  static_assert(!HW || MGV == 0, "half-wave form: serial contraction only");
  extern __shared__ float sm_all[];
  const int half = HW ? (int)(threadIdx.x >> 5) : 0;
  float* sm_raw = sm_all + half * per;
  cf* E0 = reinterpret_cast<cf*>(sm_raw);  // [N][M]
  cf* A = E0 + N * M;                      // [N][N]
  cf* fac = A + N * N;                     // [N]
  cf* ld = fac + N;                        // [K] log dets
  cf* logdet = ld + K;
  int* piv = reinterpret_cast<int*>(logdet + 1);
  const int bw = HW ? 2 * (int)blockIdx.x + half : (int)blockIdx.x;
  const bool live = bw < nw;
  const int b = live ? bw : nw - 1;  // a dead half repeats the last walker, writes nothing
  const int tid = HW ? (int)(threadIdx.x & 31) : (int)threadIdx.x, nt = HW ? 32 : 64, width = HW ? 32 : 64;
  double* cart = reinterpret_cast<double*>(piv + 2);  // [N][3] unit vectors (double: close pairs)
  DET_T(0, 0);
  for (int idx = tid; idx < N * M; idx += nt) {
    const int i = idx / M, p = idx % M;
    E0[idx] = env_leaf(x[2 * (b * N + i)], x[2 * (b * N + i) + 1], p, M, norm[p], false, 0.f, true).e0;
  }
  for (int i = tid; i < N; i += nt) {
    double st, ct, sp, cp;
    sincos((double)x[2 * (b * N + i)], &st, &ct);
    sincos((double)x[2 * (b * N + i) + 1], &sp, &cp);
    cart[3 * i] = st * cp;
    cart[3 * i + 1] = st * sp;
    cart[3 * i + 2] = ct;
  }
  __syncthreads();
  DET_T(0, 1);
  // Jastrow (blocks.py:76-121): chord distances on the unit sphere, pairs spread over the
  // wave, accumulated in double and reduced with shuffles (one 64-lane wave per walker)
  double Jw = 0.0;
  {
    const double ap = jas[0], aa = jas[1];
    for (int q = tid; q < N * N; q += nt) {
      const int i = q / N, j = q - (q / N) * N;
      if (j <= i) continue;
      const double dx = cart[3 * j] - cart[3 * i], dy = cart[3 * j + 1] - cart[3 * i + 1],
                   dz = cart[3 * j + 2] - cart[3 * i + 2];
      const double r = sqrt(dx * dx + dy * dy + dz * dz);
      const bool same = (i < n_up) == (j < n_up);
      double f1, f2;
      Jw += jastrow_pair(r, same ? ap : aa, same ? 0.25 : 0.5, &f1, &f2);
    }
    for (int o = width >> 1; o > 0; o >>= 1) Jw += __shfl_xor(Jw, o, width);
  }
  DET_T(0, 2);
  const int G = 64 / N, gj = tid % N, gg = tid / N, NK = N * K, MNK = M * NK;
  for (int k = 0; k < K; ++k) {
    if constexpr (MGV == 0) {  // small rows: one thread per entry, serial over m
      for (int idx = tid; idx < N * N; idx += nt) {
        const int i = idx / N, j = idx % N;
        const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
        const float* rp = Fp + ((size_t)b * N + i) * ldF + (size_t)blk * 2 * MNK + (size_t)j * K + k;
        cf acc{0.f, 0.f};
        // 16 harmonics' loads in flight at once (a loop with the trip count M at run time
        // waited for every pair before its FMA: 16 L2 round trips in a row at C2); the same
        // products summed in the same order
        for (int p0 = 0; p0 < M; p0 += 16) {
          float fr[16], fi[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const size_t p = (size_t)min(p0 + q, M - 1);
            fr[q] = rp[p * NK];
            fi[q] = rp[(size_t)MNK + p * NK];
          }
#pragma unroll
          for (int q = 0; q < 16; ++q)
            if (p0 + q < M) cfma(acc, cf{fr[q], fi[q]}, E0[i * M + p0 + q]);
        }
        A[idx] = acc;
      }
    }
    if constexpr (MGV > 0) {
      // row i's F loads in flight while row i - 1 is contracted (two register sets, rows in
      // pairs; round 5): one row at a time waited for every row's L2 / HBM round trip (C5: 20
      // rows, 63 % of the kernel, profiles/r05_v17_det_stamps_c5.txt).  The loads are
      // unconditional (clamped harmonic and row; out-of-range terms zeroed after the load), so
      // the compiler's counted waits leave the other set in flight.
      constexpr int NF = 2 * (MGV > 0 ? MGV : 1);
      auto ldrow = [&](int i, float (&f)[NF]) __attribute__((always_inline)) {
        const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
        const float* rp = Fp + ((size_t)b * N + i) * ldF + (size_t)blk * 2 * MNK + (size_t)gj * K + k;
#pragma unroll
        for (int u = 0; u < MGV; ++u) {
          const size_t m = (size_t)min(gg + G * u, M - 1);
          f[2 * u] = rp[m * NK];
          f[2 * u + 1] = rp[(size_t)MNK + m * NK];
        }
      };
      auto contract = [&](int i, const float (&f)[NF]) __attribute__((always_inline)) {
        cf acc{0.f, 0.f};
#pragma unroll
        for (int u = 0; u < MGV; ++u) {
          const int m = gg + G * u;
          const bool ok = gg < G && m < M;
          cfma(acc, cf{ok ? f[2 * u] : 0.f, ok ? f[2 * u + 1] : 0.f}, E0[i * M + min(m, M - 1)]);
        }
        float re = acc.re, im = acc.im;
        for (int q = 1; q < G; ++q) {
          re += __shfl(acc.re, gj + N * q, 64);
          im += __shfl(acc.im, gj + N * q, 64);
        }
        if (gg == 0) A[i * N + gj] = cf{re, im};
      };
      float fa[NF], fb[NF];
      if constexpr (MGV <= 24) {
        ldrow(0, fa);
        for (int i = 0; i < N; i += 2) {
          ldrow(min(i + 1, N - 1), fb);
          contract(i, fa);
          ldrow(min(i + 2, N - 1), fa);
          if (i + 1 < N) contract(i + 1, fb);
        }
      } else {  // (the widest forms: a second set would cost the second wave per SIMD)
        for (int i = 0; i < N; ++i) {
          ldrow(i, fa);
          contract(i, fa);
        }
      }
    }
    __syncthreads();
    DET_T(0, 3);
    if (N <= 8 && DET_LU_REG) {  // register LU, one column per lane
      cf col[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) col[r] = (r < N && tid < N) ? A[r * N + tid] : cf{0.f, 0.f};
      const cf l = lu_logdet_cols<8>(col, N, tid, width);
      if (tid == 0) ld[k] = l;
    } else {  // (a 32-row register LU for N = 10, 20 took the C5 form to 256 VGPRs, one wave per SIMD)
      eliminate(A, N, N, N, false, fac, piv, logdet, tid, nt, width);
      if (tid == 0) ld[k] = *logdet;
    }
    __syncthreads();
    DET_T(0, 4);
  }
  float* lpv = reinterpret_cast<float*>(cart + 3 * N);  // this walker's Re log psi for the epilogue
  if (tid == 0 && live) {
    // log-sum-exp over determinants (psiformer.py:74-76)
    float lmax = -INFINITY;
    for (int k = 0; k < K; ++k) lmax = fmaxf(lmax, ld[k].re);
    float zr = 0.f, zi = 0.f;
    for (int k = 0; k < K; ++k) {
      const float mag = expf(ld[k].re - lmax);
      zr += mag * cosf(ld[k].im);
      zi += mag * sinf(ld[k].im);
    }
    float val_re = 0.5f * logf(zr * zr + zi * zi) + lmax;
    float val_im = atan2f(zi, zr);
    logpsi[2 * b] = val_re + (float)Jw;
    logpsi[2 * b + 1] = val_im;
    *lpv = val_re + (float)Jw;
  }
  DET_T(0, 5);
  if (!epi.on) return;
  // ---- MCMC epilogue (McmcEpi): the accept of epi.step for this walker and its next proposal,
  // lane i < N moving electron i — accept_propose_kernel's arithmetic on the same values
  __syncthreads();
  if (!live || tid >= N) return;
  const float lp2 = 2.f * *lpv;
  const bool cond = accept_one(lp2, epi.lp[b], b, N, epi.seed, epi.step, epi.woff, epi.noise);
  const int e = b * N + tid;
  float th = epi.x[2 * e], ph = epi.x[2 * e + 1];
  if (cond) {
    th = x[2 * e];  // x is the proposal this kernel evaluated (epi.x2)
    ph = x[2 * e + 1];
    epi.x[2 * e] = th;
    epi.x[2 * e + 1] = ph;
    if (tid == 0) {
      epi.lp[b] = lp2;
      epi.nacc[b] += 1;
    }
  }
  if (epi.propose)
    propose_one(th, ph, epi.x2, epi.geo, e, b, tid, N, epi.width, epi.seed, epi.step + 1, epi.woff, epi.noise2);
  DET_T(0, 6);
}

// ------------------------------------------------------------------ envelope contraction
// For large orbital rows (2 M N K floats per channel row, C5: 2320) det_energy_kernel no
// longer contracts F itself: this kernel forms, per (walker, det kd, channel c), the
// complex N x N matrices it needs (blocks.py:64-68 with the product rule):
//   c = 0:       Phi0   = sum_m F_0 e0
//   c = 1+t:     Phi_t  = sum_m F_t e0 + [t moves i] sum_m F_0 de/dt
//   c = 1+T:     Phi_L  = sum_m F_L e0 + sum_m F_0 LB(e) + 2 sum_{t moves i} sum_m F_t de/dt
//   c = 2+T+k:   Phi_Sk = sum_m F_Sk e0 + sum_m F_0 e_flow2,k
//                         + 2 sum_t alpha_kt sum_m F_t (phh_k de/dth - thh_k de/dph)
// into PhiC[((b K + kd) C + c) N N + i N + j] (re, im).  One 256-thread workgroup per
// (walker, electron i).  Every term is linear in the harmonic sums, so each of the 4 G lane
// groups (lane (j, g) of wave w, group gg = G w + g, G = 64 / N) forms ALL of them over its
// own harmonics m = gg + 4 G u (u < MG) — partial extras included — and the partials are
// summed at the end (shuffles within a wave, LDS across the four).  A wave load instruction
// covers G consecutive harmonics = 4 G N contiguous bytes.  The channel rows stream through
// a per-wave LDS-DMA ring (global_load_lds_dword, RING rows deep: RING - 1 rows in flight
// without holding registers), counted with vmcnt; every lane reads back only its own words.
// LDS-DMA ring depth: up to 4 rows, (depth - 1) rows of 2 MG loads within vmcnt's 6 bits
#ifndef ENV_REG  // A/B knob: the segment form keeps the tangent rows' envelope factors in registers
#define ENV_REG 1
#endif
#ifndef ENV_SEG_RING  // A/B knob: rows per ring of the segment-DMA form
#define ENV_SEG_RING 4
#endif
constexpr int kEnvSegRing = ENV_SEG_RING;
__host__ __device__ constexpr int env_ring(int MG) { return (63 / (2 * MG) + 1) < 4 ? (63 / (2 * MG) + 1) : 4; }

// WU (short rows, C4): one WAVE per (walker, electron) instead of one workgroup: no
// cross-wave partials, no block barriers, 4 units per workgroup (the leaves of a unit are
// computed by its own 64 lanes).
// SEG > 0 (four waves per electron only): each wave owns a CONTIGUOUS block of MW = ceil(M / 4)
// harmonics, so a channel row's share of a wave is two contiguous segments (re, im: MW N K
// floats each) that come into the ring by SEG global_load_lds_dwordx4 pieces per segment (1 KiB
// each, lanes past the segment masked) instead of 2 MG one-dword pieces: a third of the DMA
// issue slots (an LDS-DMA piece costs ~60-180 cycles to issue, MI355X_MICROARCH.md).  Lane (j, g)
// takes the wave's harmonics g + G u.  The launcher picks it when every piece keeps a lane.
template <int MG, bool WU = false, int SEG = 0>
__global__ __launch_bounds__(256) void env_contract_kernel(const float* __restrict__ Fp, int ldF,
                                                           const float* __restrict__ x,
                                                           const float* __restrict__ geo_g,
                                                           const float* __restrict__ norm, float* __restrict__ PhiC,
                                                           int nw, int N, int n_up, int M, int K, float Q) {
  static_assert(SEG == 0 || !WU, "segment DMA: four waves per electron");
  // SEG: 4 rows per ring (ENV_SEG_RING; 5 fits 80 KiB at C5 and measured no faster)
  constexpr int Q2 = SEG ? 2 * SEG : 2 * MG, RING = SEG ? kEnvSegRing : env_ring(MG);  // load instructions per row, rows per ring
  static_assert((RING - 1) * Q2 <= 63, "vmcnt range");
  extern __shared__ float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int unit = WU ? blockIdx.x * 4 + wv : blockIdx.x;
  if (WU && unit >= nw * N) return;  // whole waves only (no block barriers in the WU form)
  const int b = unit / N, i = unit - (unit / N) * N;
  const int T = 2 * N, C = 2 * N + 5;
  // LDS: WU: per wave [wt | al | ring]; else [wt | part | al | 4 rings]
  const int wsz = WU ? 20 * M + ((3 * T + 3) & ~3) + RING * Q2 * 64 : 0;
  cf* wt = reinterpret_cast<cf*>(sm + (size_t)wv * wsz);  // [E0, DTH, DPH, LB, W0..2, SF0..2][M]
  cf* part = wt + 10 * M;                                 // [4 waves][C][N] partial sums (not WU)
  float* al = reinterpret_cast<float*>(WU ? part : part + 4 * C * N);  // [3][T]
  float* ring = al + ((3 * T + 3) & ~3);                  // [RING][Q2][64] per wave (SEG: [RING][2 segf])
  const int G = 64 / N, j = lane % N, g = lane / N, S = WU ? G : 4 * G;
  const int MW = (M + 3) / 4;                         // SEG: harmonics per wave
  const int gg = SEG ? MW * wv + g : (WU ? g : G * wv + g);
  const int mend = SEG ? min(MW * (wv + 1), M) : M;    // SEG: this wave's harmonics end
  const bool act = g < G;
  const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
  const int NK = N * K, MNK = M * NK;
  auto gsum = [&](float v) __attribute__((always_inline)) {
    float r = v;
    for (int q = 1; q < G; ++q) r += __shfl(v, j + N * q, 64);
    return r;
  };
  auto gsumc = [&](cf v) __attribute__((always_inline)) { return cf{gsum(v.re), gsum(v.im)}; };
  const float* rowbase = Fp + ((size_t)(b * N + i) * C) * ldF + (size_t)blk * 2 * MNK + (size_t)j * K;
  // lane's harmonic u (< MG) is m = gg + S u, valid when m < M (and g < G)
  const int SS = SEG ? G : S;  // harmonic stride of a lane
  auto mw = [&](int u) __attribute__((always_inline)) { return min(gg + SS * u, M - 1); };
  auto okm = [&](int u) __attribute__((always_inline)) { return act && gg + SS * u < mend; };
  const int segf = MW * N * K;  // SEG: floats of one segment
  float* wring = WU ? ring : ring + (size_t)wv * RING * (SEG ? 2 * segf : Q2 * 64);
  const uint32_t ring0 = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)wring);
  // DMA row c of det kd into ring slot c % RING
  // SEG: the wave's segments of row c (re at + 0, im at + MNK floats), lane-linear in the slot
  const float* segbase = Fp + ((size_t)(b * N + i) * C) * ldF + (size_t)blk * 2 * MNK + (size_t)MW * wv * NK;
  const int segb = (mend - MW * wv) * NK * 4;  // bytes this wave really reads per segment
  auto issue = [&](int c, int kd) __attribute__((always_inline)) {
    if constexpr (SEG > 0) {
      (void)kd;  // K == 1 (launcher)
      const int slot = c % RING;
#pragma unroll
      for (int q = 0; q < 2 * SEG; ++q) {
        const int p = q / SEG, piece = q % SEG;  // part (re / im), 1-KiB piece
        const int byte = piece * 1024 + lane * 16;
        const char* src = reinterpret_cast<const char*>(segbase + (size_t)c * ldF + (p ? (size_t)MNK : 0)) + byte;
        const uint32_t dst = __builtin_amdgcn_readfirstlane(ring0 + (uint32_t)(slot * 2 * segf * 4 + p * segf * 4 + piece * 1024));
        if (byte < segb) {  // lane 0 of every piece is inside the segment (launcher's check)
          unsigned keep;
          asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                       : "=&s"(keep)
                       : "v"(src), "s"(dst)
                       : "memory");
        }
      }
      return;
    }
    const float* rp = rowbase + (size_t)c * ldF + kd;
    const int slot = c % RING;
#pragma unroll
    for (int q = 0; q < Q2; ++q) {
      const int u = q >> 1;
      const float* src = okm(u) ? rp + ((q & 1) ? (size_t)MNK : 0) + (size_t)(gg + S * u) * NK : rowbase;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(ring0 + (uint32_t)((slot * Q2 + q) * 256));
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(dst)
                   : "memory");
    }
  };
  // wait until row c landed (rows issued after it: min(RING - 1, C - 1 - c))
  auto wait_row = [&](int c) __attribute__((always_inline)) {
    const int ahead = min(RING - 1, C - 1 - c);
    if constexpr (RING >= 5) {
      if (ahead >= 4) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * Q2) : "memory");
        return;
      }
    }
    if constexpr (RING >= 4) {
      if (ahead >= 3) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * Q2) : "memory");
        return;
      }
    }
    if constexpr (RING >= 3) {
      if (ahead == 2) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * Q2) : "memory");
        return;
      }
    }
    if (ahead == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(Q2) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto fval = [&](int c, int u) __attribute__((always_inline)) {
    if constexpr (SEG > 0) {
      const float* r = wring + (size_t)(c % RING) * 2 * segf + (size_t)(g + G * u) * NK + j;  // K == 1
      return okm(u) ? cf{r[0], r[segf]} : cf{0.f, 0.f};
    }
    const float* r = wring + (size_t)((c % RING) * Q2 + 2 * u) * 64 + lane;
    return okm(u) ? cf{r[0], r[64]} : cf{0.f, 0.f};
  };
  // the first rows' DMA goes out before the envelope leaves are computed (it does not need
  // them); the leaves' few global operands are loaded (and waited for) first, so no
  // compiler-inserted wait inside the leaves drains the DMA queue
  const int lt = WU ? lane : tid, nlt = WU ? 64 : 256;  // threads computing the leaves
  const float4 g4 = *reinterpret_cast<const float4*>(geo_g + 4 * (size_t)(b * N + i));
  const float th = x[2 * (b * N + i)], ph = x[2 * (b * N + i) + 1];
  const float4 ga = *reinterpret_cast<const float4*>(geo_g + 4 * (size_t)(b * N + (lt < T ? lt >> 1 : 0)));
  float nrm[2];  // norm of this thread's harmonics (M <= 2 nlt)
  nrm[0] = lt < M ? norm[lt] : 0.f;
  nrm[1] = lt + nlt < M ? norm[lt + nlt] : 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int c = 0; c < RING - 1 && c < C; ++c) issue(c, 0);
  {
    const float st = g4.x, ct = g4.y, sp = g4.z, cp = g4.w;
    const float gauge = env_gauge(ct, M);
    const float phh[3] = {-sp, cp, 0.f};
    const float thh[3] = {ct * cp, ct * sp, -st};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int p = lt + r * nlt;
      if (p >= M) break;
      const EnvLeaf e = env_leaf(th, ph, p, M, nrm[r], true, gauge, DET_LEAF_SQ);
      wt[p] = e.e0;
      wt[M + p] = e.dth;
      wt[2 * M + p] = e.dph;
      wt[3 * M + p] = e.lb;
      const float mf = (float)p - 0.5f * (float)(M - 1) - gauge;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        wt[(4 + k) * M + p] = cf{phh[k] * e.dth.re - thh[k] * e.dph.re, phh[k] * e.dth.im - thh[k] * e.dph.im};
        wt[(7 + k) * M + p] = env_flow2(e.e0, e.dth, e.d2th, mf, st, ct, sp, cp, k);
      }
    }
    if (lt < T) {  // alpha_kt from the geometry of the electron tangent t moves
      al[lt] = (lt & 1) ? -(ga.y * ga.w) : -ga.z;
      al[T + lt] = (lt & 1) ? -(ga.y * ga.z) : ga.w;
      al[2 * T + lt] = (lt & 1) ? ga.x : 0.f;
    }
  }
  if constexpr (WU)
    __builtin_amdgcn_wave_barrier();  // a wave's LDS operations complete in order
  else
    __syncthreads();
  // SEG: the four envelope factors every tangent row needs (e0, the three flow weights W_k) at
  // this lane's harmonics, held in registers: the row loop's LDS stores (part) would keep the
  // compiler from hoisting them, and they are 80 % of a tangent row's LDS reads
  constexpr bool RC = SEG > 0 && ENV_REG;
  cf re0[RC ? MG : 1], rw0[RC ? MG : 1], rw1[RC ? MG : 1], rw2[RC ? MG : 1];
  if constexpr (RC) {
#pragma unroll
    for (int u = 0; u < MG; ++u) {
      const int m = mw(u);
      re0[u] = wt[m];
      rw0[u] = wt[4 * M + m];
      rw1[u] = wt[5 * M + m];
      rw2[u] = wt[6 * M + m];
    }
  }
  for (int kd = 0; kd < K; ++kd) {
    cf xd{0.f, 0.f}, xp{0.f, 0.f}, xl{0.f, 0.f}, xs0{0.f, 0.f}, xs1{0.f, 0.f}, xs2{0.f, 0.f};  // F_0 extras
    cf lb2{0.f, 0.f}, gu0{0.f, 0.f}, gu1{0.f, 0.f}, gu2{0.f, 0.f};                            // lane partials
    if (kd > 0)
      for (int c = 0; c < RING - 1 && c < C; ++c) issue(c, kd);
    for (int c = 0; c < C; ++c) {
      if (c + RING - 1 < C) issue(c + RING - 1, kd);  // its slot's last reader was row c - 1
      wait_row(c);
      const bool tang = c >= 1 && c <= T;
      const int t = c - 1;
      const bool own = tang && (t >> 1) == i;
      cf e0a{0.f, 0.f};
      if (c == 0) {
#pragma unroll
        for (int u = 0; u < MG; ++u) {
          const cf fv = fval(c, u);
          const int m = mw(u);
          cfma(e0a, fv, wt[m]);
          cfma(xd, fv, wt[M + m]);
          cfma(xp, fv, wt[2 * M + m]);
          cfma(xl, fv, wt[3 * M + m]);
          cfma(xs0, fv, wt[7 * M + m]);
          cfma(xs1, fv, wt[8 * M + m]);
          cfma(xs2, fv, wt[9 * M + m]);
        }
      } else if (tang) {
        cf w0{0.f, 0.f}, w1{0.f, 0.f}, w2{0.f, 0.f}, dd{0.f, 0.f};
        const cf* wdd = wt + ((t & 1) ? 2 : 1) * M;
#pragma unroll
        for (int u = 0; u < MG; ++u) {
          const cf fv = fval(c, u);
          const int m = mw(u);
          cfma(e0a, fv, RC ? re0[RC ? u : 0] : wt[m]);
          cfma(w0, fv, RC ? rw0[RC ? u : 0] : wt[4 * M + m]);
          cfma(w1, fv, RC ? rw1[RC ? u : 0] : wt[5 * M + m]);
          cfma(w2, fv, RC ? rw2[RC ? u : 0] : wt[6 * M + m]);
          if (own) cfma(dd, fv, wdd[m]);
        }
        gu0 += al[t] * w0;
        gu1 += al[T + t] * w1;
        gu2 += al[2 * T + t] * w2;
        lb2 += dd;
        if (own) e0a += (t & 1) ? xp : xd;
      } else {
#pragma unroll
        for (int u = 0; u < MG; ++u) cfma(e0a, fval(c, u), RC ? re0[RC ? u : 0] : wt[mw(u)]);
        if (c == T + 1) e0a += xl + 2.f * lb2;
        if (c >= T + 2) {
          const int k = c - T - 2;
          e0a += (k == 0 ? xs0 : (k == 1 ? xs1 : xs2)) + 2.f * (k == 0 ? gu0 : (k == 1 ? gu1 : gu2));
        }
      }
      const cf v = gsumc(e0a);
      if constexpr (WU) {
        if (g == 0) {
          float* o = PhiC + 2 * (((size_t)(b * K + kd) * C + c) * N * N + (size_t)i * N + j);
          o[0] = v.re;
          o[1] = v.im;
        }
      } else {
        if (g == 0) part[((size_t)wv * C + c) * N + j] = v;
      }
    }
    if constexpr (WU) continue;
    __syncthreads();
    float* out = PhiC + 2 * ((size_t)(b * K + kd) * C * N * N + (size_t)i * N);
    for (int e = tid; e < C * N; e += 256) {
      const int c = e / N, jj = e - (e / N) * N;
      const cf v = (part[e] + part[C * N + e]) + (part[2 * C * N + e] + part[3 * C * N + e]);
      out[2 * ((size_t)c * N * N + jj)] = v.re;
      out[2 * ((size_t)c * N * N + jj) + 1] = v.im;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ envelope contraction, streamed
// Round 5 form of env_contract_kernel for long rows (C5: 2 M N = 2320 floats per channel row):
// the same sums, but the rows come straight into registers by plain loads, D rows ahead (the
// compiler counts them: no LDS ring, no hand-counted vmcnt), so a wave keeps D - 1 rows
// (~17 KB at C5) in flight instead of the ring's three — the ring form read F at ~3 TB/s,
// bounded by the bytes in flight per CU, not by HBM.  One 256-thread workgroup per (walker,
// electron), four waves over contiguous harmonic blocks (MW = ceil(M / 4) each), lane (j, g)
// on harmonics MW w + g + G u (u < MG); the channel loop is unrolled (C compile-time) so the
// register ring is indexed by constants.  The leaves, the per-row sums, the lane-group and
// cross-wave reductions and the PhiC layout are env_contract_kernel's (K = 1).
#ifndef DET_WAVE_LBAR  // A/B knob: det_energy_wave_kernel's channel-loop barriers wait for LDS only (1) or
#define DET_WAVE_LBAR 1  // are __syncthreads, whose vmcnt(0) drained the next channel's staging loads (0)
#endif
__device__ __forceinline__ void lds_barrier() {
#if DET_WAVE_LBAR
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#else
  __syncthreads();
#endif
}
template <int N, int MG, int D>
__global__ __launch_bounds__(256, 2) void env_stream_kernel(const float* __restrict__ Fp, int ldF,
                                                            const float* __restrict__ x,
                                                            const float* __restrict__ geo_g,
                                                            const float* __restrict__ norm, float* __restrict__ PhiC,
                                                            int n_up, int M) {
  constexpr int T = 2 * N, C = 2 * N + 5, G = 64 / N, NK = N;
  extern __shared__ float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = blockIdx.x / N, i = blockIdx.x - (blockIdx.x / N) * N;
  cf* wt = reinterpret_cast<cf*>(sm);                  // [E0, DTH, DPH, LB, W0..2, SF0..2][M + 1]
  cf* part = wt + 10 * (M + 1);                        // [4 waves][C][N]
  cf* sink = part + 4 * C * N;                         // [4 waves][64]: lanes g > 0 store here
  float* al = reinterpret_cast<float*>(sink + 256);    // [3][T]
  const int j = lane % N, g = lane / N;
  const int MW = (M + 3) / 4, gg = MW * wv + g, mend = min(MW * (wv + 1), M), M1 = M + 1;
  const bool act = g < G;
  const int blk = (i >= n_up && n_up > 0) ? 1 : 0, MNK = M * NK;
  // uniform row base (scalar address) + 32-bit lane offsets: one voffset per harmonic
  const float* rowbase = Fp + ((size_t)(b * N + i) * C) * ldF + (size_t)blk * 2 * MNK;
  // lane harmonic u: m = gg + G u (clamped for the address; masked in the sums)
  // masked lanes read harmonic M - 1 and multiply it by the zero factor at index M
  int mo[MG], mw_[MG];
#pragma unroll
  for (int u = 0; u < MG; ++u) {
    const bool ok = act && gg + G * u < mend;
    mo[u] = min(gg + G * u, M - 1) * NK + j;
    mw_[u] = ok ? gg + G * u : M;
  }
  // buffer loads: scalar resource + row soffset, 32-bit lane voffsets (no 64-bit lane addresses)
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rowbase), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int u = 0; u < MG; ++u) mo[u] *= 4;
  float fr[D][MG][2];
  auto load_row = [&](int c, float (&f)[MG][2]) __attribute__((always_inline)) {
    const int so = c * ldF * 4;
#pragma unroll
    for (int u = 0; u < MG; ++u) {
      f[u][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, mo[u], so, 0));
      f[u][1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, mo[u] + MNK * 4, so, 0));
    }
  };
  // the value row and the first D - 1 tangent rows are requested before the leaves are computed
  float f0[MG][2];
  load_row(0, f0);
#pragma unroll
  for (int d = 0; d < D - 1; ++d) load_row(1 + d, fr[d]);
  {
    const float4 g4 = *reinterpret_cast<const float4*>(geo_g + 4 * (size_t)(b * N + i));
    const float th = x[2 * (b * N + i)], ph = x[2 * (b * N + i) + 1];
    const float st = g4.x, ct = g4.y, sp = g4.z, cp = g4.w;
    const float gauge = env_gauge(ct, M);
    const float phh[3] = {-sp, cp, 0.f};
    const float thh[3] = {ct * cp, ct * sp, -st};
    if (tid < 10) wt[tid * M1 + M] = cf{0.f, 0.f};
    for (int p = tid; p < M; p += 256) {
      const EnvLeaf e = env_leaf(th, ph, p, M, norm[p], true, gauge, DET_LEAF_SQ);
      wt[p] = e.e0;
      wt[M1 + p] = e.dth;
      wt[2 * M1 + p] = e.dph;
      wt[3 * M1 + p] = e.lb;
      const float mf = (float)p - 0.5f * (float)(M - 1) - gauge;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        wt[(4 + k) * M1 + p] = cf{phh[k] * e.dth.re - thh[k] * e.dph.re, phh[k] * e.dth.im - thh[k] * e.dph.im};
        wt[(7 + k) * M1 + p] = env_flow2(e.e0, e.dth, e.d2th, mf, st, ct, sp, cp, k);
      }
    }
    if (tid < T) {  // alpha_kt from the geometry of the electron tangent t moves
      const float4 ga = *reinterpret_cast<const float4*>(geo_g + 4 * (size_t)(b * N + (tid >> 1)));
      al[tid] = (tid & 1) ? -(ga.y * ga.w) : -ga.z;
      al[T + tid] = (tid & 1) ? -(ga.y * ga.z) : ga.w;
      al[2 * T + tid] = (tid & 1) ? ga.x : 0.f;
    }
  }
  lds_barrier();  // the leaves are LDS; the D rows requested above stay in flight across it
  // the envelope factors are re-read from LDS per row (the index is laundered so that they are
  // not hoisted into registers: the VGPRs go to rows in flight instead)
  // per-row result store without a branch (a branch per row splits the unrolled bodies into
  // blocks and lets the compiler sink the row sums past them, keeping every row live)
  cf* const dst = g == 0 ? part + (size_t)wv * C * N + j : sink + tid;
  const int dstride = g == 0 ? N : 0;
  auto gsum = [&](float v) __attribute__((always_inline)) {
    float r = v;
#pragma unroll
    for (int q = 1; q < G; ++q) r += __shfl(v, j + N * q, 64);
    return r;
  };
  cf xd{0.f, 0.f}, xp{0.f, 0.f}, xl{0.f, 0.f}, xs0{0.f, 0.f}, xs1{0.f, 0.f}, xs2{0.f, 0.f};  // F_0 extras
  cf lb2{0.f, 0.f}, gu0{0.f, 0.f}, gu1{0.f, 0.f}, gu2{0.f, 0.f};                            // lane partials
  {  // value row (c = 0)
    cf e0a{0.f, 0.f};
#pragma unroll
    for (int u = 0; u < MG; ++u) {
      const cf fv{f0[u][0], f0[u][1]};
      const int m = mw_[u];
      cfma(e0a, fv, wt[m]);
      cfma(xd, fv, wt[M1 + m]);
      cfma(xp, fv, wt[2 * M1 + m]);
      cfma(xl, fv, wt[3 * M1 + m]);
      cfma(xs0, fv, wt[7 * M1 + m]);
      cfma(xs1, fv, wt[8 * M1 + m]);
      cfma(xs2, fv, wt[9 * M1 + m]);
    }
    const cf v{gsum(e0a.re), gsum(e0a.im)};
    dst[0] = v;
  }
  // tangent rows c = 1..T: branch-free bodies (own-electron terms weighted by 0/1), loads for
  // row min(c + D - 1, C - 1) issued unconditionally, so the loop is straight-line and the
  // compiler's vmcnt keeps D - 1 rows in flight
  static_assert(T % D == 0, "tangent rows come in whole groups of D");
#pragma nounroll
  for (int c0 = 1; c0 <= T; c0 += D) {
#pragma unroll
    for (int dd_ = 0; dd_ < D; ++dd_) {
      const int c = c0 + dd_, t = c - 1;
      __builtin_amdgcn_sched_barrier(0);  // keep the ring order: one row's loads per body
      load_row(min(c + D - 1, C - 1), fr[(dd_ + D - 1) % D]);
      const float (&f)[MG][2] = fr[dd_];
      const float ownf = (t >> 1) == i ? 1.f : 0.f;
      const int dsel = (t & 1) ? 2 * M1 : M1;
      cf e0a{0.f, 0.f}, w0{0.f, 0.f}, w1{0.f, 0.f}, w2{0.f, 0.f}, dd{0.f, 0.f};
#pragma unroll
      for (int u = 0; u < MG; ++u) {
        const cf fv{f[u][0], f[u][1]};
        int m = mw_[u];
        asm volatile("" : "+v"(m));
        cfma(e0a, fv, wt[m]);
        cfma(w0, fv, wt[4 * M1 + m]);
        cfma(w1, fv, wt[5 * M1 + m]);
        cfma(w2, fv, wt[6 * M1 + m]);
        cfma(dd, fv, wt[dsel + m]);
      }
      lb2 += ownf * dd;
      e0a += ownf * ((t & 1) ? xp : xd);
      gu0 += al[t] * w0;
      gu1 += al[T + t] * w1;
      gu2 += al[2 * T + t] * w2;
      const cf v{gsum(e0a.re), gsum(e0a.im)};
      dst[c * dstride] = v;
    }
  }
  // rows T + 1..T + 4 (L, S_0..2) are in ring slots 0..3
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = T + 1 + r;
    const float (&f)[MG][2] = fr[r];
    cf e0a{0.f, 0.f};
#pragma unroll
    for (int u = 0; u < MG; ++u) cfma(e0a, cf{f[u][0], f[u][1]}, wt[mw_[u]]);
    if (r == 0) e0a += xl + 2.f * lb2;
    if (r == 1) e0a += xs0 + 2.f * gu0;
    if (r == 2) e0a += xs1 + 2.f * gu1;
    if (r == 3) e0a += xs2 + 2.f * gu2;
    const cf v{gsum(e0a.re), gsum(e0a.im)};
    dst[c * dstride] = v;
  }
  lds_barrier();
  float* out = PhiC + 2 * ((size_t)b * C * N * N + (size_t)i * N);
  for (int e = tid; e < C * N; e += 256) {
    const int c = e / N, jj = e - (e / N) * N;
    const cf v = (part[e] + part[C * N + e]) + (part[2 * C * N + e] + part[3 * C * N + e]);
    out[2 * ((size_t)c * N * N + jj)] = v.re;
    out[2 * ((size_t)c * N * N + jj) + 1] = v.im;
  }
}

// dynamic LDS of env_contract_kernel<MG, WU>
size_t env_contract_smem(int N, int M, int MG, bool WU, int K = 1, bool seg = false) {
  const int T = 2 * N, C = 2 * N + 5;
  if (WU) return (size_t)4 * (20 * M + ((3 * T + 3) & ~3) + env_ring(MG) * 2 * MG * 64) * sizeof(float);
  const int ringf = seg ? kEnvSegRing * 2 * ((M + 3) / 4) * N * K : env_ring(MG) * 2 * MG * 64;  // per wave
  return (size_t)(20 * M + 8 * C * N + ((3 * T + 3) & ~3) + 4 * ringf) * sizeof(float);
}
// segment DMA (env_contract_kernel SEG > 0) usable for this shape: K == 1, 16-B aligned
// segments, every piece of every wave keeping its lane 0, the lane harmonics within MG;
// returns the pieces per segment (1, 2), or 0
int env_contract_seg(int N, int M, int K, int MG, int ldF) {
  if (K != 1) return 0;
  const int G = 64 / N, MW = (M + 3) / 4, NK = N * K, MNK = M * NK;
  if ((MW + G - 1) / G > MG || (MW * NK) % 4 || MNK % 4 || ldF % 4) return 0;
  const int seg = (MW * NK * 4 + 1023) / 1024;
  if (seg > 2) return 0;
  for (int wv = 0; wv < 4; ++wv) {
    const int bytes = (std::min(MW * (wv + 1), M) - MW * wv) * NK * 4;
    if (bytes <= (seg - 1) * 1024) return 0;  // a piece without lanes would not be issued
  }
  if (env_contract_smem(N, M, MG, false, K, true) > 163840) return 0;
  return seg;
}

// ------------------------------------------------------------------ energy kernel
struct DetSmem {
  int geo, alpha, E0, DTH, DPH, LB, D2TH, Aug, Binv, Phi, Mt, Mu, Gu, fac, ellt, ell0, ellL, ellS, red, misc;
  int Fv, Fc, LB2, asmb, dgeo, total;  // staged orbital rows (value, current channel); own-tangent LB
                                       // terms; double-precision assembly partials; double geometry
};
// Orbital rows are staged through LDS when the N rows of one channel (the electron's own
// spin block: 2 M N K floats each) fit this many floats.
constexpr int kStageFloats = 5120;
__host__ __device__ inline bool det_staged(int N, int M, int K) { return 2 * M * N * K * N <= kStageFloats; }
// pc (the precontracted path): the envelope leaves (E0 .. D2TH) and the flow first-order
// sums (Gu) are not needed and get no space, so more workgroups fit a CU (C5: 89 -> 33 KiB)
__host__ __device__ inline DetSmem det_layout(int N, int M, int K, int nwaves, bool pc = false) {
  // offsets in floats; complex arrays take 2 floats per element
  DetSmem L;
  const int T = 2 * N, NN = N * N;
  int o = 0;
  const int rows = det_staged(N, M, K) ? 2 * M * N * K * N : 0;
  L.Fv = o;
  o += rows;
  L.Fc = o;
  o += rows;
  L.LB2 = o;
  o += 2 * NN;
  L.asmb = o;  // even offset: doubles
  o += 2 * (4 * T + 10 * N + 2 * K);
  L.dgeo = o;  // even offset: (sin th, cos th, sin ph, cos ph) in double, from x
  o += 2 * 4 * N;
  L.geo = o;
  o += 4 * N;
  L.alpha = o;
  o += 3 * T;
  o = (o + 1) & ~1;
  const int nm = pc ? 0 : 2 * N * M;
  L.E0 = o;
  o += nm;
  L.DTH = o;
  o += nm;
  L.DPH = o;
  o += nm;
  L.LB = o;
  o += nm;
  L.D2TH = o;
  o += nm;
  L.Aug = o;
  o += 2 * 2 * NN;
  L.Binv = o;
  o += 2 * NN;
  L.Phi = o;
  o += 2 * NN;
  L.Mt = o;
  o += 2 * NN;
  L.Mu = o;
  o += 3 * 2 * NN;
  L.Gu = o;
  o += pc ? 0 : 3 * 2 * NN;
  L.fac = o;
  o += 2 * N;
  L.ellt = o;
  o += 2 * K * T;
  L.ell0 = o;
  o += 2 * K;
  L.ellL = o;
  o += 2 * K;
  L.ellS = o;
  o += 2 * 3 * K;
  L.red = o;
  o += 4 * nwaves + 4;
  L.misc = o;
  o += 8;
  L.total = o;
  return L;
}

// block-wide sum of 4 floats, result returned to every thread (two __syncthreads)
__device__ inline void block_sum4(float v[4], float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = wave_sum(v[q]);
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[4 * w + q] = v[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[4 * i + q];
    v[q] = s;
  }
  __syncthreads();
}

// ---- combine determinants, Jastrow, potential, assembly (double precision).
// Per-tangent terms on threads t < T, per-electron Jastrow / potential sums on threads
// T + i, partial results in LDS; thread 0 finishes with scalar sums only (no private
// arrays, so nothing goes to scratch memory).
// Shared by det_energy_kernel and det_energy_wave_kernel: ell0 [K], ellt [K T], ellL [K],
// ellS [3 K] (written by thread 0 / the lanes before the call), geometry geo (f32) / dgeo
// (f64) / al in LDS, asmb = 2 (4 T + 10 N + 2 K) floats of LDS scratch; every thread of the
// workgroup calls it (one __syncthreads inside), threads tid < T + N do the per-tangent and
// per-electron parts.
__device__ __forceinline__ void energy_assembly(int tid, int N, int n_up, int M, int K, float Q, float radius, float lambda,
                                int interaction, int b, const float* __restrict__ x, const float* __restrict__ jas,
                                const float* geo, const double* dgeo, const float* al, const cf* ell0,
                                const cf* ellt, const cf* ellL, const cf* ellS, double* asmb,
                                float* __restrict__ e_l, float* __restrict__ obs) {
  const int T = 2 * N;
  __syncthreads();  // ell* written by thread 0 in the channel loops
  double* tgr = asmb;
  double* tgi = tgr + T;
  double* lbr = tgi + T;
  double* lbi = lbr + T;
  double* Jn = lbi + T;
  double* Jlbn = Jn + N;
  double* pen = Jlbn + N;
  // per-electron terms of thread 0's sums, formed by threads T + i (their divisions off the
  // serial thread; thread 0 adds them in the same order, so the sums are unchanged)
  double* gph = pen + N;     // kappa_i phi_i
  double* sgi = gph + N;     // [3][N] the gauge terms of S_im
  double* cotn = sgi + 3 * N;
  double* mvn = cotn + N;    // [2][N] Q cos ph / sin th, Q sin ph / sin th
  double* pkr = mvn + 2 * N;  // [2][K] the determinant weights p_k for thread 0 (formed once,
                              // by threads T + N + k: thread 0 used them 4 K times)
  // determinant weights p_k = w_k / Z, w_k = exp(ell0_k - max) (every thread; K is small)
  double lmax = -1e300;
  for (int k = 0; k < K; ++k) lmax = fmax(lmax, (double)ell0[k].re);
  double zr = 0.0, zi = 0.0;
  for (int k = 0; k < K; ++k) {
    const double mag = exp((double)ell0[k].re - lmax);
    zr += mag * cos((double)ell0[k].im);
    zi += mag * sin((double)ell0[k].im);
  }
  const double zz = zr * zr + zi * zi;
  auto pk = [&](int k, double& pr, double& pi_) {
    const double mag = exp((double)ell0[k].re - lmax);
    const double wr = mag * cos((double)ell0[k].im), wi = mag * sin((double)ell0[k].im);
    pr = (wr * zr + wi * zi) / zz;
    pi_ = (wi * zr - wr * zi) / zz;
  };
  const double ap = jas[0], aa = jas[1];
  if (tid < T) {
    const int t = tid, i = t >> 1;
    double gr = 0.0, gi = 0.0, sr = 0.0, si = 0.0;
    for (int k = 0; k < K; ++k) {
      double pr, pi_;
      pk(k, pr, pi_);
      const double lr = ellt[k * T + t].re, li = ellt[k * T + t].im;
      gr += pr * lr - pi_ * li;
      gi += pr * li + pi_ * lr;
      const double l2r = lr * lr - li * li, l2i = 2.0 * lr * li;
      sr += pr * l2r - pi_ * l2i;
      si += pr * l2i + pi_ * l2r;
    }
    lbr[t] = sr - (gr * gr - gi * gi);
    lbi[t] = si - 2.0 * gr * gi;
    // Jastrow gradient along the (scaled) tangent t of electron i
    const double sti = dgeo[4 * i], cti = dgeo[4 * i + 1], spi = dgeo[4 * i + 2], cpi = dgeo[4 * i + 3];
    const double ri[3] = {sti * cpi, sti * spi, cti};
    const double et[3] = {(t & 1) ? -spi : cti * cpi, (t & 1) ? cpi : cti * spi, (t & 1) ? 0.0 : -sti};
    double jg = 0.0;
    for (int j = 0; j < N; ++j) {
      if (j == i) continue;
      const double stj = dgeo[4 * j], ctj = dgeo[4 * j + 1], spj = dgeo[4 * j + 2], cpj = dgeo[4 * j + 3];
      const double rj[3] = {stj * cpj, stj * spj, ctj};
      const double u = ri[0] * rj[0] + ri[1] * rj[1] + ri[2] * rj[2];
      const double r = sqrt(fmax(2.0 - 2.0 * u, 0.0));
      const bool same = (i < n_up) == (j < n_up);
      double f1, f2;
      (void)jastrow_pair(r, same ? ap : aa, same ? 0.25 : 0.5, &f1, &f2);
      jg += (-f1 / r) * (rj[0] * et[0] + rj[1] * et[1] + rj[2] * et[2]);
    }
    // gauge term A = i sum_i kappa_i phi_i (env_leaf) on the phi tangent
    if (t & 1) gi += (double)env_gauge(geo[4 * i + 1], M) / sti;  // the leaves' kappa
    tgr[t] = gr + jg;
    tgi[t] = gi;
  } else if (tid < T + N) {
    const int i = tid - T;
    const double sti = dgeo[4 * i], cti = dgeo[4 * i + 1], spi = dgeo[4 * i + 2], cpi = dgeo[4 * i + 3];
    const double ri[3] = {sti * cpi, sti * spi, cti};
    double J = 0.0, Jlb = 0.0, pe = 0.0;
    for (int j = i + 1; j < N; ++j) {
      const double stj = dgeo[4 * j], ctj = dgeo[4 * j + 1], spj = dgeo[4 * j + 2], cpj = dgeo[4 * j + 3];
      const double rj[3] = {stj * cpj, stj * spj, ctj};
      const double u = ri[0] * rj[0] + ri[1] * rj[1] + ri[2] * rj[2];
      const double r = sqrt(fmax(2.0 - 2.0 * u, 0.0));
      const bool same = (i < n_up) == (j < n_up);
      double f1, f2;
      J += jastrow_pair(r, same ? ap : aa, same ? 0.25 : 0.5, &f1, &f2);
      Jlb += 2.0 * ((4.0 - r * r) * r * f2 + (4.0 - 3.0 * r * r) * f1) / (4.0 * r);
      if (interaction == DH_INTERACTION_COULOMB)
        pe += 1.0 / sqrt(2.0 - 2.0 * u);
      else
        pe += 1.0 + ((double)Q + 1.0) / (double)Q * u;
    }
    Jn[i] = J;
    Jlbn[i] = Jlb;
    pen[i] = pe;
    {
      const double st = sti, ct = cti, sp = spi, cp = cpi;
      const double kap = (double)env_gauge(geo[4 * i + 1], M);  // the leaves' kappa
      gph[i] = kap * (double)x[2 * (b * N + i) + 1];
      const double cot = ct / st;
      const double tdot[3] = {-sp, cp, 0.0};
      const double thp[3] = {cp * cot, sp * cot, -1.0};
      const double dthp_dth[3] = {-cp / (st * st), -sp / (st * st), 0.0};
      const double dthp_dph[3] = {-sp * cot, cp * cot, 0.0};
#pragma unroll
      for (int kk = 0; kk < 3; ++kk) sgi[kk * N + i] = kap * (-(dthp_dth[kk] * tdot[kk] - dthp_dph[kk] * thp[kk]));
      cotn[i] = cot;
      mvn[i] = Q * cp / st;
      mvn[N + i] = Q * sp / st;
    }
  } else {  // (blockDim > 3 N for every launch: 64 or 256 threads, N <= 20)
    for (int k = tid - T - N; k < K; k += (int)blockDim.x - T - N) pk(k, pkr[k], pkr[K + k]);
  }
  __syncthreads();
  if (tid == 0) {
    const double val_re = 0.5 * log(zz) + lmax, val_im = atan2(zi, zr);
    double LB_re = 0.0, LB_im = 0.0;
    for (int k = 0; k < K; ++k) {
      const double pr = pkr[k], pi_ = pkr[K + k];
      LB_re += pr * ellL[k].re - pi_ * ellL[k].im;
      LB_im += pr * ellL[k].im + pi_ * ellL[k].re;
    }
    for (int t = 0; t < T; ++t) {
      LB_re += lbr[t];
      LB_im += lbi[t];
    }
    double S_re[3], S_im[3];
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      double a_r = 0.0, a_i = 0.0, m1r = 0.0, m1i = 0.0, m2r = 0.0, m2i = 0.0;
      for (int k = 0; k < K; ++k) {
        const double pr = pkr[k], pi_ = pkr[K + k];
        a_r += pr * ellS[3 * k + kk].re - pi_ * ellS[3 * k + kk].im;
        a_i += pr * ellS[3 * k + kk].im + pi_ * ellS[3 * k + kk].re;
        double gur = 0.0, gui = 0.0;
        for (int t = 0; t < T; ++t) {
          gur += (double)al[kk * T + t] * ellt[k * T + t].re;
          gui += (double)al[kk * T + t] * ellt[k * T + t].im;
        }
        m1r += pr * gur - pi_ * gui;
        m1i += pr * gui + pi_ * gur;
        const double g2r = gur * gur - gui * gui, g2i = 2.0 * gur * gui;
        m2r += pr * g2r - pi_ * g2i;
        m2i += pr * g2i + pi_ * g2r;
      }
      S_re[kk] = a_r + m2r - (m1r * m1r - m1i * m1i);
      S_im[kk] = a_i + m2i - 2.0 * m1r * m1i;
    }
    double J = 0.0, Jlb = 0.0, pe = 0.0;
    for (int i = 0; i < N; ++i) {
      J += Jn[i];
      Jlb += Jlbn[i];
      pe += pen[i];
    }
    if (interaction == DH_INTERACTION_COULOMB) pe /= (double)radius;
    // gauge terms: phase and the flow channels' phi acceleration (see env_flow2)
    double gauge_phase = 0.0;
    for (int i = 0; i < N; ++i) {
      gauge_phase += gph[i];
#pragma unroll
      for (int kk = 0; kk < 3; ++kk) S_im[kk] += sgi[kk * N + i];
    }
    pe *= (double)lambda;
    LB_re += Jlb;
    double sq_re = 0.0, sq_im = 0.0, mag_re = 0.0, mag_im = 0.0;
    for (int t = 0; t < T; ++t) {
      sq_re += tgr[t] * tgr[t] - tgi[t] * tgi[t];
      sq_im += 2.0 * tgr[t] * tgi[t];
    }
    double Mv[3] = {0.0, 0.0, 0.0};
    for (int i = 0; i < N; ++i) {
      const double cot = cotn[i];
      mag_re += (Q * cot) * (Q * cot);
      mag_re += -2.0 * Q * cot * tgi[2 * i + 1];  // 2 i Q cot * t_phi_scaled
      mag_im += 2.0 * Q * cot * tgr[2 * i + 1];
      Mv[0] += mvn[i];
      Mv[1] += mvn[N + i];
    }
    const double r2 = (double)radius * radius;
    const double ke_re = (-LB_re - sq_re + mag_re) / (2.0 * r2);
    const double ke_im = (-LB_im - sq_im + mag_im) / (2.0 * r2);
    double G_re[3], G_im[3];
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      double gr = 0.0, gi = 0.0;
      for (int t = 0; t < T; ++t) {
        gr += (double)al[kk * T + t] * tgr[t];
        gi += (double)al[kk * T + t] * tgi[t];
      }
      G_re[kk] = gr;
      G_im[kk] = gi;
    }
    double L2 = 0.0;
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      const double ar = G_re[kk], ai = G_im[kk] + Mv[kk];  // (G + i M)^2, real part
      L2 -= S_re[kk] + (ar * ar - ai * ai);
    }
    const double lz = G_im[2];
    const double lz2 = -(S_re[2] + G_re[2] * G_re[2] - G_im[2] * G_im[2]);
    e_l[2 * b] = (float)(ke_re + pe);
    e_l[2 * b + 1] = (float)ke_im;
    float* ob = obs + 8 * (size_t)b;
    ob[0] = (float)ke_re;
    ob[1] = (float)ke_im;
    ob[2] = (float)pe;
    ob[3] = (float)lz;
    ob[4] = (float)lz2;
    ob[5] = (float)L2;
    ob[6] = (float)(val_re + J);
    ob[7] = (float)remainder(val_im + gauge_phase, 2.0 * M_PI);
  }
}

// PF > 0: orbital rows staged through LDS, PF floats per thread in flight.
// PC: the channel matrices come precontracted from env_contract_kernel (PhiC), F unused.
// NT: threads per walker, 256 (four waves; the default) or 64 (one wave, DH_DET_WAVE=1:
// every matrix of N <= 8 has at most 64 entries and a one-wave barrier is nearly free, but
// the per-walker staging and contraction then run on a quarter of the lanes — slower).
template <int PF, bool PC = false, int NT = 256>
__global__ __launch_bounds__(NT, NT == 64 ? 8 : 4) void det_energy_kernel(const float* __restrict__ Fp, int ldF, const float* __restrict__ x,
                                  const float* __restrict__ geo_g, const float* __restrict__ jas,
                                  const float* __restrict__ norm, float* __restrict__ e_l, float* __restrict__ obs,
                                  int N, int n_up, int M, int K, float Q, float radius, float lambda,
                                  int interaction, const float* __restrict__ PhiC) {
  extern __shared__ float sm[];
  const int T = 2 * N, C = 2 * N + 5, NN = N * N;
  const int tid = threadIdx.x, nt = blockDim.x;
  const DetSmem L = det_layout(N, M, K, nt >> 6, PC);
  const int b = blockIdx.x;
  float* geo = sm + L.geo;  // st ct sp cp
  float* al = sm + L.alpha;
  cf *E0 = (cf*)(sm + L.E0), *DTH = (cf*)(sm + L.DTH), *DPH = (cf*)(sm + L.DPH), *LBe = (cf*)(sm + L.LB),
     *D2 = (cf*)(sm + L.D2TH);
  cf *Aug = (cf*)(sm + L.Aug), *Binv = (cf*)(sm + L.Binv), *Phi = (cf*)(sm + L.Phi), *Mt = (cf*)(sm + L.Mt);
  cf *Mu = (cf*)(sm + L.Mu), *Gu = (cf*)(sm + L.Gu), *fac = (cf*)(sm + L.fac);
  cf *ellt = (cf*)(sm + L.ellt), *ell0 = (cf*)(sm + L.ell0), *ellL = (cf*)(sm + L.ellL), *ellS = (cf*)(sm + L.ellS);
  float* red = sm + L.red;
  int* piv = reinterpret_cast<int*>(sm + L.misc);
  cf* logdet = reinterpret_cast<cf*>(sm + L.misc + 2);
  const FView F{Fp, ldF, M, N, K};
  auto phic = [&](int kd, int c, int idx) -> cf {
    const float* q = PhiC + 2 * (((size_t)(b * K + kd) * C + c) * NN + idx);
    return cf{q[0], q[1]};
  };
  const size_t rowbase = (size_t)b * N * C;  // row of (b, i, c) = rowbase + i*C + c
  // ---- staging of orbital rows (STAGED): the N rows of one channel, each the electron's
  // own spin block (2 M N K floats), through registers into LDS.  The value rows stay in
  // Fv; channel c's rows go to Fc while channel c+1's are already in flight.
  const int MNK = M * N * K, RW = 2 * MNK, NRW = N * RW;
  float* Fv = sm + L.Fv;
  float* Fc = sm + L.Fc;
  cf* LB2 = (cf*)(sm + L.LB2);
  constexpr bool STAGED = PF > 0;
  constexpr int PFMAX = STAGED ? PF : 1;
  float pf[PFMAX];
  auto stage_load = [&](int c) {
#pragma unroll
    for (int u = 0; u < PFMAX; ++u) {
      const int q = tid + u * nt;
      if (q < NRW) {
        const int i = q / RW, w = q - (q / RW) * RW;
        const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
        pf[u] = Fp[(rowbase + (size_t)i * C + c) * ldF + (size_t)blk * RW + w];
      }
    }
  };
  auto stage_store = [&](float* dst) {
#pragma unroll
    for (int u = 0; u < PFMAX; ++u) {
      const int q = tid + u * nt;
      if (q < NRW) dst[q] = pf[u];
    }
  };
  // element (part re/im of) orbital m, column j, det kd of electron i from a staged buffer
  auto fs = [&](const float* buf, int i, int p, int j, int kd) -> cf {
    const float* r = buf + i * RW + (p * N + j) * K + kd;
    return cf{r[0], r[MNK]};
  };
  if constexpr (STAGED) {
    stage_load(0);
    stage_store(Fv);
  }

  // the double-precision parts (pair distances of the Jastrow and the potential, the
  // assembly's geometry) take sin / cos of the walker coordinates in double: from f32
  // sin / cos a close pair's chord sqrt(2 - 2 r_i . r_j) loses ~eps_f32 / r^2
  double* dgeo = reinterpret_cast<double*>(sm + L.dgeo);
  for (int i = tid; i < N; i += nt) {
    const float4 g = *reinterpret_cast<const float4*>(geo_g + 4 * (size_t)(b * N + i));
    geo[4 * i] = g.x;
    geo[4 * i + 1] = g.y;
    geo[4 * i + 2] = g.z;
    geo[4 * i + 3] = g.w;
    double st, ct, sp, cp;
    sincos((double)x[2 * (b * N + i)], &st, &ct);
    sincos((double)x[2 * (b * N + i) + 1], &sp, &cp);
    dgeo[4 * i] = st;
    dgeo[4 * i + 1] = ct;
    dgeo[4 * i + 2] = sp;
    dgeo[4 * i + 3] = cp;
  }
  __syncthreads();
  for (int t = tid; t < T; t += nt) {
    const int i = t >> 1;
    const float st = geo[4 * i], ct = geo[4 * i + 1], sp = geo[4 * i + 2], cp = geo[4 * i + 3];
    for (int k = 0; k < 3; ++k) {
      float a;
      if ((t & 1) == 0)
        a = (k == 0) ? -sp : (k == 1 ? cp : 0.f);
      else
        a = (k == 0) ? -(ct * cp) : (k == 1 ? -(ct * sp) : st);
      al[k * T + t] = a;
    }
  }
  for (int idx = tid; idx < (PC ? 0 : N * M); idx += nt) {
    const int i = idx / M, p = idx % M;
    const float gauge = env_gauge(geo[4 * i + 1], M);
    const EnvLeaf e = env_leaf(x[2 * (b * N + i)], x[2 * (b * N + i) + 1], p, M, norm[p], true, gauge, DET_LEAF_SQ);
    E0[idx] = e.e0;
    DTH[idx] = e.dth;
    DPH[idx] = e.dph;
    LBe[idx] = e.lb;
    D2[idx] = e.d2th;
  }
  __syncthreads();

  for (int kd = 0; kd < K; ++kd) {
    if constexpr (STAGED) {
      stage_load(1);  // first tangent channel, in flight during the LU below
      for (int idx = tid; idx < NN; idx += nt) LB2[idx] = cf{0.f, 0.f};
    }
    // ---- Phi0 and its inverse (augmented Gauss-Jordan)
    for (int idx = tid; idx < NN; idx += nt) {
      const int i = idx / N, j = idx % N;
      const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
      cf acc{0.f, 0.f};
      if constexpr (PC)
        acc = phic(kd, 0, idx);
      else
        for (int p = 0; p < M; ++p)
          cfma(acc, STAGED ? fs(Fv, i, p, j, kd) : F.at(rowbase + (size_t)i * C, blk, p, j, kd), E0[i * M + p]);
      Aug[i * 2 * N + j] = acc;
      Aug[i * 2 * N + N + j] = (i == j) ? cf{1.f, 0.f} : cf{0.f, 0.f};
    }
    for (int idx = tid; idx < 3 * NN; idx += nt) {
      Mu[idx] = cf{0.f, 0.f};
      if (!PC) Gu[idx] = cf{0.f, 0.f};
    }
    __syncthreads();
    eliminate(Aug, 2 * N, N, 2 * N, true, fac, piv, logdet);
    for (int idx = tid; idx < NN; idx += nt) Binv[idx] = Aug[(idx / N) * 2 * N + N + idx % N];
    if (tid == 0) ell0[kd] = *logdet;
    __syncthreads();

    float sum_trm2_re = 0.f, sum_trm2_im = 0.f;  // uniform across threads after block_sum4
    // ---- tangent channels
    for (int t = 0; t < T; ++t) {
      const int it = t >> 1;
      const cf* dE = (t & 1) ? DPH : DTH;
      const float a0 = al[t], a1 = al[T + t], a2 = al[2 * T + t];
      if constexpr (STAGED) {  // Fc <- channel 1+t (readers of the previous channel are done)
        stage_store(Fc);
        stage_load(t + 1 < T ? t + 2 : T + 1);
        __syncthreads();
      }
      for (int idx = tid; idx < (PC ? NN : 0); idx += nt) Phi[idx] = phic(kd, 1 + t, idx);
      for (int idx = tid; idx < (PC ? 0 : NN); idx += nt) {
        const int i = idx / N, j = idx % N;
        const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
        const size_t rt = rowbase + (size_t)i * C + 1 + t;
        const float st = geo[4 * i], ct = geo[4 * i + 1], sp = geo[4 * i + 2], cp = geo[4 * i + 3];
        const float phh[3] = {-sp, cp, 0.f};
        const float thh[3] = {ct * cp, ct * sp, -st};
        cf acc{0.f, 0.f}, g0{0.f, 0.f}, g1{0.f, 0.f}, g2{0.f, 0.f};
        cf lb2{0.f, 0.f};
        for (int p = 0; p < M; ++p) {
          const cf f = STAGED ? fs(Fc, i, p, j, kd) : F.at(rt, blk, p, j, kd);
          const cf dth = DTH[i * M + p], dph = DPH[i * M + p];
          if (STAGED && i == it) cfma(lb2, f, (t & 1) ? dph : dth);
          cfma(acc, f, E0[i * M + p]);
          cfma(g0, f, phh[0] * dth - thh[0] * dph);
          cfma(g1, f, phh[1] * dth - thh[1] * dph);
          cfma(g2, f, phh[2] * dth - thh[2] * dph);
        }
        if (i == it) {
          const size_t r0 = rowbase + (size_t)i * C;
          for (int p = 0; p < M; ++p)
            cfma(acc, STAGED ? fs(Fv, i, p, j, kd) : F.at(r0, blk, p, j, kd), dE[i * M + p]);
          if (STAGED) LB2[idx] += lb2;  // own-tangent term of the Laplace-Beltrami channel
        }
        Phi[idx] = acc;
        Gu[idx] += a0 * g0;
        Gu[NN + idx] += a1 * g1;
        Gu[2 * NN + idx] += a2 * g2;
      }
      __syncthreads();
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      for (int idx = tid; idx < NN; idx += nt) {
        const int i = idx / N, j = idx % N;
        cf acc{0.f, 0.f};
        for (int l = 0; l < N; ++l) cfma(acc, Binv[i * N + l], Phi[l * N + j]);
        Mt[idx] = acc;
        Mu[idx] += a0 * acc;
        Mu[NN + idx] += a1 * acc;
        Mu[2 * NN + idx] += a2 * acc;
        if (i == j) {
          v[0] += acc.re;
          v[1] += acc.im;
        }
      }
      __syncthreads();
      for (int idx = tid; idx < NN; idx += nt) {
        const int i = idx / N, j = idx % N;
        const cf prod = Mt[idx] * Mt[j * N + i];
        v[2] += prod.re;
        v[3] += prod.im;
      }
      block_sum4(v, red);
      if (tid == 0) ellt[kd * T + t] = cf{v[0], v[1]};
      sum_trm2_re += v[2];
      sum_trm2_im += v[3];
    }

    // ---- Laplace-Beltrami channel
    {
      if constexpr (STAGED) {
        stage_store(Fc);
        stage_load(T + 2);
        __syncthreads();
      }
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      for (int idx = tid; idx < NN; idx += nt) {
        const int i = idx / N, j = idx % N;
        const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
        const size_t r0 = rowbase + (size_t)i * C;
        cf acc{0.f, 0.f}, acc2{0.f, 0.f};
        if constexpr (PC) {
          acc = phic(kd, 1 + T, idx);  // includes 2 LB2
        } else if constexpr (STAGED) {
          for (int p = 0; p < M; ++p) {
            cfma(acc, fs(Fc, i, p, j, kd), E0[i * M + p]);
            cfma(acc, fs(Fv, i, p, j, kd), LBe[i * M + p]);
          }
          acc2 = LB2[idx];
        } else {
          for (int p = 0; p < M; ++p) {
            cfma(acc, F.at(r0 + 1 + T, blk, p, j, kd), E0[i * M + p]);
            cfma(acc, F.at(r0, blk, p, j, kd), LBe[i * M + p]);
            cfma(acc2, F.at(r0 + 1 + 2 * i, blk, p, j, kd), DTH[i * M + p]);
            cfma(acc2, F.at(r0 + 2 + 2 * i, blk, p, j, kd), DPH[i * M + p]);
          }
        }
        acc += 2.f * acc2;
        // tr(B Phi) = sum_ij B[j][i] Phi[i][j]
        const cf pr = Binv[j * N + i] * acc;
        v[0] += pr.re;
        v[1] += pr.im;
      }
      block_sum4(v, red);
      if (tid == 0) ellL[kd] = cf{v[0] - sum_trm2_re, v[1] - sum_trm2_im};
    }
    // ---- flow channels
    for (int k = 0; k < 3; ++k) {
      if constexpr (STAGED) {
        stage_store(Fc);
        if (k < 2) stage_load(T + 3 + k);
        __syncthreads();
      }
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      for (int idx = tid; idx < NN; idx += nt) {
        const int i = idx / N, j = idx % N;
        const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
        const size_t r0 = rowbase + (size_t)i * C;
        const float st = geo[4 * i], ct = geo[4 * i + 1], sp = geo[4 * i + 2], cp = geo[4 * i + 3];
        cf acc{0.f, 0.f};
        if constexpr (PC) {
          acc = phic(kd, 2 + T + k, idx);  // includes 2 Gu_k
        } else {
          for (int p = 0; p < M; ++p) {
            const float m = (float)p - 0.5f * (float)(M - 1) - env_gauge(ct, M);
            const cf sf = env_flow2(E0[i * M + p], DTH[i * M + p], D2[i * M + p], m, st, ct, sp, cp, k);
            cfma(acc, STAGED ? fs(Fc, i, p, j, kd) : F.at(r0 + 2 + T + k, blk, p, j, kd), E0[i * M + p]);
            cfma(acc, STAGED ? fs(Fv, i, p, j, kd) : F.at(r0, blk, p, j, kd), sf);
          }
          acc += 2.f * Gu[k * NN + idx];
        }
        const cf pr = Binv[j * N + i] * acc;
        v[0] += pr.re;
        v[1] += pr.im;
        const cf m2 = Mu[k * NN + idx] * Mu[k * NN + j * N + i];
        v[2] += m2.re;
        v[3] += m2.im;
      }
      block_sum4(v, red);
      if (tid == 0) ellS[3 * kd + k] = cf{v[0] - v[2], v[1] - v[3]};
    }
    __syncthreads();
  }

  energy_assembly(tid, N, n_up, M, K, Q, radius, lambda, interaction, b, x, jas, geo, dgeo, al, ell0, ellt, ellL,
                  ellS, reinterpret_cast<double*>(sm + L.asmb), e_l, obs);
}


// ------------------------------------------------------------------ energy kernel, wave form
// Round 5, N <= 8 (every entry of an N x N matrix has its own lane) with staged rows: ONE
// 64-lane wave per walker (one-wave workgroups, so a barrier is a wave barrier), two phases
// instead of det_energy_kernel's 17 barrier-separated channel rounds on 256 threads:
//  (1) contraction.  The N orbital rows of channel c (each the electron's own spin block,
//      RW = 2 M N K floats) stream HBM -> registers (float4, issued one channel ahead, while
//      channel c - 1 is contracted) -> LDS; lane (i, j) forms every harmonic sum it needs:
//        c = 0         Phi0 = sum F0 e0, D0t / D0p = sum F0 de/dth | de/dph,
//                      L0 = sum F0 LB(e), S0k = sum F0 e_flow2,k
//        c = 1 + t     Phi_t = sum Ft e0 (+ D0t | D0p on the moved electron's row i_t),
//                      At / Ap = sum Ft de/dth | de/dph:  Gu_k += alpha_kt (phh_k At - thh_k Ap),
//                      LB2 += At | Ap on row i_t
//        c = 1 + T     Phi_L  = sum FL e0 + L0 + 2 LB2
//        c = 2 + T + k Phi_Sk = sum FSk e0 + S0k + 2 Gu_k
//      (det_energy_kernel's flow first-order sums sum F (phh_k de/dth - thh_k de/dph) are
//      the same two harmonic sums At, Ap recombined: 3 complex sums per tangent channel
//      instead of 5).  Phi_t goes to LDS, the other channel matrices stay in registers.
//  (2) algebra.  B = Phi0^-1 by the same Gauss-Jordan (eliminate), M_t = B Phi_t with the
//      column of Phi_t from LDS, tr M_t per t from LDS diagonals, the squared traces and the
//      L / S traces as wave sums (the transposed entry by a lane permute), then the shared
//      f64 assembly.  Same formulas as det_energy_kernel; the harmonic
//      sums are the same FMAs in the same order, the extra terms are added as separate sums.
// NV: float4 (VEC) or floats per lane per channel row set (N RW floats over 64 lanes).
struct DetWaveSmem {
  int S, LS, Fs, leaf, leaf2, Aug, fac, DG, geo, alpha, dgeo, asmb, ell, misc, xs, nrm, total;
};
__host__ __device__ inline DetWaveSmem det_wave_layout(int N, int M, int K) {
  DetWaveSmem L;
  const int T = 2 * N, NN = N * N, RW = 2 * M * N * K, NK = N * K;
  // staged row stride S = RW + pad with S = N K (mod 32): lane (i, j) reads bank K (i N + j)
  // (conflict-free for K = 1); kept even so that a float4 lands as two 8-B stores
  int want = NK & 31;
  if (NK & 1) want = (want + 1) & 31;
  L.S = RW + (((want - RW) % 32) + 32) % 32;
  L.LS = 8 * M + 4;  // leaf row stride per electron: b128 reads of different electrons on different banks
  int o = 0;
  L.Fs = o;
  o += N * L.S;
  o = (o + 3) & ~3;
  L.leaf = o;  // [i][m] (e0, de/dth, de/dph, d2e/dth2)
  o += N * L.LS;
  L.leaf2 = o;  // [i][m] (LB(e), e_flow2,0..2) for channel 0; then Phi_t [T][NN]
  o += (N * L.LS > 2 * T * NN) ? N * L.LS : 2 * T * NN;
  L.Aug = o;
  o += 4 * NN;
  L.fac = o;
  o += 2 * N;
  L.DG = o;
  o += 2 * T * N;
  L.geo = o;
  o += 4 * N;
  L.alpha = o;
  o += 3 * T;
  o = (o + 1) & ~1;
  L.dgeo = o;
  o += 8 * N;
  L.asmb = o;
  o += 2 * (4 * T + 10 * N + 2 * K);
  L.ell = o;  // ell0 [K], ellt [K T], ellL [K], ellS [3 K] (complex)
  o += 2 * K * (T + 5);
  L.misc = o;
  o += 8;
  L.xs = o;  // the walker's (theta, phi) and the harmonics' norms: the leaves read LDS only, so
  o += 2 * N;  // no global load queues behind the staged channel rows (vmcnt counts in order)
  L.nrm = o;
  o += M;
  L.total = o;
  return L;
}
constexpr int kDetWaveMaxN = 8;

#ifndef DET_WAVE_WPE  // A/B knob: waves per SIMD the det_energy_wave_kernel is compiled for (0: the compiler's choice)
#define DET_WAVE_WPE 0
#endif
#if DET_WAVE_WPE > 0
#define DET_WAVE_ATTR __attribute__((amdgpu_waves_per_eu(DET_WAVE_WPE, DET_WAVE_WPE)))
#else
#define DET_WAVE_ATTR
#endif
template <int NV, bool VEC>
__global__ __launch_bounds__(64) DET_WAVE_ATTR void det_energy_wave_kernel(const float* __restrict__ Fp, int ldF,
                                                             const float* __restrict__ x, const float* __restrict__ geo_g,
                                                             const float* __restrict__ jas, const float* __restrict__ norm,
                                                             float* __restrict__ e_l, float* __restrict__ obs, int N,
                                                             int n_up, int M, int K, float Q, float radius, float lambda,
                                                             int interaction) {
  extern __shared__ float sm[];
  const int T = 2 * N, C = 2 * N + 5, NN = N * N, NK = N * K, MNK = M * NK, RW = 2 * MNK;
  const int tid = threadIdx.x, b = blockIdx.x;
  const DetWaveSmem L = det_wave_layout(N, M, K);
  const int S = L.S, LS = L.LS;
  float* Fs = sm + L.Fs;
  float* leaf = sm + L.leaf;
  float* leaf2 = sm + L.leaf2;
  cf* Pt = reinterpret_cast<cf*>(sm + L.leaf2);  // after channel 0
  cf* Aug = reinterpret_cast<cf*>(sm + L.Aug);
  cf* fac = reinterpret_cast<cf*>(sm + L.fac);
  cf* DG = reinterpret_cast<cf*>(sm + L.DG);
  float* geo = sm + L.geo;
  float* al = sm + L.alpha;
  double* dgeo = reinterpret_cast<double*>(sm + L.dgeo);
  cf* ell0 = reinterpret_cast<cf*>(sm + L.ell);
  cf* ellt = ell0 + K;
  cf* ellL = ellt + K * T;
  cf* ellS = ellL + K;
  int* piv = reinterpret_cast<int*>(sm + L.misc);
  cf* logdet = reinterpret_cast<cf*>(sm + L.misc + 2);
  float* xs = sm + L.xs;
  float* nrm = sm + L.nrm;
  // lane (i, j): entry (i, j) of every N x N matrix (lanes >= N N carry zeros)
  const bool act = tid < NN;
  const int i = act ? tid / N : 0, j = act ? tid - (tid / N) * N : 0;
  const int tr_lane = j * N + i;  // the lane holding entry (j, i)

  // ---- staging: channel c's N rows (own spin block) -> registers -> LDS (row stride S)
  const size_t rowbase = (size_t)b * N * C;
  using PF = typename std::conditional<VEC, float4, float>::type;
  // two channels' rows in flight (DET_WAVE_PF2, round 5): channel c + 2 is requested while c is
  // contracted, into the buffer c just left
  // (one buffer for the widest float4 forms, NV >= 8: two would cost the second wave per SIMD)
  constexpr bool PF2 = !(VEC && NV >= 8);
  PF pfa[NV], pfb[NV];
  const int unit = VEC ? 4 : 1, RU = RW / unit;  // units per row
  // per unit u: element offsets of its row piece from the walker's first row (channel 0) and
  // in the staged rows, formed once; a lane without a piece (q >= N RU) re-loads piece 0 and
  // stores into the Aug area (written afresh after the channel loop), so loads and stores are
  // unconditional: branches around them made every store wait for all loads (vmcnt(0)), the
  // other buffer's included
  const float* Fw = Fp + rowbase * ldF;
  int goff[NV], soff[NV];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int q = tid + 64 * u;
    const bool ok = q < N * RU;
    const int r = ok ? q / RU : 0, w = ok ? q - r * RU : 0;
    const int blk = (r >= n_up && n_up > 0) ? 1 : 0;
    goff[u] = r * C * ldF + blk * RW + w * unit;
    soff[u] = ok ? L.Fs + r * S + w * unit : L.Aug;
  }
  auto stage_load = [&](PF (&pf)[NV], int c) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const float* src = Fw + (goff[u] + c * ldF);
      if constexpr (VEC)
        pf[u] = *reinterpret_cast<const float4*>(src);
      else
        pf[u] = *src;
    }
  };
  auto stage_store = [&](const PF (&pf)[NV]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      float* dst = sm + soff[u];
      if constexpr (VEC) {
        reinterpret_cast<float2*>(dst)[0] = make_float2(pf[u].x, pf[u].y);
        reinterpret_cast<float2*>(dst)[1] = make_float2(pf[u].z, pf[u].w);
      } else {
        *dst = pf[u];
      }
    }
  };

  DET_T(1, 0);
  // ---- geometry, flow coefficients (as det_energy_kernel)
  for (int e = tid; e < N; e += 64) {
    const float4 g = *reinterpret_cast<const float4*>(geo_g + 4 * (size_t)(b * N + e));
    geo[4 * e] = g.x;
    geo[4 * e + 1] = g.y;
    geo[4 * e + 2] = g.z;
    geo[4 * e + 3] = g.w;
    double st, ct, sp, cp;
    sincos((double)x[2 * (b * N + e)], &st, &ct);
    sincos((double)x[2 * (b * N + e) + 1], &sp, &cp);
    dgeo[4 * e] = st;
    dgeo[4 * e + 1] = ct;
    dgeo[4 * e + 2] = sp;
    dgeo[4 * e + 3] = cp;
    xs[2 * e] = x[2 * (b * N + e)];
    xs[2 * e + 1] = x[2 * (b * N + e) + 1];
  }
  for (int p = tid; p < M; p += 64) nrm[p] = norm[p];
  __syncthreads();
  for (int t = tid; t < T; t += 64) {
    const int e = t >> 1;
    const float st = geo[4 * e], ct = geo[4 * e + 1], sp = geo[4 * e + 2], cp = geo[4 * e + 3];
    for (int k = 0; k < 3; ++k) {
      float a;
      if ((t & 1) == 0)
        a = (k == 0) ? -sp : (k == 1 ? cp : 0.f);
      else
        a = (k == 0) ? -(ct * cp) : (k == 1 ? -(ct * sp) : st);
      al[k * T + t] = a;
    }
  }
  // this lane's row geometry (flow first-order coefficients phh, thh of electron i)
  const float gst = geo[4 * i], gct = geo[4 * i + 1], gsp = geo[4 * i + 2], gcp = geo[4 * i + 3];
  const float phh[3] = {-gsp, gcp, 0.f};
  const float thh[3] = {gct * gcp, gct * gsp, -gst};

  for (int kd = 0; kd < K; ++kd) {
    stage_load(pfa, 0);
    if constexpr (PF2) stage_load(pfb, 1);  // C = 2 N + 5 > 1
    // envelope leaves of every (electron, harmonic): e0, de/dth, de/dph, d2e/dth2 and, for
    // channel 0, LB(e) and the flow second derivatives (same functions as det_energy_kernel)
    lds_barrier();  // Pt of the previous determinant (aliases leaf2) is consumed
    for (int idx = tid; idx < N * M; idx += 64) {
      const int e = idx / M, p = idx - (idx / M) * M;
      const float st = geo[4 * e], ct = geo[4 * e + 1], sp = geo[4 * e + 2], cp = geo[4 * e + 3];
      const float gauge = env_gauge(ct, M);
      const EnvLeaf lf = env_leaf(xs[2 * e], xs[2 * e + 1], p, M, nrm[p], true, gauge, DET_WAVE_SQ);
      const float m = (float)p - 0.5f * (float)(M - 1) - gauge;
      float* d = leaf + e * LS + 8 * p;
      reinterpret_cast<float4*>(d)[0] = make_float4(lf.e0.re, lf.e0.im, lf.dth.re, lf.dth.im);
      reinterpret_cast<float4*>(d)[1] = make_float4(lf.dph.re, lf.dph.im, lf.d2th.re, lf.d2th.im);
      const cf f0 = env_flow2(lf.e0, lf.dth, lf.d2th, m, st, ct, sp, cp, 0);
      const cf f1 = env_flow2(lf.e0, lf.dth, lf.d2th, m, st, ct, sp, cp, 1);
      const cf f2 = env_flow2(lf.e0, lf.dth, lf.d2th, m, st, ct, sp, cp, 2);
      float* d2 = leaf2 + e * LS + 8 * p;
      reinterpret_cast<float4*>(d2)[0] = make_float4(lf.lb.re, lf.lb.im, f0.re, f0.im);
      reinterpret_cast<float4*>(d2)[1] = make_float4(f1.re, f1.im, f2.re, f2.im);
    }
    DET_T(1, 1);
    const float* Frow = Fs + i * S + j * K + kd;  // re at + m NK, im at + MNK + m NK
    const float* lrow = leaf + i * LS;
    const float* l2row = leaf2 + i * LS;
    cf P0{0.f, 0.f}, D0t{0.f, 0.f}, D0p{0.f, 0.f}, L0{0.f, 0.f}, S0[3] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
    cf Gu[3] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}}, LB2{0.f, 0.f}, PL{0.f, 0.f};
    cf PS[3] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
    auto chan = [&](int c) __attribute__((always_inline)) {
      if (c == 0) {
        for (int m = 0; m < M; ++m) {
          const cf f{Frow[m * NK], Frow[MNK + m * NK]};
          const float4 a = *reinterpret_cast<const float4*>(lrow + 8 * m);
          const float4 q = *reinterpret_cast<const float4*>(lrow + 8 * m + 4);
          const float4 u = *reinterpret_cast<const float4*>(l2row + 8 * m);
          const float4 v = *reinterpret_cast<const float4*>(l2row + 8 * m + 4);
          cfma(P0, f, cf{a.x, a.y});
          cfma(D0t, f, cf{a.z, a.w});
          cfma(D0p, f, cf{q.x, q.y});
          cfma(L0, f, cf{u.x, u.y});
          cfma(S0[0], f, cf{u.z, u.w});
          cfma(S0[1], f, cf{v.x, v.y});
          cfma(S0[2], f, cf{v.z, v.w});
        }
      } else if (c <= T) {
        const int t = c - 1;
        cf Pe{0.f, 0.f}, At{0.f, 0.f}, Ap{0.f, 0.f};
#pragma unroll 4
        for (int m = 0; m < M; ++m) {
          const cf f{Frow[m * NK], Frow[MNK + m * NK]};
          const float4 a = *reinterpret_cast<const float4*>(lrow + 8 * m);
          const float2 q = *reinterpret_cast<const float2*>(lrow + 8 * m + 4);
          cfma(Pe, f, cf{a.x, a.y});
          cfma(At, f, cf{a.z, a.w});
          cfma(Ap, f, cf{q.x, q.y});
        }
        const bool own = (i == (t >> 1));
        if (own) {
          Pe += (t & 1) ? D0p : D0t;
          LB2 += (t & 1) ? Ap : At;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float ak = al[k * T + t];
          const cf g{phh[k] * At.re - thh[k] * Ap.re, phh[k] * At.im - thh[k] * Ap.im};
          Gu[k] += ak * g;
        }
        if (act) Pt[t * NN + tid] = Pe;  // leaf2 is free: channel 0's readers passed the barriers above
      } else {
        cf Pe{0.f, 0.f};
#pragma unroll 4
        for (int m = 0; m < M; ++m) {
          const cf f{Frow[m * NK], Frow[MNK + m * NK]};
          const float2 a = *reinterpret_cast<const float2*>(lrow + 8 * m);
          cfma(Pe, f, cf{a.x, a.y});
        }
        // (register arrays indexed by compile-time constants only: a run-time index sends them to scratch)
        if (c == T + 1)
          PL = Pe + L0 + 2.f * LB2;
        else if (c == T + 2)
          PS[0] = Pe + S0[0] + 2.f * Gu[0];
        else if (c == T + 3)
          PS[1] = Pe + S0[1] + 2.f * Gu[1];
        else
          PS[2] = Pe + S0[2] + 2.f * Gu[2];
      }
    };
    // channel c from buffer c & 1, which then takes channel c + 2 (in flight while c and c + 1
    // are contracted, and across the barriers: they wait for LDS only).  The loads are
    // unconditional (past the last channel they re-read it): a load under a branch leaves the
    // compiler's counted waits at the path without it, and the stores would drain both buffers
    if constexpr (PF2) {
      for (int c = 0; c < C; c += 2) {
        lds_barrier();  // the readers of channel c - 1 are done with Fs
        stage_store(pfa);
        lds_barrier();
        stage_load(pfa, min(c + 2, C - 1));
        chan(c);
        if (c + 1 < C) {
          lds_barrier();
          stage_store(pfb);
          lds_barrier();
        }
        stage_load(pfb, min(c + 3, C - 1));
        if (c + 1 < C) chan(c + 1);
      }
    } else {
      for (int c = 0; c < C; ++c) {
        lds_barrier();
        stage_store(pfa);
        lds_barrier();
        stage_load(pfa, min(c + 1, C - 1));
        chan(c);
      }
    }
    DET_T(1, 2);
    // ---- B = Phi0^-1 (augmented Gauss-Jordan, partial pivoting), log det Phi0
    if (act) {
      Aug[i * 2 * N + j] = P0;
      Aug[i * 2 * N + N + j] = (i == j) ? cf{1.f, 0.f} : cf{0.f, 0.f};
    }
    __syncthreads();
    if (DET_GJ_REG) {  // register Gauss-Jordan, one augmented column per lane
      cf col[kDetWaveMaxN];
      const bool lc = tid < 2 * N;
#pragma unroll
      for (int r = 0; r < kDetWaveMaxN; ++r)
        col[r] = (lc && r < N) ? (tid < N ? Aug[r * 2 * N + tid] : cf{r == tid - N ? 1.f : 0.f, 0.f}) : cf{0.f, 0.f};
      const cf l = gj_inverse_cols<kDetWaveMaxN>(col, N);
      if (tid >= N && lc)
#pragma unroll
        for (int r = 0; r < kDetWaveMaxN; ++r)
          if (r < N) Aug[r * 2 * N + tid] = col[r];
      if (tid == 0) ell0[kd] = l;
      __syncthreads();
    } else {
      eliminate(Aug, 2 * N, N, 2 * N, true, fac, piv, logdet, tid, 64, 64);
      if (tid == 0) ell0[kd] = *logdet;
    }
    DET_T(1, 3);
    cf Br[kDetWaveMaxN];
#pragma unroll
    for (int l = 0; l < kDetWaveMaxN; ++l) Br[l] = (act && l < N) ? Aug[i * 2 * N + N + l] : cf{0.f, 0.f};
    const cf BT = act ? Aug[j * 2 * N + N + i] : cf{0.f, 0.f};  // B[j][i]
    // ---- M_t = B Phi_t, traces
    cf sq{0.f, 0.f}, Mu[3] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
    for (int t = 0; t < T; ++t) {
      cf mt{0.f, 0.f};
#pragma unroll
      for (int l = 0; l < kDetWaveMaxN; ++l)
        if (l < N) cfma(mt, Br[l], act ? Pt[t * NN + l * N + j] : cf{0.f, 0.f});
      const cf mT{__shfl(mt.re, tr_lane, 64), __shfl(mt.im, tr_lane, 64)};
      if (act) {
        sq += mt * mT;
        if (i == j) DG[t * N + i] = mt;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) Mu[k] += al[k * T + t] * mt;
    }
    float v[16];
    {
      const cf pl = act ? BT * PL : cf{0.f, 0.f};
      v[0] = sq.re;
      v[1] = sq.im;
      v[2] = pl.re;
      v[3] = pl.im;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const cf ps = act ? BT * PS[k] : cf{0.f, 0.f};
        const cf muT{__shfl(Mu[k].re, tr_lane, 64), __shfl(Mu[k].im, tr_lane, 64)};
        const cf m2 = act ? Mu[k] * muT : cf{0.f, 0.f};
        v[4 + 4 * k] = ps.re;
        v[5 + 4 * k] = ps.im;
        v[6 + 4 * k] = m2.re;
        v[7 + 4 * k] = m2.im;
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = wave_sum(v[q]);
    __syncthreads();  // DG written
    if (tid < T) {
      cf s{0.f, 0.f};
      for (int e = 0; e < N; ++e) s += DG[tid * N + e];
      ellt[kd * T + tid] = s;
    }
    if (tid == 0) {
      ellL[kd] = cf{v[2] - v[0], v[3] - v[1]};
#pragma unroll
      for (int k = 0; k < 3; ++k) ellS[3 * kd + k] = cf{v[4 + 4 * k] - v[6 + 4 * k], v[5 + 4 * k] - v[7 + 4 * k]};
    }
  }
  DET_T(1, 4);
  energy_assembly(tid, N, n_up, M, K, Q, radius, lambda, interaction, b, x, jas, geo, dgeo, al, ell0, ellt, ellL, ellS,
                  reinterpret_cast<double*>(sm + L.asmb), e_l, obs);
  DET_T(1, 5);
}


// ------------------------------------------------------------------ backward (parameter gradient)
// log psi = J + log sum_k det Phi_k (psiformer.py:72-76, 91).  For the per-walker cotangent
// c = ct.re + i ct.im of (Re log psi, Im log psi):
//   d log psi / d Phi_k[i][j] = w_k inv_k[j][i],  w_k = det Phi_k / sum_k det Phi_k
//   G_k = c conj(w_k inv_k^T)   (dL/dRe Phi = Re G, dL/dIm Phi = Im G)
//   dF[i, (blk_i, re|im, m, j, k)] = G_k[i][j] conj(env[i][m])   (blocks.py:64-68)
//   jg = ct.re dJ/d(alpha_par, alpha_anti),  dJ/dalpha = -c alpha (alpha + 2 r) / (alpha + r)^2
// One 64-thread workgroup per walker: pass 1 LU of every Phi_k (the log-dets), pass 2
// Gauss-Jordan inverse of each Phi_k and the owned columns of dF; the other spin block's
// and the padding columns are written 0.
__global__ __launch_bounds__(64) void det_bwd_kernel(const float* __restrict__ Fp, int ldF, const float* __restrict__ x,
                                                     const float* __restrict__ jas, const float* __restrict__ norm,
                                                     const float* __restrict__ ct, float* __restrict__ dF,
                                                     float* __restrict__ jg, int N, int n_up, int M, int K,
                                                     int orb_cols) {
  extern __shared__ float sm_raw[];
  cf* E0 = reinterpret_cast<cf*>(sm_raw);  // [N][M]
  cf* A = E0 + N * M;                      // [N][2N]
  cf* fac = A + 2 * N * N;                 // [N]
  cf* ld = fac + N;                        // [K]
  cf* logdet = ld + K;
  cf* wk = logdet + 1;                     // [K]
  int* piv = reinterpret_cast<int*>(wk + K);
  double* cart = reinterpret_cast<double*>(piv + 2);  // [N][3] (double: close pairs)
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const FView F{Fp, ldF, M, N, K};
  const int MNK = M * N * K;
  for (int idx = tid; idx < N * M; idx += nt) {
    const int i = idx / M, p = idx % M;
    E0[idx] = env_leaf(x[2 * (b * N + i)], x[2 * (b * N + i) + 1], p, M, norm[p], false, 0.f, true).e0;  // as det_value (powers by squaring)
  }
  for (int i = tid; i < N; i += nt) {
    double st, ct_, sp, cp;
    sincos((double)x[2 * (b * N + i)], &st, &ct_);
    sincos((double)x[2 * (b * N + i) + 1], &sp, &cp);
    cart[3 * i] = st * cp;
    cart[3 * i + 1] = st * sp;
    cart[3 * i + 2] = ct_;
  }
  // columns of dF this walker's rows do not own: the other spin block, the padding
  for (int idx = tid; idx < N * ldF; idx += nt) {
    const int i = idx / ldF, col = idx - (idx / ldF) * ldF;
    const int blk_i = (i >= n_up && n_up > 0) ? 1 : 0;
    const bool own = col < orb_cols && col / (2 * MNK) == blk_i;
    if (!own) dF[((size_t)b * N + i) * ldF + col] = 0.f;
  }
  const float cr = ct[2 * b], ci = ct[2 * b + 1];
  if (cr == 0.f && ci == 0.f) {
    // a walker without weight (NaN diff: the reference's nanmean / nan_to_num drop it,
    // loss.py:59-64; or psi = 0 in the KFAC Fisher pass): zero rows, so a singular matrix's
    // inf inverse cannot turn 0 * inf into NaN in every weight gradient
    for (int idx = tid; idx < N * orb_cols; idx += nt) dF[((size_t)b * N + idx / orb_cols) * ldF + idx % orb_cols] = 0.f;
    if (tid == 0) {
      jg[2 * b] = 0.f;
      jg[2 * b + 1] = 0.f;
    }
    return;
  }
  __syncthreads();
  // Jastrow parameter derivatives (double, reduced over the wave)
  {
    double gp = 0.0, ga = 0.0;
    const double ap = jas[0], aa = jas[1];
    for (int q = tid; q < N * N; q += nt) {
      const int i = q / N, j = q - (q / N) * N;
      if (j <= i) continue;
      const double dx = cart[3 * j] - cart[3 * i], dy = cart[3 * j + 1] - cart[3 * i + 1],
                   dz = cart[3 * j + 2] - cart[3 * i + 2];
      const double r = sqrt(dx * dx + dy * dy + dz * dz);
      const bool same = (i < n_up) == (j < n_up);
      const double al = same ? ap : aa, cst = same ? 0.25 : 0.5;
      const double g = -cst * al * (al + 2.0 * r) / ((al + r) * (al + r));
      if (same)
        gp += g;
      else
        ga += g;
    }
    for (int o = 32; o > 0; o >>= 1) {
      gp += __shfl_xor(gp, o, 64);
      ga += __shfl_xor(ga, o, 64);
    }
    if (tid == 0) {
      jg[2 * b] = (float)(cr * gp);
      jg[2 * b + 1] = (float)(cr * ga);
    }
  }
  auto build = [&](int k, int lda) {
    for (int idx = tid; idx < N * N; idx += nt) {
      const int i = idx / N, j = idx % N;
      const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
      const size_t row = (size_t)b * N + i;
      cf acc{0.f, 0.f};
      for (int p = 0; p < M; ++p) cfma(acc, F.at(row, blk, p, j, k), E0[i * M + p]);
      A[i * lda + j] = acc;
      if (lda > N) A[i * lda + N + j] = cf{i == j ? 1.f : 0.f, 0.f};
    }
    __syncthreads();
  };
  // pass 1: log det of every determinant -> softmax weights w_k
  if (K > 1) {
    for (int k = 0; k < K; ++k) {
      build(k, N);
      eliminate(A, N, N, N, false, fac, piv, logdet);
      if (tid == 0) ld[k] = *logdet;
      __syncthreads();
    }
    if (tid == 0) {
      float lmax = -INFINITY;
      for (int k = 0; k < K; ++k) lmax = fmaxf(lmax, ld[k].re);
      cf z{0.f, 0.f};
      for (int k = 0; k < K; ++k) {
        const float mag = expf(ld[k].re - lmax);
        z += cf{mag * cosf(ld[k].im), mag * sinf(ld[k].im)};
      }
      for (int k = 0; k < K; ++k) {
        const float mag = expf(ld[k].re - lmax);
        wk[k] = cdiv(cf{mag * cosf(ld[k].im), mag * sinf(ld[k].im)}, z);
      }
    }
  } else if (tid == 0) {
    wk[0] = cf{1.f, 0.f};
  }
  __syncthreads();
  // pass 2: inverse of each Phi_k, owned dF columns
  for (int k = 0; k < K; ++k) {
    build(k, 2 * N);
    eliminate(A, 2 * N, N, 2 * N, true, fac, piv, logdet);
    const cf w = wk[k];
    for (int idx = tid; idx < N * M * N; idx += nt) {
      const int i = idx / (M * N), rem = idx - i * (M * N), p = rem / N, j = rem - (rem / N) * N;
      const int blk = (i >= n_up && n_up > 0) ? 1 : 0;
      const cf f = w * A[j * 2 * N + N + i];  // d log psi / d Phi_k[i][j]
      // G = c conj(f); dF = G conj(env)
      const cf G{cr * f.re + ci * f.im, ci * f.re - cr * f.im};
      const cf e = E0[i * M + p];
      const cf v{G.re * e.re + G.im * e.im, G.im * e.re - G.re * e.im};
      const size_t rowoff = ((size_t)b * N + i) * ldF;
      const int off = p * N * K + j * K + k;
      dF[rowoff + (size_t)(blk * 2) * MNK + off] = v.re;
      dF[rowoff + (size_t)(blk * 2 + 1) * MNK + off] = v.im;
    }
    __syncthreads();
  }
}

__global__ void potential_kernel(const float* __restrict__ x, float* __restrict__ pe, int nw, int N, float Q,
                                 float radius, int interaction) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nw) return;
  double acc = 0.0;
  for (int i = 0; i < N; ++i) {
    const double ti = x[2 * (b * N + i)], pi_ = x[2 * (b * N + i) + 1];
    const double xi = sin(ti) * cos(pi_), yi = sin(ti) * sin(pi_), zi = cos(ti);
    for (int j = i + 1; j < N; ++j) {
      const double tj = x[2 * (b * N + j)], pj = x[2 * (b * N + j) + 1];
      const double u = xi * sin(tj) * cos(pj) + yi * sin(tj) * sin(pj) + zi * cos(tj);
      if (interaction == DH_INTERACTION_COULOMB)
        acc += 1.0 / sqrt(2.0 - 2.0 * u);
      else
        acc += 1.0 + ((double)Q + 1.0) / (double)Q * u;
    }
  }
  if (interaction == DH_INTERACTION_COULOMB) acc /= (double)radius;
  pe[b] = (float)acc;
}

}  // namespace

void launch_potential(const Dims& d, const float* x, float* pe, int nw, hipStream_t s) {
  hipLaunchKernelGGL(potential_kernel, dim3((nw + 127) / 128), dim3(128), 0, s, x, pe, nw, d.N, d.Q, d.r,
                     d.interaction);
}

void launch_det_value(const Dims& d, const float* F, const float* x, const float* jastrow, const float* norm,
                      float* logpsi, int nw, hipStream_t s, const McmcEpi& epi) {
  // floats per walker region (+1: the epilogue's log psi slot after the f64 unit vectors)
  const int per = (2 * d.N * d.M + 2 * d.N * d.N + 2 * d.N + 2 * d.K + 2 + 4 + 6 * d.N + 2 + 3 + 1) & ~3;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(nw), dim3(64), (size_t)per * sizeof(float), s, F, d.ld_orb, x, jastrow, norm,
                       logpsi, d.N, d.n_up, d.M, d.K, nw, per, epi);
  };
  const int mgv = (d.M + 64 / d.N - 1) / (64 / d.N);  // harmonics per lane
  if (mgv <= 2 && d.N * d.N <= 64) {
    // two walkers per wave (C2, M = 16, N = 6)
    hipLaunchKernelGGL((det_value_kernel<0, true>), dim3((nw + 1) / 2), dim3(64), (size_t)2 * per * sizeof(float), s, F,
                       d.ld_orb, x, jastrow, norm, logpsi, d.N, d.n_up, d.M, d.K, nw, per, epi);
  } else if (mgv <= 2)  // serial per entry (C2 at one walker per wave: 0.35 ms against 0.41 ms lane groups)
    go(det_value_kernel<0>);
  else if (mgv <= 4)
    go(det_value_kernel<4>);
  else if (mgv <= 8)
    go(det_value_kernel<8>);
  else if (mgv <= 16)
    go(det_value_kernel<16>);
  else if (mgv <= 24)
    go(det_value_kernel<24>);
  else if (mgv <= 32)
    go(det_value_kernel<32>);
  else
    go(det_value_kernel<64>);
}

void launch_det_bwd(const Dims& d, const float* F, const float* x, const float* jastrow, const float* norm,
                    const float* ct, float* dF, float* jg, int nw, hipStream_t s) {
  const size_t bytes =
      (size_t)(2 * d.N * d.M + 4 * d.N * d.N + 2 * d.N + 4 * d.K + 2 + 4 + 6 * d.N + 2) * sizeof(float);
  ensure_smem(det_bwd_kernel, bytes);
  hipLaunchKernelGGL(det_bwd_kernel, dim3(nw), dim3(64), bytes, s, F, d.ld_orb, x, jastrow, norm, ct, dF, jg, d.N,
                     d.n_up, d.M, d.K, d.orb_cols);
}

bool det_precontract(const Dims& d) {
  const bool fits = 2 * d.K * d.N <= d.D && d.N <= 32 && d.M <= 16 * 4 * (64 / d.N) && d.M <= 128;
  // the direct kernel stages small channel rows through LDS (C2: 0.64 ms against 0.93 ms
  // precontracted); larger rows (C4: 3.96 -> 1.92 ms, C5: 52 -> 15.5 ms) go through PhiC
  return fits && !(det_staged(d.N, d.M, d.K) && 2 * d.M * d.N * d.K * d.N <= 8 * 256);
}

// det_energy_wave_kernel for this shape: the template's per-lane staging width NV, or 0
static int det_wave_nv(const Dims& d, bool& vec) {
  if (d.N > kDetWaveMaxN || !det_staged(d.N, d.M, d.K)) return 0;
  const int RW = 2 * d.M * d.N * d.K;
  vec = (RW % 4 == 0) && (d.ld_orb % 4 == 0);
  const int units = vec ? d.N * RW / 4 : d.N * RW;
  const int need = (units + 63) / 64;
  for (int v : (vec ? std::initializer_list<int>{1, 2, 3, 5, 8, 12} : std::initializer_list<int>{1, 2, 4, 8, 16}))
    if (need <= v) return v;
  return 0;
}

void launch_det_energy(const Dims& d, const float* F, const float* x, const float* geo, const float* jastrow,
                       const float* norm, float* e_l, float* obs, int nw, hipStream_t s, float* phic) {
  bool vec = false;
  const int nv = phic ? 0 : det_wave_nv(d, vec);
  if (nv > 0) {
    const size_t bytes = (size_t)det_wave_layout(d.N, d.M, d.K).total * sizeof(float);
    auto go = [&](auto kern) {
      ensure_smem(kern, bytes);
      hipLaunchKernelGGL(kern, dim3(nw), dim3(64), bytes, s, F, d.ld_orb, x, geo, jastrow, norm, e_l, obs, d.N, d.n_up,
                         d.M, d.K, d.Q, d.r, d.lambda, d.interaction);
    };
    if (vec) {
      switch (nv) {
        case 1: go(det_energy_wave_kernel<1, true>); break;
        case 2: go(det_energy_wave_kernel<2, true>); break;
        case 3: go(det_energy_wave_kernel<3, true>); break;
        case 5: go(det_energy_wave_kernel<5, true>); break;
        case 8: go(det_energy_wave_kernel<8, true>); break;
        default: go(det_energy_wave_kernel<12, true>); break;
      }
    } else {
      switch (nv) {
        case 1: go(det_energy_wave_kernel<1, false>); break;
        case 2: go(det_energy_wave_kernel<2, false>); break;
        case 4: go(det_energy_wave_kernel<4, false>); break;
        case 8: go(det_energy_wave_kernel<8, false>); break;
        default: go(det_energy_wave_kernel<16, false>); break;
      }
    }
    return;
  }
  const DetSmem L = det_layout(d.N, d.M, d.K, 4, phic != nullptr);
  const size_t bytes = (size_t)L.total * sizeof(float);
  auto go = [&](auto kern) {
    ensure_smem(kern, bytes);
    hipLaunchKernelGGL(kern, dim3(nw), dim3(256), bytes, s, F, d.ld_orb, x, geo, jastrow, norm, e_l, obs, d.N, d.n_up,
                       d.M, d.K, d.Q, d.r, d.lambda, d.interaction, (const float*)phic);
  };
  const int nrw = 2 * d.M * d.N * d.K * d.N;  // floats of one channel's N staged rows
  if (phic) {
    const int G = 64 / d.N;
    const int mgw = (d.M + G - 1) / G;          // harmonics per lane, one wave per electron
    const int mg = (d.M + 4 * G - 1) / (4 * G);  // harmonics per lane, four waves per electron
    auto env = [&](auto kern, int MG, bool WU, bool seg = false) {
      const size_t eb = env_contract_smem(d.N, d.M, MG, WU, d.K, seg);
      ensure_smem(kern, eb);
      const int grid = WU ? (nw * d.N + 3) / 4 : nw * d.N;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), eb, s, F, d.ld_orb, x, geo, norm, phic, nw, d.N, d.n_up, d.M,
                         d.K, d.Q);
    };
    // C5 (N = 20, one spin block, K = 1): rows streamed through registers (env_stream_kernel)
    const int mgs = ((d.M + 3) / 4 + (64 / d.N) - 1) / (64 / d.N);  // harmonics per lane, four waves
    if (d.N == 20 && d.K == 1 && mgs <= 5) {
      const size_t eb = ((size_t)10 * (d.M + 1) * 2 + 4 * (2 * d.N + 5) * d.N * 2 + 512 + 3 * 2 * d.N) * sizeof(float);
      hipLaunchKernelGGL((env_stream_kernel<20, 5, 8>), dim3(nw * d.N), dim3(256), eb, s, F, d.ld_orb, x, geo, norm,
                         phic, d.n_up, d.M);
      go(det_energy_kernel<0, true>);
      return;
    }
    if (mgw <= 4) {  // short rows (C4: M = 24, N = 10): a wave per electron
      switch (mgw) {
        case 1: env(env_contract_kernel<1, true>, 1, true); break;
        case 2: env(env_contract_kernel<2, true>, 2, true); break;
        case 3: env(env_contract_kernel<3, true>, 3, true); break;
        default: env(env_contract_kernel<4, true>, 4, true); break;
      }
    } else {
      switch (mg) {
        case 1: env(env_contract_kernel<1>, 1, false); break;
        case 2: env(env_contract_kernel<2>, 2, false); break;
        case 3: env(env_contract_kernel<3>, 3, false); break;
        case 4: env(env_contract_kernel<4>, 4, false); break;
        case 5: {
          const int sg = env_contract_seg(d.N, d.M, d.K, 5, d.ld_orb);
          if (sg == 2)
            env(env_contract_kernel<5, false, 2>, 5, false, true);
          else if (sg == 1)
            env(env_contract_kernel<5, false, 1>, 5, false, true);
          else
            env(env_contract_kernel<5>, 5, false);
          break;
        }
        case 6: env(env_contract_kernel<6>, 6, false); break;
        case 7:
        case 8: env(env_contract_kernel<8>, 8, false); break;
        default: env(env_contract_kernel<16>, 16, false); break;
      }
    }
    go(det_energy_kernel<0, true>);
  } else if (!det_staged(d.N, d.M, d.K)) {
    go(det_energy_kernel<0>);
  }
  else if (nrw <= 8 * 256)
    go(det_energy_kernel<8>);
  else
    go(det_energy_kernel<kStageFloats / 256>);
}

size_t det_energy_smem_bytes(const Dims& d) { return (size_t)det_layout(d.N, d.M, d.K, 4).total * sizeof(float); }

namespace {
// test hook kernel: env_leaf of n angle pairs, every harmonic p < M, in the production gauge
__global__ void env_leaf_probe_kernel(const float* __restrict__ thph, int n, int M, int sq, float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * M) return;
  const int i = t / M, p = t - i * M;
  const float th = thph[2 * i], ph = thph[2 * i + 1];
  const EnvLeaf L = env_leaf(th, ph, p, M, 1.f, true, env_gauge(cosf(th), M), sq != 0);
  float* o = out + (size_t)t * 10;
  o[0] = L.e0.re, o[1] = L.e0.im, o[2] = L.dth.re, o[3] = L.dth.im, o[4] = L.dph.re;
  o[5] = L.dph.im, o[6] = L.lb.re, o[7] = L.lb.im, o[8] = L.d2th.re, o[9] = L.d2th.im;
}
}  // namespace

void launch_env_leaf_probe(const float* thph, int n, int M, int sq, float* out, hipStream_t s) {
  hipLaunchKernelGGL(env_leaf_probe_kernel, dim3((n * M + 127) / 128), dim3(128), 0, s, thph, n, M, sq, out);
}



// ------------------------------------------------------------------ envelope first (round 6)
// C4 / C5 (one spin block, one determinant, N > 8): every entry the determinant algebra reads is
// Phi_c[i][j] = sum_m F_c[i](m, j) e_m(x_i) + (own-electron / value-row leaf terms), with
// F_c[i] = h_c[i] W.  By associativity the e0 part is h_c[i] . Weff_i[:, j] with
// Weff_i = sum_m e_m(x_i) W[:, (m, j)] (256 x N complex per electron), so the 2 M N-column
// orbital map over all C channel rows (C5: 4.4 TFLOP per step, F = 34 GB written and read back)
// is replaced by
//   (1) Weff = E2 W2 — one GEMM over the electrons (rows: the envelope coefficients
//       (Re e_m | Im e_m) of each electron, K = 2 M padded to 32; columns (j, re / im, k));
//   (2) F of six special rows per electron only — the value row (with the bias), the two own
//       tangent rows, and the three flow rows hu_k = sum_t alpha_kt h_t (the tangent rows'
//       W_k terms of env_stream_kernel summed over t before the map instead of after);
//   (3) env_phi_kernel: h_c . Weff on the matrix cores (exact f32), the special rows'
//       leaf contractions (e0, d/dtheta, d/dphi, LB, flow2_k, W_k) from their F, and the
//       same assembly as env_stream_kernel -> PhiC for det_energy_kernel<0, true>.
// blocks.py:64-68 / psiformer.py:74 (the envelope sum), hamiltonian.py (the channels).
bool env_first(const Dims& d) {
  return d.K == 1 && d.NB == 1 && (d.N == 10 || d.N == 20) && d.D == 256 && 2 * d.M <= 128 && det_precontract(d);
}
int env_first_k(const Dims& d) { return round_up(2 * d.M, 32); }

namespace {

// S rows [e][6][256]: h_0, h_(1+2i), h_(2+2i), hu_0..2 (hu_k = sum_t alpha_kt h_t); the T
// tangent rows are loaded in one unrolled burst
template <int N>
__global__ __launch_bounds__(256) void srows_kernel(const float* __restrict__ h, const float* __restrict__ geo,
                                                    float* __restrict__ S) {
  const int e = blockIdx.x, b = e / N, i = e - (e / N) * N, k = threadIdx.x;
  constexpr int T = 2 * N, C = 2 * N + 5;
  const float* hr = h + (size_t)e * C * 256 + k;
  float* sr = S + (size_t)e * 6 * 256 + k;
  sr[0] = hr[0];
  sr[256] = hr[(size_t)(1 + 2 * i) * 256];
  sr[512] = hr[(size_t)(2 + 2 * i) * 256];
  float u0 = 0.f, u1 = 0.f, u2 = 0.f;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const float4 q = *reinterpret_cast<const float4*>(geo + 4 * (size_t)(b * N + (t >> 1)));  // st ct sp cp
    const float ht = hr[(size_t)(1 + t) * 256];
    if ((t & 1) == 0) {
      u0 = fmaf(-q.z, ht, u0);
      u1 = fmaf(q.w, ht, u1);
    } else {
      u0 = fmaf(-(q.y * q.w), ht, u0);
      u1 = fmaf(-(q.y * q.z), ht, u1);
      u2 = fmaf(q.x, ht, u2);
    }
  }
  sr[768] = u0;
  sr[1024] = u1;
  sr[1280] = u2;
}

// E2 [e][KE]: (Re e_m | Im e_m | 0 ...) of electron e, the leaves' own e0 (norm, gauge)
__global__ void env_coef_kernel(const float* __restrict__ x, const float* __restrict__ geo,
                                const float* __restrict__ norm, float* __restrict__ E2, int ne, int M, int KE) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ne * KE) return;
  const int e = t / KE, q = t - (t / KE) * KE;
  float v = 0.f;
  if (q < 2 * M) {
    const int p = q < M ? q : q - M;
    const float gauge = env_gauge(geo[4 * (size_t)e + 1], M);
    const EnvLeaf L = env_leaf(x[2 * (size_t)e], x[2 * (size_t)e + 1], p, M, norm[p], false, gauge, DET_LEAF_SQ);
    v = q < M ? L.e0.re : L.e0.im;
  }
  E2[t] = v;
}

// W2T [n = (2 j + part) 256 + k][KE]: Weff_re[k][j] = sum_m Wre e_re - Wim e_im, Weff_im = Wre e_im + Wim e_re
__global__ void env_w2_kernel(const float* __restrict__ Worb, int ldw, int M, int N, int D, int KE,
                              float* __restrict__ W2T) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= D * 2 * N * KE) return;
  const int n = t / KE, q = t - (t / KE) * KE;
  const int jp = n / D, k = n - (n / D) * D, j = jp >> 1, part = jp & 1;  // Weff laid out [jp][k]
  float v = 0.f;
  if (q < 2 * M) {
    const int m = q < M ? q : q - M, qim = q >= M, MN = M * N;
    const float wre = Worb[(size_t)k * ldw + m * N + j], wim = Worb[(size_t)k * ldw + MN + m * N + j];
    v = part == 0 ? (qim ? -wim : wre) : (qim ? wre : wim);
  }
  W2T[t] = v;
}

typedef float f4e __attribute__((ext_vector_type(4)));

// One 256-thread workgroup per electron, one burst of loads up front: the six special F rows
// (LDS-DMA) and the MFMA operands of h_c . Weff
// (v_mfma_f32_16x16x4_f32, exact f32) straight from global memory.  The product is split over
// K: wave w takes k in [64 w, 64 w + 64), lane (r, g) of a 16 x 16 tile row / column r and the
// 16 contiguous k at 64 w + 16 g (4 float4 per operand tile; Weff is laid out [jp][k] for
// that, env_w2_kernel).  The four per-wave partial tiles are summed in a fixed order at the
// assembly (bitwise repeatable), in LDS that the special rows free once their 14 leaf
// contractions per orbital are done.
template <int N>
__global__ __launch_bounds__(256) void env_phi_kernel(const float* __restrict__ h, const float* __restrict__ Weff,
                                                     const float* __restrict__ FS, int ldF,
                                                     const float* __restrict__ x, const float* __restrict__ geo_g,
                                                     const float* __restrict__ norm, float* __restrict__ PhiC, int M) {
  constexpr int T = 2 * N, C = 2 * N + 5, J2 = 2 * N, JP = 48, NE = 14;
  constexpr int TR = (C + 15) / 16, TC = (J2 + 15) / 16;
  static_assert(TR <= 3 && TC <= 3, "tile sizes");
  extern __shared__ float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int e = blockIdx.x, b = e / N, i = e - (e / N) * N, M1 = M + 1, MN = M * N, RW = 2 * MN;
  float* fsl = sm;                                  // [6][RW] the special rows; later [4][48][JP] partials
  cf* wt = reinterpret_cast<cf*>(sm + (6 * RW > 4 * 48 * JP ? 6 * RW : 4 * 48 * JP));  // [10][M + 1]
  cf* ext = wt + 10 * M1;                           // [NE][N]
  // ---- the load burst: the special rows by LDS-DMA (global_load_lds_dwordx4, 1-KiB pieces,
  // no VGPRs), then the MFMA operands into registers
  {
    const int RB = RW * 4, PR = (RB + 1023) / 1024;  // bytes / pieces per row
    const uint32_t base = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)fsl);
    for (int q = wv; q < 6 * PR; q += 4) {
      const int r = q / PR, piece = q - (q / PR) * PR, byte = piece * 1024 + lane * 16;
      const char* src = reinterpret_cast<const char*>(FS + ((size_t)e * 6 + r) * ldF) + byte;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(base + (uint32_t)(r * RB + piece * 1024));
      if (byte < RB) {
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(dst)
                     : "memory");
      }
    }
  }
  const int r16 = lane & 15, kq = lane >> 4, k0 = 64 * wv + 16 * kq;
  float4 av[TR][4], bv[TC][4];
#pragma unroll
  for (int t = 0; t < TR; ++t) {
    const int row = 16 * t + r16;
    const float* ap = h + ((size_t)e * C + (row < C ? row : 0)) * 256 + k0;
#pragma unroll
    for (int q = 0; q < 4; ++q) av[t][q] = *reinterpret_cast<const float4*>(ap + 4 * q);
  }
#pragma unroll
  for (int t = 0; t < TC; ++t) {
    const int col = 16 * t + r16;
    const float* bp = Weff + ((size_t)e * J2 + (col < J2 ? col : 0)) * 256 + k0;
#pragma unroll
    for (int q = 0; q < 4; ++q) bv[t][q] = *reinterpret_cast<const float4*>(bp + 4 * q);
  }
  // ---- the leaves while the loads are in flight
  {
    const float4 g4 = *reinterpret_cast<const float4*>(geo_g + 4 * (size_t)e);
    const float th = x[2 * (size_t)e], ph = x[2 * (size_t)e + 1];
    const float st = g4.x, ct = g4.y, sp = g4.z, cp = g4.w;
    const float gauge = env_gauge(ct, M);
    const float phh[3] = {-sp, cp, 0.f};
    const float thh[3] = {ct * cp, ct * sp, -st};
    for (int p = tid; p < M; p += 256) {
      const EnvLeaf L = env_leaf(th, ph, p, M, norm[p], true, gauge, DET_LEAF_SQ);
      wt[p] = L.e0;
      wt[M1 + p] = L.dth;
      wt[2 * M1 + p] = L.dph;
      wt[3 * M1 + p] = L.lb;
      const float mf = (float)p - 0.5f * (float)(M - 1) - gauge;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        wt[(4 + k) * M1 + p] = cf{phh[k] * L.dth.re - thh[k] * L.dph.re, phh[k] * L.dth.im - thh[k] * L.dph.im};
        wt[(7 + k) * M1 + p] = env_flow2(L.e0, L.dth, L.d2th, mf, st, ct, sp, cp, k);
      }
    }
  }
  // ---- the partial h_c . Weff tiles of this wave's k range
  f4e acc[TR][TC];
#pragma unroll
  for (int t = 0; t < TR; ++t)
#pragma unroll
    for (int c = 0; c < TC; ++c) {
      acc[t][c] = f4e{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t][q].x, bv[c][q].x, acc[t][c], 0, 0, 0);
        acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t][q].y, bv[c][q].y, acc[t][c], 0, 0, 0);
        acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t][q].z, bv[c][q].z, acc[t][c], 0, 0, 0);
        acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t][q].w, bv[c][q].w, acc[t][c], 0, 0, 0);
      }
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA pieces
  __syncthreads();
  // ---- the special rows' leaf contractions (row s of fsl: 0 value, 1 / 2 own tangents 2 i /
  // 2 i + 1, 3..5 the flow rows): sums over the M harmonics
  for (int q = tid; q < NE * N; q += 256) {
    const int s = q / N, j = q - (q / N) * N;
    // (row, leaf) of sum s: E0 DTH DPH LB SF0 SF1 SF2 of the value row; E0, DTH of own 2 i;
    // E0, DPH of own 2 i + 1; W0, W1, W2 of the flow rows
    const int row = s < 7 ? 0 : (s < 9 ? 1 : (s < 11 ? 2 : s - 8));
    const int leaf = s == 0 ? 0 : (s < 4 ? s : (s < 7 ? s + 3 : (s == 7 ? 0 : (s == 8 ? 1 : (s == 9 ? 0 : (s == 10 ? 2 : s - 7))))));
    const float* r = fsl + row * RW + j;
    const cf* wl = wt + leaf * M1;
    cf a0{0.f, 0.f}, a1{0.f, 0.f};
    int m = 0;
    for (; m + 1 < M; m += 2) {
      cfma(a0, cf{r[m * N], r[MN + m * N]}, wl[m]);
      cfma(a1, cf{r[(m + 1) * N], r[MN + (m + 1) * N]}, wl[m + 1]);
    }
    if (m < M) cfma(a0, cf{r[m * N], r[MN + m * N]}, wl[m]);
    ext[s * N + j] = a0 + a1;
  }
  __syncthreads();
  float* part = fsl;  // [4][48][JP]
#pragma unroll
  for (int t = 0; t < TR; ++t)
#pragma unroll
    for (int c = 0; c < TC; ++c)
#pragma unroll
      for (int v = 0; v < 4; ++v) part[(wv * 48 + 16 * t + 4 * kq + v) * JP + 16 * c + r16] = acc[t][c][v];
  __syncthreads();
  // ---- assembly (env_stream_kernel's): PhiC[b][0][c][i][j]
  for (int q = tid; q < C * N; q += 256) {
    const int c = q / N, j = q - (q / N) * N;
    cf r{0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      r.re += part[(w * 48 + c) * JP + 2 * j];
      r.im += part[(w * 48 + c) * JP + 2 * j + 1];
    }
    cf v;
    if (c == 0) {
      v = ext[j];
    } else if (c <= T) {
      const int t = c - 1;
      if ((t >> 1) == i)
        v = (t & 1) ? ext[9 * N + j] + ext[2 * N + j] : ext[7 * N + j] + ext[1 * N + j];
      else
        v = r;
    } else if (c == T + 1) {
      v = r + ext[3 * N + j] + 2.f * (ext[8 * N + j] + ext[10 * N + j]);
    } else {
      const int k = c - T - 2;
      v = r + ext[(4 + k) * N + j] + 2.f * ext[(11 + k) * N + j];
    }
    float* o = PhiC + 2 * (((size_t)b * C + c) * N * N + (size_t)i * N + j);
    o[0] = v.re;
    o[1] = v.im;
  }
}

}  // namespace

size_t env_phi_smem_bytes(const Dims& d) {
  return (size_t)std::max(6 * 2 * d.M * d.N, 4 * 48 * 48) * sizeof(float) +
         (size_t)(10 * (d.M + 1) + 14 * d.N) * sizeof(cf);
}

void launch_env_first(const Dims& d, const float* h, const float* geo, const float* x, const float* norm,
                      const float* WorbT, const float* borb, const uint16_t* WorbP, const float* W2T,
                      const uint16_t* W2P, bool x6, int nw, float* S, float* FS, float* E2, float* Weff, float* phic,
                      hipStream_t s) {
  const int ne = nw * d.N, KE = env_first_k(d), J2 = 2 * d.N;
  if (d.N == 10)
    hipLaunchKernelGGL(srows_kernel<10>, dim3(ne), dim3(256), 0, s, h, geo, S);
  else  // env_first: N = 10 or 20
    hipLaunchKernelGGL(srows_kernel<20>, dim3(ne), dim3(256), 0, s, h, geo, S);
  hipLaunchKernelGGL(env_coef_kernel, dim3((ne * KE + 255) / 256), dim3(256), 0, s, x, geo, norm, E2, ne, d.M, KE);
  if (x6) {  // split-bf16 (the default); exact-f32 NT GEMMs in DH_GEMM_F32
    launch_gemm_x6(S, 256, WorbP, x6_plane_rows(d.orb_cols), borb, nullptr, 0, FS, d.ld_orb, 6 * ne, d.orb_cols, 256,
                   6, s);
    launch_gemm_x6(E2, KE, W2P, x6_plane_rows(256 * J2), nullptr, nullptr, 0, Weff, 256 * J2, ne, 256 * J2, KE, 1, s);
  } else {
    launch_gemm_nt(S, 256, WorbT, 256, borb, nullptr, 0, FS, d.ld_orb, 6 * ne, d.orb_cols, 256, 6, s);
    launch_gemm_nt(E2, KE, W2T, KE, nullptr, nullptr, 0, Weff, 256 * J2, ne, 256 * J2, KE, 1, s);
  }
  const size_t smem = env_phi_smem_bytes(d);
  auto go = [&](auto kern) {
    ensure_smem(kern, smem);
    hipLaunchKernelGGL(kern, dim3(ne), dim3(256), smem, s, h, Weff, FS, d.ld_orb, x, geo, norm, phic, d.M);
  };
  switch (d.N) {
    case 10: go(env_phi_kernel<10>); break;
    default: go(env_phi_kernel<20>); break;  // env_first: N = 10 or 20
  }
}

void launch_env_w2(const Dims& d, const float* Worb, float* W2T, hipStream_t s) {
  const int n = 256 * 2 * d.N * env_first_k(d);
  hipLaunchKernelGGL(env_w2_kernel, dim3((n + 255) / 256), dim3(256), 0, s, Worb, d.ld_orb, d.M, d.N, 256,
                     env_first_k(d), W2T);
}

void launch_det_energy_pc(const Dims& d, const float* x, const float* geo, const float* jastrow, const float* norm,
                          float* e_l, float* obs, int nw, hipStream_t s, const float* phic) {
  const DetSmem L = det_layout(d.N, d.M, d.K, 4, true);
  const size_t bytes = (size_t)L.total * sizeof(float);
  ensure_smem(det_energy_kernel<0, true>, bytes);
  hipLaunchKernelGGL((det_energy_kernel<0, true>), dim3(nw), dim3(256), bytes, s, nullptr, d.ld_orb, x, geo, jastrow,
                     norm, e_l, obs, d.N, d.n_up, d.M, d.K, d.Q, d.r, d.lambda, d.interaction, phic);
}

}  // namespace dh
