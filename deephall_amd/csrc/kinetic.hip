// Local kinetic energy and angular momenta of an ARBITRARY log psi from its derivatives
// (hamiltonian.py:83-172, the reference's make_local_kinetic_energy(f, Q, r) for any f).
//
// The caller differentiates its own callable (first derivatives g[N][2] and the full
// Hessian H[N][2][N][2] of log psi in (theta, phi), complex); this kernel assembles
//   KE   = (-grad_grad - square_grad + magnetic) / 2 r^2                 (lines 109-133)
//   L^2  = sum_ij [2 phi_i.theta'_j h_tp - phi_i.phi_j h_tt - theta'_i.theta'_j h_pp]
//          - 2i M.V + M.M - sum_i g_theta_i / tan theta_i                 (lines 139-159)
//   Lz   = Im sum_i g_phi_i,   Lz^2 = -Re sum_ij h_pp                      (lines 165-168)
// with h_ab = H_ab + g_a g_b, M = sum_j m_j (m = Q (theta' cos theta + r_hat), real) and
// V = sum_i (phi_i g_theta_i - theta'_i g_phi_i): the reference's i x j sums of
// m_j (x) v_i and m_i (x) m_j factor into these two 3-vectors.
//
// One wave per walker, everything in double: lanes stage the per-electron terms in LDS,
// then stride over the N^2 (i, j) pairs reading three complex Hessian entries each, and
// the partial sums meet in a wave reduction.  HBM-bound on the Hessian (64 N^2 bytes per
// walker); the generic path's cost is in the caller's differentiation, not here.
#include "dh_internal.h"
#include "device_common.h"

namespace dh {
namespace {

constexpr int kWalkersPerBlock = 4;
constexpr int kElecTerms = 8;  // phi_hat x, y; theta' x, y (z = -1); g_theta re, im; g_phi re, im

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(64 * kWalkersPerBlock) void kinetic_assembly_kernel(
    const double* __restrict__ x, const double* __restrict__ g, const double* __restrict__ H, int nw, int N, double Q,
    double r, float* __restrict__ ke, float* __restrict__ mom) {
  extern __shared__ double sm[];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int b = blockIdx.x * kWalkersPerBlock + wave;
  if (b >= nw) return;  // whole waves exit; no block barrier below
  double* e = sm + (size_t)wave * N * kElecTerms;
  const double* xb = x + (size_t)b * N * 2;
  const double* gb = g + (size_t)b * N * 4;  // [i][a][re, im]
  const size_t n2 = 2 * (size_t)N;
  const double* Hb = H + (size_t)b * n2 * n2 * 2;  // [i][a][j][c][re, im]

  // per-electron terms (lanes over i)
  // (only Re L^2 is an output, and M is real, so V enters through its imaginary part)
  double ks_re = 0, ks_im = 0, l2 = 0, lz = 0;
  double Mx = 0, My = 0, Vx = 0, Vy = 0, Vz = 0;  // M_z = Q (-cos + cos) = 0
  for (int i = lane; i < N; i += 64) {
    double st, ct, sp, cp;
    sincos(xb[2 * i], &st, &ct);
    sincos(xb[2 * i + 1], &sp, &cp);
    const double cot = ct / st, s2 = st * st;
    const double gt_re = gb[4 * i], gt_im = gb[4 * i + 1], gp_re = gb[4 * i + 2], gp_im = gb[4 * i + 3];
    const double* Hi = Hb + (size_t)(2 * i) * n2 * 2;
    const double htt_re = Hi[(2 * i) * 2], htt_im = Hi[(2 * i) * 2 + 1];
    const double hpp_re = Hi[n2 * 2 + (2 * i + 1) * 2], hpp_im = Hi[n2 * 2 + (2 * i + 1) * 2 + 1];
    // -grad_grad - square_grad + magnetic (hamiltonian.py:110, 121-132), electron i
    const double sq_re = gt_re * gt_re - gt_im * gt_im + (gp_re * gp_re - gp_im * gp_im) / s2;
    const double sq_im = 2 * gt_re * gt_im + 2 * gp_re * gp_im / s2;
    const double gg_re = gt_re * cot + htt_re + hpp_re / s2, gg_im = gt_im * cot + htt_im + hpp_im / s2;
    const double qc = Q * cot;
    const double mg_re = qc * qc - 2 * Q * ct / s2 * gp_im, mg_im = 2 * Q * ct / s2 * gp_re;
    ks_re += -gg_re - sq_re + mg_re;
    ks_im += -gg_im - sq_im + mg_im;
    // L^2 diagonal extra term and Lz
    l2 -= gt_re * cot;
    lz += gp_im;
    // M, V (theta' = (cos phi cot, sin phi cot, -1), phi_hat = (-sin phi, cos phi, 0))
    const double tx = cp * cot, ty = sp * cot;
    Mx += Q * (tx * ct + st * cp);
    My += Q * (ty * ct + st * sp);
    Vx += -sp * gt_im - tx * gp_im;
    Vy += cp * gt_im - ty * gp_im;
    Vz += gp_im;  // -(theta'_z = -1) g_phi
    double* ei = e + (size_t)i * kElecTerms;
    ei[0] = -sp;
    ei[1] = cp;
    ei[2] = tx;
    ei[3] = ty;
    ei[4] = gt_re;
    ei[5] = gt_im;
    ei[6] = gp_re;
    ei[7] = gp_im;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // pair terms (lanes over (i, j))
  double lz2 = 0;
  for (int p = lane; p < N * N; p += 64) {
    const int i = p / N, j = p - i * N;
    const double* ei = e + (size_t)i * kElecTerms;
    const double* ej = e + (size_t)j * kElecTerms;
    const double* Hi0 = Hb + (size_t)(2 * i) * n2 * 2;  // row (i, theta)
    const double* Hi1 = Hi0 + n2 * 2;                   // row (i, phi)
    const double Htt_re = Hi0[(2 * j) * 2], Htp_re = Hi0[(2 * j + 1) * 2], Hpp_re = Hi1[(2 * j + 1) * 2];
    const double gti_re = ei[4], gti_im = ei[5], gpi_re = ei[6], gpi_im = ei[7];
    const double gtj_re = ej[4], gtj_im = ej[5], gpj_re = ej[6], gpj_im = ej[7];
    const double tt_re = Htt_re + gti_re * gtj_re - gti_im * gtj_im;
    const double tp_re = Htp_re + gti_re * gpj_re - gti_im * gpj_im;
    const double pp_re = Hpp_re + gpi_re * gpj_re - gpi_im * gpj_im;
    const double ph_th = ei[0] * ej[2] + ei[1] * ej[3];      // phi_i . theta'_j
    const double ph_ph = ei[0] * ej[0] + ei[1] * ej[1];      // phi_i . phi_j
    const double th_th = ei[2] * ej[2] + ei[3] * ej[3] + 1;  // theta'_i . theta'_j
    l2 += 2 * ph_th * tp_re - ph_ph * tt_re - th_th * pp_re;
    lz2 -= pp_re;
  }

  ks_re = wave_sum(ks_re);
  ks_im = wave_sum(ks_im);
  l2 = wave_sum(l2);
  lz = wave_sum(lz);
  lz2 = wave_sum(lz2);
  Mx = wave_sum(Mx);
  My = wave_sum(My);
  Vx = wave_sum(Vx);
  Vy = wave_sum(Vy);
  Vz = wave_sum(Vz);
  if (lane == 0) {
    // Re(-2i M.V + M.M) = 2 M.Im V + |M|^2 (M real)
    const double l2t = l2 + 2 * (Mx * Vx + My * Vy) + Mx * Mx + My * My;
    const double s = 0.5 / (r * r);
    ke[2 * (size_t)b] = (float)(ks_re * s);
    ke[2 * (size_t)b + 1] = (float)(ks_im * s);
    mom[3 * (size_t)b] = (float)lz;
    mom[3 * (size_t)b + 1] = (float)lz2;
    mom[3 * (size_t)b + 2] = (float)l2t;
  }
}

}  // namespace

size_t kinetic_assembly_lds_bytes(int N) { return (size_t)kWalkersPerBlock * N * kElecTerms * sizeof(double); }

void launch_kinetic_assembly(const double* x, const double* g, const double* H, int nw, int N, double Q, double r,
                             float* ke, float* mom, hipStream_t s) {
  hipLaunchKernelGGL(kinetic_assembly_kernel, dim3((nw + kWalkersPerBlock - 1) / kWalkersPerBlock),
                     dim3(64 * kWalkersPerBlock), kinetic_assembly_lds_bytes(N), s, x, g, H, nw, N, Q, r, ke, mom);
}

}  // namespace dh
