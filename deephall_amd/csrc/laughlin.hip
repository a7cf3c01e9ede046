// Laughlin wavefunction (deephall/networks/laughlin.py:19-100) and its local energy.
//
//   psi = det[ u_i^(Q1+m_j) v_i^(Q1-m_j) ] * prod_{i != j} (u_i v_j - u_j v_i)
//   u = cos(theta/2) e^(i phi/2),  v = sin(theta/2) e^(-i phi/2),  Q1 = Q - p (N - 1)
//
// ground state (N = 2 Q1 + 1, m = -Q1..Q1) and quasihole (N = 2 Q1, m = -Q1..Q1 without
// -excitation_lz; laughlin.py:36-41, 66-77).  The per-row Jastrow factor J_i of
// laughlin.py:62-63 (diagonal element 1) is the product over ordered pairs, so
//   log psi = log det E + sum_{i<j} 2 log w_ij  (+ i pi per pair: the phase of -1),
// and every derivative is analytic: the determinant part through E^-1 (its first
// derivatives tr(E^-1 dE) and second derivatives tr(E^-1 d2E) - tr(E^-1 dE E^-1 dE),
// each dE row-sparse), the pair part term by term.  The FULL complex Hessian of log psi is
// formed in double and fed to the reference's kinetic / angular-momentum formulas
// (hamiltonian.py:115-169) — the same algorithm as the reference, without autodiff.
// One 64-thread workgroup per walker, everything in LDS, double precision throughout.
#include "dh_internal.h"
#include "device_common.h"

namespace dh {
namespace {

struct zd {
  double re, im;
};
__device__ __forceinline__ zd operator+(zd a, zd b) { return zd{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ zd operator-(zd a, zd b) { return zd{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ zd operator*(zd a, zd b) { return zd{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
__device__ __forceinline__ zd operator*(double s, zd a) { return zd{s * a.re, s * a.im}; }
__device__ __forceinline__ zd zdiv(zd a, zd b) {
  const double d = b.re * b.re + b.im * b.im;
  return zd{(a.re * b.re + a.im * b.im) / d, (a.im * b.re - a.re * b.im) / d};
}
__device__ __forceinline__ zd zpow(zd b, int e) {  // e >= 0
  zd r{1.0, 0.0};
  for (int k = 0; k < e; ++k) r = r * b;
  return r;
}

// LDS layout (complex doubles unless noted)
struct LSm {
  int uv, E, dE, d2E, Einv, R, g, H, misc, total;  // offsets in zd units
};
__host__ __device__ inline LSm lsm_layout(int N) {
  LSm L;
  int o = 0;
  L.uv = o;  // per electron: u, v, du[2], dv[2], d2u[3], d2v[3] = 12
  o += 12 * N;
  L.E = o;
  o += 2 * N * N;  // augmented [E | I] -> [I | E^-1]
  L.dE = o;
  o += 2 * N * N;  // [coord theta/phi][i][j] (row i only: own electron)
  L.d2E = o;
  o += 3 * N * N;  // [tt, tp, pp][i][j]
  L.Einv = o;
  o += N * N;
  L.R = o;
  o += 2 * N * N;  // R[a][i] = sum_q dE[a][e_a][q] Einv[q][i]
  L.g = o;
  o += 2 * N;
  L.H = o;
  o += 4 * N * N;
  L.misc = o;
  o += N + 4;  // pivot factors, log det
  L.total = o;
  return L;
}

// the seven u / v derivative quantities of electron (th, ph)
__device__ void uv_derivs(double th, double ph, zd* q) {
  double sh, ch, sp, cp;
  sincos(0.5 * th, &sh, &ch);
  sincos(0.5 * ph, &sp, &cp);
  const zd eu{cp, sp}, ev{cp, -sp};  // e^(i phi/2), e^(-i phi/2)
  const zd u = ch * eu, v = sh * ev;
  const zd I{0.0, 1.0};
  q[0] = u;
  q[1] = v;
  q[2] = -0.5 * sh * eu;              // du/dth
  q[3] = 0.5 * (I * u);               // du/dph
  q[4] = 0.5 * ch * ev;               // dv/dth
  q[5] = -0.5 * (I * v);              // dv/dph
  q[6] = -0.25 * u;                   // d2u/dth2
  q[7] = 0.5 * (I * q[2]);            // d2u/dth dph
  q[8] = -0.25 * u;                   // d2u/dph2
  q[9] = -0.25 * v;                   // d2v/dth2
  q[10] = -0.5 * (I * q[4]);          // d2v/dth dph
  q[11] = -0.25 * v;                  // d2v/dph2
}

// d/dx and d2/dxdy of u^a v^b (x, y in {th, ph}; xy index 0 tt, 1 tp, 2 pp)
__device__ void monomial(const zd* q, int a, int b, zd* val, zd* d1, zd* d2) {
  const zd u = q[0], v = q[1];
  const zd ua = zpow(u, a), vb = zpow(v, b);
  const zd ua1 = a >= 1 ? zpow(u, a - 1) : zd{0, 0}, vb1 = b >= 1 ? zpow(v, b - 1) : zd{0, 0};
  const zd ua2 = a >= 2 ? zpow(u, a - 2) : zd{0, 0}, vb2 = b >= 2 ? zpow(v, b - 2) : zd{0, 0};
  *val = ua * vb;
  const zd du[2] = {q[2], q[3]}, dv[2] = {q[4], q[5]};
  for (int x = 0; x < 2; ++x) d1[x] = (double)a * (ua1 * vb * du[x]) + (double)b * (ua * vb1 * dv[x]);
  const int xs[3] = {0, 0, 1}, ys[3] = {0, 1, 1};
  for (int k = 0; k < 3; ++k) {
    const int x = xs[k], y = ys[k];
    const zd d2u = q[6 + k], d2v = q[9 + k];
    d2[k] = (double)(a * (a - 1)) * (ua2 * vb * du[x] * du[y]) + (double)a * (ua1 * vb * d2u) +
            (double)(a * b) * (ua1 * vb1 * (du[x] * dv[y] + du[y] * dv[x])) + (double)(b * (b - 1)) * (ua * vb2 * dv[x] * dv[y]) +
            (double)b * (ua * vb1 * d2v);
  }
}

template <bool ENERGY>
__global__ __launch_bounds__(64) void laughlin_kernel(const float* __restrict__ x, const int* __restrict__ expo,
                                                      float* __restrict__ out_lp, float* __restrict__ e_l,
                                                      float* __restrict__ obs, int N, double Q, double radius,
                                                      double lambda, int interaction) {
  extern __shared__ double smd[];
  zd* sm = reinterpret_cast<zd*>(smd);
  const LSm L = lsm_layout(N);
  zd *UV = sm + L.uv, *E = sm + L.E, *dE = sm + L.dE, *d2E = sm + L.d2E, *Einv = sm + L.Einv, *R = sm + L.R;
  zd *g = sm + L.g, *H = sm + L.H, *fac = sm + L.misc;
  __shared__ int piv;
  __shared__ zd logdet;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int NN = N * N, T = 2 * N;
  for (int i = tid; i < N; i += nt) uv_derivs((double)x[2 * (b * N + i)], (double)x[2 * (b * N + i) + 1], UV + 12 * i);
  __syncthreads();
  // E (augmented with I) and its coordinate derivatives (row i depends on electron i only)
  for (int idx = tid; idx < NN; idx += nt) {
    const int i = idx / N, j = idx % N;
    zd val, d1[2], d2[3];
    monomial(UV + 12 * i, expo[j], expo[N + j], &val, d1, d2);
    E[i * 2 * N + j] = val;
    E[i * 2 * N + N + j] = zd{i == j ? 1.0 : 0.0, 0.0};
    dE[idx] = d1[0];
    dE[NN + idx] = d1[1];
    for (int k = 0; k < 3; ++k) d2E[k * NN + idx] = d2[k];
  }
  if (tid == 0) logdet = zd{0.0, 0.0};
  __syncthreads();
  // Gauss-Jordan with partial pivoting on [E | I] (|re| + |im| pivot, as det.hip)
  const int ld = 2 * N;
  for (int p = 0; p < N; ++p) {
    if (tid == 0) {
      double best = -1.0;
      int bi = p;
      for (int r = p; r < N; ++r) {
        const double v = fabs(E[r * ld + p].re) + fabs(E[r * ld + p].im);
        if (v > best) {
          best = v;
          bi = r;
        }
      }
      piv = bi;
    }
    __syncthreads();
    const int pr = piv;
    if (pr != p)
      for (int c = tid; c < ld; c += nt) {
        const zd t = E[p * ld + c];
        E[p * ld + c] = E[pr * ld + c];
        E[pr * ld + c] = t;
      }
    __syncthreads();
    const zd P = E[p * ld + p];
    if (tid == 0) {
      logdet.re += 0.5 * log(P.re * P.re + P.im * P.im);
      logdet.im += atan2(P.im, P.re) + (pr != p ? M_PI : 0.0);
    }
    const zd Pinv = zdiv(zd{1.0, 0.0}, P);
    __syncthreads();
    for (int r = tid; r < N; r += nt) fac[r] = (r == p) ? zd{0.0, 0.0} : E[r * ld + p];
    for (int c = tid; c < ld; c += nt) E[p * ld + c] = E[p * ld + c] * Pinv;
    __syncthreads();
    for (int idx = tid; idx < N * ld; idx += nt) {
      const int r = idx / ld, c = idx % ld;
      if (r == p) continue;
      E[r * ld + c] = E[r * ld + c] - fac[r] * E[p * ld + c];
    }
    __syncthreads();
  }
  for (int idx = tid; idx < NN; idx += nt) Einv[idx] = E[(idx / N) * ld + N + idx % N];
  __syncthreads();
  // pair part of log psi (value): sum_{i<j} 2 log w_ij (+ i pi each: w_ji = -w_ij)
  double lre = 0.0, lim = 0.0;
  for (int q = tid; q < NN; q += nt) {
    const int i = q / N, j = q % N;
    if (j <= i) continue;
    const zd w = UV[12 * i] * UV[12 * j + 1] - UV[12 * j] * UV[12 * i + 1];
    lre += log(w.re * w.re + w.im * w.im);  // 2 log|w|
    lim += 2.0 * atan2(w.im, w.re) + M_PI;
  }
  for (int o = 32; o > 0; o >>= 1) {
    lre += __shfl_xor(lre, o, 64);
    lim += __shfl_xor(lim, o, 64);
  }
  if (!ENERGY) {
    if (tid == 0) {
      out_lp[2 * b] = (float)(logdet.re + lre);
      out_lp[2 * b + 1] = (float)remainder(logdet.im + lim, 2.0 * M_PI);
    }
    return;
  }
  // R[a][i] = sum_q dE[a][e_a][q] Einv[q][i],  a = 2 e + (0 theta | 1 phi)
  for (int idx = tid; idx < T * N; idx += nt) {
    const int a = idx / N, i = idx % N, e = a >> 1, c = a & 1;
    zd s{0.0, 0.0};
    for (int q = 0; q < N; ++q) s = s + dE[c * NN + e * N + q] * Einv[q * N + i];
    R[idx] = s;
  }
  __syncthreads();
  // gradient: determinant + pairs
  for (int a = tid; a < T; a += nt) {
    const int e = a >> 1, c = a & 1;
    zd s = R[a * N + e];
    const zd* qe = UV + 12 * e;
    for (int j = 0; j < N; ++j) {
      if (j == e) continue;
      const zd* qj = UV + 12 * j;
      const zd w = qe[0] * qj[1] - qj[0] * qe[1];
      const zd dw = qe[2 + c] * qj[1] - qj[0] * qe[4 + c];
      s = s + 2.0 * zdiv(dw, w);
    }
    g[a] = s;
  }
  // Hessian
  for (int idx = tid; idx < T * T; idx += nt) {
    const int a = idx / T, bb = idx % T, ea = a >> 1, ca = a & 1, eb = bb >> 1, cb = bb & 1;
    zd h = zd{0.0, 0.0} - R[bb * N + ea] * R[a * N + eb];
    const zd* qa = UV + 12 * ea;
    if (ea == eb) {
      const int k = ca + cb;  // 0 tt, 1 tp, 2 pp
      zd s{0.0, 0.0};
      for (int j = 0; j < N; ++j) s = s + Einv[j * N + ea] * d2E[k * NN + ea * N + j];
      h = h + s;
      for (int j = 0; j < N; ++j) {
        if (j == ea) continue;
        const zd* qj = UV + 12 * j;
        const zd w = qa[0] * qj[1] - qj[0] * qa[1];
        const zd dx = qa[2 + ca] * qj[1] - qj[0] * qa[4 + ca];
        const zd dy = qa[2 + cb] * qj[1] - qj[0] * qa[4 + cb];
        const zd dxy = qa[6 + k] * qj[1] - qj[0] * qa[9 + k];
        const zd fw = zdiv(dx, w), gw = zdiv(dy, w);
        h = h + 2.0 * (zdiv(dxy, w) - fw * gw);
      }
    } else {
      const zd* qb = UV + 12 * eb;
      const zd w = qa[0] * qb[1] - qb[0] * qa[1];
      const zd dx = qa[2 + ca] * qb[1] - qb[0] * qa[4 + ca];  // d/dx_a
      const zd dy = qa[0] * qb[4 + cb] - qb[2 + cb] * qa[1];  // d/dy_b
      const zd dxy = qa[2 + ca] * qb[4 + cb] - qb[2 + cb] * qa[4 + ca];
      h = h + 2.0 * (zdiv(dxy, w) - zdiv(dx, w) * zdiv(dy, w));
    }
    H[idx] = h;
  }
  __syncthreads();
  // hamiltonian.py:115-169 with g and the full Hessian; potential (double geometry)
  double v[4] = {0.0, 0.0, 0.0, 0.0};  // KE re, KE im, L2 re, PE
  double lz = 0.0, lz2 = 0.0;
  // per electron terms (one thread per electron i), pair terms over (i, j)
  for (int idx = tid; idx < NN; idx += nt) {
    const int i = idx / N, j = idx % N;
    double sti, cti, spi, cpi, stj, ctj, spj, cpj;
    sincos((double)x[2 * (b * N + i)], &sti, &cti);
    sincos((double)x[2 * (b * N + i) + 1], &spi, &cpi);
    sincos((double)x[2 * (b * N + j)], &stj, &ctj);
    sincos((double)x[2 * (b * N + j) + 1], &spj, &cpj);
    const zd gti = g[2 * i], gpi = g[2 * i + 1], gtj = g[2 * j], gpj = g[2 * j + 1];
    const zd htt = H[(2 * i) * T + 2 * j] + gti * gtj, htp = H[(2 * i) * T + 2 * j + 1] + gti * gpj;
    const zd hpp = H[(2 * i + 1) * T + 2 * j + 1] + gpi * gpj;
    const double phi_i[3] = {-spi, cpi, 0.0}, phi_j[3] = {-spj, cpj, 0.0};
    const double thp_i[3] = {cpi * cti / sti, spi * cti / sti, -1.0}, thp_j[3] = {cpj * ctj / stj, spj * ctj / stj, -1.0};
    const double rj[3] = {stj * cpj, stj * spj, ctj}, ri[3] = {sti * cpi, sti * spi, cti};
    double pp = 0.0, ptp = 0.0, tt = 0.0, mi_mj = 0.0, mj_phi = 0.0, mj_thp = 0.0;
    for (int k = 0; k < 3; ++k) {
      const double mj = Q * (thp_j[k] * ctj + rj[k]), mi = Q * (thp_i[k] * cti + ri[k]);
      pp += phi_i[k] * phi_j[k];
      ptp += phi_i[k] * thp_j[k];
      tt += thp_i[k] * thp_j[k];
      mi_mj += mi * mj;
      mj_phi += mj * phi_i[k];
      mj_thp += mj * thp_i[k];
    }
    // 2 phi_i.thp_j P_tp - phi_i.phi_j P_tt - thp_i.thp_j P_pp - 2i m_j.(phi_i g_t_i - thp_i g_p_i) + m_i.m_j
    zd term = 2.0 * ptp * htp - pp * htt - tt * hpp + zd{mi_mj, 0.0};
    const zd cross = mj_phi * gti - mj_thp * gpi;
    term = term - zd{-2.0 * cross.im, 2.0 * cross.re};  // - 2i * cross
    v[2] += term.re;
    lz2 -= hpp.re;
    if (i == j) {
      const double cot = cti / sti, s2 = sti * sti;
      // square_grad, grad_grad (Laplacian), magnetic (hamiltonian.py:115-133)
      const zd sq = gti * gti + (1.0 / s2) * (gpi * gpi);
      const zd lap = cot * gti + H[(2 * i) * T + 2 * i] + (1.0 / s2) * H[(2 * i + 1) * T + 2 * i + 1];
      const zd mag = zd{(Q * cot) * (Q * cot), 0.0} + zd{0.0, 2.0 * Q * cti / s2} * gpi;
      const zd ke = zd{0.0, 0.0} - lap - sq + mag;
      v[0] += ke.re;
      v[1] += ke.im;
      v[2] -= gti.re * cot;  // - sum g_theta cot theta (real part)
      lz += gpi.im;
      {
        double pe = 0.0;
        for (int jj = i + 1; jj < N; ++jj) {
          double a1, a2, a3, a4;
          sincos((double)x[2 * (b * N + jj)], &a1, &a2);
          sincos((double)x[2 * (b * N + jj) + 1], &a3, &a4);
          const double u = ri[0] * a1 * a4 + ri[1] * a1 * a3 + ri[2] * a2;
          pe += interaction == DH_INTERACTION_COULOMB ? 1.0 / sqrt(2.0 - 2.0 * u) : 1.0 + (Q + 1.0) / Q * u;
        }
        v[3] += pe;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    for (int q = 0; q < 4; ++q) v[q] += __shfl_xor(v[q], o, 64);
    lz += __shfl_xor(lz, o, 64);
    lz2 += __shfl_xor(lz2, o, 64);
  }
  if (tid == 0) {
    const double r2 = radius * radius;
    double pe = v[3];
    if (interaction == DH_INTERACTION_COULOMB) pe /= radius;
    pe *= lambda;
    const double ke_re = v[0] / (2.0 * r2), ke_im = v[1] / (2.0 * r2);
    e_l[2 * b] = (float)(ke_re + pe);
    e_l[2 * b + 1] = (float)ke_im;
    float* ob = obs + 8 * (size_t)b;
    ob[0] = (float)ke_re;
    ob[1] = (float)ke_im;
    ob[2] = (float)pe;
    ob[3] = (float)lz;
    ob[4] = (float)lz2;
    ob[5] = (float)v[2];
    ob[6] = (float)(logdet.re + lre);
    ob[7] = (float)remainder(logdet.im + lim, 2.0 * M_PI);
  }
}

}  // namespace

size_t laughlin_smem_bytes(int N) { return (size_t)lsm_layout(N).total * 2 * sizeof(double); }

void launch_laughlin(const Dims& d, const float* x, const int* expo, float* logpsi, float* e_l, float* obs, int nw,
                     hipStream_t s) {
  const size_t bytes = laughlin_smem_bytes(d.N);
  if (e_l) {
    ensure_smem(laughlin_kernel<true>, bytes);
    hipLaunchKernelGGL(laughlin_kernel<true>, dim3(nw), dim3(64), bytes, s, x, expo, logpsi, e_l, obs, d.N,
                       (double)d.Q, (double)d.r, (double)d.lambda, d.interaction);
  } else {
    ensure_smem(laughlin_kernel<false>, bytes);
    hipLaunchKernelGGL(laughlin_kernel<false>, dim3(nw), dim3(64), bytes, s, x, expo, logpsi, e_l, obs, d.N,
                       (double)d.Q, (double)d.r, (double)d.lambda, d.interaction);
  }
}

}  // namespace dh
