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
//
// Quasiparticle (N = 2 Q1 + 2, laughlin.py:82-100; expo[2N] = 1): columns 0..N-2 are the
// monomials of m = -Q1..Q1, the last column is the LLL-projected excited orbital.  Its
// Jastrow factor J_i factors out of row i as for the other states, leaving
//   X_i = -sum_{k != i} h_ik,  h_ik = (al P1_i u_k + be P2_i v_k) / (u_i v_k - u_k v_i),
//   P1 = u^A v^(B+1), P2 = u^(A+1) v^B, A = Q1 + m1, B = Q1 - m1, al = A + 1, be = B + 1
// (laughlin.py:93-99 with the diagonal term of jastrow_dv / jastrow_du cancelled).  That
// column depends on EVERY electron, so dE_a = e_n rho_a^T + c_a e_L^T (row n = electron of
// coordinate a, plus the dense column c_a[i] = dX_i / dx_a), and with w_n = E^-1 e_n,
// y_a = E^-1 c_a, z = row L of E^-1:
//   tr(E^-1 dE_a)          = rho_a . w_n + y_a[L]
//   tr(E^-1 dE_a E^-1 dE_b) = (rho_a . w_n')(rho_b . w_n) + (rho_a . y_b) z_n + z_n' (rho_b . y_a)
//                            + y_a[L] y_b[L]
//   tr(E^-1 d2E_ab)         = [n = n'] sum_j E^-1[j][n] d2E_nj + sum_i z_i d2X_i / dx_a dx_b
// with every derivative of h_ik from the quotient rule on its bilinear numerator and
// denominator (qp_pair).  The ground state and the quasihole are the case c = 0.
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
  int uv, E, dE, d2E, Einv, R, g, H, misc, P, c, Y, total;  // offsets in zd units
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
  L.P = o;
  o += 12 * N;  // quasiparticle: P1, P2 of each electron (value, d1[2], d2[3])
  L.c = o;
  o += 2 * N * N;  // c[a][i] = dX_i / dx_a
  L.Y = o;
  o += 2 * N * N;  // Y[a][j] = (E^-1 c_a)[j]
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

// h = (al P1_i u_k + be P2_i v_k) / e,  e = u_i v_k - u_k v_i, and its first / second
// derivatives in the coordinates (0 th_i, 1 ph_i, 2 th_k, 3 ph_k).  qi, qk: uv_derivs of the
// two electrons; Pi: P1 (0..5) and P2 (6..11) of electron i as value, d/dth, d/dph, d2 tt,
// tp, pp.  Numerator and denominator are bilinear in (u, v) of the two electrons, so their
// derivatives are products of uv_derivs terms; h_a = (n_a - h e_a) / e and
// h_ab = (n_ab - h_a e_b - h_b e_a - h e_ab) / e (the quotient rule twice).
struct PairD {
  zd h, d[4], dd[4][4];
};
__device__ void qp_pair(const zd* qi, const zd* qk, const zd* Pi, double al, double be, PairD& o) {
  const zd ui = qi[0], vi = qi[1], uk = qk[0], vk = qk[1];
  const zd P1 = Pi[0], P2 = Pi[6];
  // first derivatives of u, v of the electron of coordinate a (0, 1: i; 2, 3: k)
  auto du = [&](int a) { return a < 2 ? qi[2 + a] : qk[a]; };       // qk[2 + (a - 2)]
  auto dv = [&](int a) { return a < 2 ? qi[4 + a] : qk[2 + a]; };    // qk[4 + (a - 2)]
  zd n = al * (P1 * uk) + be * (P2 * vk);
  zd e = ui * vk - uk * vi;
  zd na[4], ea[4];
  for (int a = 0; a < 4; ++a) {
    if (a < 2) {
      na[a] = al * (Pi[1 + a] * uk) + be * (Pi[7 + a] * vk);
      ea[a] = du(a) * vk - uk * dv(a);
    } else {
      na[a] = al * (P1 * du(a)) + be * (P2 * dv(a));
      ea[a] = ui * dv(a) - du(a) * vi;
    }
  }
  const zd einv = zdiv(zd{1.0, 0.0}, e);
  o.h = n * einv;
  for (int a = 0; a < 4; ++a) o.d[a] = (na[a] - o.h * ea[a]) * einv;
  for (int a = 0; a < 4; ++a)
    for (int b = a; b < 4; ++b) {
      zd nab, eab;
      if (b < 2) {  // both on electron i
        const int k = a + b;  // 0 tt, 1 tp, 2 pp
        nab = al * (Pi[3 + k] * uk) + be * (Pi[9 + k] * vk);
        eab = qi[6 + k] * vk - uk * qi[9 + k];
      } else if (a >= 2) {  // both on electron k
        const int k = (a - 2) + (b - 2);
        nab = al * (P1 * qk[6 + k]) + be * (P2 * qk[9 + k]);
        eab = ui * qk[9 + k] - qk[6 + k] * vi;
      } else {  // a on i, b on k
        nab = al * (Pi[1 + a] * du(b)) + be * (Pi[7 + a] * dv(b));
        eab = du(a) * dv(b) - du(b) * dv(a);
      }
      const zd hab = (nab - o.d[a] * ea[b] - o.d[b] * ea[a] - o.h * eab) * einv;
      o.dd[a][b] = hab;
      o.dd[b][a] = hab;
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
  zd *PP = sm + L.P, *cX = sm + L.c, *Y = sm + L.Y;
  __shared__ int piv;
  __shared__ zd logdet;
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int NN = N * N, T = 2 * N;
  // quasiparticle: the last column (Lc) is the excited orbital X_i; P1 = u^A v^(B+1) with
  // weight al = A + 1, P2 = u^(A+1) v^B with be = B + 1 (A or B = -1 only with weight 0)
  const bool qp = expo[2 * N] != 0;
  const int Lc = N - 1, qa = expo[N - 1], qb = expo[2 * N - 1];
  const double al = qa + 1.0, be = qb + 1.0;
  for (int i = tid; i < N; i += nt) {
    uv_derivs((double)x[2 * (b * N + i)], (double)x[2 * (b * N + i) + 1], UV + 12 * i);
    if (qp) {
      zd* P = PP + 12 * i;
      for (int t = 0; t < 12; ++t) P[t] = zd{0.0, 0.0};
      if (al != 0.0) monomial(UV + 12 * i, qa, qb + 1, P, P + 1, P + 3);
      if (be != 0.0) monomial(UV + 12 * i, qa + 1, qb, P + 6, P + 7, P + 9);
    }
  }
  __syncthreads();
  // E (augmented with I) and its coordinate derivatives (row i depends on electron i only;
  // the quasiparticle column's derivatives go to cX below, its row entries stay zero)
  for (int idx = tid; idx < NN; idx += nt) {
    const int i = idx / N, j = idx % N;
    zd val{0.0, 0.0}, d1[2] = {{0.0, 0.0}, {0.0, 0.0}}, d2[3] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
    if (!qp || j != Lc) monomial(UV + 12 * i, expo[j], expo[N + j], &val, d1, d2);
    if (qp && j == Lc) val = zd{0.0, 0.0};  // X_i: the pair pass below
    E[i * 2 * N + j] = val;
    E[i * 2 * N + N + j] = zd{i == j ? 1.0 : 0.0, 0.0};
    dE[idx] = d1[0];
    dE[NN + idx] = d1[1];
    for (int k = 0; k < 3; ++k) d2E[k * NN + idx] = d2[k];
  }
  __syncthreads();
  if (qp) {
    // X_i and c[a][i] = dX_i / dx_a (thread i owns column i of c)
    for (int i = tid; i < N; i += nt) {
      for (int a = 0; a < T; ++a) cX[a * N + i] = zd{0.0, 0.0};
      zd X{0.0, 0.0}, own0{0.0, 0.0}, own1{0.0, 0.0};
      for (int k = 0; k < N; ++k) {
        if (k == i) continue;
        PairD pd;
        qp_pair(UV + 12 * i, UV + 12 * k, PP + 12 * i, al, be, pd);
        X = X - pd.h;
        own0 = own0 - pd.d[0];
        own1 = own1 - pd.d[1];
        cX[(2 * k) * N + i] = zd{0.0, 0.0} - pd.d[2];
        cX[(2 * k + 1) * N + i] = zd{0.0, 0.0} - pd.d[3];
      }
      cX[(2 * i) * N + i] = own0;
      cX[(2 * i + 1) * N + i] = own1;
      E[i * 2 * N + Lc] = X;
    }
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
  if (qp) {
    // Y[a][j] = (E^-1 c_a)[j]; H <- T2[a][b] = sum_i z_i d2X_i / dx_a dx_b, z = row Lc of E^-1:
    // thread per electron block (n, n'): n = n' sums the own-own terms of the pairs (n, k)
    // and the other-other terms of the pairs (k, n); n != n' takes the cross terms of the
    // pairs (n, n') and (n', n)
    for (int idx = tid; idx < T * N; idx += nt) {
      const int a = idx / N, j = idx % N;
      zd s{0.0, 0.0};
      for (int i = 0; i < N; ++i) s = s + Einv[j * N + i] * cX[a * N + i];
      Y[idx] = s;
    }
    for (int blk = tid; blk < NN; blk += nt) {
      const int n = blk / N, n2 = blk % N;
      zd t[2][2] = {{{0.0, 0.0}, {0.0, 0.0}}, {{0.0, 0.0}, {0.0, 0.0}}};
      PairD pd;
      if (n == n2) {
        for (int k = 0; k < N; ++k) {
          if (k == n) continue;
          qp_pair(UV + 12 * n, UV + 12 * k, PP + 12 * n, al, be, pd);  // X_n: n own
          const zd zn = Einv[Lc * N + n];
          for (int x2 = 0; x2 < 2; ++x2)
            for (int y2 = 0; y2 < 2; ++y2) t[x2][y2] = t[x2][y2] - zn * pd.dd[x2][y2];
          qp_pair(UV + 12 * k, UV + 12 * n, PP + 12 * k, al, be, pd);  // X_k: n other
          const zd zk = Einv[Lc * N + k];
          for (int x2 = 0; x2 < 2; ++x2)
            for (int y2 = 0; y2 < 2; ++y2) t[x2][y2] = t[x2][y2] - zk * pd.dd[2 + x2][2 + y2];
        }
      } else {
        qp_pair(UV + 12 * n, UV + 12 * n2, PP + 12 * n, al, be, pd);  // X_n: (own n, other n2)
        const zd zn = Einv[Lc * N + n];
        for (int x2 = 0; x2 < 2; ++x2)
          for (int y2 = 0; y2 < 2; ++y2) t[x2][y2] = t[x2][y2] - zn * pd.dd[x2][2 + y2];
        qp_pair(UV + 12 * n2, UV + 12 * n, PP + 12 * n2, al, be, pd);  // X_n2: (own n2, other n)
        const zd zm = Einv[Lc * N + n2];
        for (int x2 = 0; x2 < 2; ++x2)
          for (int y2 = 0; y2 < 2; ++y2) t[x2][y2] = t[x2][y2] - zm * pd.dd[2 + x2][y2];
      }
      for (int x2 = 0; x2 < 2; ++x2)
        for (int y2 = 0; y2 < 2; ++y2) H[(2 * n + x2) * T + 2 * n2 + y2] = t[x2][y2];
    }
    __syncthreads();
  }
  // gradient: determinant + pairs
  for (int a = tid; a < T; a += nt) {
    const int e = a >> 1, c = a & 1;
    zd s = R[a * N + e];
    if (qp) s = s + Y[a * N + Lc];
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
    if (qp) {
      // T2 (left in H by the pass above) - (rho_a . y_b) z_ea - z_eb (rho_b . y_a) - y_a[L] y_b[L]
      zd sab{0.0, 0.0}, sba{0.0, 0.0};
      for (int j = 0; j < N; ++j) {
        sab = sab + dE[ca * NN + ea * N + j] * Y[bb * N + j];
        sba = sba + dE[cb * NN + eb * N + j] * Y[a * N + j];
      }
      h = h + H[idx] - sab * Einv[Lc * N + ea] - Einv[Lc * N + eb] * sba - Y[a * N + Lc] * Y[bb * N + Lc];
    }
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
