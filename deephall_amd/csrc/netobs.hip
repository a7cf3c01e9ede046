// NetObs-style estimators on the device (reference
// deephall/netobs_bridge/observables/*.py):
//
//   density    (density.py:38-44): histogram of every electron's theta over [0, pi]
//   pair corr. (pair_corr.py:43-58): histogram of the pair angle theta_12 = arccos(r_i . r_j)
//              over i < j, [0, pi], weight 1 / sin theta_12 (the caller scales by
//              4 bins / (B N^2 pi), as pair_corr.py:57)
//   orbitals   (one_rdm.py:31-54): the lowest-Landau-level monopole harmonics
//              Y_{Q,Q,m}, m = -Q..Q, at given points (one-body density matrix basis)
//
// Histograms follow numpy / jnp.histogram: edges linspace(0, pi, bins + 1), the last bin
// closed, values outside [0, pi] (or NaN) dropped.  Each block accumulates into LDS with
// ds_add_f32, then adds its bins to the global histogram (vector atomics, one per bin).
// The pair geometry is evaluated in double (the chord of a close pair from f32 sin / cos
// loses eps_f32 / r^2).
#include <cmath>

#include "dh_internal.h"
#include "device_common.h"

namespace dh {
namespace {

__device__ __forceinline__ int hist_bin(double v, int bins) {
  if (!(v >= 0.0 && v <= M_PI)) return -1;  // NaN and out-of-range values are dropped
  int k = (int)(v * (bins / M_PI));
  return k >= bins ? bins - 1 : k;
}

// one block per 256-walker slice; LDS: density [db] + pair [pb] floats
__global__ __launch_bounds__(256) void hist_kernel(const float* __restrict__ x, int B, int N, int db, int pb,
                                                   float* __restrict__ dens, float* __restrict__ pair) {
  extern __shared__ float hs[];
  float* hd = hs;
  float* hp = hs + db;
  for (int k = threadIdx.x; k < db + pb; k += 256) hs[k] = 0.f;
  __syncthreads();
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b < B) {
    const float* xb = x + (size_t)b * N * 2;
    for (int i = 0; i < N; ++i) {
      if (db > 0) {
        const int k = hist_bin((double)xb[2 * i], db);
        if (k >= 0) atomicAdd(hd + k, 1.f);
      }
      if (pb > 0) {
        double sti, cti, spi, cpi;
        sincos((double)xb[2 * i], &sti, &cti);
        sincos((double)xb[2 * i + 1], &spi, &cpi);
        for (int j = i + 1; j < N; ++j) {
          double stj, ctj, spj, cpj;
          sincos((double)xb[2 * j], &stj, &ctj);
          sincos((double)xb[2 * j + 1], &spj, &cpj);
          const double c = sti * stj * (cpi * cpj + spi * spj) + cti * ctj;
          const double t = acos(c);
          const int k = hist_bin(t, pb);
          if (k >= 0) atomicAdd(hp + k, (float)(1.0 / sin(t)));
        }
      }
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < db; k += 256)
    if (hd[k] != 0.f) atomicAdd(dens + k, hd[k]);
  for (int k = threadIdx.x; k < pb; k += 256)
    if (hp[k] != 0.f) atomicAdd(pair + k, hp[k]);
}

// Y_{Q,Q,m}(theta, phi), m = -Q + k (k < flux + 1): with l = q = Q only the s = 0 term of
// one_rdm.py:36-51 survives, Y = c_m (1 - x)^((Q - m) / 2) (1 + x)^((Q + m) / 2) e^{i m phi},
// x = clip(cos theta, -1 + 1e-4, 1 - 1e-4), and norm x sum factor collapse to
// c_m = (-1)^(Q - m) 2^-Q sqrt((2Q + 1) / 4 pi) sqrt(binom(2Q, Q - m)).  Double precision.
__global__ void orbitals_kernel(const float* __restrict__ pts, int n, int flux, float* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const double th = pts[2 * p], ph = pts[2 * p + 1];
  const double x = fmin(fmax(cos(th), -1.0 + 1e-4), 1.0 - 1e-4);
  const double lm = log1p(-x), lp = log1p(x);  // log(1 - x), log(1 + x)
  const double Q = 0.5 * flux;
  float* o = out + (size_t)p * (flux + 1) * 2;
  const double lg2q = lgamma(2.0 * Q + 1.0), base = sqrt((2.0 * Q + 1.0) / (4.0 * M_PI));
  for (int k = 0; k <= flux; ++k) {
    const double m = -Q + k;  // Q - m = flux - k
    const double lbin = lg2q - lgamma(Q - m + 1.0) - lgamma(Q + m + 1.0);
    const double cm = (((flux - k) & 1) ? -base : base) * exp(0.5 * lbin - Q * M_LN2);
    const double mag = cm * exp(0.5 * (Q - m) * lm + 0.5 * (Q + m) * lp);
    double s, c;
    sincos(m * ph, &s, &c);
    o[2 * k] = (float)(mag * c);
    o[2 * k + 1] = (float)(mag * s);
  }
}

}  // namespace

void launch_histograms(const float* x, int B, int N, int db, int pb, float* dens, float* pair, hipStream_t s) {
  const size_t smem = (size_t)(db + pb) * sizeof(float);
  ensure_smem(hist_kernel, smem);
  hipLaunchKernelGGL(hist_kernel, dim3((B + 255) / 256), dim3(256), smem, s, x, B, N, db, pb, dens, pair);
}

void launch_monopole_orbitals(const float* pts, int n, int flux, float* out, hipStream_t s) {
  hipLaunchKernelGGL(orbitals_kernel, dim3((n + 127) / 128), dim3(128), 0, s, pts, n, flux, out);
}

}  // namespace dh
