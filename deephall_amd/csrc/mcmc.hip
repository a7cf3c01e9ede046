// Metropolis-Hastings pieces of the walker update (deephall/mcmc.py).
//
//   propose_kernel  sph_sampling (mcmc.py:67-102): theta' = arctan(xi * width),
//                   phi' = 2 pi U, rotate the pole onto each electron with
//                   R_z(phi) R_y(theta), back to (theta, phi) with clipping (double).
//   accept_kernel   mh_update accept/select (mcmc.py:55-62): accept the whole
//                   walker if 2 Re log psi(x') - lp > log U.
//   init_kernel     init_guess (train.py:40-54): theta = arccos U(-1,1), phi = U(-pi,pi).
//
// Random numbers: Philox4x32-10 keyed by the seed, counter (lane, global walker,
// step) — see device_common.h — or injected arrays [B][2N+1] per step
// (normals[N], phi uniforms[N], accept uniform) for parity tests.
#include <algorithm>

#include "dh_internal.h"
#include "device_common.h"
#include "mcmc_common.h"

namespace dh {
namespace {

__global__ void propose_kernel(const float* __restrict__ x, float* __restrict__ x2, float* __restrict__ geo, int nw,
                               int N, float width, uint64_t seed, uint64_t step, int64_t woff,
                               const float* __restrict__ noise) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nw * N) return;
  propose_one(x[2 * e], x[2 * e + 1], x2, geo, e, e / N, e % N, N, width, seed, step, woff, noise);
}

// accept_kernel for step `step` and the proposal of step `step + 1` in one launch: thread
// per electron; every thread of a walker recomputes the walker's accept decision (same
// random number, same inputs), moves only its own electron, and proposes its next move
// from the result (noise2: the next step's injected noise).
__global__ void accept_propose_kernel(float* __restrict__ x, float* __restrict__ x2, float* __restrict__ geo,
                                      float* __restrict__ lp, const float* __restrict__ logpsi2,
                                      int32_t* __restrict__ nacc, int nw, int N, float width, uint64_t seed,
                                      uint64_t step, int64_t woff, const float* __restrict__ noise,
                                      const float* __restrict__ noise2) {
  // blocks hold whole walkers (blockDim = N x walkers per block), so the barrier below
  // orders every read of lp[b] before its rewrite
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const bool on = e < nw * N;
  const int b = e / N, i = e % N;
  bool cond = false;
  float lp2 = 0.f, th = 0.f, ph = 0.f;
  if (on) {
    lp2 = 2.f * logpsi2[2 * b];
    cond = accept_one(lp2, lp[b], b, N, seed, step, woff, noise);
    th = x[2 * e];
    ph = x[2 * e + 1];
    if (cond) {
      th = x2[2 * e];
      ph = x2[2 * e + 1];
      x[2 * e] = th;
      x[2 * e + 1] = ph;
    }
  }
  __syncthreads();
  if (!on) return;
  if (cond && i == 0) {
    lp[b] = lp2;
    nacc[b] += 1;
  }
  propose_one(th, ph, x2, geo, e, b, i, N, width, seed, step + 1, woff, noise2);
}

__global__ void accept_kernel(float* __restrict__ x, const float* __restrict__ x2, float* __restrict__ lp,
                              const float* __restrict__ logpsi2, int32_t* __restrict__ nacc, int nw, int N,
                              uint64_t seed, uint64_t step, int64_t woff, const float* __restrict__ noise) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nw) return;
  const float lp2 = 2.f * logpsi2[2 * b];
  const bool cond = accept_one(lp2, lp[b], b, N, seed, step, woff, noise);
  if (cond) {
    for (int k = 0; k < 2 * N; ++k) x[(size_t)b * 2 * N + k] = x2[(size_t)b * 2 * N + k];
    lp[b] = lp2;
    nacc[b] += 1;
  }
}

__global__ void lp_init_kernel(const float* __restrict__ logpsi, float* __restrict__ lp, int32_t* __restrict__ nacc,
                               int nw) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nw) return;
  lp[b] = 2.f * logpsi[2 * b];
  nacc[b] = 0;
}

__global__ void init_kernel(float* __restrict__ x, int nw, int N, uint64_t seed, int64_t woff) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nw * N) return;
  const int b = e / N, i = e % N;
  u32x4 r = dh_random(seed, kPurposeInit, (uint32_t)i, (uint64_t)(woff + b), 0);
  const float u1 = u01(r.x), u2 = u01(r.y);
  x[2 * e] = acosf(2.f * u1 - 1.f);
  x[2 * e + 1] = (2.f * u2 - 1.f) * kPi;
}

}  // namespace

void launch_propose(const Dims& d, const float* x, float* x2, int nw, float width, uint64_t seed, uint64_t step,
                    int64_t walker_offset, const float* noise, int noise_stride, hipStream_t s, float* geo) {
  (void)noise_stride;
  const int n = nw * d.N;
  hipLaunchKernelGGL(propose_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, x2, geo, nw, d.N, width, seed, step,
                     walker_offset, noise);
}

void launch_accept_propose(const Dims& d, float* x, float* x2, float* geo, float* lp, const float* logpsi2,
                           int32_t* n_acc, int nw, float width, uint64_t seed, uint64_t step, int64_t walker_offset,
                           const float* noise, const float* noise2, hipStream_t s) {
  const int wpb = std::max(1, 256 / d.N);  // whole walkers per block
  hipLaunchKernelGGL(accept_propose_kernel, dim3((nw + wpb - 1) / wpb), dim3(wpb * d.N), 0, s, x, x2, geo, lp,
                     logpsi2, n_acc, nw, d.N, width, seed, step, walker_offset, noise, noise2);
}

void launch_accept(const Dims& d, float* x, const float* x2, float* lp, const float* logpsi2, int32_t* n_acc,
                   int nw, uint64_t seed, uint64_t step, int64_t walker_offset, const float* noise,
                   int noise_stride, hipStream_t s) {
  (void)noise_stride;
  hipLaunchKernelGGL(accept_kernel, dim3((nw + 255) / 256), dim3(256), 0, s, x, x2, lp, logpsi2, n_acc, nw, d.N,
                     seed, step, walker_offset, noise);
}

void launch_lp_from_logpsi(const float* logpsi, float* lp, int32_t* n_acc, int nw, hipStream_t s) {
  hipLaunchKernelGGL(lp_init_kernel, dim3((nw + 255) / 256), dim3(256), 0, s, logpsi, lp, n_acc, nw);
}

void launch_init_walkers(const Dims& d, float* x, int nw, uint64_t seed, int64_t walker_offset, hipStream_t s) {
  const int n = nw * d.N;
  hipLaunchKernelGGL(init_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, nw, d.N, seed, walker_offset);
}

}  // namespace dh
