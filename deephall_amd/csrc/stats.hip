// Device-local energy statistics of loss_and_grad (deephall/loss.py:30-38, 66-92),
// computed before the single cross-device all-reduce:
//   energy   = nanmean(E_L)                          (loss.py:73)
//   clipped  = nanmean(iqr_clip(E_L))                (loss.py:74, 30-38: quantiles of the
//              LOCAL batch, real and imaginary parts clipped separately, scale 100)
//   ere2     = nanmean(Re(E_L)^2)                    (loss.py:91; the global energy^2 is
//              subtracted after the all-reduce)
//   observables: plain means (loss.py:68-71), pmove = sum accepts / (steps * B) (mcmc.py:146)
// One 1024-thread workgroup; quantiles by an LDS bitonic sort (B <= 32768).
#include "dh_internal.h"
#include "device_common.h"

namespace dh {
namespace {

constexpr int kNT = 1024;

__device__ double block_sum_d(double v, double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

// sorts s[0..n2) ascending (n2 power of two)
__device__ void bitonic(float* s, int n2) {
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n2; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const float a = s[i], b = s[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            s[i] = b;
            s[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}

// nanquantile, linear interpolation (numpy / jnp default)
__device__ float quant(const float* s, int n, float q) {
  if (n == 0) return NAN;
  const float pos = q * (float)(n - 1);
  const int lo = (int)floorf(pos);
  const int hi = min(lo + 1, n - 1);
  const float fr = pos - (float)lo;
  return s[lo] + (s[hi] - s[lo]) * fr;
}

__global__ __launch_bounds__(kNT) void stats_kernel(const float* __restrict__ e_l, const float* __restrict__ obs,
                                                    const int32_t* __restrict__ n_acc, int B, int steps, int n2,
                                                    float* __restrict__ out) {
  extern __shared__ float s[];
  __shared__ double red[kNT / 64];
  __shared__ float bounds[4];
  const int tid = threadIdx.x;
  for (int part = 0; part < 2; ++part) {
    int cnt = 0;
    for (int i = tid; i < n2; i += blockDim.x) {
      float v = INFINITY;
      if (i < B) {
        const float x = e_l[2 * i + part];
        if (!isnan(x)) {
          v = x;
          ++cnt;
        }
      }
      s[i] = v;
    }
    const int n = (int)block_sum_d((double)cnt, red);
    __syncthreads();
    bitonic(s, n2);
    if (tid == 0) {
      const float q1 = quant(s, n, 0.25f), q3 = quant(s, n, 0.75f);
      const float iqr = q3 - q1;
      bounds[2 * part] = q1 - 100.f * iqr;
      bounds[2 * part + 1] = q3 + 100.f * iqr;
    }
    __syncthreads();
  }
  double acc[13];
  for (int q = 0; q < 13; ++q) acc[q] = 0.0;
  for (int i = tid; i < B; i += blockDim.x) {
    const float re = e_l[2 * i], im = e_l[2 * i + 1];
    const bool valid = !(isnan(re) || isnan(im));
    if (valid) {
      acc[0] += re;
      acc[1] += im;
      acc[2] += fminf(fmaxf(re, bounds[0]), bounds[1]);
      acc[3] += fminf(fmaxf(im, bounds[2]), bounds[3]);
      acc[12] += 1.0;
    }
    if (!isnan(re)) {
      acc[4] += (double)re * re;
      acc[11] += 1.0;
    }
    const float* o = obs + 8 * (size_t)i;
    acc[5] += o[0];
    acc[6] += o[1];
    acc[7] += o[2];
    acc[8] += o[3];
    acc[9] += o[4];
    acc[10] += o[5];
  }
  double pm = 0.0;
  if (n_acc)
    for (int i = tid; i < B; i += blockDim.x) pm += n_acc[i];
  double tot[14];
  for (int q = 0; q < 13; ++q) {
    tot[q] = block_sum_d(acc[q], red);
    __syncthreads();
  }
  tot[13] = block_sum_d(pm, red);
  if (tid == 0) {
    const double nv = tot[12];
    out[DH_STAT_ENERGY_RE] = (float)(tot[0] / nv);
    out[DH_STAT_ENERGY_IM] = (float)(tot[1] / nv);
    out[DH_STAT_CLIPPED_RE] = (float)(tot[2] / nv);
    out[DH_STAT_CLIPPED_IM] = (float)(tot[3] / nv);
    out[DH_STAT_ERE2] = (float)(tot[4] / tot[11]);
    out[DH_STAT_KINETIC_RE] = (float)(tot[5] / B);
    out[DH_STAT_KINETIC_IM] = (float)(tot[6] / B);
    out[DH_STAT_POTENTIAL] = (float)(tot[7] / B);
    out[DH_STAT_LZ] = (float)(tot[8] / B);
    out[DH_STAT_LZ2] = (float)(tot[9] / B);
    out[DH_STAT_L2] = (float)(tot[10] / B);
    out[DH_STAT_PMOVE] = n_acc ? (float)(tot[13] / ((double)steps * B)) : 0.f;
    out[DH_STAT_NVALID] = (float)nv;
    for (int q = DH_STAT_NVALID + 1; q < DH_NSTATS; ++q) out[q] = 0.f;
  }
}

}  // namespace

void launch_stats(const float* e_l, const float* obs, const int32_t* n_acc, int B, int steps, float* out,
                  float* scratch, hipStream_t s) {
  (void)scratch;
  int n2 = 1;
  while (n2 < B) n2 <<= 1;
  ensure_smem(stats_kernel, (size_t)n2 * sizeof(float));
  hipLaunchKernelGGL(stats_kernel, dim3(1), dim3(kNT), (size_t)n2 * sizeof(float), s, e_l, obs, n_acc, B, steps, n2,
                     out);
}

}  // namespace dh
