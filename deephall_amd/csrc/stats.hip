// Device-local energy statistics of loss_and_grad (deephall/loss.py:30-38, 66-92),
// computed before the single cross-device all-reduce:
//   energy   = nanmean(E_L)                          (loss.py:73)
//   clipped  = nanmean(iqr_clip(E_L))                (loss.py:74, 30-38: quantiles of the
//              LOCAL batch, real and imaginary parts clipped separately, scale 100)
//   ere2     = nanmean(Re(E_L)^2)                    (loss.py:91; the global energy^2 is
//              subtracted after the all-reduce)
//   observables: plain means (loss.py:68-71), pmove = sum accepts / (steps * B) (mcmc.py:146)
// One 1024-thread workgroup; quantiles by an LDS bitonic sort, the real and imaginary
// parts at once (one half of the workgroup each) for B <= 16384, else one after the other
// (B <= 32768).
#include "dh_internal.h"
#include "device_common.h"

namespace dh {
namespace {

constexpr int kNT = 1024;

// sorts s[0..n2) ascending (n2 power of two) with the threads [t0, t0 + nt) of the block;
// every thread of the block calls it (the barriers are block-wide)
__device__ void bitonic(float* s, int n2, int t0, int nt) {
  const int me = (int)threadIdx.x - t0;
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (me >= 0 && me < nt)
        for (int i = me; i < n2; i += nt) {
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

constexpr int kNQ = 14;  // accumulated sums

__global__ __launch_bounds__(kNT) void stats_kernel(const float* __restrict__ e_l, const float* __restrict__ obs,
                                                    const int32_t* __restrict__ n_acc, int B, int steps, int n2,
                                                    int conc, float* __restrict__ out) {
  extern __shared__ float s[];  // [2][n2] (real, imaginary parts) or [n2]
  __shared__ double red[kNT / 64][kNQ];
  __shared__ int cnt_s[2];
  __shared__ float bounds[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < 2) cnt_s[tid] = 0;
  __syncthreads();
  // NaN -> +inf: sorted to the end and excluded by the count.  Both parts at once (one
  // half of the block each) when 2 n2 floats fit the LDS, else one after the other.
  const bool both = conc != 0;
  for (int part = 0; part < (both ? 1 : 2); ++part) {
    int c0 = 0, c1 = 0;
    for (int i = tid; i < n2; i += blockDim.x) {
      float re = INFINITY, im = INFINITY;
      if (i < B) {
        const float x = e_l[2 * i], y = e_l[2 * i + 1];
        if (!isnan(x)) re = x, ++c0;
        if (!isnan(y)) im = y, ++c1;
      }
      if (both) {
        s[i] = re;
        s[n2 + i] = im;
      } else {
        s[i] = part == 0 ? re : im;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      c0 += __shfl_xor(c0, o, 64);
      c1 += __shfl_xor(c1, o, 64);
    }
    if (lane == 0 && part == 0) {
      atomicAdd(&cnt_s[0], c0);
      atomicAdd(&cnt_s[1], c1);
    }
    __syncthreads();
    if (both) {
      const int half = blockDim.x / 2;
      bitonic(tid < half ? s : s + n2, n2, tid < half ? 0 : half, half);
    } else {
      bitonic(s, n2, 0, blockDim.x);
    }
    if (both ? tid < 2 : tid == 0) {
      const int q = both ? tid : part;
      const float* sp = s + (both ? tid * n2 : 0);
      const int n = cnt_s[q];
      const float q1 = quant(sp, n, 0.25f), q3 = quant(sp, n, 0.75f);
      const float iqr = q3 - q1;
      bounds[2 * q] = q1 - 100.f * iqr;
      bounds[2 * q + 1] = q3 + 100.f * iqr;
    }
    __syncthreads();
  }
  double acc[kNQ];
#pragma unroll
  for (int q = 0; q < kNQ; ++q) acc[q] = 0.0;
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
    if (n_acc) acc[13] += n_acc[i];
  }
  // one block reduction of all sums: wave shuffles, then one LDS pass
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    double v = acc[q];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[w][q] = v;
  }
  __syncthreads();
  if (tid < kNQ) {
    double t = 0.0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i][tid];
    red[0][tid] = t;  // each thread reads and writes only its own column
  }
  __syncthreads();
  if (tid == 0) {
    const double* tot = red[0];
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
  const int conc = n2 <= 16384;  // 2 x 64 KiB of LDS
  const size_t bytes = (conc ? 2 : 1) * (size_t)n2 * sizeof(float);
  ensure_smem(stats_kernel, bytes);
  hipLaunchKernelGGL(stats_kernel, dim3(1), dim3(kNT), bytes, s, e_l, obs, n_acc, B, steps, n2, conc, out);
}

}  // namespace dh
