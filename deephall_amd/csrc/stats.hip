// Device-local statistics of loss_and_grad (deephall/loss.py:30-38, 66-92), computed
// before the single cross-device all-reduce, and the clipped energy difference that
// weights the parameter gradient (loss.py:75-89):
//
//   stats_kernel (dh_energy_stats)
//     energy   = nanmean(E_L)                          (loss.py:73)
//     clipped  = nanmean(iqr_clip(E_L))                (loss.py:74; iqr_clip 30-38: nanquantiles
//                of the LOCAL batch, real and imaginary parts clipped separately, scale 100)
//     ere2     = nanmean(Re(E_L)^2)                    (loss.py:91; the global energy^2 is
//                subtracted after the all-reduce)
//     observables: plain means (loss.py:68-71), pmove = sum accepts / (steps * B) (mcmc.py:146)
//     with penalties on: nanmean(iqr_clip(Lz^2)), nanmean(iqr_clip(Lz)), nanmean(iqr_clip(L^2))
//                (loss.py:79-80, 87)
//   diff_kernel (dh_loss_diff), after the all-reduce:
//     d = E_L - clipped + lz_penalty ((Lz^2 - <Lz^2>_c) - 2 lz_center (Lz - <Lz>_c))
//           + l2_penalty (L^2 - <L^2>_c)                 (loss.py:75-88)
//     diff = iqr_clip(d)                                 (loss.py:89)
//
// Quantiles: one 1024-thread workgroup selects the order statistics numpy/jnp.nanquantile
// (linear interpolation) needs — ranks floor(q (n-1)) and the next one for q = 1/4, 3/4 —
// by an MSB-first radix select over the order-preserving uint32 image of the floats:
// 4 passes of 8-bit digits, all parts and ranks at once (one LDS histogram of 256 bins per
// (part, rank)), so there is no batch-size limit and no sort.  NaN values are excluded
// from the counts, as nanquantile excludes them.
#include "dh_internal.h"
#include "device_common.h"

namespace dh {
namespace {

#ifndef STATS_ABL  // timing ablations (tools/stats_bench.py only)
#define STATS_ABL 0
#endif
constexpr int kNT = 1024;
constexpr int kNW = kNT / 64;
constexpr int kMaxParts = 5;
#ifndef STATS_CACHE  // values per thread held in registers by iqr_bounds
#define STATS_CACHE 4
#endif
#ifndef STATS_CPARTS  // parts cached in registers (more, the penalty form: the uncached path)
#define STATS_CPARTS 2
#endif
// (B <= 4096 and the two E_L parts, round 5: with 8 values of all 5 parts the 128-VGPR budget
// of a 1024-thread workgroup spilled the keys to scratch: 42.8 -> 37.3 us per call at B = 4096;
// the penalty form, 5 parts, now takes the uncached path: 71 -> 97 us, profiles/r05_v24_stats.txt)
constexpr int kCache = STATS_CACHE, kCP = STATS_CPARTS;

// order-preserving float -> uint32 (NaN excluded by the caller)
__device__ __forceinline__ uint32_t fkey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kfloat(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// The per-walker values whose quantiles are needed.
struct Src {
  const float* e_l;  // [B][2]
  const float* obs;  // [B][8]: KE re, KE im, PE, Lz, Lz^2, L^2, logpsi re, im
  int diff;          // 0: stats parts (Re E, Im E, Lz^2, Lz, L^2); 1: the difference d (re, im)
  float cl_re, cl_im, lz_pen, lz_center, l2_pen, c_lz2, c_lz, c_l2;
};

__device__ __forceinline__ float diff_re(const Src& s, int i) {
  float d = s.e_l[2 * i] - s.cl_re;
  if (s.lz_pen != 0.f) {
    const float* o = s.obs + 8 * (size_t)i;
    d += s.lz_pen * ((o[4] - s.c_lz2) - 2.f * s.lz_center * (o[3] - s.c_lz));
  }
  if (s.l2_pen != 0.f) d += s.l2_pen * (s.obs[8 * (size_t)i + 5] - s.c_l2);
  return d;
}

__device__ __forceinline__ float part_value(const Src& s, int p, int i) {
  if (s.diff) return p == 0 ? diff_re(s, i) : s.e_l[2 * i + 1] - s.cl_im;
  if (p < 2) return s.e_l[2 * i + p];
  const float* o = s.obs + 8 * (size_t)i;
  return p == 2 ? o[4] : (p == 3 ? o[3] : o[5]);
}

struct SelectLds {
  uint32_t hist[kMaxParts * 4][256];
  uint32_t prefix[kMaxParts * 4];
  int kleft[kMaxParts * 4];
  int src[kMaxParts * 4];  // per pass: the first rank of the part with the same prefix (its histogram)
  int cnt[kMaxParts];
  int wcnt[kNW][kMaxParts];
  float lo[kMaxParts], hi[kMaxParts];  // clip bounds
};

// Clip bounds q1 - 100 iqr, q3 + 100 iqr of the first np parts (NaN bounds for a part with
// no valid value).  Every thread of the block calls it.  (noinline: inlined into
// stats_kernel, ROCm 7.2 clang -O2/-O3 crashes in instruction selection.)
__device__ __noinline__ void iqr_bounds(const Src& s, int B, int np, SelectLds& L) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // the order-preserving keys of this thread's values, read once (B <= kCache * kNT): the
  // passes below then run on registers instead of re-reading global memory between atomics
  const bool cached = B <= kCache * kNT && np <= kCP;
  uint32_t kc[kCache][kCP];
  uint64_t okm = 0;  // bit u * kCP + p: value (u, p) is not NaN
  if (cached) {
#pragma unroll
    for (int u = 0; u < kCache; ++u) {
      const int i = tid + u * kNT;
#pragma unroll
      for (int p = 0; p < kCP; ++p) {
        const float v = (p < np && i < B) ? part_value(s, p, i) : NAN;
        const bool ok = !isnan(v);
        kc[u][p] = ok ? fkey(v) : 0u;
        if (ok) okm |= 1ull << (u * kCP + p);
      }
    }
  }
  // valid counts
  int c[kMaxParts] = {0, 0, 0, 0, 0};
  if (cached) {
#pragma unroll
    for (int u = 0; u < kCache; ++u) {
#pragma unroll
      for (int p = 0; p < kCP; ++p) c[p] += (okm >> (u * kCP + p)) & 1ull ? 1 : 0;
    }
  } else {
    for (int i = tid; i < B; i += kNT)
      for (int p = 0; p < np; ++p) c[p] += isnan(part_value(s, p, i)) ? 0 : 1;
  }
  for (int p = 0; p < np; ++p) {
    int v = c[p];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) L.wcnt[w][p] = v;
  }
  __syncthreads();
  const int nh = 4 * np;
  if (tid < np) {
    int n = 0;
    for (int j = 0; j < kNW; ++j) n += L.wcnt[j][tid];
    L.cnt[tid] = n;
    // ranks: floor(q (n-1)) and the next one, q = 1/4, 3/4 (exact in float for n < 2^24)
    for (int q = 0; q < 2; ++q) {
      const float pos = (q == 0 ? 0.25f : 0.75f) * (float)max(n - 1, 0);
      const int r0 = (int)floorf(pos);
      L.kleft[4 * tid + 2 * q] = r0;
      L.kleft[4 * tid + 2 * q + 1] = min(r0 + 1, max(n - 1, 0));
    }
    for (int r = 0; r < 4; ++r) L.prefix[4 * tid + r] = 0u;
  }
  __syncthreads();
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const uint32_t hmask = pass == 0 ? 0u : (0xffffffffu << (shift + 8));
    // ranks of a part whose prefixes agree so far share one histogram (pass 0: all four; later
    // the two ranks of a quartile, usually): counted once (round 5, half the count work)
    if (tid < nh) {
      int sr = tid;
      for (int r = (tid & ~3); r < tid; ++r)
        if (L.prefix[r] == L.prefix[tid]) {
          sr = r;
          break;
        }
      L.src[tid] = sr;
    }
    for (int j = tid; j < nh * 256; j += kNT) (&L.hist[0][0])[j] = 0u;
    __syncthreads();
    auto count = [&](bool ok, uint32_t u, int p) __attribute__((always_inline)) {
        const uint32_t dig = (u >> shift) & 255u;
        for (int r = 0; r < 4; ++r) {
          if (L.src[4 * p + r] != 4 * p + r) continue;  // block-uniform
          const bool take = ok && ((u ^ L.prefix[4 * p + r]) & hmask) == 0u;
          // the common case of a wave sharing one digit (leading bits of similar values)
          // becomes one atomic; the rest fall back to per-lane atomics
          const uint64_t act = __ballot(take);
          if (act == 0) continue;
          const int lead = __ffsll((long long)act) - 1;
          const uint32_t ldig = __shfl(dig, lead, 64);
          const uint64_t same = __ballot(take && dig == ldig);
          if (lane == lead) atomicAdd(&L.hist[4 * p + r][ldig], (uint32_t)__popcll(same));
          if (take && dig != ldig) atomicAdd(&L.hist[4 * p + r][dig], 1u);
        }
    };
    if (cached) {
#pragma unroll
      for (int u = 0; u < kCache; ++u) {
        if (u * kNT >= B) break;  // block-uniform
#pragma unroll
        for (int p = 0; p < kCP; ++p)
          if (p < np) count((okm >> (u * kCP + p)) & 1ull, kc[u][p], p);
      }
    } else {
      for (int i0 = 0; i0 < B; i0 += kNT) {
        const int i = i0 + tid;
        for (int p = 0; p < np; ++p) {
          const float v = i < B ? part_value(s, p, i) : NAN;
          const bool ok = !isnan(v);
          count(ok, ok ? fkey(v) : 0u, p);
        }
      }
    }
    __syncthreads();
    // one wave per histogram: find the bin holding rank kleft, descend into it
    for (int hh = w; hh < nh; hh += kNW) {
      const uint32_t* hb = L.hist[L.src[hh]];
      uint32_t b0 = hb[4 * lane], b1 = hb[4 * lane + 1], b2 = hb[4 * lane + 2], b3 = hb[4 * lane + 3];
      const uint32_t loc = b0 + b1 + b2 + b3;
      uint32_t incl = loc;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      const int k = L.kleft[hh];
      const uint64_t over = __ballot(incl > (uint32_t)k);
      if (over != 0 && lane == __ffsll((long long)over) - 1) {
        uint32_t below = incl - loc;
        const uint32_t bins[4] = {b0, b1, b2, b3};
        int j = 0;
        while (j < 3 && below + bins[j] <= (uint32_t)k) below += bins[j++];
        L.prefix[hh] |= (uint32_t)(4 * lane + j) << shift;
        L.kleft[hh] = k - (int)below;
      }
    }
    __syncthreads();
  }
  if (tid < np) {
    const int n = L.cnt[tid];
    float lo = NAN, hi = NAN;
    if (n > 0) {
      float q[2];
      for (int qq = 0; qq < 2; ++qq) {
        const float pos = (qq == 0 ? 0.25f : 0.75f) * (float)(n - 1);
        const float fr = pos - floorf(pos);
        const float a = kfloat(L.prefix[4 * tid + 2 * qq]), b = kfloat(L.prefix[4 * tid + 2 * qq + 1]);
        q[qq] = a + (b - a) * fr;
      }
      const float iqr = q[1] - q[0];
      lo = q[0] - 100.f * iqr;
      hi = q[1] + 100.f * iqr;
    }
    L.lo[tid] = lo;
    L.hi[tid] = hi;
  }
  __syncthreads();
}

// jnp.clip: NaN stays NaN (fmaxf alone would return the bound)
__device__ __forceinline__ float clip(float x, float lo, float hi) {
  return isnan(x) ? x : fminf(fmaxf(x, lo), hi);
}

constexpr int kNQ = 18;  // accumulated sums

__global__ __launch_bounds__(kNT) void stats_kernel(const float* __restrict__ e_l, const float* __restrict__ obs,
                                                    const int32_t* __restrict__ n_acc, int B, int steps,
                                                    int penalties, float* __restrict__ out) {
  __shared__ SelectLds L;
  __shared__ double red[kNW][kNQ];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  Src src{e_l, obs, 0, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  iqr_bounds(src, B, penalties ? 5 : 2, L);
#if STATS_ABL & 2  // ablation (timing tools only): quantiles only
  if (tid == 0) out[0] = L.lo[0] + L.hi[1];
  return;
#endif
  double acc[kNQ];
#pragma unroll
  for (int q = 0; q < kNQ; ++q) acc[q] = 0.0;
  for (int i = tid; i < B; i += kNT) {
    const float re = e_l[2 * i], im = e_l[2 * i + 1];
    if (!(isnan(re) || isnan(im))) {  // nanmean of a complex array skips NaN in either part
      acc[0] += re;
      acc[1] += im;
      acc[2] += clip(re, L.lo[0], L.hi[0]);
      acc[3] += clip(im, L.lo[1], L.hi[1]);
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
    if (penalties) {  // nanmean(iqr_clip(x)) of the real observables Lz^2, Lz, L^2
      const float v[3] = {o[4], o[3], o[5]};
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (!isnan(v[j])) {
          acc[14 + j] += clip(v[j], L.lo[2 + j], L.hi[2 + j]);
        }
    }
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
    for (int i = 0; i < kNW; ++i) t += red[i][tid];
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
    out[DH_STAT_CLIPPED_LZ2] = penalties ? (float)(tot[14] / L.cnt[2]) : 0.f;
    out[DH_STAT_CLIPPED_LZ] = penalties ? (float)(tot[15] / L.cnt[3]) : 0.f;
    out[DH_STAT_CLIPPED_L2] = penalties ? (float)(tot[16] / L.cnt[4]) : 0.f;
  }
}

// diff = iqr_clip(d) (loss.py:75-89) -> diff[B][2] (NaN where d is NaN), and
// wsum[0] = number of walkers whose complex diff is not NaN (the nanmean count of
// loss_prod, loss.py:64).
__global__ __launch_bounds__(kNT) void diff_kernel(Src s, const float* __restrict__ g, int B,
                                                   float* __restrict__ diff, float* __restrict__ nvalid) {
  __shared__ SelectLds L;
  __shared__ int wn[kNW];
  // the reduced (global) clipped means, DH_STAT_* layout
  s.cl_re = g[DH_STAT_CLIPPED_RE];
  s.cl_im = g[DH_STAT_CLIPPED_IM];
  s.c_lz2 = g[DH_STAT_CLIPPED_LZ2];
  s.c_lz = g[DH_STAT_CLIPPED_LZ];
  s.c_l2 = g[DH_STAT_CLIPPED_L2];
  iqr_bounds(s, B, 2, L);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int n = 0;
  for (int i = tid; i < B; i += kNT) {
    const float dr = clip(part_value(s, 0, i), L.lo[0], L.hi[0]);
    const float di = clip(part_value(s, 1, i), L.lo[1], L.hi[1]);
    diff[2 * i] = dr;
    diff[2 * i + 1] = di;
    n += (isnan(dr) || isnan(di)) ? 0 : 1;
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
  if (lane == 0) wn[w] = n;
  __syncthreads();
  if (tid == 0) {
    int t = 0;
    for (int j = 0; j < kNW; ++j) t += wn[j];
    nvalid[0] = (float)t;
  }
}

}  // namespace

void launch_stats(const float* e_l, const float* obs, const int32_t* n_acc, int B, int steps, int penalties,
                  float* out, hipStream_t s) {
  hipLaunchKernelGGL(stats_kernel, dim3(1), dim3(kNT), 0, s, e_l, obs, n_acc, B, steps, penalties, out);
}

void launch_loss_diff(const float* e_l, const float* obs, int B, const float* g, float lz_penalty, float lz_center,
                      float l2_penalty, float* diff, float* nvalid, hipStream_t s) {
  // g = device pointer to the reduced stats (DH_STAT_* layout)
  Src src{e_l, obs, 1, 0.f, 0.f, lz_penalty, lz_center, l2_penalty, 0.f, 0.f, 0.f};
  hipLaunchKernelGGL(diff_kernel, dim3(1), dim3(kNT), 0, s, src, g, B, diff, nvalid);
}

}  // namespace dh
