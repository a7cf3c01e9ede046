// Input layer: electron features of every channel times W0 (psiformer.py:42,51-60),
// and — folded — layer 1's attention projections q|k|v = f (W0 Wqkv) + b (the
// product of two linear maps with nothing in between; W0 Wqkv is formed on the host
// in float64).  This replaces the first K=256 GEMM by a K=4 streaming kernel.
//
// Channel c of row (walker b, electron i):
//   c = 0        [cos th, sin th cos ph, sin th sin ph, s_i]                 (value)
//   c = 1+t      derivative along seed t (only if t/2 == i):
//                t even: d/dth  = [-sin th, cos th cos ph, cos th sin ph, 0]
//                t odd : d/dph / sin th = [0, -sin ph, cos ph, 0]
//   c = 2N+1     Laplace-Beltrami of r_hat = -2 r_hat
//   c = 2N+2+k   second derivative along the rotation flow about axis k:
//                e_k (e_k . r_hat) - r_hat
// Feature order is [z, x, y, spin] as in the reference's input_feature.
#include "dh_internal.h"
#include "device_common.h"

namespace dh {
namespace {

constexpr int kRows = 32;  // rows per workgroup

__global__ __launch_bounds__(256) void input_kernel(const float* __restrict__ x, const float* __restrict__ W0,
                                                    const float* __restrict__ W0qkv,
                                                    const float* __restrict__ bqkv, float* __restrict__ h,
                                                    float* __restrict__ qkv, float* __restrict__ geo, int rows,
                                                    int N, int n_up, int C, int D) {
  extern __shared__ float4 smem4[];
  const int E = qkv ? 4 * D : D;  // output columns per row (h, then q|k|v)
  float4* Ws = smem4;             // [4][E/4]: W0 rows then W0qkv rows, per input feature
  float4* F = Ws + E;             // [kRows] features
  const int tid = threadIdx.x;
  const int E4 = E / 4, D4 = D / 4;
  for (int q = tid; q < 4 * E4; q += blockDim.x) {
    const int k = q / E4, c4 = q - k * E4;
    Ws[q] = (c4 < D4) ? reinterpret_cast<const float4*>(W0 + (size_t)k * D)[c4]
                      : reinterpret_cast<const float4*>(W0qkv + (size_t)k * 3 * D)[c4 - D4];
  }
  const int row0 = blockIdx.x * kRows;
  if (tid < kRows && row0 + tid < rows) {
    const int row = row0 + tid;
    const int c = row % C;
    const int e = row / C;  // walker*N + electron
    const int i = e % N;
    const float th = x[2 * e], ph = x[2 * e + 1];
    float st, ct, sp, cp;
    sincosf(th, &st, &ct);
    sincosf(ph, &sp, &cp);
    const float rx = st * cp, ry = st * sp, rz = ct;
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    const int T = 2 * N;
    if (c == 0) {
      f = make_float4(rz, rx, ry, (i < n_up) ? 1.f : -1.f);
      *reinterpret_cast<float4*>(geo + 4 * (size_t)e) = make_float4(st, ct, sp, cp);
    } else if (c <= T) {
      const int t = c - 1;
      if ((t >> 1) == i) f = ((t & 1) == 0) ? make_float4(-st, ct * cp, ct * sp, 0.f) : make_float4(0.f, -sp, cp, 0.f);
    } else if (c == T + 1) {
      f = make_float4(-2.f * rz, -2.f * rx, -2.f * ry, 0.f);
    } else {
      const int k = c - T - 2;  // 0:x 1:y 2:z
      f = make_float4((k == 2) ? 0.f : -rz, (k == 0) ? 0.f : -rx, (k == 1) ? 0.f : -ry, 0.f);
    }
    F[tid] = f;
  }
  if (!h && !qkv) return;  // geometry only (the log-psi layer-1 residual is formed later)
  __syncthreads();
  const int nr = min(kRows, rows - row0);
  for (int q = tid; q < nr * E4; q += blockDim.x) {
    const int r = q / E4, c4 = q - r * E4;
    const float4 f = F[r];
    const float4 w0 = Ws[c4], w1 = Ws[E4 + c4], w2 = Ws[2 * E4 + c4], w3 = Ws[3 * E4 + c4];
    float4 o;
    o.x = f.x * w0.x + f.y * w1.x + f.z * w2.x + f.w * w3.x;
    o.y = f.x * w0.y + f.y * w1.y + f.z * w2.y + f.w * w3.y;
    o.z = f.x * w0.z + f.y * w1.z + f.z * w2.z + f.w * w3.z;
    o.w = f.x * w0.w + f.y * w1.w + f.z * w2.w + f.w * w3.w;
    const size_t row = (size_t)(row0 + r);
    if (c4 < D4) {
      reinterpret_cast<float4*>(h + row * D)[c4] = o;
    } else {
      const int q4 = c4 - D4;
      if (row % C == 0) {
        const float4 bb = reinterpret_cast<const float4*>(bqkv)[q4];
        o.x += bb.x;
        o.y += bb.y;
        o.z += bb.z;
        o.w += bb.w;
      }
      reinterpret_cast<float4*>(qkv + row * 3 * D)[q4] = o;
    }
  }
}

}  // namespace

void launch_input(const Dims& d, const float* x, const float* W0, const float* W0qkv, const float* bqkv, float* h,
                  float* qkv, float* geo, int nw, int C, hipStream_t s) {
  const int rows = nw * d.N * C;
  const int E = qkv ? 4 * d.D : d.D;
  const size_t smem = (size_t)(4 * E / 4 + kRows) * sizeof(float4);
  ensure_smem(input_kernel, smem);
  hipLaunchKernelGGL(input_kernel, dim3((rows + kRows - 1) / kRows), dim3(256), smem, s, x, W0, W0qkv, bqkv, h, qkv,
                     geo, rows, d.N, d.n_up, C, d.D);
}

}  // namespace dh
