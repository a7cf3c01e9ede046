// Input layer: electron features of every channel times W0 (psiformer.py:42,51-60).
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

__global__ void input_kernel(const float* __restrict__ x, const float* __restrict__ W0, float* __restrict__ h,
                             float* __restrict__ geo, int nw, int N, int n_up, int C, int D) {
  const int D4 = D >> 2;
  const long total = (long)nw * N * C * D4;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int d4 = idx % D4;
    const long row = idx / D4;
    const int c = row % C;
    const long e = row / C;  // walker*N + electron
    const int i = e % N;
    const float th = x[2 * e], ph = x[2 * e + 1];
    float st, ct, sp, cp;
    sincosf(th, &st, &ct);
    sincosf(ph, &sp, &cp);
    const float rx = st * cp, ry = st * sp, rz = ct;
    float f0 = 0.f, f1 = 0.f, f2 = 0.f, f3 = 0.f;
    const int T = 2 * N;
    if (c == 0) {
      f0 = rz;
      f1 = rx;
      f2 = ry;
      f3 = (i < n_up) ? 1.f : -1.f;
      if (d4 == 0) {
        float4 g = make_float4(st, ct, sp, cp);
        *reinterpret_cast<float4*>(geo + 4 * e) = g;
      }
    } else if (c <= T) {
      const int t = c - 1;
      if ((t >> 1) == i) {
        if ((t & 1) == 0) {
          f0 = -st;
          f1 = ct * cp;
          f2 = ct * sp;
        } else {
          f1 = -sp;
          f2 = cp;
        }
      }
    } else if (c == T + 1) {
      f0 = -2.f * rz;
      f1 = -2.f * rx;
      f2 = -2.f * ry;
    } else {
      const int k = c - T - 2;  // 0:x 1:y 2:z
      f0 = (k == 2) ? 0.f : -rz;
      f1 = (k == 0) ? 0.f : -rx;
      f2 = (k == 1) ? 0.f : -ry;
    }
    const float4 w0 = reinterpret_cast<const float4*>(W0)[d4];
    const float4 w1 = reinterpret_cast<const float4*>(W0 + D)[d4];
    const float4 w2 = reinterpret_cast<const float4*>(W0 + 2 * D)[d4];
    const float4 w3 = reinterpret_cast<const float4*>(W0 + 3 * D)[d4];
    float4 o;
    o.x = f0 * w0.x + f1 * w1.x + f2 * w2.x + f3 * w3.x;
    o.y = f0 * w0.y + f1 * w1.y + f2 * w2.y + f3 * w3.y;
    o.z = f0 * w0.z + f1 * w1.z + f2 * w2.z + f3 * w3.z;
    o.w = f0 * w0.w + f1 * w1.w + f2 * w2.w + f3 * w3.w;
    reinterpret_cast<float4*>(h + row * D)[d4] = o;
  }
}

}  // namespace

void launch_input(const Dims& d, const float* x, const float* W0, float* h, float* geo, int nw, int C,
                  hipStream_t s) {
  const long total = (long)nw * d.N * C * (d.D / 4);
  int blocks = (int)std::min<long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(input_kernel, dim3(blocks), dim3(256), 0, s, x, W0, h, geo, nw, d.N, d.n_up, C, d.D);
}

}  // namespace dh
