// Channel-row linear map + channel LayerNorm in ONE launch (local energy, D = 256):
//
//   MODE 0:  h = LN_ch(h + X W + b)            psiformer.py:44-46  (X = o, W = Wo Wl folded)
//   MODE 1:  h = LN_ch(h + tanh_ch(h W + b))   psiformer.py:47-48  (X = h)
//   MODE 2:  layer 1 whole (round 6), from the o~ rows of attention_feat2_kernel:
//            h = LN_ch2(h1 + tanh_ch(h1 Wm + bm)),  h1 = LN_ch1(f W0 + o~ U + b)
//
// in place over h [rows = ne * C][256], C = 2N + 5 channel rows per (walker, electron),
// bias b on the value rows only; LN_ch / tanh_ch are layernorm.hip's channel rules.  It
// replaces gemm_x6q (the GEMM writing t to HBM) + layernorm_ch_wave (reading t and h back):
// the GEMM output never leaves the CU.
//
// Why a new tile shape.  The channel LayerNorm of one electron mixes its C rows feature by
// feature (u_k = sum_t alpha_kt z_t, tanh_ch's sum_t z_t^2) and needs full-row sums over the
// 256 features (means, z0 . z_c, |z_t|^2, |u_k|^2).  Here the MFMA column dimension is the
// ELECTRON: a tile is 16 electrons x C channels (= 16 C rows, electron-aligned), and
// wave w computes output features 32 w .. 32 w + 31 of all C channels of all 16 electrons.
// With the weights as the MFMA A operand (v_mfma_f32_16x16x32_bf16: D col = lane & 15 =
// electron, D row = 4 (lane >> 4) + reg = feature), lane (e, g) ends the k loop holding,
// for electron e, features 32 w + 16 cb + 4 g .. +3 (cb = 0, 1) of EVERY channel row: the
// channel algebra is lane-local, the feature sums are 8 lane-local values and one LDS
// reduction over the 32 lanes (8 waves x 4 lane rows) holding that electron.
//
// Split-bf16 arithmetic (gemm_x6.hip header): weights as pre-split planes Wp[3][ldp][K]
// streamed L2 -> registers one k-step ahead (each wave uses only its own 32 feature columns,
// so they need no LDS); the activation k-step (16 C rows x 32 k f32) is loaded by all 512
// threads one step ahead into registers, split ONCE into three bf16 planes in LDS (every
// element split by one thread; the MFMA loop reads the planes, no VALU split in it), two
// plane buffers, one barrier per 32 k.  LDS plane image: [p][c][e][64 B], 16-B slot s of
// electron e at s ^ f(e), f = {0, 2, 3, 1}[(e >> 2) & 3] (conflict-free ds_read_b128 for the
// 16x16x32 lane groups, checked exhaustively).  Six MFMAs per product block, smallest
// terms first (as gemm_x6m).
//
// MODE 2: layer 1 in coefficient space.  Every pre-LN1 channel row is a combination of 26 fixed
// vectors: x_c = f_c W0 + o~_c U + [c = 0] b (f_c: the input features' channel seeds, 4; o~_c:
// the attention's feature-space outputs, 5 per head, dh_internal.h ofeat_k), and centring
// subtracts mean_c times the all-ones vector, so z_c = zh_c E with E = [W0; U; b; 1] and
// zh_c = (f_c, o~_c, [c = 0], -mean_c).  LN_ch1's outputs are linear in the z rows with
// per-electron scalars (s, a_t, cl, au_k, cs_k, computed from the real x rows as MODE 0 does),
// so h1_c = r_c B with r_c = the same combination of the zh rows and B = [E diag(gamma); beta]
// (27 rows), and h1_c Wm + bm = r_c V with V = B Wm (+ bm on the beta row): the 256-deep Wm
// product becomes a 32-deep one over the tile's r rows, and h1 never exists outside the
// registers.  Passes: o~ U (K = 32) -> LN1 statistics -> r rows into the planes -> r V (K = 32)
// -> tanh_ch -> += r B (K = 32: the residual h1) -> LN2 -> h.  The weights B, V (planes of B^T,
// V^T) are formed once per parameter upload (api.cpp, launch_l1_basis, f64 sums).
//
// Traffic per launch: X once (the k loop), h once (the epilogue; in MODE 1 the same rows
// as X, from MALL), h written once: 12 * rows * 256 B, against 20 (MODE 0) / 24 (MODE 1)
// for the two-kernel form; MODE 2: the o~ rows (128 B per row) read, h written once.
#include <cstdlib>

#include "dh_internal.h"
#include "device_common.h"

#ifndef LNCH_STAMP
#define LNCH_STAMP 0
#endif
#ifndef LNCH_STAMP_MODE  // stamp builds: only launches of this MODE write (-1: every launch)
#define LNCH_STAMP_MODE -1
#endif

namespace dh {

#if LNCH_STAMP
// diagnostic builds only (tools/lnch_one.py): per-workgroup phase timestamps (s_memtime) of
// the first LNCH_STAMP_WG tiles, written by thread 0 into a buffer nothing else reads
// (slots 0-6 the phases, 8-9 real time at start / end; MODE 2 also 10-14)
constexpr int LNCH_STAMP_WG = 4096, LNCH_NSTAMP = 16;
__device__ unsigned long long g_lnch_stamp[LNCH_STAMP_WG * LNCH_NSTAMP];
#define LNCH_T(i)                                                                    \
  do {                                                                               \
    if ((LNCH_STAMP_MODE < 0 || LNCH_STAMP_MODE == MODE) && threadIdx.x == 0 && blockIdx.x < LNCH_STAMP_WG) \
      g_lnch_stamp[blockIdx.x * LNCH_NSTAMP + (i)] = __builtin_amdgcn_s_memtime();   \
  } while (0)
#define LNCH_RT(i)                                                                   \
  do {                                                                               \
    if ((LNCH_STAMP_MODE < 0 || LNCH_STAMP_MODE == MODE) && threadIdx.x == 0 && blockIdx.x < LNCH_STAMP_WG) \
      g_lnch_stamp[blockIdx.x * LNCH_NSTAMP + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LNCH_T(i)
#define LNCH_RT(i)
#endif

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int LN_NWV = 8;   // waves per workgroup (one workgroup per CU)
constexpr int LN_EPT = 16;  // electrons per tile (the MFMA column dimension)
constexpr int LN_D = 256;   // features (= K of MODE 1)
constexpr int LN_BK = 32;   // k per step
constexpr int LN_KB = 32;   // MODE 2: coefficient-row length (27 used: 4 + 5 H + 3, H = 4)
constexpr int LN_SCF = 32;  // MODE 2: floats of one electron's LN_ch1 scalar table (8 + T <= 32)
// epilogue residual through LDS: chunks of LN_RCH channel rows of all 16 electrons (LN_RCH * 16
// rows of 1 KB) in two buffers over the stage area
constexpr int LN_RCH = 4;
constexpr int LN_RBUF = LN_RCH * LN_EPT * LN_D * 4;  // bytes of one chunk buffer

__host__ __device__ constexpr int lnch_nr(int N) { return (2 * N + 5) + 2 * N + 3; }  // second moments
__host__ __device__ constexpr int lnch_ts(int N) { return lnch_nr(N) | 1; }          // odd stride
// LDS bytes: the two k-step plane stages / the residual chunk buffers (the epilogue's reduction
// scratch and totals, then MODE 2's zh rows), then the walkers' geometry
__host__ __device__ constexpr int lnch_geo_off(int N) {
  return (6 * (2 * N + 5) * LN_EPT * 64 > 2 * LN_RBUF) ? 6 * (2 * N + 5) * LN_EPT * 64 : 2 * LN_RBUF;
}
__host__ __device__ constexpr int lnch_smem(int N) { return lnch_geo_off(N) + ((LN_EPT + N - 1) / N + 1) * N * 16; }
__host__ __device__ constexpr int lnch_z_off(int N) {
  return (LN_NWV * lnch_nr(N) * 64 * 4 + LN_EPT * lnch_ts(N) * 4 + 15) & ~15;
}

__device__ __forceinline__ uint32_t pkbf(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){x, y}, bf16x2));
}
__device__ __forceinline__ float lo_of(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_of(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ int lnch_sw(int e) { return (0x78 >> (2 * ((e >> 2) & 3))) & 3; }
// 4 consecutive k values of one (channel, electron) row as their three bf16 terms, at byte
// offset loff of each plane (the k-step plane image above)
__device__ __forceinline__ void put_split4(char* P, int plane, int loff, float x, float y, float z, float w) {
  const uint32_t h0 = pkbf(x, y), h1 = pkbf(z, w);
  const float rx = x - lo_of(h0), ry = y - hi_of(h0), rz = z - lo_of(h1), rw = w - hi_of(h1);
  const uint32_t m0 = pkbf(rx, ry), m1 = pkbf(rz, rw);
  const uint32_t s0 = pkbf(rx - lo_of(m0), ry - hi_of(m0)), s1 = pkbf(rz - lo_of(m1), rw - hi_of(m1));
  *reinterpret_cast<uint2*>(P + loff) = make_uint2(h0, h1);
  *reinterpret_cast<uint2*>(P + plane + loff) = make_uint2(m0, m1);
  *reinterpret_cast<uint2*>(P + 2 * plane + loff) = make_uint2(s0, s1);
}
// input.hip's channel seed f_c of electron ie (geometry st ct sp cp) for channel c
template <int N>
__device__ __forceinline__ float4 chan_feature(int c, int ie, float4 g4, int n_up) {
  constexpr int T = 2 * N;
  const float st = g4.x, ct = g4.y, sp = g4.z, cp = g4.w;
  const float rx = st * cp, ry = st * sp, rz = ct;
  float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c == 0) {
    f = make_float4(rz, rx, ry, (ie < n_up) ? 1.f : -1.f);
  } else if (c <= T) {
    const int t = c - 1;
    if ((t >> 1) == ie) f = ((t & 1) == 0) ? make_float4(-st, ct * cp, ct * sp, 0.f) : make_float4(0.f, -sp, cp, 0.f);
  } else if (c == T + 1) {
    f = make_float4(-2.f * rz, -2.f * rx, -2.f * ry, 0.f);
  } else {
    const int k = c - T - 2;  // 0:x 1:y 2:z
    f = make_float4((k == 2) ? 0.f : -rz, (k == 0) ? 0.f : -rx, (k == 1) ? 0.f : -ry, 0.f);
  }
  return f;
}
// flow coefficient alpha_kt (layernorm.hip) from the walker's geometry gw[electron]
__device__ __forceinline__ float alpha_of(const float4* gw, int k, int t) {
  const float4 q = gw[t >> 1];
  if ((t & 1) == 0) return k == 0 ? -q.z : (k == 1 ? q.w : 0.f);
  return k == 0 ? -(q.y * q.w) : (k == 1 ? -(q.y * q.z) : q.x);
}
// the channel LayerNorm's per-electron scalars from its second moments mt (lnch_nr of them:
// <z0 z_c>, <z_t^2>, <u_k^2>)
template <int N>
struct LnScalars {
  float s, s2, cl, aL, au[3], cs[3];
  __device__ __forceinline__ void from(const float* mt, const float4* gw) {
    constexpr int C = 2 * N + 5, T = 2 * N;
    s = 1.f / sqrtf(mt[0] + 1e-5f);
    s2 = s * s;
    cl = 0.f;
    au[0] = au[1] = au[2] = 0.f;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float a = s2 * mt[1 + t];
      cl += 3.f * a * a - s2 * mt[C + t];
#pragma unroll
      for (int k = 0; k < 3; ++k) au[k] = fmaf(alpha_of(gw, k, t), a, au[k]);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) cs[k] = 3.f * au[k] * au[k] - s2 * mt[C + T + k];
    aL = s2 * mt[1 + T];
  }
};

template <int N, int MODE, bool FRES = false>
__global__ __launch_bounds__(LN_NWV * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_lnch_kernel(
    const float* X, const uint16_t* __restrict__ Wp, int ldp, const float* __restrict__ bias,
    const float* __restrict__ ln, const float* __restrict__ geo, float* h, int ne, const float* __restrict__ W0f,
    int n_up, int kx, const uint16_t* __restrict__ Wv, const uint16_t* __restrict__ Wb) {
  // K: the contraction length = X's row length, a multiple of BK (256; layer 1 from the o~
  // rows: ofeat_k, dh_internal.h); a compile-time 256 in MODE 1
  constexpr int NWV = LN_NWV, C = 2 * N + 5, T = 2 * N, EPT = LN_EPT, D = LN_D, BK = LN_BK;
  const int K = MODE == 1 ? LN_D : kx, NK = K / BK;
  constexpr int ROWS = EPT * C;                    // activation rows per tile
  constexpr int NT = NWV * 64, CB = D / (16 * NWV);  // threads; 16-column blocks per wave
  constexpr int PLANE = C * EPT * 64;              // bytes of one bf16 plane per step
  constexpr int STAGE = 3 * PLANE;
  constexpr int NQ = (ROWS * 8 + NT - 1) / NT;     // 16-B activation pieces per thread per step
  constexpr int NR = lnch_nr(N);                   // second-moment statistics per electron
  constexpr int TS = lnch_ts(N);
  constexpr int KB = LN_KB;
  static_assert(2 * STAGE <= lnch_geo_off(N) && lnch_smem(N) <= 163840, "LDS");
  static_assert(NWV * NR * 64 * 4 + EPT * TS * 4 <= 2 * STAGE, "reduction scratch");
  static_assert(MODE != 2 || lnch_z_off(N) + (EPT * C * KB + EPT * LN_SCF) * 4 <= lnch_geo_off(N), "MODE 2 zh rows");
  static_assert(MODE != 2 || (EPT * KB == NT && 8 + T <= LN_SCF), "MODE 2: thread (electron, column)");
  static_assert(MODE != 2 || NWV * NR * 64 * 4 >= STAGE, "MODE 2: the r planes stay clear of the totals");
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kg = lane >> 4;
  const int tile = blockIdx.x;
  // every barrier here orders LDS only (planes, residual chunks after their counted DMA waits,
  // statistics): global loads in flight may cross it
  auto lbar = []() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const int e0 = tile * EPT;                       // first electron of the tile
  const size_t row0 = (size_t)e0 * C;
  const int rows_valid = min(ROWS, (ne - e0) * C);
  LNCH_T(0);
  LNCH_RT(8);

  // geometry of the walkers the tile's electrons belong to, staged once in LDS past the
  // stage buffers (visible after the k loop's barriers)
  constexpr int GW = (EPT + N - 1) / N + 1;  // walkers a 16-electron tile can touch
  float4* gl = reinterpret_cast<float4*>(smem + lnch_geo_off(N));
  if (tid < GW * N) {
    const int ge = (e0 / N) * N + tid;
    gl[tid] = ge < ne ? reinterpret_cast<const float4*>(geo)[ge] : make_float4(0.f, 1.f, 0.f, 1.f);
  }
  // ---- activation pieces of this thread: piece i = tid + NT j -> (row i >> 3, quad i & 7)
  // buffer descriptor over the tile's activation rows (tile-uniform base; rows past the last
  // electron are out of range: their loads return 0)
  const uint32_t xbytes = (uint32_t)rows_valid * K * 4;
  const auto rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X) + row0 * K, (short)0, xbytes, 0x00020000);
  int goff[NQ], loff[NQ];
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    const int i = tid + NT * j;
    const int r = i >> 3, q = i & 7;
    const int e = r / C, c = r - e * C;
    goff[j] = i < ROWS * 8 ? (r * K + 4 * q) * 4 : 0x7fffffff;  // bytes from row0 (k step in soffset)
    loff[j] = (c * EPT + e) * 64 + (((q >> 1) ^ lnch_sw(e)) * 16) + (q & 1) * 8;
    if (!(i < ROWS * 8)) loff[j] = -1;
  }
  auto load_a = [&](int kt, float4 (&ra)[NQ]) {
#pragma unroll
    for (int j = 0; j < NQ; ++j)
      ra[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsX, goff[j], kt * BK * 4, 0));
  };
  auto split_store = [&](const float4 (&ra)[NQ], int buf) {
    char* P = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      if (loff[j] < 0) continue;
      const float4 u = ra[j];
      put_split4(P, PLANE, loff[j], u.x, u.y, u.z, u.w);
    }
  };
  // ---- weight fragments of this wave: feature n = 16 (CB wid + cb) + l16, k = 32 kt + 8 kg
  const uint16_t* wbase = Wp + (size_t)(16 * CB * wid + l16) * K + 8 * kg;
  const size_t wplane = (size_t)ldp * K;
  auto load_w = [&](int kt, int cb, bf16x8 (&wf)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
      wf[p] = *reinterpret_cast<const bf16x8*>(wbase + p * wplane + (size_t)cb * 16 * K + kt * BK);
  };
  const int xoff = l16 * 64 + ((kg ^ lnch_sw(l16)) * 16);  // + c * EPT * 64 within a plane

  // ---- the residual rows h through LDS by DMA (global_load_lds_dwordx4, no VGPRs): chunk k =
  // channel rows LN_RCH k .. + LN_RCH - 1 of the tile's 16 electrons, one 1-KB row per wave
  // instruction, into chunk buffer k & 1 at row q = (c - LN_RCH k) * 16 + e.  16-B slot s of
  // a row holds the row's quad s ^ e (the swizzle is on the SOURCE address: the DMA writes
  // lane-linearly), so the epilogue's ds_read_b128 of quad Q = 8 w + 4 cb + g by lane (e, g)
  // hits slot Q ^ e: 16 distinct slots in every lane group.  Rows of electrons past the end
  // re-read the tile's first row into their (never read) slot, so every wave issues the same
  // compile-time number of DMAs per chunk and "chunk k landed" is vmcnt(DMAs of chunk k + 1).
  constexpr int NCHK = (C + LN_RCH - 1) / LN_RCH;
  auto rows_of = [](int k) { return EPT * (C - LN_RCH * k < LN_RCH ? C - LN_RCH * k : LN_RCH); };
  static_assert(EPT * LN_RCH % NWV == 0 && EPT % NWV == 0, "DMA rows must divide over the waves");
  const uint32_t lds0 = (uint32_t)(size_t)((__attribute__((address_space(3))) char*)smem);
  auto rdma = [&](int k) {
    const int nrow = rows_of(k);
#pragma unroll
    for (int j = 0; j < LN_RCH * EPT / NWV; ++j) {
      const int q = wid + NWV * j;  // wave-uniform
      if (q < nrow) {
        const int c = LN_RCH * k + q / EPT, e = q % EPT;
        const int er = e0 + e < ne ? e : 0;
        // row base in SGPRs, the lane's swizzled 16-B quad as a 32-bit VGPR offset (formed here,
        // not hoisted: 64-bit per-lane addresses of every chunk held across the epilogue spill)
        const float* rowp = h + (row0 + (size_t)(er * C + c)) * D;
        const int le = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        uint32_t voff = (uint32_t)(le ^ e) << 4;
        asm volatile("" : "+v"(voff));
        const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)((k & 1) * LN_RBUF + q * D * 4));
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(rowp), "s"(dst)
                     : "memory");
      }
    }
  };
  // layer 1 (MODE 0 with W0f, MODE 2): the residual h0 = f W0 is formed from the walkers'
  // geometry in the epilogue (round 5), so h0 is never written by the input kernel nor read back
  constexpr bool fres = (MODE == 0 && FRES) || MODE == 2;
  // the accumulators start from zero (the residual is added in the epilogue: starting them
  // from h rounds every k-step's partial sum at |h| and measurably loosened the tangent
  // channels against float64 on ill-conditioned walkers)
  f32x4 acc[C][CB];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc[c][cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  {
    // column block outermost: one block's weight fragments (12 VGPRs) live at a time, the next
    // block's streaming in behind them; the activation fragments are re-read from LDS per block
    float4 ra[NQ];
    bf16x8 wf[3], wn[3];
    load_a(0, ra);
    load_w(0, 0, wf);
    split_store(ra, 0);
    if (NK > 1) load_a(1, ra);
#pragma unroll 1
    for (int kt = 0; kt < NK; ++kt) {
      lbar();  // planes of step kt complete; step kt - 1's buffer is free
      if (kt == 0) LNCH_T(1);
      const char* P = smem + (kt & 1) * STAGE + xoff;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        // a compiler memory fence per block: the fragments are re-read, not kept live (CSE
        // across blocks would hold all C channels' fragments in registers)
        asm volatile("" ::: "memory");
        if (cb + 1 < CB)
          load_w(kt, cb + 1, wn);
        else if (kt + 1 < NK)
          load_w(kt + 1, 0, wn);
        bf16x8 xf[2][3];
        auto ldx = [&](int c, bf16x8 (&x)[3]) {
          x[0] = *reinterpret_cast<const bf16x8*>(P + c * EPT * 64);
          x[1] = *reinterpret_cast<const bf16x8*>(P + PLANE + c * EPT * 64);
          x[2] = *reinterpret_cast<const bf16x8*>(P + 2 * PLANE + c * EPT * 64);
        };
        ldx(0, xf[0]);
#pragma unroll
        for (int c = 0; c < C; ++c) {
          if (c + 1 < C) ldx(c + 1, xf[(c + 1) & 1]);  // one channel ahead
          const bf16x8 x0 = xf[c & 1][0], x1 = xf[c & 1][1], x2 = xf[c & 1][2];
          f32x4 a = acc[c][cb];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0], x2, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[2], x0, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1], x1, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0], x1, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1], x0, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0], x0, a, 0, 0, 0);
          acc[c][cb] = a;
          if (cb == 0 && c == C / 2 && kt + 1 < NK) {
            split_store(ra, (kt + 1) & 1);
            if (kt + 2 < NK) load_a(kt + 2, ra);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) wf[p] = wn[p];
      }
    }
  }
  lbar();  // every wave is past its last plane read: the stage buffers become scratch
  LNCH_T(2);
  // the epilogue's lane indices, re-derived from the lane id (mbcnt) rather than kept live
  // across the k loop from threadIdx (holding them there made MODE 1 spill)
  const int lane_e = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (MODE == 0 && !fres) {
    rdma(0);
    if (NCHK > 1) rdma(1);
  }
  const int l16e = lane_e & 15, kge = lane_e >> 4, tide = wid * 64 + lane_e;
  // lane = electron l16 of the tile; its accumulators hold features nf + 16 cb + 0..3 of every
  // channel row (MFMA D layout: col = lane & 15, row = 4 (lane >> 4) + reg)
  const int E = e0 + l16e;
  const bool valid = E < ne;
  const int b = (valid ? E : e0) / N;
  const int nf = 16 * CB * wid + 4 * kge;  // + 16 cb
  // this lane's rows of h (invalid electrons read the tile's first rows and store nothing);
  // 32-bit offsets from the tile's base, each passed through an opaque asm so the compiler
  // forms them one at a time (precomputing all 2 C row addresses spills)
  char* const htile = reinterpret_cast<char*>(h + row0 * D);  // tile-uniform base (SGPRs)
  const uint32_t hv = (uint32_t)(((valid ? l16e : 0) * C * D + nf) * 4);
  auto roff = [&](int c, int cb) {  // 32-bit byte offset of (row c, block cb): saddr + voffset
    uint32_t o = hv + (uint32_t)((c * D + 16 * cb) * 4);
    asm volatile("" : "+v"(o));
    return o;
  };
  auto sth = [&](int c, int cb, float4 v) {
    if (valid) *reinterpret_cast<float4*>(htile + roff(c, cb)) = v;
  };

  // ---- epilogue: lane = electron l16, features nf + 16 cb + 0..3 of every channel row
  // geometry of the walker's electrons (st, ct, sp, cp) from the tile's LDS copy (read where
  // used: holding N float4 per lane would spill the accumulators)
  const float4* gw = gl + (b - e0 / N) * N;
  // tanh_ch of the pre-activation rows in acc (layernorm.hip: y0 = tanh z0, y_t = d1 z_t,
  // y_L = d1 z_L + d2 sum_t z_t^2, y_Sk = d1 z_Sk + d2 u_k^2)
  float chain = 0.f;
  auto tanh_ch = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      // the value row's tanh first, one feature at a time (its temporaries never overlap
      // the channel algebra's); tanh_ocml = tanhf bit for bit, without tanhf's branch
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        acc[0][cb][v] = tanh_ocml(acc[0][cb][v]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float y0 = acc[0][cb][v], d1 = 1.f - y0 * y0, d2 = -2.f * y0 * d1;
        float sq = 0.f, u0 = 0.f, u1 = 0.f, u2 = 0.f;
        // the geometry is re-read per feature, not held (spills): its offset is opaque and
        // depends on the previous feature's last result, so the reads cannot be batched early
        int gi = 0;
        asm volatile("" : "+v"(gi) : "v"(y0), "v"(chain));
#pragma unroll
        for (int i = 0; i < N; ++i) {
          const float4 q = gw[gi + i];
          const float za = acc[1 + 2 * i][cb][v], zb = acc[2 + 2 * i][cb][v];
          sq = fmaf(za, za, fmaf(zb, zb, sq));
          u0 = fmaf(-q.z, za, fmaf(-(q.y * q.w), zb, u0));
          u1 = fmaf(q.w, za, fmaf(-(q.y * q.z), zb, u1));
          u2 = fmaf(q.x, zb, u2);
          acc[1 + 2 * i][cb][v] = d1 * za;
          acc[2 + 2 * i][cb][v] = d1 * zb;
        }
        acc[1 + T][cb][v] = d1 * acc[1 + T][cb][v] + d2 * sq;
        acc[2 + T][cb][v] = d1 * acc[2 + T][cb][v] + d2 * (u0 * u0);
        acc[3 + T][cb][v] = d1 * acc[3 + T][cb][v] + d2 * (u1 * u1);
        acc[4 + T][cb][v] = d1 * acc[4 + T][cb][v] + d2 * (u2 * u2);
        chain = acc[4 + T][cb][v];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // pre-LN rows x_c (in acc): bias (value rows), MODE 1's tanh_ch, then + h
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + nf + 16 * cb) : make_float4(0.f, 0.f, 0.f, 0.f);
    acc[0][cb][0] += bv.x;
    acc[0][cb][1] += bv.y;
    acc[0][cb][2] += bv.z;
    acc[0][cb][3] += bv.w;
  }
  if constexpr (MODE == 1) {
    tanh_ch();
    // the tanh_ch results are materialised here, before the DMA blocks (otherwise the
    // compiler sinks the channel algebra past them and its live ranges spill)
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) asm volatile("" : "+v"(acc[c][cb]));
    rdma(0);
    if (NCHK > 1) rdma(1);
  }
  if constexpr (fres) {
    // input.hip's channel features of this lane's electron (the geometry staged in gl) times
    // W0's columns nf + 16 cb .. + 3, the input kernel's expression, then added as the
    // residual rows are (r + acc)
    const float4 g4 = gl[valid ? E - (e0 / N) * N : 0];  // st ct sp cp
    const int ie = (valid ? E : e0) % N;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const float4 w0 = *reinterpret_cast<const float4*>(W0f + nf + 16 * cb);
      const float4 w1 = *reinterpret_cast<const float4*>(W0f + D + nf + 16 * cb);
      const float4 w2 = *reinterpret_cast<const float4*>(W0f + 2 * D + nf + 16 * cb);
      const float4 w3 = *reinterpret_cast<const float4*>(W0f + 3 * D + nf + 16 * cb);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float4 f = chan_feature<N>(c, ie, g4, n_up);
        f32x4& a = acc[c][cb];
        a[0] = (f.x * w0.x + f.y * w1.x + f.z * w2.x + f.w * w3.x) + a[0];
        a[1] = (f.x * w0.y + f.y * w1.y + f.z * w2.y + f.w * w3.y) + a[1];
        a[2] = (f.x * w0.z + f.y * w1.z + f.z * w2.z + f.w * w3.z) + a[2];
        a[3] = (f.x * w0.w + f.y * w1.w + f.z * w2.w + f.w * w3.w) + a[3];
      }
    }
  } else {
    // this lane's row in a chunk buffer (+ channel / buffer offsets) and its two quad slots
    const char* const rb0 = smem + l16e * D * 4;
    int rsl[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) rsl[cb] = 16 * ((4 * CB * wid + 4 * cb + kge) ^ l16e);
#pragma unroll
    for (int k = 0; k < NCHK; ++k) {
      // this wave's chunk-k DMAs landed (the younger ones are chunk k + 1's, issued before this
      // wait), then every wave's
      if (k + 1 < NCHK)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"((k + 1 < NCHK ? rows_of(k + 1) : 0) / NWV) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lbar();
#pragma unroll
      for (int cc = 0; cc < LN_RCH; ++cc) {
        const int c = LN_RCH * k + cc;
        if (c < C) {
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) {
            const float4 r = *reinterpret_cast<const float4*>(rb0 + (k & 1) * LN_RBUF + cc * EPT * D * 4 + rsl[cb]);
            f32x4& a = acc[c][cb];
            a[0] = r.x + a[0];
            a[1] = r.y + a[1];
            a[2] = r.z + a[2];
            a[3] = r.w + a[3];
            asm volatile("" : "+v"(a));  // consumed here (keeps the reads from being batched)
          }
        }
      }
      if (k + 2 < NCHK) {
        lbar();  // every wave is done with chunk k's buffer
        rdma(k + 2);
      }
    }
    lbar();  // the chunk buffers become the statistics scratch
    LNCH_T(3);
  }
  float* red = reinterpret_cast<float*>(smem);   // [NWV waves][NR][64 lanes] partial sums
  float* tot = red + NWV * NR * 64;               // [EPT][TS] totals (odd stride: 16 banks)
  auto lane_sum = [&](int c) {
    float r = 0.f;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) r += (acc[c][cb][0] + acc[c][cb][1]) + (acc[c][cb][2] + acc[c][cb][3]);
    return r;
  };
  // reduce NS per-lane partials part(j) over the tile's 256 features -> mean in tot[e][j]
  auto reduce = [&](auto part, auto NS_) {
    constexpr int NS = decltype(NS_)::value;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      red[(wid * NS + j) * 64 + lane_e] = part(j);  // every lane's 8-feature partial (no cross-lane ops)
      __builtin_amdgcn_sched_barrier(0);          // one statistic at a time (register pressure)
    }
    lbar();
    for (int i = tide; i < NS * EPT; i += NT) {
      const int j = i / EPT, e = i - j * EPT;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w)
#pragma unroll
        for (int g = 0; g < 4; ++g) s += red[(w * NS + j) * 64 + 16 * g + e];
      tot[e * TS + j] = s * (1.f / D);
    }
    lbar();
  };
  const float* mt = tot + l16e * TS;  // this lane's electron
  auto center = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float mu = mt[c];
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[c][cb][v] -= mu;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // flow vector u_k = sum_t alpha_kt z_t of columns block cb (recomputed where needed)
  auto flow = [&](int k, int cb) {
    f32x4 r = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (k == 2 && (t & 1) == 0) continue;  // alpha_2,2i = 0
      const float a = alpha_of(gw, k, t);
      r[0] = fmaf(a, acc[1 + t][cb][0], r[0]);
      r[1] = fmaf(a, acc[1 + t][cb][1], r[1]);
      r[2] = fmaf(a, acc[1 + t][cb][2], r[2]);
      r[3] = fmaf(a, acc[1 + t][cb][3], r[3]);
    }
    return r;
  };
  auto dot4 = [](const f32x4& x, const f32x4& y) { return (x[0] * y[0] + x[1] * y[1]) + (x[2] * y[2] + x[3] * y[3]); };
  // p_c = <z0 z_c>, q_t = <z_t^2>, uu_k = <u_k^2>
  auto reduce2 = [&]() __attribute__((always_inline)) {
    reduce(
        [&](int j) {
          float r = 0.f;
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) {
            if (j < C) {
              r += dot4(acc[0][cb], acc[j][cb]);
            } else if (j < C + T) {
              r += dot4(acc[1 + j - C][cb], acc[1 + j - C][cb]);
            } else {
              const f32x4 u = flow(j - C - T, cb);
              r += dot4(u, u);
            }
          }
          return r;
        },
        std::integral_constant<int, NR>{});
  };
  // channel means, centre
  reduce([&](int c) { return lane_sum(c); }, std::integral_constant<int, C>{});
  LNCH_T(4);
  if constexpr (MODE == 2) {
    // ---- zh rows (header): thread (e, c) -> Z[e][c][0..31] = (f_c, o~_c (5 per head), [c = 0],
    // -mean_c, 0 ...), o~ re-read from global memory (the tile's rows, L2-resident)
    float* Z = reinterpret_cast<float*>(smem + lnch_z_off(N));
    if (tid < EPT * C) {
      const int e = tid / C, c = tid - (tid / C) * C;
      const int Ee = e0 + e;
      const float4 g4 = gl[Ee < ne ? Ee - (e0 / N) * N : 0];
      const float4 f = chan_feature<N>(c, (Ee < ne ? Ee : e0) % N, g4, n_up);
      float* zr = Z + (e * C + c) * KB;
      *reinterpret_cast<float4*>(zr) = f;
      const int ro = (e * C + c) * K * 4;  // bytes from the tile's first o~ row (range-checked)
#pragma unroll
      for (int hh = 0; hh < 4; ++hh) {
        const float4 o4 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsX, ro + 32 * hh, 0, 0));
        const float o5 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsX, ro + 32 * hh + 16, 0, 0));
        zr[4 + 5 * hh] = o4.x;
        zr[5 + 5 * hh] = o4.y;
        zr[6 + 5 * hh] = o4.z;
        zr[7 + 5 * hh] = o4.w;
        zr[8 + 5 * hh] = o5;
      }
      zr[24] = c == 0 ? 1.f : 0.f;
      zr[25] = -tot[e * TS + c];
#pragma unroll
      for (int j = 26; j < KB; ++j) zr[j] = 0.f;
    }
    // (the next barrier is reduce2's, after every lane's partials are written)
  }
  center();
  reduce2();
  LNCH_T(5);
  if constexpr (MODE == 2) {
    // ---- r rows: LN_ch1's combinations of the zh rows (the output block's formulas below, with
    // z -> zh), written into plane buffer 0 as the next B operand.  First the per-electron
    // scalars into a table past the zh rows (thread e), then thread (e, j) forms column j of
    // every channel row of electron e: C + 4 T FMAs from C zh values, no serial chains.
    {
      const float* Z = reinterpret_cast<const float*>(smem + lnch_z_off(N));
      float* SC = reinterpret_cast<float*>(smem + lnch_z_off(N)) + EPT * C * KB;  // [EPT][LN_SCF]
      if (tid < EPT) {
        const int Ee = e0 + tid;
        const float4* gwe = gl + ((Ee < ne ? Ee : e0) / N - e0 / N) * N;
        LnScalars<N> S1;
        S1.from(tot + tid * TS, gwe);
        float* sc = SC + tid * LN_SCF;
        sc[0] = S1.s;
        sc[1] = S1.aL - S1.cl;  // y_L = s (z_L - (aL - cl) z0 - 2 sum_t a_t z_t)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          sc[2 + k] = S1.s2 * tot[tid * TS + 2 + T + k] - S1.cs[k];  // y_Sk = s (z_Sk - (ak - cs_k) z0 - 2 au_k u_k)
          sc[5 + k] = 2.f * S1.au[k];
        }
#pragma unroll
        for (int t = 0; t < T; ++t) sc[8 + t] = S1.s2 * tot[tid * TS + 1 + t];  // a_t
      }
      lbar();
      const int e = tid >> 5, j = tid & 31, Ee = e0 + e;
      const float4* gwe = gl + ((Ee < ne ? Ee : e0) / N - e0 / N) * N;
      const float* sc = SC + e * LN_SCF;
      const float* zc = Z + (e * C) * KB + j;  // + c KB
      const float sv = sc[0], z0 = zc[0];
      float sat = 0.f, u0 = 0.f, u1 = 0.f, u2 = 0.f;
      char* P = smem;  // plane buffer 0 (clear of the totals: static_assert above)
      const int lo = e * 64 + ((((j >> 2) >> 1) ^ lnch_sw(e)) * 16) + ((j >> 2) & 1) * 8 + (j & 3) * 2;
      auto put = [&](int c, float y) __attribute__((always_inline)) {  // element (c, e, k = j), three bf16 terms
        const uint32_t h2 = pkbf(y, 0.f);
        const float ry = y - lo_of(h2);
        const uint32_t m2 = pkbf(ry, 0.f);
        const uint32_t l2 = pkbf(ry - lo_of(m2), 0.f);
        char* q = P + c * EPT * 64 + lo;
        *reinterpret_cast<uint16_t*>(q) = (uint16_t)h2;
        *reinterpret_cast<uint16_t*>(q + PLANE) = (uint16_t)m2;
        *reinterpret_cast<uint16_t*>(q + 2 * PLANE) = (uint16_t)l2;
      };
      put(0, j == 26 ? 1.f : sv * z0);  // row 26: the beta row (zh has 0 there)
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const float zt = zc[(1 + t) * KB], at = sc[8 + t];
        sat = fmaf(at, zt, sat);
        u0 = fmaf(alpha_of(gwe, 0, t), zt, u0);
        u1 = fmaf(alpha_of(gwe, 1, t), zt, u1);
        if (t & 1) u2 = fmaf(alpha_of(gwe, 2, t), zt, u2);
        put(1 + t, sv * (zt - at * z0));
      }
      put(1 + T, sv * (zc[(1 + T) * KB] - sc[1] * z0 - 2.f * sat));
      const float uk[3] = {u0, u1, u2};
#pragma unroll
      for (int k = 0; k < 3; ++k) put(2 + T + k, sv * (zc[(2 + T + k) * KB] - sc[2 + k] * z0 - sc[5 + k] * uk[k]));
    }
    LNCH_T(10);    lbar();
    // ---- 32-deep passes over the r planes (buffer 0): acc (+)= r W^T, W = Wv or Wb planes
    const int xo = l16e * 64 + ((kge ^ lnch_sw(l16e)) * 16);
    auto pass = [&](const uint16_t* __restrict__ Wq) __attribute__((always_inline)) {
      const uint16_t* wq = Wq + (size_t)(16 * CB * wid + l16e) * KB + 8 * kge;
      const size_t wpl = (size_t)ldp * KB;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        asm volatile("" ::: "memory");
        bf16x8 wf[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) wf[p] = *reinterpret_cast<const bf16x8*>(wq + p * wpl + (size_t)cb * 16 * KB);
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const char* P = smem + xo + c * EPT * 64;
          const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(P);
          const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(P + PLANE);
          const bf16x8 x2 = *reinterpret_cast<const bf16x8*>(P + 2 * PLANE);
          f32x4 a = acc[c][cb];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0], x2, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[2], x0, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1], x1, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0], x1, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1], x0, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0], x0, a, 0, 0, 0);
          acc[c][cb] = a;
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) acc[c][cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
    pass(Wv);   // the pre-activation h1 Wm + bm (bm on the beta row of V)
    LNCH_T(11);
    tanh_ch();
    LNCH_T(12);
    pass(Wb);   // + h1 (beta on the beta row of B)
    lbar();     // every wave is past its plane reads: the reduction scratch overlaps them
    LNCH_T(13);
    reduce([&](int c) { return lane_sum(c); }, std::integral_constant<int, C>{});
    center();
    reduce2();
    LNCH_T(14);
  }
  LnScalars<N> S;
  S.from(mt, gw);
  const float s = S.s;
  // the LayerNorm scale / shift of both column blocks before the first store: a load between
  // two stores waits for every earlier store (vmcnt counts in order)
  float4 lng[CB], lnb[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    lng[cb] = *reinterpret_cast<const float4*>(ln + nf + 16 * cb);
    lnb[cb] = *reinterpret_cast<const float4*>(ln + D + nf + 16 * cb);
  }
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const float4 gv = lng[cb];
    const float4 bb = lnb[cb];
    const float gg[4] = {gv.x, gv.y, gv.z, gv.w}, bq[4] = {bb.x, bb.y, bb.z, bb.w};
    float gs[4], z0[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      gs[v] = gg[v] * s;
      z0[v] = acc[0][cb][v];
    }
    sth(0, cb, make_float4(gg[0] * (s * z0[0]) + bq[0], gg[1] * (s * z0[1]) + bq[1], gg[2] * (s * z0[2]) + bq[2],
                           gg[3] * (s * z0[3]) + bq[3]));
    float sat[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float at = S.s2 * mt[1 + t];
      float y[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float zt = acc[1 + t][cb][v];
        sat[v] = fmaf(at, zt, sat[v]);
        y[v] = gs[v] * (zt - at * z0[v]);
      }
      sth(1 + t, cb, make_float4(y[0], y[1], y[2], y[3]));
      __builtin_amdgcn_sched_barrier(0);
    }
    {
      float y[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) y[v] = gs[v] * (acc[1 + T][cb][v] - S.aL * z0[v] - 2.f * sat[v] + S.cl * z0[v]);
      sth(1 + T, cb, make_float4(y[0], y[1], y[2], y[3]));
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const f32x4 uk = flow(k, cb);
      const float ak = S.s2 * mt[2 + T + k];
      float y[4];
#pragma unroll
      for (int v = 0; v < 4; ++v)
        y[v] = gs[v] * (acc[2 + T + k][cb][v] - ak * z0[v] - 2.f * S.au[k] * uk[v] + S.cs[k] * z0[v]);
      sth(2 + T + k, cb, make_float4(y[0], y[1], y[2], y[3]));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  LNCH_T(6);
  LNCH_RT(9);
}

template <int N>
void launch_lnch_n(const float* X, const uint16_t* Wp, int ldp, const float* bias, const float* ln, const float* geo,
                   float* h, int ne, int mode, hipStream_t s, const float* W0f, int n_up, int K, const uint16_t* Wv,
                   const uint16_t* Wb) {
  const size_t smem = lnch_smem(N);
  const int grid = (ne + LN_EPT - 1) / LN_EPT;
  auto go = [&](auto kern) {
    ensure_smem(kern, smem);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(LN_NWV * 64), smem, s, X, Wp, ldp, bias, ln, geo, h, ne, W0f, n_up, K, Wv,
                       Wb);
  };
  if (mode == 2)
    go(gemm_lnch_kernel<N, 2>);
  else if (mode == 0 && W0f)
    go(gemm_lnch_kernel<N, 0, true>);
  else if (mode == 0)
    go(gemm_lnch_kernel<N, 0>);
  else
    go(gemm_lnch_kernel<N, 1>);
}

}  // namespace

#if LNCH_STAMP
extern "C" int dh_debug_lnch_stamps(unsigned long long* out, int n) {
  n = n < LNCH_STAMP_WG * LNCH_NSTAMP ? n : LNCH_STAMP_WG * LNCH_NSTAMP;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lnch_stamp), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif

// 1 = gemm_lnch_kernel (16-electron tiles, one per CU), 0 = the GEMM + layernorm_ch pair
// (dh_debug_set_lnch_form: tests and tools only)
static int g_lnch_form = 1;

int set_lnch_form(int f) {
  const int old = g_lnch_form;
  if (f >= 0 && f <= 1) g_lnch_form = f;
  return old;
}

bool gemm_lnch_supported(int N, int D) {
  if (D != LN_D || N < 1) return false;
  return g_lnch_form == 1 && N <= 6;
}

void launch_gemm_lnch(int N, const float* X, const uint16_t* Wp, int ldp, const float* bias, const float* ln,
                      const float* geo, float* h, int ne, int mode, hipStream_t s, const float* W0f, int n_up, int K,
                      const uint16_t* Wv, const uint16_t* Wb) {
  if (mode == 1) {
    W0f = nullptr;
    K = LN_D;
  }
  switch (N) {
    case 1: launch_lnch_n<1>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K, Wv, Wb); return;
    case 2: launch_lnch_n<2>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K, Wv, Wb); return;
    case 3: launch_lnch_n<3>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K, Wv, Wb); return;
    case 4: launch_lnch_n<4>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K, Wv, Wb); return;
    case 5: launch_lnch_n<5>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K, Wv, Wb); return;
    default: launch_lnch_n<6>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K, Wv, Wb); return;
  }
}

}  // namespace dh
