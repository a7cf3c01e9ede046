// Channel-row linear map + channel LayerNorm in ONE launch (local energy, D = K = 256):
//
//   MODE 0:  h = LN_ch(h + X W + b)            psiformer.py:44-46  (X = o, W = Wo Wl folded)
//   MODE 1:  h = LN_ch(h + tanh_ch(h W + b))   psiformer.py:47-48  (X = h)
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
// Traffic per launch: X once (the k loop), h once (the epilogue; in MODE 1 the same rows
// as X, from MALL), h written once: 12 * rows * 256 B, against 20 (MODE 0) / 24 (MODE 1)
// for the two-kernel form.
//
// Build knobs (tools/lnch_one.py A/B builds; defaults are the production kernel):
// LNCH_COUTER channel-outer k loop; LNCH_SB per-channel sched barrier; LNCH_PF residual
// loads in flight; LNCH_OPQ opaque residual offsets (register pressure); LNCH_ABL ablations
// (bit 0: no LayerNorm epilogue, bit 1: no MFMAs — wrong results, timing only); LNCH_RPF MODE 0
// residual-line touch during the k loop.
#include <cstdlib>

#include "dh_internal.h"
#include "device_common.h"

#ifndef LNCH_COUTER
#define LNCH_COUTER 0
#endif
#ifndef LNCH_SB
#define LNCH_SB 1
#endif
#ifndef LNCH_PF
#define LNCH_PF 8
#endif
#ifndef LNCH_ABL
#define LNCH_ABL 0
#endif
#ifndef LNCH_OPQ
#define LNCH_OPQ 1
#endif
#ifndef LNCH_LBAR  // A/B knob: barriers that wait for LDS only (lgkmcnt(0) + s_barrier), round 5: __syncthreads'
#define LNCH_LBAR 1  // vmcnt(0) drained the next k-step's activation loads every step and the next residual chunk
#endif
#ifndef LNCH_RPF
#define LNCH_RPF 0
#endif
#ifndef LNCH_RDMA
#define LNCH_RDMA 1
#endif
#ifndef LNCH_RDMA_LATE
#define LNCH_RDMA_LATE 1
#endif
#ifndef LNCH_PERMLANE  // round-3 variant kept for the electron-slot study: the
#define LNCH_PERMLANE 0  // four lane rows' partials summed by permlane32/16 swaps, not in LDS
#endif
#ifndef LNCH_LNP  // A/B knob: the LayerNorm scale / shift loaded before the output stores (1) or between them (0)
#define LNCH_LNP 1
#endif
#ifndef LNCH_STAMP
#define LNCH_STAMP 0
#endif

namespace dh {

#if LNCH_STAMP
// diagnostic builds only (tools/lnch_one.py): per-workgroup phase timestamps (s_memtime) of
// the first LNCH_STAMP_WG tiles, written by thread 0 into a buffer nothing else reads
constexpr int LNCH_STAMP_WG = 4096, LNCH_NSTAMP = 10;
__device__ unsigned long long g_lnch_stamp[LNCH_STAMP_WG * LNCH_NSTAMP];
#define LNCH_T(i)                                                                    \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < LNCH_STAMP_WG)                              \
      g_lnch_stamp[blockIdx.x * LNCH_NSTAMP + (i)] = __builtin_amdgcn_s_memtime();   \
  } while (0)
#define LNCH_RT(i)                                                                   \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < LNCH_STAMP_WG)                              \
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
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

constexpr int LN_EPT = 16;  // electrons per tile (the MFMA column dimension)
constexpr int LN_D = 256;   // features (= K)
constexpr int LN_BK = 32;   // k per step
// epilogue residual through LDS (LNCH_RDMA): chunks of LN_RCH channel rows of all 16
// electrons (LN_RCH * 16 rows of 1 KB).  LNCH_R3 (round 5): 3-row chunks in three buffers —
// two over the stage area, the third past the geometry, free during the k loop, so chunk 0 is
// requested at kernel start (its latency hides behind the first k-step's own loads) and two
// chunks are in flight behind the one being added; else 4-row chunks in two buffers
#ifndef LNCH_R3
#define LNCH_R3 0  // measured neutral (profiles/r05_v13_ab.txt): kept off
#endif
constexpr int LN_RCH = LNCH_R3 ? 3 : 4;
constexpr int LN_NBUF = LNCH_R3 ? 3 : 2;
constexpr int LN_RBUF = LN_RCH * LN_EPT * LN_D * 4;  // bytes of one chunk buffer

// LDS bytes of the kernel: the two k-step plane stages (reused by the epilogue's residual
// chunks and statistics), then the walkers' geometry, then (LNCH_R3) the third chunk buffer
__host__ __device__ constexpr int lnch_geo_off(int N) {
  return (6 * (2 * N + 5) * LN_EPT * 64 > (LNCH_RDMA ? 2 * LN_RBUF : 0)) ? 6 * (2 * N + 5) * LN_EPT * 64
                                                                       : 2 * LN_RBUF;
}
__host__ __device__ constexpr int lnch_bx_off(int N) {
  return (lnch_geo_off(N) + ((LN_EPT + N - 1) / N + 1) * N * 16 + 1023) & ~1023;
}
__host__ __device__ constexpr int lnch_smem(int N) {
  return (LNCH_RDMA && LN_NBUF == 3) ? lnch_bx_off(N) + LN_RBUF
                                     : lnch_geo_off(N) + ((LN_EPT + N - 1) / N + 1) * N * 16;
}
// byte offset of chunk k's buffer
__host__ __device__ constexpr int lnch_cbuf(int N, int k) {
  return LN_NBUF == 3 ? (k % 3 == 0 ? lnch_bx_off(N) : (k % 3 - 1) * LN_RBUF) : (k & 1) * LN_RBUF;
}

__device__ __forceinline__ uint32_t pkbf(float x, float y) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){x, y}, bf16x2));
}
__device__ __forceinline__ float lo_of(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_of(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ int lnch_sw(int e) { return (0x78 >> (2 * ((e >> 2) & 3))) & 3; }
#if LNCH_PERMLANE
// sum over the four lanes e, e + 16, e + 32, e + 48 (the round-3 permlane form)
__device__ __forceinline__ float lnch_sum4g(float v) {
  const int x = __float_as_int(v);
  const auto a = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  v = __int_as_float(a[0]) + __int_as_float(a[1]);
  const int y = __float_as_int(v);
  const auto b = __builtin_amdgcn_permlane16_swap(y, y, false, false);
  return __int_as_float(b[0]) + __int_as_float(b[1]);
}
#endif

template <int N, int MODE, int NWV, bool FRES = false>
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(NWV >= 8 ? 2 : 1, NWV >= 8 ? 2 : 1))) void gemm_lnch_kernel(const float* X, const uint16_t* __restrict__ Wp, int ldp,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ ln,
                                                         const float* __restrict__ geo, float* h, int ne,
                                                         const float* __restrict__ W0f, int n_up, int kx) {
  // K: the contraction length = X's row length, a multiple of BK (256; MODE 0 of layer 1 from
  // the o~ rows: ofeat_k, dh_internal.h); a compile-time 256 in MODE 1
  constexpr int C = 2 * N + 5, T = 2 * N, EPT = LN_EPT, D = LN_D, BK = LN_BK;
  const int K = MODE == 1 ? LN_D : kx, NK = K / BK;
  constexpr int ROWS = EPT * C;                    // activation rows per tile
  constexpr int NT = NWV * 64, CB = D / (16 * NWV);  // threads; 16-column blocks per wave
  constexpr int PLANE = C * EPT * 64;              // bytes of one bf16 plane per step
  constexpr int STAGE = 3 * PLANE;
  constexpr int NQ = (ROWS * 8 + NT - 1) / NT;     // 16-B activation pieces per thread per step
  constexpr int NR = C + T + 3;                    // second-moment statistics per electron
  constexpr int TS = NR | 1;                       // odd row stride of the totals
  static_assert(2 * STAGE <= lnch_geo_off(N) && lnch_smem(N) <= 163840, "LDS");
  static_assert(NWV * NR * 64 * 4 + EPT * TS * 4 <= 2 * STAGE, "reduction scratch");
  extern __shared__ float4 smem4[];
  char* smem = reinterpret_cast<char*>(smem4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kg = lane >> 4;
  const int tile = blockIdx.x;
  // every barrier here orders LDS only (planes, residual chunks after their counted DMA waits,
  // statistics): global loads in flight may cross it
  auto lbar = []() __attribute__((always_inline)) {
#if LNCH_LBAR
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#else
    __syncthreads();
#endif
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
  const uint32_t tbytes = (uint32_t)rows_valid * D * 4, xbytes = (uint32_t)rows_valid * K * 4;
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
      const uint32_t h0 = pkbf(u.x, u.y), h1 = pkbf(u.z, u.w);
      const float rx = u.x - lo_of(h0), ry = u.y - hi_of(h0), rz = u.z - lo_of(h1), rw = u.w - hi_of(h1);
      const uint32_t m0 = pkbf(rx, ry), m1 = pkbf(rz, rw);
      const uint32_t s0 = pkbf(rx - lo_of(m0), ry - hi_of(m0)), s1 = pkbf(rz - lo_of(m1), rw - hi_of(m1));
      *reinterpret_cast<uint2*>(P + loff[j]) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(P + PLANE + loff[j]) = make_uint2(m0, m1);
      *reinterpret_cast<uint2*>(P + 2 * PLANE + loff[j]) = make_uint2(s0, s1);
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

#if LNCH_RDMA
  // ---- the residual rows h through LDS by DMA (global_load_lds_dwordx4, no VGPRs): chunk k =
  // channel rows LN_RCH k .. + LN_RCH - 1 of the tile's 16 electrons, one 1-KB row per wave
  // instruction, into chunk buffer lnch_cbuf(k) at row q = (c - LN_RCH k) * 16 + e.  16-B slot s of
  // a row holds the row's quad s ^ e (the swizzle is on the SOURCE address: the DMA writes
  // lane-linearly), so the epilogue's ds_read_b128 of quad Q = 8 w + 4 cb + g by lane (e, g)
  // hits slot Q ^ e: 16 distinct slots in every lane group.  Rows of electrons past the end
  // re-read the tile's first row into their (never read) slot, so every wave issues the same
  // compile-time number of DMAs per chunk and "chunk k landed" is vmcnt(DMAs of the younger
  // chunks k + 1 .. k + LN_NBUF - 1).
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
        const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(lnch_cbuf(N, k) + q * D * 4));
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(rowp), "s"(dst)
                     : "memory");
      }
    }
  };
  // MODE 0 of layer 1 (W0f): the residual h0 = f W0 is formed from the walkers' geometry in the
  // epilogue (round 5), so h0 is never written by the input kernel nor read back here
  constexpr bool fres = MODE == 0 && FRES;
  if (LN_NBUF == 3 && !fres) rdma(0);  // LNCH_R3: chunk 0 into the buffer past the stages, now
#endif
  // the accumulators start from zero (the residual is added in the epilogue: starting them
  // from h rounds every k-step's partial sum at |h| and measurably loosened the tangent
  // channels against float64 on ill-conditioned walkers)
  f32x4 acc[C][CB];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc[c][cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  {
#if LNCH_COUTER
    // channel outermost: each activation fragment read from LDS once per step and used by
    // all CB column blocks (half the LDS reads of the block-outer order); all CB blocks'
    // weight fragments live, the next step's streaming in behind them
    float4 ra[NQ];
    bf16x8 wf[CB][3], wn[CB][3];
    load_a(0, ra);
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) load_w(0, cb, wf[cb]);
    split_store(ra, 0);
    if (NK > 1) load_a(1, ra);
#pragma unroll 1
    for (int kt = 0; kt < NK; ++kt) {
      lbar();  // planes of step kt complete; step kt - 1's buffer is free
      const char* P = smem + (kt & 1) * STAGE + xoff;
      if (kt + 1 < NK) {
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) load_w(kt + 1, cb, wn[cb]);
      }
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
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) {
          f32x4 a = acc[c][cb];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][0], x2, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][2], x0, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][1], x1, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][0], x1, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][1], x0, a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cb][0], x0, a, 0, 0, 0);
          acc[c][cb] = a;
        }
        if (c == C / 2 && kt + 1 < NK) {
          split_store(ra, (kt + 1) & 1);
          if (kt + 2 < NK) load_a(kt + 2, ra);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (kt + 1 < NK) {
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
#pragma unroll
          for (int p = 0; p < 3; ++p) wf[cb][p] = wn[cb][p];
      }
    }
  }
#else
    // column block outermost: one block's weight fragments (12 VGPRs) live at a time, the next
    // block's streaming in behind them; the activation fragments are re-read from LDS per block
    float4 ra[NQ];
    bf16x8 wf[3], wn[3];
    // MODE 0 (X = o, not h): one dword of every 128-B line of the tile's residual rows is
    // touched during the k loop (one line per thread per step), so the epilogue's residual
    // loads find the lines in the MALL / L2 instead of HBM; the touched values are folded
    // into an opaque word, consumed a step later (the load never stalls the loop)
    constexpr int RLINES = ROWS * D * 4 / 128;
    const auto rsH = __builtin_amdgcn_make_buffer_rsrc(h + row0 * D, (short)0, tbytes, 0x00020000);
    uint32_t rpf = 0, rpv = 0;
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
#if LNCH_ABL & 2
          if (a[0] == 1.2345e-33f)  // ablation (tools only): MFMAs skipped
#endif
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
            if (MODE == 0 && LNCH_RPF) {
              rpf ^= rpv;
              const int li = kt * NT + tid;
              rpv = li < RLINES ? __builtin_amdgcn_raw_buffer_load_b32(rsH, li * 128, 0, 0) : 0u;
            }
          }
#if LNCH_SB
          __builtin_amdgcn_sched_barrier(0);
#endif
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) wf[p] = wn[p];
      }
    }
    if (MODE == 0 && LNCH_RPF && (rpf ^ rpv) == 0x7fc00001u && ne < 0) h[0] = 0.f;  // never taken
  }
#endif
  lbar();  // every wave is past its last plane read: the stage buffers become scratch
  LNCH_T(2);
  // the epilogue's lane indices, re-derived from the lane id (mbcnt) rather than kept live
  // across the k loop from threadIdx (holding them there made MODE 1 spill)
  const int lane_e = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
#if LNCH_RDMA
  if ((MODE == 0 || !LNCH_RDMA_LATE) && !fres) {
    if (LN_NBUF == 2) rdma(0);
#pragma unroll
    for (int x = 1; x < LN_NBUF; ++x)
      if (x < NCHK) rdma(x);
  }
#endif
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
#if !LNCH_RDMA
  auto ldh = [&](int c, int cb) { return *reinterpret_cast<const float4*>(htile + roff(c, cb)); };
#endif
  auto sth = [&](int c, int cb, float4 v) {
    if (valid) *reinterpret_cast<float4*>(htile + roff(c, cb)) = v;
  };
#if LNCH_ABL & 1
  {  // ablation (tools only): no LayerNorm epilogue, the raw accumulators stored
    const int E = e0 + l16;
    if (E < ne) {
      float* hr = h + (row0 + (size_t)l16 * C) * D + 16 * CB * wid + 4 * kg;
      for (int c = 0; c < C; ++c)
        for (int cb = 0; cb < CB; ++cb) *reinterpret_cast<f32x4*>(hr + c * D + 16 * cb) = acc[c][cb];
    }
    return;
  }
#endif

  // ---- epilogue: lane = electron l16, features nf + 16 cb + 0..3 of every channel row
  // geometry of the walker's electrons (st, ct, sp, cp) from the tile's LDS copy (read where
  // used: holding N float4 per lane would spill the accumulators)
  const float4* gw = gl + (b - e0 / N) * N;
  auto al = [&](int k, int t) -> float {  // flow coefficient alpha_kt (layernorm.hip)
    const float4 q = gw[t >> 1];
    if ((t & 1) == 0) return k == 0 ? -q.z : (k == 1 ? q.w : 0.f);
    return k == 0 ? -(q.y * q.w) : (k == 1 ? -(q.y * q.z) : q.x);
  };
  // pre-LN rows x_c (in acc): bias (value rows), MODE 1's tanh_ch, then + h
  float chain = 0.f;
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + nf + 16 * cb) : make_float4(0.f, 0.f, 0.f, 0.f);
    acc[0][cb][0] += bv.x;
    acc[0][cb][1] += bv.y;
    acc[0][cb][2] += bv.z;
    acc[0][cb][3] += bv.w;
    if (MODE == 1) {
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
  }
#if LNCH_RDMA
  if (MODE == 1) {
    // the tanh_ch results are materialised here, before the DMA blocks (otherwise the
    // compiler sinks the channel algebra past them and its live ranges spill)
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) asm volatile("" : "+v"(acc[c][cb]));
  }
  if (MODE == 1 && LNCH_RDMA_LATE) {
    if (LN_NBUF == 2) rdma(0);
#pragma unroll
    for (int x = 1; x < LN_NBUF; ++x)
      if (x < NCHK) rdma(x);
  }
  if constexpr (fres) {
    // input.hip's channel features of this lane's electron (the geometry staged in gl) times
    // W0's columns nf + 16 cb .. + 3, the input kernel's expression, then added as the
    // residual rows are (r + acc)
    const float4 g4 = gl[valid ? E - (e0 / N) * N : 0];  // st ct sp cp
    const float st = g4.x, ct = g4.y, sp = g4.z, cp = g4.w;
    const int ie = (valid ? E : e0) % N;
    const float rx = st * cp, ry = st * sp, rz = ct;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const float4 w0 = *reinterpret_cast<const float4*>(W0f + nf + 16 * cb);
      const float4 w1 = *reinterpret_cast<const float4*>(W0f + D + nf + 16 * cb);
      const float4 w2 = *reinterpret_cast<const float4*>(W0f + 2 * D + nf + 16 * cb);
      const float4 w3 = *reinterpret_cast<const float4*>(W0f + 3 * D + nf + 16 * cb);
#pragma unroll
      for (int c = 0; c < C; ++c) {
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
      // this wave's chunk-k DMAs landed (the younger ones are chunks k + 1 .. k + LN_NBUF - 1,
      // issued before this wait), then every wave's
      const int YNG = (k + 1 < NCHK ? rows_of(k + 1) : 0) / NWV + (LN_NBUF == 3 && k + 2 < NCHK ? rows_of(k + 2) : 0) / NWV;
      if (YNG > 0)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"((k + 1 < NCHK ? rows_of(k + 1) : 0) / NWV +
                                                (LN_NBUF == 3 && k + 2 < NCHK ? rows_of(k + 2) : 0) / NWV)
                     : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lbar();
#pragma unroll
      for (int cc = 0; cc < LN_RCH; ++cc) {
        const int c = LN_RCH * k + cc;
        if (c < C) {
#pragma unroll
          for (int cb = 0; cb < CB; ++cb) {
            const float4 r = *reinterpret_cast<const float4*>(rb0 + lnch_cbuf(N, k) + cc * EPT * D * 4 + rsl[cb]);
            f32x4& a = acc[c][cb];
            a[0] = r.x + a[0];
            a[1] = r.y + a[1];
            a[2] = r.z + a[2];
            a[3] = r.w + a[3];
#if LNCH_OPQ
            asm volatile("" : "+v"(a));  // consumed here (keeps the reads from being batched)
#endif
          }
        }
      }
      if (k + LN_NBUF < NCHK) {
        lbar();  // every wave is done with chunk k's buffer
        rdma(k + LN_NBUF);
      }
    }
    lbar();  // the chunk buffers become the statistics scratch
    LNCH_T(3);
  }
#else
  static_assert(!fres, "the feature residual needs the LNCH_RDMA build (the default)");
  {
    // residual rows, PF float4 loads in flight (ldh's opaque offsets keep the compiler from
    // hoisting all C * CB of them, which would spill the accumulators)
    constexpr int NRES = C * CB, PF = LNCH_PF;
    float4 rb[PF];
#pragma unroll
    for (int i = 0; i < PF && i < NRES; ++i) rb[i] = ldh(i / CB, i % CB);
#pragma unroll
    for (int i = 0; i < NRES; ++i) {
      const float4 r = rb[i % PF];
      if (i + PF < NRES) rb[i % PF] = ldh((i + PF) / CB, (i + PF) % CB);
      f32x4& a = acc[i / CB][i % CB];
      a[0] = r.x + a[0];
      a[1] = r.y + a[1];
      a[2] = r.z + a[2];
      a[3] = r.w + a[3];
#if LNCH_OPQ
      asm volatile("" : "+v"(a));  // consumed here, before the next load is issued
#endif
    }
  }
#endif
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
#if LNCH_PERMLANE
      const float v = lnch_sum4g(part(j));
      if (kge == 0) red[(wid * NS + j) * 64 + l16e] = v;
#else
      red[(wid * NS + j) * 64 + lane_e] = part(j);  // every lane's 8-feature partial (no cross-lane ops)
#endif
      __builtin_amdgcn_sched_barrier(0);          // one statistic at a time (register pressure)
    }
    lbar();
    for (int i = tide; i < NS * EPT; i += NT) {
      const int j = i / EPT, e = i - j * EPT;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w)
#pragma unroll
        for (int g = 0; g < (LNCH_PERMLANE ? 1 : 4); ++g) s += red[(w * NS + j) * 64 + 16 * g + e];
      tot[e * TS + j] = s * (1.f / D);
    }
    lbar();
  };
  const float* mt = tot + l16e * TS;  // this lane's electron
  // channel means, centre
  reduce([&](int c) { return lane_sum(c); }, std::integral_constant<int, C>{});
  LNCH_T(4);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float mu = mt[c];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[c][cb][v] -= mu;
    __builtin_amdgcn_sched_barrier(0);
  }
  // flow vector u_k = sum_t alpha_kt z_t of columns block cb (recomputed where needed)
  auto flow = [&](int k, int cb) {
    f32x4 r = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (k == 2 && (t & 1) == 0) continue;  // alpha_2,2i = 0
      const float a = al(k, t);
      r[0] = fmaf(a, acc[1 + t][cb][0], r[0]);
      r[1] = fmaf(a, acc[1 + t][cb][1], r[1]);
      r[2] = fmaf(a, acc[1 + t][cb][2], r[2]);
      r[3] = fmaf(a, acc[1 + t][cb][3], r[3]);
    }
    return r;
  };
  auto dot4 = [](const f32x4& x, const f32x4& y) { return (x[0] * y[0] + x[1] * y[1]) + (x[2] * y[2] + x[3] * y[3]); };
  // p_c = <z0 z_c>, q_t = <z_t^2>, uu_k = <u_k^2>
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
  LNCH_T(5);
  const float s = 1.f / sqrtf(mt[0] + 1e-5f), s2 = s * s;
  float cl = 0.f, au[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const float a = s2 * mt[1 + t];
    cl += 3.f * a * a - s2 * mt[C + t];
#pragma unroll
    for (int k = 0; k < 3; ++k) au[k] = fmaf(al(k, t), a, au[k]);
  }
  float cs[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) cs[k] = 3.f * au[k] * au[k] - s2 * mt[C + T + k];
  const float aL = s2 * mt[1 + T];
  // the LayerNorm scale / shift of both column blocks before the first store: a load between
  // two stores waits for every earlier store (vmcnt counts in order)
  float4 lng[CB], lnb[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    lng[cb] = LNCH_LNP ? *reinterpret_cast<const float4*>(ln + nf + 16 * cb) : make_float4(0.f, 0.f, 0.f, 0.f);
    lnb[cb] = LNCH_LNP ? *reinterpret_cast<const float4*>(ln + D + nf + 16 * cb) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const float4 gv = LNCH_LNP ? lng[cb] : *reinterpret_cast<const float4*>(ln + nf + 16 * cb);
    const float4 bb = LNCH_LNP ? lnb[cb] : *reinterpret_cast<const float4*>(ln + D + nf + 16 * cb);
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
      const float at = s2 * mt[1 + t];
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
      for (int v = 0; v < 4; ++v) y[v] = gs[v] * (acc[1 + T][cb][v] - aL * z0[v] - 2.f * sat[v] + cl * z0[v]);
      sth(1 + T, cb, make_float4(y[0], y[1], y[2], y[3]));
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const f32x4 uk = flow(k, cb);
      const float ak = s2 * mt[2 + T + k];
      float y[4];
#pragma unroll
      for (int v = 0; v < 4; ++v)
        y[v] = gs[v] * (acc[2 + T + k][cb][v] - ak * z0[v] - 2.f * au[k] * uk[v] + cs[k] * z0[v]);
      sth(2 + T + k, cb, make_float4(y[0], y[1], y[2], y[3]));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  LNCH_T(6);
  LNCH_RT(9);
}

template <int N, int NWV>
void launch_lnch_t(const float* X, const uint16_t* Wp, int ldp, const float* bias, const float* ln, const float* geo,
                   float* h, int ne, int mode, hipStream_t s, const float* W0f, int n_up, int K) {
  const size_t smem = lnch_smem(N);
  const int grid = (ne + LN_EPT - 1) / LN_EPT;
  if (mode == 0 && W0f) {
    ensure_smem(gemm_lnch_kernel<N, 0, NWV, true>, smem);
    hipLaunchKernelGGL((gemm_lnch_kernel<N, 0, NWV, true>), dim3(grid), dim3(NWV * 64), smem, s, X, Wp, ldp, bias, ln, geo,
                       h, ne, W0f, n_up, K);
  } else if (mode == 0) {
    ensure_smem(gemm_lnch_kernel<N, 0, NWV>, smem);
    hipLaunchKernelGGL((gemm_lnch_kernel<N, 0, NWV>), dim3(grid), dim3(NWV * 64), smem, s, X, Wp, ldp, bias, ln, geo, h,
                       ne, W0f, n_up, K);
  } else {
    ensure_smem(gemm_lnch_kernel<N, 1, NWV>, smem);
    hipLaunchKernelGGL((gemm_lnch_kernel<N, 1, NWV>), dim3(grid), dim3(NWV * 64), smem, s, X, Wp, ldp, bias, ln, geo, h,
                       ne, nullptr, 0, LN_D);
  }
}

template <int N>
void launch_lnch_n(const float* X, const uint16_t* Wp, int ldp, const float* bias, const float* ln, const float* geo,
                   float* h, int ne, int mode, hipStream_t s, const float* W0f, int n_up, int K) {
  launch_lnch_t<N, 8>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K);
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
                      const float* geo, float* h, int ne, int mode, hipStream_t s, const float* W0f, int n_up, int K) {
  if (mode != 0) {
    W0f = nullptr;
    K = LN_D;
  }
  switch (N) {
    case 1: launch_lnch_n<1>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K); return;
    case 2: launch_lnch_n<2>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K); return;
    case 3: launch_lnch_n<3>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K); return;
    case 4: launch_lnch_n<4>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K); return;
    case 5: launch_lnch_n<5>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K); return;
    default: launch_lnch_n<6>(X, Wp, ldp, bias, ln, geo, h, ne, mode, s, W0f, n_up, K); return;
  }
}

}  // namespace dh
