// C ABI of the MI355X-native DeepHall VMC inner loop (include/deephall_amd.h).
// Sequences the HIP kernels of one Psiformer pass:
//
//   input (features x W0) -> per layer [ QKV GEMM -> attention -> (O.Wl) GEMM + residual
//   -> LayerNorm -> MLP GEMM -> tanh + residual + LayerNorm ] -> orbital GEMM -> det
//
// with either 1 channel (log psi, MCMC) or 2N+5 channels (local energy).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "dh_internal.h"

using namespace dh;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(DH_EHIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

int check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(DH_EHIP, std::string("kernel launch: ") + hipGetErrorString(e));
  return DH_OK;
}

size_t align64(size_t n) { return (n + 63) / 64 * 64; }

// Workspace of one pass (floats), carved from the caller's buffer.
struct Work {
  float *h, *qkv, *o, *t, *F, *geo, *x2, *logpsi, *lp;
  int32_t* nacc;
  size_t total_bytes;
};

Work carve(const Dims& d, int nw, int C, void* base) {
  const int rows = nw * d.N * C;
  const size_t rp = (size_t)round_up(std::max(rows, 1), kRowPad);
  const size_t nh = align64(rp * d.D);
  const size_t nqkv = align64(rp * (size_t)std::max(3 * d.D, d.ld_orb));
  Work w{};
  size_t off = 0;
  auto take = [&](size_t n) {
    float* p = base ? reinterpret_cast<float*>(base) + off : nullptr;
    off += align64(n);
    return p;
  };
  w.h = take(nh);
  w.qkv = take(nqkv);
  w.o = take(nh);
  w.t = take(nh);
  w.F = w.qkv;  // orbital features reuse the QKV buffer (free after the last attention)
  w.geo = take((size_t)nw * d.N * 4);
  w.x2 = take((size_t)nw * d.N * 2);
  w.logpsi = take((size_t)nw * 2);
  w.lp = take((size_t)nw);
  w.nacc = reinterpret_cast<int32_t*>(take((size_t)nw));
  w.total_bytes = off * sizeof(float);
  return w;
}

}  // namespace

// Optional per-kernel HIP-event timing (bench.py reads it to compute the live roofline).
enum ProfKind { PK_GEMM = 0, PK_ATTN, PK_LN, PK_INPUT, PK_DET_VALUE, PK_DET_ENERGY, PK_MCMC, PK_COUNT };
// channel-mode (C > 1) launches of GEMM/attention/LayerNorm/input are recorded as kind + PK_CH
constexpr int PK_CH = PK_COUNT, PK_TOTAL = PK_COUNT + 4;
struct ProfRec {
  hipEvent_t a, b;
  int kind;
  double flops, bytes;
};
struct Profiler {
  bool on = false;
  std::vector<ProfRec> recs;
  size_t used = 0;
};

struct dh_handle {
  dh_config cfg;
  Dims d;
  Params p{};
  std::vector<size_t> offsets;  // nseg + 1
  float* params = nullptr;
  float* norm = nullptr;  // sqrt(binom(2Q, Q-m)), M floats (device)
  float* wt = nullptr;    // transposed GEMM weights for the NT kernels (device)
  uint16_t* wp = nullptr;  // split-bf16 weight planes for the x6 kernels (device)
  int gemm_mode = DH_GEMM_X6_ALL;
  std::vector<float> norm_host;
  bool params_set = false;
  Profiler prof;
};

namespace {
struct ProfScope {
  dh_handle* h;
  hipStream_t s;
  ProfRec* r = nullptr;
  ProfScope(dh_handle* h_, int kind, double flops, double bytes, hipStream_t s_) : h(h_), s(s_) {
    if (!h->prof.on) return;
    Profiler& P = h->prof;
    if (P.used == P.recs.size()) {
      ProfRec nr{};
      (void)hipEventCreate(&nr.a);
      (void)hipEventCreate(&nr.b);
      P.recs.push_back(nr);
    }
    r = &P.recs[P.used++];
    r->kind = kind;
    r->flops = flops;
    r->bytes = bytes;
    (void)hipEventRecord(r->a, s);
  }
  ~ProfScope() {
    if (r) (void)hipEventRecord(r->b, s);
  }
};
}  // namespace
#define PROF(kind, flops, bytes) ProfScope prof_scope_##__LINE__(h, kind, (double)(flops), (double)(bytes), s)

extern "C" {

const char* dh_last_error(void) { return g_err.c_str(); }
const char* dh_version(void) { return "deephall_amd 0.1 (gfx950)"; }

int dh_create(const dh_config* cfg, dh_handle** out) {
  if (!cfg || !out) return fail(DH_EINVAL, "null argument");
  const int N = cfg->n_up + cfg->n_dn;
  if (cfg->n_up < 0 || cfg->n_dn < 0 || N < 1 || N > 32) return fail(DH_EINVAL, "need 1 <= N <= 32 electrons");
  if (cfg->flux < 0 || cfg->flux > 126) return fail(DH_EINVAL, "need 0 <= flux <= 126");
  if (cfg->num_layers < 0 || cfg->num_layers > 16) return fail(DH_EINVAL, "need num_layers <= 16");
  if (cfg->ndets < 1 || cfg->ndets > 16) return fail(DH_EINVAL, "need 1 <= determinants <= 16");
  if (cfg->num_heads < 1 || cfg->heads_dim < 1) return fail(DH_EINVAL, "bad attention shape");
  if (cfg->orbital_type != DH_ORBITAL_FULL) return fail(DH_EINVAL, "only orbital type 'full' is supported");
  if (cfg->interaction_type != DH_INTERACTION_COULOMB && cfg->interaction_type != DH_INTERACTION_HARMONIC)
    return fail(DH_EINVAL, "bad interaction type");
  const int D = cfg->num_heads * cfg->heads_dim;
  if (D % 4 != 0) return fail(DH_EINVAL, "num_heads * heads_dim must be a multiple of 4");
  if (cfg->flux == 0 && cfg->interaction_type == DH_INTERACTION_HARMONIC)
    return fail(DH_EINVAL, "harmonic potential needs flux > 0");
  auto* h = new dh_handle();
  h->cfg = *cfg;
  Dims& d = h->d;
  d.N = N;
  d.n_up = cfg->n_up;
  d.n_dn = cfg->n_dn;
  d.T = 2 * N;
  d.C = 2 * N + 5;
  d.M = cfg->flux + 1;
  d.Q = 0.5f * cfg->flux;
  d.r = cfg->radius > 0.f ? cfg->radius : std::sqrt(d.Q);
  d.H = cfg->num_heads;
  d.dh = cfg->heads_dim;
  d.D = D;
  d.L = cfg->num_layers;
  d.K = cfg->ndets;
  d.NB = (cfg->n_dn > 0 && cfg->n_up > 0) ? 2 : 1;
  d.orb_cols = d.NB * 2 * d.M * N * d.K;
  d.ld_orb = round_up(d.orb_cols, 128);
  d.interaction = cfg->interaction_type;
  d.lambda = cfg->interaction_strength;
  // packed layout
  std::vector<size_t> sizes;
  sizes.push_back((size_t)4 * D);
  for (int l = 0; l < d.L; ++l) {
    sizes.push_back((size_t)D * 3 * D);
    sizes.push_back((size_t)3 * D);
    sizes.push_back((size_t)D * D);
    sizes.push_back((size_t)D);
    sizes.push_back((size_t)2 * D);
    sizes.push_back((size_t)D * D);
    sizes.push_back((size_t)D);
    sizes.push_back((size_t)2 * D);
  }
  sizes.push_back((size_t)D * d.ld_orb);
  sizes.push_back((size_t)d.ld_orb);
  sizes.push_back(2);
  sizes.push_back((size_t)4 * 3 * D);  // W0 @ Wqkv of layer 0 (folded input projection)
  size_t off = 0;
  for (size_t s : sizes) {
    h->offsets.push_back(off);
    off += align64(s);
  }
  h->offsets.push_back(off);
  // monopole-harmonic normalisation sqrt(C(2Q, Q-m)) (blocks.py:45-46), index p = Q+m
  std::vector<float> norm(d.M);
  for (int p = 0; p < d.M; ++p) {
    const int n = d.M - 1, k = d.M - 1 - p;
    const double lc = std::lgamma(n + 1.0) - std::lgamma(k + 1.0) - std::lgamma(n - k + 1.0);
    norm[p] = (float)std::sqrt(std::exp(lc));
  }
  h->norm_host = norm;  // uploaded by dh_set_params (dh_create makes no HIP calls)
  *out = h;
  return DH_OK;
}

void dh_destroy(dh_handle* h) {
  if (!h) return;
  for (auto& r : h->prof.recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  if (h->params) (void)hipFree(h->params);
  if (h->norm) (void)hipFree(h->norm);
  if (h->wt) (void)hipFree(h->wt);
  if (h->wp) (void)hipFree(h->wp);
  delete h;
}

int dh_param_layout(const dh_handle* h, size_t* offsets, int n) {
  if (!h) return fail(DH_EINVAL, "null handle");
  const int nseg = (int)h->offsets.size() - 1;
  for (int i = 0; i < n && i <= nseg; ++i) offsets[i] = h->offsets[i];
  return nseg;
}

int dh_set_params(dh_handle* h, const float* params, size_t count, void* stream) {
  if (!h || !params) return fail(DH_EINVAL, "null argument");
  if (count != h->offsets.back()) return fail(DH_EINVAL, "parameter count mismatch");
  if (!h->params) HIP_TRY(hipMalloc(&h->params, count * sizeof(float)));
  if (!h->norm) {
    HIP_TRY(hipMalloc(&h->norm, h->norm_host.size() * sizeof(float)));
    HIP_TRY(hipMemcpy(h->norm, h->norm_host.data(), h->norm_host.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMemcpyAsync(h->params, params, count * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  const Dims& d = h->d;
  const float* P = h->params;
  int s = 0;
  h->p.W0 = P + h->offsets[s++];
  for (int l = 0; l < d.L; ++l) {
    LayerParams& lp = h->p.layer[l];
    lp.Wqkv = P + h->offsets[s++];
    lp.bqkv = P + h->offsets[s++];
    lp.Wol = P + h->offsets[s++];
    lp.bol = P + h->offsets[s++];
    lp.ln1 = P + h->offsets[s++];
    lp.Wm = P + h->offsets[s++];
    lp.bm = P + h->offsets[s++];
    lp.ln2 = P + h->offsets[s++];
  }
  h->p.Worb = P + h->offsets[s++];
  h->p.borb = P + h->offsets[s++];
  h->p.jastrow = P + h->offsets[s++];
  h->p.W0qkv = P + h->offsets[s++];
  // Transposed copies Wt[n][k] (rows zero-padded to 256) of every GEMM weight, for the
  // NT GEMM kernels whose LDS-DMA staging wants k contiguous in both operands.
  if (d.D % 32 == 0) {
    const int D = d.D;
    const size_t sq = (size_t)round_up(D, kRowPad) * D, sqkv = (size_t)round_up(3 * D, kRowPad) * D;
    const size_t sorb = (size_t)round_up(d.orb_cols, kRowPad) * D;
    const size_t total = (size_t)d.L * (sqkv + 2 * sq) + sorb;
    if (!h->wt) HIP_TRY(hipMalloc(&h->wt, total * sizeof(float)));
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(h->wt, 0, total * sizeof(float), st));
    float* q = h->wt;
    for (int l = 0; l < d.L; ++l) {
      LayerParams& lp = h->p.layer[l];
      launch_transpose(lp.Wqkv, 3 * D, D, 3 * D, q, D, st);
      lp.WqkvT = q;
      q += sqkv;
      launch_transpose(lp.Wol, D, D, D, q, D, st);
      lp.WolT = q;
      q += sq;
      launch_transpose(lp.Wm, D, D, D, q, D, st);
      lp.WmT = q;
      q += sq;
    }
    launch_transpose(h->p.Worb, d.ld_orb, D, d.orb_cols, q, D, st);
    h->p.WorbT = q;
    // split-bf16 planes of the same weights (gemm_x6.hip), from the transposed copies
    const size_t pq = (size_t)3 * x6_plane_rows(3 * D) * D, pd = (size_t)3 * x6_plane_rows(D) * D;
    const size_t po = (size_t)3 * x6_plane_rows(d.orb_cols) * D;
    const size_t ptotal = (size_t)d.L * (pq + 2 * pd) + po;
    if (!h->wp) HIP_TRY(hipMalloc(&h->wp, ptotal * sizeof(uint16_t)));
    uint16_t* w = h->wp;
    for (int l = 0; l < d.L; ++l) {
      LayerParams& lp = h->p.layer[l];
      launch_split_planes(lp.WqkvT, D, 3 * D, D, w, st);
      lp.WqkvP = w;
      w += pq;
      launch_split_planes(lp.WolT, D, D, D, w, st);
      lp.WolP = w;
      w += pd;
      launch_split_planes(lp.WmT, D, D, D, w, st);
      lp.WmP = w;
      w += pd;
    }
    launch_split_planes(h->p.WorbT, D, d.orb_cols, D, w, st);
    h->p.WorbP = w;
    HIP_TRY(hipGetLastError());
  }
  h->params_set = true;
  return DH_OK;
}

int dh_set_gemm_mode(dh_handle* h, int mode) {
  if (!h) return fail(DH_EINVAL, "null handle");
  if (mode != DH_GEMM_F32 && mode != DH_GEMM_X6 && mode != DH_GEMM_X6_ALL) return fail(DH_EINVAL, "bad GEMM mode");
  h->gemm_mode = mode;
  return DH_OK;
}

size_t dh_workspace_bytes(const dh_handle* h, int batch, int op) {
  if (!h || batch < 1) return 0;
  return carve(h->d, batch, op == 1 ? h->d.C : 1, nullptr).total_bytes;
}

}  // extern "C"

namespace {

// One Psiformer pass over nw walkers with C channels; leaves orbital features in w.F.
int run_trunk(dh_handle* h, const float* x, int nw, int C, const Work& w, hipStream_t s) {
  const Dims& d = h->d;
  const Params& P = h->p;
  const int rows = nw * d.N * C;
  const int D = d.D;
  const double R = rows, DD = D, f4 = 4.0;
  const bool nt = P.WorbT != nullptr;
  // channel rows (local energy) take the split-bf16 GEMM unless exact-f32 is requested;
  // the log-psi rows only in DH_GEMM_X6_ALL, the LayerNorm-carrying GEMMs with their
  // LayerNorm in the split-bf16 epilogue (96-row tiles of 3 x 4 waves: 34 / 38 us at
  // 24576 x 256 x 256 against 43 / 47 us for the exact-f32 gemm_ln_kernel;
  // tools/ln_gemm_bench.py on MI355X)
  const bool x6 = nt && gemm_x6_supported(D) &&
                  (C > 1 ? h->gemm_mode != DH_GEMM_F32 : h->gemm_mode == DH_GEMM_X6_ALL);
  const bool ln_fused = nt && C == 1 && gemm_ln_supported(D, D);
  auto gemm = [&](const float* X, int ldx, const float* W, const float* Wt, const uint16_t* Wp, int ldw,
                  const float* bias, const float* Res, int ldr, float* Y, int ldy, int ncols, int K) {
    PROF(PK_GEMM + (C > 1 ? PK_CH : 0), 2.0 * R * ncols * K, f4 * (R * K + (double)K * ncols + R * ncols * (Res ? 2 : 1)));
    if (x6)
      launch_gemm_x6(X, ldx, Wp, x6_plane_rows(ncols), bias, Res, ldr, Y, ldy, rows, ncols, K, C, s);
    else if (nt)
      launch_gemm_nt(X, ldx, Wt, K, bias, Res, ldr, Y, ldy, rows, ncols, K, C, s);
    else
      launch_gemm(X, ldx, W, ldw, bias, Res, ldr, Y, ldy, rows, ncols, K, C, s);
  };
  // Layer-1 q|k|v come straight from the K=4 features through the folded W0 Wqkv: inside
  // the attention kernel when it supports that (fused), else written by the input kernel.
  const bool fold = d.L > 0;
  const bool fused = fold && attention_takes_features(d);
  // log psi, split-bf16: layer 1's residual h = features W0 is formed in the epilogue of
  // its LayerNorm GEMM from geo, so the input kernel only writes the geometry
  const bool h_feat = C == 1 && fused && x6 && ln_fused;
  {
    const bool wq = fold && !fused;
    PROF(PK_INPUT + (C > 1 ? PK_CH : 0), 8.0 * R * DD * (wq ? 4 : 1), f4 * R * DD * (wq ? 4 : 1));
    launch_input(d, x, P.W0, wq ? P.W0qkv : nullptr, wq ? P.layer[0].bqkv : nullptr, h_feat ? nullptr : w.h,
                 wq ? w.qkv : nullptr, w.geo, nw, C, s);
  }
  for (int l = 0; l < d.L; ++l) {
    const LayerParams& lp = P.layer[l];
    if (l > 0) gemm(w.h, D, lp.Wqkv, lp.WqkvT, lp.WqkvP, 3 * D, lp.bqkv, nullptr, 0, w.qkv, 3 * D, 3 * D, D);
    {
      const bool f = fused && l == 0;
      PROF(PK_ATTN + (C > 1 ? PK_CH : 0), 0.0, f4 * R * (f ? 1.0 : 4.0) * DD);
      launch_attention(d, w.qkv, w.geo, w.o, nw, C, s, f ? P.W0qkv : nullptr, f ? lp.bqkv : nullptr);
    }
    if (ln_fused) {
      // log psi: each GEMM carries its LayerNorm in the epilogue, in place over h
      {
        PROF(PK_GEMM, 2.0 * R * DD * DD, f4 * (3.0 * R * DD + DD * DD));
        if (x6)
          launch_gemm_x6_ln(w.o, D, lp.WolP, x6_plane_rows(D), lp.bol, lp.ln1, w.h, rows, D, 0, 0, s,
                            (h_feat && l == 0) ? X6Feat{P.W0, w.geo, d.N, d.n_up} : X6Feat{});
        else
          launch_gemm_ln(w.o, D, lp.WolT, D, lp.bol, lp.ln1, w.h, rows, D, 0, 0, s);
      }
      {
        PROF(PK_GEMM, 2.0 * R * DD * DD, f4 * (2.0 * R * DD + DD * DD));
        if (x6)
          launch_gemm_x6_ln(w.h, D, lp.WmP, x6_plane_rows(D), lp.bm, lp.ln2, w.h, rows, D, 1, 0, s);
        else
          launch_gemm_ln(w.h, D, lp.WmT, D, lp.bm, lp.ln2, w.h, rows, D, 1, 0, s);
      }
      continue;
    }
    // t = h + o (Wo Wl) + bo Wl    (psiformer.py:44-45, two adjacent linear maps folded)
    gemm(w.o, D, lp.Wol, lp.WolT, lp.WolP, D, lp.bol, w.h, D, w.t, D, D, D);
    {
      PROF(PK_LN + (C > 1 ? PK_CH : 0), 0.0, f4 * R * 2.0 * DD);
      launch_layernorm(d, w.t, nullptr, lp.ln1, w.geo, w.h, nw, C, 0, s);
    }
    gemm(w.h, D, lp.Wm, lp.WmT, lp.WmP, D, lp.bm, nullptr, 0, w.o, D, D, D);
    {
      PROF(PK_LN + (C > 1 ? PK_CH : 0), 0.0, f4 * R * 3.0 * DD);
      launch_layernorm(d, nullptr, w.o, lp.ln2, w.geo, w.h, nw, C, 1, s);
    }
  }
  gemm(w.h, D, P.Worb, P.WorbT, P.WorbP, d.ld_orb, P.borb, nullptr, 0, w.F, d.ld_orb, d.orb_cols, D);
  return check_launch();
}

int check_common(dh_handle* h, const void* x, int B, void* ws, size_t ws_bytes, size_t need) {
  if (!h) return fail(DH_EINVAL, "null handle");
  if (!h->params_set) return fail(DH_ESTATE, "parameters not set");
  if (!x || B < 1) return fail(DH_EINVAL, "bad walkers");
  if (!ws || ws_bytes < need) return fail(DH_ENOMEM, "workspace too small");
  return DH_OK;
}

}  // namespace

extern "C" {

int dh_logpsi(dh_handle* h, const float* x, int B, float* logpsi, void* ws, size_t ws_bytes, void* stream) {
  const size_t need = h ? dh_workspace_bytes(h, B, 0) : 0;
  if (int rc = check_common(h, x, B, ws, ws_bytes, need)) return rc;
  if (!logpsi) return fail(DH_EINVAL, "null output");
  hipStream_t s = (hipStream_t)stream;
  Work w = carve(h->d, B, 1, ws);
  if (int rc = run_trunk(h, x, B, 1, w, s)) return rc;
  {
    PROF(PK_DET_VALUE, 0.0, 4.0 * B * h->d.N * h->d.ld_orb);
    launch_det_value(h->d, w.F, x, h->p.jastrow, h->norm, logpsi, B, s);
  }
  return check_launch();
}

int dh_mcmc_step(dh_handle* h, float* x, float* lp, int32_t* n_accept, int B, int steps, float width, uint64_t seed,
                 uint64_t counter, int64_t walker_offset, const float* noise, void* ws, size_t ws_bytes,
                 void* stream) {
  const size_t need = h ? dh_workspace_bytes(h, B, 0) : 0;
  if (int rc = check_common(h, x, B, ws, ws_bytes, need)) return rc;
  if (!lp || !n_accept || steps < 0) return fail(DH_EINVAL, "bad MCMC arguments");
  hipStream_t s = (hipStream_t)stream;
  const Dims& d = h->d;
  Work w = carve(d, B, 1, ws);
  // initial log-probability (mcmc.py:142)
  if (int rc = run_trunk(h, x, B, 1, w, s)) return rc;
  {
    PROF(PK_DET_VALUE, 0.0, 4.0 * B * d.N * d.ld_orb);
    launch_det_value(d, w.F, x, h->p.jastrow, h->norm, w.logpsi, B, s);
  }
  launch_lp_from_logpsi(w.logpsi, lp, n_accept, B, s);
  const size_t nstride = (size_t)B * (2 * d.N + 1);
  for (int st = 0; st < steps; ++st) {
    const float* nz = noise ? noise + st * nstride : nullptr;
    const uint64_t step = counter + (uint64_t)st;
    {
      PROF(PK_MCMC, 0.0, 16.0 * B * d.N);
      launch_propose(d, x, w.x2, B, width, seed, step, walker_offset, nz, 0, s);
    }
    if (int rc = run_trunk(h, w.x2, B, 1, w, s)) return rc;
    {
      PROF(PK_DET_VALUE, 0.0, 4.0 * B * d.N * d.ld_orb);
      launch_det_value(d, w.F, w.x2, h->p.jastrow, h->norm, w.logpsi, B, s);
    }
    {
      PROF(PK_MCMC, 0.0, 16.0 * B * d.N);
      launch_accept(d, x, w.x2, lp, w.logpsi, n_accept, B, seed, step, walker_offset, nz, 0, s);
    }
  }
  return check_launch();
}

int dh_local_energy(dh_handle* h, const float* x, int B, float* e_l, float* obs, void* ws, size_t ws_bytes,
                    void* stream) {
  const size_t need1 = h ? dh_workspace_bytes(h, 1, 1) : 0;
  if (int rc = check_common(h, x, B, ws, ws_bytes, need1)) return rc;
  if (!e_l || !obs) return fail(DH_EINVAL, "null output");
  const Dims& d = h->d;
  // largest chunk that fits the workspace
  int chunk = B;
  while (chunk > 1 && dh_workspace_bytes(h, chunk, 1) > ws_bytes) chunk = (chunk + 1) / 2;
  hipStream_t s = (hipStream_t)stream;
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nw = std::min(chunk, B - b0);
    Work w = carve(d, nw, d.C, ws);
    const float* xc = x + (size_t)b0 * d.N * 2;
    if (int rc = run_trunk(h, xc, nw, d.C, w, s)) return rc;
    {
      PROF(PK_DET_ENERGY, 0.0, 4.0 * nw * d.N * d.C * d.ld_orb);
      launch_det_energy(d, w.F, xc, w.geo, h->p.jastrow, h->norm, e_l + 2 * (size_t)b0, obs + 8 * (size_t)b0, nw, s);
    }
    if (int rc = check_launch()) return rc;
  }
  return DH_OK;
}

int dh_energy_stats(dh_handle* h, const float* e_l, const float* obs, const int32_t* n_accept, int B, int steps,
                    float* out, void* ws, size_t ws_bytes, void* stream) {
  (void)ws;
  (void)ws_bytes;
  if (!h || !e_l || !obs || !out) return fail(DH_EINVAL, "null argument");
  if (B < 1 || B > 32768) return fail(DH_EINVAL, "dh_energy_stats supports 1 <= B <= 32768");
  launch_stats(e_l, obs, n_accept, B, steps, out, nullptr, (hipStream_t)stream);
  return check_launch();
}

// Debug hook (tests only): run input + trunk + orbital GEMM for B walkers with
// C = 1 (op 0) or 2N+5 (op 1) channels and leave the results in the workspace:
// final trunk activations at float offset 0 ([rows][D]) and orbital features at
// float offset dh_debug_offsets()[1] ([rows][ld_orb]).
int dh_debug_trunk(dh_handle* h, const float* x, int B, int op, void* ws, size_t ws_bytes, void* stream) {
  const size_t need = h ? dh_workspace_bytes(h, B, op) : 0;
  if (int rc = check_common(h, x, B, ws, ws_bytes, need)) return rc;
  Work w = carve(h->d, B, op == 1 ? h->d.C : 1, ws);
  return run_trunk(h, x, B, op == 1 ? h->d.C : 1, w, (hipStream_t)stream);
}

size_t dh_debug_f_offset(const dh_handle* h, int B, int op) {
  Work w = carve(h->d, B, op == 1 ? h->d.C : 1, reinterpret_cast<void*>(size_t(64)));
  return (size_t)(w.F - reinterpret_cast<float*>(size_t(64)));
}

// Test hook: one GEMM launch of kernel variant `variant` (-1 = default).
int dh_debug_gemm(int variant, const float* X, int ldx, const float* W, int ldw, const float* bias, const float* R,
                  int ldr, float* Y, int ldy, int rows, int ncols, int K, int C, void* stream) {
  if (variant >= 100) {
    if (K % 32 != 0) return fail(DH_EINVAL, "NT GEMM needs K % 32 == 0");
    launch_gemm_nt_variant(variant - 100, X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C,
                           (hipStream_t)stream);
  } else {
    launch_gemm_variant(variant < 0 ? 0 : variant, X, ldx, W, ldw, bias, R, ldr, Y, ldy, rows, ncols, K, C,
                        (hipStream_t)stream);
  }
  return check_launch();
}

int dh_debug_x6_plane_rows(int ncols) { return x6_plane_rows(ncols); }

int dh_debug_split_planes(const float* Wt, int ldw, int ncols, int K, uint16_t* Wp, void* stream) {
  if (!Wt || !Wp || ncols < 1 || K < 1) return fail(DH_EINVAL, "bad split_planes args");
  launch_split_planes(Wt, ldw, ncols, K, Wp, (hipStream_t)stream);
  return check_launch();
}

int dh_debug_gemm_x6(int variant, const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias,
                     const float* R, int ldr, float* Y, int ldy, int rows, int ncols, int K, int C, void* stream) {
  if (!gemm_x6_supported(K) || ldp < x6_plane_rows(ncols)) return fail(DH_EINVAL, "bad gemm_x6 args");
  if (variant >= 10 && K > 256) return fail(DH_EINVAL, "persistent gemm_x6 needs K <= 256");
  if (variant < 0)
    launch_gemm_x6(X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, (hipStream_t)stream);
  else
    launch_gemm_x6_variant(variant, X, ldx, Wp, ldp, bias, R, ldr, Y, ldy, rows, ncols, K, C, (hipStream_t)stream);
  return check_launch();
}

int dh_debug_gemm_x6_ln(int mode, int nw, const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias,
                        const float* ln, float* h, int rows, int K, void* stream) {
  if (!gemm_x6_supported(K) || K > 256 || ldp < x6_plane_rows(256) || rows < 1 || (mode != 0 && mode != 1))
    return fail(DH_EINVAL, "bad gemm_x6_ln args");
  launch_gemm_x6_ln(X, ldx, Wp, ldp, bias, ln, h, rows, K, mode, nw, (hipStream_t)stream);
  return check_launch();
}

int dh_debug_gemm_ln(int mode, int bm, const float* X, int ldx, const float* Wt, int ldw, const float* bias,
                     const float* ln, float* h, int rows, int K, void* stream) {
  if (!gemm_ln_supported(256, K) || rows < 1 || (mode != 0 && mode != 1)) return fail(DH_EINVAL, "bad gemm_ln args");
  launch_gemm_ln(X, ldx, Wt, ldw, bias, ln, h, rows, K, mode, bm, (hipStream_t)stream);
  return check_launch();
}

int dh_profile_enable(dh_handle* h, int on) {
  if (!h) return fail(DH_EINVAL, "null handle");
  h->prof.on = on != 0;
  h->prof.used = 0;
  return DH_OK;
}

int dh_profile_read(dh_handle* h, double* out, int reset) {
  if (!h || !out) return fail(DH_EINVAL, "null argument");
  for (int i = 0; i < 4 * PK_TOTAL; ++i) out[i] = 0.0;
  for (size_t i = 0; i < h->prof.used; ++i) {
    ProfRec& r = h->prof.recs[i];
    HIP_TRY(hipEventSynchronize(r.b));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
    out[4 * r.kind + 0] += 1.0;
    out[4 * r.kind + 1] += ms;
    out[4 * r.kind + 2] += r.flops;
    out[4 * r.kind + 3] += r.bytes;
  }
  if (reset) h->prof.used = 0;
  return PK_TOTAL;
}

int dh_potential(dh_handle* h, const float* x, int B, float* pe, void* stream) {
  if (!h || !x || !pe || B < 1) return fail(DH_EINVAL, "bad arguments");
  launch_potential(h->d, x, pe, B, (hipStream_t)stream);
  return check_launch();
}

int dh_init_walkers(dh_handle* h, float* x, int B, uint64_t seed, int64_t walker_offset, void* stream) {
  if (!h || !x || B < 1) return fail(DH_EINVAL, "bad arguments");
  launch_init_walkers(h->d, x, B, seed, walker_offset, (hipStream_t)stream);
  return check_launch();
}

}  // extern "C"
