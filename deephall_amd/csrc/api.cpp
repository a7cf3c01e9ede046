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

// envelope first (det.hip): floats of S, FS, E2, Weff for nw walkers (each padded to 256 rows)
size_t env_first_floats(const Dims& d, int nw) {
  const size_t ne = (size_t)nw * d.N, r6 = (size_t)round_up((int)(6 * ne), 256), r1 = (size_t)round_up((int)ne, 256);
  return align64(r6 * 256) + align64(r6 * d.ld_orb) + align64(r1 * env_first_k(d)) + align64(r1 * 256 * 2 * d.N);
}

Work carve(const Dims& d, int nw, int C, void* base) {
  const int rows = nw * d.N * C;
  // + CH_BM rows: the channel chain's electron-aligned 96-row tiles read past the last row
  const size_t rp = (size_t)round_up(std::max(rows, 1) + 96, kWalkerRowPad);
  const size_t nh = align64(rp * d.D);
  size_t nqkv = align64(rp * (size_t)std::max(3 * d.D, d.ld_orb));
  if (C > 1 && env_first(d))  // no F over the channel rows: S, FS, E2, Weff share the q|k|v buffer
    nqkv = align64(std::max(rp * (size_t)(3 * d.D), env_first_floats(d, nw)));
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
// channel-mode (C > 1) launches of GEMM/attention/LayerNorm/input are recorded as kind + PK_CH;
// PK_L1CH: the local energy's layer 1 in one launch (gemm_lnch MODE 2)
constexpr int PK_CH = PK_COUNT, PK_L1CH = PK_COUNT + 4, PK_TOTAL = PK_COUNT + 5;
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

// KFAC plan (dh_kfac_*): factor slots of the statistics buffer, the dense blocks and the
// generic parameters (oracle/kfac.py restates the algorithm), plus device job tables.
struct KfacLayerSlots {
  int A_h, G_q, G_k, G_v, A_o, G_T, A_Wl, G_out, A_h1, G_z;
};
struct KfacHost {
  std::vector<KfacSlot> slots;
  size_t nmat = 0;     // floats of all factor slots
  size_t nstats = 0;   // + the generic diagonal
  int s_feat = -1, s_h0 = -1;
  KfacLayerSlots lay[16];
  int A_orb[2] = {-1, -1}, G_orb[2][2] = {{-1, -1}, {-1, -1}};
  int A_lll = -1, G_lll = -1;  // "sparse" orbitals: the complex lll_weight block
  struct Blk {
    int kseg, bseg, din, dout, a, g;
    float scale;
  };
  std::vector<Blk> blocks;
  std::vector<KfacInvJob> inv;
  std::vector<KfacBlockJob> bjobs;
  std::vector<KfacGemmJob> g1, g2;
  size_t kbuf_doubles = 0;  // inverse matrices + V, T, P V per block
  KfacDevPlan dev{};
  void* dev_mem = nullptr;  // one allocation for the device tables
};

struct dh_handle {
  dh_config cfg;
  Dims d;
  Params p{};
  std::vector<size_t> offsets;      // packed layout, nseg + 1
  std::vector<size_t> ref_offsets;  // reference-tree layout (dh_ref_layout), nseg + 1
  float* params = nullptr;
  float* ref = nullptr;      // reference-layout copy (dh_set_params_ref; needed by the VJP)
  uint16_t* wb = nullptr;    // backward split-bf16 planes (untransposed weights)
  float* wbt = nullptr;      // backward exact-f32 transposed weights (D % 32 != 0)
  float* norm = nullptr;  // sqrt(binom(2Q, Q-m)), M floats (device)
  float* wt = nullptr;    // transposed GEMM weights for the NT kernels (device)
  uint16_t* wp = nullptr;  // split-bf16 weight planes for the x6 kernels (device)
  float* mqk = nullptr;    // layer 1's per-head score forms (attn_val.h, launch_lowrank_qk)
  float* ofw = nullptr;    // layer 1's feature-space output map U^T [256 pad][KO] (launch_ofeat_weight)
  uint16_t* ofp = nullptr;  // its split-bf16 planes [3][x6_plane_rows(D)][KO]
  float* l1w = nullptr;     // layer 1's coefficient-space maps B^T, V^T (launch_l1_basis)
  float* w2t = nullptr;     // envelope first: W2T [256 2N][KE] (launch_env_w2)
  uint16_t* w2p = nullptr;  // its planes
  uint16_t* l1p = nullptr;  // their planes
  int gemm_mode = DH_GEMM_X6_ALL;
  std::vector<float> norm_host;
  bool params_set = false;
  bool ref_set = false;
  bool laughlin = false;          // DH_NETWORK_LAUGHLIN: no parameters, laughlin.hip kernels
  std::vector<int> expo_host;     // Laughlin exponents [2][N] = (Q1 + m_j, Q1 - m_j)
  int* expo = nullptr;            // device copy (uploaded at first use)
  KfacHost* kfac = nullptr;       // KFAC plan (built at first dh_kfac_* call)
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

namespace {
// Laughlin(nspins, flux, cf_flux, excitation_lz) (laughlin.py:19-46): exponents of the
// composite-fermion orbitals, in doubled units (2 Q1, 2 m are integers)
int laughlin_exponents(const dh_config* cfg, std::vector<int>& ex) {
  const int N = cfg->n_up + cfg->n_dn;
  const int p = cfg->cf_flux < 1 ? 1 : cfg->cf_flux;
  const int q2 = cfg->flux - 2 * p * (N - 1);  // 2 Q1
  if (q2 < 0) return fail(DH_EINVAL, "Laughlin: flux too small for N electrons (Q1 < 0)");
  std::vector<int> m2;  // 2 m
  if (N == q2 + 1) {  // ground state
    for (int m = -q2; m <= q2; m += 2) m2.push_back(m);
  } else if (N == q2) {  // quasihole: m = -Q1 .. Q1 without -lz (laughlin.py:66-73)
    const double lz2 = 2.0 * cfg->excitation_lz;
    const int l2 = (int)std::lround(lz2);
    if (std::fabs(lz2 - l2) > 1e-6 || ((l2 - q2) % 2) != 0 || std::abs(l2) > q2)
      return fail(DH_EINVAL, "Laughlin quasihole: impossible excitation_lz");
    for (int m = -q2; m < -l2; m += 2) m2.push_back(m);
    for (int m = q2; m > -l2; m -= 2) m2.push_back(m);
  } else if (N == q2 + 2) {  // quasiparticle: m = -Q1 .. Q1, then the excited orbital (laughlin.py:82-100)
    const double lz2 = 2.0 * cfg->excitation_lz;
    const int l2 = (int)std::lround(lz2);
    if (std::fabs(lz2 - l2) > 1e-6 || ((l2 - q2) % 2) != 0 || std::abs(l2) > q2 + 2)
      return fail(DH_EINVAL, "Laughlin quasiparticle: impossible excitation_lz");
    for (int m = -q2; m <= q2; m += 2) m2.push_back(m);
    m2.push_back(l2);  // last column: A = Q1 + m1, B = Q1 - m1 (each >= -1)
  } else {
    return fail(DH_EINVAL, "Laughlin: filling not supported");
  }
  if ((int)m2.size() != N) return fail(DH_EINVAL, "Laughlin: orbital count mismatch");
  ex.assign(2 * N + 1, 0);
  for (int j = 0; j < N; ++j) {
    ex[j] = (q2 + m2[j]) / 2;
    ex[N + j] = (q2 - m2[j]) / 2;
  }
  ex[2 * N] = N == q2 + 2 ? 1 : 0;  // the kernel's quasiparticle flag
  if (laughlin_smem_bytes(N) > 160 * 1024)
    return fail(DH_EINVAL, "Laughlin: N too large for the one-workgroup kernel's LDS (160 KiB)");
  return DH_OK;
}
}  // namespace

int dh_create(const dh_config* cfg, dh_handle** out) {
  if (!cfg || !out) return fail(DH_EINVAL, "null argument");
  if (cfg->struct_size != sizeof(dh_config))
    return fail(DH_EINVAL, "dh_config.struct_size must equal sizeof(dh_config) (" + std::to_string(sizeof(dh_config)) +
                               " bytes); the caller's binding has a different layout");
  if (cfg->network_type == DH_NETWORK_LAUGHLIN) {
    const int N = cfg->n_up + cfg->n_dn;
    if (cfg->n_up < 0 || cfg->n_dn < 0 || N < 1 || N > 32) return fail(DH_EINVAL, "need 1 <= N <= 32 electrons");
    if (cfg->flux < 1 || cfg->flux > 126) return fail(DH_EINVAL, "Laughlin needs 1 <= flux <= 126");
    if (cfg->interaction_type != DH_INTERACTION_COULOMB && cfg->interaction_type != DH_INTERACTION_HARMONIC)
      return fail(DH_EINVAL, "bad interaction type");
    std::vector<int> ex;
    if (int rc = laughlin_exponents(cfg, ex)) return rc;
    auto* h = new dh_handle();
    h->cfg = *cfg;
    h->laughlin = true;
    h->expo_host = ex;
    Dims& d = h->d;
    d = Dims{};
    d.N = N;
    d.n_up = cfg->n_up;
    d.n_dn = cfg->n_dn;
    d.T = 2 * N;
    d.C = 2 * N + 5;
    d.M = 1;
    d.Q = 0.5f * cfg->flux;
    d.r = cfg->radius > 0.f ? cfg->radius : std::sqrt(d.Q);
    d.H = 1;
    d.dh = 4;
    d.D = 4;
    d.L = 0;
    d.K = 1;
    d.NB = 1;
    d.orb_cols = 0;
    d.ld_orb = 0;
    d.interaction = cfg->interaction_type;
    d.lambda = cfg->interaction_strength;
    h->offsets = {0};
    h->ref_offsets = {0};
    h->params_set = h->ref_set = true;  // nothing to upload
    *out = h;
    return DH_OK;
  }
  if (cfg->network_type != DH_NETWORK_PSIFORMER) return fail(DH_EINVAL, "bad network type");
  const int N = cfg->n_up + cfg->n_dn;
  if (cfg->n_up < 0 || cfg->n_dn < 0 || N < 1 || N > 32) return fail(DH_EINVAL, "need 1 <= N <= 32 electrons");
  if (cfg->flux < 0 || cfg->flux > 126) return fail(DH_EINVAL, "need 0 <= flux <= 126");
  if (cfg->num_layers < 0 || cfg->num_layers > 16) return fail(DH_EINVAL, "need num_layers <= 16");
  if (cfg->ndets < 1 || cfg->ndets > 16) return fail(DH_EINVAL, "need 1 <= determinants <= 16");
  if (cfg->num_heads < 1 || cfg->heads_dim < 1) return fail(DH_EINVAL, "bad attention shape");
  if (cfg->orbital_type != DH_ORBITAL_FULL && cfg->orbital_type != DH_ORBITAL_SPARSE)
    return fail(DH_EINVAL, "orbital type must be DH_ORBITAL_FULL or DH_ORBITAL_SPARSE");
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
  d.sparse = cfg->orbital_type == DH_ORBITAL_SPARSE;
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
  // reference parameter tree, flattened in SURVEY.md Appendix B order (ref_seg below)
  {
    const size_t DD = (size_t)D * D, FNK = (size_t)(d.sparse ? kSparseFeatures : d.M) * N * d.K;
    std::vector<size_t> rs;
    rs.push_back((size_t)4 * D);
    for (int l = 0; l < d.L; ++l)
      for (size_t v : {DD, (size_t)D, DD, (size_t)D, DD, (size_t)D, DD, (size_t)D, DD, (size_t)D, (size_t)D, DD,
                       (size_t)D, (size_t)D, (size_t)D})
        rs.push_back(v);
    for (int i = 0; i < 2 * d.NB; ++i) {
      rs.push_back((size_t)D * FNK);
      rs.push_back(FNK);
    }
    if (d.sparse) {  // Orbitals_0/lll_weight
      rs.push_back((size_t)kSparseFeatures * d.M);
      rs.push_back((size_t)d.M);
    }
    rs.push_back(1);
    rs.push_back(1);
    size_t ro = 0;
    for (size_t v : rs) {
      h->ref_offsets.push_back(ro);
      ro += align64(v);
    }
    h->ref_offsets.push_back(ro);
  }
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
  if (h->mqk) (void)hipFree(h->mqk);
  if (h->ofw) (void)hipFree(h->ofw);
  if (h->ofp) (void)hipFree(h->ofp);
  if (h->l1w) (void)hipFree(h->l1w);
  if (h->w2t) (void)hipFree(h->w2t);
  if (h->w2p) (void)hipFree(h->w2p);
  if (h->l1p) (void)hipFree(h->l1p);
  if (h->ref) (void)hipFree(h->ref);
  if (h->wb) (void)hipFree(h->wb);
  if (h->wbt) (void)hipFree(h->wbt);
  if (h->expo) (void)hipFree(h->expo);
  if (h->kfac) {
    if (h->kfac->dev_mem) (void)hipFree(h->kfac->dev_mem);
    delete h->kfac;
  }
  delete h;
}

int dh_param_layout(const dh_handle* h, size_t* offsets, int n) {
  if (!h) return fail(DH_EINVAL, "null handle");
  const int nseg = (int)h->offsets.size() - 1;
  for (int i = 0; i < n && i <= nseg; ++i) offsets[i] = h->offsets[i];
  return nseg;
}

}  // extern "C"

namespace {

// Reference-tree segment indices (dh_ref_layout)
struct RefSeg {
  int L, NB, sparse;
  int W0() const { return 0; }
  int lay(int l, int k) const { return 1 + 15 * l + k; }  // k: Wq bq Wk bk Wv bv Wo bo Wl ln1s ln1b Wm bm ln2s ln2b
  int orb_kernel(int i) const { return 1 + 15 * L + 2 * i; }
  int orb_bias(int i) const { return 2 + 15 * L + 2 * i; }
  int lll(int k) const { return 1 + 15 * L + 4 * NB + k; }  // "sparse": lll_weight kernel, bias
  int jas(int k) const { return 1 + 15 * L + 4 * NB + (sparse ? 2 : 0) + k; }
};
enum { RWq = 0, Rbq, RWk, Rbk, RWv, Rbv, RWo, Rbo, RWl, Rln1s, Rln1b, RWm, Rbm, Rln2s, Rln2b };

// Device pointers of the packed segments.
void assign_packed(dh_handle* h) {
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
}

// Derived weight copies: transposed + split-bf16 planes for the forward NT/x6 GEMMs, and the
// backward copies (planes of the untransposed weights, or W^T when D % 32 != 0).
int derive_weights(dh_handle* h, hipStream_t st) {
  const Dims& d = h->d;
  const int D = d.D;
  if (d.L > 0 && d.dh == 64) {  // layer 1's score forms of the feature-space attention
    if (!h->mqk) HIP_TRY(hipMalloc(&h->mqk, (size_t)d.H * kMqkStride * sizeof(float)));
    launch_lowrank_qk(d, h->p.W0qkv, h->p.layer[0].bqkv, h->mqk, st);
    h->p.Mqk = h->mqk;
    // layer 1's attention output in feature space (round 6): o = o~ Wv~, so o Wol = o~ U with
    // U = Wv~ Wol per head (8 H rows, zero padded to KO); the NT / x6 kernels read U^T
    const int KO = ofeat_k(d);
    const size_t nu = (size_t)round_up(d.D, kRowPad) * KO;
    if (!h->ofw) HIP_TRY(hipMalloc(&h->ofw, nu * sizeof(float)));
    if (!h->ofp) HIP_TRY(hipMalloc(&h->ofp, (size_t)3 * x6_plane_rows(d.D) * KO * sizeof(uint16_t)));
    HIP_TRY(hipMemsetAsync(h->ofw, 0, nu * sizeof(float), st));
    launch_ofeat_weight(d, h->p.W0qkv, h->p.layer[0].bqkv, h->p.layer[0].Wol, h->ofw, st);
    launch_split_planes(h->ofw, KO, d.D, KO, h->ofp, st);
    h->p.UT = h->ofw;
    h->p.UP = h->ofp;
    // layer 1 in coefficient space (gemm_lnch MODE 2): B^T, V^T [256 pad][32] and their planes
    if (d.H == 4) {
      const size_t nb = (size_t)round_up(d.D, kRowPad) * 32, pb = (size_t)3 * x6_plane_rows(d.D) * 32;
      if (!h->l1w) HIP_TRY(hipMalloc(&h->l1w, 2 * nb * sizeof(float)));
      if (!h->l1p) HIP_TRY(hipMalloc(&h->l1p, 2 * pb * sizeof(uint16_t)));
      HIP_TRY(hipMemsetAsync(h->l1w, 0, 2 * nb * sizeof(float), st));
      const LayerParams& l0 = h->p.layer[0];
      launch_l1_basis(d, h->p.W0, h->ofw, l0.bol, l0.ln1, l0.Wm, l0.bm, h->l1w, h->l1w + nb, st);
      launch_split_planes(h->l1w, 32, d.D, 32, h->l1p, st);
      launch_split_planes(h->l1w + nb, 32, d.D, 32, h->l1p + pb, st);
      h->p.L1BP = h->l1p;
      h->p.L1VP = h->l1p + pb;
      h->p.L1VT = h->l1w + nb;
    }
  }
  if (d.D % 32 == 0) {
    // Transposed copies Wt[n][k] (rows zero-padded to 256) of every GEMM weight, for the
    // NT GEMM kernels whose LDS-DMA staging wants k contiguous in both operands.
    const size_t sq = (size_t)round_up(D, kRowPad) * D, sqkv = (size_t)round_up(3 * D, kRowPad) * D;
    const size_t sorb = (size_t)round_up(d.orb_cols, kRowPad) * D;
    const size_t total = (size_t)d.L * (sqkv + 2 * sq) + sorb;
    if (!h->wt) HIP_TRY(hipMalloc(&h->wt, total * sizeof(float)));
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
    if (env_first(d)) {  // envelope first (C4 / C5): the envelope-coefficient map of Worb
      const int KE = env_first_k(d), n2 = 256 * 2 * d.N;
      if (!h->w2t) HIP_TRY(hipMalloc(&h->w2t, (size_t)n2 * KE * sizeof(float)));
      if (!h->w2p) HIP_TRY(hipMalloc(&h->w2p, (size_t)3 * x6_plane_rows(n2) * KE * sizeof(uint16_t)));
      launch_env_w2(d, h->p.Worb, h->w2t, st);
      launch_split_planes(h->w2t, KE, n2, KE, h->w2p, st);
      h->p.W2T = h->w2t;
      h->p.W2P = h->w2p;
    }
    // backward planes: the untransposed W [K = D][n] read as a transposed weight with D
    // output rows and contraction length n (dX = dY W^T)
    const int pr = x6_plane_rows(D);
    const size_t bq = (size_t)3 * pr * 3 * D, bd = (size_t)3 * pr * D, bo = (size_t)3 * pr * d.ld_orb;
    const size_t btotal = (size_t)d.L * (bq + 2 * bd) + bo;
    if (!h->wb) HIP_TRY(hipMalloc(&h->wb, btotal * sizeof(uint16_t)));
    uint16_t* b = h->wb;
    for (int l = 0; l < d.L; ++l) {
      LayerParams& lp = h->p.layer[l];
      launch_split_planes(lp.Wqkv, 3 * D, D, 3 * D, b, st);
      lp.WqkvB = b;
      b += bq;
      launch_split_planes(lp.Wol, D, D, D, b, st);
      lp.WolB = b;
      b += bd;
      launch_split_planes(lp.Wm, D, D, D, b, st);
      lp.WmB = b;
      b += bd;
    }
    launch_split_planes(h->p.Worb, d.ld_orb, D, d.ld_orb, b, st);
    h->p.WorbB = b;
  } else {
    // exact-f32 backward: W^T [n][D]
    const size_t total = (size_t)d.L * (5 * (size_t)D * D) + (size_t)d.ld_orb * D;
    if (!h->wbt) HIP_TRY(hipMalloc(&h->wbt, total * sizeof(float)));
    HIP_TRY(hipMemsetAsync(h->wbt, 0, total * sizeof(float), st));
    float* q = h->wbt;
    for (int l = 0; l < d.L; ++l) {
      LayerParams& lp = h->p.layer[l];
      launch_transpose(lp.Wqkv, 3 * D, D, 3 * D, q, D, st);
      lp.WqkvBT = q;
      q += (size_t)3 * D * D;
      launch_transpose(lp.Wol, D, D, D, q, D, st);
      lp.WolBT = q;
      q += (size_t)D * D;
      launch_transpose(lp.Wm, D, D, D, q, D, st);
      lp.WmBT = q;
      q += (size_t)D * D;
    }
    launch_transpose(h->p.Worb, d.ld_orb, D, d.orb_cols, q, D, st);
    h->p.WorbBT = q;
  }
  HIP_TRY(hipGetLastError());
  return DH_OK;
}

int ensure_param_buffers(dh_handle* h) {
  if (!h->params) HIP_TRY(hipMalloc(&h->params, h->offsets.back() * sizeof(float)));
  if (!h->norm) {
    HIP_TRY(hipMalloc(&h->norm, h->norm_host.size() * sizeof(float)));
    HIP_TRY(hipMemcpy(h->norm, h->norm_host.data(), h->norm_host.size() * sizeof(float), hipMemcpyHostToDevice));
  }
  return DH_OK;
}

// Pack the reference tree (h->ref) into the kernel layout: concatenations, zero padding and
// the three folds (Wo Wl, bo Wl, W0 Wqkv) as double-accumulated products.
void pack_from_ref(dh_handle* h, hipStream_t st) {
  const Dims& d = h->d;
  const int D = d.D, MNK = d.M * d.N * d.K;
  const RefSeg R{d.L, d.NB, d.sparse};
  auto ref = [&](int seg) { return h->ref + h->ref_offsets[seg]; };
  auto pk = [&](int seg) { return h->params + h->offsets[seg]; };
  launch_copy2d(ref(R.W0()), D, pk(0), D, 4, D, st);
  for (int l = 0; l < d.L; ++l) {
    const int b = 1 + 8 * l;
    for (int part = 0; part < 3; ++part) {
      launch_copy2d(ref(R.lay(l, RWq + 2 * part)), D, pk(b + 0) + part * D, 3 * D, D, D, st);
      launch_copy2d(ref(R.lay(l, Rbq + 2 * part)), D, pk(b + 1) + part * D, 3 * D, 1, D, st);
    }
    launch_small_gemm(D, D, D, ref(R.lay(l, RWo)), D, 0, ref(R.lay(l, RWl)), D, 0, pk(b + 2), D, 0, st);
    launch_small_gemm(1, D, D, ref(R.lay(l, Rbo)), D, 0, ref(R.lay(l, RWl)), D, 0, pk(b + 3), D, 0, st);
    launch_copy2d(ref(R.lay(l, Rln1s)), D, pk(b + 4), D, 1, D, st);
    launch_copy2d(ref(R.lay(l, Rln1b)), D, pk(b + 4) + D, D, 1, D, st);
    launch_copy2d(ref(R.lay(l, RWm)), D, pk(b + 5), D, D, D, st);
    launch_copy2d(ref(R.lay(l, Rbm)), D, pk(b + 6), D, 1, D, st);
    launch_copy2d(ref(R.lay(l, Rln2s)), D, pk(b + 7), D, 1, D, st);
    launch_copy2d(ref(R.lay(l, Rln2b)), D, pk(b + 7) + D, D, 1, D, st);
  }
  const int so = 1 + 8 * d.L;
  launch_copy2d(nullptr, 0, pk(so), d.ld_orb, D, d.ld_orb, st);
  launch_copy2d(nullptr, 0, pk(so + 1), d.ld_orb, 1, d.ld_orb, st);
  for (int i = 0; i < 2 * d.NB; ++i) {
    if (d.sparse)  // fold lll_weight into the full layout (blocks.py:52-62)
      launch_sparse_fold(ref(R.orb_kernel(i)), ref(R.orb_bias(i)), ref(R.lll(0)), ref(R.lll(1)), i % 2 == 0, D,
                         d.N * d.K, d.M, pk(so) + i * MNK, d.ld_orb, pk(so + 1) + i * MNK, st);
    else {
      launch_copy2d(ref(R.orb_kernel(i)), MNK, pk(so) + i * MNK, d.ld_orb, D, MNK, st);
      launch_copy2d(ref(R.orb_bias(i)), MNK, pk(so + 1) + i * MNK, d.ld_orb, 1, MNK, st);
    }
  }
  launch_copy2d(ref(R.jas(0)), 1, pk(so + 2), 1, 1, 1, st);
  launch_copy2d(ref(R.jas(1)), 1, pk(so + 2) + 1, 1, 1, 1, st);
  if (d.L > 0) launch_small_gemm(4, 3 * D, D, pk(0), D, 0, pk(1), 3 * D, 0, pk(so + 3), 3 * D, 0, st);
}

}  // namespace

extern "C" {

int dh_set_params(dh_handle* h, const float* params, size_t count, void* stream) {
  if (h && h->laughlin) return count == 0 ? DH_OK : fail(DH_EINVAL, "the Laughlin wavefunction has no parameters");
  if (!h || !params) return fail(DH_EINVAL, "null argument");
  if (count != h->offsets.back()) return fail(DH_EINVAL, "parameter count mismatch");
  if (int rc = ensure_param_buffers(h)) return rc;
  HIP_TRY(hipMemcpyAsync(h->params, params, count * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  assign_packed(h);
  if (int rc = derive_weights(h, (hipStream_t)stream)) return rc;
  h->params_set = true;
  h->ref_set = false;  // a packed upload has no reference tree (the VJP needs one)
  return DH_OK;
}

int dh_ref_layout(const dh_handle* h, size_t* offsets, int n) {
  if (!h) return fail(DH_EINVAL, "null handle");
  const int nseg = (int)h->ref_offsets.size() - 1;
  for (int i = 0; i < n && i <= nseg; ++i) offsets[i] = h->ref_offsets[i];
  return nseg;
}

int dh_set_params_ref(dh_handle* h, const float* ref, size_t count, void* stream) {
  if (h && h->laughlin) return count == 0 ? DH_OK : fail(DH_EINVAL, "the Laughlin wavefunction has no parameters");
  if (!h || !ref) return fail(DH_EINVAL, "null argument");
  if (count != h->ref_offsets.back()) return fail(DH_EINVAL, "reference parameter count mismatch");
  if (int rc = ensure_param_buffers(h)) return rc;
  if (!h->ref) HIP_TRY(hipMalloc(&h->ref, count * sizeof(float)));
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(hipMemcpyAsync(h->ref, ref, count * sizeof(float), hipMemcpyDeviceToDevice, st));
  pack_from_ref(h, st);
  HIP_TRY(hipGetLastError());
  assign_packed(h);
  if (int rc = derive_weights(h, st)) return rc;
  h->params_set = true;
  h->ref_set = true;
  return DH_OK;
}

int dh_set_gemm_mode(dh_handle* h, int mode) {
  if (!h) return fail(DH_EINVAL, "null handle");
  if (mode != DH_GEMM_F32 && mode != DH_GEMM_X6 && mode != DH_GEMM_X6_ALL && mode != DH_GEMM_X6_ALL_UNFUSED)
    return fail(DH_EINVAL, "bad GEMM mode");
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
// geo_ready: w.geo already holds the walkers' geometry (written by the MCMC proposal); the
// input kernel is then skipped when the geometry is all it would write.
int run_trunk(dh_handle* h, const float* x, int nw, int C, const Work& w, hipStream_t s, bool geo_ready = false,
              bool keep_h = false) {
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
                  (C > 1 ? h->gemm_mode != DH_GEMM_F32
                         : (h->gemm_mode == DH_GEMM_X6_ALL || h->gemm_mode == DH_GEMM_X6_ALL_UNFUSED));
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
  const bool fused = fold && attention_takes_features(d, C);
  const int KO = ofeat_k(d);  // layer 1's o~ row length (fused channel attention, chain prologue)
  // log psi, split-bf16: layer 1's residual h = features W0 is formed in the epilogue of
  // its LayerNorm GEMM from geo, so the input kernel only writes the geometry
  const bool h_feat = C == 1 && fused && x6 && ln_fused;
  // log psi, split-bf16, D = 256: each layer's tail (Wo Wl + LN1, Wm + LN2) and the next
  // linear map (the next layer's q|k|v, or the orbitals) run as ONE launch (chain_x6s_kernel).
  // Its 96-row tiles suit up to ~64K walker rows (C2 24576: 256 tiles, C4 40960: 427); at
  // C5 (81920 rows, 2320 orbital columns) the separate GEMMs with 128-row LayerNorm tiles are
  // faster (102.6 vs 103.6 ms per step, tools/chain_bench.py, profiles/)
  // At N = 20 (C5) the chain is taken past 64K rows too (round 6): layer 1 with its attention in
  // the prologue (attention, two LayerNorm GEMMs and layer 2's q|k|v in one launch), layer 2 with
  // the 2320-column orbital map as its last pass (C5 73.5 -> 74.2 K E_L/s, 2.53 -> 2.59 M
  // walker-steps/s same box, profiles/r06_v35_chain_big20_ab.txt)
  const bool chain_any = C == 1 && x6 && ln_fused && D == 256;
  auto chain_at = [&](int l) {
    (void)l;
    return chain_any && (rows < 65536 || d.N >= 20);
  };
  // local energy, split-bf16, D = 256, N <= 8: GEMM + channel LayerNorm fused per map
  const bool lnch = C > 1 && x6 && C == 2 * d.N + 5 && h->gemm_mode != DH_GEMM_X6_ALL_UNFUSED &&
                    gemm_lnch_supported(d.N, D);
  // local energy, gemm_lnch: layer 1's residual h0 = f W0 is formed in the first launch's
  // epilogue from geo
  const bool lnch_feat = lnch && fused;  // fused: the input kernel writes no q|k|v
  // local energy at N = 10, 20 (GEMM + layernorm_ch_quad): the same residual formed by the
  // first LayerNorm launch, the GEMM writing t without it
  const bool ln_feat = C > 1 && !lnch && fused && D == 256 && (d.N == 10 || d.N == 20);
  {
    const bool wq = fold && !fused;
    if (!(geo_ready && h_feat && !wq)) {
      PROF(PK_INPUT + (C > 1 ? PK_CH : 0), 8.0 * R * DD * (wq ? 4 : 1), f4 * R * DD * (wq ? 4 : 1));
      launch_input(d, x, P.W0, wq ? P.W0qkv : nullptr, wq ? P.layer[0].bqkv : nullptr, (h_feat || lnch_feat || ln_feat) ? nullptr : w.h,
                   wq ? w.qkv : nullptr, w.geo, nw, C, s);
    }
  }
  for (int l = 0; l < d.L; ++l) {
    const LayerParams& lp = P.layer[l];
    const bool chain = chain_at(l);
    if (l > 0 && !chain_at(l - 1))  // (a chained layer's last pass wrote this layer's q|k|v)
      gemm(w.h, D, lp.Wqkv, lp.WqkvT, lp.WqkvP, 3 * D, lp.bqkv, nullptr, 0, w.qkv, 3 * D, 3 * D, D);
    // log psi, chain form: layer 1's attention runs in the chain kernel's prologue (its o
    // never leaves the CU; attn_val.h)
    const bool attn_in_chain = chain && fused && l == 0 && chain_attn_supported(d.N, d.H, d.dh);
    if (!attn_in_chain) {
      const bool f = fused && l == 0;
      PROF(PK_ATTN + (C > 1 ? PK_CH : 0), 0.0, f4 * R * (f ? 1.0 : 4.0) * DD);
      launch_attention(d, w.qkv, w.geo, w.o, nw, C, s, f ? P.W0qkv : nullptr, f ? lp.bqkv : nullptr,
                       f ? P.Mqk : nullptr);
    }
    if (chain) {
      const bool last = l + 1 == d.L;
      const int n3 = last ? d.orb_cols : 3 * D;
      PROF(PK_GEMM, 2.0 * R * DD * (2.0 * DD + n3), f4 * (2.0 * R * DD + R * n3 + 2.0 * DD * DD + DD * n3));
      X6Feat feat{};
      if (h_feat && l == 0) feat = X6Feat{P.W0, w.geo, d.N, d.n_up};
      if (attn_in_chain) {
        feat.W0qkv = P.W0qkv;
        feat.bqkv = lp.bqkv;
        feat.Mqk = P.Mqk;
        feat.L1V = P.L1VP;
        feat.L1B = P.L1BP;
      }
      // layer 1 with its attention in the prologue: P1 contracts the o~ planes with U (K = 32)
      launch_chain_x6(w.o, attn_in_chain ? P.UP : lp.WolP, x6_plane_rows(D), lp.bol, lp.ln1, lp.WmP, x6_plane_rows(D),
                      lp.bm, lp.ln2, last ? P.WorbP : P.layer[l + 1].WqkvP, x6_plane_rows(n3),
                      last ? P.borb : P.layer[l + 1].bqkv, n3, last ? w.F : w.qkv, last ? d.ld_orb : 3 * D, w.h, rows,
                      feat, s, /*store_h=*/!last || keep_h);  // the last layer's h is dead: only its orbitals are read
      continue;
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
    if (lnch && l == 0 && fused && d.H == 4) {
      // layer 1 whole in one launch from the o~ rows (gemm_lnch MODE 2: LN1, Wm and tanh_ch in
      // coefficient space, the residual h1 from the same 32-deep rows, LN2)
      PROF(PK_L1CH, 2.0 * R * DD * 3.0 * KO, f4 * (R * KO + R * DD));
      launch_gemm_lnch(d.N, w.o, P.UP, x6_plane_rows(D), lp.bol, lp.ln2, w.geo, w.h, nw * d.N, 2, s, P.W0, d.n_up, KO,
                       P.L1VP, P.L1BP);
      continue;
    }
    if (lnch) {
      // channel rows: each linear map and its channel LayerNorm in one launch, in place over h
      // (gemm_lnch.hip; the GEMM output never reaches HBM)
      {
        // layer 1 (fused attention): the o~ rows against U, K = ofeat_k
        const bool of = fused && l == 0;
        const double KK = of ? KO : DD;
        PROF(PK_GEMM + PK_CH, 2.0 * R * DD * KK, f4 * (R * KK + 2.0 * R * DD + DD * KK));
        launch_gemm_lnch(d.N, w.o, of ? P.UP : lp.WolP, x6_plane_rows(D), lp.bol, lp.ln1, w.geo, w.h, nw * d.N, 0, s,
                         (lnch_feat && l == 0) ? P.W0 : nullptr, d.n_up, of ? KO : D);
      }
      {
        PROF(PK_GEMM + PK_CH, 2.0 * R * DD * DD, f4 * (3.0 * R * DD + DD * DD));
        launch_gemm_lnch(d.N, w.h, lp.WmP, x6_plane_rows(D), lp.bm, lp.ln2, w.geo, w.h, nw * d.N, 1, s);
      }
      continue;
    }
    if (C > 1 && l == 0 && fused && ln_feat && P.L1VT && layer1_ch_supported(d) &&
        h->gemm_mode != DH_GEMM_X6_ALL_UNFUSED) {  // (the unfused mode keeps the two-kernel form: tests)
      // layer 1 at N = 10, 20 in one launch from the o~ rows (layernorm.hip layer1_ch_kernel:
      // LN_ch1, Wm in coefficient space, tanh_ch, LN_ch2)
      PROF(PK_L1CH, 2.0 * R * DD * (24.0 + 27.0), f4 * (R * KO + R * DD));
      launch_layer1_ch(d, w.o, P.UT, P.L1VT, P.W0, lp.bol, lp.ln1, lp.ln2, w.geo, w.h, nw, s);
      continue;
    }
    // t = h + o (Wo Wl) + bo Wl    (psiformer.py:44-45, two adjacent linear maps folded);
    // layer 1 with ln_feat: t = o (Wo Wl) + bo Wl, the LayerNorm adds h0 = f W0
    const bool lf = ln_feat && l == 0;
    if (fused && l == 0 && C > 1)  // layer 1's o~ rows (attention_feat2_kernel) against U
      gemm(w.o, KO, nullptr, P.UT, P.UP, KO, lp.bol, lf ? nullptr : w.h, D, w.t, D, D, KO);
    else
      gemm(w.o, D, lp.Wol, lp.WolT, lp.WolP, D, lp.bol, lf ? nullptr : w.h, D, w.t, D, D, D);
    {
      PROF(PK_LN + (C > 1 ? PK_CH : 0), 0.0, f4 * R * 2.0 * DD);
      launch_layernorm(d, w.t, nullptr, lp.ln1, w.geo, w.h, nw, C, 0, s, lf ? P.W0 : nullptr);
    }
    gemm(w.h, D, lp.Wm, lp.WmT, lp.WmP, D, lp.bm, nullptr, 0, w.o, D, D, D);
    {
      PROF(PK_LN + (C > 1 ? PK_CH : 0), 0.0, f4 * R * 3.0 * DD);
      launch_layernorm(d, nullptr, w.o, lp.ln2, w.geo, w.h, nw, C, 1, s);
    }
  }
  // (the envelope-first local energy maps only six special rows per electron, det.hip)
  if ((d.L == 0 || !chain_at(d.L - 1)) && !(C > 1 && env_first(d)))
    gemm(w.h, D, P.Worb, P.WorbT, P.WorbP, d.ld_orb, P.borb, nullptr, 0, w.F, d.ld_orb, d.orb_cols, D);
  return check_launch();
}

int ensure_expo(dh_handle* h) {
  if (h->expo) return DH_OK;
  HIP_TRY(hipMalloc(&h->expo, h->expo_host.size() * sizeof(int)));
  HIP_TRY(hipMemcpy(h->expo, h->expo_host.data(), h->expo_host.size() * sizeof(int), hipMemcpyHostToDevice));
  return DH_OK;
}

// log psi of nw walkers into logpsi [nw][2]: the Psiformer pass or the Laughlin kernel
// epi (Psiformer only): the MCMC accept / next proposal fused into the value kernel
int value_pass(dh_handle* h, const float* x, int nw, const Work& w, float* logpsi, hipStream_t s,
               bool geo_ready = false, const McmcEpi& epi = McmcEpi{}) {
  if (h->laughlin) {
    if (int rc = ensure_expo(h)) return rc;
    PROF(PK_DET_VALUE, 0.0, 8.0 * nw * h->d.N);
    launch_laughlin(h->d, x, h->expo, logpsi, nullptr, nullptr, nw, s);
    return check_launch();
  }
  if (int rc = run_trunk(h, x, nw, 1, w, s, geo_ready)) return rc;
  {
    PROF(PK_DET_VALUE, 0.0, 4.0 * nw * h->d.N * h->d.ld_orb);
    launch_det_value(h->d, w.F, x, h->p.jastrow, h->norm, logpsi, nw, s, epi);
  }
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
  return value_pass(h, x, B, w, logpsi, s);
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
  if (int rc = value_pass(h, x, B, w, w.logpsi, s)) return rc;
  launch_lp_from_logpsi(w.logpsi, lp, n_accept, B, s);
  const size_t nstride = (size_t)B * (2 * d.N + 1);
  // step st: accept of st - 1 and the proposal of st in one launch (which also writes the
  // proposal's geometry, so the trunk skips its input kernel); the last accept alone
  const bool geo = !h->laughlin;
  // Psiformer: step st's accept and step st + 1's proposal run in the epilogue of step st's
  // value kernel (McmcEpi, det.hip): one launch fewer per move, bit-identical results; the
  // Laughlin kernel keeps the separate accept / proposal launches
  const bool fuse = geo;
  for (int st = 0; st < steps; ++st) {
    const float* nz = noise ? noise + st * nstride : nullptr;
    const uint64_t step = counter + (uint64_t)st;
    if (!fuse || st == 0) {
      PROF(PK_MCMC, 0.0, 16.0 * B * d.N);
      if (st == 0)
        launch_propose(d, x, w.x2, B, width, seed, step, walker_offset, nz, 0, s, geo ? w.geo : nullptr);
      else
        launch_accept_propose(d, x, w.x2, geo ? w.geo : nullptr, lp, w.logpsi, n_accept, B, width, seed, step - 1,
                              walker_offset, noise ? noise + (st - 1) * nstride : nullptr, nz, s);
    }
    McmcEpi epi{};
    if (fuse) {
      epi.on = 1;
      epi.propose = st + 1 < steps;
      epi.x = x;
      epi.x2 = w.x2;
      epi.geo = w.geo;
      epi.lp = lp;
      epi.nacc = n_accept;
      epi.width = width;
      epi.seed = seed;
      epi.step = step;
      epi.woff = walker_offset;
      epi.noise = nz;
      epi.noise2 = (noise && st + 1 < steps) ? noise + (st + 1) * nstride : nullptr;
    }
    if (int rc = value_pass(h, w.x2, B, w, w.logpsi, s, geo, epi)) return rc;
  }
  if (steps > 0 && !fuse) {
    PROF(PK_MCMC, 0.0, 16.0 * B * d.N);
    launch_accept(d, x, w.x2, lp, w.logpsi, n_accept, B, seed, counter + (uint64_t)(steps - 1), walker_offset,
                  noise ? noise + (steps - 1) * nstride : nullptr, 0, s);
  }
  return check_launch();
}

int dh_local_energy(dh_handle* h, const float* x, int B, float* e_l, float* obs, void* ws, size_t ws_bytes,
                    void* stream) {
  const size_t need1 = h ? dh_workspace_bytes(h, 1, 1) : 0;
  if (int rc = check_common(h, x, B, ws, ws_bytes, need1)) return rc;
  if (!e_l || !obs) return fail(DH_EINVAL, "null output");
  const Dims& d = h->d;
  if (h->laughlin) {
    if (int rc = ensure_expo(h)) return rc;
    hipStream_t s = (hipStream_t)stream;
    PROF(PK_DET_ENERGY, 0.0, 48.0 * B);
    launch_laughlin(d, x, h->expo, nullptr, e_l, obs, B, s);
    return check_launch();
  }
  // largest chunk that fits the workspace
  int chunk = B;
  while (chunk > 1 && dh_workspace_bytes(h, chunk, 1) > ws_bytes) chunk = (chunk + 1) / 2;
  hipStream_t s = (hipStream_t)stream;
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nw = std::min(chunk, B - b0);
    Work w = carve(d, nw, d.C, ws);
    const float* xc = x + (size_t)b0 * d.N * 2;
    if (int rc = run_trunk(h, xc, nw, d.C, w, s)) return rc;
    if (env_first(d)) {
      // envelope first (det.hip): PhiC straight from h, then the determinant algebra
      const size_t ne = (size_t)nw * d.N, r6 = (size_t)round_up((int)(6 * ne), 256);
      const size_t r1 = (size_t)round_up((int)ne, 256);
      float* S = w.qkv;
      float* FS = S + align64(r6 * 256);
      float* E2 = FS + align64(r6 * d.ld_orb);
      float* Weff = E2 + align64(r1 * env_first_k(d));
      {
        PROF(PK_GEMM + PK_CH, 2.0 * 6 * ne * d.D * d.orb_cols + 2.0 * ne * env_first_k(d) * 256 * 2 * d.N +
                                  2.0 * ne * d.C * 256 * 2 * d.N,
             4.0 * ne * (7.0 * 256 + 6.0 * d.ld_orb + env_first_k(d) + 2.0 * 256 * 2 * d.N + d.C * 256));
        launch_env_first(d, w.h, w.geo, xc, h->norm, h->p.WorbT, h->p.borb, h->p.WorbP, h->p.W2T, h->p.W2P,
                         h->gemm_mode != DH_GEMM_F32, nw, S, FS, E2, Weff, w.o, s);
      }
      {
        PROF(PK_DET_ENERGY, 0.0, 8.0 * nw * d.C * d.N * d.N);
        launch_det_energy_pc(d, xc, w.geo, h->p.jastrow, h->norm, e_l + 2 * (size_t)b0, obs + 8 * (size_t)b0, nw, s, w.o);
      }
      if (int rc = check_launch()) return rc;
      continue;
    }
    {
      PROF(PK_DET_ENERGY, 0.0, 4.0 * nw * d.N * d.C * d.ld_orb);
      // the trunk's o buffer (rows x D floats) is free here and holds nw K C N N complex when 2 K N <= D
      launch_det_energy(d, w.F, xc, w.geo, h->p.jastrow, h->norm, e_l + 2 * (size_t)b0, obs + 8 * (size_t)b0, nw, s,
                        det_precontract(d) ? w.o : nullptr);
    }
    if (int rc = check_launch()) return rc;
  }
  return DH_OK;
}

}  // extern "C"

namespace {

// Workspace of one gradient (VJP) pass over nw walkers (floats).
struct GradWork {
  float *geo, *logpsi, *F, *dF, *jg;
  float *hs[17], *qkv[16], *o[16], *t[16], *h1[16], *z[16];  // saved activations per layer
  float *dh, *dA, *dz, *dqkv, *dO;                            // backward temporaries
  float *P, *dWol, *dbol;                                     // chunk partials, folded-weight grads
  float *dWorb, *dborb;                                       // full-layout orbital grads ("sparse")
  float *fgrad, *ctf;                                         // KFAC: Fisher tangent (ref layout), cotangent
  float *kfs0, *kfs1;                                         // KFAC "sparse": featured-orbital rows
  size_t total_bytes;
};

GradWork carve_grad(const Dims& d, int nw, void* base, size_t nref = 0) {
  const int rows = nw * d.N;
  const size_t rp = (size_t)round_up(std::max(rows, 1), kRowPad);
  const size_t D = d.D, nh = align64(rp * D);
  GradWork w{};
  size_t off = 0;
  auto take = [&](size_t n) {
    float* p = base ? reinterpret_cast<float*>(base) + off : nullptr;
    off += align64(n);
    return p;
  };
  w.geo = take((size_t)rows * 4);
  w.logpsi = take((size_t)nw * 2);
  w.jg = take((size_t)nw * 2);
  w.F = take(rp * d.ld_orb);
  w.dF = take(rp * d.ld_orb);
  for (int l = 0; l <= d.L; ++l) w.hs[l] = take(nh);
  for (int l = 0; l < d.L; ++l) {
    w.qkv[l] = take(3 * nh);
    w.o[l] = take(nh);
    w.t[l] = take(nh);
    w.h1[l] = take(nh);
    w.z[l] = take(nh);
  }
  w.dh = take(nh);
  w.dA = take(nh);
  w.dz = take(nh);
  w.dqkv = take(3 * nh);
  w.dO = take(nh);
  const size_t nch = (size_t)grad_chunks(rows);
  const size_t MNK = (size_t)d.M * d.N * d.K;
  // (KFAC: the orbital output Gram matrices need MNK^2 per chunk)
  // ("sparse" KFAC: the featured-orbital tangent Gram (8 N K)^2, the lll_weight factors over
  //  N K times as many rows: 64 and M^2 per chunk of those)
  const size_t F8 = (size_t)8 * d.N * d.K, pls = (nref && d.sparse) ? std::max(F8 * F8, (size_t)d.N * d.K *
                                                                       std::max<size_t>(64, (size_t)d.M * d.M)) : 0;
  const size_t pw = std::max({D * 3 * D, D * (size_t)d.ld_orb, (size_t)4 * D, nref ? MNK * MNK : (size_t)0, pls});
  const size_t pc = std::max((size_t)3 * D, (size_t)d.ld_orb);
  w.P = take(std::max({nch * pw, nch * pc, (size_t)ln_bwd_blocks(rows) * 2 * D, (size_t)nw * 2}));
  w.dWol = take(D * D);
  w.dbol = take(D);
  if (d.sparse) {
    w.dWorb = take(D * d.ld_orb);
    w.dborb = take(d.ld_orb);
  }
  if (nref) {
    w.fgrad = take(nref);
    w.ctf = take((size_t)nw * 2);
    if (d.sparse) {
      w.kfs0 = take(rp * 8 * d.N * d.K);
      w.kfs1 = take(rp * 8 * d.N * d.K);
    }
  }
  w.total_bytes = off * sizeof(float);
  return w;
}

// KFAC statistics accumulated by a Fisher-mode backward pass (vjp_backward with kf != null):
// factor Gram matrices into `stats` (KfacHost slots), normalised by the total row counts.
struct KfacAcc {
  const KfacHost* plan;
  float* stats;
  float inv_rows;         // 1 / (B N)
  float inv_rows_blk[2];  // 1 / (B N_alpha) (orbital blocks)
  int acc;                // accumulate into stats (chunks after the first)
};

// forward with saved activations (the same arithmetic as the log-psi pass)
void vjp_forward(dh_handle* h, const float* x, int nw, float* logpsi, const GradWork& w, hipStream_t s) {
  const Dims& d = h->d;
  const Params& P = h->p;
  const int rows = nw * d.N, D = d.D;
  const bool x6 = d.D % 32 == 0 && gemm_x6_supported(D);
  auto fwd = [&](const float* X, const float* W, const float* Wt, const uint16_t* Wp, int ncols, const float* bias,
                 const float* Rr, float* Y) {
    if (x6)
      launch_gemm_x6(X, D, Wp, x6_plane_rows(ncols), bias, Rr, ncols, Y, ncols, rows, ncols, D, 1, s);
    else if (Wt)
      launch_gemm_nt(X, D, Wt, D, bias, Rr, ncols, Y, ncols, rows, ncols, D, 1, s);
    else
      launch_gemm(X, D, W, ncols, bias, Rr, ncols, Y, ncols, rows, ncols, D, 1, s);
  };
  launch_input(d, x, P.W0, nullptr, nullptr, w.hs[0], nullptr, w.geo, nw, 1, s);
  for (int l = 0; l < d.L; ++l) {
    const LayerParams& lp = P.layer[l];
    fwd(w.hs[l], lp.Wqkv, lp.WqkvT, lp.WqkvP, 3 * D, lp.bqkv, nullptr, w.qkv[l]);
    launch_attention(d, w.qkv[l], w.geo, w.o[l], nw, 1, s);
    fwd(w.o[l], lp.Wol, lp.WolT, lp.WolP, D, lp.bol, w.hs[l], w.t[l]);
    launch_ln_fwd(w.t[l], nullptr, lp.ln1, w.h1[l], rows, D, s);
    fwd(w.h1[l], lp.Wm, lp.WmT, lp.WmP, D, lp.bm, nullptr, w.z[l]);
    launch_ln_fwd(w.h1[l], w.z[l], lp.ln2, w.hs[l + 1], rows, D, s);
  }
  {
    const float* hL = w.hs[d.L];
    if (x6)
      launch_gemm_x6(hL, D, P.WorbP, x6_plane_rows(d.orb_cols), P.borb, nullptr, 0, w.F, d.ld_orb, rows, d.orb_cols,
                     D, 1, s);
    else if (P.WorbT)
      launch_gemm_nt(hL, D, P.WorbT, D, P.borb, nullptr, 0, w.F, d.ld_orb, rows, d.orb_cols, D, 1, s);
    else
      launch_gemm(hL, D, P.Worb, d.ld_orb, P.borb, nullptr, 0, w.F, d.ld_orb, rows, d.orb_cols, D, 1, s);
  }
  launch_det_value(d, w.F, x, P.jastrow, h->norm, logpsi ? logpsi : w.logpsi, nw, s);
}

// Reverse pass over the saved activations of vjp_forward: the parameter gradient for the
// per-walker cotangents ct, written (acc = 0) or accumulated (acc = 1) into `grad`
// (dh_ref_layout).  Fisher mode (kf != null): the dense weight gradients are skipped (only
// the LayerNorm and Jastrow entries of `grad` are written — KFAC's generic tangents) and
// every dense layer's input / output-tangent Gram matrices go into kf->stats.
int vjp_backward(dh_handle* h, const float* x, int nw, const float* ct, float* grad, int acc, const GradWork& w,
                 hipStream_t s, const KfacAcc* kf = nullptr) {
  const Dims& d = h->d;
  const Params& P = h->p;
  const int rows = nw * d.N, D = d.D, nch = grad_chunks(rows);
  const bool x6 = d.D % 32 == 0 && gemm_x6_supported(D);
  const RefSeg RS{d.L, d.NB, d.sparse};
  const bool fisher = kf != nullptr;
  auto g = [&](int seg) { return grad + h->ref_offsets[seg]; };
  auto ref = [&](int seg) { return (const float*)h->ref + h->ref_offsets[seg]; };
  // backward GEMM dX = dY W^T (+ R) with W [D][n]
  auto bwd = [&](const float* dY, int n, const uint16_t* WB, const float* WBT, const float* Rr, float* dX) {
    if (x6)
      launch_gemm_x6(dY, n, WB, x6_plane_rows(D), nullptr, Rr, D, dX, D, rows, D, n, 1, s);
    else
      launch_gemm(dY, n, WBT, D, nullptr, Rr, D, dX, D, rows, D, n, 1, s);
  };
  // weight gradient: out[:, c0:c0+nc] (ldo) (+)= X^T dY[:, c0:c0+nc] over this chunk's rows
  auto wgrad = [&](const float* X, const float* dY, int n) { launch_tn_partial(X, D, dY, n, rows, D, n, w.P, s); };
  auto wout = [&](int n, int c0, int nc, float* out, int ldo) {
    launch_reduce2d(w.P + c0, nch, (size_t)D * n, n, D, nc, out, ldo, 1.f, acc, s);
  };
  auto bgrad = [&](const float* dY, int n, int c0, int nc, float* out) {
    launch_colsum_partial(dY, n, rows, n, w.P, s);
    launch_reduce2d(w.P + c0, nch, (size_t)n, n, 1, nc, out, nc, 1.f, acc, s);
  };
  // KFAC Gram matrices: slot (+)= scale X^T X (n columns of X, row stride ldx, `nr` rows),
  // with the bias row / column / corner of [X, 1] when aug
  // (accum: add to the slot instead of overwriting it; default kf->acc, the chunk loop's flag)
  auto gram = [&](const float* X, int ldx, int n, int slot, float scale, int nr, bool aug, int accum = -1) {
    const KfacSlot& sl = kf->plan->slots[slot];
    float* out = kf->stats + sl.off;
    const int nc2 = grad_chunks(nr);
    const int a = accum < 0 ? kf->acc : accum;
    launch_tn_partial(X, ldx, X, ldx, nr, n, n, w.P, s);
    launch_reduce2d(w.P, nc2, (size_t)n * n, n, n, n, out, sl.n, scale, a, s);
    if (aug) {
      launch_colsum_partial(X, ldx, nr, n, w.P, s);
      launch_kfac_aug(w.P, nc2, n, out, sl.n, scale, (float)nr * scale, a, s);
    }
  };
  // ---- backward
  launch_det_bwd(d, w.F, x, P.jastrow, h->norm, ct, w.dF, w.jg, nw, s);
  launch_reduce2d(w.jg, nw, 2, 2, 1, 1, g(RS.jas(0)), 1, 1.f, acc, s);
  launch_reduce2d(w.jg + 1, nw, 2, 2, 1, 1, g(RS.jas(1)), 1, 1.f, acc, s);
  {
    const int MNK = d.M * d.N * d.K;
    if (fisher) {
      const KfacHost& K = *kf->plan;
      const int NK = d.N * d.K, F8 = 8 * NK;
      const float inv_lll = kf->inv_rows / (float)NK;  // rows of the lll block: B N N K
      int lo = 0;
      for (int a = 0, blk = 0; a < 2; ++a) {
        const int na = a == 0 ? d.n_up : d.n_dn;
        if (na == 0) continue;
        const int nr = d.NB == 1 ? rows : nw * na;
        if (!d.sparse)
          for (int part = 0; part < 2; ++part)
            gram(w.dF + (size_t)(blk * 2 + part) * MNK, d.ld_orb, MNK, K.G_orb[blk][part], kf->inv_rows_blk[blk],
                 rows, false);
        const float* hb = w.hs[d.L];
        if (d.NB > 1) {  // this spin block's rows of every walker, gathered
          launch_copy2d(w.hs[d.L] + (size_t)lo * D, d.N * D, w.dqkv, na * D, nw, na * D, s);
          hb = w.dqkv;
        }
        gram(hb, D, D, K.A_orb[blk], kf->inv_rows_blk[blk], nr, true);
        if (d.sparse) {
          const int nlo = d.NB == 1 ? 0 : lo, nna = d.NB == 1 ? d.N : na;
          // featured-orbital tangents (lll dF) -> the DenseGeneral G factors
          for (int part = 0; part < 2; ++part) {
            launch_kfac_sparse_dphi(w.dF, d.ld_orb, ref(RS.lll(0)), d.M, NK, blk * 2 + part, nr, nna, d.N, nlo,
                                    w.kfs0, s);
            gram(w.kfs0, F8, F8, K.G_orb[blk][part], kf->inv_rows_blk[blk], nr, false);
          }
          // the lll_weight input (the real featured orbitals h W + b, exact f32) in rows of 8,
          // its output tangent (the real feature segment) in rows of M; spin blocks accumulate
          const int acc_lll = (kf->acc || blk > 0) ? 1 : 0;
          launch_gemm(hb, D, ref(RS.orb_kernel(2 * blk)), F8, ref(RS.orb_bias(2 * blk)), nullptr, 0, w.kfs1, F8, nr,
                      F8, D, 1, s);
          gram(w.kfs1, 8, 8, K.A_lll, inv_lll, nr * NK, false, acc_lll);
          // scratch for the regrouped tangent: w.F, the saved orbital matrix of this chunk's
          // forward — dead here, because this (Fisher) reverse pass is its last reader: the
          // gradient pass ran first and this pass's launch_det_bwd above has consumed it; the
          // next chunk's forward rewrites it.  dh_kfac_vjp must keep that order.
          launch_kfac_sparse_regroup(w.dF, d.ld_orb, d.M, NK, blk * 2, nr, nna, d.N, nlo, w.F, s);
          gram(w.F, d.M, d.M, K.G_lll, inv_lll, nr * NK, false, acc_lll);
          // the generic lll bias tangent: sum over rows of the real feature segment
          launch_colsum_partial(w.F, d.M, nr * NK, d.M, w.P, s);
          launch_reduce2d(w.P, grad_chunks(nr * NK), (size_t)d.M, d.M, 1, d.M, g(RS.lll(1)), d.M, 1.f, acc || blk > 0,
                          s);
        }
        lo += na;
        ++blk;
      }
    } else {
      wgrad(w.hs[d.L], w.dF, d.ld_orb);
      if (!d.sparse) {
        for (int i = 0; i < 2 * d.NB; ++i) wout(d.ld_orb, i * MNK, MNK, g(RS.orb_kernel(i)), MNK);
        launch_colsum_partial(w.dF, d.ld_orb, rows, d.ld_orb, w.P, s);
        for (int i = 0; i < 2 * d.NB; ++i)
          launch_reduce2d(w.P + i * MNK, nch, (size_t)d.ld_orb, d.ld_orb, 1, MNK, g(RS.orb_bias(i)), MNK, 1.f, acc,
                          s);
      } else {
        // full-layout gradients of this chunk, then through the lll_weight fold
        launch_reduce2d(w.P, nch, (size_t)D * d.ld_orb, d.ld_orb, D, d.orb_cols, w.dWorb, d.ld_orb, 1.f, 0, s);
        launch_colsum_partial(w.dF, d.ld_orb, rows, d.ld_orb, w.P, s);
        launch_reduce2d(w.P, nch, (size_t)d.ld_orb, d.ld_orb, 1, d.orb_cols, w.dborb, d.ld_orb, 1.f, 0, s);
        SparseBlocks sb{};
        sb.n = 2 * d.NB;
        for (int i = 0; i < sb.n; ++i) {
          sb.W8[i] = ref(RS.orb_kernel(i));
          sb.b8[i] = ref(RS.orb_bias(i));
          launch_sparse_unfold(w.dWorb + i * MNK, d.ld_orb, w.dborb + i * MNK, ref(RS.lll(0)), D, d.N * d.K, d.M,
                               g(RS.orb_kernel(i)), g(RS.orb_bias(i)), acc, s);
        }
        launch_sparse_lll_grad(sb, w.dWorb, d.ld_orb, w.dborb, D, d.N * d.K, d.M, g(RS.lll(0)), g(RS.lll(1)), acc,
                               s);
      }
    }
    bwd(w.dF, d.ld_orb, P.WorbB, P.WorbBT, nullptr, w.dh);
  }
  for (int l = d.L - 1; l >= 0; --l) {
    const LayerParams& lp = P.layer[l];
    const int nb = ln_bwd_blocks(rows);
    // h_{l+1} = LN2(h1 + tanh z): dU -> dA (the residual path into h1), dz
    launch_ln_bwd(w.h1[l], w.z[l], lp.ln2, w.dh, nullptr, w.dA, w.dz, w.P, rows, D, s);
    launch_reduce2d(w.P, nb, (size_t)2 * D, D, 1, D, g(RS.lay(l, Rln2s)), D, 1.f, acc, s);
    launch_reduce2d(w.P + D, nb, (size_t)2 * D, D, 1, D, g(RS.lay(l, Rln2b)), D, 1.f, acc, s);
    // z = h1 Wm + bm
    if (fisher) {
      gram(w.dz, D, D, kf->plan->lay[l].G_z, kf->inv_rows, rows, false);
      gram(w.h1[l], D, D, kf->plan->lay[l].A_h1, kf->inv_rows, rows, true);
    } else {
      wgrad(w.h1[l], w.dz, D);
      wout(D, 0, D, g(RS.lay(l, RWm)), D);
      bgrad(w.dz, D, 0, D, g(RS.lay(l, Rbm)));
    }
    bwd(w.dz, D, lp.WmB, lp.WmBT, w.dA, w.dh);  // dh1 = dU + dz Wm^T
    // h1 = LN1(t): dT -> dA
    launch_ln_bwd(w.t[l], nullptr, lp.ln1, w.dh, nullptr, w.dA, nullptr, w.P, rows, D, s);
    launch_reduce2d(w.P, nb, (size_t)2 * D, D, 1, D, g(RS.lay(l, Rln1s)), D, 1.f, acc, s);
    launch_reduce2d(w.P + D, nb, (size_t)2 * D, D, 1, D, g(RS.lay(l, Rln1b)), D, 1.f, acc, s);
    // t = h + o Wol + bol: folded-weight gradients, then unfolded onto Wo, bo, Wl
    if (fisher) {
      // Dense_{2l+1}'s output tangent is dT; the attention output's input is o
      gram(w.dA, D, D, kf->plan->lay[l].G_T, kf->inv_rows, rows, false);
      gram(w.o[l], D, D, kf->plan->lay[l].A_o, kf->inv_rows, rows, true);
    } else {
      wgrad(w.o[l], w.dA, D);
      launch_reduce2d(w.P, nch, (size_t)D * D, D, D, D, w.dWol, D, 1.f, 0, s);
      launch_colsum_partial(w.dA, D, rows, D, w.P, s);
      launch_reduce2d(w.P, nch, (size_t)D, D, 1, D, w.dbol, D, 1.f, 0, s);
      //   Wol = Wo Wl, bol = bo Wl:  dWo = dWol Wl^T, dbo = dbol Wl^T, dWl = Wo^T dWol + bo^T dbol
      launch_small_gemm(D, D, D, w.dWol, D, 0, ref(RS.lay(l, RWl)), D, 1, g(RS.lay(l, RWo)), D, acc, s);
      launch_small_gemm(1, D, D, w.dbol, D, 0, ref(RS.lay(l, RWl)), D, 1, g(RS.lay(l, Rbo)), D, acc, s);
      launch_small_gemm(D, D, D, ref(RS.lay(l, RWo)), D, 1, w.dWol, D, 0, g(RS.lay(l, RWl)), D, acc, s);
      launch_small_gemm(D, D, 1, ref(RS.lay(l, Rbo)), 1, 0, w.dbol, D, 0, g(RS.lay(l, RWl)), D, 1, s);
    }
    bwd(w.dA, D, lp.WolB, lp.WolBT, nullptr, w.dO);  // dO = dT Wol^T
    launch_attn_bwd(d, w.qkv[l], w.dO, w.dqkv, nw, s);
    // qkv = h Wqkv + bqkv
    if (fisher) {
      const KfacLayerSlots& ls = kf->plan->lay[l];
      const int gs[3] = {ls.G_q, ls.G_k, ls.G_v};
      for (int part = 0; part < 3; ++part) gram(w.dqkv + part * D, 3 * D, D, gs[part], kf->inv_rows, rows, false);
      gram(w.hs[l], D, D, ls.A_h, kf->inv_rows, rows, true);
    } else {
      wgrad(w.hs[l], w.dqkv, 3 * D);
      for (int part = 0; part < 3; ++part) wout(3 * D, part * D, D, g(RS.lay(l, RWq + 2 * part)), D);
      launch_colsum_partial(w.dqkv, 3 * D, rows, 3 * D, w.P, s);
      for (int part = 0; part < 3; ++part)
        launch_reduce2d(w.P + part * D, nch, (size_t)3 * D, 3 * D, 1, D, g(RS.lay(l, Rbq + 2 * part)), D, 1.f, acc,
                        s);
    }
    bwd(w.dqkv, 3 * D, lp.WqkvB, lp.WqkvBT, w.dA, w.dh);  // dh_l = dT + dqkv Wqkv^T
  }
  // h_0 = features W0
  if (fisher) {
    gram(w.dh, D, D, kf->plan->s_h0, kf->inv_rows, rows, false);
    const KfacSlot& sl = kf->plan->slots[kf->plan->s_feat];
    launch_kfac_feat_gram(d, w.geo, rows, w.P, s);
    launch_reduce2d(w.P, nch, 16, 4, 4, 4, kf->stats + sl.off, 4, kf->inv_rows, kf->acc, s);
  } else {
    launch_w0_partial(d, w.geo, w.dh, D, rows, w.P, s);
    launch_reduce2d(w.P, nch, (size_t)4 * D, D, 4, D, g(RS.W0()), D, 1.f, acc, s);
  }
  return check_launch();
}

// One chunk of the VJP: forward with saved activations, then the chain rule back to every
// reference parameter; gradient written (acc = 0) or accumulated (acc = 1) into `grad`
// (dh_ref_layout).  ct: per-walker cotangents [nw][2].
int run_vjp(dh_handle* h, const float* x, int nw, const float* ct, float* grad, float* logpsi, int acc,
            const GradWork& w, hipStream_t s) {
  vjp_forward(h, x, nw, logpsi, w, s);
  return vjp_backward(h, x, nw, ct, grad, acc, w, s);
}


// ---- KFAC (optimizers/kfac.py:195-241; oracle/kfac.py)

// Build the factor slots, dense blocks, generic segments and device job tables.
int kfac_plan(dh_handle* h) {
  if (h->kfac) return DH_OK;
  const Dims& d = h->d;
  if (d.L > 16) return fail(DH_EINVAL, "KFAC: too many layers");
  auto* K = new KfacHost();
  const int D = d.D, N = d.N, MNK = d.M * d.N * d.K;
  auto slot = [&](int n) {
    K->slots.push_back(KfacSlot{n, K->nmat});
    K->nmat += align64((size_t)n * n);
    return (int)K->slots.size() - 1;
  };
  const RefSeg RS{d.L, d.NB, d.sparse};
  auto blk = [&](int kseg, int bseg, int din, int dout, int a, int g, float scale) {
    K->blocks.push_back(KfacHost::Blk{kseg, bseg, din, dout, a, g, scale});
  };
  K->s_feat = slot(4);
  K->s_h0 = slot(D);
  blk(RS.W0(), -1, 4, D, K->s_feat, K->s_h0, (float)N);
  for (int l = 0; l < d.L; ++l) {
    KfacLayerSlots& L = K->lay[l];
    L.A_h = slot(D + 1);
    L.G_q = slot(D);
    L.G_k = slot(D);
    L.G_v = slot(D);
    L.A_o = slot(D + 1);
    L.G_out = slot(D);
    L.A_Wl = slot(D);
    L.G_T = slot(D);
    L.A_h1 = slot(D + 1);
    L.G_z = slot(D);
    blk(RS.lay(l, RWq), RS.lay(l, Rbq), D, D, L.A_h, L.G_q, (float)N);
    blk(RS.lay(l, RWk), RS.lay(l, Rbk), D, D, L.A_h, L.G_k, (float)N);
    blk(RS.lay(l, RWv), RS.lay(l, Rbv), D, D, L.A_h, L.G_v, (float)N);
    blk(RS.lay(l, RWo), RS.lay(l, Rbo), D, D, L.A_o, L.G_out, (float)(N * d.H));  // x [B, N, H, dh]
    blk(RS.lay(l, RWl), -1, D, D, L.A_Wl, L.G_T, (float)N);
    blk(RS.lay(l, RWm), RS.lay(l, Rbm), D, D, L.A_h1, L.G_z, (float)N);
  }
  // featured orbitals: M N K outputs, or 8 N K for "sparse" (then mixed by lll_weight)
  const int FNK = d.sparse ? 8 * N * d.K : MNK;
  for (int a = 0, b = 0; a < 2; ++a) {
    const int na = a == 0 ? d.n_up : d.n_dn;
    if (na == 0) continue;
    K->A_orb[b] = slot(D + 1);
    for (int part = 0; part < 2; ++part) {
      K->G_orb[b][part] = slot(FNK);
      blk(RS.orb_kernel(2 * b + part), RS.orb_bias(2 * b + part), D, FNK, K->A_orb[b], K->G_orb[b][part], (float)na);
    }
    ++b;
  }
  if (d.sparse) {
    // lll_weight: kfac.py's repeated_dense_complex_no_bias block, its statistics as
    // RepeatedDenseBlock computes them (inputs regrouped into rows of 8, scale 8 N^2)
    K->A_lll = slot(8);
    K->G_lll = slot(d.M);
    blk(RS.lll(0), -1, 8, d.M, K->A_lll, K->G_lll, (float)(8 * N * N));
  }
  // generic (diagonal) parameters: LayerNorm scale / bias, Jastrow alphas
  KfacGenTable& G = K->dev.gen;
  G = KfacGenTable{};
  auto gen = [&](int seg, int n) {
    G.ref[G.n] = h->ref_offsets[seg];
    G.cmp[G.n] = G.total;
    G.total += n;
    ++G.n;
  };
  for (int l = 0; l < d.L; ++l)
    for (int k : {Rln1s, Rln1b, Rln2s, Rln2b}) gen(RS.lay(l, k), D);
  if (d.sparse) gen(RS.lll(1), d.M);  // lll_weight's bias: no pattern covers it
  gen(RS.jas(0), 1);
  gen(RS.jas(1), 1);
  K->nstats = K->nmat + (size_t)G.total;
  // inverse jobs (2 per block: A side, G side), then V / T / P V per block, all in one f64 buffer
  size_t off = 0;
  int nmax = 0, max_v = 0, max_m = 0, max_n = 0;
  for (const auto& b : K->blocks) {
    for (int side = 0; side < 2; ++side) {
      KfacInvJob j{};
      j.slot = side == 0 ? b.a : b.g;
      j.partner = side == 0 ? b.g : b.a;
      j.is_a = side == 0;
      j.n = K->slots[j.slot].n;
      j.sqrt_scale = std::sqrt(b.scale);
      j.gj_off = off;
      off += (size_t)j.n * j.n;
      nmax = std::max(nmax, j.n);
      K->inv.push_back(j);
    }
  }
  for (size_t i = 0; i < K->blocks.size(); ++i) {
    const auto& b = K->blocks[i];
    const int dA = b.din + (b.bseg >= 0 ? 1 : 0);
    KfacBlockJob j{};
    j.kernel_off = h->ref_offsets[b.kseg];
    j.bias_off = b.bseg >= 0 ? (long long)h->ref_offsets[b.bseg] : -1;
    j.din = b.din;
    j.dout = b.dout;
    const size_t nv = (size_t)dA * b.dout;
    j.v_off = off;
    j.t_off = off + nv;
    j.pv_off = off + 2 * nv;
    off += 3 * nv;
    K->bjobs.push_back(j);
    K->g1.push_back(KfacGemmJob{K->inv[2 * i].gj_off, j.v_off, j.t_off, dA, b.dout, dA});
    K->g2.push_back(KfacGemmJob{j.t_off, K->inv[2 * i + 1].gj_off, j.pv_off, dA, b.dout, b.dout});
    max_v = std::max(max_v, (int)nv);
    max_m = std::max(max_m, dA);
    max_n = std::max(max_n, b.dout);
  }
  K->kbuf_doubles = off;
  K->dev.nslots = (int)K->slots.size();
  K->dev.njobs = (int)K->inv.size();
  K->dev.nblocks = (int)K->blocks.size();
  K->dev.nmax = nmax;
  K->dev.max_v = max_v;
  K->dev.max_m = max_m;
  K->dev.max_n = max_n;
  h->kfac = K;
  return DH_OK;
}

// Upload the job tables (once, at the first device call).
int kfac_device(dh_handle* h) {
  if (int rc = kfac_plan(h)) return rc;
  KfacHost* K = h->kfac;
  if (K->dev_mem) return DH_OK;
  // device tables
  const size_t b1 = K->slots.size() * sizeof(KfacSlot), b2 = K->inv.size() * sizeof(KfacInvJob),
               b3 = K->bjobs.size() * sizeof(KfacBlockJob), b4 = K->g1.size() * sizeof(KfacGemmJob);
  auto al = [](size_t n) { return (n + 255) / 256 * 256; };
  char* mem = nullptr;
  if (hipMalloc(&mem, al(b1) + al(b2) + al(b3) + 2 * al(b4)) != hipSuccess) {
    return fail(DH_EHIP, "KFAC: device table allocation failed");
  }
  K->dev_mem = mem;
  K->dev.slots = reinterpret_cast<KfacSlot*>(mem);
  K->dev.inv_jobs = reinterpret_cast<KfacInvJob*>(mem + al(b1));
  K->dev.block_jobs = reinterpret_cast<KfacBlockJob*>(mem + al(b1) + al(b2));
  K->dev.gemm1 = reinterpret_cast<KfacGemmJob*>(mem + al(b1) + al(b2) + al(b3));
  K->dev.gemm2 = reinterpret_cast<KfacGemmJob*>(mem + al(b1) + al(b2) + al(b3) + al(b4));
  bool ok = hipMemcpy(K->dev.slots, K->slots.data(), b1, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(K->dev.inv_jobs, K->inv.data(), b2, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(K->dev.block_jobs, K->bjobs.data(), b3, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(K->dev.gemm1, K->g1.data(), b4, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(K->dev.gemm2, K->g2.data(), b4, hipMemcpyHostToDevice) == hipSuccess;
  if (!ok) {
    (void)hipFree(mem);
    K->dev_mem = nullptr;
    return fail(DH_EHIP, "KFAC: device table upload failed");
  }
  return DH_OK;
}

size_t kfac_step_ws(const KfacHost* K) {
  // kbuf (inverses, V, T, P V) | traces | GJ panel temporaries, doubles
  const size_t nd = align64(K->kbuf_doubles) + align64(K->slots.size()) +
                    align64(kfac_gj_tmp_doubles(K->dev.njobs, K->dev.nmax));
  return nd * sizeof(double);
}

}  // namespace

extern "C" {

size_t dh_vjp_workspace_bytes(const dh_handle* h, int batch) {
  if (!h || batch < 1) return 0;
  return carve_grad(h->d, batch, nullptr).total_bytes;
}

int dh_logpsi_vjp(dh_handle* h, const float* x, int B, const float* ct, float* grad, float* logpsi, void* ws,
                  size_t ws_bytes, void* stream) {
  const size_t need1 = h ? dh_vjp_workspace_bytes(h, 1) : 0;
  if (int rc = check_common(h, x, B, ws, ws_bytes, need1)) return rc;
  if (h && h->laughlin) return fail(DH_EINVAL, "the Laughlin wavefunction has no parameters to differentiate");
  if (!h->ref_set) return fail(DH_ESTATE, "the VJP needs parameters uploaded with dh_set_params_ref");
  if (!ct || !grad) return fail(DH_EINVAL, "null argument");
  if (h->d.D > 1024 || h->d.dh > 1024) return fail(DH_EINVAL, "VJP supports D <= 1024");
  int chunk = B;
  while (chunk > 1 && dh_vjp_workspace_bytes(h, chunk) > ws_bytes) chunk = (chunk + 1) / 2;
  hipStream_t s = (hipStream_t)stream;
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nw = std::min(chunk, B - b0);
    GradWork w = carve_grad(h->d, nw, ws);
    if (int rc = run_vjp(h, x + (size_t)b0 * h->d.N * 2, nw, ct + 2 * (size_t)b0, grad,
                         logpsi ? logpsi + 2 * (size_t)b0 : nullptr, b0 > 0, w, s))
      return rc;
  }
  return DH_OK;
}

int dh_kfac_layout(dh_handle* h, size_t* out, int n) {
  if (!h || h->laughlin) return fail(DH_EINVAL, "KFAC needs a Psiformer handle");
  if (int rc = kfac_plan(h)) return rc;
  const KfacHost& K = *h->kfac;
  // [0] statistics floats, [1] factor-matrix floats, [2] slots, [3] dense blocks, [4] generic
  // floats, [5] dh_kfac_step workspace bytes, then per block (kernel seg, bias seg or -1 as
  // SIZE_MAX, din, dout, A slot, G slot, scale x 1000), then per slot (n, offset)
  std::vector<size_t> v = {K.nstats, K.nmat, K.slots.size(), K.blocks.size(), (size_t)K.dev.gen.total,
                           kfac_step_ws(&K)};
  for (const auto& b : K.blocks)
    v.insert(v.end(), {(size_t)b.kseg, b.bseg >= 0 ? (size_t)b.bseg : SIZE_MAX, (size_t)b.din, (size_t)b.dout,
                       (size_t)b.a, (size_t)b.g, (size_t)std::lround(b.scale * 1000.f)});
  for (const auto& sl : K.slots) v.insert(v.end(), {(size_t)sl.n, sl.off});
  if (out)
    for (int i = 0; i < n && i < (int)v.size(); ++i) out[i] = v[i];
  return (int)v.size();
}

size_t dh_kfac_workspace_bytes(const dh_handle* h, int batch) {
  if (!h || batch < 1) return 0;
  return carve_grad(h->d, batch, nullptr, h->ref_offsets.back()).total_bytes;
}

int dh_kfac_vjp(dh_handle* h, const float* x, int B, const float* ct, float* grad, float* stats, float* logpsi,
                void* ws, size_t ws_bytes, void* stream) {
  if (!h || h->laughlin) return fail(DH_EINVAL, "KFAC needs a Psiformer handle");
  const size_t nref = h->ref_offsets.back();
  const size_t need1 = dh_kfac_workspace_bytes(h, 1);
  if (int rc = check_common(h, x, B, ws, ws_bytes, need1)) return rc;
  if (!h->ref_set) return fail(DH_ESTATE, "KFAC needs parameters uploaded with dh_set_params_ref");
  if (!stats) return fail(DH_EINVAL, "null statistics buffer");
  if (ct && !grad) return fail(DH_EINVAL, "ct given without grad");
  if (h->d.D > 1024 || h->d.dh > 1024) return fail(DH_EINVAL, "KFAC supports D <= 1024");
  if (int rc = kfac_device(h)) return rc;
  const KfacHost& K = *h->kfac;
  const Dims& d = h->d;
  int chunk = B;
  while (chunk > 1 && carve_grad(d, chunk, nullptr, nref).total_bytes > ws_bytes) chunk = (chunk + 1) / 2;
  hipStream_t s = (hipStream_t)stream;
  KfacAcc kf{};
  kf.plan = &K;
  kf.stats = stats;
  kf.inv_rows = 1.f / ((float)B * d.N);
  for (int a = 0, b = 0; a < 2; ++a) {
    const int na = a == 0 ? d.n_up : d.n_dn;
    if (na) kf.inv_rows_blk[b++] = 1.f / ((float)B * na);
  }
  const GradWork w = carve_grad(d, chunk, ws, nref);  // one layout: fgrad accumulates over chunks
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nw = std::min(chunk, B - b0);
    const float* xc = x + (size_t)b0 * d.N * 2;
    float* lp = logpsi ? logpsi + 2 * (size_t)b0 : w.logpsi;
    vjp_forward(h, xc, nw, lp, w, s);
    if (ct)
      if (int rc = vjp_backward(h, xc, nw, ct + 2 * (size_t)b0, grad, b0 > 0, w, s)) return rc;
    launch_kfac_fisher_ct(lp, nw, w.ctf, s);
    kf.acc = b0 > 0;
    if (int rc = vjp_backward(h, xc, nw, w.ctf, w.fgrad, b0 > 0, w, s, &kf)) return rc;
  }
  // derived factors of the folded attention output (the kernels run Wol = Wo Wl as one map):
  // Dense_{2l+1}'s input a = [o, 1] [Wo; bo]:  A_Wl = [Wo; bo]^T A_o [Wo; bo]
  // the attention output's tangent dT Wl^T:    G_out = Wl G_T Wl^T
  const RefSeg RS{d.L, d.NB, d.sparse};
  const int D = d.D;
  auto ref = [&](int seg) { return (const float*)h->ref + h->ref_offsets[seg]; };
  float* Wt = w.P;                        // [D + 1][D]
  float* T = w.P + (size_t)(D + 1) * D;   // [D + 1][D]
  for (int l = 0; l < d.L; ++l) {
    const KfacLayerSlots& L = K.lay[l];
    launch_copy2d(ref(RS.lay(l, RWo)), D, Wt, D, D, D, s);
    launch_copy2d(ref(RS.lay(l, Rbo)), D, Wt + (size_t)D * D, D, 1, D, s);
    launch_small_gemm(D + 1, D, D + 1, stats + K.slots[L.A_o].off, D + 1, 0, Wt, D, 0, T, D, 0, s);
    launch_small_gemm(D, D, D + 1, Wt, D, 1, T, D, 0, stats + K.slots[L.A_Wl].off, D, 0, s);
    launch_small_gemm(D, D, D, ref(RS.lay(l, RWl)), D, 0, stats + K.slots[L.G_T].off, D, 0, T, D, 0, s);
    launch_small_gemm(D, D, D, T, D, 0, ref(RS.lay(l, RWl)), D, 1, stats + K.slots[L.G_out].off, D, 0, s);
  }
  launch_kfac_generic(w.fgrad, K.dev.gen, stats + K.nmat, 1.f / (float)B, s);
  return check_launch();
}

int dh_kfac_step(dh_handle* h, float* raw, const float* stats, float ema, float weight, const float* grad,
                 float* params, float lr, float damping, float norm_constraint, float* pgrad, double* info, void* ws,
                 size_t ws_bytes, void* stream) {
  if (!h || h->laughlin) return fail(DH_EINVAL, "KFAC needs a Psiformer handle");
  if (!raw || !grad || !pgrad || !info || !ws) return fail(DH_EINVAL, "null argument");
  if (!(weight > 0.f) || !(damping > 0.f)) return fail(DH_EINVAL, "KFAC needs weight > 0 and damping > 0");
  if (int rc = kfac_device(h)) return rc;
  const KfacHost& K = *h->kfac;
  const size_t nref = h->ref_offsets.back();
  if (ws_bytes < kfac_step_ws(&K)) return fail(DH_ENOMEM, "KFAC step workspace too small");
  hipStream_t s = (hipStream_t)stream;
  double* kbuf = reinterpret_cast<double*>(ws);
  double* tr = kbuf + align64(K.kbuf_doubles);
  double* tmp = tr + align64(K.slots.size());
  if (stats) launch_kfac_ema(raw, stats, K.nstats, ema, s);
  launch_kfac_invert(K.dev, raw, 1.0 / weight, std::sqrt((double)damping), tr, kbuf, tmp, s);
  launch_kfac_precondition(K.dev, grad, raw + K.nmat, 1.0 / weight, damping, kbuf, pgrad, nref, info, s);
  if (params) launch_kfac_update(params, pgrad, nref, info, lr, norm_constraint, s);
  return check_launch();
}

int dh_grad_cotangent(const float* diff, const float* nvalid, int B, int part, float* ct, void* stream) {
  if (!diff || !nvalid || !ct || B < 1 || (part != 0 && part != 1)) return fail(DH_EINVAL, "bad arguments");
  launch_cotangent(diff, nvalid, B, part, ct, (hipStream_t)stream);
  return check_launch();
}

int dh_adam_update(float* params, const float* grad, float* mu, float* nu, size_t n, float lr, float b1, float b2,
                   float eps, int step, void* stream) {
  if (!params || !grad || !mu || !nu || n == 0 || step < 0) return fail(DH_EINVAL, "bad arguments");
  launch_adam(params, grad, mu, nu, n, lr, b1, b2, eps, step, (hipStream_t)stream);
  return check_launch();
}

int dh_energy_stats(dh_handle* h, const float* e_l, const float* obs, const int32_t* n_accept, int B, int steps,
                    int penalties, float* out, void* stream) {
  (void)h;  // statistics of any wavefunction's E_L (NULL: a log-psi callable of the caller)
  if (!e_l || !obs || !out) return fail(DH_EINVAL, "null argument");
  if (B < 1) return fail(DH_EINVAL, "dh_energy_stats needs B >= 1");
  launch_stats(e_l, obs, n_accept, B, steps, penalties, out, (hipStream_t)stream);
  return check_launch();
}

int dh_loss_diff(dh_handle* h, const float* e_l, const float* obs, int B, const float* stats, float lz_penalty,
                 float lz_center, float l2_penalty, float* diff, float* nvalid, void* stream) {
  (void)h;  // as dh_energy_stats: h may be NULL
  if (!e_l || !obs || !stats || !diff || !nvalid) return fail(DH_EINVAL, "null argument");
  if (B < 1) return fail(DH_EINVAL, "dh_loss_diff needs B >= 1");
  launch_loss_diff(e_l, obs, B, stats, lz_penalty, lz_center, l2_penalty, diff, nvalid, (hipStream_t)stream);
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
  // keep_h: the chain form writes the last layer's h too (the production path skips it)
  return run_trunk(h, x, B, op == 1 ? h->d.C : 1, w, (hipStream_t)stream, false, /*keep_h=*/true);
}

int dh_debug_env_leaf(const float* thph, int n, int M, int sq, float* out, void* stream) {
  if (!thph || !out || n < 1 || M < 1) return fail(DH_EINVAL, "bad env_leaf probe args");
  launch_env_leaf_probe(thph, n, M, sq, out, (hipStream_t)stream);
  return check_launch();
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

int dh_debug_chain_x6(const float* X1, const uint16_t* Wp1, int ldp1, const float* b1, const float* ln1,
                      const uint16_t* Wp2, int ldp2, const float* b2, const float* ln2, const uint16_t* Wp3,
                      int ldp3, const float* b3, int n3, float* Y3, int ldy3, float* h, int rows, void* stream) {
  if (!X1 || !Wp1 || !Wp2 || !b1 || !ln1 || !b2 || !ln2 || !h || rows < 1 || ldp1 < x6_plane_rows(256) ||
      ldp2 < x6_plane_rows(256) || (Wp3 && (!b3 || !Y3 || n3 < 1 || ldy3 < n3 || ldy3 % 4 || ldp3 < x6_plane_rows(n3))))
    return fail(DH_EINVAL, "bad chain_x6 args");
  launch_chain_x6(X1, Wp1, ldp1, b1, ln1, Wp2, ldp2, b2, ln2, Wp3, ldp3, b3, n3, Y3, ldy3, h, rows, X6Feat{},
                  (hipStream_t)stream);
  return check_launch();
}

int dh_debug_gemm_lnch(int N, int mode, const float* X, const uint16_t* Wp, int ldp, const float* bias,
                       const float* ln, const float* geo, float* h, int ne, void* stream) {
  if (!gemm_lnch_supported(N, 256) || (mode != 0 && mode != 1) || (mode == 0 && !X) || !Wp || !ln || !geo || !h ||
      ne < 1 || ldp < x6_plane_rows(256) || ne % N)
    return fail(DH_EINVAL, "bad gemm_lnch args");
  launch_gemm_lnch(N, mode == 0 ? X : h, Wp, ldp, bias, ln, geo, h, ne, mode, (hipStream_t)stream);
  return check_launch();
}

// which fused channel-tail kernel the local energy uses (DH_LNCH at start-up): tests only
int dh_debug_set_lnch_form(int form) { return set_lnch_form(form); }

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

int dh_histograms(const float* x, int B, int nelec, int density_bins, int pair_bins, float* density, float* pair,
                  void* stream) {
  if (!x || B < 1 || nelec < 1 || density_bins < 0 || pair_bins < 0 || density_bins + pair_bins < 1 ||
      density_bins + pair_bins > 8192 || (density_bins && !density) || (pair_bins && !pair))
    return fail(DH_EINVAL, "bad arguments");
  launch_histograms(x, B, nelec, density_bins, pair_bins, density, pair, (hipStream_t)stream);
  return check_launch();
}

int dh_monopole_orbitals(const float* points, int n, int flux, float* out, void* stream) {
  if (!points || !out || n < 1 || flux < 0 || flux > 126) return fail(DH_EINVAL, "bad arguments");
  launch_monopole_orbitals(points, n, flux, out, (hipStream_t)stream);
  return check_launch();
}

// ---- log psi supplied by the caller (arbitrary callables, mcmc.py:105 / hamiltonian.py:83) ----

int dh_mh_init(const float* logpsi, float* lp, int32_t* n_accept, int B, void* stream) {
  if (!logpsi || !lp || !n_accept || B < 1) return fail(DH_EINVAL, "bad arguments");
  launch_lp_from_logpsi(logpsi, lp, n_accept, B, (hipStream_t)stream);
  return check_launch();
}

int dh_mh_propose(const float* x, float* x2, int B, int nelec, float width, uint64_t seed, uint64_t step,
                  int64_t walker_offset, const float* noise, void* stream) {
  if (!x || !x2 || B < 1 || nelec < 1 || x == x2) return fail(DH_EINVAL, "bad arguments");
  Dims d{};
  d.N = nelec;
  launch_propose(d, x, x2, B, width, seed, step, walker_offset, noise, 0, (hipStream_t)stream);
  return check_launch();
}

int dh_mh_accept(float* x, const float* x2, float* lp, const float* logpsi2, int32_t* n_accept, int B, int nelec,
                 uint64_t seed, uint64_t step, int64_t walker_offset, const float* noise, void* stream) {
  if (!x || !x2 || !lp || !logpsi2 || !n_accept || B < 1 || nelec < 1) return fail(DH_EINVAL, "bad arguments");
  Dims d{};
  d.N = nelec;
  launch_accept(d, x, x2, lp, logpsi2, n_accept, B, seed, step, walker_offset, noise, 0, (hipStream_t)stream);
  return check_launch();
}

int dh_kinetic_from_derivatives(const double* x, const double* grad, const double* hess, int B, int nelec, double Q,
                                double r, float* ke, float* mom, void* stream) {
  if (!x || !grad || !hess || !ke || !mom || B < 1 || nelec < 1 || !(r > 0.0) || Q < 0.0)
    return fail(DH_EINVAL, "bad arguments");
  if (kinetic_assembly_lds_bytes(nelec) > 64 * 1024) return fail(DH_EINVAL, "nelec > 256");
  launch_kinetic_assembly(x, grad, hess, B, nelec, Q, r, ke, mom, (hipStream_t)stream);
  return check_launch();
}

int dh_init_walkers(dh_handle* h, float* x, int B, uint64_t seed, int64_t walker_offset, void* stream) {
  if (!h || !x || B < 1) return fail(DH_EINVAL, "bad arguments");
  launch_init_walkers(h->d, x, B, seed, walker_offset, (hipStream_t)stream);
  return check_launch();
}

}  // extern "C"
