// Internal declarations shared by the HIP kernel files and the C ABI (api.cpp).
#pragma once
#include <algorithm>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/deephall_amd.h"

namespace dh {

// Static network geometry derived from dh_config (all sizes in elements).
struct Dims {
  int N, n_up, n_dn;   // electrons
  int T;               // 2N first-order tangent channels
  int C;               // 2N + 5 channels (local energy)
  int M;               // 2Q + 1 monopole harmonics
  float Q, r;          // monopole strength, sphere radius
  int H, dh, D, L, K;  // heads, head dim, model dim, layers, determinants
  int NB;              // spin blocks of the orbital layer (1 or 2)
  int orb_cols;        // NB * 2 * M * N * K
  int ld_orb;          // orb_cols rounded up to 128
  int interaction;     // DH_INTERACTION_*
  float lambda;        // interaction strength
  int sparse;          // orbital type "sparse": F = 8 features per (j, k) (blocks.py:52-62)
};
constexpr int kSparseFeatures = 8;
constexpr int kMqkStride = 32;  // floats per head of layer 1's score forms Mqk (25 used; attn_val.h)

// Device pointers into the packed parameter buffer.
struct LayerParams {
  const float *Wqkv, *bqkv, *Wol, *bol, *ln1, *Wm, *bm, *ln2;
  // backward (x^T-side) copies of the same weights for dX = dY W^T: split-bf16 planes of the
  // untransposed W (x6 path) or W^T [ncols][D] (exact-f32 path)
  const uint16_t *WqkvB, *WolB, *WmB;
  const float *WqkvBT, *WolBT, *WmBT;
  const float *WqkvT, *WolT, *WmT;  // transposed copies [ncols pad 256][D] for the NT GEMM
  const uint16_t *WqkvP, *WolP, *WmP;  // split-bf16 planes [3][x6_plane_rows(ncols)][D] (gemm_x6)
};
struct Params {
  const float* W0;
  LayerParams layer[16];
  const float *Worb, *borb, *jastrow;
  const float* W0qkv;  // [4][3D] = W0 @ Wqkv of layer 0 (folded at packing)
  const float* WorbT;  // [orb_cols pad 256][D]
  const uint16_t* WorbP;  // split-bf16 planes of Worb
  const uint16_t* WorbB;  // backward planes (untransposed Worb [D][ld_orb])
  const float* WorbBT;    // backward exact-f32 copy Worb^T [ld_orb][D]
  const float* Mqk;       // layer 1's score forms Wq~ Wk~^T / 8, [H][kMqkStride] (attn_val.h)
  // layer 1's output map in feature space (round 6): U^T [n < D, pad 256][k < ofeat_k] with
  // U[8 h + a][n] = sum_d Wv~[a][h dh + d] Wol[h dh + d][n] (a < 5; a = 5..7 zero), and its planes
  const float* UT;
  const uint16_t* UP;
  // layer 1 in coefficient space (gemm_lnch MODE 2, H = 4): planes of V^T and B^T [3][ldp][32],
  // and V^T [256][32] itself (layer1_ch_kernel, N = 10, 20)
  const uint16_t *L1VP, *L1BP;
  const float* L1VT;
  const float* W2T;     // envelope first (env_first): W2T [256 2N][KE] and its planes
  const uint16_t* W2P;
};
// Layer 1's attention output in feature space (attention.hip feat2, the chain prologue): per
// row o~ [ofeat_k] = per head h the five sums o~_h[a] = sum_j A_ij f~_j[a] (f~ = (z, x, y,
// spin, 1)) at columns 8 h + a, zeros elsewhere, so o = o~_h Wv~ and o Wol = o~ U (K = ofeat_k)
inline int ofeat_k(const Dims& d) { return (8 * d.H + 31) / 32 * 32; }

// Channel bookkeeping for one pass: C = 1 (log psi only) or 2N+5 (local energy).
struct Pass {
  int nw;      // walkers in this pass
  int C;       // channels
  int rows;    // nw * N * C
  int rows_pad;
};

constexpr int kRowPad = 256;
// walker-row buffers (h, qkv, o, t) are padded to 768 = lcm(96, 256) rows, so the log-psi
// LayerNorm GEMM may take 64-, 96- or 128-row tiles without reading past the buffer
constexpr int kWalkerRowPad = 768;
inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

// Opt a kernel into more than 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU).
template <typename Kern>
inline void ensure_smem(Kern kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
}

// ---- kernel launchers (each .hip file) ----------------------------------------
// gemm.hip: Y[r][n] = sum_k X[r][k] W[k][n] + (r % C == 0 ? bias[n] : 0) + (R ? R[r][n] : 0)
void launch_gemm(const float* X, int ldx, const float* W, int ldw, const float* bias, const float* R, int ldr,
                 float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s);
void launch_gemm_variant(int v, const float* X, int ldx, const float* W, int ldw, const float* bias, const float* R,
                         int ldr, float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s);
// NT form: Y = X Wt^T, Wt[n][k] (row stride ldw), K % 32 == 0, Wt rows padded to 256.
void launch_gemm_nt_variant(int v, const float* X, int ldx, const float* Wt, int ldw, const float* bias,
                            const float* R, int ldr, float* Y, int ldy, int rows, int ncols, int K, int C,
                            hipStream_t s);
void set_gemm_variant(int v);
// NT GEMM with the tile shape chosen from (rows, ncols, residual): Wt[n][k], row stride ldw.
void launch_gemm_nt(const float* X, int ldx, const float* Wt, int ldw, const float* bias, const float* R, int ldr,
                    float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s);
// Log-psi rows (C = 1), D = 256: GEMM + bias, then (mode 0) + h or (mode 1) h + tanh(.),
// then LayerNorm (ln = gamma|beta), written in place over h [rows][256].
bool gemm_ln_supported(int D, int K);
void launch_gemm_ln(const float* X, int ldx, const float* Wt, int ldw, const float* bias, const float* ln, float* h,
                    int rows, int K, int mode, int bm, hipStream_t s);
// gemm_x6.hip: split-bf16 GEMM (f32-accurate, 6 bf16 MFMAs per product block).
// Wp = three bf16 planes [3][ldp][K] of the transposed weight (launch_split_planes),
// ldp = x6_plane_rows(ncols); K % 32 == 0; X holds round_up(rows, 256) readable rows.
int x6_plane_rows(int ncols);
void launch_split_planes(const float* Wt, int ldw, int ncols, int K, uint16_t* Wp, hipStream_t s);
bool gemm_x6_supported(int K);
void launch_gemm_x6_variant(int v, const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias,
                            const float* R, int ldr, float* Y, int ldy, int rows, int ncols, int K, int C,
                            hipStream_t s);
void launch_gemm_x6(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* R, int ldr,
                    float* Y, int ldy, int rows, int ncols, int K, int C, hipStream_t s);
// h = LN(h + X W + b) (mode 0) or LN(h + tanh(X W + b)) (mode 1), in place, split-bf16
// arithmetic; h [rows][256], ln = [gamma(256), beta(256)]; nw = tile form (0: pick; gemm_x6.hip).
// feat (layer 1 of log psi, mode 0): the residual h = features W0 is formed in the epilogue
// from geo [rows][4] = (sin th, cos th, sin ph, cos ph) and W0 [4][256] instead of read.
struct X6Feat {
  const float* W0 = nullptr;
  const float* geo = nullptr;
  int N = 1, n_up = 0;
  // launch_chain_x6 only: layer 1's attention formed in the chain prologue from the features
  // (folded W0 Wqkv [4][3D], bqkv [3D]) instead of read from X1 (chain_attn_supported)
  const float* W0qkv = nullptr;
  const float* bqkv = nullptr;
  const float* Mqk = nullptr;  // [H][kMqkStride] (attn_val.h attn_feat_core)
  // with W0qkv: layer 1's coefficient-space maps (planes of V^T, B^T; launch_l1_basis)
  const uint16_t* L1V = nullptr;
  const uint16_t* L1B = nullptr;
};
void launch_gemm_x6_ln(const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias, const float* ln,
                       float* h, int rows, int K, int mode, int nw, hipStream_t s, X6Feat feat = X6Feat{});
// gemm_lnch.hip: channel rows (C = 2N + 5 per electron, ne electrons), D = K = 256, N <= 8:
// h = LN_ch(h + X W + b) (mode 0) or LN_ch(h + tanh_ch(h W + b)) (mode 1) in ONE launch,
// in place over h [ne * C][256]; X [ne * C][256] (mode 1: X = h); split-bf16 arithmetic.
// DH_LNCH=0 selects the GEMM + layernorm_ch pair instead.
bool gemm_lnch_supported(int N, int D);
int set_lnch_form(int f);  // 0 off, 1 gemm_lnch_kernel; returns the previous form
// K: X's row length and the contraction (mode 0 / 2; 256, or layer 1's ofeat_k o~ rows with
// Wp = the planes of U^T); mode 1 contracts over h's 256 features.  Mode 2 (layer 1 whole, H = 4:
// LN1, Wm, tanh_ch, LN2 from the o~ rows; ln = LN2's scale | shift, bias = bol, W0f = W0): Wv /
// Wb = the planes of layer 1's coefficient-space maps V^T / B^T (launch_l1_basis, K = 32).
void launch_gemm_lnch(int N, const float* X, const uint16_t* Wp, int ldp, const float* bias, const float* ln,
                      const float* geo, float* h, int ne, int mode, hipStream_t s,
                      const float* W0f = nullptr, int n_up = 0, int K = 256, const uint16_t* Wv = nullptr,
                      const uint16_t* Wb = nullptr);
// Layer 1 in coefficient space (gemm_lnch.hip MODE 2): with E = [W0 (4); U's 5 H nonzero rows;
// bol; ones] and row 26 = beta, BT[n][j] = gamma_n E[j][n] (j < 26), beta_n (j = 26), and
// VT[n][j] = sum_k B[j][k] Wm[k][n] (+ bm_n for j = 26); 32 columns, f64 sums; H = 4.
void launch_l1_basis(const Dims& d, const float* W0, const float* UT, const float* bol, const float* ln1,
                     const float* Wm, const float* bm, float* BT, float* VT, hipStream_t s);
bool chain_attn_supported(int N, int H, int dh);
// Log-psi layer tail in one launch (D = K = 256): h1 = LN1(h + X1 Wol + b1) (feature
// residual when feat.W0), h = LN2(h1 + tanh(h1 Wm + b2)), then Y3 = h W3 + b3 if Wp3.
void launch_chain_x6(const float* X1, const uint16_t* Wp1, int ldp1, const float* b1, const float* ln1,
                     const uint16_t* Wp2, int ldp2, const float* b2, const float* ln2, const uint16_t* Wp3, int ldp3,
                     const float* b3, int n3, float* Y3, int ldy3, float* h, int rows, X6Feat feat, hipStream_t s,
                     bool store_h = true);
// dst[c][r] = src[r][c] for r < rows, c < cols (row strides ld_src / ld_dst).
void launch_transpose(const float* src, int ld_src, int rows, int cols, float* dst, int ld_dst, hipStream_t s);

// input.hip
// Features (psiformer.py:51-60) of every channel times W0 -> h [rows][D]; also
// writes geo[nw][N][4] = (sin th, cos th, sin ph, cos ph).
// With W0qkv != nullptr it also writes layer 1's q|k|v = f (W0 Wqkv) (+ bqkv on value
// rows): the first attention projection is folded into the K=4 input map.
void launch_input(const Dims& d, const float* x, const float* W0, const float* W0qkv, const float* bqkv, float* h,
                  float* qkv, float* geo, int nw, int C, hipStream_t s);
// Proposal (mcmc.py:67-102): x2 = sph_sampling(x, noise).
// geo (optional): the proposal's geometry (sin/cos of the f32 angles, as input_kernel).
void launch_propose(const Dims& d, const float* x, float* x2, int nw, float width, uint64_t seed, uint64_t step,
                    int64_t walker_offset, const float* noise, int noise_stride, hipStream_t s, float* geo = nullptr);
// accept of `step` + proposal of `step + 1` (and its geometry) in one launch.
void launch_accept_propose(const Dims& d, float* x, float* x2, float* geo, float* lp, const float* logpsi2,
                           int32_t* n_acc, int nw, float width, uint64_t seed, uint64_t step, int64_t walker_offset,
                           const float* noise, const float* noise2, hipStream_t s);
void launch_init_walkers(const Dims& d, float* x, int nw, uint64_t seed, int64_t walker_offset, hipStream_t s);

// attention.hip: channel self-attention for all heads.
// W0qkv/bqkv non-null: layer-1 q|k|v formed in-kernel from the input features (only when
// attention_takes_features(d)); otherwise read from qkv [rows][3D].
bool attention_takes_features(const Dims& d, int C);
// channel attention on the matrix cores (attention_mfma.hip): C > 1, dh = 64, N = 10, 20
bool attention_mfma_supported(const Dims& d);
void launch_attention_mfma(const Dims& d, const float* qkv, const float* geo, float* o, int nw, hipStream_t s,
                           const float* W0qkv, const float* bqkv);
void launch_attention(const Dims& d, const float* qkv, const float* geo, float* o, int nw, int C, hipStream_t s,
                      const float* W0qkv = nullptr, const float* bqkv = nullptr, const float* Mqk = nullptr);
// layer 1's 5 x 5 score forms per head, Mqk[h][a][b] = sum_d Wq~[a][h dh + d] Wk~[b][h dh + d] / 8
// (Wq~ / Wk~ = the folded W0 Wqkv rows with the bias as row 4; dh = 64; f64 sums)
void launch_lowrank_qk(const Dims& d, const float* W0qkv, const float* bqkv, float* Mqk, hipStream_t s);
// U^T [n][ofeat_k] (row stride ofeat_k, rows n < D; f64 sums) from the folded W0 Wqkv, bqkv and Wol
void launch_ofeat_weight(const Dims& d, const float* W0qkv, const float* bqkv, const float* Wol, float* UT,
                         hipStream_t s);

// layernorm.hip
//   mode 0: h = LN_ch(X)           (X may alias h)
//   mode 1: h = LN_ch(h + tanh_ch(Z))
void launch_layernorm(const Dims& d, const float* X, const float* Z, const float* ln, const float* geo, float* h,
                      int nw, int C, int mode, hipStream_t s,
                      const float* W0f = nullptr);
// layer 1 of the local energy at N = 10, 20 in one launch from the o~ rows O [ne C][KO]
// (layernorm.hip layer1_ch_kernel): UT = U^T [256][KO], VT = V^T [256][32] (launch_l1_basis)
bool layer1_ch_supported(const Dims& d);
void launch_layer1_ch(const Dims& d, const float* O, const float* UT, const float* VT, const float* W0f,
                      const float* bol, const float* ln1, const float* ln2, const float* geo, float* h, int nw,
                      hipStream_t s);

// det.hip
//   value mode (C == 1): logpsi[nw][2]
//   energy mode (C == 2N+5): e_l[nw][2], obs[nw][8]
// MCMC epilogue of the value kernel (round 5): after log psi of the proposal x2 (= the x the
// kernel evaluates), the accept of `step` (mcmc.py:55-62: x, lp, nacc updated) and, when
// `propose`, the next proposal of step + 1 into x2 / geo (mcmc.py:67-102) — what
// launch_accept_propose / launch_accept do, per walker, bit for bit, without their launch.
struct McmcEpi {
  int on = 0, propose = 0;
  float* x = nullptr;
  float* x2 = nullptr;
  float* geo = nullptr;
  float* lp = nullptr;
  int32_t* nacc = nullptr;
  float width = 0.f;
  uint64_t seed = 0, step = 0;
  int64_t woff = 0;
  const float* noise = nullptr;   // this step's injected noise (accept uniform)
  const float* noise2 = nullptr;  // the next step's (its proposal)
};
void launch_det_value(const Dims& d, const float* F, const float* x, const float* jastrow, const float* norm,
                      float* logpsi, int nw, hipStream_t s, const McmcEpi& epi = McmcEpi{});
// phic != nullptr (det_precontract(d)): the channel matrices are first contracted from F by
// env_contract_kernel into phic [nw][K][C][N][N] complex, then assembled from there
// NetObs estimators (netobs.hip): theta / pair-angle histograms, LLL monopole harmonics
void launch_histograms(const float* x, int B, int N, int db, int pb, float* dens, float* pair, hipStream_t s);
void launch_monopole_orbitals(const float* pts, int n, int flux, float* out, hipStream_t s);
bool det_precontract(const Dims& d);
void launch_det_energy(const Dims& d, const float* F, const float* x, const float* geo, const float* jastrow,
                       const float* norm, float* e_l, float* obs, int nw, hipStream_t s, float* phic);
size_t det_energy_smem_bytes(const Dims& d);
// envelope first (round 6, C4 / C5: one spin block, one determinant, N > 8; det.hip): the
// channel matrices PhiC from h directly — Weff = E2 W2 per electron, F of six special rows per
// electron, env_phi_kernel — instead of the full orbital map F and env_stream / env_contract
bool env_first(const Dims& d);
int env_first_k(const Dims& d);  // KE: the envelope-coefficient row length (2 M padded to 32)
// W2T [256 * 2N][KE] from the packed Worb (launch_split_planes makes its planes)
void launch_env_w2(const Dims& d, const float* Worb, float* W2T, hipStream_t s);
// S [round_up(6 ne, 256)][256], FS [round_up(6 ne, 256)][ld_orb], E2 [round_up(ne, 256)][KE],
// Weff [round_up(ne, 256)][256 * 2N] (ne = nw N): workspace; phic [nw][C][N][N] complex
void launch_env_first(const Dims& d, const float* h, const float* geo, const float* x, const float* norm,
                      const float* WorbT, const float* borb, const uint16_t* WorbP, const float* W2T,
                      const uint16_t* W2P, bool x6, int nw, float* S, float* FS, float* E2, float* Weff, float* phic,
                      hipStream_t s);
// det_energy_kernel<0, true> alone on precontracted channel matrices
void launch_det_energy_pc(const Dims& d, const float* x, const float* geo, const float* jastrow, const float* norm,
                          float* e_l, float* obs, int nw, hipStream_t s, const float* phic);
// test hook: env_leaf (e0, dth, dph, lb, d2th as re / im pairs: 10 floats) of n (theta, phi)
// pairs for every harmonic p < M, norm 1, the production gauge; sq: powers by squaring
void launch_env_leaf_probe(const float* thph, int n, int M, int sq, float* out, hipStream_t s);
void launch_potential(const Dims& d, const float* x, float* pe, int nw, hipStream_t s);
// mcmc.hip: accept/reject (mcmc.py:55-62).
void launch_accept(const Dims& d, float* x, const float* x2, float* lp, const float* logpsi2, int32_t* n_acc,
                   int nw, uint64_t seed, uint64_t step, int64_t walker_offset, const float* noise,
                   int noise_stride, hipStream_t s);
void launch_lp_from_logpsi(const float* logpsi, float* lp, int32_t* n_acc, int nw, hipStream_t s);

// kinetic.hip: KE / Lz / Lz^2 / L^2 of an arbitrary log psi from its derivatives
size_t kinetic_assembly_lds_bytes(int N);
void launch_kinetic_assembly(const double* x, const double* g, const double* H, int nw, int N, double Q, double r,
                             float* ke, float* mom, hipStream_t s);

// stats.hip
void launch_stats(const float* e_l, const float* obs, const int32_t* n_acc, int B, int steps, int penalties,
                  float* out, hipStream_t s);
// g: device pointer to the reduced stats; diff [B][2]; nvalid [1]
void launch_loss_diff(const float* e_l, const float* obs, int B, const float* g, float lz_penalty, float lz_center,
                      float l2_penalty, float* diff, float* nvalid, hipStream_t s);

// grad.hip: reverse mode of log psi w.r.t. the parameters (see the file header)
constexpr int kGradChunk = 512;       // rows per weight-gradient partial
constexpr int kLnRowsPerBlock = 64;   // rows per LayerNorm-backward block (one partial each)
int grad_chunks(int rows);
int ln_bwd_blocks(int rows);
void launch_ln_fwd(const float* a, const float* z, const float* ln, float* out, int rows, int D, hipStream_t s);
void launch_ln_bwd(const float* a, const float* z, const float* ln, const float* dy, const float* dres, float* da,
                   float* dz, float* pg, int rows, int D, hipStream_t s);
void launch_attn_bwd(const Dims& d, const float* qkv, const float* dO, float* dqkv, int nw, hipStream_t s);
void launch_tn_partial(const float* X, int ldx, const float* Y, int ldy, int rows, int M, int Nc, float* P,
                       hipStream_t s);
void launch_colsum_partial(const float* Y, int ldy, int rows, int Nc, float* P, hipStream_t s);
void launch_w0_partial(const Dims& d, const float* geo, const float* Y, int ldy, int rows, float* P, hipStream_t s);
// out[r * ldo + c] = scale * sum_ch P[ch * stride + r * ldp + c] (+ out if acc), r < nr, c < nc
void launch_reduce2d(const float* P, int nchunk, size_t stride, int ldp, int nr, int nc, float* out, int ldo,
                     float scale, int acc, hipStream_t s);
void launch_small_gemm(int M, int N, int K, const float* A, int lda, int ta, const float* B, int ldb, int tb, float* C,
                       int ldc, int acc, hipStream_t s);
void launch_copy2d(const float* src, int lds, float* dst, int ldd, int nr, int nc, hipStream_t s);
void launch_cotangent(const float* diff, const float* nvalid, int B, int part, float* ct, hipStream_t s);
void launch_adam(float* p, const float* g, float* mu, float* nu, size_t n, float lr, float b1, float b2, float eps,
                 int step, hipStream_t s);
// "sparse" orbitals (blocks.py:52-62): featured orbitals with 8 features per (j, k),
// mixed into the M harmonics by lll_weight (DenseGeneral over axis 1, real kernel, bias on
// the real part), folded into the full layout:
//   Wfull[d][m NK + jk] = sum_a W8[d][a NK + jk] Wl[a][m]  (rows d < D; row D = the bias,
//   with + bl[m] when `real_part`)
void launch_sparse_fold(const float* W8, const float* b8, const float* Wl, const float* bl, int real_part, int D,
                        int NK, int M, float* Wfull, int ldw, float* bfull, hipStream_t s);
// gradient: dW8[d][a NK + jk] (+)= sum_m dWfull[d][m NK + jk] Wl[a][m] (rows d < D, row D bias)
void launch_sparse_unfold(const float* dWfull, int ldw, const float* dbfull, const float* Wl, int D, int NK, int M,
                          float* dW8, float* db8, int acc, hipStream_t s);
// dWl[a][m] (+)= sum_{blocks i} [sum_d W8_i[d][a NK + jk] dWfull_i[d][m NK + jk] + b8_i . dbfull_i];
// dbl[m] (+)= sum_{real blocks} sum_jk dbfull_i[m NK + jk].  W8s/b8s: per-block pointers.
struct SparseBlocks {
  const float* W8[4];
  const float* b8[4];
  int n;
};
void launch_sparse_lll_grad(SparseBlocks blk, const float* dWfull, int ldw, const float* dbfull, int D, int NK, int M,
                            float* dWl, float* dbl, int acc, hipStream_t s);

// laughlin.hip: log psi (e_l == nullptr) or the local energy (e_l [nw][2], obs [nw][8])
// of the Laughlin wavefunction; expo [2][N] = (Q1 + m_j, Q1 - m_j)
size_t laughlin_smem_bytes(int N);
void launch_laughlin(const Dims& d, const float* x, const int* expo, float* logpsi, float* e_l, float* obs, int nw,
                     hipStream_t s);

// det.hip: backward of log psi = J + log sum_k det Phi_k for per-walker cotangents ct[nw][2]:
// dF [nw*N][ld_orb] (all columns written) and jg[nw][2] = ct.re * dJ / d(ee_par, ee_anti)
void launch_det_bwd(const Dims& d, const float* F, const float* x, const float* jastrow, const float* norm,
                    const float* ct, float* dF, float* jg, int nw, hipStream_t s);

// kfac.hip: KFAC curvature statistics, damped inverses and update (api.cpp dh_kfac_*)
struct KfacSlot {  // one factor matrix n x n (f32) at float offset `off` of the statistics buffer
  int n;
  size_t off;
};
struct KfacInvJob {  // one damped inverse: slot, the paired factor's slot (for pi), A or G side
  int slot, partner, is_a, n;
  float sqrt_scale;  // sqrt(fixed_scale) of the block
  size_t gj_off;     // f64 offset of the n x n matrix in the inverse buffer
};
struct KfacBlockJob {  // one dense block: gradient segments (ref layout) and f64 work offsets
  size_t kernel_off;
  long long bias_off;  // -1: no bias
  int din, dout;
  size_t v_off, t_off, pv_off;
};
struct KfacGemmJob {  // C[M][N] = A[M][K] B[K][N], f64 offsets into one buffer
  size_t a_off, b_off, c_off;
  int M, N, K;
};
constexpr int kKfacMaxGen = 80;
struct KfacGenTable {  // generic (diagonal) parameter segments: ref offset, compact offset
  int n, total;
  size_t ref[kKfacMaxGen];
  int cmp[kKfacMaxGen];
};
struct KfacDevPlan {  // device copies of the job tables (owned by the handle)
  KfacSlot* slots;
  KfacInvJob* inv_jobs;
  KfacBlockJob* block_jobs;
  KfacGemmJob *gemm1, *gemm2;
  int nslots, njobs, nblocks, nmax, max_v, max_m, max_n;
  KfacGenTable gen;
};
void launch_kfac_aug(const float* P, int nch, int n, float* out, int ld, float scale, float corner, int acc,
                     hipStream_t s);
void launch_kfac_feat_gram(const Dims& d, const float* geo, int rows, float* P, hipStream_t s);
// "sparse" orbitals: the featured-orbital tangent lll dF and the lll output tangent as rows of M
void launch_kfac_sparse_dphi(const float* dF, int ld, const float* lll, int M, int NK, int seg, int nr, int na, int N,
                             int lo, float* out, hipStream_t s);
void launch_kfac_sparse_regroup(const float* dF, int ld, int M, int NK, int seg, int nr, int na, int N, int lo,
                                float* out, hipStream_t s);
void launch_kfac_fisher_ct(const float* logpsi, int nw, float* ct, hipStream_t s);
void launch_kfac_generic(const float* fgrad, const KfacGenTable& tab, float* diag, float scale, hipStream_t s);
void launch_kfac_ema(float* raw, const float* st, size_t n, float ema, hipStream_t s);
size_t kfac_gj_tmp_doubles(int njobs, int nmax);
void launch_kfac_invert(const KfacDevPlan& p, const float* raw, double inv_weight, double sqrt_lambda, double* tr,
                        double* gj, double* tmp, hipStream_t s);
void launch_kfac_precondition(const KfacDevPlan& p, const float* grad, const float* raw_diag, double inv_weight,
                              double lambda, double* buf, float* pg, size_t nref, double* info, hipStream_t s);
void launch_kfac_update(float* params, const float* pg, size_t n, double* info, double lr, double norm_constraint,
                        hipStream_t s);

}  // namespace dh

