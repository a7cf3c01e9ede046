/*
 * deephall_amd.h — C ABI of the MI355X-native DeepHall VMC inner loop.
 *
 * The reference (peterzjx/DeepHall) has no FFI: its hot path is a set of Python
 * callables transformed by JAX.  This ABI is the native drop-in underneath the
 * Python mirror of those callables (deephall_amd/), one entry point per
 * reference interface:
 *
 *   dh_create / dh_set_params   <-> make_network(system, network)
 *                                   deephall/networks/__init__.py:22-37, and the
 *                                   parameter tree of model.init (train.py:62)
 *   dh_logpsi                   <-> Psiformer.__call__ / model.apply, vmapped
 *                                   deephall/networks/psiformer.py:72-76, train.py:69,84
 *   dh_mcmc_step                <-> make_mcmc_step(...)(params, data, key, width)
 *                                   deephall/mcmc.py:105-150 (mh_update 25-64,
 *                                   sph_sampling 67-102)
 *   dh_local_energy             <-> local_energy(f, system) vmapped
 *                                   deephall/hamiltonian.py:175-212 (+ make_local_kinetic_energy 83-172,
 *                                   make_potential 63-80), loss.py:51
 *   dh_energy_stats             <-> device-local statistics of loss_and_grad
 *                                   deephall/loss.py:30-38, 66-92 (before pmean)
 *   dh_init_walkers             <-> init_guess, deephall/train.py:40-54
 *
 * Conventions
 *   - Every pointer argument except `cfg`/`out`/`offsets` is a DEVICE pointer.
 *     Buffers (including the workspace) are owned by the caller; the library
 *     owns only the handle and the packed parameter copy made by dh_set_params.
 *   - Calls are asynchronous on `stream` (a hipStream_t; NULL = default stream).
 *     One handle per device; a handle is not thread-safe.
 *   - Return 0 on success, a negative DH_E* code on error; dh_last_error()
 *     returns a thread-local message.  No C++ exception crosses the ABI.
 *     NaN walkers propagate as NaN exactly as in the reference (loss.py uses
 *     nanmean; train.py:159 aborts on a NaN energy).
 *   - Walker coordinates: float32 [B][N][2] = (theta, phi), as the reference's
 *     data[B, N, 2] (train.py:53).
 */
#ifndef DEEPHALL_AMD_H
#define DEEPHALL_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DH_OK 0
#define DH_EINVAL -1   /* bad argument / shape / unsupported config */
#define DH_EHIP -2     /* HIP runtime error */
#define DH_ENOMEM -3   /* workspace too small */
#define DH_ESTATE -4   /* parameters not set */

#define DH_INTERACTION_COULOMB 0
#define DH_INTERACTION_HARMONIC 1
#define DH_NETWORK_PSIFORMER 0
#define DH_NETWORK_LAUGHLIN 1 /* networks/laughlin.py: ground state, quasihole, quasiparticle (no parameters) */
#define DH_ORBITAL_FULL 0
#define DH_ORBITAL_SPARSE 1 /* blocks.py:52-62: 8 features per (j, k) mixed into the M harmonics by
                               lll_weight; folded into the full layout when parameters are set */

/* System + Network fields of deephall/config.py:56-104 that the hot path reads.
 * The first field is the caller's sizeof(dh_config): dh_create rejects any other
 * value with DH_EINVAL, so a binding written against an older (shorter) layout fails
 * loudly instead of letting the library read past the caller's struct.  Set it with
 * DH_CONFIG_INIT or `cfg.struct_size = sizeof(dh_config)`. */
typedef struct dh_config {
  uint32_t struct_size;       /* = sizeof(dh_config) = 60 bytes        */
  int n_up, n_dn;             /* System.nspins                          */
  int flux;                   /* System.flux = 2Q                       */
  float radius;               /* System.radius; <= 0 means sqrt(Q)      */
  float interaction_strength; /* System.interaction_strength            */
  int interaction_type;       /* DH_INTERACTION_*                       */
  int num_heads;              /* PsiformerNetwork.num_heads             */
  int heads_dim;              /* PsiformerNetwork.heads_dim             */
  int num_layers;             /* PsiformerNetwork.num_layers            */
  int ndets;                  /* PsiformerNetwork.determinants          */
  int orbital_type;           /* Network.orbital, DH_ORBITAL_*          */
  int network_type;           /* Network.type, DH_NETWORK_*             */
  float excitation_lz;        /* Laughlin: System.lz_center (networks/__init__.py:26) */
  int cf_flux;                /* Laughlin: composite-fermion flux p (laughlin.py:23), >= 1 */
} dh_config;
#define DH_CONFIG_INIT {sizeof(dh_config)}

typedef struct dh_handle dh_handle;

int dh_create(const dh_config* cfg, dh_handle** out);
void dh_destroy(dh_handle* h);
const char* dh_last_error(void);
const char* dh_version(void);

/* Packed parameter layout.  Segment s starts at float offset
 * offsets[s] of the packed buffer (each segment 64-float aligned); segment
 * order:
 *   0                  W0        [4][D]           PsiformerLayers_0/Dense_0/kernel
 *   per layer l (8 segments, base 1+8l):
 *     +0 Wqkv [D][3D]  query|key|value kernels, columns (h, d) per block
 *     +1 bqkv [3D]
 *     +2 Wol  [D][D]   out/kernel (as [H*dh][D]) @ Dense_{2l+1}/kernel  (folded)
 *     +3 bol  [D]      out/bias @ Dense_{2l+1}/kernel
 *     +4 ln1  [2][D]   LayerNorm_{2l}: scale, bias
 *     +5 Wm   [D][D]   Dense_{2l+2}/kernel
 *     +6 bm   [D]      Dense_{2l+2}/bias
 *     +7 ln2  [2][D]   LayerNorm_{2l+1}: scale, bias
 *   1+8L     Worb [D][ld_orb]  columns ((blk*2+part)*M + m)*N*K + j*K + k,
 *                              blk = spin block, part 0 = real / 1 = imag,
 *                              zero padded to ld_orb (multiple of 128)
 *   2+8L     borb [ld_orb]
 *   3+8L     jastrow [2]       ee_par, ee_anti
 *   4+8L     W0qkv [4][3D]     W0 @ Wqkv of layer 0: the first attention projection
 *                              folded into the K=4 input map (unused if L == 0)
 * Returns the number of segments (5+8L) and writes up to `n` offsets; the
 * total float count is offsets[nseg] (written if n > nseg). */
int dh_param_layout(const dh_handle* h, size_t* offsets, int n);
/* Copy the packed parameter buffer (device pointer, `count` floats) into the
 * handle.  `count` must equal the total from dh_param_layout. */
int dh_set_params(dh_handle* h, const float* params, size_t count, void* stream);

/* Reference parameter tree, flattened (SURVEY.md Appendix B names, Flax order):
 *   0                 PsiformerLayers_0/Dense_0/kernel [4][D]
 *   per layer l (15 segments, base 1+15l):
 *     MultiHeadAttention_l/{query,key,value}/{kernel [D][H*dh], bias [H*dh]}  (+0..+5)
 *     MultiHeadAttention_l/out/{kernel [H*dh][D], bias [D]}                   (+6, +7)
 *     Dense_{2l+1}/kernel [D][D]; LayerNorm_{2l}/{scale, bias} [D]             (+8..+10)
 *     Dense_{2l+2}/{kernel [D][D], bias [D]}; LayerNorm_{2l+1}/{scale, bias}   (+11..+14)
 *   1+15L+2i, +1      Orbitals_0/featured_orbitals/DenseGeneral_i/{kernel [D][F*N*K],
 *                     bias [F*N*K]}, i < 2 * (spin blocks); F = M ("full") or 8 ("sparse")
 *   "sparse" only:    Orbitals_0/lll_weight/{kernel [8][M], bias [M]}
 *   then              Jastrow_0/ee_par [1], Jastrow_0/ee_anti [1]
 * Segments are 64-float aligned.  Returns the segment count; offsets[nseg] = total floats.
 * Parameter gradients (dh_logpsi_vjp) use the same layout. */
int dh_ref_layout(const dh_handle* h, size_t* offsets, int n);
/* Upload the reference tree (device pointer, `count` = total floats of dh_ref_layout) and
 * pack it on the device: concatenations, zero padding, and the folds Wo Wl, bo Wl,
 * W0 Wqkv (double-accumulated), transposed / split-bf16 copies.  Replaces the host
 * packing of dh_set_params; required by dh_logpsi_vjp. */
int dh_set_params_ref(dh_handle* h, const float* ref, size_t count, void* stream);

/* Parameter gradient by reverse mode (loss.py:53-64, 93-108 with jax.grad of the network):
 *   grad = sum_b ct[b][0] d Re log psi_b / dp + ct[b][1] d Im log psi_b / dp
 * ct [B][2] per-walker cotangents (dh_grad_cotangent), grad [dh_ref_layout total] f32,
 * logpsi [B][2] optional (NULL) log psi of the walkers from the same forward pass.
 * Processes walkers in chunks sized to the workspace (dh_vjp_workspace_bytes per chunk). */
size_t dh_vjp_workspace_bytes(const dh_handle* h, int batch);
int dh_logpsi_vjp(dh_handle* h, const float* x, int B, const float* ct, float* grad, float* logpsi, void* ws,
                  size_t ws_bytes, void* stream);
/* KFAC — the reference's default optimizer (deephall/optimizers/kfac.py:195-241, kfac_jax
 * Optimizer with "fisher_exact" curvature, repeated-dense Kronecker blocks, pi-adjusted
 * damping, norm constraint; restated in oracle/kfac.py).  Orbital "full" only.
 *
 * dh_kfac_layout: describes the curvature statistics buffer; returns the number of size_t
 *   values, writes up to n of them: [0] statistics floats, [1] factor-matrix floats,
 *   [2] factor slots S, [3] dense blocks nb, [4] generic (diagonal) floats, [5] dh_kfac_step
 *   workspace bytes, then per block (kernel segment, bias segment or SIZE_MAX, d_in, d_out,
 *   A slot, G slot, 1000 x fixed scale), then per slot (n, float offset).
 * dh_kfac_vjp: one forward pass over x [B][N][2] with saved activations, then
 *   (ct != NULL) the gradient of dh_logpsi_vjp into grad, and the Fisher reverse pass
 *   (cotangent sqrt(2) on Re log psi; 0 for a walker with non-finite log psi) whose layer
 *   Gram matrices A = x~^T x~ / rows, G = dy^T dy / rows and generic diagonal
 *   (sum_b tangent)^2 / B are WRITTEN to stats (this device's batch; average over devices
 *   before dh_kfac_step).  logpsi [B][2] optional.  Workspace per chunk:
 *   dh_kfac_workspace_bytes.
 * dh_kfac_step: raw = ema * raw + stats (stats may be NULL: no EMA update), then with the
 *   EMA weight `weight` (sum of ema^k): damped inverses, P g into pgrad (dh_ref_layout
 *   floats), info[0] = <P g, g>, info[1] = c = min(1, sqrt(norm_constraint / (lr^2 <P g, g>))),
 *   info[2] = lr c (device doubles), and params -= lr c P g when params != NULL. */
int dh_kfac_layout(dh_handle* h, size_t* out, int n);
size_t dh_kfac_workspace_bytes(const dh_handle* h, int batch);
int dh_kfac_vjp(dh_handle* h, const float* x, int B, const float* ct, float* grad, float* stats, float* logpsi,
                void* ws, size_t ws_bytes, void* stream);
int dh_kfac_step(dh_handle* h, float* raw, const float* stats, float ema, float weight, const float* grad,
                 float* params, float lr, float damping, float norm_constraint, float* pgrad, double* info, void* ws,
                 size_t ws_bytes, void* stream);

/* Cotangents of the gradient estimator 2 nanmean(conj(d log psi) diff) (loss.py:59-64):
 * part 0 (its real part, ENERGY_GRAD): ct = 2 (Re diff, Im diff) / n;
 * part 1 (its imaginary part, SR_F_VECTOR): ct = 2 (Im diff, -Re diff) / n;
 * n = nvalid[0] (device), NaN diffs give 0. */
int dh_grad_cotangent(const float* diff, const float* nvalid, int B, int part, float* ct, void* stream);
/* optax.adam step in place (optimizers/adam.py:24-43): b1, b2, eps as optax, lr = the
 * schedule value at `step` (config.py:125-137), bias correction with step + 1; NaN
 * gradients count as 0 (loss.py:64 nan_to_num). */
int dh_adam_update(float* params, const float* grad, float* mu, float* nu, size_t n, float lr, float b1, float b2,
                   float eps, int step, void* stream);

/* GEMM arithmetic of the local-energy (2N+5 channel) pass:
 *   DH_GEMM_F32   exact-f32 MFMA (v_mfma_f32_32x32x2_f32), f32 rounding per product;
 *   DH_GEMM_X6    split-bf16 MFMA: each f32 operand split exactly into three bf16 terms,
 *                 six bf16 products per pair (dropped terms <= 2^-24 |ab|, f32 accumulate);
 *                 error at the level of the f32 GEMM (tests/test_gpu_kernels.py), 2.67x the
 *                 f32 matrix rate.
 *   DH_GEMM_X6_ALL  split-bf16 also for the log-psi / MCMC GEMMs (the two per layer that
 *                 carry a LayerNorm with it in their epilogue).  Default.
 *   DH_GEMM_X6_ALL_UNFUSED  as DH_GEMM_X6_ALL, but the local energy's channel LayerNorms run
 *                 as separate passes after their GEMMs instead of inside them (test hook for
 *                 the fused gemm_lnch kernel; same arithmetic up to f32 summation order).
 * In DH_GEMM_F32 and DH_GEMM_X6 the log-psi / MCMC passes use the exact-f32 kernels. */
#define DH_GEMM_F32 0
#define DH_GEMM_X6 1
#define DH_GEMM_X6_ALL 2
#define DH_GEMM_X6_ALL_UNFUSED 3
int dh_set_gemm_mode(dh_handle* h, int mode);

/* Workspace bytes needed to process `batch` walkers: op 0 = log psi / MCMC,
 * op 1 = local energy.  Local energy processes walkers in chunks sized to the
 * workspace it is given (at least one walker). */
size_t dh_workspace_bytes(const dh_handle* h, int batch, int op);

/* log psi for B walkers: logpsi[B][2] = (Re, Im), Im the principal phase. */
int dh_logpsi(dh_handle* h, const float* x, int B, float* logpsi, void* ws, size_t ws_bytes, void* stream);

/* `steps` Metropolis-Hastings all-electron moves on B walkers, in place.
 *   x       [B][N][2]  walkers, updated in place (the reference donates data)
 *   lp      [B]        work/out: 2 Re log psi of the current walkers (computed
 *                      here at entry, mcmc.py:142)
 *   n_accept[B] int32  out: accepted moves per walker in this call
 *   width              proposal width (MCMC.width, mcmc.py:69-70)
 *   seed, counter      counter-based RNG (Philox4x32-10): the draw for walker g
 *                      (global index = walker_offset + b), step s uses counter
 *                      (g, counter + s, electron, 0) under key seed; results do
 *                      not depend on how walkers are sharded over devices
 *   noise              NULL, or injected noise [steps][B][2N+1] floats:
 *                      normals [N], phi uniforms in [0,1) [N], accept uniform [1]
 */
int dh_mcmc_step(dh_handle* h, float* x, float* lp, int32_t* n_accept, int B, int steps, float width,
                 uint64_t seed, uint64_t counter, int64_t walker_offset, const float* noise, void* ws,
                 size_t ws_bytes, void* stream);

/* Local energy for B walkers.
 *   e_l [B][2]   E_L = KE + lambda * PE (complex)
 *   obs [B][8]   KE re, KE im, PE (already times interaction_strength),
 *                Lz, Lz^2, L^2, logpsi re, logpsi im                         */
int dh_local_energy(dh_handle* h, const float* x, int B, float* e_l, float* obs, void* ws, size_t ws_bytes,
                    void* stream);

/* Device-local energy statistics (loss.py:66-92 before the pmean).  Writes
 * out[DH_NSTATS] floats: see DH_STAT_* indices.  Any B >= 1 (quantiles by a radix
 * select, no sort).  penalties != 0 also computes the clipped Lz^2, Lz, L^2 means that
 * System.lz_penalty / l2_penalty need (loss.py:76-88); else those entries are 0. */
#define DH_NSTATS 16
#define DH_STAT_ENERGY_RE 0    /* nanmean Re E_L                     */
#define DH_STAT_ENERGY_IM 1    /* nanmean Im E_L                     */
#define DH_STAT_CLIPPED_RE 2   /* nanmean Re iqr_clip(E_L)           */
#define DH_STAT_CLIPPED_IM 3   /* nanmean Im iqr_clip(E_L)           */
#define DH_STAT_ERE2 4         /* nanmean (Re E_L)^2                 */
#define DH_STAT_KINETIC_RE 5   /* mean KE re                         */
#define DH_STAT_KINETIC_IM 6   /* mean KE im                         */
#define DH_STAT_POTENTIAL 7    /* mean PE                            */
#define DH_STAT_LZ 8           /* mean Lz                            */
#define DH_STAT_LZ2 9          /* mean Lz^2                          */
#define DH_STAT_L2 10          /* mean L^2                           */
#define DH_STAT_PMOVE 11       /* sum n_accept / (steps * B)         */
#define DH_STAT_NVALID 12      /* number of non-NaN E_L              */
#define DH_STAT_CLIPPED_LZ2 13 /* nanmean iqr_clip(Lz^2)  (penalties) */
#define DH_STAT_CLIPPED_LZ 14  /* nanmean iqr_clip(Lz)    (penalties) */
#define DH_STAT_CLIPPED_L2 15  /* nanmean iqr_clip(L^2)   (penalties) */
/* h may be NULL (E_L of a log-psi callable evaluated outside the library). */
int dh_energy_stats(dh_handle* h, const float* e_l, const float* obs, const int32_t* n_accept, int B, int steps,
                    int penalties, float* out, void* stream);

/* The clipped energy difference that weights the parameter gradient (loss.py:75-89):
 *   d = E_L - <E_L>_clip + lz_penalty ((Lz^2 - <Lz^2>_clip) - 2 lz_center (Lz - <Lz>_clip))
 *         + l2_penalty (L^2 - <L^2>_clip),    diff = iqr_clip(d)  (local quantiles)
 * with the <.>_clip means read from `stats` (device, DH_STAT_* layout, already averaged
 * over devices).  diff[B][2] (re, im; NaN where E_L is NaN); nvalid[1] = number of
 * walkers with a non-NaN diff (the nanmean count of loss.py:64).  h may be NULL. */
int dh_loss_diff(dh_handle* h, const float* e_l, const float* obs, int B, const float* stats, float lz_penalty,
                 float lz_center, float l2_penalty, float* diff, float* nvalid, void* stream);

/* Potential energy only (make_potential, hamiltonian.py:63-80), NOT multiplied by
 * interaction_strength: pe[B]. */
int dh_potential(dh_handle* h, const float* x, int B, float* pe, void* stream);

/* ---- NetObs-style estimators (deephall/netobs_bridge/observables/NAME.py) ----------------
 * dh_histograms ADDS to density[density_bins] the counts of every electron's theta and
 * to pair[pair_bins] the 1/sin(theta_12)-weighted counts of every pair angle
 * theta_12 = arccos(r_i . r_j), i < j, both over [0, pi] with numpy's bin rule
 * (density.py:38-44, pair_corr.py:43-58; the caller applies pair_corr.py:57's scale).
 * Either count may be 0 (its pointer then unused).  Walkers x[B][nelec][2]. */
int dh_histograms(const float* x, int B, int nelec, int density_bins, int pair_bins, float* density, float* pair,
                  void* stream);
/* Lowest-Landau-level monopole harmonics Y_{Q,Q,m}, m = -Q..Q, Q = flux / 2, at n points
 * (theta, phi): out[n][flux + 1] complex (re, im), one_rdm.py:31-54 (cos theta clipped to
 * +-(1 - 1e-4) as there). */
int dh_monopole_orbitals(const float* points, int n, int flux, float* out, void* stream);

/* ---- log psi supplied by the caller: the arbitrary-callable boundary ---------------------
 * The reference's make_mcmc_step(batch_network, ...) (mcmc.py:105-150) and
 * make_local_kinetic_energy(f, Q, r) (hamiltonian.py:83-172) accept ANY log psi.  For one
 * that is not a network of this library the caller evaluates log psi (and, for the energy,
 * its derivatives) itself; these entry points do the rest on the device.
 *
 * MCMC with the same random streams as dh_mcmc_step (so a caller-evaluated network walks
 * exactly as the native one):
 *   dh_mh_init     lp[b] = 2 Re logpsi[b][0], n_accept[b] = 0           (mcmc.py:142)
 *   dh_mh_propose  x2 = sph_sampling(x) for step `step` = counter + s    (mcmc.py:67-102)
 *   dh_mh_accept   accept/select with logpsi2[B][2] = log psi(x2) (re, im): x, lp, n_accept
 *                  updated where 2 Re log psi(x2) - lp > log U             (mcmc.py:25-64)
 * noise: NULL or this step's injected [B][2N+1] (dh_mcmc_step layout).
 *
 * dh_kinetic_from_derivatives: KE (complex) and Lz, Lz^2, L^2 from x[B][N][2], the complex
 * first derivatives grad[B][N][2][2] (d/dtheta, d/dphi; re, im) and complex Hessian
 * hess[B][N][2][N][2][2] of log psi, all double; Q monopole strength, r radius; nelec <= 256.
 * Out: ke[B][2] (re, im), mom[B][3] (Lz, Lz^2, L^2). */
int dh_mh_init(const float* logpsi, float* lp, int32_t* n_accept, int B, void* stream);
int dh_mh_propose(const float* x, float* x2, int B, int nelec, float width, uint64_t seed, uint64_t step,
                  int64_t walker_offset, const float* noise, void* stream);
int dh_mh_accept(float* x, const float* x2, float* lp, const float* logpsi2, int32_t* n_accept, int B, int nelec,
                 uint64_t seed, uint64_t step, int64_t walker_offset, const float* noise, void* stream);
int dh_kinetic_from_derivatives(const double* x, const double* grad, const double* hess, int B, int nelec, double Q,
                                double r, float* ke, float* mom, void* stream);

/* Kernel timing with HIP events on the launch stream (bench / roofline).
 * dh_profile_enable(h, 1) starts recording every kernel launch of this handle;
 * dh_profile_read fills out[k*4 + {0,1,2,3}] = {launches, total ms, algorithmic
 * FLOPs, algorithmic bytes} for kernel class k (returns the number of classes):
 *   0 GEMM  1 attention  2 LayerNorm  3 input  4 det (log psi)  5 det (energy)
 *   6 MCMC proposal/accept; 7-10 = classes 0-3 launched with 2N+5 channels
 *   (local energy); 11 = layer 1 of the local energy in one launch (gemm_lnch MODE 2:
 *   LayerNorms, tanh and three 32-deep products).  out holds 4 * 12 doubles.
 *   Synchronises on the recorded events. */
int dh_profile_enable(dh_handle* h, int on);
int dh_profile_read(dh_handle* h, double* out, int reset);

/* Test hooks: run the network trunk + orbital GEMM only and leave the
 * activations in the workspace (trunk output at float offset 0, orbital
 * features at float offset dh_debug_f_offset). */
int dh_debug_trunk(dh_handle* h, const float* x, int B, int op, void* ws, size_t ws_bytes, void* stream);
size_t dh_debug_f_offset(const dh_handle* h, int B, int op);
/* Test hook: the envelope leaves of det.hip's env_leaf (e0, d/dtheta, d/dphi / sin theta,
 * Laplace-Beltrami, d2/dtheta2 as re / im pairs: 10 floats) of n (theta, phi) pairs thph[n][2]
 * for every harmonic p < M (norm 1, the kernels' gauge kappa = env_gauge(cos theta)) into
 * out[n][M][10]; sq = 1: integer powers by squaring (the production form), 0: powf. */
int dh_debug_env_leaf(const float* thph, int n, int M, int sq, float* out, void* stream);
/* Test hook: one launch of GEMM kernel variant `variant` (-1 = default):
 * Y = X W (+ bias on rows r % C == 0) (+ R).  X must hold round_up(rows, 256) rows.
 * variant >= 100 selects the NT kernels: W is then the TRANSPOSED weight Wt[n][k]
 * (row stride ldw) holding round_up(ncols, 256) rows, and K % 32 == 0. */
int dh_debug_gemm(int variant, const float* X, int ldx, const float* W, int ldw, const float* bias, const float* R,
                  int ldr, float* Y, int ldy, int rows, int ncols, int K, int C, void* stream);

/* Test hook: the log-psi GEMM with the LayerNorm fused into its epilogue (D = 256):
 * h = LN(h + X Wt^T + bias) (mode 0) or LN(h + tanh(X Wt^T + bias)) (mode 1), in place;
 * Wt[256][K] transposed weight (row stride ldw), ln = gamma[256] | beta[256];
 * bm = rows per workgroup (32, 64, 96; 0 = automatic).  X, h hold round_up(rows, 96) rows. */
int dh_debug_gemm_ln(int mode, int bm, const float* X, int ldx, const float* Wt, int ldw, const float* bias,
                     const float* ln, float* h, int rows, int K, void* stream);

/* Split-bf16 form of dh_debug_gemm_ln (weight as the planes of dh_debug_split_planes,
 * ldp >= dh_debug_x6_plane_rows(256)); nw = tile form: 1 = 96 rows x (3 x 4 waves),
 * 2 = 64 rows x (2 x 4 waves), 3 / 4 = 96 / 128 rows of whole-row waves, 0 = choose. */
int dh_debug_gemm_x6_ln(int mode, int nw, const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias,
                        const float* ln, float* h, int rows, int K, void* stream);
/* Chained log-psi layer tail (gemm_x6.hip chain_x6_kernel; D = K = 256, rows padded to 768):
 * h1 = LN1(h + X1 W1 + b1); h = LN2(h1 + tanh(h1 W2 + b2)); Y3 = h W3 + b3 when Wp3. */
int dh_debug_chain_x6(const float* X1, const uint16_t* Wp1, int ldp1, const float* b1, const float* ln1,
                      const uint16_t* Wp2, int ldp2, const float* b2, const float* ln2, const uint16_t* Wp3,
                      int ldp3, const float* b3, int n3, float* Y3, int ldy3, float* h, int rows, void* stream);

/* Fused channel GEMM + channel LayerNorm (gemm_lnch.hip; D = K = 256, N <= 6): in place over
 * h [ne * (2N + 5)][256], mode 0: h = LN_ch(h + X W + b), mode 1: h = LN_ch(h + tanh_ch(h W + b))
 * (X ignored); geo [ne][4] = (sin th, cos th, sin ph, cos ph) of the walkers' electrons. */
int dh_debug_gemm_lnch(int N, int mode, const float* X, const uint16_t* Wp, int ldp, const float* bias,
                       const float* ln, const float* geo, float* h, int ne, void* stream);

/* Test hooks of the split-bf16 GEMM (gemm_x6.hip): the transposed weight Wt[ncols][K]
 * is split into three bf16 planes Wp[3][ldp][K] (ldp = dh_debug_x6_plane_rows(ncols),
 * uint16 bit patterns), then Y = X Wt^T (+ bias on rows r % C == 0) (+ R) with
 * K % 32 == 0 and X holding round_up(rows, 256) rows; variant -1 = automatic. */
int dh_debug_x6_plane_rows(int ncols);
int dh_debug_split_planes(const float* Wt, int ldw, int ncols, int K, uint16_t* Wp, void* stream);
int dh_debug_gemm_x6(int variant, const float* X, int ldx, const uint16_t* Wp, int ldp, const float* bias,
                     const float* R, int ldr, float* Y, int ldy, int rows, int ncols, int K, int C, void* stream);

/* init_guess with the device RNG: theta = arccos U(-1,1), phi = U(-pi,pi). */
int dh_init_walkers(dh_handle* h, float* x, int B, uint64_t seed, int64_t walker_offset, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DEEPHALL_AMD_H */
