/*
 * tci.h -- C ABI of the MI355X-native TranscriptionCycleInference likelihood path.
 *
 * Drop-in boundary: mcmcstat's model.ssfun handle, ss = ssfun(theta, data), set at
 *   /root/reference/src/TranscriptionCycleMCMC.m:186 (closure over `construct`) and :258,
 *   called by mcmcrun at :273. The handle wraps
 *   SumofSquaresFunction_TranscriptionCycleMCMC(construct,data,x)
 *   (/root/reference/src/SumofSquaresFunction_TranscriptionCycleMCMC.m:1-64), which runs
 *   ConstantElongationSim (src/dependencies/ConstantElongationSim.m:1-67) and
 *   GetFluorFromPolPos (src/GetFluorFromPolPos.m:1-71).
 *
 * The reference's FFI for this path would be a MATLAB MEX gateway; its source is
 * matlab/tci_mex.cpp and the binding is shown in INTEGRATION.md.
 *
 * Conventions: every entry point returns int status (TCI_OK = 0, negative = error) and
 * never throws; tci_last_error(ctx) gives the message. Plain pointers and sizes only.
 * A context is bound to one device and is NOT thread-safe (one context per host thread).
 * Theta layout (TranscriptionCycleMCMC.m:210, SumofSquares...m:35-42):
 *   theta = [v, tau, ton, MS2_basal, PP7_basal, A, R, dR_1 .. dR_N]   (P = 7 + N doubles)
 */
#ifndef TCI_H_
#define TCI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCI_OK 0
#define TCI_EINVAL (-1)  /* bad argument (null pointer, size, construct table) */
#define TCI_EHIP (-2)    /* HIP runtime error */
#define TCI_ENOMEM (-3)  /* host or device allocation failed */
#define TCI_EDIM (-4)    /* grid length != data length: the reference errors at
                            ConstantElongationSim.m:47 ("Matrix dimensions must agree") */
#define TCI_ERANGE (-5)  /* cell id out of range, or ld_theta < 7 + N of that cell */

#define TCI_MAX_SEG 4    /* stem-loop segments per dye (GetFluorFromPolPos.m:47 loop) */
#define TCI_MAX_POINTS 2048 /* acquisition points per cell: <= 513 run the register-resident kernels,
                               longer cells the long-cell kernel (its tables in LDS, 64 B per point) */

typedef struct tci_ctx tci_ctx;

/* Ragged struct-of-arrays cell table: cell c owns t/ms2/pp7[offsets[c] .. offsets[c+1]).
 * Replaces the per-cell data struct {xdata = time, ydata = [MS2, PP7]} built at
 * TranscriptionCycleMCMC.m:163-181 (schema README.md:11-16). NaN = missing sample.
 * Borrowed for the duration of tci_create only (copied to the device). */
typedef struct {
  int64_t n_cells;
  const int64_t* offsets; /* [n_cells + 1] */
  const double* t;
  const double* ms2;
  const double* pp7;
} tci_cells;

/* Reporter construct (GetFluorFromPolPos.m:18-30): gene length L = L0 + tau*v (kb) and,
 * per segment s, the MS2 and PP7 stem-loop start/end (kb) and loop count (fluorval =
 * loopn/24). Requirements (checked): 1 <= n_seg <= TCI_MAX_SEG, 0 <= start < end. */
typedef struct {
  double L0;
  int32_t n_seg;
  const double* ms2_start;
  const double* ms2_end;
  const double* ms2_loopn;
  const double* pp7_start;
  const double* pp7_end;
  const double* pp7_loopn;
} tci_construct;

typedef struct {
  int32_t device;
  int32_t rows_per_lane;   /* kernel variant selected from the longest cell (0: the long-cell kernel) */
  int64_t n_cells;
  int64_t max_points;
  int64_t device_bytes;    /* resident cell-table bytes in HBM */
} tci_info;

/* Fill *out with the construct named by `name`; pointers refer to static storage.
 * Only "P2P-MS2v5-LacZ-PP7v4" is built in (GetFluorFromPolPos.m:18); any other name
 * returns TCI_EINVAL, as the reference errors on an undefined construct. */
int tci_construct_by_name(const char* name, tci_construct* out);

/* Create a context on HIP device `device`: validates the cells, builds each cell's
 * uniform grid t(1):mean(diff(t)):t(end) (SumofSquares...m:29-30, MATLAB colon rule),
 * interpolation indices/weights and time steps, and uploads everything to HBM. */
int tci_create(const tci_cells* cells, const tci_construct* construct, int device, tci_ctx** out);
int tci_destroy(tci_ctx* ctx);
const char* tci_last_error(const tci_ctx* ctx);
int tci_get_info(const tci_ctx* ctx, tci_info* out);

/* Test hook. flags bit 0: run the exact sequential loading-counter scan in every evaluation
 * (normally only when the parallel scan cannot prove floor() exact); bit 1: run the exact
 * per-(row, cohort) position sweep (normally only when the uniform-grid distance table cannot
 * prove every stem-loop/gene-end comparison). 0 restores the default. */
int tci_set_force_exact_scan(tci_ctx* ctx, int flags);

/* Batched likelihood, HOST pointers, synchronous: for b in [0,B)
 *   ss_out[b] = SumofSquaresFunction_TranscriptionCycleMCMC(construct, cell[cell_id[b]], theta[b,:])
 * theta is B rows of ld_theta doubles (ld_theta >= 7 + N of the row's cell).
 * active (may be NULL = all active): rows with active[b] == 0 are skipped (mcmcstat
 * rejects out-of-bounds proposals without calling ssfun) and get ss_out[b] = +Inf.
 * Non-finite theta entries give ss_out[b] = NaN (mcmcstat treats it as a rejection). */
int tci_ss_batch(tci_ctx* ctx, const double* theta, int64_t ld_theta, const int32_t* cell_id,
                 const uint8_t* active, int64_t B, double* ss_out);

/* Same on DEVICE pointers, asynchronous on `stream` (a hipStream_t; NULL = the HIP default
 * stream, as in every HIP API). Inputs stay resident in HBM; nothing is copied or
 * synchronised. Rows whose cell id is out of range or whose ld_theta is too short get NaN. */
int tci_ss_batch_async(tci_ctx* ctx, const double* d_theta, int64_t ld_theta, const int32_t* d_cell_id,
                       const uint8_t* d_active, int64_t B, double* d_ss_out, void* stream);

/* One evaluation: the literal ssfun(theta, data) call for one cell (host pointers).
 * P must be >= 7 + N of the cell. */
int tci_ssfun(tci_ctx* ctx, int32_t cell, const double* theta, int64_t P, double* ss_out);

#define TCI_GRID_INTERP 0 /* through the uniform grid + interp1, as inside the SS
                             (SumofSquares...m:28-56) */
#define TCI_GRID_RAW 1    /* on the raw acquisition times, as the plot/summary call
                             TranscriptionCycleMCMC.m:307-309 (no grid, no interp1) */

/* Batched forward model, HOST pointers, synchronous: simulated MS2 (already x A) and
 * PP7 at the acquisition times of each row's cell. Row b writes N(cell) values at
 * ms2_out[b*ld_out] and pp7_out[b*ld_out] (ld_out >= N of the cell); NaN where the
 * grid does not cover a time (interp1 out of range). */
int tci_forward(tci_ctx* ctx, const double* theta, int64_t ld_theta, const int32_t* cell_id, int64_t B,
                int grid_mode, double* ms2_out, double* pp7_out, int64_t ld_out);

/* Number of HIP devices visible to this process (*n_out = 0 when there is none; never an error
 * for that). Lets a caller spread contexts over a node's GPUs, e.g. the reference's parfor worker k
 * (TranscriptionCycleMCMC.m:161) on device (k - 1) mod n (matlab/tci_ssfun.m). */
int tci_device_count(int* n_out);

/* Number of acquisition points of a cell, and the grid the SS uses for it (M points). */
int tci_cell_points(const tci_ctx* ctx, int32_t cell, int64_t* n_out);
int tci_cell_grid(const tci_ctx* ctx, int32_t cell, double* t_interp_out, int64_t cap, int64_t* m_out);

/* ---- GPU-resident batched DRAM: the caller of ssfun ----------------
 * mcmcrun(model, data, params, options) for many independent chains at once, one chain per
 * row (TranscriptionCycleMCMC.m:161-273): proposals, bounds rejection, delayed rejection,
 * adaptive covariance, Gaussian priors and the sigma^2 Gibbs update all run on the device; every
 * ssfun call is the batched likelihood kernel. mcmcstat is restated from its published algorithm
 * (version unpinned); MATLAB's RNG is not reproducible, so parity is statistical. */
typedef struct {
  int64_t n_steps;      /* nsimu: chain rows including the initial state (:264) */
  int64_t burnintime;   /* options.burnintime (:267): steps before covariance adaptation starts */
  int64_t adaptint;     /* options.adaptint (:268); 0 = no adaptation */
  int32_t ntry;         /* 2 = DRAM ('dram', :269), 1 = adaptive Metropolis only */
  int32_t updatesigma;  /* options.updatesigma (:265) */
  double drscale;       /* stage-2 proposal shrink (mcmcstat default 5) */
  double adascale;      /* adapted proposal scale; <= 0 = 2.4/sqrt(npar) */
  double qcovadj;       /* diagonal added before the Cholesky (1e-5) */
  double burnin_scale;  /* burn-in proposal scaling factor (10) */
  int64_t stats_from;   /* first chain row (1-based) of the posterior summaries (n_burn, :276) */
  int64_t thin;         /* keep every thin-th chain row in outputs.chain (0 = keep none) */
  uint64_t seed;
  int32_t engine;       /* TCI_DRAM_AUTO / _FUSED / _BATCHED / _WALK (below) */
  int32_t max_chunk;    /* FUSED/WALK: at most this many chain rows per draws pass + walk (0 = automatic:
                           adaptint, or the draws buffer's 2 GiB cap); same chains whatever it is */
  const int64_t* chain_keys; /* optional [n_chains]: chain c draws from RNG stream chain_keys[c]
                                (NULL: stream c). Keying chains by their global cell index makes a
                                shard of a run (its cells on one GPU) reproduce the unsharded chains */
  int64_t adapt_pmax;   /* 0, or the largest P = 7 + N over every chain of a larger fit that this run is one
                           shard of: the covariance adaptation kernel is picked by the largest P
                           (k_adapt_gt past 208), so a shard passing the whole fit's value adapts with the
                           same kernel, hence the same bits, as the unsharded fit (parallel.fit_sharded) */
  int64_t kernel_times; /* 1: time every kernel launch of the FUSED / WALK engines with HIP events on the
                           launch stream (tci_dram_outputs.kernel_ms); 0 (default): no events */
} tci_dram_options;

/* DRAM engines; all give identical chains for the same seed.
 *   FUSED:   per chunk of steps (up to the next adaptation) one wide launch draws every
 *            state-independent random quantity (proposal offsets z*R on MFMA, uniforms, Gamma
 *            variates), then one workgroup per chain walks the chunk with its ssfun evaluations in
 *            the loop (one workgroup barrier per step): latency-bound runs (few chains). The draws
 *            that do not need the adapted R (normals, uniforms, Gamma variates) are drawn on a
 *            second stream one chunk ahead, under the previous chunk's walk.
 *   BATCHED: one launch per stage, every chain's ssfun in the batched likelihood kernel, replayed
 *            as a hipGraph per adaptation window: many chains, or cells too long for FUSED.
 *   WALK:    FUSED's draws pass, then ONE WAVEFRONT per chain walks the chunk (stage 2 evaluated
 *            only after a stage-1 rejection, no workgroup barriers): many chains (configs 4/5).
 *   AUTO:    FUSED whenever its draws pass fits a CU's LDS (P <= ~225), as WALK beyond two chains
 *            per CU; BATCHED otherwise. */
#define TCI_DRAM_AUTO 0
#define TCI_DRAM_FUSED 1
#define TCI_DRAM_BATCHED 2
#define TCI_DRAM_WALK 3

/* Host buffers filled by tci_dram_run (any may be NULL). Per-chain vectors have stride ld.
 * Padding (entries j >= P = 7 + N of a chain whose row is shorter than ld): mean and std are NaN
 * (also every entry when no row is in the statistics range, stats_from > n_steps); final_theta keeps
 * theta0's padding unchanged; chain rows and qcov_R are 0 there. */
typedef struct {
  double* mean;         /* mean(chain(stats_from:end, :)) (:286-301) */
  double* std;          /* std(chain(stats_from:end, :), 1) */
  double* final_theta;  /* last chain row */
  double* sigma_mean;   /* sqrt(mean(s2chain)) over all rows (:302) */
  double* sigma_std;    /* std(sqrt(s2chain), 1) (:303) */
  double* accept_rate;  /* accepted moves / (n_steps - 1) */
  int64_t* n_evals;     /* ssfun calls: the initial one + every in-bounds proposal */
  double* chain;        /* [ceil(n_steps/thin)][n_chains][ld] thinned rows (rows 1, 1+thin, ...) */
  double* s2chain;      /* [ceil(n_steps/thin)][n_chains] */
  double* qcov_R;       /* [n_chains][ld][ld] final proposal factor R (upper): qcov = R'R (mcmcstat results.qcov) */
  double elapsed_ms;    /* device time of the step loop (HIP events) */
  double kernel_ms[4];  /* with opt.kernel_times (FUSED / WALK): device ms summed per kernel class -- [0] the
                           draws pass (k_draws), [1] the chain walk (k_chain / k_walk), [2] the covariance
                           adaptation (k_adapt_*), [3] FUSED's split draws: the normals and scalar draws
                           (k_draws_rng, on a second stream one chunk ahead, overlapping the walk) --
                           written by tci_dram_run, 0 otherwise */
  int64_t kernel_launches[4]; /* launches per class behind kernel_ms */
} tci_dram_outputs;

int tci_dram_defaults(tci_dram_options* opt);

/* Run n_chains chains; chain c evaluates cell cell_id[c] of the context. Inputs (host, n_chains x
 * ld row-major, ld >= 7 + N of every chain's cell): theta0 = x0 (:210), lower/upper = parameter
 * bounds (:242-255), prior_mu/prior_sig = Gaussian priors (sig = +Inf: none; dR: 0, 50, :254),
 * qcov_diag = the initial proposal covariance diagonal J0 (:230); sigma2_0 = model.sigma2 (:259,
 * per chain). The number of observations per chain is 2 N_c, NaNs included (:260). */
int tci_dram_run(tci_ctx* ctx, const tci_dram_options* opt, int64_t n_chains, const int32_t* cell_id,
                 const double* theta0, const double* lower, const double* upper, const double* prior_mu,
                 const double* prior_sig, const double* qcov_diag, const double* sigma2_0, int64_t ld,
                 tci_dram_outputs* out);

const char* tci_version(void);

#ifdef __cplusplus
}
#endif

#endif /* TCI_H_ */
