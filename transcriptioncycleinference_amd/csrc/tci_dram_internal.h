// tci_dram_internal.h -- device state of the GPU-resident batched DRAM sampler.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "tci.h"
#include "tci_internal.h"

namespace tci {

// Optional device time per kernel class (tci_dram_options.kernel_times): a HIP event pair around each
// launch of the fused / walk engines, on the launch stream, summed after the run's final
// synchronisation. Classes: 0 the draws pass (k_draws), 1 the chain walk (k_chain / k_walk), 2 the
// covariance adaptation (k_adapt_*), 3 the split draws' first chunk (k_draws_rng; the later chunks'
// are drawn inside the k_chain launches, class 1).
struct LaunchTimer {
  static constexpr int kClasses = 4;
  struct Mark {
    int cls;
    hipEvent_t a, b;
  };
  std::vector<Mark> marks;
  hipEvent_t open = nullptr;
  void begin(hipStream_t s) {
    if (hipEventCreate(&open) == hipSuccess) (void)hipEventRecord(open, s);
    else open = nullptr;
  }
  void end(int cls, hipStream_t s) {
    hipEvent_t e = nullptr;
    if (open && hipEventCreate(&e) == hipSuccess) {
      (void)hipEventRecord(e, s);
      marks.push_back({cls, open, e});
    } else if (open) {
      (void)hipEventDestroy(open);
    }
    open = nullptr;
  }
  // after the stream is synchronised: total ms and launches per class; releases the events
  void collect(double* ms, int64_t* launches) {
    for (Mark& m : marks) {
      float t = 0.f;
      if (hipEventElapsedTime(&t, m.a, m.b) == hipSuccess) {
        ms[m.cls] += t;
        launches[m.cls] += 1;
      }
      (void)hipEventDestroy(m.a);
      (void)hipEventDestroy(m.b);
    }
    marks.clear();
  }
  ~LaunchTimer() {
    for (Mark& m : marks) {
      (void)hipEventDestroy(m.a);
      (void)hipEventDestroy(m.b);
    }
  }
};

// One workgroup (256 threads) per chain. All arrays are indexed by chain c; vectors have stride ld (= max parameter count P_max),
// matrices stride ld*ld (row-major, P_c x P_c used).
// Doubles per chain of DramState::Rd: the packed triangle ld(ld+1)/2 rounded up to 128 doubles, so a
// chain's triangle starts 1 KiB-aligned and is copied to LDS in whole 1 KiB pieces (k_draws).
constexpr int64_t dram_tri_stride(int64_t ld) { return (ld * (ld + 1) / 2 + 127) / 128 * 128; }
// Doubles per chain of DramState::cov: the ld x ld matrix (k_adapt_gt), or k_adapt_mfma's owned-tile
// layout (the NT (NT + 1) / 2 upper 16 x 16 tiles of 256 doubles, NT = ceil(ld / 16)), whichever is larger.
constexpr int64_t dram_cov_stride(int64_t ld) {
  return ld * ld > (ld + 15) / 16 * ((ld + 15) / 16 + 1) / 2 * 256 ? ld * ld : (ld + 15) / 16 * ((ld + 15) / 16 + 1) / 2 * 256;
}

// The fused engines' draws buffer: at most this many GiB (sets the chunk length). 4 GiB holds a whole
// 100-step window of configs 4/5's 10,000 chains (2 GiB split it into two 50-step chunks, whose
// second draws pass filled 36 of its 64 rows): config 4 127.5 -> 123.8 us per step, config 5 135.8
// -> 131.9, bitwise equal (r05dg; round 4's 8 GiB test predates the short-pass draws and measured
// within noise, r04s).
constexpr int64_t kDrawsGiB = 4;
// Rows longer than this adapt with k_adapt_gt (tiles in global memory); k_adapt_mfma<8, 13, 12> up to
// here (k_adapt_gt at config 4's P = 207: 5,207 -> 5,887 us, r04q).
constexpr int64_t kAdaptGtFrom = 208;

struct DramState {
  int64_t n_chains;
  int64_t ld;
  const int32_t* cell;     // chain -> cell of the context
  const int64_t* key;      // chain -> RNG stream key (tci_dram_options.chain_keys; identity when absent)
  const int32_t* npar;     // P_c = 7 + N_c
  const int32_t* nobs;     // N = length(ydata) = 2 N_c (TranscriptionCycleMCMC.m:260)
  const double* lower;     // bounds (TranscriptionCycleMCMC.m:242-255)
  const double* upper;
  const double* pmu;       // Gaussian prior mean / sd (sd = +Inf: no prior), :254
  const double* psig;
  double* theta;           // current state
  double* ss;              // SS of the current state
  double* prior;           // prior SS of the current state
  double* sigma2;          // error variance (model.sigma2, :259)
  double* Rd;              // proposal Cholesky factor R (upper: proposal = theta + z * R) in FP64, as packed
                           // upper triangles (chain c at c * dram_tri_stride(ld)); the
                           // [ld][ld] double form is built on the host for the results only
  double* cov;             // running chain covariance (mcmcstat covupd), dram_cov_stride(ld) per chain
  double* cmean;
  double* wsum;
  double* window;          // chain rows by window slot (DramParams::win per chain): the covupd window, and
                           // every engine's per-row log (k_stats)
  double* s2log;           // s2 of each row of the window, by window slot
  double* wsumv;           // column sums of the window's rows (row order; the adaptation's batch mean); during a
                           // window that spans k_chain launches, its running sums so far with
  double* wacc1;           //   the shifted sums S1, S2 of the statistics rows (n_chains x ld)
  double* wacc2;
  double* s2acc;           //   and the s2 sums: sum, S1, S2 per chain (n_chains x 3)
  double* prop1;           // stage-1 / stage-2 proposals (n_chains x ld)
  double* prop2;
  uint8_t* act1;           // in-bounds flags (ssfun is called only for these)
  uint8_t* act2;
  uint8_t* acc1;           // stage 1 accepted this step
  double* ss1;             // SS of the proposals (+Inf when out of bounds)
  double* ss2;
  double* prior1;
  double* a12;             // stage-1 acceptance probability
  int32_t* naccept;        // accepted moves
  int32_t* nrej_win;       // rejections in the current adaptation window (burn-in scaling)
  int64_t* nevals;         // ssfun evaluations (in-bounds proposals)
  double* smean;           // posterior mean / M2 (Welford) over rows >= stats_from
  double* sm2;
  double* s2sum;           // sum of s2 and Welford of sqrt(s2) over all rows (:302-303)
  double* sq_mean;
  double* sq_m2;
  double* chain_out;       // optional thinned chain rows (n_keep x n_chains x ld) or null
  double* s2_out;          // optional thinned s2 rows
  double* work;            // Cholesky tile grid of k_adapt_gt (n_chains x gt_lt(ld)^2)
  int64_t* step;           // current chain row (1-based), advanced on device after each step
  int64_t* prof;           // TCI_CHAIN_PROFILE builds only: k_chain phase cycles, summed over chains
  double* draws;           // fused engine: per chain, p.chunk rows of draw_stride(ld) doubles (k_draws)
  uint8_t* runf;           // 1 where a window row's step moved the chain (a new run of equal rows: the
                           // adaptation scatters each run once), by window slot
};

// One chain row's state-independent draws (fused engine): u1 = z1*R [ld], u2 = z2*R [ld], then
// the scalars |z2/drscale - z1|^2, |z1|^2, the two acceptance uniforms and the unit Gamma variate.
constexpr int64_t draw_stride(int64_t ld) { return 2 * ld + 8; }

struct DramParams {
  uint64_t seed;
  int32_t ntry;
  int32_t updatesigma;
  double drscale;
  double adascale;  // <= 0: 2.4 / sqrt(P_c) per chain
  double qcovadj;
  double burnin_scale;
  int64_t adaptint;
  int64_t burnintime;
  int64_t stats_from;
  int64_t thin;
  int64_t n_keep;
  int64_t pmax;        // max parameter count over the chains, or tci_dram_options.adapt_pmax if larger (picks
                       // the adaptation kernel)
  int64_t chunk;       // fused engine: rows per chain of the draws buffer (>= the longest chunk)
  int64_t walk;        // fused engine: 1 = one wavefront per chain walks the chunk (k_walk), 0 = k_chain
  int64_t win;         // window rows per chain: adaptint, or (no adaptation) 100; the
                       // records are merged window by window (k_stats), the same partition for every engine
  int64_t split;       // k_chain's engine: the draws split in two (the state-independent ones drawn one chunk
                       // ahead by extra k_chain workgroups; k_draws multiplies by R only). Same bits.
};

int dram_launch_init(const DramState& st, const double* qcov_diag, const double* sigma2_0, void* stream);
int dram_launch_propose1(const DramState& st, const DramParams& p, void* stream);
int dram_launch_accept1(const DramState& st, const DramParams& p, void* stream);
int dram_launch_accept2(const DramState& st, const DramParams& p, void* stream);
int dram_launch_adapt(const DramState& st, const DramParams& p, void* stream,
                      LaunchTimer* timer = nullptr);  // no-op unless step % adaptint == 0
int dram_launch_step_incr(const DramState& st, void* stream);
int dram_launch_init_stats(const DramState& st, const DramParams& p, void* stream);
// Fused engine: chain rows s_begin..s_end (each chain's ssfun inside the kernel); leaves *st.step = s_end.
// with_records: s_end ends a window (or the run) -- the window's records are kept by the same kernel.
// The split draws (DramParams::split): k_chain's launch also draws the next chunk's normals and scalar
// draws (rows s_begin..s_end) into that chunk's buffer with `wgs` extra workgroups.
struct ChainNext {
  double* draws;
  int64_t s_begin, s_end;
  int wgs;
};
int dram_launch_chain(const DramState& st, const DramParams& p, const KParams& kp, int rpl, int64_t s_begin,
                      int64_t s_end, int with_records, void* stream, LaunchTimer* timer = nullptr,
                      const ChainNext* next = nullptr);
int64_t dram_chain_lds_bytes(int64_t ld, int rpl);
// Split draws (DramParams::split): the normals, q1 and scalar draws of chain rows s_begin..s_end into
// st.draws (that chunk's buffer) by `wgs` workgroups -- the first chunk's; k_chain draws the later ones
// (ChainNext). Timer class 3.
int dram_launch_draws_rng(const DramState& st, const DramParams& p, int64_t s_begin, int64_t s_end, int wgs,
                          void* stream, LaunchTimer* timer = nullptr);
int64_t dram_draws_rng_lds_bytes(int64_t ld);  // LDS per workgroup of the fused engine
// LDS of the adaptation kernel dram_launch_adapt picks for (pmax, adaptint), dynamic plus the kernel's
// static __shared__: the window's run table grows with adaptint (4 bytes per row), so tci_dram_run
// refuses an adaptint past the CU's LDS before any launch.
int64_t dram_adapt_lds_bytes(int64_t pmax, int64_t adaptint);
// The records of the window of chain rows ending at row *st.step (posterior mean / M2, window column
// sums, s2 statistics, thinned outputs) from the rows every engine logs: run after a window's last
// row (a multiple of p.win) and after the chain's last row (the batched engine; the fused engines
// keep them in the chain kernel, dram_launch_chain).
int dram_launch_stats(const DramState& st, const DramParams& p, void* stream);

}  // namespace tci
