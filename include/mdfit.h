/*
 * mdfit.h — C-ABI of the MI355X-native per-TaxID ancient-DNA damage-fit engine.
 *
 * This is the drop-in boundary for the hot path of metadamage's fits.py
 * (reference: /root/reference/metadamage/fits.py).  The reference has no FFI;
 * its operator boundary is the per-taxon numpyro call chain
 *
 *     fit_single_group_without_timeout(group, cfg, ...)   fits.py:428-469
 *       group_to_numpyro_data                              fits.py:398-419
 *       fit_mcmc(mcmc_PMD / mcmc_null, data)               fits.py:382-387, 438-439
 *       compute_fit_results                                fits.py:230-295
 *         add_assymetry_results_to_fit_results             fits.py:298-356
 *         add_noise_estimates                              fits.py:359-376
 *
 * dispatched by compute_fits (fits.py:709-730).  mdfit_fit_batch replaces the
 * whole chain for a batch of taxa in one stream-ordered launch: one call per
 * device, outputs in input order (so the reference's reorder step,
 * fits.py:422-425, is a no-op).
 *
 * Conventions
 *  - Every pointer argument of mdfit_fit_batch is a DEVICE pointer (HBM); the
 *    caller owns all buffers (PyTorch tensors in the Python host).  The library
 *    allocates no persistent device memory.
 *  - The call is asynchronous on `hip_stream` (a hipStream_t, NULL = default
 *    stream) and never synchronises the host.
 *  - Return value: 0 on success, otherwise a negative MDFIT_E* code or a
 *    positive hipError_t; mdfit_last_error() gives a message (thread-local).
 *  - Per-taxon failures are reported in status[] and never abort the batch.
 */
#ifndef MDFIT_H
#define MDFIT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDFIT_ABI_VERSION 2

/* Dense count layout: one row of MDFIT_LD uint32 per taxon.
 * Column i < 15 is forward position z = i+1 (y = CT, N = C by default);
 * column 15 <= i < 30 is reverse position z = -(i-14) (y = GA, N = G).
 * Columns 30, 31 are padding (ignored).  This is group_to_numpyro_data
 * (fits.py:398-419) packed for a whole batch. */
#define MDFIT_NPOS 30
#define MDFIT_NHALF 15
#define MDFIT_LD 32

/* Mismatch counts for the noise estimate (fits.py:359-376): uint32
 * mm[T][30][12], columns in the reference order AC AG AT CA CG CT GA GC GT TA TC TG. */
#define MDFIT_NMM 12

/* Fit modes. */
#define MDFIT_MODE_MAP 0  /* maximum a posteriori of model_PMD / model_null (fits.py:43-67) */
#define MDFIT_MODE_NUTS 1 /* NUTS posterior sampling as fits.py:382-387 (MDFIT-NUTS v1) */

/* Per-taxon status codes (status[t]). */
#define MDFIT_OK 0
#define MDFIT_MAXITER 1   /* a sub-fit hit max_iter before converging */
#define MDFIT_NONFINITE 2 /* non-finite objective at the returned point */
#define MDFIT_INVALID 3   /* invalid input (y > N somewhere) */

/* Error codes (return values). */
#define MDFIT_E_ARG (-1)
#define MDFIT_E_HIP (-2)

/* Output record: double out[T][MDFIT_NOUT].  Fields 0..24 are the numeric
 * columns of fit_results (fits.py:244-293, 317-356, 374-376) in the reference
 * column order; the rest are per-sub-fit diagnostics. */
enum mdfit_field {
  MDFIT_F_D_MAX = 0,
  MDFIT_F_N_SIGMA,
  MDFIT_F_D_MAX_LOWER_HPDI,
  MDFIT_F_D_MAX_UPPER_HPDI,
  MDFIT_F_Q_MEAN,
  MDFIT_F_CONCENTRATION_MEAN,
  MDFIT_F_D_MAX_MARGINALIZED_MEAN,
  MDFIT_F_N_Z1_FORWARD,
  MDFIT_F_N_Z1_REVERSE,
  MDFIT_F_N_SUM_FORWARD,
  MDFIT_F_N_SUM_REVERSE,
  MDFIT_F_N_SUM_TOTAL,
  MDFIT_F_Y_SUM_FORWARD,
  MDFIT_F_Y_SUM_REVERSE,
  MDFIT_F_Y_SUM_TOTAL,
  MDFIT_F_N_SIGMA_FORWARD,
  MDFIT_F_D_MAX_FORWARD,
  MDFIT_F_Q_MEAN_FORWARD,
  MDFIT_F_N_SIGMA_REVERSE,
  MDFIT_F_D_MAX_REVERSE,
  MDFIT_F_Q_MEAN_REVERSE,
  MDFIT_F_ASYMMETRY,
  MDFIT_F_NORMALIZED_NOISE,
  MDFIT_F_NORMALIZED_NOISE_FORWARD,
  MDFIT_F_NORMALIZED_NOISE_REVERSE,
  MDFIT_NRESULT, /* = 25 result columns */
  /* diagnostics: sub-fit k in {0 PMD-all, 1 null-all, 2 PMD-fwd, 3 PMD-rev,
   * 4 null-fwd, 5 null-rev} occupies MDFIT_F_DIAG + 8*k + {q, A, c, phi,
   * objective, evaluations, status, polished}.  Null sub-fits store A = c = 0.
   * MAP: `polished` = 1 when the fit entered its polish phase (DESIGN.md
   * §3.4); its objective is then the cancellation-free form (the full log-pmf,
   * log C(N,y) included), else the lnGamma-sum form.  After the MDFIT-MAP
 * v1.1 quadratic-contraction stop the returned point is u + d
 * (the last Newton step taken without evaluating its end) while `objective`
 * holds F at the last EVALUATED point u: it exceeds F(u + d) by O(|g.d|) <=
 * ~1e-9 relative (the oracle stores the same).  NUTS: {posterior means
   * of q, A, c, phi, adapted step size, leapfrogs per draw, status,
   * divergences}. */
  MDFIT_F_DIAG = 32,
  MDFIT_NOUT = 80
};

#define MDFIT_NSUBFIT 6
#define MDFIT_DIAG_STRIDE 8

/* Prediction record: float pred[T][3][30] = (median, hdpi_lower, hdpi_upper)
 * per position, the payload of fit_predictions (fits.py:632-665). */
#define MDFIT_NPRED 3

typedef struct mdfit_opts {
  int32_t mode;       /* MDFIT_MODE_MAP or MDFIT_MODE_NUTS */
  int32_t max_iter;   /* MAP: objective evaluations per sub-fit (default 200) */
  double tol_step;    /* MAP: convergence, max |Newton step| in unconstrained units (default 1e-9) */
  uint64_t seed;      /* NUTS: key of the Philox streams (default 0, the reference's Key(0)) */
  int32_t num_warmup; /* NUTS: adaptation iterations (default 500, fits.py:792-799) */
  int32_t num_samples;/* NUTS: kept iterations (default 1000) */
  int64_t index_base; /* NUTS: global index of taxon 0 of this call -- the random streams are keyed
                         by it, so a sharded run draws the same numbers as one call (default 0) */
} mdfit_opts;

/* Fill `opts` with defaults. */
void mdfit_default_opts(mdfit_opts* opts);

/*
 * Fit a batch of taxa.
 *   y, N      : const uint32_t[n_taxa][MDFIT_LD]           (device)
 *   mm        : const uint32_t[n_taxa][30][MDFIT_NMM] or NULL (device; NULL -> noise columns NaN)
 *   out       : double[n_taxa][MDFIT_NOUT]                  (device)
 *   pred      : float[n_taxa][MDFIT_NPRED][MDFIT_NPOS] or NULL (device)
 *   status    : int32_t[n_taxa]                             (device)
 *   workspace : device buffer of mdfit_workspace_bytes(n_taxa) bytes (work
 *               queues, the PMD-all mode for the HPDI, the wide-window list:
 *               MAP 256 B + 48 B per taxon below 60k taxa, + 4,800 B more
 *               per taxon from 60k (160 B per position's wide-window record),
 *               + the HPDI stream's defer list: min(120 B per taxon, 512 KB);
 *               NUTS 256 B + 6 x num_samples x 32 B per taxon, the draws)
 *   hip_stream: hipStream_t or NULL.  MAP: parts of the call run on two
 *               library-owned side streams (one set per device, created once),
 *               forked from and joined back into hip_stream by events on every
 *               return path, so the call stays ordered on hip_stream and
 *               capturable in a graph: below 60k taxa the early HPDI launch
 *               beside the fit kernel and the late HPDI launch beside the
 *               record assembly (which follows the fit on hip_stream); from
 *               60k taxa the record assembly beside the HPDI launches (which
 *               stay on hip_stream).  MAP below 60k taxa: the predictive
 *               HPDI kernel runs beside the fit kernel and waits for modes
 *               the fit kernel's waves publish (relaxed, order-free: each
 *               field of a ready-list entry is written once as the bit
 *               complement of its value into a list the call zeroed, and an
 *               entry is taken when every field reads non-zero -- no fence,
 *               DESIGN.md §4); the two grids are sized to be co-resident on
 *               an otherwise idle device.
 *               The waits are bounded: a wave that makes no progress for 1 ms
 *               hands its items to the HPDI launch after the fit and exits, so
 *               concurrent calls or other kernels on the device (e.g. an RCCL
 *               collective) cost time, never a hang.  Fastest when calls on
 *               one device run one after another.
 *   n_taxa    : at most 2^25 per call (MAP: int32 position indices)
 * Replaces compute_fits' per-taxon loop (fits.py:477-526, 569-626, 709-730).
 */
int mdfit_fit_batch(const uint32_t* y, const uint32_t* N, const uint32_t* mm,
                    int64_t n_taxa, const mdfit_opts* opts, double* out,
                    float* pred, int32_t* status, void* workspace,
                    void* hip_stream);

/* Bytes of device workspace mdfit_fit_batch needs for n_taxa taxa under
 * `opts` (NULL = defaults; NUTS keeps every chain's samples there:
 * 6 x num_samples x 4 doubles per taxon). */
int64_t mdfit_workspace_bytes(int64_t n_taxa, const mdfit_opts* opts);

/*
 * Noise columns of records fitted with mm = NULL (both modes): the three
 * normalized_noise columns of out[n_taxa][MDFIT_NOUT] from the mismatch counts
 * mm[n_taxa][30][12] (add_noise_estimates, fits.py:359-376) -- the values a
 * call with mm writes, bit for bit; taxa with y > N (status 3, NaN record) are
 * left alone.  Device pointers, stream-ordered.  Lets a host ship the 1,440 B
 * per taxon of mismatch counts while the fit runs (engine.ChunkedFitter).
 */
int mdfit_noise(const uint32_t* y, const uint32_t* N, const uint32_t* mm, int64_t n_taxa, double* out,
                void* hip_stream);

/*
 * Pointwise beta-binomial log-pmf (numpyro BetaBinomial.log_prob, used by
 * fits.py:59,67 and log_likelihood fits.py:126-133):
 *   out[i] = log C(N,y) + lnB(y+alpha, N-y+beta) - lnB(alpha, beta)
 * plus d/dalpha, d/dbeta (grad[i][2]).  Device pointers; for parity tests.
 * The value is computed in the cancellation-free form the record assembly
 * uses for its pointwise log-likelihoods (rising-factorial ratios).
 */
int mdfit_betabinom_logpmf(const double* y, const double* N, const double* alpha,
                           const double* beta, int64_t n, double* out,
                           double* grad, void* hip_stream);

/*
 * Device special functions on an array (parity tests): out[i] =
 * (lgamma(x), digamma(x), trigamma(x)) for x[i] > 0.  Device pointers.
 */
int mdfit_special(const double* x, int64_t n, double* out3, void* hip_stream);

/*
 * Test helper: fills every CU's LDS with NaN (one launch of blocks holding the
 * largest LDS a block may take, several per CU), so that a kernel launched after
 * it on the stream that reads LDS it did not write sees NaN there.  The library's
 * kernels never do; tests/test_gpu_paths.py checks that records are bit-identical
 * after a poisoning.
 */
int mdfit_poison_lds(void* hip_stream);

/*
 * MAP predictive HPDI (MDFIT-HPDI v2): the 68 % highest-
 * probability window [lo, hi] (integer counts, returned as double) of
 * BetaBinomial(alpha, beta, N), the population form of numpyro's
 * hpdi(obs/N, 0.68) over predictive draws (fits.py:112-120, 260-261).  The
 * fit's D_max_{lower,upper}_hpdi and the pred bounds are lo/N, hi/N at the
 * PMD-all mode.  Device pointers; N[i] = 0 -> NaN.  For parity tests.
 */
int mdfit_hpdi68(const double* N, const double* alpha, const double* beta, int64_t n, double* lo,
                 double* hi, void* hip_stream);

/*
 * Objective of one sub-fit at given unconstrained parameters, evaluated by
 * the fit kernel's own lane layout and code (parity tests).  Per item i:
 * model[i] (0 PMD, 1 null), subset[i] (0 all, 1 forward, 2 reverse),
 * y/N rows [n][MDFIT_LD], u[n][4] = (logit q, logit A, c, log delta) -- c on
 * its own scale (MDFIT-MAP v1; the sampler uses logit c).
 * Outputs F[n] = -(sum ell + log prior), g[n][4], H[n][4][4] (d/du),
 * ell[n][30] (pointwise log-lik without log C(N,y); 0 outside the subset).
 */
int mdfit_objective(const int32_t* model, const int32_t* subset, const uint32_t* y,
                    const uint32_t* N, const double* u, int64_t n, double* F, double* g,
                    double* H, double* ell, void* hip_stream);

/*
 * Register-only throughput probe of the per-point evaluation the fit kernel
 * runs (value + gradient + Hessian of one beta-binomial point): launches
 * `n_waves` waves that each do `iters` evaluations; `sink` is a device
 * double[n_waves*64].  Used by bench.py for the compute roofline.
 */
int mdfit_peak_probe(int64_t n_waves, int32_t iters, double* sink, void* hip_stream);

/*
 * The same for the sampling mode: the chain kernel's potential evaluation
 * (value + gradient of 15 beta-binomial points per 16-lane chain slot, the
 * unconstrained transform, the row sums) at the chain kernel's occupancy;
 * 60 point-evaluations per wave-iteration.  bench.py's NUTS compute roofline.
 */
int mdfit_nuts_peak_probe(int64_t n_waves, int32_t iters, double* sink, void* hip_stream);

/*
 * Sampling-mode potential -(log density + log|J|) and its gradient in the
 * unconstrained v = (logit q, logit A, logit c, log delta) (numpyro's
 * potential of model_PMD / model_null, fits.py:43-67), evaluated by the chain
 * kernel's own lane layout and code (parity tests).  Per item i: model[i]
 * (0 PMD, 1 null), subset[i] (0 all, 1 forward, 2 reverse), y/N rows
 * [n][MDFIT_LD], v[n][4] -> U[n], g[n][4]; infeasible -> U = +inf, g = 0.
 */
int mdfit_nuts_potential(const int32_t* model, const int32_t* subset, const uint32_t* y,
                         const uint32_t* N, const double* v, int64_t n, double* U, double* g,
                         void* hip_stream);

/* Profiling hooks (bench / roofline): while enabled, every mdfit_fit_batch
 * records HIP events on its stream around the whole call and around the fit
 * kernel (up to 256 calls); on = 2 records only the two events around the fit
 * kernel (call_ms then reads -1).  mdfit_profile_read synchronises on them and
 * returns the summed milliseconds and the number of calls, then resets. */
int mdfit_profile_enable(int on);
int mdfit_profile_read(double* call_ms, double* fit_ms, int32_t* n_calls);

const char* mdfit_last_error(void);
int mdfit_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MDFIT_H */
