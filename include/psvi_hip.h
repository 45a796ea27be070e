/*
 * psvi_hip.h -- C ABI of the MI355X (gfx950) coreset-ELBO inner-loop library
 * (libpsvi_hip.so).  Plain C: no HIP, torch or C++ types, so ctypes / cgo /
 * JNI / N-API can bind it directly (binding stubs: INTEGRATION.md).
 *
 * What it replaces (reference = souravc83/Blackbox-Coresets-VI, paths relative
 * to its repo root):
 *   one inner step of PSVI.nested_step / PSVI.hyper_step, i.e.
 *     PSVI.inner_elbo                     psvi/inference/psvi_classes.py:488-511
 *       -> VILinear.forward / rsample      psvi/models/neural_net.py:155-179
 *       -> VILinearMultivariateNormal      neural_net.py:408-491
 *       -> Categorical.log_prob, .matmul(N f(v)), sum, + sum(m.kl())
 *     DifferentiableOptimizer.step         psvi/robust_higher/optim.py:152-257
 *       -> DifferentiableAdam._update      optim.py:299-367      (trainer nested)
 *     hypergrad DifferentiableAdam.step    psvi/hypergrad/diff_optimizers.py:107-154
 *       -> adam_step                       diff_optimizers.py:184-213 (trainer hyper)
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer (fp32 unless stated) owned by
 *     the caller; the library never allocates device memory inside a step
 *     (psvi_plan_create allocates its immutable work lists and the plan-owned
 *     split-K scratch of the full-cov sample phase and the LeNet activation
 *     scratch; a plan's calls must not
 *     run concurrently on different streams).
 *   - Steps are stream-ordered and asynchronous on `stream` (a hipStream_t
 *     passed as void*; NULL = default stream); no host synchronisation inside.
 *   - Return 0 on success, <0 for an invalid argument / shape (PSVI_E*),
 *     >0 for a hipError_t.  psvi_last_error() gives a thread-local message.
 *   - Parameter vectors use the reference's parameters_to_vector order:
 *       mean-field layer (in,out): [mu_W (out*in), mu_b (out), rho_W (out*in), rho_b (out)]
 *       full-cov   layer (in,out): n = out*in + out;
 *                                  [mean (n), sd (n), corr ((n-1)(n-2)/2)]
 *     corr is the packed row-major strict lower triangle of the top-left
 *     (n-1)x(n-1) block of L (neural_net.py:452-461): row r starts at r(r-1)/2.
 *   - Noise `eps` uses the reference draw order (Normal/MultivariateNormal
 *     rsample in forward order): mean-field per layer eps_W (S,out,in) then
 *     eps_b (S,out); full-cov per layer eps (S, n).  S is the GLOBAL sample
 *     count of the plan; every rank passes the full eps.
 *   - z holds int32 class ids; w holds the coreset weights N*f(v) (M floats,
 *     psvi_classes.py:505).
 *   - Scalar objective outputs (elbo_out, nll_out, kl_out) are DOUBLE device
 *     accumulators: the kernels add thousands of per-block partials into them
 *     and fp32 accumulation would bias the sum (rounding of similar-size adds
 *     into a large running total).  They are accumulated into (+=) unless a
 *     call documents that it zeroes them.
 */
#ifndef PSVI_HIP_H
#define PSVI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSVI_MAX_LAYERS 8

/* error codes (<0) */
#define PSVI_EINVAL   (-1)   /* bad descriptor / shape / pointer            */
#define PSVI_ENOSPC   (-2)   /* workspace too small                         */
#define PSVI_EUNSUP   (-3)   /* configuration not supported by the kernels  */
#define PSVI_ESTATE   (-4)   /* call not valid for this plan (family/world) */

/* model families */
#define PSVI_FAMILY_MEANFIELD 0   /* VILinear stack: logistic_regression, fn   */
#define PSVI_FAMILY_FULLCOV   1   /* VILinearMultivariateNormal stack: fn2,
                                     logistic_regression_fullcov              */
#define PSVI_FAMILY_LENET     2   /* make_lenet (neural_net.py:334-359): VIConv2d(1,6,5,p2)
                                     ReLU BatchMaxPool2d(2) VIConv2d(6,16,5) ReLU pool
                                     VILinear 400-120-84-10 (the last one ONE shared
                                     sample, mc_samples=1); u is (M,1,28,28).  The
                                     architecture is fixed: n_layers / dims of the
                                     descriptor are ignored.  Parameters: the
                                     mean-field layout per layer (conv weights in
                                     (out,in,5,5) order); eps per layer in draw order,
                                     W (S,n_w) then b (S,n_b), the last layer (n_w)
                                     then (n_b) without S.  KL on the VILinear layers
                                     only (psvi_classes.py:506-510).  Entry points:
                                     inner_step, elbo_grad, inner_loop and the
                                     mean-field phases; the plan owns the activation
                                     scratch (about S*M*7.9 KB).                  */

/* Adam variants */
#define PSVI_ADAM_HIGHER    0   /* robust_higher DifferentiableAdam (optim.py:318-367):
                                   denom = sqrt(v + 1e-8)/sqrt(bc2) + eps            */
#define PSVI_ADAM_HYPERGRAD 1   /* hypergrad adam_step (diff_optimizers.py:197-213):
                                   v += 1e-12 stored; denom = sqrt(v/bc2) + eps      */
#define PSVI_ADAM_TORCH     2   /* torch.optim.Adam (the MFVI baselines' optim_vi,
                                   baselines.py:870, 1020): denom = sqrt(v)/sqrt(bc2) + eps;
                                   not differentiable here (psvi_adam_adjoint refuses) */

typedef struct psvi_net_desc {
    int32_t n_layers;                     /* affine VI layers                     */
    int32_t dims[PSVI_MAX_LAYERS + 1];    /* dims[0] = D ... dims[n_layers] = C   */
    int32_t S;                            /* GLOBAL Monte-Carlo samples           */
    int32_t M;                            /* pseudopoints                         */
    float   prior_sd;                     /* sigma_0 (neural_net.py:61, 409)      */
} psvi_net_desc;

typedef struct psvi_adam_hp {
    float   lr;
    float   beta1;
    float   beta2;
    float   eps;
    int32_t step;      /* 1-based Adam step t (bias corrections 1 - beta^t) */
    int32_t kind;      /* PSVI_ADAM_HIGHER | PSVI_ADAM_HYPERGRAD            */
} psvi_adam_hp;

typedef struct psvi_plan psvi_plan;       /* opaque, immutable after create */

/* psvi_plan_query keys */
#define PSVI_Q_PARAM_COUNT   1  /* floats in params / adam_m / adam_v / grad          */
#define PSVI_Q_EPS_COUNT     2  /* floats of eps for all S (reference draw order)     */
#define PSVI_Q_WS_BYTES      3  /* workspace bytes for psvi_inner_step/elbo_grad      */
#define PSVI_Q_S_LOCAL       4  /* samples owned by this rank                         */
#define PSVI_Q_S_OFFSET      5  /* first global sample owned by this rank             */
#define PSVI_Q_ACC_COUNT     6  /* mean-field: floats in the all-reduced accumulator
                                   [sum_s dW | sum_s dW*eps] = 2 * sum_l n_l         */
#define PSVI_Q_ROWS_LOCAL    7  /* full-cov: x/g columns owned (sum over layers)      */
#define PSVI_Q_XSHARD_COUNT  8  /* full-cov: floats of x_shard / g_shard = S*ROWS_LOCAL */
#define PSVI_Q_XRECV_COUNT   9  /* full-cov: floats of x_recv / g_send = S_LOCAL*n_tot */
#define PSVI_Q_LOOP_WS_BYTES 10 /* workspace bytes for psvi_inner_loop                 */
#define PSVI_Q_TILED_FLOATS  11 /* floats of the tiled corr/m/v state (0: the plan has
                                   none -- it needs full-cov, world 1, S <= 128)      */
#define PSVI_Q_OUTER_WS_BYTES 12 /* workspace bytes for psvi_outer_elbo_grad          */
#define PSVI_Q_HVP_WS_BYTES  13 /* workspace bytes for psvi_hvp                       */
#define PSVI_Q_EVAL_WS_BYTES 14 /* workspace bytes for psvi_evaluate                  */
#define PSVI_Q_NET_PART_OK   15 /* full-cov: 1 if psvi_mvn_phase_net_part takes sample
                                   ranges (no per-chunk gradient slots), else 0    */

/* Create a plan for `family` over `world` ranks, this process being `rank`.
 * Samples are split in contiguous blocks; for FULLCOV at world > 1 the rows
 * of the layers' L are split in whole 64-row bands, balanced by their 64 x 64
 * tile counts over all layers (ranks own the matching mean/sd/corr rows and
 * their Adam state; a rank's rows need not be contiguous -- see
 * psvi_plan_shard_runs). */
int psvi_plan_create(int32_t family, const psvi_net_desc* d, int32_t world,
                     int32_t rank, psvi_plan** out);
int psvi_plan_destroy(psvi_plan* plan);
int psvi_plan_query(const psvi_plan* plan, int32_t key, int64_t* value);
/* rows (full-cov) and samples owned by rank `r` of the plan's world:
 * out[0] = s_offset, out[1] = s_count, out[2] = rows_total,
 * out[3 + l] = first row of layer l when the rank's rows of layer l are one
 * contiguous run (-1 when they are several), out[3 + PSVI_MAX_LAYERS + l] =
 * row count of layer l. */
int psvi_plan_shard_info(const psvi_plan* plan, int32_t r, int64_t* out);
/* The rows of rank `r` as runs, in x-shard column order (layer-major, rows
 * ascending): out[4 i .. 4 i + 3] = (layer, first row, row count, x-shard
 * column of the first row) for i < *count.  out == NULL: *count only;
 * PSVI_ENOSPC when cap < *count.  x_shard / g_shard hold [S][ROWS_LOCAL] in
 * this column order; x_recv / g_send hold, per source rank q in rank order,
 * [S_LOCAL][rows_total of q] in q's column order. */
int psvi_plan_shard_runs(const psvi_plan* plan, int32_t r, int64_t* out, int32_t cap,
                         int32_t* count);

/* ---- single-process fused step (world == 1) --------------------------------
 * One inner step = reparameterise, batched forward over (S x M), weighted NLL
 * + KL, hand-derived backward, Adam update of params/adam_m/adam_v in place.
 * elbo_out[0] (double, zeroed by the call) <- negative inner ELBO (the value
 * inner_elbo returns) at the incoming params.  eps == NULL is invalid (draw
 * it with psvi_randn, or pass the reference-order draws). */
int psvi_inner_step(const psvi_plan* plan, const float* u, const int32_t* z,
                    const float* w, const float* eps, float* params,
                    float* adam_m, float* adam_v, const psvi_adam_hp* hp,
                    double* elbo_out, void* ws, size_t ws_bytes, void* stream);

/* Same objective without the update: grad_out (PARAM_COUNT floats) <- d elbo
 * / d params, elbo_out[0] (double, zeroed by the call) <- elbo.  Used by the
 * autograd.Function boundary.  include_kl = 0 drops the KL term and its
 * gradient. */
int psvi_elbo_grad(const psvi_plan* plan, const float* u, const int32_t* z,
                   const float* w, const float* eps, const float* params,
                   int32_t include_kl, double* elbo_out, float* grad_out,
                   void* ws, size_t ws_bytes, void* stream);

/* T chained inner steps (world == 1): the loop the reference runs as
 *   for t in range(T): diffopt.step(inner_elbo(fmodel))   (psvi_classes.py:549-555)
 * with Adam steps hp->step .. hp->step + T - 1 on params/adam_m/adam_v in place.
 * elbo_out[t] (T doubles) <- negative inner ELBO before step t.  eps: the T
 * steps' noise as [T][EPS_COUNT] floats, or NULL to draw step t's noise in the
 * library with psvi_randn(seed, offset + t * round_up(EPS_COUNT, 4)).  For
 * full-cov plans each update also samples the next step's weights from the
 * updated parameters (one fused kernel when S <= 128; the separate sample
 * phase otherwise): the same numbers as T psvi_inner_step calls up to fp32
 * summation order.  ws: PSVI_Q_LOOP_WS_BYTES. */
int psvi_inner_loop(const psvi_plan* plan, const float* u, const int32_t* z,
                    const float* w, const float* eps, uint64_t seed, uint64_t offset,
                    int32_t T, float* params, float* adam_m, float* adam_v,
                    const psvi_adam_hp* hp, double* elbo_out, void* ws, size_t ws_bytes,
                    void* stream);

/* psvi_inner_loop with the loop's state kept across calls (full-cov plans with a
 * tiled state, Philox mode).  The calls of a run of inner steps split over
 * several calls repeat the first steps' fixed work -- corr / m / v into the
 * tiled layout, step 0's draw and sample -- because one call cannot know that
 * the next continues it:
 *   PSVI_LOOP_KEEP   the last step also draws (seed, offset + T * stride) and
 *                    samples the next step's weights (the fused update, as
 *                    every other step), the tiled corr / m / v stay in ws, and
 *                    the packed params / adam_m / adam_v are written as usual;
 *   PSVI_LOOP_RESUME start from that resident state when this call continues
 *                    the last KEEP call on this plan: the same ws, params,
 *                    adam_m, adam_v pointers and seed, and offset = its offset
 *                    + T * stride.  The caller asserts that nothing wrote
 *                    params / adam_m / adam_v / ws since (the Python
 *                    InnerLoopPlan checks the tensors' version counters);
 *                    otherwise -- or when the state does not match -- the call
 *                    starts cold, as psvi_inner_loop.
 * Every call drops the resident state first, so a RESUME after any other loop
 * call on the plan starts cold.  RESUME without KEEP takes the state up and
 * ends as a plain call.  Calls of T1, T2, ... steps, each resuming the last
 * and all but the last with KEEP, give the numbers of one call of T1 + T2 +
 * ... steps bit for bit (a KEEP call's last step is the fused update with the
 * next sample, as every step but the last of a call; a plain call's last step
 * writes the packed arrays directly: the same values up to fp32 rounding).
 * Other plans and eps != NULL: the flags are ignored. */
#define PSVI_LOOP_KEEP   1
#define PSVI_LOOP_RESUME 2
int psvi_inner_loop_ex(const psvi_plan* plan, const float* u, const int32_t* z,
                       const float* w, const float* eps, uint64_t seed, uint64_t offset,
                       int32_t T, float* params, float* adam_m, float* adam_v,
                       const psvi_adam_hp* hp, double* elbo_out, void* ws, size_t ws_bytes,
                       int32_t flags, void* stream);

/* ---- sharded phases (any world; the caller runs the collectives) ------------
 * MEANFIELD (sample-parallel, replicated params):
 *   acc (ACC_COUNT floats, overwritten) <- [sum_s dW | sum_s dW*eps] over this
 *   rank's samples, summed in a fixed order from per-(sample, chunk) slots
 *   (plan-owned scratch: one call on a plan at a time; bitwise reproducible),
 *   nll_out[0] += their weighted NLL;  caller
 *   all-reduces acc (sum);  update applies KL gradient + Adam identically on
 *   every rank (grad_out != NULL: write the gradient instead), kl_out[0] +=
 *   KL (nullable; count it on one rank). */
int psvi_mf_phase_accumulate(const psvi_plan* plan, const float* u,
                             const int32_t* z, const float* w, const float* eps,
                             const float* params, float* acc, double* nll_out,
                             void* stream);
int psvi_mf_phase_update(const psvi_plan* plan, const float* acc, float* params,
                         float* adam_m, float* adam_v, const psvi_adam_hp* hp,
                         double* kl_out, float* grad_out, int32_t include_kl,
                         void* stream);

/* FULLCOV (rows of L sharded, samples sharded):
 *   sample: x_shard[S][ROWS_LOCAL] <- mean + L eps for this rank's rows, all S
 *   (all_to_all: rank r sends rows s in shard q to q -> x_recv)
 *   net:    x_recv[S_LOCAL][n_tot, blocked by source rank] -> g_send (same
 *           layout) = per-sample gradients; nll_out[0] += local weighted NLL
 *   (all_to_all back -> g_shard[S][ROWS_LOCAL])
 *   update: corr/mean/sd Adam for owned rows; kl_out[0] += owned KL part.
 *           grad_out != NULL writes the gradient instead of updating. */
int psvi_mvn_phase_sample(const psvi_plan* plan, const float* eps,
                          const float* params, float* x_shard, void* stream);
int psvi_mvn_phase_net(const psvi_plan* plan, const float* u, const int32_t* z,
                       const float* w, const float* x_recv, float* g_send,
                       double* nll_out, void* stream);
/* the net phase with the next step's noise drawn in the same launch (the
 * sharded inner loop: every rank draws the whole global eps of the next step,
 * normals [0, n) of the psvi_randn stream (seed, offset) into eps_out -- the
 * same values psvi_randn writes -- split over the network kernel's workgroups
 * after their gradients; no separate draw launch).  offset % 4 == 0. */
int psvi_mvn_phase_net_draw(const psvi_plan* plan, const float* u, const int32_t* z,
                            const float* w, const float* x_recv, float* g_send,
                            double* nll_out, float* eps_out, int64_t n, uint64_t seed,
                            uint64_t offset, void* stream);
/* the net phase (with, optionally, one part of the next step's draw) for the
 * rank's local samples [s_begin, s_begin + s_count) only -- the sharded loop's
 * sample halves, whose exchanges overlap the other half's network.  The
 * buffers are the whole rank's (x_recv / g_send [source rank][S_LOCAL][rows]);
 * this launch reads and writes its samples' rows.  Draw: normals of quad range
 * part of nparts (contiguous, in order) of [0, n) into eps_out (NULL, n = 0:
 * none).  Plans whose pseudopoint chunks use per-chunk slots (not looped)
 * take whole launches only (PSVI_EUNSUP). */
int psvi_mvn_phase_net_part(const psvi_plan* plan, const float* u, const int32_t* z,
                            const float* w, const float* x_recv, float* g_send,
                            double* nll_out, int32_t s_begin, int32_t s_count, float* eps_out,
                            int64_t n, uint64_t seed, uint64_t offset, int32_t part,
                            int32_t nparts, void* stream);
int psvi_mvn_phase_update(const psvi_plan* plan, const float* eps,
                          const float* g_shard, float* params, float* adam_m,
                          float* adam_v, const psvi_adam_hp* hp, double* kl_out,
                          float* grad_out, int32_t include_kl, void* stream);
/* update (Adam) followed by the next step's sample phase from the updated
 * parameters: x_next[S][ROWS_LOCAL] <- mean' + L' eps_next for this rank's
 * rows.  One fused kernel when the plan allows (world == 1, S <= 128). */
int psvi_mvn_phase_update_sample(const psvi_plan* plan, const float* eps,
                                 const float* g_shard, float* params, float* adam_m,
                                 float* adam_v, const psvi_adam_hp* hp, double* kl_out,
                                 int32_t include_kl, const float* eps_next,
                                 float* x_next, void* stream);

/* Tiled corr / m / v state for a run of inner steps (full-cov, world 1,
 * S <= 128): the packed triangles re-laid as 64x64 tiles in the update
 * kernel's fragment order, so every corr/m/v access is a contiguous 1 KB
 * wave transaction (the packed rows' scattered 256-byte runs stream at about
 * two thirds of that rate).  tstate: PSVI_Q_TILED_FLOATS floats.
 * to_tiled = 1 copies the corr parts of params / adam_m / adam_v in; 0 copies
 * them back (the mean / sd parts always stay in params / adam_m / adam_v).
 * psvi_inner_loop does this itself. */
int psvi_mvn_tiled_convert(const psvi_plan* plan, float* params, float* adam_m,
                           float* adam_v, float* tstate, int32_t to_tiled, void* stream);
/* psvi_mvn_phase_update with corr and its Adam state in tstate (mean / sd
 * and theirs stay in params / adam_m / adam_v; the packed corr parts are
 * neither read nor written until psvi_mvn_tiled_convert(..., 0)); with
 * eps_next / x_next also the next step's sample (fused). */
int psvi_mvn_phase_update_tiled(const psvi_plan* plan, const float* eps,
                                const float* g_shard, float* params, float* adam_m,
                                float* adam_v, float* tstate, const psvi_adam_hp* hp,
                                double* kl_out, int32_t include_kl,
                                const float* eps_next, float* x_next, void* stream);

/* ---- outer objective ------------------------------------------------------
 * PSVI.psvi_elbo (psvi/inference/psvi_classes.py:445-486) with the sampled KL
 * of every layer (VIMixin.sampled_nkl, psvi/models/neural_net.py:110-115;
 * MultivariateNormalVIMixin.sampled_nkl, neural_net.py:438-442), world == 1,
 * 2 <= S <= 2048.  The plan's M counts ALL rows of the batch: x_all
 * ([M][D]) = cat(u, xbatch) with the n_pseudo pseudopoints first, z_all their
 * class ids, w_all the row weights -- N f(v)_m for the pseudopoints, N / Nx
 * for the data rows -- and eps the draw order of model(all_data).
 *   loss_out[0] (double, written) <- sum_s W_s (data_s - pseudo_s) - mean_s lw_s,
 *       lw_s = -pseudo_s + nkl_s, W = softmax_s(lw)
 *   grad_params (PARAM_COUNT, nullable) <- d loss / d params (first order)
 *   grad_u ([n_pseudo][D], nullable; needs grad_params) <- d loss / d u
 *   grad_w (n_pseudo, nullable) <- d loss / d w_m (chain to v / alpha on the host)
 *   sample_out ([S][4] doubles, nullable) <- pseudo_s, data_s, nkl_s, W_s
 * The sampled KL uses L^-1 (x_s - mean) = eps_s (the reference's fp32
 * triangular solve overflows at fn2 sizes).  ws: PSVI_Q_OUTER_WS_BYTES. */
int psvi_outer_elbo_grad(const psvi_plan* plan, int32_t n_pseudo, const float* x_all,
                         const int32_t* z_all, const float* w_all, const float* eps,
                         const float* params, double* loss_out, float* grad_params,
                         float* grad_u, float* grad_w, double* sample_out, void* ws,
                         size_t ws_bytes, void* stream);

/* PSVI_Ablated.psvi_elbo (psvi/inference/psvi_classes.py:1397-1408; also
 * PSVI_No_IW's, 1411): the outer objective without importance weighting,
 * over the data batch only (x_all = xbatch, the plan's M = Nx rows, w_all =
 * N / Nx each; no pseudopoints), 1 <= S <= 2048:
 *   loss_out[0] (double, written) <- mean_s data_s - mean_s nkl_s,
 *       data_s = sum_m w_m NLL_sm, nkl_s the sampled KL of the VILinear
 *       layers (every mean-field layer; LeNet's three linear layers)
 *   grad_params (PARAM_COUNT, nullable) <- d loss / d params (first order)
 *   sample_out ([S][4] doubles, nullable) <- 0, data_s, nkl_s, 1/S
 * A full-covariance plan returns PSVI_EUNSUP: the reference's sum over
 * VILinear modules is then the int 0 and 0.mean() raises.
 * ws: PSVI_Q_OUTER_WS_BYTES. */
int psvi_outer_ablated_elbo_grad(const psvi_plan* plan, const float* x_all,
                                 const int32_t* z_all, const float* w_all, const float* eps,
                                 const float* params, double* loss_out, float* grad_params,
                                 double* sample_out, void* ws, size_t ws_bytes, void* stream);

/* The backward half of psvi_outer_elbo_grad with caller-given per-sample
 * coefficients instead of the plan's own softmax over its S samples
 * (replaces the autograd backward of PSVI.psvi_elbo, psvi_classes.py:463-486,
 * when the samples are split over ranks):
 *   coef = [rowcoef (S x 2): d loss / d pseudo_s, d loss / d data_s |
 *           ck (S): d loss / d nkl_s | sck (1): the sum of ck over these samples]
 * (floats, device).  For the sample-sharded outer objective:
 * each rank runs psvi_outer_elbo_grad on a plan of its own samples for the
 * per-sample terms (sample_out), the host forms the softmax over ALL samples
 * (psvi.runtime.sharded.ShardedOuter), and each rank's grad_params / grad_u /
 * grad_w from this call are partial sums over its samples (sum over ranks).
 * S may be 1 here.  ws: PSVI_Q_OUTER_WS_BYTES. */
int psvi_outer_elbo_grad_coef(const psvi_plan* plan, int32_t n_pseudo, const float* x_all,
                              const int32_t* z_all, const float* w_all, const float* eps,
                              const float* params, const float* coef, float* grad_params,
                              float* grad_u, float* grad_w, void* ws, size_t ws_bytes,
                              void* stream);

/* Importance-weighted predictive evaluation of one test batch: PSVI.evaluate
 * (psvi_classes.py:1031-1108) and pred_on_grid (1130-1175), world == 1,
 * 2 <= S <= 2048.  Rows as psvi_outer_elbo_grad: x_all = cat(u, xtest), the
 * n_pseudo pseudopoints first; z_all their labels (test labels after);
 * w_all: N f(v) for the pseudopoints (the data rows' entries are unused).
 * Weights W = softmax_s(+sum_m w_m NLL_sm + sampled_nkl_s) -- the reference's
 * sign there (its pseudo_nll is the log-likelihood); correction = 0: W = 1/S.
 *   probs_out ([M - n_pseudo][C], nullable) <- sum_s W_s softmax(logits_s)
 *   stats_out[4] (double, written) <- entropy of W (over W > 0), normalised
 *     ESS (sum W)^2 / sum W^2 / S, correct predictions, summed test NLL
 *     (-log of the normalised probability of the label, clamped to fp32 eps).
 * ws: PSVI_Q_EVAL_WS_BYTES. */
int psvi_evaluate(const psvi_plan* plan, int32_t n_pseudo, const float* x_all,
                  const int32_t* z_all, const float* w_all, const float* eps,
                  const float* params, int32_t correction, float* probs_out,
                  double* stats_out, void* ws, size_t ws_bytes, void* stream);

/* ---- second order (the `hyper` trainer's implicit hypergradient) ----------
 * Hessian-vector product of the negative inner ELBO (psvi_inner_step's
 * objective, KL included) at fixed eps, world == 1:
 *   hv_out (PARAM_COUNT) <- H vec
 *   du_out ([M][D], nullable) <- d/du (vec . d elbo / d params)
 *   dw_out (M, nullable)      <- d/dw (vec . d elbo / d params)
 * -- the products hypergrad's CG_normaleq takes from autograd through
 * GradientDescent's fp_map (psvi/hypergrad/hypergradients.py:199-244, 300-311,
 * diff_optimizers.py:51-60; PSVI.hyper_step psvi_classes.py:602-687):
 * J^T x = x - lr H x, J x = x - lr H x (jvp), torch_grad(w_mapped, hparams, v)
 * = -lr (du_out, dw_out chained to v).  Forward-over-reverse (R-op) through
 * the per-sample network, one workgroup per sample (the model's per-sample
 * weights and row chunks in LDS; PSVI_EUNSUP when they do not fit).
 * ws: PSVI_Q_HVP_WS_BYTES. */
int psvi_hvp(const psvi_plan* plan, const float* u, const int32_t* z, const float* w,
             const float* eps, const float* params, const float* vec, float* hv_out,
             float* du_out, float* dw_out, void* ws, size_t ws_bytes, void* stream);

/* psvi_hvp over this plan's samples only, for the sample-sharded second-order
 * trainers (PSVI.hyper_step's CG_normaleq products and PSVI.nested_step's
 * reverse pass, psvi/hypergrad/hypergradients.py:199-244, 300-311;
 * psvi_classes.py:541-687, split over ranks): each rank runs it on a world-1
 * plan of its own samples with its slice of the global eps; include_kl = 1 on
 * exactly one rank adds the KL Hessian (sample-independent), 0 leaves it out,
 * so hv_out / du_out / dw_out summed over ranks (one all-reduce) equal
 * psvi_hvp over all S samples.  psvi_hvp == psvi_hvp_partial(include_kl = 1). */
int psvi_hvp_partial(const psvi_plan* plan, const float* u, const int32_t* z, const float* w,
                     const float* eps, const float* params, const float* vec,
                     int32_t include_kl, float* hv_out, float* du_out, float* dw_out, void* ws,
                     size_t ws_bytes, void* stream);

/* Reverse of one Adam step (either variant) for the nested trainer's
 * reverse-mode pass through the unrolled inner loop (PSVI.nested_step,
 * psvi_classes.py:541-600; DifferentiableAdam._update optim.py:318-367 /
 * adam_step diff_optimizers.py:184-213).  The step took (p, m, v, grad) to
 * (p', adam_m, adam_v) with Adam step hp->step; given lt = adjoint of p' and
 * lm / lv = adjoints of (adam_m, adam_v) (in/out: replaced by the adjoints of
 * the step's incoming m, v), writes lg_out = adjoint of grad.  The adjoint of
 * p is lt + H^T lg_out (psvi_hvp at p). */
int psvi_adam_adjoint(int64_t n, const float* lt, float* lm, float* lv, const float* adam_m,
                      const float* adam_v, const float* grad, float* lg_out,
                      const psvi_adam_hp* hp, void* stream);

/* ---- utilities ----------------------------------------------------------- */
/* out[i] ~ N(0,1), Philox4x32-10 counter (seed, offset + i) + Box-Muller.
 * Throughput-mode replacement for torch's normal_() draw (not bit-identical
 * to torch's generator; parity mode passes torch-drawn eps instead). */
int psvi_randn(float* out, int64_t n, uint64_t seed, uint64_t offset, void* stream);
/* flag[0] |= 1 when any of the n values at data (dtype 0: float, 1: double;
 * device) is NaN or +-inf; flag is a caller-zeroed device int32.  The HIP
 * path's stand-in for torch.autograd.set_detect_anomaly, which the reference
 * driver turns on (psvi/experiments/flow_psvi.py:50): PSVI's trainers check
 * their ELBO / loss / gradient buffers with it and read the flag once per
 * outer step when anomaly detection is enabled. */
int psvi_nonfinite(const void* data, int64_t n, int32_t dtype, int32_t* flag, void* stream);
/* Generic fused Adam over n floats (either variant). */
int psvi_adam_update(int64_t n, float* params, const float* grad, float* adam_m,
                     float* adam_v, const psvi_adam_hp* hp, void* stream);

/* ---- hyper_step's conjugate-gradient iteration (CG_normaleq) ----
 * Replaces the vector work of one iteration of the reference's
 * psvi/hypergrad/CG_torch.py:21-43 cg() over hypergradients.py:217-230's
 * normal-equation operator A(p) = vmj - J vmj, vmj = lr H_A p, J y = y - lr
 * H_B y, given the two fp32 Hessian-vector products hv1 = H_A p (from p32)
 * and hv2 = H_B vmj32 (psvi_hvp):
 *   psvi_cg_scale:    vmj32 = float(lr hv1)  (hv2's input)
 *   psvi_cg_pap:      state[1] = p . A p
 *   psvi_cg_residual: alpha = state[0] / state[1]; r -= alpha A p; state[2] =
 *                     r . r; done (state[3]) |= sqrt(state[2]) < tol; the step
 *                     length for x (state[4]: 0 once done), beta (state[5]),
 *                     and rTr (state[0]) unless done
 *   psvi_cg_update:   x += state[4] p; unless done p = r + beta p, p32 = float(p)
 * state: 7 float64 on the device, [0] = r . r and the rest 0 on entry to the
 * first iteration; x = 0, r = p = b (float64), p32 = float(b).  Where the
 * reference breaks, x keeps its last iterate and p freezes (the step length
 * is selected, never multiplied by a non-finite alpha); the caller reads
 * state[3] when it wants to stop.  ws: psvi_cg_ws_bytes() bytes, zeroed once
 * (the grid sums leave their counter at 0).  The sums are deterministic. */
size_t psvi_cg_ws_bytes(void);
int psvi_cg_scale(int64_t n, const float* hv, double lr, float* out, void* stream);
int psvi_cg_pap(int64_t n, const float* hv1, const float* hv2, double lr, const double* p,
                double* state, void* ws, size_t ws_bytes, void* stream);
int psvi_cg_residual(int64_t n, const float* hv1, const float* hv2, double lr, double* r,
                     double* state, double tol, void* ws, size_t ws_bytes, void* stream);
int psvi_cg_update(int64_t n, double* x, double* p, float* p32, const double* r,
                   const double* state, void* stream);

const char* psvi_last_error(void);
const char* psvi_version(void);

/* Diagnostics (ablation masks, A/B switches, per-phase stamps:
   psvi_debug_set / psvi_debug_set_ptr / psvi_debug_loop_timing) are exported
   for profiling tools but are not part of this interface: they are declared
   in the library's internal header csrc/psvi_diag.h. */

#ifdef __cplusplus
}
#endif
#endif /* PSVI_HIP_H */
