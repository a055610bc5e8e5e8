/*
 * insfm_ba.h -- C ABI of the MI355X-native sparse bundle-adjustment core.
 *
 * This library replaces the engine row under InstantSfM's TorchBA processor:
 *   - the per-step call  `loss = optimizer.step(input)`  of  `bae.optim.LM(model, strategy=TrustRegion(...),
 *     solver=PCG(tol=1e-5), kernel=Huber(thres), reject=30)`   (instantsfm/processors/bundle_adjustment.py:115-119, :132)
 *     -> insfm_ba_step();
 *   - the residual model `ReprojNonBatched.forward` = `reproject_funcs[model](points_3d[pi], pose[ci], pp[ci]) - points_2d`
 *     (bundle_adjustment.py:51-64, cost_function.py:32-208) and its TrackingTensor sparse Jacobian
 *     (bae.autograd.function, un-vendored)  -> fused into the library's linearize kernels;
 *   - `bae.utils.pysolvers.PCG` and the cuDSS sparse solve (un-vendored)  -> explicit Schur complement on the camera
 *     blocks + PCG kernels with the same relative-residual stopping rule; preconditioner `desc.precond`: 2 (default,
 *     the product's: TorchBA.Solve, bench.py) a camera-cluster coarse space (similarity + intrinsic modes per cluster,
 *     the build's choice) applied as an A-DEF2 deflation on top of block-Jacobi, 1 = the same coarse space as an
 *     additive correction, 0 = block-Jacobi only (the closest restatement of PCG(tol=1e-5));
 *   - `model.loss(input)` (pypose RobustModel, Huber kernel)  -> insfm_ba_cost().
 * Creation corresponds to the LM/model construction at bundle_adjustment.py:115-119 (packed inputs of :98-113).
 *
 * Plain C types only.  Device pointers are HIP device memory (e.g. the data_ptr() of a torch ROCm tensor).
 * All functions return INSFM_BA_OK (0) or a negative error code; insfm_ba_last_error() gives text.
 * One handle per device and stream; calls on a handle must be serialised by the caller.
 */
#ifndef INSFM_BA_H
#define INSFM_BA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define INSFM_BA_OK 0
#define INSFM_BA_EINVAL (-22)   /* bad descriptor / inputs (e.g. obs not track-major, unsupported model) */
#define INSFM_BA_ENOMEM (-12)   /* device or host allocation failed */
#define INSFM_BA_EHIP (-100)    /* HIP runtime error (message in insfm_ba_last_error) */
#define INSFM_BA_ECOMM (-101)   /* cross-rank all-reduce callback failed */
#define INSFM_BA_ESOLVER (-102) /* linear solver breakdown: params unchanged, loss == previous loss
                                   (mirrors "Linear solver failed. Breaking optimization step..." in the LM) */

typedef struct insfm_ba insfm_ba;

/* Sum `count` doubles starting at `dev_buf` across ranks, in place, ordered after all work the library
 * has queued on its stream (a torch.distributed all_reduce on the current stream satisfies this). */
typedef int (*insfm_ba_allreduce_fn)(void* ctx, double* dev_buf, int64_t count);

/* Optional asynchronous form: enqueue the in-place sum of `count` doubles at `dev_buf` on the HIP stream `stream`
 * (the library's exchange stream, already ordered after the work that produced the range) and return without waiting
 * for it (an RCCL all_reduce issued on that stream).  With it the library all-reduces the reduced camera system in row
 * chunks while the Schur complement of the next chunk is still being built (desc.exchange_chunks). */
typedef int (*insfm_ba_allreduce_async_fn)(void* ctx, double* dev_buf, int64_t count, void* stream);

typedef struct {
    int32_t n_cams;        /* C: rows of camera_params (registered, observed images after compaction) */
    int32_t n_points;      /* P: rows of points_3d */
    int32_t n_obs;         /* N: observations (after the cheirality filter, bundle_adjustment.py:102-107) */
    int32_t cam_model;     /* CameraModelId value (defs.py:101-113); 7 (FOV) and 10 (THIN_PRISM) -> EINVAL */
    int32_t optimize_poses;/* 0: cameras frozen, points-only solve (track_retriangulation.py:247-249) */
    int32_t deterministic; /* 1: fixed-order reductions everywhere (bitwise reproducible Schur build) */
    double huber_delta;    /* BUNDLE_ADJUSTER_OPTIONS['thres_loss_function'] */
    double tr_radius, tr_max, tr_min, tr_up, tr_down, tr_factor, tr_high, tr_low; /* TrustRegion(1e4, 1e10, .., 2, 1/16, ..) */
    double clamp_min, clamp_max;   /* A.diagonal().clamp_(1e-6, 1e32) */
    int32_t max_rejects;           /* LM(reject=30) */
    int32_t pcg_max_iter;          /* PCG iteration cap */
    double pcg_tol;                /* PCG(tol=1e-5): ||b - S x|| <= tol ||b|| */
    int32_t world_size, rank;      /* track-sharded multi-GPU; 1 / 0 for a single GPU */
    int32_t shard_point_begin;     /* points [begin, end) (and their observations) belong to this rank */
    int32_t shard_point_end;
    insfm_ba_allreduce_fn allreduce;  /* required when world_size > 1 */
    void* allreduce_ctx;
    int32_t precond;       /* PCG preconditioner: 0 block-Jacobi (the reference's), 1 two-level: block-Jacobi plus an
                              additive coarse correction on camera clusters (7 similarity modes + intrinsics per
                              cluster), 2 (default) = the same coarse space as an A-DEF2 deflation (x0 = Z E^-1 Z^T r0,
                              then M^-1 r = r + Z E^-1 Z^T (r - S r) -- Tang, Nabben, Vuik & Erlangga 2009): about half
                              the iterations of 1.  2 runs on the persistent CG (D = 8; insfm_ba_cg_info path 4, and 5
                              in its fixed-order form: deterministic mode, every rank of a multi-rank run); the
                              launch-per-iteration CG (other D, ranks sharing a GPU) runs 2 as 1.  An A-DEF2 solve that
                              breaks down is repeated with 1 (insfm_ba_cg_fallbacks).  Same stopping rule
                              (||b - S x|| <= tol ||b||), 5-20x fewer iterations than 0. */
    int32_t cluster_size;  /* target cameras per coarse cluster (default 24; grown until nclust*(D+1) <= 768) */
    int32_t schur_variant; /* reduced-system build: must be 0 (EINVAL otherwise).  Kept for the struct layout: the
                              round-2/3 variants 1-3 (re-derived or compact camera-point blocks) were measured slower
                              or even and removed. */
    insfm_ba_allreduce_async_fn allreduce_async; /* optional (see above); uses allreduce_ctx */
    int32_t exchange_chunks;  /* row chunks of the [S | b] exchange overlapped with the Schur build when allreduce_async
                                 is set (default 4; 1 = one all-reduce after the whole build) */
} insfm_ba_desc;

typedef struct {
    double loss;            /* robust (Huber) loss after the step, == LM.step() return value */
    double loss_before;     /* loss at the start of the step */
    double damping;         /* 1 / TrustRegion radius after the step */
    int32_t trials;         /* linear solves this step (1 + rejected trials) */
    int32_t rejects;
    int32_t pcg_iters_last; /* PCG iterations of the final trial */
    int32_t pcg_iters_total;
    int32_t solver_failed;
    int32_t cg_launches;    /* CG iteration launches this step (incl. the cheap early-exit ones after convergence;
                               the persistent two-level CG k_tl_cgp counts one per solve) */
    double time_ms[8];      /* device time per phase (hipEvent on the library stream), filled when stats != NULL:
                               [0] linearize  [1] k_schur  [2] whole linear solve (point prep .. CG finish, incl. the
                               host polls of the CG status)  [3] back-substitution + update  [4] trial cost
                               [5] CG iteration launches (k_cg_dots + k_cg_iter chunks, no host gaps)  [6] the
                               two-level coarse-inverse chains that finished during the step (side stream: E build +
                               Gauss-Jordan; overlaps the other phases)  [7] multi-rank: the chunked [S | b] exchange's
                               span on the exchange stream (0 otherwise)
                               Only filled after insfm_ba_set_timing(h, 1): the events cost a little. */
    int32_t coarse_used;    /* two-level preconditioner: 1 if the coarse correction was active in the final trial
                               (0 with precond 0, or when the coarse matrix was not positive definite) */
} insfm_ba_stats;

/* Fill `desc` with the reference's defaults (TorchBA + BUNDLE_ADJUSTER_OPTIONS, config/colmap.py:47-54). */
/* Provenance of this build: "src=<16 hex digits> arch=<gfx> flags=<hipcc flags>", the hash taken over the library's
 * sources and headers by instantsfm_amd/build.py (the Python loader refuses a library whose hash differs from the
 * tree it is loaded from). */
const char* insfm_build_info(void);

void insfm_ba_default_desc(insfm_ba_desc* desc);

/* Create a solver.  obs_uv [N,2] f64, cam_idx [N] i32 (compacted camera row), pt_idx [N] i32 (compacted point row,
 * nondecreasing = track-major as TorchBA packs them), pp [C,2] f64: HOST pointers, copied.  `stream` is a hipStream_t
 * (NULL = default stream).  Device memory is allocated here and freed by insfm_ba_destroy. */
int insfm_ba_create(const insfm_ba_desc* desc, const double* obs_uv, const int32_t* cam_idx, const int32_t* pt_idx,
                    const double* pp, void* stream, insfm_ba** out);

/* One LM step (bae.optim.LM.step semantics).  cam_params [C, 7+n_intr] ([t, q_xyzw, intrinsics without pp]) and
 * points [P,3] are DEVICE pointers, read at the start and updated in place at the end (on a multi-rank run each
 * rank updates only its shard's points).  `stats` may be NULL.  Per trial the host waits for the trial cost (five
 * scalars published into host-mapped memory by the last kernel of the trial, read by a spin on a sequence word).
 * The buffers are read in place as the step's linearization point (they must not be written by other work while the
 * step runs); an accepted trial is copied into them by that same kernel, the last work enqueued on the handle's
 * stream (stream-ordered: work queued after the call on that stream sees it; other streams or host reads
 * synchronize with the stream first). */
int insfm_ba_step(insfm_ba* h, double* cam_params, double* points, insfm_ba_stats* stats);

/* Enable (1) / disable (0, default) the per-phase hipEvent timing reported in insfm_ba_stats.time_ms. */
int insfm_ba_set_timing(insfm_ba* h, int32_t on);

/* Robust loss and raw reprojection RMSE (sqrt(sum ||r||^2 / N)) at the given DEVICE parameters. */
int insfm_ba_cost(insfm_ba* h, const double* cam_params, const double* points, double* loss, double* rmse);

/* Multi-rank runs: the reduced system [S | b | U | g_c | scalars] must live in a caller-owned DEVICE buffer that the
 * allreduce callback can reach (e.g. a torch tensor).  Query the size after create, then hand the buffer over before
 * the first step.  The callback is then only ever called with sub-ranges of this buffer. */
int64_t insfm_ba_exchange_count(const insfm_ba* h);
int insfm_ba_set_exchange(insfm_ba* h, double* dev_buf, int64_t count);

/* Multi-rank runs: how many ranks of the group (this one included) share this rank's GPU; every rank passes the same
 * count before the first step.  The replicated two-level CG runs as one persistent launch per solve (k_tl_cgp) only
 * when that many of its grids fit on the device at once (else the ranks' workgroups could hold each other off the CUs
 * until a grid barrier times out); otherwise every rank takes the launch-per-iteration CG, so that all ranks round
 * alike.  Default 1 (one GPU per rank). */
int insfm_ba_set_ranks_per_device(insfm_ba* h, int32_t ranks);
/* Which CG this handle runs: out[0] = 0 the launch-per-iteration two-level / block-Jacobi CG, 1 the persistent
 * k_tl_cgp with atomic cluster sums (single rank), 2 the persistent k_tl_cgp in its fixed-order form (deterministic
 * mode, replicated multi-rank CG), 3 the row-partitioned multi-rank CG; out[1] the k_tl_cgp grid (workgroups), out[2]
 * the workgroups of it the device holds at once, out[3] its register blocks per row (0: not eligible). */
int insfm_ba_cg_info(const insfm_ba* h, int32_t* out);
/* on = 0: this handle leaves the persistent k_tl_cgp for the launch-per-iteration CG (ranks of a replicated
 * multi-rank CG must all take the same path: the engine all-gathers insfm_ba_cg_info and turns it off everywhere
 * unless every rank runs the fixed-order k_tl_cgp and every GPU holds all grids placed on it).  on = 1: EINVAL unless
 * the handle already runs it. */
int insfm_ba_set_persistent_cg(insfm_ba* h, int32_t on);

/* A-DEF2 solves (precond 2) of this handle that broke down (single-reduction recurrence, status 2: possible under a
 * lagged coarse inverse) and were repeated with the additive coarse correction (precond 1) instead of failing the LM
 * step; a count (>= 0) or a negative error code. */
int32_t insfm_ba_cg_fallbacks(const insfm_ba* h);

/* Row-partitioned two-level CG across ranks (multi-rank handles with precond 1): each rank applies
 * the reduced camera matrix to its own rows (whole camera clusters) and writes those rows' CG partials straight into
 * every rank's exchange window over peer-to-peer mappings; the recurrence scalars and the coarse correction stay
 * replicated, so the result is bitwise the replicated CG's.  After create (and set_exchange): insfm_ba_cg_window
 * allocates this rank's window and returns its IPC handle (hipIpcMemHandle_t, 64 bytes) in ipc_handle; every rank then
 * passes all ranks' handles (world_size x 64 bytes, in rank order) to insfm_ba_cg_attach before the first step.  Ranks
 * must not destroy their handle while a peer may still write into its window (barrier first).  Replaces the replicated
 * CG of the reference's PCG(tol=1e-5) solve (bundle_adjustment.py:117) on multi-rank runs.
 * insfm_ba_cg_partition: this rank's rows as [begin, end) cluster-ordered positions. */
int insfm_ba_cg_window(insfm_ba* h, void* ipc_handle);
int insfm_ba_cg_attach(insfm_ba* h, const void* handles);
int insfm_ba_cg_partition(const insfm_ba* h, int32_t* rows_begin_end);
/* Collective timing probe of the partitioned CG's exchange: `reps` back-to-back flag exchanges with every peer (the
 * k_xsignal / k_xwait pair each CG iteration pays), average microseconds per exchange into *us. */
int insfm_ba_debug_time_xchg(insfm_ba* h, int32_t reps, double* us);

/* A fresh LM on the same problem, as TorchBA builds one per Solve: forgets the cached loss, the damping / TrustRegion
 * state and the lagged coarse inverse of the two-level preconditioner (the next solve factorizes its own). */
int insfm_ba_reset(insfm_ba* h);

/* Free the device buffers that destroyed handles parked for reuse (process-wide cache, at most
 * INSFM_DEVICE_CACHE_MB, default 4096 MB; invisible to PyTorch's caching allocator).  Returns the bytes released. */
int64_t insfm_ba_release_cache(void);

void insfm_ba_destroy(insfm_ba* h);
const char* insfm_ba_last_error(const insfm_ba* h);

/* ---- introspection used by the parity tests (not needed by TorchBA) -------------------------------------- */
/* Linearize at DEVICE params (fills W, V, g_p, U, g_c). */
int insfm_ba_debug_linearize(insfm_ba* h, const double* cam_params, const double* points);
/* Build and solve the damped system for cumulative damping factor f; returns PCG iterations or a negative code. */
int insfm_ba_debug_solve(insfm_ba* h, double f);
/* Copy an internal buffer to HOST memory: 0 the camera-point records Y[N,3,D] (Y_o = W_o R_p^-T, R_p the Cholesky
 * factor of point p's block damped for the first trial: S = U - sum Y Y^T; column-major blocks) 1 V[P,6] 2 g_p[P,3] 3 U[C,D,D] 4 g_c[C,D] 5 S(scaled after a
 * solve)[nnzb,D,D] 6 b[C,D] 7 dc[C,D] 8 dp[P,3].  Returns the number of doubles copied or a negative code. */
int64_t insfm_ba_debug_get(insfm_ba* h, int32_t which, double* host_out);
/* Device time per launch (us, hipEvents on the library stream) of `reps` back-to-back launches of one kernel on the
 * data of the last solve: which = 0 k_cg_iter (one block-Jacobi CG iteration), 1 k_schur, 2 one two-level CG
 * iteration (k_tl_pc + k_tl_pspmv), 3 k_tl_pspmv alone, 4 the two-level setup (k_tl_basis, the E build k_tl_erow +
 * k_tl_ereduce, the Gauss-Jordan inversion k_gj_pinv0 + k_gj_step), 5 k_lin_points at the last trial's parameters
 * (BA with stored W records only), 6 the coarse inverse alone (k_gj_pinv0 + one k_gj_step per 32-wide block of E),
 * 7 the E build alone (k_tl_erow + k_tl_ereduce).  Overwrites CG scratch state. */
int insfm_ba_debug_time_kernel(insfm_ba* h, int32_t which, int32_t reps, double* us_per_launch);
/* The persistent two-level CG (k_tl_cgp, the default D = 8 solve) of the last solve, re-run `reps` times from its
 * right-hand side: out[0] device microseconds per k_tl_cgp launch (a whole solve: the coarse solve of r0, the in-kernel
 * setup and every iteration), out[1] 0 (reserved: the setup launch that preceded it until round 4), out[2] PCG
 * iterations per solve.  EINVAL when the handle does not
 * run k_tl_cgp.  Overwrites CG scratch state.  (Measurement of PCG(tol=1e-5), bundle_adjustment.py:117.) */
int insfm_ba_debug_time_cgp(insfm_ba* h, int32_t reps, double* out);
/* INSFM_DIAG=stamps only (else returns 0): the device-clock timestamps (wall_clock64, 100 MHz) of the last
 * min(steps taken, 1024, max_steps) LM steps, oldest first, [steps][10 kernels][entry, exit] as int64 into HOST
 * memory: kernels k_lin_points, k_schur, k_tl_cgp, k_cg_finish, k_publish, k_cg_factor, k_tl_basis, k_backsub_rc,
 * k_cost, k_final (the trial's: the last launch of each in the step; entry = workgroup 0's, exit = the latest
 * workgroup end; 0 = not launched).  Tracer-free main-queue busy time and gaps.  Returns the number of steps copied. */
int32_t insfm_ba_debug_stamps(insfm_ba* h, int64_t* host_out, int32_t max_steps);
/* Camera cluster labels [C] of the two-level preconditioner's coarse space (HOST out); returns the cluster count. */
int32_t insfm_ba_debug_clusters(const insfm_ba* h, int32_t* labels);
/* Number of upper-triangular camera blocks of the reduced system (incl. the diagonal). */
int64_t insfm_ba_nnzb(const insfm_ba* h);
/* E^-1 of a dense SPD matrix (DEVICE pointers, row-major m x m, 1 <= m <= 4096) by the two-level preconditioner's
 * blocked Gauss-Jordan kernels (k_gj_pinv0 / k_gj_step), on `stream` (NULL: the default stream); blocks until done.
 * Returns 1 when E is positive definite, 0 when a pivot was not positive (Einv is then meaningless), or a negative
 * code.  If us_per_inverse is non-NULL, the inversion is repeated `reps` times and the mean device time stored. */
int insfm_ba_debug_spd_inverse(int32_t m, const double* E, double* Einv, void* stream, int32_t reps,
                               double* us_per_inverse);

#ifdef __cplusplus
}
#endif
#endif /* INSFM_BA_H */
