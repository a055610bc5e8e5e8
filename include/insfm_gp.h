/*
 * insfm_gp.h -- C ABI of the MI355X-native global-positioning solver (same handle type and library as insfm_ba.h).
 *
 * This replaces the engine under InstantSfM's TorchGP processor:
 *   - `loss = optimizer.step(input)` of `bae.optim.LM(model, strategy=TrustRegion(radius=1e3, max=1e8, up=2.0,
 *     down=0.5**4), solver=PCG(tol=1e-5), kernel=Huber(GLOBAL_POSITIONER_OPTIONS['thres_loss_function']), reject=30)`
 *     (instantsfm/processors/global_positioning.py:158-161, :176)  -> insfm_gp_step();
 *   - the residual model `PairwiseNonBatched.forward` = `pairwise_cost(points_3d[pi], translations[ci], scales,
 *     translations_obs, is_calibrated[ci])` (global_positioning.py:51-71, utils/cost_function.py:23-29) and its
 *     TrackingTensor Jacobian, with `scales.optimize_indices` excluding observations that carry a valid depth
 *     (global_positioning.py:57-59, :145-152)  -> the library's GP linearize / scale-elimination kernels;
 *   - `bae.utils.pysolvers.PCG` -> the shared Schur complement + (two-level) PCG kernels with 3x3 camera blocks.
 * The depth-only variant (PairwiseNonBatchedDepthOnly, :73-83) is the same problem with every scale fixed
 * (scale_free all 0).
 *
 * Parameters are camera POSITIONS (TorchGP optimizes image.world2cam[:3, 3] as positions and converts them to
 * translations afterwards, ConvertResults :41-43), track points, and one scale per observation.
 */
#ifndef INSFM_GP_H
#define INSFM_GP_H

#include "insfm_ba.h"

#ifdef __cplusplus
extern "C" {
#endif

/* insfm_ba_default_desc() with TorchGP's values: huber_delta 0.1, TrustRegion radius 1e3 / max 1e8
 * (global_positioning.py:158-161, config/colmap.py:41-46).  cam_model and optimize_poses are ignored. */
void insfm_gp_default_desc(insfm_ba_desc* desc);

/* Create a global-positioning solver.  HOST inputs, copied: trans [N,3] f64 world-frame rays
 * (R_img^T features_undist, global_positioning.py:135), cam_idx [N] / pt_idx [N] i32 (pt_idx nondecreasing, as
 * TorchGP packs them track by track), cam_factor [C] f64 (1.0 if the camera has a prior focal length else 0.5,
 * cost_function.py:27), scale_free [N] i32 (0: scale fixed at its given value -- observation with a valid depth;
 * NULL: all free).  desc->n_cams/n_points/n_obs give C/P/N.  Destroy with insfm_ba_destroy. */
int insfm_gp_create(const insfm_ba_desc* desc, const double* trans, const int32_t* cam_idx, const int32_t* pt_idx,
                    const double* cam_factor, const int32_t* scale_free, void* stream, insfm_ba** out);

/* One LM step.  positions [C,3], points [P,3], scales [N] (per observation, the caller's order): DEVICE pointers,
 * updated in place (multi-rank: this rank's points and their observations' scales only).  Loaded into the LM state
 * and written back by one launch each on the handle's stream (stream-ordered like insfm_ba_step: no host wait after
 * the write-back). */
int insfm_gp_step(insfm_ba* h, double* positions, double* points, double* scales, insfm_ba_stats* stats);

/* Robust loss and raw RMSE sqrt(sum ||r||^2 / N) at DEVICE parameters. */
int insfm_gp_cost(insfm_ba* h, const double* positions, const double* points, const double* scales, double* loss,
                  double* rmse);

/* ---- introspection used by the parity tests ---- */
/* Linearize at DEVICE parameters; then insfm_ba_debug_solve(h, f) solves the damped system and
 * insfm_ba_debug_get gives 0 W as [N,4] records {u, beta^2} (W_o = -beta^2 (I - u u^T), scale-eliminated) 1 V[P,6]
 * (damped) 2 g'_p 5 S 6 b 7 dc[C,3] 8 dp[P,3]. */
int insfm_gp_debug_linearize(insfm_ba* h, const double* positions, const double* points, const double* scales);
/* Scale steps of the last solve in the caller's observation order (HOST out, [N]); returns N. */
int64_t insfm_gp_debug_get_ds(insfm_ba* h, double* host_out);

#ifdef __cplusplus
}
#endif
#endif /* INSFM_GP_H */
