/*
 * insfm_passes.h -- C ABI of the between-round caller passes, same library as insfm_ba.h.
 *
 * global_mapper.py runs these between the bundle-adjustment rounds (:130-150, :160-166) and around global
 * positioning (:107-112):
 *   - UndistortImages (processors/image_undistortion.py:3-10 + Camera.img2cam, scene/defs.py:315-369)
 *       -> insfm_undistort(): every feature of every image -> unit ray [x, y, 1] / ||.||;
 *   - FilterTracksByReprojectionNormalized (processors/track_filter.py:26-66) -> insfm_filter_reproj_normalized();
 *   - FilterTracksByAngle (track_filter.py:5-24)                            -> insfm_filter_angle();
 *   - FilterTracksTriangulationAngle (track_filter.py:116-137)             -> insfm_filter_tri_angle().
 * The kernels compute per feature / observation / track; the scene bookkeeping (gathering the arrays from the scene
 * objects, the per-track compaction, the counters) stays in the host processors (instantsfm_amd/processors/).
 *
 * All array arguments are DEVICE pointers; `stream` is a hipStream_t (NULL = default).  The calls only enqueue work.
 * Return 0 or INSFM_BA_EINVAL / INSFM_BA_EHIP.
 */
#ifndef INSFM_PASSES_H
#define INSFM_PASSES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Camera.img2cam + normalization for n features.  xy [n,2] is float32 when xy_f32 != 0 (the database's feature
 * type; cv2.undistortPoints then returns float32, which is reproduced), else float64.  feat_cam [n] int32: row of
 * the feature's camera in cam_model [ncam] (CameraModelId value; 0-10) and cam_params [ncam,12] (the reference's
 * Camera.params vector, zero padded).  Output rays [n,3] float64. */
int insfm_undistort(int64_t n, const void* xy, int32_t xy_f32, const int32_t* feat_cam, const int32_t* cam_model,
                    const double* cam_params, double* rays, void* stream);

/* Per observation x (image obs_img[x], track obs_track[x], ray rays[obs_ray[x]]):
 *   p = world2cam[img] (4x4, row-major) * [xyz[track], 1];
 *   valid[x] = p.z > 1e-10  &&  || p.xy / (p.z + 1e-10) - ray.xy / (ray.z + 1e-10) || < max_err.
 * err (nullable) receives the reprojection error. */
int insfm_filter_reproj_normalized(int64_t n_obs, const int32_t* obs_img, const int32_t* obs_track,
                                   const int64_t* obs_ray, const double* world2cam, const double* track_xyz,
                                   const double* rays, double max_err, uint8_t* valid, double* err, void* stream);

/* valid[x] = p.z >= 1e-10 && dot(p / ||p||, ray) > cos_thres, p = R[img] xyz[track] + t[img] (track_filter.py:5-24). */
int insfm_filter_angle(int64_t n_obs, const int32_t* obs_img, const int32_t* obs_track, const int64_t* obs_ray,
                       const double* world2cam, const double* track_xyz, const double* rays, double cos_thres,
                       uint8_t* valid, void* stream);

/* Per track t (observations [track_ptr[t], track_ptr[t+1]) of obs_img): remove[t] = 1 when every pair of its
 * images' viewing directions (xyz - center, normalized with +1e-10) has cosine > cos_thres (track_filter.py:116-137;
 * duplicate images do not change the outcome, so no np.unique is needed).  centers [M,3]. */
int insfm_filter_tri_angle(int64_t n_tracks, const int64_t* track_ptr, const int32_t* obs_img, const double* centers,
                           const double* track_xyz, double cos_thres, uint8_t* remove, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* INSFM_PASSES_H */
