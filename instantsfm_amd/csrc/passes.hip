// Between-round caller passes of the global mapper (include/insfm_passes.h): per-feature undistortion and the
// per-observation / per-track filters.  Elementwise, HBM- and gather-bound: one thread per item, 16-byte loads where
// the layout allows, no LDS.  Floating-point contraction is off in this file so the arithmetic sequence is the one
// the reference (numpy / OpenCV scalar code, no FMA) performs.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/insfm_ba.h"
#include "../../include/insfm_passes.h"

#pragma clang fp contract(off)

#include "ba_device.h"  // eval_obs<M>: the reproject_funcs restatement shared with the BA kernels

namespace {

constexpr int kT = 256;
constexpr double kEps = 1e-10;

// cvUndistortPointsInternal (OpenCV 4.10, calib3d/src/undistort.dispatch.cpp) for R = I, no tilt, default criteria
// COUNT 5: fixed-point iteration x <- (x0 - delta(x)) * icdist(x) on the K-normalized point.
__device__ void cv_undistort(double u, double v, double fx, double fy, double cx, double cy, const double k[12], double& xo,
                             double& yo) {
    const double ifx = 1.0 / fx, ify = 1.0 / fy;
    double x = (u - cx) * ifx, y = (v - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; ++j) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        if (icdist < 0) {  // regression_14583
            x = (u - cx) * ifx;
            y = (v - cy) * ify;
            break;
        }
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    xo = x;
    yo = y;
}

// Camera.img2cam (scene/defs.py:315-369) for one feature; the reference's parameter vector p (Camera.set_params).
// f32: the features are float32, so cv2 returns float32 and the fisheye post-processing runs in float32 (numpy).
__device__ void img2cam(int model, const double* p, double u, double v, bool f32, double& x, double& y) {
    const bool single = model == 0 || model == 2 || model == 3 || model == 8 || model == 9;
    const double fx = p[0], fy = single ? p[0] : p[1];
    const double cx = single ? p[1] : p[2], cy = single ? p[2] : p[3];
    if (model == 0) {  // (xy - pp) / focal(), focal() = mean(focal_length)
        const double f = (fx + fy) / 2;
        x = (u - cx) / f;
        y = (v - cy) / f;
        return;
    }
    if (model == 1) {
        x = (u - cx) / fx;
        y = (v - cy) / fy;
        return;
    }
    if (model == 7 && f32) {  // FOV on float32 features: numpy keeps r2 / factor in float32 (omega is a Python float)
        const double omega = p[4], omega2 = omega * omega, eps = 1e-4;
        const float uf = (float)u, vf = (float)v;
        const float r2 = uf * uf + vf * vf;
        float factor;
        if (omega2 < eps) factor = (float)((omega2 * r2) / 3 - omega2 / 12 + 1);
        else if (r2 < eps) factor = (float)((omega * (omega2 * r2 + 3)) / (6 * tan(omega / 2)));
        else {
            // numpy 2 promotion: tan(radius * omega) is float32 (omega a weak Python float), the denominator
            // radius * 2 * np.tan(omega / 2) is float64 (np.float64 scalar), the quotient is stored as float32.
            // tan of the float32 argument is evaluated in double and rounded: the correctly rounded tanf.
            const float radius = sqrtf(r2);
            const float num = (float)tan((double)(radius * (float)omega));
            factor = (float)((double)num / ((double)(radius * 2.0f) * tan(omega / 2)));
        }
        x = (u - cx) / fx * (double)factor;
        y = (v - cy) / fy * (double)factor;
        return;
    }
    if (model == 7) {  // FOV, as written in the reference (r2 of the raw pixel coordinates)
        const double omega = p[4], omega2 = omega * omega, eps = 1e-4;
        const double r2 = u * u + v * v;
        double factor;
        if (omega2 < eps) factor = (omega2 * r2) / 3 - omega2 / 12 + 1;
        else if (r2 < eps) factor = (omega * (omega2 * r2 + 3)) / (6 * tan(omega / 2));
        else {
            const double radius = sqrt(r2);
            factor = tan(radius * omega) / (radius * 2 * tan(omega / 2));
        }
        x = (u - cx) / fx * factor;
        y = (v - cy) / fy * factor;
        return;
    }
    double k[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    switch (model) {
        case 2: case 8: k[0] = p[3]; break;
        case 3: case 9: k[0] = p[3]; k[1] = p[4]; break;
        case 4: k[0] = p[4]; k[1] = p[5]; k[2] = p[6]; k[3] = p[7]; break;
        case 5: k[0] = p[4]; k[1] = p[5]; k[4] = p[6]; break;
        case 6: k[0] = p[4]; k[1] = p[5]; k[2] = p[6]; k[3] = p[7]; k[4] = p[8]; k[5] = p[9]; k[6] = p[10]; k[7] = p[11]; break;
        case 10: k[0] = p[4]; k[1] = p[5]; k[2] = p[6]; k[3] = p[7]; k[4] = p[8]; k[8] = p[10]; k[9] = p[11]; break;
        default: break;
    }
    cv_undistort(u, v, fx, fy, cx, cy, k, x, y);
    const bool fisheye = model == 5 || model == 8 || model == 9 || model == 10;
    if (f32) {
        const float xf = (float)x, yf = (float)y;
        if (fisheye) {  // normal_from_fisheye in float32: uv * sin(theta) / (theta cos(theta))
            const float th = sqrtf(xf * xf + yf * yf);
            const float tc = th * cosf(th), s = sinf(th);
            x = (double)(xf * s / tc);
            y = (double)(yf * s / tc);
        } else {
            x = (double)xf;
            y = (double)yf;
        }
    } else if (fisheye) {
        const double th = sqrt(x * x + y * y);
        const double tc = th * cos(th), s = sin(th);
        x = x * s / tc;
        y = y * s / tc;
    }
}

__global__ __launch_bounds__(kT) void k_undistort(int64_t n, const void* __restrict__ xy, int f32,
                                                  const int32_t* __restrict__ feat_cam, const int32_t* __restrict__ cam_model,
                                                  const double* __restrict__ cam_params, double* __restrict__ rays) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    double u, v;
    if (f32) {
        const float2 q = reinterpret_cast<const float2*>(xy)[i];
        u = q.x;
        v = q.y;
    } else {
        const double2 q = reinterpret_cast<const double2*>(xy)[i];
        u = q.x;
        v = q.y;
    }
    const int c = feat_cam[i];
    double x, y;
    img2cam(cam_model[c], cam_params + 12 * (size_t)c, u, v, f32 != 0, x, y);
    // np.hstack([uv, 1]) / np.linalg.norm(axis=1): sqrt((x*x + y*y) + 1*1)
    const double nrm = sqrt(x * x + y * y + 1.0 * 1.0);
    rays[3 * i] = x / nrm;
    rays[3 * i + 1] = y / nrm;
    rays[3 * i + 2] = 1.0 / nrm;
}

__global__ __launch_bounds__(kT) void k_filter_reproj(int64_t n, const int32_t* __restrict__ obs_img,
                                                      const int32_t* __restrict__ obs_track, const int64_t* __restrict__ obs_ray,
                                                      const double* __restrict__ w2c, const double* __restrict__ xyz,
                                                      const double* __restrict__ rays, double max_err,
                                                      uint8_t* __restrict__ valid, double* __restrict__ err_out) {
    const int64_t x = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (x >= n) return;
    const double* W = w2c + 16 * (size_t)obs_img[x];
    const double* X = xyz + 3 * (size_t)obs_track[x];
    const double* r = rays + 3 * obs_ray[x];
    const double X0 = X[0], X1 = X[1], X2 = X[2];
    // einsum('ijk,ik->ij', world2cam, [xyz, 1])[:, :3]
    const double p0 = W[0] * X0 + W[1] * X1 + W[2] * X2 + W[3];
    const double p1 = W[4] * X0 + W[5] * X1 + W[6] * X2 + W[7];
    const double p2 = W[8] * X0 + W[9] * X1 + W[10] * X2 + W[11];
    const double rz = r[2] + kEps, pz = p2 + kEps;
    const double d0 = p0 / pz - r[0] / rz, d1 = p1 / pz - r[1] / rz;
    const double e = sqrt(d0 * d0 + d1 * d1);
    valid[x] = (p2 > kEps) && (e < max_err);
    if (err_out) err_out[x] = e;
}

__global__ __launch_bounds__(kT) void k_filter_angle(int64_t n, const int32_t* __restrict__ obs_img,
                                                     const int32_t* __restrict__ obs_track, const int64_t* __restrict__ obs_ray,
                                                     const double* __restrict__ w2c, const double* __restrict__ xyz,
                                                     const double* __restrict__ rays, double cos_thres,
                                                     uint8_t* __restrict__ valid) {
    const int64_t x = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (x >= n) return;
    const double* W = w2c + 16 * (size_t)obs_img[x];
    const double* X = xyz + 3 * (size_t)obs_track[x];
    const double* r = rays + 3 * obs_ray[x];
    // world2cam[:3, :3] @ xyz + world2cam[:3, 3]
    const double p0 = (W[0] * X[0] + W[1] * X[1] + W[2] * X[2]) + W[3];
    const double p1 = (W[4] * X[0] + W[5] * X[1] + W[6] * X[2]) + W[7];
    const double p2 = (W[8] * X[0] + W[9] * X[1] + W[10] * X[2]) + W[11];
    if (p2 < kEps) { valid[x] = 0; return; }
    const double nrm = sqrt(p0 * p0 + p1 * p1 + p2 * p2);
    const double dot = (p0 / nrm) * r[0] + (p1 / nrm) * r[1] + (p2 / nrm) * r[2];
    valid[x] = dot > cos_thres;
}

// One thread per track: all pairs of its observations' viewing directions (L^2 / 2 dot products, L ~ 2..200).
__global__ __launch_bounds__(kT) void k_filter_tri_angle(int64_t nt, const int64_t* __restrict__ track_ptr,
                                                         const int32_t* __restrict__ obs_img, const double* __restrict__ centers,
                                                         const double* __restrict__ xyz, double cos_thres,
                                                         uint8_t* __restrict__ remove) {
    const int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (t >= nt) return;
    const double X0 = xyz[3 * t], X1 = xyz[3 * t + 1], X2 = xyz[3 * t + 2];
    const int64_t b = track_ptr[t], e = track_ptr[t + 1];
    bool all = true;
    for (int64_t i = b; i < e && all; ++i) {
        const double* ci = centers + 3 * (size_t)obs_img[i];
        double a0 = X0 - ci[0], a1 = X1 - ci[1], a2 = X2 - ci[2];
        const double na = sqrt(a0 * a0 + a1 * a1 + a2 * a2) + kEps;
        a0 /= na; a1 /= na; a2 /= na;
        // diagonal term (i, i) included, as the reference's result_matrix
        for (int64_t j = i; j < e; ++j) {
            const double* cj = centers + 3 * (size_t)obs_img[j];
            double b0 = X0 - cj[0], b1 = X1 - cj[1], b2 = X2 - cj[2];
            const double nb = sqrt(b0 * b0 + b1 * b1 + b2 * b2) + kEps;
            b0 /= nb; b1 /= nb; b2 /= nb;
            if (!(a0 * b0 + a1 * b1 + a2 * b2 > cos_thres)) { all = false; break; }
        }
    }
    remove[t] = all ? 1 : 0;
}

// Camera.cam2img (scene/defs.py:371-412) of one camera-frame point, with Camera.Distortion (defs.py:257-313) and
// fisheye_from_normal (defs.py:246-250) in numpy's operation order; p is the reference's Camera.params vector.
// Integer powers follow numpy: r2**2 is a square (r2 * r2), r2**3 goes through pow().
__device__ void cam2img(int model, const double* p, double X, double Y, double Z, double& xo, double& yo) {
    const bool single = model == 0 || model == 2 || model == 3 || model == 8 || model == 9;
    const double fx = p[0], fy = single ? p[0] : p[1];
    const double cx = single ? p[1] : p[2], cy = single ? p[2] : p[3];
    const double f = (fx + fy) / 2;  // np.mean(focal_length)
    const double zz = Z + 1e-10;
    double u = X / zz, v = Y / zz;
    const bool fisheye = model == 5 || model == 8 || model == 9 || model == 10;
    if (fisheye) {  // uv * arctan(r) / r, r = max(||uv||, 1e-8)
        double r = sqrt(u * u + v * v);
        r = r < 1e-8 ? 1e-8 : r;
        const double th = atan(r);
        u = u * th / r;
        v = v * th / r;
    }
    const double r2 = u * u + v * v;
    bool use_ff = false;
    switch (model) {
        case 0: break;
        case 1: use_ff = true; break;
        case 2: case 8: {
            const double du = u * p[3] * r2, dv = v * p[3] * r2;
            u += du; v += dv;
        } break;
        case 3: case 9: {
            const double du = u * p[3] * r2 + u * p[4] * (r2 * r2), dv = v * p[3] * r2 + v * p[4] * (r2 * r2);
            u += du; v += dv;
        } break;
        case 4: case 6: case 10: {
            use_ff = true;
            double radial;
            if (model == 4) radial = p[4] * r2 + p[5] * (r2 * r2);
            else if (model == 6)
                radial = (1 + p[4] * r2 + p[5] * (r2 * r2) + p[8] * pow(r2, 3.0)) /
                         (1 + p[9] * r2 + p[10] * (r2 * r2) + p[11] * pow(r2, 3.0)) - 1;
            else radial = p[4] * r2 + p[5] * (r2 * r2) + p[8] * pow(r2, 3.0);
            const double p0 = p[6], p1 = p[7], uv_ = u * v;
            double dx = u * radial + 2 * p0 * uv_, dy = v * radial + 2 * p1 * uv_;
            dx += p1 * (r2 + 2 * (u * u));
            dy += p0 * (r2 + 2 * (v * v));
            if (model == 10) { dx += p[10] * r2; dy += p[11] * r2; }
            u += dx; v += dy;
        } break;
        case 5: {
            use_ff = true;
            const double radial = p[4] * r2 + p[5] * (r2 * r2) + p[6] * pow(r2, 3.0);
            const double du = u * radial, dv = v * radial;
            u += du; v += dv;
        } break;
        case 7: {  // FOV: uv = Distortion(uv), then the mean focal
            const double omega = p[4], omega2 = omega * omega, eps = 1e-4;
            double factor;
            if (omega2 < eps) factor = (omega2 * r2) / 3 - omega2 / 12 + 1;
            else if (r2 < eps) {
                const double th = tan(omega / 2);
                factor = (-2 * th * (4 * r2 * (th * th) - 3)) / (3 * omega);
            } else {
                const double radius = sqrt(r2);
                factor = atan(radius * 2 * tan(omega / 2)) / (radius * omega);
            }
            u = u * factor; v = v * factor;
        } break;
        default: break;
    }
    xo = use_ff ? u * fx + cx : u * f + cx;
    yo = use_ff ? v * fy + cy : v * f + cy;
}

// FilterTracksByReprojection (track_filter.py:68-113): p = world2cam[img] [xyz, 1] (einsum order as k_filter_reproj),
// pixel reprojection through the image's camera, error against the raw feature (float32 or float64).
__global__ __launch_bounds__(kT) void k_filter_reproj_pixel(int64_t n, const int32_t* __restrict__ obs_img,
                                                            const int32_t* __restrict__ obs_track,
                                                            const int64_t* __restrict__ obs_feat, const void* __restrict__ feats,
                                                            int f32, const int32_t* __restrict__ img_cam,
                                                            const int32_t* __restrict__ cam_model,
                                                            const double* __restrict__ cam_params, const double* __restrict__ w2c,
                                                            const double* __restrict__ xyz, double max_err,
                                                            uint8_t* __restrict__ valid, double* __restrict__ err_out) {
    const int64_t x = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (x >= n) return;
    const int im = obs_img[x];
    const double* W = w2c + 16 * (size_t)im;
    const double* X = xyz + 3 * (size_t)obs_track[x];
    const double X0 = X[0], X1 = X[1], X2 = X[2];
    const double p0 = W[0] * X0 + W[1] * X1 + W[2] * X2 + W[3];
    const double p1 = W[4] * X0 + W[5] * X1 + W[6] * X2 + W[7];
    const double p2 = W[8] * X0 + W[9] * X1 + W[10] * X2 + W[11];
    const int c = img_cam[im];
    double px, py;
    cam2img(cam_model[c], cam_params + 12 * (size_t)c, p0, p1, p2, px, py);
    double fu, fv;
    if (f32) {
        const float2 q = reinterpret_cast<const float2*>(feats)[obs_feat[x]];
        fu = q.x; fv = q.y;
    } else {
        const double2 q = reinterpret_cast<const double2*>(feats)[obs_feat[x]];
        fu = q.x; fv = q.y;
    }
    const double d0 = px - fu, d1 = py - fv;
    const double e = sqrt(d0 * d0 + d1 * d1);
    valid[x] = (p2 > kEps) && (e < max_err);
    if (err_out) err_out[x] = e;
}

// complete_tracks' candidate test (track_retriangulation.py:58-90): reproject_funcs[M] (eval_obs, the BA kernels'
// projection) with the image's row [t, q_xyzw, intrinsics without pp] and pp; valid = z > 1e-7 && ||err|| <= thr.
template <int M>
__global__ __launch_bounds__(kT) void k_reproj_candidates(int64_t n, const int32_t* __restrict__ cand_img,
                                                          const int32_t* __restrict__ cand_track,
                                                          const int64_t* __restrict__ cand_feat,
                                                          const void* __restrict__ feats, int f32,
                                                          const double* __restrict__ rows, const double* __restrict__ pps,
                                                          const double* __restrict__ xyz, double thr,
                                                          uint8_t* __restrict__ valid, double* __restrict__ err_out) {
    constexpr int S = insfm::kStride<M>;
    const int64_t x = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (x >= n) return;
    const int im = cand_img[x];
    double cam[S];
#pragma unroll
    for (int j = 0; j < S; ++j) cam[j] = rows[(size_t)im * S + j];
    const double Xp[3] = {xyz[3 * (size_t)cand_track[x]], xyz[3 * (size_t)cand_track[x] + 1],
                          xyz[3 * (size_t)cand_track[x] + 2]};
    const double pp[2] = {pps[2 * (size_t)im], pps[2 * (size_t)im + 1]};
    double uv[2];
    if (f32) {
        const float2 q = reinterpret_cast<const float2*>(feats)[cand_feat[x]];
        uv[0] = q.x; uv[1] = q.y;
    } else {
        const double2 q = reinterpret_cast<const double2*>(feats)[cand_feat[x]];
        uv[0] = q.x; uv[1] = q.y;
    }
    double r[2];
    insfm::eval_obs<M, false>(cam, Xp, pp, uv, r, nullptr, nullptr);
    // rotate_quat z (the same expression eval_obs evaluates)
    const double qx = cam[3], qy = cam[4], qw = cam[6];
    const double c1z = qx * Xp[1] - qy * Xp[0];
    const double c1x = qy * Xp[2] - cam[5] * Xp[1], c1y = cam[5] * Xp[0] - qx * Xp[2];
    const double c2z = qx * c1y - qy * c1x;
    const double pz = Xp[2] + 2.0 * (qw * c1z + c2z) + cam[2];
    const double e = sqrt(r[0] * r[0] + r[1] * r[1]);
    valid[x] = (e <= thr) && (pz > 1e-7);
    if (err_out) err_out[x] = e;
}

inline unsigned grid(int64_t n) { return (unsigned)((n + kT - 1) / kT); }

int finish() {
    return hipGetLastError() == hipSuccess ? INSFM_BA_OK : INSFM_BA_EHIP;
}

}  // namespace

extern "C" {

int insfm_undistort(int64_t n, const void* xy, int32_t xy_f32, const int32_t* feat_cam, const int32_t* cam_model,
                    const double* cam_params, double* rays, void* stream) {
    if (n < 0 || (n > 0 && (!xy || !feat_cam || !cam_model || !cam_params || !rays))) return INSFM_BA_EINVAL;
    if (n == 0) return INSFM_BA_OK;
    k_undistort<<<grid(n), kT, 0, reinterpret_cast<hipStream_t>(stream)>>>(n, xy, xy_f32, feat_cam, cam_model, cam_params,
                                                                         rays);
    return finish();
}

int insfm_filter_reproj_normalized(int64_t n_obs, const int32_t* obs_img, const int32_t* obs_track, const int64_t* obs_ray,
                                   const double* world2cam, const double* track_xyz, const double* rays, double max_err,
                                   uint8_t* valid, double* err, void* stream) {
    if (n_obs < 0 || (n_obs > 0 && (!obs_img || !obs_track || !obs_ray || !world2cam || !track_xyz || !rays || !valid)))
        return INSFM_BA_EINVAL;
    if (n_obs == 0) return INSFM_BA_OK;
    k_filter_reproj<<<grid(n_obs), kT, 0, reinterpret_cast<hipStream_t>(stream)>>>(n_obs, obs_img, obs_track, obs_ray,
                                                                                  world2cam, track_xyz, rays, max_err, valid,
                                                                                  err);
    return finish();
}

int insfm_filter_angle(int64_t n_obs, const int32_t* obs_img, const int32_t* obs_track, const int64_t* obs_ray,
                       const double* world2cam, const double* track_xyz, const double* rays, double cos_thres,
                       uint8_t* valid, void* stream) {
    if (n_obs < 0 || (n_obs > 0 && (!obs_img || !obs_track || !obs_ray || !world2cam || !track_xyz || !rays || !valid)))
        return INSFM_BA_EINVAL;
    if (n_obs == 0) return INSFM_BA_OK;
    k_filter_angle<<<grid(n_obs), kT, 0, reinterpret_cast<hipStream_t>(stream)>>>(n_obs, obs_img, obs_track, obs_ray,
                                                                                 world2cam, track_xyz, rays, cos_thres, valid);
    return finish();
}

int insfm_filter_tri_angle(int64_t n_tracks, const int64_t* track_ptr, const int32_t* obs_img, const double* centers,
                           const double* track_xyz, double cos_thres, uint8_t* remove, void* stream) {
    if (n_tracks < 0 || (n_tracks > 0 && (!track_ptr || !obs_img || !centers || !track_xyz || !remove)))
        return INSFM_BA_EINVAL;
    if (n_tracks == 0) return INSFM_BA_OK;
    k_filter_tri_angle<<<grid(n_tracks), kT, 0, reinterpret_cast<hipStream_t>(stream)>>>(n_tracks, track_ptr, obs_img,
                                                                                        centers, track_xyz, cos_thres, remove);
    return finish();
}

int insfm_filter_reproj_pixel(int64_t n_obs, const int32_t* obs_img, const int32_t* obs_track, const int64_t* obs_feat,
                              const void* feats, int32_t feats_f32, const int32_t* img_cam, const int32_t* cam_model,
                              const double* cam_params, const double* world2cam, const double* track_xyz, double max_err,
                              uint8_t* valid, double* err, void* stream) {
    if (n_obs < 0 || (n_obs > 0 && (!obs_img || !obs_track || !obs_feat || !feats || !img_cam || !cam_model || !cam_params ||
                                    !world2cam || !track_xyz || !valid)))
        return INSFM_BA_EINVAL;
    if (n_obs == 0) return INSFM_BA_OK;
    k_filter_reproj_pixel<<<grid(n_obs), kT, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        n_obs, obs_img, obs_track, obs_feat, feats, feats_f32, img_cam, cam_model, cam_params, world2cam, track_xyz, max_err,
        valid, err);
    return finish();
}

int insfm_reproj_candidates(int64_t n, int32_t cam_model, const int32_t* cand_img, const int32_t* cand_track,
                            const int64_t* cand_feat, const void* feats, int32_t feats_f32, const double* image_rows,
                            const double* image_pps, const double* track_xyz, double max_err, uint8_t* valid, double* err,
                            void* stream) {
    if (n < 0 || (n > 0 && (!cand_img || !cand_track || !cand_feat || !feats || !image_rows || !image_pps || !track_xyz ||
                            !valid)))
        return INSFM_BA_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define INSFM_CAND(M)                                                                                                      \
    case M:                                                                                                                \
        if (n > 0)                                                                                                         \
            k_reproj_candidates<M><<<grid(n), kT, 0, s>>>(n, cand_img, cand_track, cand_feat, feats, feats_f32, image_rows, \
                                                          image_pps, track_xyz, max_err, valid, err);                      \
        break;
    switch (cam_model) {
        INSFM_CAND(0) INSFM_CAND(1) INSFM_CAND(2) INSFM_CAND(3) INSFM_CAND(4) INSFM_CAND(5) INSFM_CAND(6) INSFM_CAND(8)
        INSFM_CAND(9)
        default: return INSFM_BA_EINVAL;  // FOV / THIN_PRISM_FISHEYE: reproject_funcs raises (cost_function.py:125,179)
    }
#undef INSFM_CAND
    return n > 0 ? finish() : INSFM_BA_OK;
}

}  // extern "C"
