/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Linked by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg; never by the product path (instantsfm_amd/).
 *
 * Plain-C (C99 + OpenMP) float64 restatement of the reference's BA hot path:
 *   - per-observation reprojection, cost_function.py:32-208 (9 implemented models), with
 *     bae.utils.ba.rotate_quat restated as p + 2w(qv x p) + 2 qv x (qv x p) + t (pypose [t, q_xyzw]);
 *   - residual = reproject(...) - points_2d, bundle_adjustment.py:59-64;
 *   - the un-vendored LM step (bae.optim.LM + pypose@bae TrustRegion/Huber) as reconstructed in
 *     SURVEY.md section 3.3 / Appendix A, with the options TorchBA passes at
 *     bundle_adjustment.py:115-119 (TrustRegion(1e4, 1e10, 2, 1/16), PCG(tol=1e-5), Huber(delta), reject=30):
 *       * Huber kernel + Triggs corrector: w = 1 if sqrt(s) < delta else delta/sqrt(s); r~ = sqrt(w) r, J~ = sqrt(w) J
 *       * A = J~^T J~ with diag clamped to [1e-6, 1e32]; per trial diag *= (1 + damping) (cumulative)
 *       * damped system solved by explicit Schur complement on the camera blocks + PCG, preconditioned by block-Jacobi
 *         (precond 0) or the two-level block-Jacobi + camera-cluster coarse correction (precond 1, the default)
 *         (relative residual tol, x0 = 0); back-substitution for points
 *       * SE3 left retraction X <- Exp([rho, phi]) X (pypose se3 = [rho, phi]); intrinsics and points +=
 *       * gain ratio (last - new) / -((J~D)^T (2 r~ + J~D)) -> TrustRegion radius update; reject while
 *         new > last and rejects < 30.
 * The LM/PCG/TrustRegion arithmetic lives in un-vendored bae / pypose@bae (no pinned commit): that
 * part is PARITY UNPINNED against the reference; projection is pinned by tests/golden/projection_golden.npz.
 *
 * Reductions are deterministic (fixed 4096-element chunks, chunk partials summed in order), so results
 * do not depend on the OpenMP thread count.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXD 16
#define ORA_GP 100   /* ora_create "model" of the global-positioning problem (ora_gp_create) */
#define CHUNK 4096

/* ------------------------------------------------------------------------------------------ */
/* camera models                                                                               */
/* ------------------------------------------------------------------------------------------ */
int ora_n_intr(int model) {
    switch (model) {
        case 0: return 1; case 1: return 2; case 2: return 2; case 3: return 3;
        case 4: return 6; case 5: return 6; case 6: return 10; case 8: return 2; case 9: return 3;
        default: return -1;
    }
}
static int n_focal(int model) { return (model == 1 || model == 4 || model == 5 || model == 6) ? 2 : 1; }

/* atan(r)/r and its derivative w.r.t. r2 (series near 0 for the derivative). */
static void fisheye_g(double r2, double* g, double* dg) {
    if (r2 == 0.0) { *g = 1.0; *dg = -1.0 / 3.0; return; }
    double r = sqrt(r2);
    *g = atan(r) / r;
    if (r2 < 1e-3) {
        double s = 0.0, pw = 1.0;
        for (int n = 1; n <= 8; ++n) { s += ((n & 1) ? -1.0 : 1.0) * n * pw / (2 * n + 1); pw *= r2; }
        *dg = s;
    } else {
        *dg = (1.0 / (1.0 + r2) - *g) / (2.0 * r2);
    }
}

/* Distortion of normalized coords: out (du,dv), Jd = d(du,dv)/d(u,v) (row-major 2x2),
 * Jk = d(du,dv)/d(k_j) (row-major 2 x nk), k = distortion params (after the focal lengths). */
static void distort(int model, const double* k, double u, double v, double* du, double* dv, double* Jd, double* Jk, int nk) {
    double r2 = u * u + v * v;
    if (model == 0 || model == 1) {
        *du = u; *dv = v; Jd[0] = 1; Jd[1] = 0; Jd[2] = 0; Jd[3] = 1;
        return;
    }
    if (model == 4 || model == 6) {
        double rad, radp, dr[8];
        double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3];
        if (model == 4) {
            rad = k1 * r2 + k2 * r2 * r2;
            radp = k1 + 2 * k2 * r2;
            dr[0] = r2; dr[1] = r2 * r2;
        } else {
            double k3 = k[4], k4 = k[5], k5 = k[6], k6 = k[7];
            double r4 = r2 * r2, r6 = r4 * r2;
            double Nn = 1 + k1 * r2 + k2 * r4 + k3 * r6, Dn = 1 + k4 * r2 + k5 * r4 + k6 * r6;
            rad = Nn / Dn - 1;
            double Np = k1 + 2 * k2 * r2 + 3 * k3 * r4, Dp = k4 + 2 * k5 * r2 + 3 * k6 * r4;
            radp = (Np * Dn - Nn * Dp) / (Dn * Dn);
            dr[0] = r2 / Dn; dr[1] = r4 / Dn; dr[4] = r6 / Dn;
            dr[5] = -Nn * r2 / (Dn * Dn); dr[6] = -Nn * r4 / (Dn * Dn); dr[7] = -Nn * r6 / (Dn * Dn);
        }
        double uv = u * v;
        *du = u + u * rad + 2 * p1 * uv + p2 * (r2 + 2 * u * u);
        *dv = v + v * rad + 2 * p2 * uv + p1 * (r2 + 2 * v * v);
        Jd[0] = 1 + rad + 2 * u * u * radp + 2 * p1 * v + 6 * p2 * u;
        Jd[1] = 2 * uv * radp + 2 * p1 * u + 2 * p2 * v;
        Jd[2] = 2 * uv * radp + 2 * p2 * v + 2 * p1 * u;
        Jd[3] = 1 + rad + 2 * v * v * radp + 2 * p2 * u + 6 * p1 * v;
        for (int j = 0; j < nk; ++j) { Jk[j] = 0; Jk[nk + j] = 0; }
        /* k1, k2 (and k3..k6 for FULL) act through rad */
        int radial_idx[6] = {0, 1, 4, 5, 6, 7};
        int nrad = (model == 4) ? 2 : 6;
        for (int a = 0; a < nrad; ++a) { int j = radial_idx[a]; Jk[j] = u * dr[j]; Jk[nk + j] = v * dr[j]; }
        Jk[2] = 2 * uv;          Jk[nk + 2] = r2 + 2 * v * v;   /* p1 */
        Jk[3] = r2 + 2 * u * u;  Jk[nk + 3] = 2 * uv;           /* p2 */
        return;
    }
    /* radial-h family: (du,dv) = h(r2) (u,v) */
    double h, hp, dh[4] = {0, 0, 0, 0};
    if (model == 2) { h = 1 + k[0] * r2; hp = k[0]; dh[0] = r2; }
    else if (model == 3) { h = 1 + k[0] * r2 + k[1] * r2 * r2; hp = k[0] + 2 * k[1] * r2; dh[0] = r2; dh[1] = r2 * r2; }
    else { /* fisheye: 5, 8, 9 */
        double g, gp, P, Pp;
        fisheye_g(r2, &g, &gp);
        if (model == 5) {
            P = 1 + k[0] * r2 + k[1] * r2 * r2 + k[2] * r2 * r2 * r2;
            Pp = k[0] + 2 * k[1] * r2 + 3 * k[2] * r2 * r2;
            dh[0] = g * r2; dh[1] = g * r2 * r2; dh[2] = g * r2 * r2 * r2; dh[3] = 0.0; /* k4 ignored by the reference */
        } else if (model == 8) {
            P = 1 + k[0] * r2; Pp = k[0]; dh[0] = g * r2;
        } else {
            P = 1 + k[0] * r2 + k[1] * r2 * r2; Pp = k[0] + 2 * k[1] * r2; dh[0] = g * r2; dh[1] = g * r2 * r2;
        }
        h = g * P; hp = gp * P + g * Pp;
    }
    *du = u * h; *dv = v * h;
    Jd[0] = h + 2 * u * u * hp; Jd[1] = 2 * u * v * hp;
    Jd[2] = 2 * u * v * hp;     Jd[3] = h + 2 * v * v * hp;
    for (int j = 0; j < nk; ++j) { Jk[j] = u * dh[j]; Jk[nk + j] = v * dh[j]; }
}

/* Evaluate one observation.  cam = [t(3), q_xyzw(4), intr(ni)].  Outputs:
 *   r (2) = projection - uv (uv may be NULL -> projection only),
 *   Jc (2 x D row-major, D = 6 + ni; pose tangent [rho, phi] left-perturbation, then intrinsics),
 *   Jp (2 x 3 row-major).  Jc/Jp may be NULL.  Also returns z_cam via *zc if non-NULL. */
void ora_eval_one(int model, const double* cam, const double* X, const double* pp, const double* uv,
                  double* r, double* Jc, double* Jp, double* zc) {
    int ni = ora_n_intr(model), nf = n_focal(model), nk = ni - nf, D = 6 + ni;
    const double *t = cam, *q = cam + 3, *intr = cam + 7;
    double qx = q[0], qy = q[1], qz = q[2], w = q[3];
    /* p_c = X + 2 w (qv x X) + 2 qv x (qv x X) + t ; linear in X with matrix M */
    double c1[3] = {qy * X[2] - qz * X[1], qz * X[0] - qx * X[2], qx * X[1] - qy * X[0]};
    double c2[3] = {qy * c1[2] - qz * c1[1], qz * c1[0] - qx * c1[2], qx * c1[1] - qy * c1[0]};
    double pc[3];
    for (int i = 0; i < 3; ++i) pc[i] = X[i] + 2.0 * (w * c1[i] + c2[i]) + t[i];
    if (zc) *zc = pc[2];
    double iz = 1.0 / pc[2];
    double u = pc[0] * iz, v = pc[1] * iz;
    double du, dv, Jd[4], Jk[2 * 10];
    distort(model, intr + nf, u, v, &du, &dv, Jd, Jk, nk);
    double fx = intr[0], fy = (nf == 2) ? intr[1] : intr[0];
    if (r) {
        r[0] = fx * du + pp[0] - (uv ? uv[0] : 0.0);
        r[1] = fy * dv + pp[1] - (uv ? uv[1] : 0.0);
    }
    if (!Jc && !Jp) return;
    /* A = diag(f) Jd duv/dpc  (2x3) */
    double duv[6] = {iz, 0, -u * iz, 0, iz, -v * iz};
    double A[6];
    for (int a = 0; a < 2; ++a) {
        double fa = a == 0 ? fx : fy;
        for (int c = 0; c < 3; ++c) A[a * 3 + c] = fa * (Jd[a * 2 + 0] * duv[c] + Jd[a * 2 + 1] * duv[3 + c]);
    }
    if (Jp) {
        /* M = I + 2w[q]x + 2[q]x[q]x  => dpc/dX */
        double M[9];
        double K[9] = {0, -qz, qy, qz, 0, -qx, -qy, qx, 0};
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                double kk = 0;
                for (int l = 0; l < 3; ++l) kk += K[i * 3 + l] * K[l * 3 + j];
                M[i * 3 + j] = (i == j ? 1.0 : 0.0) + 2.0 * w * K[i * 3 + j] + 2.0 * kk;
            }
        for (int a = 0; a < 2; ++a)
            for (int j = 0; j < 3; ++j) Jp[a * 3 + j] = A[a * 3 + 0] * M[0 * 3 + j] + A[a * 3 + 1] * M[1 * 3 + j] + A[a * 3 + 2] * M[2 * 3 + j];
    }
    if (Jc) {
        double ex[3][3] = {{0, -pc[2], pc[1]}, {pc[2], 0, -pc[0]}, {-pc[1], pc[0], 0}}; /* e_k x p_c */
        for (int a = 0; a < 2; ++a) {
            double* row = Jc + a * D;
            row[0] = A[a * 3 + 0]; row[1] = A[a * 3 + 1]; row[2] = A[a * 3 + 2];
            for (int k = 0; k < 3; ++k) row[3 + k] = A[a * 3 + 0] * ex[k][0] + A[a * 3 + 1] * ex[k][1] + A[a * 3 + 2] * ex[k][2];
            if (nf == 1) row[6] = (a == 0) ? du : dv;
            else { row[6] = (a == 0) ? du : 0.0; row[7] = (a == 0) ? 0.0 : dv; }
            double fa = a == 0 ? fx : fy;
            for (int j = 0; j < nk; ++j) row[6 + nf + j] = fa * Jk[a * nk + j];
        }
    }
}

void ora_eval(int model, int n, const double* X, const double* cam, const double* pp, const double* uv,
              double* r, double* Jc, double* Jp) {
    int stride = 7 + ora_n_intr(model), D = 6 + ora_n_intr(model);
    #pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i)
        ora_eval_one(model, cam + (size_t)i * stride, X + 3 * (size_t)i, pp + 2 * (size_t)i, uv ? uv + 2 * (size_t)i : NULL,
                     r + 2 * (size_t)i, Jc ? Jc + (size_t)i * 2 * D : NULL, Jp ? Jp + 6 * (size_t)i : NULL, NULL);
}

/* ------------------------------------------------------------------------------------------ */
/* SE3 (pypose conventions): se3 = [rho, phi]; Exp -> (q_phi, J_l(phi) rho); left composition    */
/* ------------------------------------------------------------------------------------------ */
void ora_retract_pose(const double* x /*7*/, const double* d /*6*/, double* out /*7*/) {
    const double *rho = d, *phi = d + 3;
    double th2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
    double th = sqrt(th2);
    double s_half, c_half, A, B; /* q = [s_half*phi, c_half]; J_l = I + A[phi]x + B[phi]x^2 */
    if (th < 1e-5) {
        s_half = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0;
        c_half = 1.0 - th2 / 8.0 + th2 * th2 / 384.0;
        A = 0.5 - th2 / 24.0 + th2 * th2 / 720.0;
        B = 1.0 / 6.0 - th2 / 120.0 + th2 * th2 / 5040.0;
    } else {
        s_half = sin(0.5 * th) / th;
        c_half = cos(0.5 * th);
        A = (1.0 - cos(th)) / th2;
        B = (th - sin(th)) / (th2 * th);
    }
    double qd[4] = {s_half * phi[0], s_half * phi[1], s_half * phi[2], c_half};
    double px = phi[0], py = phi[1], pz = phi[2];
    double cr[3] = {py * rho[2] - pz * rho[1], pz * rho[0] - px * rho[2], px * rho[1] - py * rho[0]};
    double cr2[3] = {py * cr[2] - pz * cr[1], pz * cr[0] - px * cr[2], px * cr[1] - py * cr[0]};
    double tau[3];
    for (int i = 0; i < 3; ++i) tau[i] = rho[i] + A * cr[i] + B * cr2[i];
    /* rotate t by q_d: t' = t + 2 w (qv x t) + 2 qv x (qv x t) */
    const double* t = x;
    double c1[3] = {qd[1] * t[2] - qd[2] * t[1], qd[2] * t[0] - qd[0] * t[2], qd[0] * t[1] - qd[1] * t[0]};
    double c2[3] = {qd[1] * c1[2] - qd[2] * c1[1], qd[2] * c1[0] - qd[0] * c1[2], qd[0] * c1[1] - qd[1] * c1[0]};
    for (int i = 0; i < 3; ++i) out[i] = t[i] + 2.0 * (qd[3] * c1[i] + c2[i]) + tau[i];
    /* q' = q_d (x) q (Hamilton, xyzw) */
    const double* q = x + 3;
    double ax = qd[0], ay = qd[1], az = qd[2], aw = qd[3];
    double bx = q[0], by = q[1], bz = q[2], bw = q[3];
    out[3] = aw * bx + ax * bw + ay * bz - az * by;
    out[4] = aw * by - ax * bz + ay * bw + az * bx;
    out[5] = aw * bz + ax * by - ay * bx + az * bw;
    out[6] = aw * bw - ax * bx - ay * by - az * bz;
}

/* ------------------------------------------------------------------------------------------ */
/* small dense helpers                                                                         */
/* ------------------------------------------------------------------------------------------ */
/* inverse of a symmetric positive definite n x n matrix (row-major, full) via Cholesky.
 * Returns 0 on success, -1 if not positive definite. */
static int spd_inverse(int n, const double* A, double* Ainv) {
    double L[MAXD * MAXD], Li[MAXD * MAXD];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = A[i * n + j];
            for (int k = 0; k < j; ++k) s -= L[i * MAXD + k] * L[j * MAXD + k];
            if (i == j) {
                if (!(s > 0.0)) return -1;
                L[i * MAXD + i] = sqrt(s);
            } else {
                L[i * MAXD + j] = s / L[j * MAXD + j];
            }
        }
    /* Li = L^{-1} (lower) */
    for (int i = 0; i < n; ++i) {
        Li[i * MAXD + i] = 1.0 / L[i * MAXD + i];
        for (int j = 0; j < i; ++j) {
            double s = 0;
            for (int k = j; k < i; ++k) s -= L[i * MAXD + k] * Li[k * MAXD + j];
            Li[i * MAXD + j] = s / L[i * MAXD + i];
        }
    }
    /* Ainv = Li^T Li */
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = 0;
            for (int k = i; k < n; ++k) s += Li[k * MAXD + i] * Li[k * MAXD + j];
            Ainv[i * n + j] = s;
            Ainv[j * n + i] = s;
        }
    return 0;
}

/* symmetric 3x3 stored as [xx, xy, xz, yy, yz, zz] */
static void sym3_full(const double* s, double* f) {
    f[0] = s[0]; f[1] = s[1]; f[2] = s[2];
    f[3] = s[1]; f[4] = s[3]; f[5] = s[4];
    f[6] = s[2]; f[7] = s[4]; f[8] = s[5];
}

static double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* ------------------------------------------------------------------------------------------ */
/* problem                                                                                    */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int model, ni, D, stride, C, P, N;
    double* uv; double* pp; int* cam; int* pt;
    int *pt_ptr, *cam_ptr, *cam_obs;
    int *row_ptr, *col, nnzb;
    int *lo_ptr, *lo_col, *lo_blk;
    /* options */
    double delta, radius0, rmax, rmin, up, down0, factor, high, low, cmin, cmax, pcg_tol;
    int max_rejects, pcg_max_iter, optimize_poses;
    int precond, cluster_size;   /* 0 block-Jacobi, 1 two-level (block-Jacobi + camera-cluster similarity coarse space) */
    /* summation-order perturbation (test yardstick, 0 = off): order_seed != 0 visits each camera row's observations
     * in ora_schur in a seeded pseudo-random order (the same terms summed in another order, as the GPU's LDS-atomic
     * row accumulation does); order_mode bit 1 also sums the PCG's dot products in reverse chunk order */
    int order_seed, order_mode;
    int *clab, nclust;           /* cluster label per camera, number of clusters */
    int *csize;                  /* cameras per cluster */
    double* lin_cams;            /* copy of the linearization point (coarse basis) */
    double* prev_einv;           /* coarse inverse of the previous solve (lag rule: see ora_pcg) */
    int kind;                    /* 0 bundle adjustment, 1 global positioning (ora_gp_*) */
    int u_predamped;             /* U already holds the damped camera blocks (global positioning) */
    /* global positioning (TorchGP.Optimize): per obs ray t, factor f, scale-free flag, linearization terms */
    double *gp_t, *gp_f, *gp_beta, *gp_a, *gp_r, *gp_hss, *gp_gs, *gp_ds, *gp_hx, *gp_hc, *gp_gx, *gp_gc;
    double *gp_scales_new;
    int* gp_sfree;
    int prev_ok, have_prev, fresh_lin;
    /* LM state */
    double damping, down, loss;
    int have_loss;
    /* work */
    double *W, *V, *gp, *U, *gc, *Vinv, *y, *S, *b, *Minv, *x, *r, *z, *p, *q, *dp;
    double *cams_new, *pts_new, *partial;
    /* stats of the last step: trials, pcg iters (last trial), total pcg iters, f */
    double stats[9];  /* trials, pcg last, pcg total, damping factor, damping, failed, rejects, coarse used,
                         A-DEF2 solves of the step repeated with the additive correction (breakdown) */
    int adef2_fallbacks;  /* (since the last ora_step) */
} ora_t;

static double det_sum_order(const double* v, size_t n, int reverse) {
    /* deterministic sum: fixed chunks, partial sums in order (reverse: chunks and their elements backwards) */
    size_t nch = (n + CHUNK - 1) / CHUNK;
    double* part = (double*)malloc((nch ? nch : 1) * sizeof(double));
    #pragma omp parallel for schedule(static)
    for (long c = 0; c < (long)nch; ++c) {
        double s = 0;
        size_t e = (c + 1) * (size_t)CHUNK; if (e > n) e = n;
        if (reverse)
            for (size_t i = e; i-- > (size_t)c * CHUNK;) s += v[i];
        else
            for (size_t i = (size_t)c * CHUNK; i < e; ++i) s += v[i];
        part[c] = s;
    }
    double s = 0;
    if (reverse)
        for (size_t c = nch; c-- > 0;) s += part[c];
    else
        for (size_t c = 0; c < nch; ++c) s += part[c];
    free(part);
    return s;
}
static double det_sum(const double* v, size_t n) { return det_sum_order(v, n, 0); }

static int cmp_int(const void* a, const void* b) { int x = *(const int*)a, y = *(const int*)b; return (x > y) - (x < y); }


/* ------------------------------------------------------------------------------------------ */
/* camera clustering for the two-level preconditioner                                          */
/* ------------------------------------------------------------------------------------------ */
/* Co-visibility weight w(i,j) = number of (obs of i, obs of j) pairs that share a track.  Greedy aggregation:
 * seeds in increasing camera id; an aggregate grows by the unassigned camera with the largest summed weight to it
 * (ties: smallest id) until it has K members or no connected unassigned camera is left.  Aggregates smaller than
 * K/2 are then dissolved: each member joins the aggregate of size >= K/2 it is most connected to (ties: smallest
 * aggregate id).  Labels are renumbered in order of first appearance by camera id. */
static int ora_aggregate(ora_t* h, int K);
/* The coarse dimension nclust * (D + 1) is capped at COARSE_MAX (the GPU's k_tl_pc keeps a cluster's rows of E^-1
 * in registers; csrc/ba_twolevel.h COARSE_MAX_DIM): while the aggregation yields more clusters, it is redone with the
 * target size grown in proportion to the excess, K' = max(K + 1, ceil(K nclust (D + 1) / COARSE_MAX)) rounded up to
 * even (aggregates below K / 2 are dissolved, so an odd K would keep singletons), at most C.  With K = C the clusters
 * are the co-visibility components; if even those exceed the cap, the solver falls back to block-Jacobi (precond 0):
 * returns 0 then, 1 when the clusters fit. */
#define COARSE_MAX 768
static int ora_cluster_cameras(ora_t* h) {
    int K = h->cluster_size < h->C ? h->cluster_size : h->C, nc;
    while ((nc = ora_aggregate(h, K)) * (h->D + 1) > COARSE_MAX && K < h->C) {
        long g = ((long)K * nc * (h->D + 1) + COARSE_MAX - 1) / COARSE_MAX;
        if (g < K + 1) g = K + 1;
        if (g > h->C) g = h->C;
        K = (int)g;
        K += K & 1;
        if (K > h->C) K = h->C;
    }
    return nc * (h->D + 1) <= COARSE_MAX;
}

static int ora_aggregate(ora_t* h, int K) {
    const int C = h->C;
    /* symmetric weighted adjacency (CSR) */
    int* deg = (int*)calloc(C + 1, sizeof(int));
    long* wsum = NULL;
    int* mark = (int*)malloc(sizeof(int) * C);
    long* acc = (long*)calloc(C, sizeof(long));
    for (int c = 0; c < C; ++c) mark[c] = -1;
    /* pass 1: neighbour lists per camera (both directions), weights by counting (o,q) pairs */
    int** nb = (int**)calloc(C, sizeof(int*));
    long** nw = (long**)calloc(C, sizeof(long*));
    int* nn = (int*)calloc(C, sizeof(int));
    int* buf = (int*)malloc(sizeof(int) * C);
    for (int i = 0; i < C; ++i) {
        int n = 0;
        for (int e = h->cam_ptr[i]; e < h->cam_ptr[i + 1]; ++e) {
            int o = h->cam_obs[e], p = h->pt[o];
            for (int q = h->pt_ptr[p]; q < h->pt_ptr[p + 1]; ++q) {
                if (q == o) continue;
                int j = h->cam[q];
                if (j == i) continue;
                if (mark[j] != i) { mark[j] = i; acc[j] = 0; buf[n++] = j; }
                acc[j] += 1;
            }
        }
        qsort(buf, n, sizeof(int), cmp_int);
        nb[i] = (int*)malloc(sizeof(int) * (n ? n : 1));
        nw[i] = (long*)malloc(sizeof(long) * (n ? n : 1));
        for (int k = 0; k < n; ++k) { nb[i][k] = buf[k]; nw[i][k] = acc[buf[k]]; }
        nn[i] = n;
    }
    (void)deg; (void)wsum;
    int* lab = h->clab;
    for (int c = 0; c < C; ++c) lab[c] = -1;
    long* score = (long*)calloc(C, sizeof(long));
    int* cand = (int*)malloc(sizeof(int) * C);
    char* incand = (char*)calloc(C, 1);
    int nagg = 0;
    int* asize = (int*)calloc(C, sizeof(int));
    for (int seed = 0; seed < C; ++seed) {
        if (lab[seed] >= 0) continue;
        int ncand = 0, size = 0;
        int cur = seed;
        for (;;) {
            lab[cur] = nagg; ++size;
            for (int k = 0; k < nn[cur]; ++k) {
                int j = nb[cur][k];
                if (lab[j] >= 0) continue;
                if (!incand[j]) { incand[j] = 1; score[j] = 0; cand[ncand++] = j; }
                score[j] += nw[cur][k];
            }
            if (size >= K) break;
            int best = -1; long bs = 0;
            for (int k = 0; k < ncand; ++k) {
                int j = cand[k];
                if (lab[j] >= 0) continue;
                if (score[j] > bs || (score[j] == bs && bs > 0 && j < best)) { bs = score[j]; best = j; }
            }
            if (best < 0) break;
            cur = best;
        }
        for (int k = 0; k < ncand; ++k) incand[cand[k]] = 0;
        asize[nagg] = size;
        ++nagg;
    }
    /* dissolve small aggregates */
    const int minsz = K / 2 > 1 ? K / 2 : 1;
    long* to = (long*)calloc(nagg, sizeof(long));
    int* newlab = (int*)malloc(sizeof(int) * C);
    for (int i = 0; i < C; ++i) newlab[i] = lab[i];
    for (int i = 0; i < C; ++i) {
        if (asize[lab[i]] >= minsz) continue;
        int best = -1; long bs = 0;
        for (int k = 0; k < nn[i]; ++k) { int a = lab[nb[i][k]]; if (asize[a] >= minsz) to[a] += nw[i][k]; }
        for (int k = 0; k < nn[i]; ++k) {
            int a = lab[nb[i][k]];
            if (asize[a] >= minsz && to[a] > 0) {
                if (to[a] > bs || (to[a] == bs && a < best)) { bs = to[a]; best = a; }
            }
        }
        for (int k = 0; k < nn[i]; ++k) to[lab[nb[i][k]]] = 0;
        if (best >= 0) newlab[i] = best;
    }
    /* renumber by first appearance */
    int* ren = (int*)malloc(sizeof(int) * nagg);
    for (int a = 0; a < nagg; ++a) ren[a] = -1;
    int nc = 0;
    for (int i = 0; i < C; ++i) {
        if (ren[newlab[i]] < 0) ren[newlab[i]] = nc++;
        lab[i] = ren[newlab[i]];
    }
    h->nclust = nc;
    for (int c = 0; c < C; ++c) h->csize[c] = 0;
    for (int i = 0; i < C; ++i) h->csize[lab[i]]++;
    for (int i = 0; i < C; ++i) { free(nb[i]); free(nw[i]); }
    free(nb); free(nw); free(nn); free(buf); free(mark); free(acc); free(score); free(cand); free(incand);
    free(asize); free(to); free(newlab); free(ren); free(deg);
    return nc;
}

int ora_clusters(const ora_t* h, int* lab) {
    if (lab) memcpy(lab, h->clab, sizeof(int) * h->C);
    return h->nclust;
}

/* Coarse basis of camera i (D x MC, row-major, MC = D + 1): the camera's tangent [rho, phi, intr] induced by an
 * infinitesimal similarity of the world (tau, omega, sigma) that leaves every projection unchanged
 *   rho = -R tau - [t]x R omega + sigma t,   phi = -R omega,
 * plus one column per intrinsic.  A camera alone in its cluster gets [I_D | 0] instead (the 7 similarity modes of a
 * single camera are linearly dependent). */
static void coarse_basis(int D, const double* cam, int alone, double* G, int kind) {
    const int MC = D + 1;
    for (int k = 0; k < D * MC; ++k) G[k] = 0.0;
    if (alone) { for (int a = 0; a < D; ++a) G[a * MC + a] = 1.0; return; }
    if (kind == 1) {  /* global positioning: camera position c; gauge = translation (I) and scaling about 0 (c) */
        for (int a = 0; a < 3; ++a) { G[a * MC + a] = 1.0; G[a * MC + 3] = cam[a]; }
        return;
    }
    const double *t = cam, *q = cam + 3;
    double qx = q[0], qy = q[1], qz = q[2], w = q[3];
    double Kq[9] = {0, -qz, qy, qz, 0, -qx, -qy, qx, 0}, R[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double kk = 0;
            for (int l = 0; l < 3; ++l) kk += Kq[i * 3 + l] * Kq[l * 3 + j];
            R[i * 3 + j] = (i == j ? 1.0 : 0.0) + 2.0 * w * Kq[i * 3 + j] + 2.0 * kk;
        }
    double tx[9] = {0, -t[2], t[1], t[2], 0, -t[0], -t[1], t[0], 0};
    for (int a = 0; a < 3; ++a)
        for (int k = 0; k < 3; ++k) {
            G[a * MC + k] = -R[a * 3 + k];
            double s = 0;
            for (int l = 0; l < 3; ++l) s += tx[a * 3 + l] * R[l * 3 + k];
            G[a * MC + 3 + k] = -s;
            G[(3 + a) * MC + 3 + k] = -R[a * 3 + k];
        }
    for (int a = 0; a < 3; ++a) G[a * MC + 6] = t[a];
    for (int k = 0; k < D - 6; ++k) G[(6 + k) * MC + 7 + k] = 1.0;
}

ora_t* ora_create(int model, int C, int P, int N, const double* uv, const int* cam, const int* pt, const double* pp,
                  const double* dopt, const int* iopt) {
    const int gpk = (model == ORA_GP);
    if ((!gpk && ora_n_intr(model) < 0) || C <= 0 || P <= 0 || N <= 0) return NULL;
    for (int i = 1; i < N; ++i) if (pt[i] < pt[i - 1]) return NULL; /* track-major required */
    ora_t* h = (ora_t*)calloc(1, sizeof(ora_t));
    h->model = model; h->kind = gpk;
    h->ni = gpk ? 0 : ora_n_intr(model); h->D = gpk ? 3 : 6 + h->ni; h->stride = gpk ? 3 : 7 + h->ni;
    h->C = C; h->P = P; h->N = N;
    h->delta = dopt[0]; h->radius0 = dopt[1]; h->rmax = dopt[2]; h->rmin = dopt[3]; h->up = dopt[4];
    h->down0 = dopt[5]; h->factor = dopt[6]; h->high = dopt[7]; h->low = dopt[8]; h->cmin = dopt[9];
    h->cmax = dopt[10]; h->pcg_tol = dopt[11];
    h->max_rejects = iopt[0]; h->pcg_max_iter = iopt[1]; h->optimize_poses = iopt[2];
    h->precond = iopt[4]; h->cluster_size = iopt[5] > 0 ? iopt[5] : 24;
    h->order_seed = iopt[6]; h->order_mode = iopt[7];
#ifdef _OPENMP
    if (iopt[3] > 0) omp_set_num_threads(iopt[3]);
#endif
    h->damping = 1.0 / h->radius0; h->down = h->down0;
    int D = h->D;
    if (!gpk) {
        h->uv = (double*)malloc(sizeof(double) * 2 * N); memcpy(h->uv, uv, sizeof(double) * 2 * N);
        h->pp = (double*)malloc(sizeof(double) * 2 * C); memcpy(h->pp, pp, sizeof(double) * 2 * C);
    }
    h->cam = (int*)malloc(sizeof(int) * N); memcpy(h->cam, cam, sizeof(int) * N);
    h->pt = (int*)malloc(sizeof(int) * N); memcpy(h->pt, pt, sizeof(int) * N);
    /* track pointers */
    h->pt_ptr = (int*)calloc(P + 1, sizeof(int));
    for (int i = 0; i < N; ++i) h->pt_ptr[pt[i] + 1]++;
    for (int p = 0; p < P; ++p) h->pt_ptr[p + 1] += h->pt_ptr[p];
    /* camera-major list (stable: obs order within a camera follows track-major order) */
    h->cam_ptr = (int*)calloc(C + 1, sizeof(int));
    for (int i = 0; i < N; ++i) h->cam_ptr[cam[i] + 1]++;
    for (int c = 0; c < C; ++c) h->cam_ptr[c + 1] += h->cam_ptr[c];
    h->cam_obs = (int*)malloc(sizeof(int) * N);
    {
        int* fill = (int*)malloc(sizeof(int) * C);
        memcpy(fill, h->cam_ptr, sizeof(int) * C);
        for (int i = 0; i < N; ++i) h->cam_obs[fill[cam[i]]++] = i;
        free(fill);
    }
    /* upper block pattern: row i holds i and every co-visible camera j > i, sorted */
    int* cnt = (int*)calloc(C, sizeof(int));
    int** cols = (int**)calloc(C, sizeof(int*));
    #pragma omp parallel
    {
        int* mark = (int*)malloc(sizeof(int) * C);
        for (int c = 0; c < C; ++c) mark[c] = -1;
        int* buf = (int*)malloc(sizeof(int) * C);
        #pragma omp for schedule(dynamic, 4)
        for (int i = 0; i < C; ++i) {
            int n = 0;
            mark[i] = i; buf[n++] = i;
            for (int e = h->cam_ptr[i]; e < h->cam_ptr[i + 1]; ++e) {
                int o = h->cam_obs[e], p = pt[o];
                for (int qq = h->pt_ptr[p]; qq < h->pt_ptr[p + 1]; ++qq) {
                    int j = cam[qq];
                    if (j > i && mark[j] != i) { mark[j] = i; buf[n++] = j; }
                }
            }
            qsort(buf, n, sizeof(int), cmp_int);
            cols[i] = (int*)malloc(sizeof(int) * n);
            memcpy(cols[i], buf, sizeof(int) * n);
            cnt[i] = n;
        }
        free(mark); free(buf);
    }
    h->row_ptr = (int*)calloc(C + 1, sizeof(int));
    for (int i = 0; i < C; ++i) h->row_ptr[i + 1] = h->row_ptr[i] + cnt[i];
    (void)0;
    h->nnzb = h->row_ptr[C];
    h->col = (int*)malloc(sizeof(int) * (h->nnzb ? h->nnzb : 1));
    for (int i = 0; i < C; ++i) { memcpy(h->col + h->row_ptr[i], cols[i], sizeof(int) * cnt[i]); free(cols[i]); }
    free(cols); free(cnt);
    h->clab = (int*)malloc(sizeof(int) * C);
    h->csize = (int*)calloc(C, sizeof(int));
    if (!ora_cluster_cameras(h) && h->precond >= 1) h->precond = 0;
    /* lower references: row j lists (i < j, blk of (i,j)) in increasing i */
    h->lo_ptr = (int*)calloc(C + 1, sizeof(int));
    for (int i = 0; i < C; ++i)
        for (int e = h->row_ptr[i] + 1; e < h->row_ptr[i + 1]; ++e) h->lo_ptr[h->col[e] + 1]++;
    for (int c = 0; c < C; ++c) h->lo_ptr[c + 1] += h->lo_ptr[c];
    int nlo = h->lo_ptr[C];
    h->lo_col = (int*)malloc(sizeof(int) * (nlo ? nlo : 1));
    h->lo_blk = (int*)malloc(sizeof(int) * (nlo ? nlo : 1));
    {
        int* fill = (int*)malloc(sizeof(int) * C);
        memcpy(fill, h->lo_ptr, sizeof(int) * C);
        for (int i = 0; i < C; ++i)
            for (int e = h->row_ptr[i] + 1; e < h->row_ptr[i + 1]; ++e) {
                int j = h->col[e]; int k = fill[j]++;
                h->lo_col[k] = i; h->lo_blk[k] = e;
            }
        free(fill);
    }
    size_t nb = (size_t)h->nnzb * D * D;
    h->W = (double*)malloc(sizeof(double) * (size_t)N * D * 3);
    h->V = (double*)malloc(sizeof(double) * (size_t)P * 6);
    h->gp = (double*)malloc(sizeof(double) * (size_t)P * 3);
    h->U = (double*)malloc(sizeof(double) * (size_t)C * D * D);
    h->gc = (double*)malloc(sizeof(double) * (size_t)C * D);
    h->Vinv = (double*)malloc(sizeof(double) * (size_t)P * 9);
    h->y = (double*)malloc(sizeof(double) * (size_t)P * 3);
    h->S = (double*)malloc(sizeof(double) * (nb ? nb : 1));
    h->b = (double*)malloc(sizeof(double) * (size_t)C * D);
    h->Minv = (double*)malloc(sizeof(double) * (size_t)C * D * D);
    h->x = (double*)malloc(sizeof(double) * (size_t)C * D);
    h->r = (double*)malloc(sizeof(double) * (size_t)C * D);
    h->z = (double*)malloc(sizeof(double) * (size_t)C * D);
    h->p = (double*)malloc(sizeof(double) * (size_t)C * D);
    h->q = (double*)malloc(sizeof(double) * (size_t)C * D);
    h->dp = (double*)malloc(sizeof(double) * (size_t)P * 3);
    h->cams_new = (double*)malloc(sizeof(double) * (size_t)C * h->stride);
    h->pts_new = (double*)malloc(sizeof(double) * (size_t)P * 3);
    size_t np = (size_t)N > (size_t)P ? (size_t)N : (size_t)P;
    h->partial = (double*)malloc(sizeof(double) * np * 2);
    return h;
}

void ora_destroy(ora_t* h) {
    if (!h) return;
    void* ptrs[] = {h->uv, h->pp, h->cam, h->pt, h->pt_ptr, h->cam_ptr, h->cam_obs, h->row_ptr, h->col, h->lo_ptr,
                    h->lo_col, h->lo_blk, h->W, h->V, h->gp, h->U, h->gc, h->Vinv, h->y, h->S, h->b, h->Minv, h->x,
                    h->r, h->z, h->p, h->q, h->dp, h->cams_new, h->pts_new, h->partial,
                    h->clab, h->csize, h->lin_cams, h->prev_einv, h->gp_t, h->gp_f, h->gp_beta, h->gp_a,
                    h->gp_r, h->gp_hss, h->gp_gs, h->gp_ds, h->gp_hx, h->gp_hc, h->gp_gx, h->gp_gc,
                    h->gp_scales_new, h->gp_sfree};
    for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); ++i) free(ptrs[i]);
    free(h);
}

int ora_nnzb(const ora_t* h) { return h->nnzb; }
void ora_pattern(const ora_t* h, int* row_ptr, int* col) {
    memcpy(row_ptr, h->row_ptr, sizeof(int) * (h->C + 1));
    memcpy(col, h->col, sizeof(int) * h->nnzb);
}

/* Huber loss (pypose.optim.kernel.Huber) summed over observations; also sum of squared norms. */
double ora_cost(ora_t* h, const double* cams, const double* pts, double* sq_out) {
    double* e = h->partial;
    double* s2 = h->partial + h->N;
    double d = h->delta;
    #pragma omp parallel for schedule(static)
    for (int i = 0; i < h->N; ++i) {
        double r[2];
        ora_eval_one(h->model, cams + (size_t)h->cam[i] * h->stride, pts + 3 * (size_t)h->pt[i], h->pp + 2 * (size_t)h->cam[i],
                     h->uv + 2 * (size_t)i, r, NULL, NULL, NULL);
        double s = r[0] * r[0] + r[1] * r[1];
        double rs = sqrt(s);
        e[i] = rs < d ? s : 2.0 * d * rs - d * d;
        s2[i] = s;
    }
    double loss = det_sum(e, h->N);
    if (sq_out) *sq_out = det_sum(s2, h->N);
    return loss;
}

/* Linearize at (cams, pts): W_o = J~c^T J~p (D x 3), V_p = sum J~p^T J~p (sym6), g_p = -sum J~p^T r~,
 * U_c = sum J~c^T J~c (D x D), g_c = -sum J~c^T r~.  Unclamped, undamped. */
void ora_linearize(ora_t* h, const double* cams, const double* pts) {
    h->fresh_lin = 1;
    if (!h->lin_cams) h->lin_cams = (double*)malloc(sizeof(double) * (size_t)h->C * h->stride);
    memcpy(h->lin_cams, cams, sizeof(double) * (size_t)h->C * h->stride);
    int D = h->D, model = h->model;
    double delta = h->delta;
    #pragma omp parallel for schedule(static)
    for (int p = 0; p < h->P; ++p) {
        double Vs[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
        for (int o = h->pt_ptr[p]; o < h->pt_ptr[p + 1]; ++o) {
            double r[2], Jc[2 * MAXD], Jp[6];
            int c = h->cam[o];
            ora_eval_one(model, cams + (size_t)c * h->stride, pts + 3 * (size_t)p, h->pp + 2 * (size_t)c, h->uv + 2 * (size_t)o, r, Jc, Jp, NULL);
            double s = r[0] * r[0] + r[1] * r[1];
            double wgt = sqrt(s) < delta ? 1.0 : delta / sqrt(s);
            double sw = sqrt(wgt);
            for (int k = 0; k < 2; ++k) { r[k] *= sw; }
            for (int k = 0; k < 2 * D; ++k) Jc[k] *= sw;
            for (int k = 0; k < 6; ++k) Jp[k] *= sw;
            double* Wo = h->W + (size_t)o * D * 3;
            for (int a = 0; a < D; ++a)
                for (int k = 0; k < 3; ++k) Wo[a * 3 + k] = Jc[a] * Jp[k] + Jc[D + a] * Jp[3 + k];
            Vs[0] += Jp[0] * Jp[0] + Jp[3] * Jp[3];
            Vs[1] += Jp[0] * Jp[1] + Jp[3] * Jp[4];
            Vs[2] += Jp[0] * Jp[2] + Jp[3] * Jp[5];
            Vs[3] += Jp[1] * Jp[1] + Jp[4] * Jp[4];
            Vs[4] += Jp[1] * Jp[2] + Jp[4] * Jp[5];
            Vs[5] += Jp[2] * Jp[2] + Jp[5] * Jp[5];
            for (int k = 0; k < 3; ++k) g[k] -= Jp[k] * r[0] + Jp[3 + k] * r[1];
        }
        memcpy(h->V + 6 * (size_t)p, Vs, sizeof(Vs));
        memcpy(h->gp + 3 * (size_t)p, g, sizeof(g));
    }
    #pragma omp parallel for schedule(dynamic, 4)
    for (int c = 0; c < h->C; ++c) {
        double Uc[MAXD * MAXD], g[MAXD];
        memset(Uc, 0, sizeof(double) * D * D); memset(g, 0, sizeof(double) * D);
        for (int e = h->cam_ptr[c]; e < h->cam_ptr[c + 1]; ++e) {
            int o = h->cam_obs[e], p = h->pt[o];
            double r[2], Jc[2 * MAXD];
            ora_eval_one(model, cams + (size_t)c * h->stride, pts + 3 * (size_t)p, h->pp + 2 * (size_t)c, h->uv + 2 * (size_t)o, r, Jc, NULL, NULL);
            double s = r[0] * r[0] + r[1] * r[1];
            double wgt = sqrt(s) < delta ? 1.0 : delta / sqrt(s);
            double sw = sqrt(wgt);
            r[0] *= sw; r[1] *= sw;
            for (int k = 0; k < 2 * D; ++k) Jc[k] *= sw;
            for (int a = 0; a < D; ++a) {
                for (int bb = 0; bb < D; ++bb) Uc[a * D + bb] += Jc[a] * Jc[bb] + Jc[D + a] * Jc[D + bb];
                g[a] -= Jc[a] * r[0] + Jc[D + a] * r[1];
            }
        }
        memcpy(h->U + (size_t)c * D * D, Uc, sizeof(double) * D * D);
        memcpy(h->gc + (size_t)c * D, g, sizeof(double) * D);
    }
}

/* Points-side preparation for damping factor f: Vinv = (clamp(diag) * f)^-1, y = Vinv g_p. */
static int prep_points(ora_t* h, double f) {
    int bad = 0;
    #pragma omp parallel for schedule(static) reduction(|:bad)
    for (int p = 0; p < h->P; ++p) {
        double Vs[6];
        memcpy(Vs, h->V + 6 * (size_t)p, sizeof(Vs));
        Vs[0] = clampd(Vs[0], h->cmin, h->cmax) * f;
        Vs[3] = clampd(Vs[3], h->cmin, h->cmax) * f;
        Vs[5] = clampd(Vs[5], h->cmin, h->cmax) * f;
        double full[9], inv[9];
        sym3_full(Vs, full);
        if (spd_inverse(3, full, inv)) { bad = 1; continue; }
        memcpy(h->Vinv + 9 * (size_t)p, inv, sizeof(inv));
        const double* g = h->gp + 3 * (size_t)p;
        for (int k = 0; k < 3; ++k) h->y[3 * (size_t)p + k] = inv[k * 3 + 0] * g[0] + inv[k * 3 + 1] * g[1] + inv[k * 3 + 2] * g[2];
    }
    return bad ? -1 : 0;
}

/* Reduced camera system for damping factor f: S (upper blocks) and b. */
void ora_schur(ora_t* h, double f) {
    int D = h->D, C = h->C;
    #pragma omp parallel
    {
        int* slot = (int*)malloc(sizeof(int) * C);
        for (int c = 0; c < C; ++c) slot[c] = -1;
        #pragma omp for schedule(dynamic, 1)
        for (int i = 0; i < C; ++i) {
            int rb = h->row_ptr[i], re = h->row_ptr[i + 1];
            for (int e = rb; e < re; ++e) slot[h->col[e]] = e;
            double* Srow = h->S + (size_t)rb * D * D;
            memset(Srow, 0, sizeof(double) * (size_t)(re - rb) * D * D);
            double bi[MAXD];
            for (int a = 0; a < D; ++a) bi[a] = h->gc[(size_t)i * D + a];
            const int eb = h->cam_ptr[i], ne = h->cam_ptr[i + 1] - eb;
            int* perm = NULL;
            if (h->order_seed && ne > 1) {  /* seeded Fisher-Yates over the row's observations (test yardstick) */
                perm = (int*)malloc(sizeof(int) * (size_t)ne);
                for (int k = 0; k < ne; ++k) perm[k] = k;
                unsigned long long st = 0x9E3779B97F4A7C15ull * (unsigned long long)(h->order_seed * 1000003LL + i + 1);
                for (int k = ne - 1; k > 0; --k) {
                    st ^= st >> 12; st ^= st << 25; st ^= st >> 27;
                    const int r = (int)((st * 0x2545F4914F6CDD1Dull) % (unsigned long long)(k + 1));
                    const int tmp = perm[k]; perm[k] = perm[r]; perm[r] = tmp;
                }
            }
            for (int e = eb; e < eb + ne; ++e) {
                int o = h->cam_obs[perm ? eb + perm[e - eb] : e], p = h->pt[o];
                const double* Wo = h->W + (size_t)o * D * 3;
                const double* Vi = h->Vinv + 9 * (size_t)p;
                const double* yp = h->y + 3 * (size_t)p;
                double Wh[MAXD * 3];
                for (int a = 0; a < D; ++a) {
                    for (int k = 0; k < 3; ++k) Wh[a * 3 + k] = Wo[a * 3 + 0] * Vi[0 * 3 + k] + Wo[a * 3 + 1] * Vi[1 * 3 + k] + Wo[a * 3 + 2] * Vi[2 * 3 + k];
                    bi[a] -= Wo[a * 3 + 0] * yp[0] + Wo[a * 3 + 1] * yp[1] + Wo[a * 3 + 2] * yp[2];
                }
                for (int qq = h->pt_ptr[p]; qq < h->pt_ptr[p + 1]; ++qq) {
                    int j = h->cam[qq];
                    if (j < i) continue;
                    double* blk = h->S + (size_t)slot[j] * D * D;
                    const double* Wq = h->W + (size_t)qq * D * 3;
                    for (int a = 0; a < D; ++a)
                        for (int bb = 0; bb < D; ++bb)
                            blk[a * D + bb] -= Wh[a * 3 + 0] * Wq[bb * 3 + 0] + Wh[a * 3 + 1] * Wq[bb * 3 + 1] + Wh[a * 3 + 2] * Wq[bb * 3 + 2];
                }
            }
            free(perm);
            /* + U_i with clamped, damped diagonal */
            const double* Ui = h->U + (size_t)i * D * D;
            for (int a = 0; a < D; ++a)
                for (int bb = 0; bb < D; ++bb) {
                    double u = Ui[a * D + bb];
                    if (a == bb && !h->u_predamped) u = clampd(u, h->cmin, h->cmax) * f;
                    Srow[a * D + bb] += u;
                }
            memcpy(h->b + (size_t)i * D, bi, sizeof(double) * D);
            for (int e = rb; e < re; ++e) slot[h->col[e]] = -1;
        }
        free(slot);
    }
}

/* w = S~ v using the upper storage of the scaled matrix; diagonal blocks of S~ are exactly I.
 * Row i: own upper blocks (j > i) + transposed blocks of rows j < i. */
static void spmv_scaled_d(ora_t* h, const double* v, double* w, int with_diag) {
    int D = h->D;
    #pragma omp parallel for schedule(static)
    for (int i = 0; i < h->C; ++i) {
        double acc[MAXD];
        for (int a = 0; a < D; ++a) acc[a] = with_diag ? v[(size_t)i * D + a] : 0.0;
        for (int e = h->row_ptr[i] + 1; e < h->row_ptr[i + 1]; ++e) {
            const double* blk = h->S + (size_t)e * D * D;
            const double* xj = v + (size_t)h->col[e] * D;
            for (int a = 0; a < D; ++a) {
                double s = 0;
                for (int bb = 0; bb < D; ++bb) s += blk[a * D + bb] * xj[bb];
                acc[a] += s;
            }
        }
        for (int e = h->lo_ptr[i]; e < h->lo_ptr[i + 1]; ++e) {
            const double* blk = h->S + (size_t)h->lo_blk[e] * D * D;
            const double* xj = v + (size_t)h->lo_col[e] * D;
            for (int a = 0; a < D; ++a) {
                double s = 0;
                for (int bb = 0; bb < D; ++bb) s += blk[bb * D + a] * xj[bb];
                acc[a] += s;
            }
        }
        for (int a = 0; a < D; ++a) w[(size_t)i * D + a] = acc[a];
    }
}
static void spmv_scaled(ora_t* h, const double* v, double* w) { spmv_scaled_d(h, v, w, 1); }

static int g_dot_reverse = 0;  /* set per solve from order_mode bit 1 (test yardstick) */
static double dot(const double* a, const double* b, size_t n, double* tmp) {
    for (size_t i = 0; i < n; ++i) tmp[i] = a[i] * b[i];
    return det_sum_order(tmp, n, g_dot_reverse);
}

/* Cholesky S_ii = L L^T (D x D, lower, row-major).  Returns -1 if not positive definite. */
static int chol(int n, const double* A, double* L) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) L[i * n + j] = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = A[i * n + j];
            for (int k = 0; k < j; ++k) s -= L[i * n + k] * L[j * n + k];
            if (i == j) {
                if (!(s > 0.0)) return -1;
                L[i * n + i] = sqrt(s);
            } else {
                L[i * n + j] = s / L[j * n + j];
            }
        }
    return 0;
}

/* inverse of a lower-triangular matrix (forward substitution per column) */
static void tri_inv(int n, const double* L, double* Li) {
    for (int i = 0; i < n * n; ++i) Li[i] = 0.0;
    for (int i = 0; i < n; ++i) {
        Li[i * n + i] = 1.0 / L[i * n + i];
        for (int j = 0; j < i; ++j) {
            double s = 0;
            for (int k = j; k < i; ++k) s -= L[i * n + k] * Li[k * n + j];
            Li[i * n + j] = s / L[i * n + i];
        }
    }
}

/* E^-1 in place by blocked Gauss-Jordan inversion, 32-wide blocks (the last one partial), the GPU's algorithm
 * (csrc/ba_twolevel.h k_gj_pinv0 / k_gj_step) with its fused multiply-adds -- the pivot update a - aip * rpc as
 * fma(-aip, rpc, a), every tile product as one fma chain in k order (v_mfma_f64_16x16x4f64 accumulates like that) --
 * so the two round alike: per block step k with pivot block P = A_kk
 *   P^-1 by scalar in-place Gauss-Jordan (pivots in order), A_kj <- P^-1 A_kj, A_ij <- A_ij - A_ik A_kj (new A_kj),
 *   A_ik <- -A_ik P^-1, A_kk <- P^-1.
 * Same pivot order and blocking as the GPU, so the two round alike (an ill-conditioned E amplifies the rounding of
 * a different inversion algorithm far beyond the PCG parity tolerance).  Returns -1 if a pivot is not positive. */
#define GJB 32
static int gj_inverse(int m, double* A) {
    double* P = (double*)malloc(sizeof(double) * GJB * GJB);
    double* Cc = (double*)malloc(sizeof(double) * (size_t)m * GJB);
    int bad = 0;
    for (int k0 = 0; k0 < m; k0 += GJB) {
        const int nk = (m - k0) < GJB ? (m - k0) : GJB;
        for (int r = 0; r < nk; ++r)
            for (int c = 0; c < nk; ++c) P[r * GJB + c] = A[(size_t)(k0 + r) * m + k0 + c];
        for (int p = 0; p < nk; ++p) {
            double piv = P[p * GJB + p];
            if (!(piv > 0.0)) { bad = 1; piv = 1.0; }
            const double inv = 1.0 / piv;
            double rp[GJB];
            for (int c = 0; c < nk; ++c) rp[c] = P[p * GJB + c] * inv;
            for (int r = 0; r < nk; ++r) {
                if (r == p) continue;
                const double aip = P[r * GJB + p];
                for (int c = 0; c < nk; ++c)
                    if (c != p) P[r * GJB + c] = fma(-aip, rp[c], P[r * GJB + c]);
                P[r * GJB + p] = -aip * inv;
            }
            for (int c = 0; c < nk; ++c)
                if (c != p) P[p * GJB + c] = rp[c];
            P[p * GJB + p] = inv;
        }
        /* old column tiles */
        for (int i = 0; i < m; ++i)
            for (int c = 0; c < nk; ++c) Cc[(size_t)i * GJB + c] = A[(size_t)i * m + k0 + c];
        /* row k: A_kj <- P^-1 A_kj */
        #pragma omp parallel for schedule(static)
        for (int j = 0; j < m; ++j) {
            if (j >= k0 && j < k0 + nk) continue;
            double col[GJB];
            for (int q = 0; q < nk; ++q) col[q] = A[(size_t)(k0 + q) * m + j];
            for (int r = 0; r < nk; ++r) {
                double s = 0.0;
                for (int q = 0; q < nk; ++q) s = fma(P[r * GJB + q], col[q], s);
                A[(size_t)(k0 + r) * m + j] = s;
            }
        }
        /* rows i outside block k */
        #pragma omp parallel for schedule(static)
        for (int i = 0; i < m; ++i) {
            if (i >= k0 && i < k0 + nk) continue;
            const double* ci = Cc + (size_t)i * GJB;
            double* Ai = A + (size_t)i * m;
            for (int j = 0; j < m; ++j) {
                if (j >= k0 && j < k0 + nk) continue;
                double s = Ai[j];
                for (int q = 0; q < nk; ++q) s = fma(-ci[q], A[(size_t)(k0 + q) * m + j], s);
                Ai[j] = s;
            }
            for (int c = 0; c < nk; ++c) {
                double s = 0.0;
                for (int q = 0; q < nk; ++q) s = fma(-ci[q], P[q * GJB + c], s);
                Ai[k0 + c] = s;
            }
        }
        for (int r = 0; r < nk; ++r)
            for (int c = 0; c < nk; ++c) A[(size_t)(k0 + r) * m + k0 + c] = P[r * GJB + c];
    }
    free(P); free(Cc);
    return bad ? -1 : 0;
}

/* Coarse operator of the two-level preconditioner (scaled space).  Z~_i = L_i^T G_i (D x MC) with G_i the coarse
 * basis of camera i at the linearization point; E = Z~^T S~ Z~ (m x m, m = nclust * MC), accumulated per camera row
 * in increasing row order: diagonal term Z~_i^T Z~_i, then for every upper block (i,j>i) Z~_i^T S~_ij Z~_j into
 * (c_i,c_j) and its transpose into (c_j,c_i).  A zero diagonal entry (unused column of a single-camera cluster)
 * becomes 1.  E^-1 is formed explicitly by blocked Gauss-Jordan inversion (gj_inverse) of the symmetrically
 * equilibrated E.  Returns 0 when E is not positive definite (the solve then runs with plain block-Jacobi). */
static int ora_coarse_setup(ora_t* h, const double* Lfac, double* Zt, double* Einv) {
    const int D = h->D, C = h->C, MC = D + 1, nc = h->nclust, m = nc * MC;
    const size_t DD = (size_t)D * D;
    for (int i = 0; i < C; ++i) {
        double G[MAXD * (MAXD + 1)];
        coarse_basis(D, h->lin_cams + (size_t)i * h->stride, h->csize[h->clab[i]] < 2, G, h->kind);
        const double* L = Lfac + (size_t)i * DD;
        double* Z = Zt + (size_t)i * D * MC;
        for (int a = 0; a < D; ++a)
            for (int k = 0; k < MC; ++k) {
                double s = 0;
                for (int l = a; l < D; ++l) s += L[l * D + a] * G[l * MC + k];
                Z[a * MC + k] = s;
            }
    }
    double* E = (double*)calloc((size_t)m * m, sizeof(double));
    for (int i = 0; i < C; ++i) {
        const double* Zi = Zt + (size_t)i * D * MC;
        const int ci = h->clab[i];
        for (int k = 0; k < MC; ++k)
            for (int l = 0; l < MC; ++l) {
                double s = 0;
                for (int a = 0; a < D; ++a) s += Zi[a * MC + k] * Zi[a * MC + l];
                E[(size_t)(ci * MC + k) * m + ci * MC + l] += s;
            }
        for (int e = h->row_ptr[i] + 1; e < h->row_ptr[i + 1]; ++e) {
            const int j = h->col[e], cj = h->clab[j];
            const double* B = h->S + (size_t)e * DD;
            const double* Zj = Zt + (size_t)j * D * MC;
            double T[MAXD * (MAXD + 1)];            /* T = S~_ij Z~_j  (D x MC) */
            for (int a = 0; a < D; ++a)
                for (int l = 0; l < MC; ++l) {
                    double s = 0;
                    for (int bb = 0; bb < D; ++bb) s += B[a * D + bb] * Zj[bb * MC + l];
                    T[a * MC + l] = s;
                }
            for (int k = 0; k < MC; ++k)
                for (int l = 0; l < MC; ++l) {
                    double s = 0;
                    for (int a = 0; a < D; ++a) s += Zi[a * MC + k] * T[a * MC + l];
                    E[(size_t)(ci * MC + k) * m + cj * MC + l] += s;
                    E[(size_t)(cj * MC + l) * m + ci * MC + k] += s;
                }
        }
    }
    for (int k = 0; k < m; ++k)
        if (E[(size_t)k * m + k] == 0.0) E[(size_t)k * m + k] = 1.0;
    /* symmetric equilibration d = 1 / sqrt(diag E) (the GPU's k_gj_equil; NaN for a non-positive diagonal, which
     * fails the first pivot test), then E^-1 = diag(d) (diag(d) E diag(d))^-1 diag(d) */
    double* dq = (double*)malloc(sizeof(double) * (size_t)m);
    for (int k = 0; k < m; ++k) dq[k] = 1.0 / sqrt(E[(size_t)k * m + k]);
    for (int r = 0; r < m; ++r)
        for (int q = 0; q < m; ++q) E[(size_t)r * m + q] = E[(size_t)r * m + q] * dq[r] * dq[q];
    int ok = gj_inverse(m, E) == 0;
    if (ok)
        for (int r = 0; r < m; ++r)
            for (int q = 0; q < m; ++q) Einv[(size_t)r * m + q] = E[(size_t)r * m + q] * dq[r] * dq[q];
    free(dq);
    free(E);
    return ok;
}

/* The coarse inverse exactly as ora_coarse_setup forms it (equilibration, gj_inverse, scaling back), exported for
 * the GPU kernels' bitwise test.  Returns 1 when E is positive definite, 0 when not. */
int ora_spd_inverse(int m, const double* E, double* Einv) {
    double* A = (double*)malloc(sizeof(double) * (size_t)m * m);
    double* dq = (double*)malloc(sizeof(double) * (size_t)m);
    for (int k = 0; k < m; ++k) dq[k] = 1.0 / sqrt(E[(size_t)k * m + k]);
    for (int r = 0; r < m; ++r)
        for (int q = 0; q < m; ++q) A[(size_t)r * m + q] = E[(size_t)r * m + q] * dq[r] * dq[q];
    const int ok = gj_inverse(m, A) == 0;
    for (int r = 0; r < m; ++r)
        for (int q = 0; q < m; ++q) Einv[(size_t)r * m + q] = A[(size_t)r * m + q] * dq[r] * dq[q];
    free(A); free(dq);
    return ok;
}

/* u = v + Z~ E^-1 Z~^T r (v null: u = Z~ E^-1 Z~^T r).  Restriction per cluster sums camera rows in increasing camera
 * order. */
static void coarse_apply_v(ora_t* h, const double* Zt, const double* Einv, double* Rc, double* yc, const double* r,
                           const double* v, double* u) {
    const int D = h->D, C = h->C, MC = D + 1, m = h->nclust * MC;
    for (int k = 0; k < m; ++k) Rc[k] = 0.0;
    for (int i = 0; i < C; ++i) {
        const double* Zi = Zt + (size_t)i * D * MC;
        const double* ri = r + (size_t)i * D;
        double* R = Rc + (size_t)h->clab[i] * MC;
        for (int k = 0; k < MC; ++k) {
            double s = 0;
            for (int a = 0; a < D; ++a) s += Zi[a * MC + k] * ri[a];
            R[k] += s;
        }
    }
    #pragma omp parallel for schedule(static)
    for (int k = 0; k < m; ++k) {
        double s = 0;
        for (int l = 0; l < m; ++l) s += Einv[(size_t)k * m + l] * Rc[l];
        yc[k] = s;
    }
    #pragma omp parallel for schedule(static)
    for (int i = 0; i < C; ++i) {
        const double* Zi = Zt + (size_t)i * D * MC;
        const double* y = yc + (size_t)h->clab[i] * MC;
        for (int a = 0; a < D; ++a) {
            double s = 0;
            for (int k = 0; k < MC; ++k) s += Zi[a * MC + k] * y[k];
            u[(size_t)i * D + a] = v ? v[(size_t)i * D + a] + s : s;
        }
    }
}
/* the additive two-level preconditioner (precond 1): u = r + Z~ E^-1 Z~^T r */
static void coarse_apply(ora_t* h, const double* Zt, const double* Einv, double* Rc, double* yc, const double* r,
                         double* u) {
    coarse_apply_v(h, Zt, Einv, Rc, yc, r, r, u);
}
/* A-DEF2 (precond 2; Tang, Nabben, Vuik & Erlangga 2009): u = P^T r + Q r = r + Z~ E^-1 Z~^T (r - S~ r), with
 * r - S~ r = -(the off-diagonal part of S~ r) (the diagonal blocks of S~ are I); t: scratch [C * D] */
static void adef2_apply(ora_t* h, const double* Zt, const double* Einv, double* Rc, double* yc, const double* r,
                        double* u, double* t) {
    const size_t n = (size_t)h->C * h->D;
    spmv_scaled_d(h, r, t, 0);
    for (size_t e = 0; e < n; ++e) t[e] = -t[e];
    coarse_apply_v(h, Zt, Einv, Rc, yc, t, r, u);
}

/* Block-Jacobi (precond 0) or two-level (precond 1) PCG on S x = b, as conjugate gradients on the symmetrically scaled system
 * S~ = L^-1 S L^-T (S_ii = L_i L_i^T, so diag blocks of S~ are I) with the single-reduction
 * Chronopoulos-Gear recurrence.  In exact arithmetic this is the standard block-Jacobi PCG;
 * convergence is tested on the true residual ||b - S x|| = ||L r~|| <= tol ||b||, x0 = 0.
 * S is scaled in place.  Returns iterations >= 0, or -1 on breakdown (solver failure). */
int ora_pcg(ora_t* h, double* xout) {
    int D = h->D, C = h->C;
    g_dot_reverse = (h->order_mode & 2) != 0;
    size_t n = (size_t)C * D;
    size_t DD = (size_t)D * D;
    int bad = 0;
    /* h->Minv holds L_i^-1; L_i kept in a scratch array */
    double* Lfac = (double*)malloc(sizeof(double) * (size_t)C * DD);
    #pragma omp parallel for schedule(static) reduction(|:bad)
    for (int i = 0; i < C; ++i) {
        const double* blk = h->S + (size_t)h->row_ptr[i] * DD; /* diagonal block is first in row */
        if (chol(D, blk, Lfac + (size_t)i * DD)) { bad = 1; continue; }
        tri_inv(D, Lfac + (size_t)i * DD, h->Minv + (size_t)i * DD);
    }
    if (bad) { free(Lfac); return -1; }
    /* S~_ij = Li^-1 S_ij Lj^-T for off-diagonal upper blocks; diag = I */
    #pragma omp parallel for schedule(dynamic, 4)
    for (int i = 0; i < C; ++i) {
        const double* Li = h->Minv + (size_t)i * DD;
        for (int e = h->row_ptr[i]; e < h->row_ptr[i + 1]; ++e) {
            double* blk = h->S + (size_t)e * DD;
            if (e == h->row_ptr[i]) {
                for (int a = 0; a < D; ++a) for (int bb = 0; bb < D; ++bb) blk[a * D + bb] = (a == bb) ? 1.0 : 0.0;
                continue;
            }
            const double* Lj = h->Minv + (size_t)h->col[e] * DD;
            double T[MAXD * MAXD];
            for (int a = 0; a < D; ++a)           /* T = Li^-1 S_ij (Li^-1 lower: k <= a) */
                for (int bb = 0; bb < D; ++bb) {
                    double s = 0;
                    for (int k = 0; k <= a; ++k) s += Li[a * D + k] * blk[k * D + bb];
                    T[a * D + bb] = s;
                }
            for (int a = 0; a < D; ++a)           /* blk = T Lj^-T : (T Lj^-T)_ab = sum_k T_ak Lj^-1_bk, k <= b */
                for (int bb = 0; bb < D; ++bb) {
                    double s = 0;
                    for (int k = 0; k <= bb; ++k) s += T[a * D + k] * Lj[bb * D + k];
                    blk[a * D + bb] = s;
                }
        }
    }
    double* tmp = h->partial;
    double* w = h->q;
    double* sv = h->z;
    double* rt = (double*)malloc(sizeof(double) * n);
    /* two-level preconditioner M~^-1 = I + Z~ E^-1 Z~^T in the scaled space (block-Jacobi + coarse correction) */
    const int MC = D + 1, nc = h->nclust, m = nc * MC;
    int twolev = h->precond >= 1 && nc > 0;
    /* precond 2: the coarse correction as A-DEF2 (u = r + Z~ E^-1 Z~^T (r - S~ r)) started from the coarse solution
     * x0 = Z~ E^-1 Z~^T r0 (with that start A-DEF2 has BNN's iterates in exact arithmetic, which keeps the
     * single-reduction recurrence sound; from x0 = 0 it broke down on config 3).  Config 3, 10 LM steps: 213 -> 111
     * iterations, the same RMSE. */
    int adef2 = h->precond == 2;
    double* tdef = adef2 ? (double*)malloc(sizeof(double) * n) : NULL;
    const int pipelined = twolev;  /* the two-level path uses the pipelined recurrence (with or without a usable E) */
    double *Zt = NULL, *Einv = NULL, *Rc = NULL, *yc = NULL, *u = h->r;
    if (twolev) {
        Zt = (double*)malloc(sizeof(double) * (size_t)C * D * MC);
        Einv = (double*)malloc(sizeof(double) * (size_t)m * m);
        Rc = (double*)malloc(sizeof(double) * (size_t)m);
        yc = (double*)malloc(sizeof(double) * (size_t)m);
        u = (double*)malloc(sizeof(double) * n);
        /* Lag rule: the first solve after a linearization runs with the coarse inverse of the previous solve, so the
         * GPU factorizes E_k on a side stream while that CG runs; later solves at the same linearization (rejected LM
         * trials, whose damping can jump by 16x per retry) and the very first solve use their own E.  Any SPD E^-1
         * keeps M~ SPD, so the lag only changes the iteration count (a few percent). */
        int okc = ora_coarse_setup(h, Lfac, Zt, Einv);
        if (!h->prev_einv) h->prev_einv = (double*)malloc(sizeof(double) * (size_t)m * m);
        if (h->have_prev && h->fresh_lin) {
            for (size_t e = 0; e < (size_t)m * m; ++e) { double tmp = Einv[e]; Einv[e] = h->prev_einv[e]; h->prev_einv[e] = tmp; }
            int o = h->prev_ok; h->prev_ok = okc; okc = o;
        } else {
            memcpy(h->prev_einv, Einv, sizeof(double) * (size_t)m * m);
            h->prev_ok = okc;
            h->have_prev = 1;
        }
        h->fresh_lin = 0;
        if (!okc) twolev = 0;
    }
    /* A-DEF2 breakdown (the recurrence's denominator <= 0: possible under the lag rule, whose E^-1 is the previous
     * solve's, so Z~^T r is not exactly zeroed by the coarse start): the solve is repeated from r0 with the additive
     * correction (pass 1), as the GPU's adef2_fallback does. */
    for (int pass = 0;; ++pass) {
    for (int i = 0; i < C; ++i) {
        const double* Li = h->Minv + (size_t)i * DD;
        for (int a = 0; a < D; ++a) {
            double s = 0;
            for (int k = 0; k <= a; ++k) s += Li[a * D + k] * h->b[(size_t)i * D + k];
            h->r[(size_t)i * D + a] = s;
        }
    }
    for (size_t e = 0; e < n; ++e) { h->x[e] = 0; h->p[e] = 0; sv[e] = 0; }
    if (twolev && adef2) {  /* x0 = Z~ E^-1 Z~^T r0; r0 -= x0 + off(S~) x0 */
        coarse_apply_v(h, Zt, Einv, Rc, yc, h->r, NULL, h->x);
        spmv_scaled_d(h, h->x, tdef, 0);
        for (size_t e = 0; e < n; ++e) h->r[e] = h->r[e] - h->x[e] - tdef[e];
    }
    if (twolev) {
        if (adef2) adef2_apply(h, Zt, Einv, Rc, yc, h->r, u, tdef);
        else coarse_apply(h, Zt, Einv, Rc, yc, h->r, u);
    }
    spmv_scaled(h, u, w);
    double bb2 = dot(h->b, h->b, n, tmp);
    if (pipelined) {
        /* Pipelined PCG (Ghysels & Vanroose 2014, preconditioned variant): the same iterates as PCG in exact
         * arithmetic, with the preconditioner and the operator applied to w (m = M~^-1 w, n = S~ m) so that every
         * iteration needs ONE reduction phase (gamma, delta, rho, and the coarse restriction of w) followed by one
         * coarse solve and one SpMV; the GPU runs it as two kernels per iteration (k_tl_pc + k_tl_pspmv). */
        double *mv = (double*)malloc(sizeof(double) * n), *nv = (double*)malloc(sizeof(double) * n);
        double *qv = (double*)calloc(n, sizeof(double)), *zv = (double*)calloc(n, sizeof(double));
        double gam = dot(h->r, u, n, tmp), del = dot(w, u, n, tmp), rho = bb2;
        double gam_prev = 1.0, alpha_prev = 1.0;
        double tol2 = h->pcg_tol * h->pcg_tol * bb2;
        int k = 0, fail = 0;
        for (;; ++k) {
            if (rho <= tol2 || k >= h->pcg_max_iter) break;
            double alpha, beta, den;
            if (k == 0) { beta = 0.0; den = del; }
            else { beta = gam / gam_prev; den = del - beta * gam / alpha_prev; }
            if (!(den > 0.0)) { fail = 1; break; }
            alpha = gam / den;
            if (twolev) {
                if (adef2) adef2_apply(h, Zt, Einv, Rc, yc, w, mv, tdef);
                else coarse_apply(h, Zt, Einv, Rc, yc, w, mv);
            } else {
                memcpy(mv, w, sizeof(double) * n);
            }
            spmv_scaled(h, mv, nv);
            for (size_t e = 0; e < n; ++e) {
                zv[e] = nv[e] + beta * zv[e];
                qv[e] = mv[e] + beta * qv[e];
                sv[e] = w[e] + beta * sv[e];
                h->p[e] = u[e] + beta * h->p[e];
                h->x[e] += alpha * h->p[e];
                h->r[e] -= alpha * sv[e];
                u[e] -= alpha * qv[e];
                w[e] -= alpha * zv[e];
            }
            gam_prev = gam; alpha_prev = alpha;
            gam = dot(h->r, u, n, tmp);
            del = dot(w, u, n, tmp);
            for (int i = 0; i < C; ++i) {
                const double* L = Lfac + (size_t)i * DD;
                for (int a = 0; a < D; ++a) {
                    double s = 0;
                    for (int kk = 0; kk <= a; ++kk) s += L[a * D + kk] * h->r[(size_t)i * D + kk];
                    rt[(size_t)i * D + a] = s;
                }
            }
            rho = dot(rt, rt, n, tmp);
        }
        free(mv); free(nv); free(qv); free(zv);
        if (fail && twolev && adef2 && pass == 0) {
            adef2 = 0;
            h->adef2_fallbacks++;
            continue;
        }
        free(tdef);
        free(rt);
        free(Lfac);
        if (Zt) { free(Zt); free(Einv); free(Rc); free(yc); free(u); }
        h->stats[7] = twolev;
        if (fail) return -1;
        for (int i = 0; i < C; ++i) {
            const double* Li = h->Minv + (size_t)i * DD;
            for (int a = 0; a < D; ++a) {
                double s = 0;
                for (int kk = a; kk < D; ++kk) s += Li[kk * D + a] * h->x[(size_t)i * D + kk];
                xout[(size_t)i * D + a] = s;
            }
        }
        return k;
    }
    double gam = dot(h->r, u, n, tmp), del = dot(w, u, n, tmp), rho = bb2;
    double gam_prev = 1.0, alpha_prev = 1.0;
    double tol2 = h->pcg_tol * h->pcg_tol * bb2;
    int k = 0, fail = 0;
    for (;; ++k) {
        if (rho <= tol2 || k >= h->pcg_max_iter) break;
        double alpha, beta, den;
        if (k == 0) { beta = 0.0; den = del; }
        else { beta = gam / gam_prev; den = del - beta * gam / alpha_prev; }
        if (!(den > 0.0)) { fail = 1; break; }
        alpha = gam / den;
        for (size_t e = 0; e < n; ++e) {
            h->p[e] = u[e] + beta * h->p[e];
            sv[e] = w[e] + beta * sv[e];
            h->x[e] += alpha * h->p[e];
            h->r[e] -= alpha * sv[e];
        }
        if (twolev) coarse_apply(h, Zt, Einv, Rc, yc, h->r, u);
        spmv_scaled(h, u, w);
        gam_prev = gam; alpha_prev = alpha;
        gam = dot(h->r, u, n, tmp);
        del = dot(w, u, n, tmp);
        /* true residual norm^2 = ||L r~||^2 */
        for (int i = 0; i < C; ++i) {
            const double* L = Lfac + (size_t)i * DD;
            for (int a = 0; a < D; ++a) {
                double s = 0;
                for (int kk = 0; kk <= a; ++kk) s += L[a * D + kk] * h->r[(size_t)i * D + kk];
                rt[(size_t)i * D + a] = s;
            }
        }
        rho = dot(rt, rt, n, tmp);
    }
    free(tdef);
    free(rt);
    free(Lfac);
    if (Zt) { free(Zt); free(Einv); free(Rc); free(yc); free(u); }
    h->stats[7] = twolev;
    if (fail) return -1;
    /* x = L^-T x~ */
    for (int i = 0; i < C; ++i) {
        const double* Li = h->Minv + (size_t)i * DD;
        for (int a = 0; a < D; ++a) {
            double s = 0;
            for (int kk = a; kk < D; ++kk) s += Li[kk * D + a] * h->x[(size_t)i * D + kk];
            xout[(size_t)i * D + a] = s;
        }
    }
    return k;
    }  /* (pass) */
}

/* back-substitution: dp = Vinv (g_p - sum_o W_o^T dc_{c(o)}) */
static void backsub(ora_t* h, const double* dc) {
    int D = h->D;
    #pragma omp parallel for schedule(static)
    for (int p = 0; p < h->P; ++p) {
        double t[3];
        for (int k = 0; k < 3; ++k) t[k] = h->gp[3 * (size_t)p + k];
        if (dc) {
            for (int o = h->pt_ptr[p]; o < h->pt_ptr[p + 1]; ++o) {
                const double* Wo = h->W + (size_t)o * D * 3;
                const double* d = dc + (size_t)h->cam[o] * D;
                for (int k = 0; k < 3; ++k) {
                    double s = 0;
                    for (int a = 0; a < D; ++a) s += Wo[a * 3 + k] * d[a];
                    t[k] -= s;
                }
            }
        }
        const double* Vi = h->Vinv + 9 * (size_t)p;
        for (int k = 0; k < 3; ++k) h->dp[3 * (size_t)p + k] = Vi[k * 3 + 0] * t[0] + Vi[k * 3 + 1] * t[1] + Vi[k * 3 + 2] * t[2];
    }
}

/* predicted-change term -((J~D)^T (2 r~ + J~D)) evaluated per observation at the linearization point */
static double model_decrease(ora_t* h, const double* cams, const double* pts, const double* dc) {
    int D = h->D;
    double* e = h->partial;
    double delta = h->delta;
    #pragma omp parallel for schedule(static)
    for (int o = 0; o < h->N; ++o) {
        int c = h->cam[o], p = h->pt[o];
        double r[2], Jc[2 * MAXD], Jp[6];
        ora_eval_one(h->model, cams + (size_t)c * h->stride, pts + 3 * (size_t)p, h->pp + 2 * (size_t)c, h->uv + 2 * (size_t)o, r, Jc, Jp, NULL);
        double s = r[0] * r[0] + r[1] * r[1];
        double wgt = sqrt(s) < delta ? 1.0 : delta / sqrt(s);
        double sw = sqrt(wgt);
        double jd[2];
        for (int a = 0; a < 2; ++a) {
            double v = 0;
            if (dc) for (int k = 0; k < D; ++k) v += Jc[a * D + k] * dc[(size_t)c * D + k];
            for (int k = 0; k < 3; ++k) v += Jp[a * 3 + k] * h->dp[3 * (size_t)p + k];
            jd[a] = sw * v;
        }
        e[o] = jd[0] * (2.0 * sw * r[0] + jd[0]) + jd[1] * (2.0 * sw * r[1] + jd[1]);
    }
    return -det_sum(e, h->N);
}

/* Build (without solving) the reduced camera system S (upper blocks, unscaled) and b for factor f. */
int ora_build_reduced(ora_t* h, double f) {
    if (prep_points(h, f)) return -1;
    ora_schur(h, f);
    return 0;
}

/* Solve the damped system for factor f; fills h->x (dc) and h->dp.  Returns pcg iterations or -1. */
int ora_solve(ora_t* h, double f) {
    if (prep_points(h, f)) return -1;
    int it = 0;
    if (h->optimize_poses) {
        ora_schur(h, f);
        it = ora_pcg(h, h->x);
        if (it < 0) return -1;
        backsub(h, h->x);
    } else {
        backsub(h, NULL);
    }
    return it;
}

/* One LM step (bae.optim.LM.step as reconstructed in SURVEY.md 3.3).  cams/pts updated in place.
 * Returns 0; *loss_out = loss after the step (== previous loss when the linear solver failed). */
int ora_step(ora_t* h, double* cams, double* pts, double* loss_out) {
    int C = h->C, P = h->P, D = h->D, st = h->stride;
    if (!h->have_loss) { h->loss = ora_cost(h, cams, pts, NULL); h->have_loss = 1; }
    double last = h->loss;
    ora_linearize(h, cams, pts);
    h->adef2_fallbacks = 0;
    double f = 1.0;
    int rejects = 0, trials = 0, pcg_total = 0, pcg_last = 0, failed = 0;
    for (;;) {
        f *= (1.0 + h->damping);
        int it = ora_solve(h, f);
        trials++;
        if (it < 0) { failed = 1; h->loss = last; break; }
        pcg_last = it; pcg_total += it;
        for (int c = 0; c < C; ++c) {
            const double* xc = cams + (size_t)c * st;
            double* nc = h->cams_new + (size_t)c * st;
            if (h->optimize_poses) {
                const double* d = h->x + (size_t)c * D;
                ora_retract_pose(xc, d, nc);
                for (int k = 0; k < h->ni; ++k) nc[7 + k] = xc[7 + k] + d[6 + k];
            } else {
                memcpy(nc, xc, sizeof(double) * st);
            }
        }
        for (size_t k = 0; k < (size_t)P * 3; ++k) h->pts_new[k] = pts[k] + h->dp[k];
        double loss_new = ora_cost(h, h->cams_new, h->pts_new, NULL);
        double denom = model_decrease(h, cams, pts, h->optimize_poses ? h->x : NULL);
        double quality = (last - loss_new) / denom;
        /* pypose TrustRegion.update */
        double radius = 1.0 / h->damping;
        if (quality > h->high) { radius = h->up * radius; h->down = h->down0; }
        else if (quality > h->low) { h->down = h->down0; }
        else { radius = radius * h->down; h->down = h->down * h->factor; }
        radius = clampd(radius, h->rmin, h->rmax);
        h->damping = 1.0 / radius;
        if (last < loss_new && rejects < h->max_rejects) {
            rejects++;
            h->loss = last;
            continue;
        }
        memcpy(cams, h->cams_new, sizeof(double) * (size_t)C * st);
        memcpy(pts, h->pts_new, sizeof(double) * (size_t)P * 3);
        h->loss = loss_new;
        break;
    }
    h->stats[0] = trials; h->stats[1] = pcg_last; h->stats[2] = pcg_total; h->stats[3] = f;
    h->stats[4] = h->damping; h->stats[5] = failed; h->stats[6] = rejects; h->stats[8] = h->adef2_fallbacks;
    *loss_out = h->loss;
    return 0;
}


/* ------------------------------------------------------------------------------------------ */
/* global positioning (TorchGP.Optimize, global_positioning.py:45-206)                         */
/* ------------------------------------------------------------------------------------------ */
/* Residual per observation o (pairwise_cost, cost_function.py:22-29):
 *     r_o = f_o (t_o - s_o (X_p - c_c))          (3-D; f_o = 1 calibrated camera, 0.5 otherwise)
 * Parameters: camera positions c [C,3], points X [P,3], per-observation scales s [N] (those with a valid depth are
 * fixed: TorchGP's scale_indices / depth_only).  LM as bundle adjustment (Huber + Triggs, diag clamp, cumulative
 * damping, TrustRegion, rejects), additive updates.  Linear solve: with the weighted Jacobian rows
 *     J_c = beta I,  J_X = -beta I,  J_s = a = -f (X - c) sqrt(w),   beta = s f sqrt(w)
 * the scale blocks (1x1) are eliminated first (h_ss = clamp(a.a) * damping), which leaves, per observation, the
 * camera-point block W_o = -beta^2 (I - a a^T / h_ss) and rank-1 corrections of the damped camera and point diagonals;
 * the points are then eliminated exactly as in bundle adjustment (S = U' - sum W V^-1 W^T, D = 3), the reduced
 * camera system is solved by the same PCG, and the back-substitution also returns the scale steps. */
ora_t* ora_gp_create(int C, int P, int N, const double* trans, const int* cam, const int* pt, const double* fcam,
                     const int* sfree, const double* dopt, const int* iopt) {
    ora_t* h = ora_create(ORA_GP, C, P, N, NULL, cam, pt, NULL, dopt, iopt);
    if (!h) return NULL;
    h->u_predamped = 1;
    h->gp_t = (double*)malloc(sizeof(double) * 3 * (size_t)N); memcpy(h->gp_t, trans, sizeof(double) * 3 * (size_t)N);
    h->gp_f = (double*)malloc(sizeof(double) * (size_t)N);
    for (int o = 0; o < N; ++o) h->gp_f[o] = fcam[cam[o]];
    h->gp_sfree = (int*)malloc(sizeof(int) * (size_t)N); memcpy(h->gp_sfree, sfree, sizeof(int) * (size_t)N);
    h->gp_beta = (double*)malloc(sizeof(double) * (size_t)N);
    h->gp_a = (double*)malloc(sizeof(double) * 3 * (size_t)N);
    h->gp_r = (double*)malloc(sizeof(double) * 3 * (size_t)N);
    h->gp_hss = (double*)malloc(sizeof(double) * (size_t)N);
    h->gp_gs = (double*)malloc(sizeof(double) * (size_t)N);
    h->gp_ds = (double*)malloc(sizeof(double) * (size_t)N);
    h->gp_hx = (double*)malloc(sizeof(double) * (size_t)P);
    h->gp_hc = (double*)malloc(sizeof(double) * (size_t)C);
    h->gp_gx = (double*)malloc(sizeof(double) * 3 * (size_t)P);
    h->gp_gc = (double*)malloc(sizeof(double) * 3 * (size_t)C);
    h->gp_scales_new = (double*)malloc(sizeof(double) * (size_t)N);
    return h;
}

static void gp_residual(const ora_t* h, int o, const double* cams, const double* pts, const double* scales, double r[3],
                        double e[3]) {
    const double* c = cams + 3 * (size_t)h->cam[o];
    const double* X = pts + 3 * (size_t)h->pt[o];
    const double* t = h->gp_t + 3 * (size_t)o;
    const double f = h->gp_f[o], s = scales[o];
    for (int k = 0; k < 3; ++k) {
        e[k] = X[k] - c[k];
        r[k] = f * (t[k] - s * e[k]);
    }
}

double ora_gp_cost(ora_t* h, const double* cams, const double* pts, const double* scales, double* sq_out) {
    double* e2 = h->partial;
    double* q2 = h->partial + h->N;
    const double delta = h->delta;
    #pragma omp parallel for schedule(static)
    for (int o = 0; o < h->N; ++o) {
        double r[3], e[3];
        gp_residual(h, o, cams, pts, scales, r, e);
        const double s = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
        e2[o] = sqrt(s) < delta ? s : 2.0 * delta * sqrt(s) - delta * delta;
        q2[o] = s;
    }
    double loss = det_sum(e2, h->N);
    if (sq_out) *sq_out = det_sum(q2, h->N);
    return loss;
}

void ora_gp_linearize(ora_t* h, const double* cams, const double* pts, const double* scales) {
    h->fresh_lin = 1;
    if (!h->lin_cams) h->lin_cams = (double*)malloc(sizeof(double) * (size_t)h->C * 3);
    memcpy(h->lin_cams, cams, sizeof(double) * (size_t)h->C * 3);
    const double delta = h->delta;
    #pragma omp parallel for schedule(static)
    for (int o = 0; o < h->N; ++o) {
        double r[3], e[3];
        gp_residual(h, o, cams, pts, scales, r, e);
        const double s2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
        const double wgt = sqrt(s2) < delta ? 1.0 : delta / sqrt(s2);
        const double sw = sqrt(wgt);
        const double f = h->gp_f[o];
        h->gp_beta[o] = scales[o] * f * sw;
        for (int k = 0; k < 3; ++k) {
            h->gp_r[3 * (size_t)o + k] = sw * r[k];
            h->gp_a[3 * (size_t)o + k] = h->gp_sfree[o] ? -f * e[k] * sw : 0.0;
        }
    }
    #pragma omp parallel for schedule(static)
    for (int p = 0; p < h->P; ++p) {
        double hx = 0, g[3] = {0, 0, 0};
        for (int o = h->pt_ptr[p]; o < h->pt_ptr[p + 1]; ++o) {
            const double b = h->gp_beta[o];
            hx += b * b;
            for (int k = 0; k < 3; ++k) g[k] += b * h->gp_r[3 * (size_t)o + k];
        }
        h->gp_hx[p] = hx;
        for (int k = 0; k < 3; ++k) h->gp_gx[3 * (size_t)p + k] = g[k];
    }
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < h->C; ++c) {
        double hc = 0, g[3] = {0, 0, 0};
        for (int e = h->cam_ptr[c]; e < h->cam_ptr[c + 1]; ++e) {
            const int o = h->cam_obs[e];
            const double b = h->gp_beta[o];
            hc += b * b;
            for (int k = 0; k < 3; ++k) g[k] -= b * h->gp_r[3 * (size_t)o + k];
        }
        h->gp_hc[c] = hc;
        for (int k = 0; k < 3; ++k) h->gp_gc[3 * (size_t)c + k] = g[k];
    }
}

/* Damped system after the scale elimination: W_o, V_p (packed sym), g'_x (into gp), U'_c (into U), g'_c (into gc). */
static void gp_prep(ora_t* h, double f) {
    #pragma omp parallel for schedule(static)
    for (int o = 0; o < h->N; ++o) {
        const double* a = h->gp_a + 3 * (size_t)o;
        const double* r = h->gp_r + 3 * (size_t)o;
        const double b2 = h->gp_beta[o] * h->gp_beta[o];
        double hss = 0.0, gs = 0.0;
        if (h->gp_sfree[o]) {
            hss = clampd(a[0] * a[0] + a[1] * a[1] + a[2] * a[2], h->cmin, h->cmax) * f;
            gs = -(a[0] * r[0] + a[1] * r[1] + a[2] * r[2]);
        }
        h->gp_hss[o] = hss;
        h->gp_gs[o] = gs;
        double* Wo = h->W + (size_t)o * 9;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                const double q = (i == j ? 1.0 : 0.0) - (hss > 0.0 ? a[i] * a[j] / hss : 0.0);
                Wo[i * 3 + j] = -b2 * q;
            }
    }
    #pragma omp parallel for schedule(static)
    for (int p = 0; p < h->P; ++p) {
        const double d = clampd(h->gp_hx[p], h->cmin, h->cmax) * f;
        double Vs[6] = {d, 0, 0, d, 0, d};
        double g[3];
        for (int k = 0; k < 3; ++k) g[k] = h->gp_gx[3 * (size_t)p + k];
        for (int o = h->pt_ptr[p]; o < h->pt_ptr[p + 1]; ++o) {
            const double hss = h->gp_hss[o];
            if (!(hss > 0.0)) continue;
            const double* a = h->gp_a + 3 * (size_t)o;
            const double b = h->gp_beta[o], c2 = b * b / hss, cg = b * h->gp_gs[o] / hss;
            Vs[0] -= c2 * a[0] * a[0]; Vs[1] -= c2 * a[0] * a[1]; Vs[2] -= c2 * a[0] * a[2];
            Vs[3] -= c2 * a[1] * a[1]; Vs[4] -= c2 * a[1] * a[2]; Vs[5] -= c2 * a[2] * a[2];
            for (int k = 0; k < 3; ++k) g[k] += cg * a[k];
        }
        memcpy(h->V + 6 * (size_t)p, Vs, sizeof(Vs));
        for (int k = 0; k < 3; ++k) h->gp[3 * (size_t)p + k] = g[k];
    }
    #pragma omp parallel for schedule(static)
    for (int c = 0; c < h->C; ++c) {
        const double d = clampd(h->gp_hc[c], h->cmin, h->cmax) * f;
        double Uc[9] = {d, 0, 0, 0, d, 0, 0, 0, d};
        double g[3];
        for (int k = 0; k < 3; ++k) g[k] = h->gp_gc[3 * (size_t)c + k];
        for (int e = h->cam_ptr[c]; e < h->cam_ptr[c + 1]; ++e) {
            const int o = h->cam_obs[e];
            const double hss = h->gp_hss[o];
            if (!(hss > 0.0)) continue;
            const double* a = h->gp_a + 3 * (size_t)o;
            const double b = h->gp_beta[o], c2 = b * b / hss, cg = b * h->gp_gs[o] / hss;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) Uc[i * 3 + j] -= c2 * a[i] * a[j];
            for (int k = 0; k < 3; ++k) g[k] -= cg * a[k];
        }
        memcpy(h->U + 9 * (size_t)c, Uc, sizeof(Uc));
        memcpy(h->gc + 3 * (size_t)c, g, sizeof(g));
    }
}

/* V^-1, y = V^-1 g'_x for the (already damped) point blocks. */
static int gp_prep_points(ora_t* h) {
    int bad = 0;
    #pragma omp parallel for schedule(static) reduction(|:bad)
    for (int p = 0; p < h->P; ++p) {
        double full[9], inv[9];
        sym3_full(h->V + 6 * (size_t)p, full);
        if (spd_inverse(3, full, inv)) { bad = 1; continue; }
        memcpy(h->Vinv + 9 * (size_t)p, inv, sizeof(inv));
        const double* g = h->gp + 3 * (size_t)p;
        for (int k = 0; k < 3; ++k) h->y[3 * (size_t)p + k] = inv[k * 3 + 0] * g[0] + inv[k * 3 + 1] * g[1] + inv[k * 3 + 2] * g[2];
    }
    return bad ? -1 : 0;
}

/* scale steps: ds_o = (g_s - beta a.(dc_c - dX_p)) / h_ss */
static void gp_scale_steps(ora_t* h, const double* dc) {
    #pragma omp parallel for schedule(static)
    for (int o = 0; o < h->N; ++o) {
        const double hss = h->gp_hss[o];
        if (!(hss > 0.0)) { h->gp_ds[o] = 0.0; continue; }
        const double* a = h->gp_a + 3 * (size_t)o;
        const double* d = dc + 3 * (size_t)h->cam[o];
        const double* dX = h->dp + 3 * (size_t)h->pt[o];
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += a[k] * (d[k] - dX[k]);
        h->gp_ds[o] = (h->gp_gs[o] - h->gp_beta[o] * s) / hss;
    }
}

int ora_gp_solve(ora_t* h, double f) {
    gp_prep(h, f);
    if (gp_prep_points(h)) return -1;
    ora_schur(h, f);
    int it = ora_pcg(h, h->x);
    if (it < 0) return -1;
    backsub(h, h->x);
    gp_scale_steps(h, h->x);
    return it;
}

static double gp_model_decrease(ora_t* h) {
    double* e = h->partial;
    #pragma omp parallel for schedule(static)
    for (int o = 0; o < h->N; ++o) {
        const double* a = h->gp_a + 3 * (size_t)o;
        const double* r = h->gp_r + 3 * (size_t)o;
        const double* d = h->x + 3 * (size_t)h->cam[o];
        const double* dX = h->dp + 3 * (size_t)h->pt[o];
        const double b = h->gp_beta[o], ds = h->gp_ds[o];
        double acc = 0.0;
        for (int k = 0; k < 3; ++k) {
            const double jd = b * (d[k] - dX[k]) + a[k] * ds;
            acc += jd * (2.0 * r[k] + jd);
        }
        e[o] = acc;
    }
    return -det_sum(e, h->N);
}

/* One LM step of TorchGP's optimizer (LM semantics as ora_step); cams [C,3], pts [P,3], scales [N] in place. */
int ora_gp_step(ora_t* h, double* cams, double* pts, double* scales, double* loss_out) {
    const int C = h->C, P = h->P, N = h->N;
    if (!h->have_loss) { h->loss = ora_gp_cost(h, cams, pts, scales, NULL); h->have_loss = 1; }
    const double last = h->loss;
    ora_gp_linearize(h, cams, pts, scales);
    h->adef2_fallbacks = 0;
    double f = 1.0;
    int rejects = 0, trials = 0, pcg_total = 0, pcg_last = 0, failed = 0;
    for (;;) {
        f *= (1.0 + h->damping);
        const int it = ora_gp_solve(h, f);
        trials++;
        if (it < 0) { failed = 1; h->loss = last; break; }
        pcg_last = it; pcg_total += it;
        for (size_t k = 0; k < (size_t)C * 3; ++k) h->cams_new[k] = cams[k] + h->x[k];
        for (size_t k = 0; k < (size_t)P * 3; ++k) h->pts_new[k] = pts[k] + h->dp[k];
        for (int o = 0; o < N; ++o) h->gp_scales_new[o] = scales[o] + h->gp_ds[o];
        const double loss_new = ora_gp_cost(h, h->cams_new, h->pts_new, h->gp_scales_new, NULL);
        const double denom = gp_model_decrease(h);
        const double quality = (last - loss_new) / denom;
        double radius = 1.0 / h->damping;
        if (quality > h->high) { radius = h->up * radius; h->down = h->down0; }
        else if (quality > h->low) { h->down = h->down0; }
        else { radius = radius * h->down; h->down = h->down * h->factor; }
        radius = clampd(radius, h->rmin, h->rmax);
        h->damping = 1.0 / radius;
        if (last < loss_new && rejects < h->max_rejects) {
            rejects++;
            h->loss = last;
            continue;
        }
        memcpy(cams, h->cams_new, sizeof(double) * (size_t)C * 3);
        memcpy(pts, h->pts_new, sizeof(double) * (size_t)P * 3);
        memcpy(scales, h->gp_scales_new, sizeof(double) * (size_t)N);
        h->loss = loss_new;
        break;
    }
    h->stats[0] = trials; h->stats[1] = pcg_last; h->stats[2] = pcg_total; h->stats[3] = f;
    h->stats[4] = h->damping; h->stats[5] = failed; h->stats[6] = rejects; h->stats[8] = h->adef2_fallbacks;
    *loss_out = h->loss;
    return 0;
}

/* scale steps of the last solve */
void ora_gp_get_ds(const ora_t* h, double* out) { memcpy(out, h->gp_ds, sizeof(double) * (size_t)h->N); }

void ora_stats(const ora_t* h, double* out) { memcpy(out, h->stats, sizeof(h->stats)); }
double ora_damping(const ora_t* h) { return h->damping; }

/* copy internal buffers out (parity tests) */
int ora_get(const ora_t* h, int which, double* out) {
    size_t C = h->C, P = h->P, N = h->N, D = h->D;
    switch (which) {
        case 0: memcpy(out, h->W, sizeof(double) * N * D * 3); return 0;
        case 1: memcpy(out, h->V, sizeof(double) * P * 6); return 0;
        case 2: memcpy(out, h->gp, sizeof(double) * P * 3); return 0;
        case 3: memcpy(out, h->U, sizeof(double) * C * D * D); return 0;
        case 4: memcpy(out, h->gc, sizeof(double) * C * D); return 0;
        case 5: memcpy(out, h->S, sizeof(double) * (size_t)h->nnzb * D * D); return 0;
        case 6: memcpy(out, h->b, sizeof(double) * C * D); return 0;
        case 7: memcpy(out, h->x, sizeof(double) * C * D); return 0;
        case 8: memcpy(out, h->dp, sizeof(double) * P * 3); return 0;
        default: return -1;
    }
}
