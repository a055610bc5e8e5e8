/* Native host half of TorchBA.Solve's packing (instantsfm/processors/bundle_adjustment.py:66-113), used by
 * processors/bundle_adjustment.py pack().  CPython extension module `_packx` (plain C, numpy C API, OpenMP).
 *
 * The reference packs with a Python double loop over tracks x observations (~6.8 us per observation).  The vectorized
 * numpy pack still paid ~0.4 us per Track object inside np.concatenate (200k observation arrays and 200k xyz arrays
 * on config 3) plus single-threaded gathers for the cheirality test; here
 *   collect(track_vals, min_len)  reads every Track's `observations` / `xyz` arrays in place (numpy C API) in one loop;
 *   finish(...)                   does the registered-image filter, the feature gather, the cheirality test
 *                                 (z of rotate_quat > 0.1, the same operations in the same order as numpy, no FMA
 *                                 contraction) and the torch.unique compaction, on the host cores.
 * collect returns None when an object is not the plain ndarray layout it expects (a Python list, another dtype or
 * shape); pack() then takes the numpy path, which gives the same result.
 *
 * The parallel parts run on a small pthread pool whose idle workers block on a condition variable.  (Until round 5
 * they were OpenMP regions: libgomp's idle workers spin for a while after every region (GOMP_SPINCOUNT), and on a host
 * share of 16 cores that spinning slowed the GIL-held Python work right after the pack -- the engine creation and the
 * 200k `track.xyz` assignments of the write-back -- by up to 2x) */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- blocking worker pool -------------------------------------------------------------------------------------
 * par_run(fn, ctx) calls fn(ctx, t, T) for t in [0, T) -- t = 0 on the caller -- and returns when all have finished.
 * T = PACKX_THREADS, else OMP_NUM_THREADS (the GPU box sets it to its share of host cores), else the CPUs of the
 * process's affinity mask; at most kMaxThreads.  The workers start on first use and live for the process; between
 * jobs they sleep on a condition variable (no spinning).  Jobs come from one thread at a time (the GIL holder). */
enum { kMaxThreads = 32 };
typedef void (*par_fn)(void* ctx, int t, int T);
static struct {
    pthread_mutex_t m;
    pthread_cond_t go, done;
    int T, started;
    long long gen, gen0;  /* job generation; its value when the workers started */
    int pending;
    par_fn fn;
    void* ctx;
} g_pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0, 0, 0, 0, NULL, NULL};

static int pool_threads(void) {
    const char* e = getenv("PACKX_THREADS");
    if (!e || !*e) e = getenv("OMP_NUM_THREADS");
    int v = e && *e ? atoi(e) : 0;
    if (v <= 0) {
        cpu_set_t cs;
        v = sched_getaffinity(0, sizeof(cs), &cs) == 0 ? CPU_COUNT(&cs) : 1;
    }
    return v < 1 ? 1 : (v > kMaxThreads ? kMaxThreads : v);
}

static void* pool_worker(void* arg) {
    const int t = (int)(intptr_t)arg;
    pthread_mutex_lock(&g_pool.m);
    long long seen = g_pool.gen0;  /* (a job issued before this worker got here is still run) */
    pthread_mutex_unlock(&g_pool.m);
    for (;;) {
        pthread_mutex_lock(&g_pool.m);
        while (g_pool.gen == seen) pthread_cond_wait(&g_pool.go, &g_pool.m);
        seen = g_pool.gen;
        par_fn fn = g_pool.fn;
        void* ctx = g_pool.ctx;
        const int T = g_pool.T;
        pthread_mutex_unlock(&g_pool.m);
        fn(ctx, t, T);
        pthread_mutex_lock(&g_pool.m);
        if (--g_pool.pending == 0) pthread_cond_signal(&g_pool.done);
        pthread_mutex_unlock(&g_pool.m);
    }
    return NULL;
}

/* A forked child has none of the parent's workers: it starts its own on first use. */
static void pool_after_fork(void) {
    pthread_mutex_init(&g_pool.m, NULL);
    pthread_cond_init(&g_pool.go, NULL);
    pthread_cond_init(&g_pool.done, NULL);
    g_pool.started = 0;
    g_pool.pending = 0;
}

/* The pool size (starting the workers on first use; a worker that cannot be started shrinks the pool). */
static int pool_size(void) {
    static int atfork = 0;
    if (!atfork) atfork = pthread_atfork(NULL, NULL, pool_after_fork) == 0;
    if (!g_pool.started) {
        g_pool.started = 1;
        g_pool.gen0 = g_pool.gen;
        const int want = pool_threads();
        int n = 1;
        for (int t = 1; t < want; ++t) {
            pthread_t th;
            pthread_attr_t at;
            pthread_attr_init(&at);
            pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
            const int rc = pthread_create(&th, &at, pool_worker, (void*)(intptr_t)t);
            pthread_attr_destroy(&at);
            if (rc != 0) break;
            ++n;
        }
        g_pool.T = n;
    }
    return g_pool.T;
}

static void par_run(par_fn fn, void* ctx) {
    const int T = pool_size();
    if (T == 1) { fn(ctx, 0, 1); return; }
    pthread_mutex_lock(&g_pool.m);
    g_pool.fn = fn;
    g_pool.ctx = ctx;
    g_pool.pending = T - 1;
    ++g_pool.gen;
    pthread_cond_broadcast(&g_pool.go);
    pthread_mutex_unlock(&g_pool.m);
    fn(ctx, 0, T);
    pthread_mutex_lock(&g_pool.m);
    while (g_pool.pending > 0) pthread_cond_wait(&g_pool.done, &g_pool.m);
    pthread_mutex_unlock(&g_pool.m);
}

static PyObject *s_obs = NULL, *s_xyz = NULL;  /* interned attribute names */

/* 8: int64, 4: int32, 0: not a C-contiguous [k, 2] integer array */
static int obs_kind(PyObject* o) {
    if (!PyArray_Check(o)) return 0;
    PyArrayObject* a = (PyArrayObject*)o;
    if (PyArray_NDIM(a) != 2 || PyArray_DIM(a, 1) != 2 || !PyArray_IS_C_CONTIGUOUS(a) || !PyArray_ISNOTSWAPPED(a))
        return 0;
    const int t = PyArray_TYPE(a);
    if (t == NPY_INT64 || (t == NPY_LONGLONG && sizeof(long long) == 8) || (t == NPY_LONG && sizeof(long) == 8)) return 8;
    if (t == NPY_INT32 || (t == NPY_INT && sizeof(int) == 4)) return 4;
    return 0;
}

/* 8: float64, 4: float32, 0: not a C-contiguous (3,) float array */
static int xyz_kind(PyObject* o) {
    if (!PyArray_Check(o)) return 0;
    PyArrayObject* a = (PyArrayObject*)o;
    if (PyArray_NDIM(a) != 1 || PyArray_DIM(a, 0) != 3 || !PyArray_IS_C_CONTIGUOUS(a) || !PyArray_ISNOTSWAPPED(a)) return 0;
    const int t = PyArray_TYPE(a);
    return t == NPY_FLOAT64 ? 8 : (t == NPY_FLOAT32 ? 4 : 0);
}

struct copy_ctx {
    Py_ssize_t T;
    long long min_len;
    const int64_t* lengths;
    const int64_t* dst_off;
    const void** src;
    const unsigned char* kind;
    int64_t* out;
};

/* worker t of T: tracks [T_tracks * t / T, T_tracks * (t + 1) / T) */
static void copy_obs(void* p, int t, int T) {
    const struct copy_ctx* c = (const struct copy_ctx*)p;
    const Py_ssize_t a = (Py_ssize_t)((long long)c->T * t / T), b = (Py_ssize_t)((long long)c->T * (t + 1) / T);
    for (Py_ssize_t k = a; k < b; ++k) {
        if (c->lengths[k] < c->min_len) continue;
        const Py_ssize_t n = 2 * c->lengths[k];
        int64_t* o = c->out + c->dst_off[k];
        if (c->kind[k] == 8) {
            memcpy(o, c->src[k], sizeof(int64_t) * (size_t)n);
        } else {
            const int32_t* s32 = (const int32_t*)c->src[k];
            for (Py_ssize_t q = 0; q < n; ++q) o[q] = s32[q];
        }
    }
}

/* collect(track_vals, min_len) -> (lengths int64[T], obs int64[n, 2] of the tracks with >= min_len observations,
 * xyz float64[T, 3]) as bytes, or None (take the numpy path).  The arrays are read in place (numpy C API): one
 * attribute lookup and a few header reads per Track object. */
static PyObject* collect(PyObject* self, PyObject* args) {
    (void)self;
    PyObject* seq;
    long long min_len;
    if (!PyArg_ParseTuple(args, "OL", &seq, &min_len)) return NULL;
    PyObject* fast = PySequence_Fast(seq, "collect: a sequence of tracks");
    if (!fast) return NULL;
    const Py_ssize_t T = PySequence_Fast_GET_SIZE(fast);
    PyObject** items = PySequence_Fast_ITEMS(fast);
    PyObject** ob = (PyObject**)PyMem_Calloc(T > 0 ? (size_t)T : 1, sizeof(PyObject*));
    /* per track: its data pointer, element width and output offset (the copy below runs without the GIL) */
    const void** src = (const void**)PyMem_Calloc(T > 0 ? (size_t)T : 1, sizeof(void*));
    int64_t* dst_off = (int64_t*)PyMem_Calloc(T > 0 ? (size_t)T : 1, sizeof(int64_t));
    unsigned char* kind = (unsigned char*)PyMem_Calloc(T > 0 ? (size_t)T : 1, 1);
    PyObject *lb = NULL, *obb = NULL, *xb = NULL, *res = NULL;
    if (!ob || !src || !dst_off || !kind) {
        PyMem_Free(ob); PyMem_Free(src); PyMem_Free(dst_off); PyMem_Free(kind);
        Py_DECREF(fast);
        return PyErr_NoMemory();
    }
    lb = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)(sizeof(int64_t) * (size_t)T));
    xb = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)(sizeof(double) * 3 * (size_t)T));
    if (!lb || !xb) goto done;
    int64_t* lengths = (int64_t*)PyBytes_AS_STRING(lb);
    double* xo = (double*)PyBytes_AS_STRING(xb);
    Py_ssize_t nvalid = 0;
    for (Py_ssize_t t = 0; t < T; ++t) {
        PyObject* o = PyObject_GetAttr(items[t], s_obs);
        if (!o) goto done;
        ob[t] = o;
        const int ok_ = obs_kind(o);
        if (!ok_) goto fallback;
        kind[t] = (unsigned char)ok_;
        src[t] = PyArray_DATA((PyArrayObject*)o);
        lengths[t] = PyArray_DIM((PyArrayObject*)o, 0);
        dst_off[t] = 2 * nvalid;
        if (lengths[t] >= min_len) nvalid += lengths[t];
        PyObject* x = PyObject_GetAttr(items[t], s_xyz);
        if (!x) goto done;
        const int k = xyz_kind(x);
        if (k == 8) {
            memcpy(xo + 3 * t, PyArray_DATA((PyArrayObject*)x), 3 * sizeof(double));
        } else if (k == 4) {
            const float* f = (const float*)PyArray_DATA((PyArrayObject*)x);
            xo[3 * t] = f[0]; xo[3 * t + 1] = f[1]; xo[3 * t + 2] = f[2];
        }
        Py_DECREF(x);
        if (!k) goto fallback;
    }
    obb = PyBytes_FromStringAndSize(NULL, (Py_ssize_t)(sizeof(int64_t) * 2 * (size_t)nvalid));
    if (!obb) goto done;
    {
        /* the copy from the 200k arrays (references held in ob[]) on the pool, without the GIL: every track writes its
         * own slice of the output, so the result is the sequential loop's */
        struct copy_ctx cc = {(Py_ssize_t)T, min_len, lengths, dst_off, src, kind, (int64_t*)PyBytes_AS_STRING(obb)};
        Py_BEGIN_ALLOW_THREADS
        par_run(copy_obs, &cc);
        Py_END_ALLOW_THREADS
    }
    res = PyTuple_Pack(3, lb, obb, xb);
    goto done;
fallback:
    res = Py_None;
    Py_INCREF(res);
done:
    for (Py_ssize_t t = 0; t < T; ++t) Py_XDECREF(ob[t]);
    PyMem_Free(ob);
    PyMem_Free(src);
    PyMem_Free(dst_off);
    PyMem_Free(kind);
    Py_XDECREF(lb);
    Py_XDECREF(obb);
    Py_XDECREF(xb);
    Py_DECREF(fast);
    return res;
}

/* A C-contiguous buffer of exactly the expected element type: kind 'i' = 8-byte signed integer, 'f' = 8-byte float,
 * 'b' = one byte (uint8 / int8 / bool).  A buffer of another dtype is refused even when its byte length happens to
 * divide (an int32 obs array or float32 features would otherwise be reinterpreted). */
static int get_buf(PyObject* o, Py_buffer* b, char kind, const char* what) {
    if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) < 0) return -1;
    const char* f = b->format ? b->format : "B";
    while (*f == '@' || *f == '=' || *f == '<') ++f;  /* native / little-endian byte order only */
    int ok = 0;
    if (kind == 'i') ok = b->itemsize == 8 && (f[0] == 'l' || f[0] == 'q') && f[1] == 0;
    else if (kind == 'f') ok = b->itemsize == 8 && f[0] == 'd' && f[1] == 0;
    else ok = b->itemsize == 1 && (f[0] == 'B' || f[0] == 'b' || f[0] == '?') && f[1] == 0;
    if (!ok) {
        PyErr_Format(PyExc_TypeError, "finish: %s has the wrong dtype (buffer format '%s', itemsize %zd)", what,
                     b->format ? b->format : "B", b->itemsize);
        PyBuffer_Release(b);
        return -1;
    }
    return 0;
}

/* finish's three passes over the observations; worker t of T takes observations [n t / T, n (t + 1) / T) */
struct fin_ctx {
    const int64_t *obs, *foff, *tid;
    const uint8_t* reg;
    const double *feat, *pts, *pose;
    int64_t n, nI, nF;
    int stride;
    int* bad;
    uint8_t* ok;
    char *pc, *pp;
    int64_t *cnt, *cmap, *pmap, *oci, *opi;
    double* o2d;
    int32_t *oc32, *op32;
};

static void fin_check(void* p, int t, int T) {
    const struct fin_ctx* c = (const struct fin_ctx*)p;
    const int64_t a = c->n * t / T, b = c->n * (t + 1) / T;
    int bad = 0;
    for (int64_t k = a; k < b; ++k) {
        const int64_t im = c->obs[2 * k];
        if (im < 0 || im >= c->nI) { bad |= 1; continue; }
        if (c->reg[im]) {
            const int64_t f = c->foff[im] + c->obs[2 * k + 1];
            if (c->obs[2 * k + 1] < 0 || f >= c->foff[im + 1] || f >= c->nF) bad |= 2;
        }
    }
    c->bad[t] = bad;
}

static void fin_cheirality(void* p, int t, int T) {
    const struct fin_ctx* c = (const struct fin_ctx*)p;
    const int64_t a = c->n * t / T, b = c->n * (t + 1) / T;
    int64_t cn = 0;
    for (int64_t k = a; k < b; ++k) {
        const int64_t im = c->obs[2 * k];
        uint8_t keep = 0;
        if (c->reg[im]) {
            const double* X = c->pts + 3 * c->tid[k];
            const double* Q = c->pose + (int64_t)c->stride * im;
            const double px = X[0], py = X[1], pz = X[2];
            const double qx = Q[3], qy = Q[4], qz = Q[5], w = Q[6];
            const double uvx = qy * pz - qz * py;
            const double uvy = qz * px - qx * pz;
            const double uvz = qx * py - qy * px;
            const double z = pz + 2.0 * (w * uvz + (qx * uvy - qy * uvx)) + Q[2];
            keep = z > 0.1;
        }
        c->ok[k] = keep;
        /* the flags are written only when not yet set: every thread marks the same ~1000 image bytes, and
         * unconditional stores would ping-pong their cache lines between cores */
        if (keep) {
            if (!c->pc[im]) c->pc[im] = 1;
            if (!c->pp[c->tid[k]]) c->pp[c->tid[k]] = 1;
            ++cn;
        }
    }
    c->cnt[t + 1] = cn;
}

static void fin_write(void* p, int t, int T) {
    const struct fin_ctx* c = (const struct fin_ctx*)p;
    const int64_t a = c->n * t / T, b = c->n * (t + 1) / T;
    int64_t w = c->cnt[t];
    for (int64_t k = a; k < b; ++k) {
        if (!c->ok[k]) continue;
        const int64_t im = c->obs[2 * k];
        const double* fp = c->feat + 2 * (c->foff[im] + c->obs[2 * k + 1]);
        c->o2d[2 * w] = fp[0];
        c->o2d[2 * w + 1] = fp[1];
        c->oci[w] = c->cmap[im];
        c->opi[w] = c->pmap[c->tid[k]];
        c->oc32[w] = (int32_t)c->cmap[im];
        c->op32[w] = (int32_t)c->pmap[c->tid[k]];
        ++w;
    }
}

/* finish(obs int64[n,2], lengths int64[T], min_len, registered uint8[I], features float64[F,2], foff int64[I+1],
 *        points float64[T,3], poses float64[I,stride], stride)
 *   -> (points_2d float64[m,2], camera_indices int64[m], point_indices int64[m], unique_cameras int64[], unique_points
 *       int64[], camera_indices int32[m], point_indices int32[m]) as bytearrays (writable): the observations of
 *       registered images whose point lies in front of the camera (bundle_adjustment.py:85-113); the int32 copies are
 *       what insfm_ba_create takes (written in the same pass instead of a numpy conversion per Solve). */
static PyObject* finish(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *o_obs, *o_len, *o_reg, *o_feat, *o_foff, *o_pts, *o_pose;
    long long min_len;
    int stride;
    if (!PyArg_ParseTuple(args, "OOLOOOOOi", &o_obs, &o_len, &min_len, &o_reg, &o_feat, &o_foff, &o_pts, &o_pose, &stride))
        return NULL;
    Py_buffer bo = {0}, bl = {0}, br = {0}, bf = {0}, bff = {0}, bp = {0}, bq = {0};
    PyObject* res = NULL;
    char *pc = NULL, *pp = NULL;
    int64_t *tid = NULL, *cnt = NULL;
    if (get_buf(o_obs, &bo, 'i', "obs") || get_buf(o_len, &bl, 'i', "lengths") || get_buf(o_reg, &br, 'b', "registered") ||
        get_buf(o_feat, &bf, 'f', "features") || get_buf(o_foff, &bff, 'i', "foff") || get_buf(o_pts, &bp, 'f', "points") ||
        get_buf(o_pose, &bq, 'f', "poses"))
        goto done;
    {
        const int64_t* obs = (const int64_t*)bo.buf;
        const int64_t* len = (const int64_t*)bl.buf;
        const uint8_t* reg = (const uint8_t*)br.buf;
        const double* feat = (const double*)bf.buf;
        const int64_t* foff = (const int64_t*)bff.buf;
        const double* pts = (const double*)bp.buf;
        const double* pose = (const double*)bq.buf;
        const int64_t n = bo.len / 16, nT = bl.len / 8, nI = br.len, nF = bf.len / 16;
        if (bff.len / 8 != nI + 1 || bp.len / 24 != nT || stride < 7 || bq.len / 8 != nI * (int64_t)stride) {
            PyErr_SetString(PyExc_ValueError, "finish: inconsistent array sizes");
            goto done;
        }
        /* the valid tracks' lengths must sum to the observation count exactly (checked before any write) */
        {
            int64_t tot = 0;
            for (int64_t t = 0; t < nT; ++t)
                if (len[t] >= min_len) {
                    if (len[t] < 0) { tot = -1; break; }
                    tot += len[t];
                }
            if (tot != n) { PyErr_SetString(PyExc_ValueError, "finish: lengths do not match obs"); goto done; }
        }
        /* track id of every observation (valid tracks only, in order) */
        tid = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
        if (!tid) { PyErr_NoMemory(); goto done; }
        {
            int64_t k = 0;
            for (int64_t t = 0; t < nT; ++t) {
                if (len[t] < min_len) continue;
                for (int64_t q = 0; q < len[t]; ++q) tid[k++] = t;
            }
        }
        const int nth = pool_size();
        struct fin_ctx fc;
        memset(&fc, 0, sizeof(fc));
        fc.obs = obs; fc.reg = reg; fc.feat = feat; fc.foff = foff; fc.pts = pts; fc.pose = pose; fc.tid = tid;
        fc.n = n; fc.nI = nI; fc.nF = nF; fc.stride = stride;
        int bad = 0;
        {
            int badv[kMaxThreads] = {0};
            fc.bad = badv;
            par_run(fin_check, &fc);
            for (int t = 0; t < nth; ++t) bad |= badv[t];
        }
        if (bad) {
            PyErr_SetString(PyExc_IndexError, (bad & 1) ? "finish: image id out of range" : "finish: feature id out of range");
            goto done;
        }
        cnt = (int64_t*)PyMem_Calloc((size_t)nth + 1, sizeof(int64_t));
        pc = (char*)PyMem_Calloc((size_t)(nI > 0 ? nI : 1), 1);
        pp = (char*)PyMem_Calloc((size_t)(nT > 0 ? nT : 1), 1);
        uint8_t* ok = (uint8_t*)PyMem_Malloc((size_t)(n > 0 ? n : 1));
        if (!cnt || !pc || !pp || !ok) { PyMem_Free(ok); PyErr_NoMemory(); goto done; }
        /* cheirality: z of rotate_quat(points[tid], pose[img]) exactly as _rotated_z's numpy expression */
        fc.ok = ok; fc.pc = pc; fc.pp = pp; fc.cnt = cnt;
        par_run(fin_cheirality, &fc);
        for (int t = 0; t < nth; ++t) cnt[t + 1] += cnt[t];
        const int64_t m = cnt[nth];
        /* compaction maps */
        int64_t nuc = 0, nup = 0;
        for (int64_t i = 0; i < nI; ++i) nuc += pc[i];
        for (int64_t i = 0; i < nT; ++i) nup += pp[i];
        PyObject *b2d = PyByteArray_FromStringAndSize(NULL, 16 * m), *bci = PyByteArray_FromStringAndSize(NULL, 8 * m);
        PyObject *bpi = PyByteArray_FromStringAndSize(NULL, 8 * m), *buc = PyByteArray_FromStringAndSize(NULL, 8 * nuc);
        PyObject* bup = PyByteArray_FromStringAndSize(NULL, 8 * nup);
        PyObject *bc32 = PyByteArray_FromStringAndSize(NULL, 4 * m), *bp32 = PyByteArray_FromStringAndSize(NULL, 4 * m);
        int64_t* cmap = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(nI > 0 ? nI : 1));
        int64_t* pmap = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(nT > 0 ? nT : 1));
        if (!b2d || !bci || !bpi || !buc || !bup || !bc32 || !bp32 || !cmap || !pmap) {
            Py_XDECREF(b2d); Py_XDECREF(bci); Py_XDECREF(bpi); Py_XDECREF(buc); Py_XDECREF(bup);
            Py_XDECREF(bc32); Py_XDECREF(bp32);
            PyMem_Free(cmap); PyMem_Free(pmap); PyMem_Free(ok);
            if (!PyErr_Occurred()) PyErr_NoMemory();
            goto done;
        }
        int64_t* uc = (int64_t*)PyByteArray_AS_STRING(buc);
        int64_t* up = (int64_t*)PyByteArray_AS_STRING(bup);
        for (int64_t i = 0, r = 0; i < nI; ++i) { cmap[i] = r; if (pc[i]) uc[r++] = i; }
        for (int64_t i = 0, r = 0; i < nT; ++i) { pmap[i] = r; if (pp[i]) up[r++] = i; }
        fc.cmap = cmap; fc.pmap = pmap;
        fc.o2d = (double*)PyByteArray_AS_STRING(b2d);
        fc.oci = (int64_t*)PyByteArray_AS_STRING(bci);
        fc.opi = (int64_t*)PyByteArray_AS_STRING(bpi);
        fc.oc32 = (int32_t*)PyByteArray_AS_STRING(bc32);
        fc.op32 = (int32_t*)PyByteArray_AS_STRING(bp32);
        par_run(fin_write, &fc);
        PyMem_Free(cmap); PyMem_Free(pmap); PyMem_Free(ok);
        res = PyTuple_Pack(7, b2d, bci, bpi, buc, bup, bc32, bp32);
        Py_DECREF(b2d); Py_DECREF(bci); Py_DECREF(bpi); Py_DECREF(buc); Py_DECREF(bup);
        Py_DECREF(bc32); Py_DECREF(bp32);
    }
done:
    PyMem_Free(tid); PyMem_Free(cnt); PyMem_Free(pc); PyMem_Free(pp);
    if (bo.obj) PyBuffer_Release(&bo);
    if (bl.obj) PyBuffer_Release(&bl);
    if (br.obj) PyBuffer_Release(&br);
    if (bf.obj) PyBuffer_Release(&bf);
    if (bff.obj) PyBuffer_Release(&bff);
    if (bp.obj) PyBuffer_Release(&bp);
    if (bq.obj) PyBuffer_Release(&bq);
    return res;
}

/* assign_xyz(track_vals, unique_points int64[n], points float64[n, 3]): track_vals[unique_points[i]].xyz = a float64
 * [3] array holding points[i] (bundle_adjustment.py:18-36 assigns the row views of one array; the values are the same).
 * When the track's current xyz is an array nothing else can see -- an exact float64 [3] ndarray that owns its
 * writable buffer, referenced only by the track's attribute (refcount 2 with ours) and by no weak reference -- the
 * point is written into it: no caller can tell that apart from a new array, and no allocation or free happens (a
 * scene whose tracks were built one array each, or written back by an earlier call).  Otherwise the track gets a new
 * array that owns its 24 bytes (so the next call can take the first path).  Round 5 assigned row views of `points`:
 * one allocation per track for two frees when the old arrays owned their buffers, and the 200k chunks left in
 * glibc's bins made the next allocation of a kilobyte or more sort them all (malloc_consolidate / the unsorted-bin
 * scan: ~5 ms on the GPU box's host, 20 ms on this container's). */
static PyObject* assign_xyz(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *seq, *o_idx, *o_pts;
    if (!PyArg_ParseTuple(args, "OOO", &seq, &o_idx, &o_pts)) return NULL;
    if (!PyArray_Check(o_idx) || !PyArray_Check(o_pts)) { PyErr_SetString(PyExc_TypeError, "assign_xyz: arrays"); return NULL; }
    PyArrayObject *ai = (PyArrayObject*)o_idx, *ap = (PyArrayObject*)o_pts;
    if (PyArray_TYPE(ai) != NPY_INT64 || !PyArray_IS_C_CONTIGUOUS(ai) || PyArray_TYPE(ap) != NPY_FLOAT64 ||
        !PyArray_IS_C_CONTIGUOUS(ap) || PyArray_NDIM(ap) != 2 || PyArray_DIM(ap, 1) != 3 ||
        PyArray_SIZE(ai) != PyArray_DIM(ap, 0)) {
        PyErr_SetString(PyExc_ValueError, "assign_xyz: int64 [n] indices and a C-contiguous float64 [n, 3] array");
        return NULL;
    }
    PyObject* fast = PySequence_Fast(seq, "assign_xyz: a sequence of tracks");
    if (!fast) return NULL;
    const Py_ssize_t T = PySequence_Fast_GET_SIZE(fast);
    PyObject** items = PySequence_Fast_ITEMS(fast);
    const int64_t* idx = (const int64_t*)PyArray_DATA(ai);
    const double* base = (const double*)PyArray_DATA(ap);
    const npy_intp n = PyArray_DIM(ap, 0);
    npy_intp dims[1] = {3};
    for (npy_intp i = 0; i < n; ++i) {
        if (idx[i] < 0 || idx[i] >= T) {
            PyErr_SetString(PyExc_IndexError, "assign_xyz: track index");
            Py_DECREF(fast);
            return NULL;
        }
        PyObject* cur = PyObject_GetAttr(items[idx[i]], s_xyz);
        if (!cur) PyErr_Clear();
        else if (PyArray_CheckExact(cur) && Py_REFCNT(cur) == 2) {
            PyArrayObject* ca = (PyArrayObject*)cur;
            if (PyArray_NDIM(ca) == 1 && PyArray_DIM(ca, 0) == 3 && PyArray_TYPE(ca) == NPY_FLOAT64 &&
                PyArray_ISNOTSWAPPED(ca) && PyArray_IS_C_CONTIGUOUS(ca) && PyArray_ISWRITEABLE(ca) &&
                PyArray_CHKFLAGS(ca, NPY_ARRAY_OWNDATA) && ((PyArrayObject_fields*)ca)->weakreflist == NULL) {
                memcpy(PyArray_DATA(ca), base + 3 * i, 3 * sizeof(double));
                Py_DECREF(cur);
                continue;
            }
        }
        Py_XDECREF(cur);
        PyObject* row = PyArray_SimpleNew(1, dims, NPY_FLOAT64);
        if (!row) { Py_DECREF(fast); return NULL; }
        memcpy(PyArray_DATA((PyArrayObject*)row), base + 3 * i, 3 * sizeof(double));
        const int r = PyObject_SetAttr(items[idx[i]], s_xyz, row);
        Py_DECREF(row);
        if (r < 0) { Py_DECREF(fast); return NULL; }
    }
    Py_DECREF(fast);
    Py_RETURN_NONE;
}

static PyMethodDef methods[] = {
    {"assign_xyz", assign_xyz, METH_VARARGS, "track.xyz = the optimized point (an owned float64 [3]), per packed point."},
    {"collect", collect, METH_VARARGS, "Track observations / xyz through the buffer protocol (or None)."},
    {"finish", finish, METH_VARARGS, "Registered filter, feature gather, cheirality test and compaction."},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_packx", NULL, -1, methods, NULL, NULL, NULL, NULL};

/* SRC_HASH: instantsfm_amd/build.py passes the hash of this file (packx_hash()); the loader compares it with the tree */
#ifndef PACKX_SRC_HASH
#define PACKX_SRC_HASH "unknown"
#endif

PyMODINIT_FUNC PyInit__packx(void) {
    import_array();
    s_obs = PyUnicode_InternFromString("observations");
    s_xyz = PyUnicode_InternFromString("xyz");
    if (!s_obs || !s_xyz) return NULL;
    PyObject* m = PyModule_Create(&mod);
    if (m && PyModule_AddStringConstant(m, "SRC_HASH", PACKX_SRC_HASH) < 0) {
        Py_DECREF(m);
        return NULL;
    }
    return m;
}
