// Track establishment (include/insfm_tracks.h): union-find over the inlier matches and track collection, on the GPU.
//
// The work is integer gather/scatter over the edge list (HBM- and atomic-bound; no FLOPs), in eight passes:
//   1. k_link       -- lock-free union-find (hook the larger root under the smaller, CAS on the root, pointer
//                      jumping in the finds), plus each node's first entry and reference count;
//   2. k_label      -- every node -> component minimum;
//   3. k_first_edge / k_edge_key + radix sort -- edges grouped by component, components in order of first
//                      appearance, edges in their original order inside a component (the sort is stable);
//   4. k_heads + scan -- component index of each grouped edge, component starts;
//   5. k_replay     -- one thread per component replays the reference's sequential UnionFind on that component's edges
//                      only (components are independent), which yields the reference's root, hence its track id;
//   6. k_entries + scan -- the distinct observations of each component in order of first appearance;
//   7. k_row_key + radix sort (stable) -- observations grouped by (component, image), first appearance inside;
//   8. k_rows       -- per (component, image): inconsistency test over the group's pairs and the kept observation.
// Scratch comes from the stream-ordered allocator and is released before the call returns.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <vector>

#include "../../include/insfm_ba.h"
#include "../../include/insfm_tracks.h"

#pragma clang fp contract(off)

namespace {

constexpr int kT = 256;
constexpr int kNone = 0x7fffffff;

inline unsigned grid(int64_t n) { return (unsigned)((n + kT - 1) / kT); }

__device__ __forceinline__ int ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Root of v while other threads link: parents only ever decrease, so a stale read is still an ancestor.
__device__ __forceinline__ int rep(int* par, int v) {
    int cur = ld(par + v);
    if (cur != v) {
        int prev = v, next;
        while (cur > (next = ld(par + cur))) {
            __hip_atomic_store(par + prev, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            prev = cur;
            cur = next;
        }
    }
    return cur;
}

__global__ __launch_bounds__(kT) void k_init(int64_t n, int* __restrict__ par, int* __restrict__ par2,
                                             int* __restrict__ first_entry, int* __restrict__ deg, int* __restrict__ first_edge) {
    const int64_t v = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (v >= n) return;
    par[v] = (int)v;
    par2[v] = (int)v;
    first_entry[v] = kNone;
    deg[v] = 0;
    first_edge[v] = kNone;
}

__global__ __launch_bounds__(kT) void k_link(int64_t ne, const int32_t* __restrict__ ea, const int32_t* __restrict__ eb,
                                             int* __restrict__ par, int* __restrict__ first_entry, int* __restrict__ deg) {
    const int64_t k = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (k >= ne) return;
    const int a = ea[k], b = eb[k];
    atomicMin(first_entry + a, (int)(2 * k));
    atomicMin(first_entry + b, (int)(2 * k + 1));
    atomicAdd(deg + a, 1);
    atomicAdd(deg + b, 1);
    int ra = rep(par, a), rb = rep(par, b);
    while (ra != rb) {
        if (ra < rb) {
            const int got = atomicCAS(par + rb, rb, ra);
            if (got == rb) break;
            rb = got;
        } else {
            const int got = atomicCAS(par + ra, ra, rb);
            if (got == ra) break;
            ra = got;
        }
        ra = rep(par, ra);
        rb = rep(par, rb);
    }
}

__global__ __launch_bounds__(kT) void k_label(int64_t n, int* __restrict__ par) {
    const int64_t v = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (v >= n) return;
    int cur = par[v];
    const int old = cur;
    int next;
    while (cur > (next = par[cur])) cur = next;
    if (cur != old) par[v] = cur;
}

__global__ __launch_bounds__(kT) void k_first_edge(int64_t ne, const int32_t* __restrict__ ea, const int* __restrict__ label,
                                                   int* __restrict__ first_edge) {
    const int64_t k = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (k >= ne) return;
    atomicMin(first_edge + label[ea[k]], (int)k);
}

__global__ __launch_bounds__(kT) void k_edge_key(int64_t ne, const int32_t* __restrict__ ea, const int* __restrict__ label,
                                                 const int* __restrict__ first_edge, int* __restrict__ key, int* __restrict__ val) {
    const int64_t k = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (k >= ne) return;
    key[k] = first_edge[label[ea[k]]];
    val[k] = (int)k;
}

template <typename K>
__global__ __launch_bounds__(kT) void k_heads(int64_t n, const K* __restrict__ key, int* __restrict__ head) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    head[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}

// seg[i] = inclusive scan of heads - 1 = segment of element i; start[seg] = i at heads; start[nseg] = n.
__global__ __launch_bounds__(kT) void k_starts(int64_t n, const int* __restrict__ head, const int* __restrict__ incl,
                                               int* __restrict__ start) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    if (head[i]) start[incl[i] - 1] = (int)i;
    if (i == n - 1) start[incl[i]] = (int)n;
}

__global__ __launch_bounds__(kT) void k_minus_one(int64_t n, const int* __restrict__ in, int* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (i < n) out[i] = in[i] - 1;
}

__device__ __forceinline__ int find_seq(int* par, int v) {
    while (par[v] != v) {
        const int g = par[par[v]];
        par[v] = g;
        v = g;
    }
    return v;
}

// UnionFind.Union(larger, smaller) (union_find.py:16-20, track_establishment.py:31-37) replayed in edge order.
__global__ __launch_bounds__(kT) void k_replay(int nt, const int* __restrict__ cstart, const int* __restrict__ sedge,
                                               const int32_t* __restrict__ ea, const int32_t* __restrict__ eb,
                                               int* __restrict__ par2, int32_t* __restrict__ root) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t >= nt) return;
    const int s = cstart[t], e = cstart[t + 1];
    for (int i = s; i < e; ++i) {
        const int k = sedge[i];
        const int a = ea[k], b = eb[k];
        const int x = a > b ? a : b, y = a > b ? b : a;
        const int rx = find_seq(par2, x), ry = find_seq(par2, y);
        if (rx != ry) par2[rx] = ry;
    }
    root[t] = find_seq(par2, ea[sedge[s]]);
}

// Entry 2i + j of the grouped sequence is node (j ? b : a) of grouped edge i; it is the node's first appearance when
// its original entry number 2k + j is the node's minimum.
__global__ __launch_bounds__(kT) void k_entry_flags(int64_t ne, const int* __restrict__ sedge, const int32_t* __restrict__ ea,
                                                    const int32_t* __restrict__ eb, const int* __restrict__ first_entry,
                                                    int* __restrict__ flag) {
    const int64_t q = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (q >= 2 * ne) return;
    const int k = sedge[q >> 1];
    const int j = (int)(q & 1);
    const int node = j ? eb[k] : ea[k];
    flag[q] = first_entry[node] == 2 * k + j ? 1 : 0;
}

__global__ __launch_bounds__(kT) void k_entries(int64_t ne, const int* __restrict__ sedge, const int32_t* __restrict__ ea,
                                                const int32_t* __restrict__ eb, const int* __restrict__ flag,
                                                const int* __restrict__ pos, const int* __restrict__ ecomp,
                                                const int32_t* __restrict__ node_img, int* __restrict__ obs_node,
                                                unsigned long long* __restrict__ obs_key) {
    const int64_t q = (int64_t)blockIdx.x * kT + threadIdx.x;
    if (q >= 2 * ne || !flag[q]) return;
    const int k = sedge[q >> 1];
    const int node = (q & 1) ? eb[k] : ea[k];
    const int p = pos[q];
    obs_node[p] = node;
    obs_key[p] = ((unsigned long long)(unsigned)ecomp[q >> 1] << 32) | (unsigned)node_img[node];
}

__global__ __launch_bounds__(kT) void k_track_nodes(int nt, const int* __restrict__ cstart, const int* __restrict__ pos,
                                                    int total, int64_t ne, int32_t* __restrict__ nodes) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t >= nt) return;
    const int64_t a = 2 * (int64_t)cstart[t], b = 2 * (int64_t)cstart[t + 1];
    nodes[t] = (b == 2 * ne ? total : pos[b]) - pos[a];
}

// numpy's float32 / float64 norm: sqrt(dx*dx + dy*dy), no contraction, compared in the features' type.
template <typename F>
__device__ __forceinline__ bool too_far(const F* xy, int i, int j, F thres) {
    const F dx = xy[2 * (size_t)i] - xy[2 * (size_t)j];
    const F dy = xy[2 * (size_t)i + 1] - xy[2 * (size_t)j + 1];
    return sqrt(dx * dx + dy * dy) > thres;
}

template <typename F>
__global__ __launch_bounds__(kT) void k_rows(int ng, const int* __restrict__ gstart, const int* __restrict__ snode,
                                             const unsigned long long* __restrict__ skey, const int* __restrict__ deg,
                                             const F* __restrict__ xy, F thres, uint8_t* __restrict__ bad,
                                             int32_t* __restrict__ row_node, int32_t* __restrict__ row_track) {
    const int g = blockIdx.x * kT + threadIdx.x;
    if (g >= ng) return;
    const int s = gstart[g], e = gstart[g + 1];
    const int t = (int)(skey[s] >> 32);
    int best = snode[s], bestc = deg[best];
    bool far = false;
    for (int i = s; i < e; ++i) {
        const int ni = snode[i];
        if (deg[ni] > bestc) {  // np.unique on (image, -count) keeps the first row of the highest count
            best = ni;
            bestc = deg[ni];
        }
        for (int j = s; j < i && !far; ++j) far = too_far(xy, snode[j], ni, thres);
    }
    if (far) bad[t] = 1;
    row_node[g] = best;
    row_track[g] = t;
}

int bits_for(int64_t n) {
    int b = 1;
    while (b < 62 && ((int64_t)1 << b) < n) ++b;
    return b;
}

struct Scratch {
    hipStream_t s;
    std::vector<void*> ptrs;
    bool ok = true;
    template <typename T>
    T* get(size_t n) {
        void* p = nullptr;
        if (hipMallocAsync(&p, (n ? n : 1) * sizeof(T), s) != hipSuccess) {
            ok = false;
            return nullptr;
        }
        ptrs.push_back(p);
        return static_cast<T*>(p);
    }
    ~Scratch() {
        for (void* p : ptrs) (void)hipFreeAsync(p, s);
        (void)hipStreamSynchronize(s);
    }
};

}  // namespace

extern "C" int insfm_tracks_establish(int64_t n_nodes, const int32_t* node_img, const void* node_xy, int32_t xy_f32,
                                      int64_t n_edges, const int32_t* edge_a, const int32_t* edge_b,
                                      double thres_inconsistency, int32_t* track_root, uint8_t* track_bad,
                                      int32_t* track_nodes, int32_t* row_node, int32_t* row_track, int64_t* counts,
                                      void* stream) {
    if (!counts || n_nodes < 0 || n_edges < 0 || n_nodes >= kNone || 2 * n_edges >= kNone) return INSFM_BA_EINVAL;
    counts[0] = counts[1] = 0;
    if (n_edges == 0) return INSFM_BA_OK;
    if (!node_img || !node_xy || !edge_a || !edge_b || !track_root || !track_bad || !track_nodes || !row_node || !row_track)
        return INSFM_BA_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t n = n_nodes, ne = n_edges, nq = 2 * n_edges;
    Scratch w{s};
    int* par = w.get<int>(n);
    int* par2 = w.get<int>(n);
    int* first_entry = w.get<int>(n);
    int* deg = w.get<int>(n);
    int* first_edge = w.get<int>(n);
    int* key = w.get<int>(ne);
    int* val = w.get<int>(ne);
    int* skey = w.get<int>(ne);
    int* sedge = w.get<int>(ne);
    int* head = w.get<int>(nq);
    int* incl = w.get<int>(nq);
    int* cstart = w.get<int>(ne + 1);
    int* flag = w.get<int>(nq);
    int* pos = w.get<int>(nq);
    int* obs_node = w.get<int>(nq);
    int* snode = w.get<int>(nq);
    unsigned long long* obs_key = w.get<unsigned long long>(nq);
    unsigned long long* skey64 = w.get<unsigned long long>(nq);
    int* gstart = w.get<int>(nq + 1);
    int* host = nullptr;
    if (!w.ok || hipHostMalloc(reinterpret_cast<void**>(&host), 4 * sizeof(int)) != hipSuccess) return INSFM_BA_ENOMEM;
    struct HostFree {
        int* p;
        ~HostFree() { (void)hipHostFree(p); }
    } host_guard{host};

    // temp storage for the sorts and scans: the largest requirement of the four shapes
    size_t tmp_bytes = 0, b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, key, skey, val, sedge, (int)ne, 0, bits_for(ne), s);
    tmp_bytes = b > tmp_bytes ? b : tmp_bytes;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, obs_key, skey64, obs_node, snode, (int)nq, 0, 64, s);
    tmp_bytes = b > tmp_bytes ? b : tmp_bytes;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, head, incl, (int)nq, s);
    tmp_bytes = b > tmp_bytes ? b : tmp_bytes;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, flag, pos, (int)nq, s);
    tmp_bytes = b > tmp_bytes ? b : tmp_bytes;
    void* tmp = w.get<unsigned char>(tmp_bytes);
    if (!w.ok) return INSFM_BA_ENOMEM;

    k_init<<<grid(n), kT, 0, s>>>(n, par, par2, first_entry, deg, first_edge);
    k_link<<<grid(ne), kT, 0, s>>>(ne, edge_a, edge_b, par, first_entry, deg);
    k_label<<<grid(n), kT, 0, s>>>(n, par);
    k_first_edge<<<grid(ne), kT, 0, s>>>(ne, edge_a, par, first_edge);
    k_edge_key<<<grid(ne), kT, 0, s>>>(ne, edge_a, par, first_edge, key, val);
    b = tmp_bytes;
    (void)hipcub::DeviceRadixSort::SortPairs(tmp, b, key, skey, val, sedge, (int)ne, 0, bits_for(ne), s);
    k_heads<int><<<grid(ne), kT, 0, s>>>(ne, skey, head);
    b = tmp_bytes;
    (void)hipcub::DeviceScan::InclusiveSum(tmp, b, head, incl, (int)ne, s);
    k_starts<<<grid(ne), kT, 0, s>>>(ne, head, incl, cstart);
    (void)hipMemcpyAsync(host, incl + ne - 1, sizeof(int), hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess) return INSFM_BA_EHIP;
    const int nt = host[0];

    k_replay<<<grid(nt), kT, 0, s>>>(nt, cstart, sedge, edge_a, edge_b, par2, track_root);
    (void)hipMemsetAsync(track_bad, 0, (size_t)nt, s);
    k_entry_flags<<<grid(nq), kT, 0, s>>>(ne, sedge, edge_a, edge_b, first_entry, flag);
    b = tmp_bytes;
    (void)hipcub::DeviceScan::ExclusiveSum(tmp, b, flag, pos, (int)nq, s);
    // component of grouped edge i: incl[i] - 1
    int* ecomp = val;  // the unsorted edge ids are no longer needed
    k_minus_one<<<grid(ne), kT, 0, s>>>(ne, incl, ecomp);
    k_entries<<<grid(nq), kT, 0, s>>>(ne, sedge, edge_a, edge_b, flag, pos, ecomp, node_img, obs_node, obs_key);
    (void)hipMemcpyAsync(host, pos + nq - 1, sizeof(int), hipMemcpyDeviceToHost, s);
    (void)hipMemcpyAsync(host + 1, flag + nq - 1, sizeof(int), hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess) return INSFM_BA_EHIP;
    const int nobs = host[0] + host[1];
    k_track_nodes<<<grid(nt), kT, 0, s>>>(nt, cstart, pos, nobs, ne, track_nodes);

    b = tmp_bytes;
    (void)hipcub::DeviceRadixSort::SortPairs(tmp, b, obs_key, skey64, obs_node, snode, nobs, 0, 32 + bits_for(nt), s);
    k_heads<unsigned long long><<<grid(nobs), kT, 0, s>>>(nobs, skey64, head);
    b = tmp_bytes;
    (void)hipcub::DeviceScan::InclusiveSum(tmp, b, head, incl, nobs, s);
    k_starts<<<grid(nobs), kT, 0, s>>>(nobs, head, incl, gstart);
    (void)hipMemcpyAsync(host, incl + nobs - 1, sizeof(int), hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess) return INSFM_BA_EHIP;
    const int ng = host[0];
    if (xy_f32)
        k_rows<float><<<grid(ng), kT, 0, s>>>(ng, gstart, snode, skey64, deg, static_cast<const float*>(node_xy),
                                              (float)thres_inconsistency, track_bad, row_node, row_track);
    else
        k_rows<double><<<grid(ng), kT, 0, s>>>(ng, gstart, snode, skey64, deg, static_cast<const double*>(node_xy),
                                               thres_inconsistency, track_bad, row_node, row_track);
    if (hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess) return INSFM_BA_EHIP;
    counts[0] = nt;
    counts[1] = ng;
    return INSFM_BA_OK;
}
