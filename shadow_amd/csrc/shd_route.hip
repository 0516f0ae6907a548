// shd_route.hip -- MI355X (gfx950) routing engine behind include/shd_route.h.
//
// Replaces the igraph path computation of Shadow 1.14 src/main/routing/topology.c:
//   K1+K2 sssp_rows_kernel  : igraph_get_shortest_paths_dijkstra (topology.c:1756) +
//                             _topology_computePathProperties (topology.c:1407-1523), one
//                             workgroup per source, many sources per launch
//   K3    direct_rows_kernel: _topology_lookupDirectPath (topology.c:1877-1927)
//   K5    min_reduce_kernel : minimumPathLatency (topology.c:1374-1385)
//   self_kernel             : _topology_computeShortestPathToSelf (topology.c:1545-1653)
//
// Host side (C++): graph validation as topology.c:565-1185, igraph-compatible edge
// lookup (get_eid), CSR construction, device residency.  See DESIGN.md for the data
// layout in HBM/LDS and the roofline of each kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <new>
#include <numeric>
#include <vector>

#include "../../include/shd_route.h"

namespace {

constexpr int kBlock = 256;              // 4 waves of 64
constexpr int kWaves = kBlock / 64;
constexpr size_t kLdsBudget = 160 * 1024; // gfx950 LDS per CU
constexpr unsigned long long kInfBits = 0x7FF0000000000000ull;  // +inf as u64

__host__ __device__ inline size_t a16(size_t x) { return (x + 15) & ~size_t(15); }

// Per-source state layout (bytes), shared by the LDS-resident and HBM-resident paths.
struct StateLayout {
    size_t dist, relv, q0, q1, bits, total;
    __host__ __device__ static StateLayout make(int n) {
        StateLayout L;
        size_t o = 0;
        L.dist = o; o += a16(sizeof(unsigned long long) * n);
        L.relv = o; o += a16(sizeof(double) * n);
        L.q0 = o;   o += a16(sizeof(int) * n);
        L.q1 = o;   o += a16(sizeof(int) * n);
        L.bits = o; o += a16(sizeof(unsigned) * ((n + 31) / 32));
        L.total = o;
        return L;
    }
};

// small per-block scratch carved from the start of dynamic LDS
struct Small {
    int off[kBlock + 1];
    int u[kBlock];
    int beg[kBlock];
    int wsum[kWaves];
    int qnext;
    int flag;
    unsigned long long rmin;
};
constexpr size_t kSmallBytes = (sizeof(Small) + 15) & ~size_t(15);

struct DevGraph {
    int n;
    int prefer_direct;
    const int* __restrict__ row;     // out-CSR  (n+1)
    const int* __restrict__ col;
    const double* __restrict__ w;
    const double* __restrict__ r;
    const int* __restrict__ row_in;  // in-CSR (== out-CSR for undirected graphs)
    const int* __restrict__ col_in;
    const double* __restrict__ w_in;
    const double* __restrict__ r_in;
    const double* __restrict__ vf;     // 1 - vertex loss, NaN = absent
    const double* __restrict__ self_w; // self-loop latency, NaN = none
    const double* __restrict__ self_r;
};

__device__ inline double as_d(unsigned long long b) { return __longlong_as_double((long long)b); }
__device__ inline unsigned long long as_u(double d) { return (unsigned long long)__double_as_longlong(d); }

__device__ inline void raise_err(int* err, int code) { atomicCAS(err, 0, code); }

// dist[] is updated with atomicMin; in the HBM-resident variant those atomics run in
// L2, so reads must bypass this CU's L1 (agent-scope relaxed load -> sc1).
template <bool kLds>
__device__ inline unsigned long long ld_dist(unsigned long long* p) {
    if constexpr (kLds) return *p;
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool kLds>
__device__ inline unsigned ld_bits(unsigned* p) {
    if constexpr (kLds) return *p;
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive block scan of one int per thread; returns prefix, writes total.
__device__ inline int block_excl_scan(int x, Small* sm, int* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) sm->wsum[wv] = incl;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kWaves; k++) {
        int s = sm->wsum[k];
        pre += (k < wv) ? s : 0;
        tot += s;
    }
    *total = tot;
    return pre + incl - x;
}

// Binary search in row [lo,hi) of a sorted col array for `key`; -1 if absent.
__device__ inline int find_arc(const int* __restrict__ col, int lo, int hi, int key) {
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        int c = col[mid];
        if (c < key) lo = mid + 1;
        else if (c > key) hi = mid;
        else {
            while (mid > lo && col[mid - 1] == key) mid--;  // first of equal run (lowest eid)
            return mid;
        }
    }
    return -1;
}

// -----------------------------------------------------------------------------
// K1+K2: one workgroup per source.
//   phase A  frontier Bellman-Ford (push), dist as IEEE-754 bits with atomicMin
//            (non-negative doubles order like u64), load-balanced arc expansion
//            (block scan of frontier degrees + binary search of the owner), frontier
//            dedup by a bitmask, compaction by an LDS counter.
//   phase B  deterministic parent: tight in-arc with min (dist[u], u, eid).
//   phase C  reliability down the tree, level-synchronous (exact left fold from s).
//   phase D  row output (+ prefer-direct dispatch) and row min (K5 partial).
// kLds: per-source state in LDS (small graphs) or in a per-workgroup HBM slice.
template <bool kLds>
__global__ __launch_bounds__(kBlock) void sssp_rows_kernel(
    DevGraph g, const int* __restrict__ src, int ns, const int* __restrict__ tgt, int nt,
    long long ld, double* __restrict__ lat_out, double* __restrict__ rel_out,
    double* __restrict__ row_min, int* __restrict__ err, char* __restrict__ ws,
    size_t ws_stride, int dispatch) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Small* sm = reinterpret_cast<Small*>(smem);
    const int n = g.n;
    const int tid = threadIdx.x;
    const StateLayout L = StateLayout::make(n);
    char* base = kLds ? (smem + kSmallBytes) : (ws + (size_t)blockIdx.x * ws_stride);
    unsigned long long* dist = reinterpret_cast<unsigned long long*>(base + L.dist);
    double* relv = reinterpret_cast<double*>(base + L.relv);
    int* q0 = reinterpret_cast<int*>(base + L.q0);
    int* q1 = reinterpret_cast<int*>(base + L.q1);
    unsigned* bits = reinterpret_cast<unsigned*>(base + L.bits);
    const int nwords = (n + 31) >> 5;

    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (s < 0 || s >= n) {
            if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL);
            continue;
        }
        for (int v = tid; v < n; v += kBlock) dist[v] = kInfBits;
        for (int k = tid; k < nwords; k += kBlock) bits[k] = 0u;
        __syncthreads();
        if (tid == 0) {
            dist[s] = 0ull;
            q0[0] = s;
        }
        int* qc = q0;
        int* qn = q1;
        int qlen = 1;
        __syncthreads();

        // ---- phase A: frontier Bellman-Ford -------------------------------
        while (qlen > 0) {
            if (tid == 0) sm->qnext = 0;
            for (int c0 = 0; c0 < qlen; c0 += kBlock) {
                const int k = c0 + tid;
                int u = -1, beg = 0, deg = 0;
                if (k < qlen) {
                    u = qc[k];
                    atomicAnd(&bits[u >> 5], ~(1u << (u & 31)));  // u leaves the queue
                    beg = g.row[u];
                    deg = g.row[u + 1] - beg;
                }
                int total;
                int off = block_excl_scan(deg, sm, &total);
                const int cnt = min(kBlock, qlen - c0);
                sm->off[tid] = off;
                sm->u[tid] = u;
                sm->beg[tid] = beg;
                __syncthreads();
                for (int e = tid; e < total; e += kBlock) {
                    int lo = 0, hi = cnt;  // first index with off > e, minus one
                    while (lo < hi) {
                        int mid = (lo + hi) >> 1;
                        if (sm->off[mid] <= e) lo = mid + 1; else hi = mid;
                    }
                    const int o = lo - 1;
                    const int uu = sm->u[o];
                    const int a = sm->beg[o] + (e - sm->off[o]);
                    const int v = g.col[a];
                    const double nd = as_d(ld_dist<kLds>(&dist[uu])) + g.w[a];
                    const unsigned long long nb = as_u(nd);
                    if (nb < ld_dist<kLds>(&dist[v])) {
                        const unsigned long long old = atomicMin(&dist[v], nb);
                        if (nb < old) {
                            const unsigned m = 1u << (v & 31);
                            if (!(atomicOr(&bits[v >> 5], m) & m)) {
                                const int slot = atomicAdd(&sm->qnext, 1);
                                qn[slot] = v;
                            }
                        }
                    }
                }
                __syncthreads();
            }
            qlen = sm->qnext;
            int* t = qc; qc = qn; qn = t;
            __syncthreads();
        }

        // ---- phase B: deterministic parents (reuse q0 as parent[]) ----------
        int* par = q0;
        for (int v = tid; v < n; v += kBlock) {
            int pa = -1;
            const double dv = as_d(ld_dist<kLds>(&dist[v]));
            if (v != s && dv < INFINITY) {
                double bd = INFINITY;
                int bu = 0x7fffffff;
                const int e1 = g.row_in[v + 1];
                for (int a = g.row_in[v]; a < e1; a++) {
                    const int u = g.col_in[a];
                    const double du = as_d(ld_dist<kLds>(&dist[u]));
                    if (du + g.w_in[a] == dv && (du < bd || (du == bd && u < bu))) {
                        bd = du; bu = u; pa = a;
                    }
                }
            }
            par[v] = pa;
        }
        const double fs = g.vf[s];
        const double cs = isnan(fs) ? 1.0 : 1.0 * fs;
        for (int v = tid; v < n; v += kBlock) relv[v] = (v == s) ? cs : -1.0;
        __syncthreads();

        // ---- phase C: reliability down the tree, level-synchronous ----------
        for (;;) {
            if (tid == 0) sm->flag = 0;
            __syncthreads();
            int progressed = 0;
            for (int v = tid; v < n; v += kBlock) {
                const int pa = par[v];
                if (pa >= 0 && relv[v] < 0.0) {
                    const double ru = relv[g.col_in[pa]];
                    if (ru >= 0.0) {
                        relv[v] = ru * g.r_in[pa];
                        progressed = 1;
                    }
                }
            }
            if (progressed) sm->flag = 1;
            __syncthreads();
            const int again = sm->flag;
            __syncthreads();
            if (!again) break;
        }

        // ---- phase D: prefer-direct adjacency mask, row output, row min ------
        const bool pd = dispatch && g.prefer_direct;
        if (pd) {
            for (int k = tid; k < nwords; k += kBlock) bits[k] = 0u;
            __syncthreads();
            const int e1 = g.row[s + 1];
            for (int a = g.row[s] + tid; a < e1; a += kBlock) {
                const int v = g.col[a];
                atomicOr(&bits[v >> 5], 1u << (v & 31));
            }
            __syncthreads();
        }
        if (tid == 0) sm->rmin = kInfBits;
        __syncthreads();
        double lmin = INFINITY;
        double* lrow = lat_out ? lat_out + (long long)i * ld : nullptr;
        double* rrow = rel_out ? rel_out + (long long)i * ld : nullptr;
        for (int j = tid; j < nt; j += kBlock) {
            const int t = tgt[j];
            double Lv, Rv;
            if (t < 0 || t >= n) {
                raise_err(err, SHD_ROUTE_EINVAL);
                Lv = Rv = NAN;
            } else if (t == s) {
                const double ws_ = g.self_w[s];
                if (isnan(ws_)) {
                    raise_err(err, SHD_ROUTE_ENOEDGE);
                    Lv = Rv = NAN;
                } else if (pd) {  // direct (s,s): f_s applied twice (topology.c:1887-1921)
                    Lv = 0.0 + ws_;
                    double R = 1.0;
                    if (!isnan(fs)) R *= fs;
                    if (!isnan(fs)) R *= fs;
                    Rv = R * g.self_r[s];
                } else {          // batch path [s]: one self-loop hop (topology.c:1471-1499)
                    Lv = 0.0 + ws_;
                    Rv = cs * g.self_r[s];
                }
            } else if (pd && (ld_bits<kLds>(&bits[t >> 5]) & (1u << (t & 31)))) {
                const int a = find_arc(g.col, g.row[s], g.row[s + 1], t);
                const double ft = g.vf[t];
                double R = 1.0;
                if (!isnan(fs)) R *= fs;
                if (!isnan(ft)) R *= ft;
                Lv = 0.0 + g.w[a];
                Rv = R * g.r[a];
            } else {
                Lv = as_d(ld_dist<kLds>(&dist[t]));
                if (!(Lv < INFINITY)) {
                    raise_err(err, SHD_ROUTE_EUNREACH);
                    Lv = Rv = NAN;
                } else {
                    if (Lv == 0.0) Lv = 1.0;  // topology.c:1848-1852
                    const double ft = g.vf[t];
                    Rv = isnan(ft) ? relv[t] : relv[t] * ft;
                }
            }
            if (lrow) lrow[j] = Lv;
            if (rrow) rrow[j] = Rv;
            lmin = fmin(lmin, Lv);
        }
        if (row_min) {
            // wave min, then one LDS atomic per wave
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
            if ((tid & 63) == 0 && lmin < INFINITY) atomicMin(&sm->rmin, as_u(lmin));
            __syncthreads();
            if (tid == 0) row_min[i] = as_d(sm->rmin);
        }
        __syncthreads();
    }
}

// K3: direct paths from dense per-pair latency / reliability (complete graphs).
__global__ __launch_bounds__(kBlock) void direct_rows_kernel(
    int n, const double* __restrict__ W, const double* __restrict__ R, const double* __restrict__ vf,
    const int* __restrict__ src, int ns, const int* __restrict__ tgt, int nt, long long ld,
    double* __restrict__ lat_out, double* __restrict__ rel_out, double* __restrict__ row_min,
    int* __restrict__ err) {
    __shared__ unsigned long long rmin;
    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (threadIdx.x == 0) rmin = kInfBits;
        __syncthreads();
        double lmin = INFINITY;
        const double fs = (s >= 0 && s < n) ? vf[s] : NAN;
        for (int j = threadIdx.x; j < nt; j += kBlock) {
            const int t = tgt[j];
            double Lv = NAN, Rv = NAN;
            if (s < 0 || s >= n || t < 0 || t >= n) {
                raise_err(err, SHD_ROUTE_EINVAL);
            } else {
                const double w = W[(long long)s * n + t];
                if (isnan(w)) {
                    raise_err(err, SHD_ROUTE_ENOEDGE);
                } else {
                    const double ft = vf[t];
                    double Rr = 1.0;
                    if (!isnan(fs)) Rr *= fs;
                    if (!isnan(ft)) Rr *= ft;
                    Lv = 0.0 + w;
                    Rv = Rr * R[(long long)s * n + t];
                }
            }
            if (lat_out) lat_out[(long long)i * ld + j] = Lv;
            if (rel_out) rel_out[(long long)i * ld + j] = Rv;
            lmin = fmin(lmin, Lv);
        }
        if (row_min) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
            if ((threadIdx.x & 63) == 0 && lmin < INFINITY) atomicMin(&rmin, as_u(lmin));
            __syncthreads();
            if (threadIdx.x == 0) row_min[i] = as_d(rmin);
        }
        __syncthreads();
    }
}

// Self path: first minimum-latency incident edge in igraph incident order
// (ascending neighbour, the self-loop at its own position), used twice.
__global__ void self_kernel(DevGraph g, const int* __restrict__ vs, int nv, double* __restrict__ lat,
                            double* __restrict__ rel, int* __restrict__ err) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nv) return;
    const int v = vs[k];
    if (v < 0 || v >= g.n) { raise_err(err, SHD_ROUTE_EINVAL); lat[k] = rel[k] = NAN; return; }
    double mn = 0.0, rm = 0.0;
    bool any = false;
    const double sw = g.self_w[v];
    bool self_done = isnan(sw);
    const int e1 = g.row[v + 1];
    for (int a = g.row[v]; a <= e1; a++) {
        // interleave the self-loop before the first neighbour > v
        if (!self_done && (a == e1 || g.col[a] > v)) {
            if (mn == 0 || sw < mn) { mn = sw; rm = g.self_r[v]; }
            self_done = true; any = true;
        }
        if (a == e1) break;
        const double w = g.w[a];
        if (mn == 0 || w < mn) { mn = w; rm = g.r[a]; }
        any = true;
    }
    if (!any) { raise_err(err, SHD_ROUTE_ENOEDGE); lat[k] = rel[k] = NAN; return; }
    lat[k] = 2.0f * mn;
    rel[k] = rm * rm;
}

// K5: device-wide min of non-negative doubles; *out must hold +inf/0xFF.. bits first.
__global__ __launch_bounds__(kBlock) void min_reduce_kernel(const double* __restrict__ vals, long long count,
                                                            unsigned long long* __restrict__ out) {
    double m = INFINITY;
    for (long long k = blockIdx.x * (long long)kBlock + threadIdx.x; k < count;
         k += (long long)gridDim.x * kBlock)
        m = fmin(m, vals[k]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = fmin(m, __shfl_xor(m, d, 64));
    if ((threadIdx.x & 63) == 0 && m < INFINITY) atomicMin(out, as_u(m));
}

// Blocked min-plus Floyd-Warshall (K4), 32x32 tiles of doubles in LDS.
constexpr int kT = 32;
__global__ __launch_bounds__(kT * 8) void fw_diag_kernel(double* d, int n, int k0) {
    __shared__ double t[kT][kT + 1];
    const int tx = threadIdx.x & (kT - 1), ty0 = threadIdx.x / kT;
    for (int y = ty0; y < kT; y += 8) {
        int gi = k0 + y, gj = k0 + tx;
        t[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
    }
    __syncthreads();
    for (int k = 0; k < kT; k++) {
        for (int y = ty0; y < kT; y += 8) {
            double c = t[y][k] + t[k][tx];
            if (c < t[y][tx]) t[y][tx] = c;
        }
        __syncthreads();
    }
    for (int y = ty0; y < kT; y += 8) {
        int gi = k0 + y, gj = k0 + tx;
        if (gi < n && gj < n) d[(long long)gi * n + gj] = t[y][tx];
    }
}
__global__ __launch_bounds__(kT * 8) void fw_panel_kernel(double* d, int n, int k0) {
    // blockIdx.x = other tile index b (skip diagonal), blockIdx.y = 0 row panel, 1 col panel
    __shared__ double dg[kT][kT + 1];
    __shared__ double t[kT][kT + 1];
    const int nb = (n + kT - 1) / kT;
    int b = blockIdx.x;
    const int kb = k0 / kT;
    if (b >= kb) b++;
    if (b >= nb) return;
    const int tx = threadIdx.x & (kT - 1), ty0 = threadIdx.x / kT;
    const bool rowp = blockIdx.y == 0;  // tile (kb, b)
    const int bi = rowp ? k0 : b * kT, bj = rowp ? b * kT : k0;
    for (int y = ty0; y < kT; y += 8) {
        int gi = k0 + y, gj = k0 + tx;
        dg[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
        gi = bi + y; gj = bj + tx;
        t[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
    }
    __syncthreads();
    for (int k = 0; k < kT; k++) {
        for (int y = ty0; y < kT; y += 8) {
            double c = rowp ? dg[y][k] + t[k][tx] : t[y][k] + dg[k][tx];
            if (c < t[y][tx]) t[y][tx] = c;
        }
        __syncthreads();
    }
    for (int y = ty0; y < kT; y += 8) {
        int gi = bi + y, gj = bj + tx;
        if (gi < n && gj < n) d[(long long)gi * n + gj] = t[y][tx];
    }
}
__global__ __launch_bounds__(kT * 8) void fw_rest_kernel(double* d, int n, int k0) {
    __shared__ double rp[kT][kT + 1];  // row panel tile (k, bj)
    __shared__ double cp[kT][kT + 1];  // col panel tile (bi, k)
    const int bi = blockIdx.y * kT, bj = blockIdx.x * kT;
    if (bi == k0 || bj == k0) return;
    const int tx = threadIdx.x & (kT - 1), ty0 = threadIdx.x / kT;
    double acc[kT / 8];
    for (int q = 0; q < kT / 8; q++) {
        int y = ty0 + 8 * q;
        int gi = k0 + y, gj = bj + tx;
        rp[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
        gi = bi + y; gj = k0 + tx;
        cp[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
        gi = bi + y; gj = bj + tx;
        acc[q] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
    }
    __syncthreads();
    for (int k = 0; k < kT; k++) {
        const double b = rp[k][tx];
#pragma unroll
        for (int q = 0; q < kT / 8; q++) {
            double c = cp[ty0 + 8 * q][k] + b;
            acc[q] = c < acc[q] ? c : acc[q];
        }
    }
    for (int q = 0; q < kT / 8; q++) {
        int gi = bi + ty0 + 8 * q, gj = bj + tx;
        if (gi < n && gj < n) d[(long long)gi * n + gj] = acc[q];
    }
}

}  // namespace

// =============================================================================
// Host side
// =============================================================================
struct shd_route {
    int device = 0;
    int n = 0, m = 0, nnz = 0;
    int directed = 0, prefer_direct = 0, complete = 0, integer_w = 0, multigraph = 0;
    double min_w = 0;
    // device graph
    int* d_row = nullptr; int* d_col = nullptr; double* d_w = nullptr; double* d_r = nullptr;
    int* d_row_in = nullptr; int* d_col_in = nullptr; double* d_w_in = nullptr; double* d_r_in = nullptr;
    double* d_vf = nullptr; double* d_self_w = nullptr; double* d_self_r = nullptr;
    double* d_W = nullptr; double* d_R = nullptr;  // dense direct tables (complete graphs, lazy)
    int* d_err = nullptr;
    char* d_ws = nullptr; size_t ws_stride = 0; int ws_slots = 0;
    bool lds = false;
    size_t lds_bytes = 0;
    uint64_t device_bytes = 0;
    // host copies needed for lazy dense build
    std::vector<int32_t> e_src, e_dst;
    std::vector<double> e_lat, e_rel;
    std::vector<void*> allocs;
};

namespace {

int hip_check(hipError_t e) { return e == hipSuccess ? SHD_ROUTE_OK : SHD_ROUTE_EDEVICE; }

template <typename T>
int upload(shd_route* c, T** dptr, const std::vector<T>& h) {
    size_t bytes = sizeof(T) * (h.empty() ? 1 : h.size());
    if (hipMalloc((void**)dptr, bytes) != hipSuccess) return SHD_ROUTE_ENOMEM;
    c->allocs.push_back(*dptr);
    c->device_bytes += bytes;
    if (!h.empty() && hipMemcpy(*dptr, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    return SHD_ROUTE_OK;
}

DevGraph dev_graph(const shd_route* c) {
    DevGraph g;
    g.n = c->n; g.prefer_direct = c->prefer_direct;
    g.row = c->d_row; g.col = c->d_col; g.w = c->d_w; g.r = c->d_r;
    g.row_in = c->d_row_in; g.col_in = c->d_col_in; g.w_in = c->d_w_in; g.r_in = c->d_r_in;
    g.vf = c->d_vf; g.self_w = c->d_self_w; g.self_r = c->d_self_r;
    return g;
}

// Build a CSR (rows by `key`, columns by `other`), arcs sorted by (row, col, eid).
void build_csr(int n, const std::vector<int32_t>& rows, const std::vector<int32_t>& cols,
               const std::vector<int32_t>& eids, const std::vector<double>& lat,
               const std::vector<double>& rel, std::vector<int>& row, std::vector<int>& col,
               std::vector<double>& w, std::vector<double>& r) {
    const size_t k = rows.size();
    std::vector<size_t> idx(k);
    std::iota(idx.begin(), idx.end(), 0);
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
        if (rows[a] != rows[b]) return rows[a] < rows[b];
        if (cols[a] != cols[b]) return cols[a] < cols[b];
        return eids[a] < eids[b];
    });
    row.assign(n + 1, 0);
    col.resize(k); w.resize(k); r.resize(k);
    for (size_t q = 0; q < k; q++) {
        size_t a = idx[q];
        row[rows[a] + 1]++;
        col[q] = cols[a];
        w[q] = lat[eids[a]];
        r[q] = rel[eids[a]];
    }
    for (int v = 0; v < n; v++) row[v + 1] += row[v];
}

bool strongly_connected(int n, const std::vector<int>& row, const std::vector<int>& col,
                        const std::vector<int>& row_in, const std::vector<int>& col_in) {
    auto reach_all = [&](const std::vector<int>& R, const std::vector<int>& Cc) {
        std::vector<char> seen(n, 0);
        std::vector<int> st{0};
        seen[0] = 1;
        int cnt = 1;
        while (!st.empty()) {
            int u = st.back(); st.pop_back();
            for (int a = R[u]; a < R[u + 1]; a++)
                if (!seen[Cc[a]]) { seen[Cc[a]] = 1; cnt++; st.push_back(Cc[a]); }
        }
        return cnt == n;
    };
    return reach_all(row, col) && reach_all(row_in, col_in);
}

int alloc_ws(shd_route* c) {
    // per-source state in HBM when it cannot live in LDS
    StateLayout L = StateLayout::make(c->n);
    c->ws_stride = a16(L.total) + 256;
    c->ws_slots = 1024;  // 256 CUs x 4 workgroups
    size_t bytes = c->ws_stride * (size_t)c->ws_slots;
    if (hipMalloc((void**)&c->d_ws, bytes) != hipSuccess) return SHD_ROUTE_ENOMEM;
    c->allocs.push_back(c->d_ws);
    return SHD_ROUTE_OK;
}

int ensure_dense(shd_route* c) {
    if (c->d_W) return SHD_ROUTE_OK;
    const size_t nn = (size_t)c->n * c->n;
    std::vector<double> W(nn, NAN), R(nn, NAN);
    // igraph_get_eid on a simple graph returns the unique edge; for parallel edges we
    // keep the lowest edge id (documented deviation, SURVEY hazard H3).
    for (int e = c->m - 1; e >= 0; e--) {
        int a = c->e_src[e], b = c->e_dst[e];
        W[(size_t)a * c->n + b] = c->e_lat[e];
        R[(size_t)a * c->n + b] = c->e_rel[e];
        if (!c->directed) {
            W[(size_t)b * c->n + a] = c->e_lat[e];
            R[(size_t)b * c->n + a] = c->e_rel[e];
        }
    }
    int rc = upload(c, &c->d_W, W);
    if (rc) return rc;
    return upload(c, &c->d_R, R);
}

int take_err(shd_route* c) {
    int h = 0;
    if (hipMemcpy(&h, c->d_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (h) {
        int z = 0;
        if (hipMemcpy(c->d_err, &z, sizeof(int), hipMemcpyHostToDevice) != hipSuccess) return SHD_ROUTE_EDEVICE;
    }
    return h;
}

}  // namespace

extern "C" {

const char* shd_route_strerror(int code) {
    switch (code) {
        case SHD_ROUTE_OK: return "success";
        case SHD_ROUTE_EINVAL: return "invalid argument or topology failed validation";
        case SHD_ROUTE_ENOMEM: return "out of memory";
        case SHD_ROUTE_EDEVICE: return "HIP device error";
        case SHD_ROUTE_ENOEDGE: return "path hop without an edge (missing self-loop?)";
        case SHD_ROUTE_EUNREACH: return "target unreachable";
        case SHD_ROUTE_EUNSUPPORTED: return "unsupported request";
        default: return "unknown error";
    }
}

int shd_route_create(shd_route_t** out, const shd_graph_t* g, int device) {
    if (!out || !g) return SHD_ROUTE_EINVAL;
    *out = nullptr;
    const int n = g->n_vertices, m = g->n_edges;
    if (n <= 0 || m < 0 || (m > 0 && (!g->edge_src || !g->edge_dst || !g->edge_latency || !g->edge_packetloss)))
        return SHD_ROUTE_EINVAL;
    // validation as topology.c:1041-1124 (edges) and 811-978 (vertex packetloss)
    for (int e = 0; e < m; e++) {
        int a = g->edge_src[e], b = g->edge_dst[e];
        double w = g->edge_latency[e], p = g->edge_packetloss[e];
        if (a < 0 || a >= n || b < 0 || b >= n) return SHD_ROUTE_EINVAL;
        if (!(w > 0.0) || std::isinf(w)) return SHD_ROUTE_EINVAL;
        if (!(p >= 0.0 && p <= 1.0)) return SHD_ROUTE_EINVAL;
    }
    if (g->vertex_packetloss)
        for (int v = 0; v < n; v++) {
            double p = g->vertex_packetloss[v];
            if (!std::isnan(p) && !(p >= 0.0 && p <= 1.0)) return SHD_ROUTE_EINVAL;
        }
    if (hipSetDevice(device) != hipSuccess) return SHD_ROUTE_EDEVICE;

    shd_route* c = new (std::nothrow) shd_route();
    if (!c) return SHD_ROUTE_ENOMEM;
    c->device = device; c->n = n; c->m = m;
    c->directed = g->directed ? 1 : 0;
    c->prefer_direct = g->prefer_direct ? 1 : 0;
    c->e_src.assign(g->edge_src, g->edge_src + m);
    c->e_dst.assign(g->edge_dst, g->edge_dst + m);
    c->e_lat.assign(g->edge_latency, g->edge_latency + m);
    c->e_rel.resize(m);
    for (int e = 0; e < m; e++) c->e_rel[e] = (1.0f - g->edge_packetloss[e]);  // topology.c:437

    // arcs for SSSP (self-loops excluded: w > 0 never relaxes them)
    std::vector<int32_t> ar, ac, ae, ir, ic, ie;
    std::vector<double> self_w(n, NAN), self_r(n, NAN);
    std::vector<int> loops(n, 0), degm(n, 0);
    double maxw = 0;
    c->min_w = m ? INFINITY : 0;
    bool integral = true;
    for (int e = 0; e < m; e++) {
        int a = g->edge_src[e], b = g->edge_dst[e];
        double w = g->edge_latency[e];
        maxw = std::max(maxw, w);
        c->min_w = std::min(c->min_w, w);
        if (w != std::floor(w) || w > 1048576.0) integral = false;
        if (a == b) {
            if (std::isnan(self_w[a])) { self_w[a] = w; self_r[a] = c->e_rel[e]; }
            loops[a]++;
            continue;
        }
        ar.push_back(a); ac.push_back(b); ae.push_back(e);
        degm[a]++;
        if (!c->directed) { ar.push_back(b); ac.push_back(a); ae.push_back(e); degm[b]++; }
        else { ir.push_back(b); ic.push_back(a); ie.push_back(e); }
    }
    c->integer_w = integral && (double)n * maxw < 2147483647.0;
    std::vector<int> row, col, row_in, col_in;
    std::vector<double> w, r, w_in, r_in;
    build_csr(n, ar, ac, ae, c->e_lat, c->e_rel, row, col, w, r);
    if (c->directed) build_csr(n, ir, ic, ie, c->e_lat, c->e_rel, row_in, col_in, w_in, r_in);
    c->nnz = (int)col.size();
    for (int v = 0; v < n && !c->multigraph; v++)
        for (int a = row[v] + 1; a < row[v + 1]; a++)
            if (col[a] == col[a - 1]) { c->multigraph = 1; break; }
    for (int v = 0; v < n; v++) if (loops[v] > 1) c->multigraph = 1;

    // topology.c:738-806: strongly connected, one cluster
    if (!strongly_connected(n, row, col, c->directed ? row_in : row, c->directed ? col_in : col)) {
        delete c;
        return SHD_ROUTE_EINVAL;
    }
    // topology.c:450-552 isComplete: OUT-incident count (undirected: loops twice, minus one)
    c->complete = 1;
    for (int v = 0; v < n; v++) {
        long long ecount;
        if (c->directed) ecount = (row[v + 1] - row[v]) + loops[v];
        else ecount = (row[v + 1] - row[v]) + 2LL * loops[v] - (loops[v] > 0 ? 1 : 0);
        if (ecount < n) { c->complete = 0; break; }
    }

    std::vector<double> vf(n, NAN);
    if (g->vertex_packetloss)
        for (int v = 0; v < n; v++)
            if (!std::isnan(g->vertex_packetloss[v])) vf[v] = (1.0f - g->vertex_packetloss[v]);

    int rc = SHD_ROUTE_OK;
    if (!rc) rc = upload(c, &c->d_row, row);
    if (!rc) rc = upload(c, &c->d_col, col);
    if (!rc) rc = upload(c, &c->d_w, w);
    if (!rc) rc = upload(c, &c->d_r, r);
    if (c->directed) {
        if (!rc) rc = upload(c, &c->d_row_in, row_in);
        if (!rc) rc = upload(c, &c->d_col_in, col_in);
        if (!rc) rc = upload(c, &c->d_w_in, w_in);
        if (!rc) rc = upload(c, &c->d_r_in, r_in);
    } else {
        c->d_row_in = c->d_row; c->d_col_in = c->d_col; c->d_w_in = c->d_w; c->d_r_in = c->d_r;
    }
    if (!rc) rc = upload(c, &c->d_vf, vf);
    if (!rc) rc = upload(c, &c->d_self_w, self_w);
    if (!rc) rc = upload(c, &c->d_self_r, self_r);
    if (!rc) {
        std::vector<int> z(1, 0);
        rc = upload(c, &c->d_err, z);
    }
    StateLayout L = StateLayout::make(n);
    c->lds_bytes = kSmallBytes + L.total;
    c->lds = c->lds_bytes <= kLdsBudget;
    if (!rc) {
        if (c->lds) {
            rc = hip_check(hipFuncSetAttribute((const void*)sssp_rows_kernel<true>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds_bytes));
        } else {
            rc = alloc_ws(c);
        }
    }
    if (rc) {
        shd_route_destroy(c);
        return rc;
    }
    *out = c;
    return SHD_ROUTE_OK;
}

void shd_route_destroy(shd_route_t* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (void* p : c->allocs) (void)hipFree(p);
    delete c;
}

int shd_route_get_info(const shd_route_t* c, shd_route_info_t* info) {
    if (!c || !info) return SHD_ROUTE_EINVAL;
    info->n_vertices = c->n;
    info->n_edges = c->m;
    info->n_arcs = c->nnz;
    info->is_complete = c->complete;
    info->directed = c->directed;
    info->prefer_direct = c->prefer_direct;
    info->integer_weights = c->integer_w;
    info->multigraph = c->multigraph;
    info->device = c->device;
    info->lds_resident = c->lds ? 1 : 0;
    info->device_bytes = c->device_bytes;
    info->min_edge_latency = c->min_w;
    return SHD_ROUTE_OK;
}

int shd_route_rows_async(shd_route_t* c, const int32_t* d_src, int32_t ns, const int32_t* d_tgt,
                         int32_t nt, int64_t ld, uint32_t flags, double* d_lat, double* d_rel,
                         double* d_row_min, void* stream) {
    if (!c || ns < 0 || nt < 0 || (ns && !d_src) || (nt && !d_tgt) || ld < nt) return SHD_ROUTE_EINVAL;
    if (ns == 0) return SHD_ROUTE_OK;
    hipStream_t st = (hipStream_t)stream;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if ((flags & SHD_ROUTE_DISPATCH) && c->complete) {
        int rc = ensure_dense(c);
        if (rc) return rc;
        int grid = std::min(ns, 65535);
        hipLaunchKernelGGL(direct_rows_kernel, dim3(grid), dim3(kBlock), 0, st, c->n, c->d_W, c->d_R,
                           c->d_vf, d_src, ns, d_tgt, nt, (long long)ld, d_lat, d_rel, d_row_min, c->d_err);
        return hip_check(hipGetLastError());
    }
    DevGraph g = dev_graph(c);
    const int dispatch = (flags & SHD_ROUTE_DISPATCH) ? 1 : 0;
    if (c->lds) {
        int grid = std::min(ns, 1 << 20);
        hipLaunchKernelGGL(sssp_rows_kernel<true>, dim3(grid), dim3(kBlock), c->lds_bytes, st, g, d_src, ns,
                           d_tgt, nt, (long long)ld, d_lat, d_rel, d_row_min, c->d_err, nullptr, (size_t)0,
                           dispatch);
    } else {
        int grid = std::min(ns, c->ws_slots);
        hipLaunchKernelGGL(sssp_rows_kernel<false>, dim3(grid), dim3(kBlock), kSmallBytes, st, g, d_src, ns,
                           d_tgt, nt, (long long)ld, d_lat, d_rel, d_row_min, c->d_err, c->d_ws, c->ws_stride,
                           dispatch);
    }
    return hip_check(hipGetLastError());
}

int shd_route_sync(shd_route_t* c, void* stream) {
    if (!c) return SHD_ROUTE_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return SHD_ROUTE_EDEVICE;
    return take_err(c);
}

}  // extern "C"

namespace {
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
    int alloc(size_t b) { return hipMalloc(&p, b ? b : 1) == hipSuccess ? SHD_ROUTE_OK : SHD_ROUTE_ENOMEM; }
};

// Host-pointer wrapper: chunks rows so device output stays bounded, copies back.
template <typename Launch>
int host_rows(shd_route* c, const int32_t* src, int32_t ns, const int32_t* tgt, int32_t nt, double* lat_out,
              double* rel_out, double* row_min_out, Launch launch) {
    if (!c || ns < 0 || nt < 0 || (ns && !src) || (nt && !tgt)) return SHD_ROUTE_EINVAL;
    if (ns == 0) return SHD_ROUTE_OK;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    const size_t row_bytes = sizeof(double) * (size_t)std::max(nt, 1);
    int32_t chunk = (int32_t)std::max<size_t>(1, std::min<size_t>(ns, (size_t)(1u << 30) / row_bytes));
    DevBuf dsrc, dtgt, dlat, drel, dmin;
    int rc;
    if ((rc = dsrc.alloc(sizeof(int32_t) * chunk)) || (rc = dtgt.alloc(sizeof(int32_t) * std::max(nt, 1))) ||
        (rc = dlat.alloc(row_bytes * chunk)) || (rc = drel.alloc(row_bytes * chunk)) ||
        (rc = dmin.alloc(sizeof(double) * chunk)))
        return rc;
    if (nt && hipMemcpy(dtgt.p, tgt, sizeof(int32_t) * nt, hipMemcpyHostToDevice) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    for (int32_t i0 = 0; i0 < ns; i0 += chunk) {
        int32_t k = std::min(chunk, ns - i0);
        if (hipMemcpy(dsrc.p, src + i0, sizeof(int32_t) * k, hipMemcpyHostToDevice) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
        rc = launch((const int32_t*)dsrc.p, k, (const int32_t*)dtgt.p, (double*)dlat.p, (double*)drel.p,
                    (double*)dmin.p);
        if (rc) return rc;
        if ((rc = shd_route_sync(c, nullptr))) return rc;
        if (lat_out && hipMemcpy(lat_out + (size_t)i0 * nt, dlat.p, row_bytes * k, hipMemcpyDeviceToHost) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
        if (rel_out && hipMemcpy(rel_out + (size_t)i0 * nt, drel.p, row_bytes * k, hipMemcpyDeviceToHost) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
        if (row_min_out && hipMemcpy(row_min_out + i0, dmin.p, sizeof(double) * k, hipMemcpyDeviceToHost) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
    }
    return SHD_ROUTE_OK;
}
}  // namespace

extern "C" {

int shd_route_rows(shd_route_t* c, const int32_t* src, int32_t ns, const int32_t* tgt, int32_t nt,
                   uint32_t flags, double* lat_out, double* rel_out, double* row_min_out) {
    return host_rows(c, src, ns, tgt, nt, lat_out, rel_out, row_min_out,
                     [&](const int32_t* ds, int32_t k, const int32_t* dt, double* dl, double* dr, double* dm) {
                         return shd_route_rows_async(c, ds, k, dt, nt, nt, flags, dl, dr, dm, nullptr);
                     });
}

int shd_route_direct(shd_route_t* c, const int32_t* src, int32_t ns, const int32_t* tgt, int32_t nt,
                     double* lat_out, double* rel_out, double* row_min_out) {
    if (!c) return SHD_ROUTE_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    int rc = ensure_dense(c);
    if (rc) return rc;
    return host_rows(c, src, ns, tgt, nt, lat_out, rel_out, row_min_out,
                     [&](const int32_t* ds, int32_t k, const int32_t* dt, double* dl, double* dr, double* dm) {
                         int grid = std::min(k, 65535);
                         hipLaunchKernelGGL(direct_rows_kernel, dim3(grid), dim3(kBlock), 0, nullptr, c->n, c->d_W,
                                            c->d_R, c->d_vf, ds, k, dt, nt, (long long)nt, dl, dr, dm, c->d_err);
                         return hip_check(hipGetLastError());
                     });
}

int shd_route_self(shd_route_t* c, const int32_t* v, int32_t nv, double* lat_out, double* rel_out) {
    if (!c || nv < 0 || (nv && (!v || !lat_out || !rel_out))) return SHD_ROUTE_EINVAL;
    if (nv == 0) return SHD_ROUTE_OK;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    DevBuf dv, dl, dr;
    int rc;
    if ((rc = dv.alloc(sizeof(int32_t) * nv)) || (rc = dl.alloc(sizeof(double) * nv)) ||
        (rc = dr.alloc(sizeof(double) * nv)))
        return rc;
    if (hipMemcpy(dv.p, v, sizeof(int32_t) * nv, hipMemcpyHostToDevice) != hipSuccess) return SHD_ROUTE_EDEVICE;
    DevGraph g = dev_graph(c);
    hipLaunchKernelGGL(self_kernel, dim3((nv + 255) / 256), dim3(256), 0, nullptr, g, (const int*)dv.p, nv,
                       (double*)dl.p, (double*)dr.p, c->d_err);
    if ((rc = hip_check(hipGetLastError()))) return rc;
    if ((rc = shd_route_sync(c, nullptr))) return rc;
    if (hipMemcpy(lat_out, dl.p, sizeof(double) * nv, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(rel_out, dr.p, sizeof(double) * nv, hipMemcpyDeviceToHost) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    return SHD_ROUTE_OK;
}

int shd_route_min_reduce_async(shd_route_t* c, const double* d_vals, int64_t count, double* d_out, void* stream) {
    if (!c || count < 0 || !d_out || (count && !d_vals)) return SHD_ROUTE_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (hipMemsetAsync(d_out, 0xFF, sizeof(double), st) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (count == 0) return SHD_ROUTE_OK;
    long long blocks = std::min<long long>((count + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(min_reduce_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, d_vals, (long long)count,
                       (unsigned long long*)d_out);
    return hip_check(hipGetLastError());
}

int shd_route_fw_async(shd_route_t* c, double* d_dist, void* stream) {
    if (!c || !d_dist) return SHD_ROUTE_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    const int n = c->n;
    const int nb = (n + kT - 1) / kT;
    for (int kb = 0; kb < nb; kb++) {
        const int k0 = kb * kT;
        hipLaunchKernelGGL(fw_diag_kernel, dim3(1), dim3(kT * 8), 0, st, d_dist, n, k0);
        if (nb > 1)
            hipLaunchKernelGGL(fw_panel_kernel, dim3(nb - 1, 2), dim3(kT * 8), 0, st, d_dist, n, k0);
        hipLaunchKernelGGL(fw_rest_kernel, dim3(nb, nb), dim3(kT * 8), 0, st, d_dist, n, k0);
    }
    return hip_check(hipGetLastError());
}

}  // extern "C"
