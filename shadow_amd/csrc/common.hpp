#pragma once
// common.hpp -- shared device helpers and layouts for the routing kernels.
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
#include <type_traits>
#include <vector>

#include "../../include/shd_route.h"

namespace shd {

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

}  // namespace shd
