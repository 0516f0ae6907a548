#pragma once
// "KB": batched multi-source shortest-path distances + deterministic parents for small
// topologies whose compressed in-CSR fits in LDS (C2-class: n ~ 2k, 20k arcs).
//
// Replaces igraph_get_shortest_paths_dijkstra (topology.c:1756) for KB_SRC sources per
// workgroup at once.  Integer latencies only (exact, see sssp_k32.hpp); the engine
// proves every shortest-path latency <= bound < 0xFFFF, so u16 distances are exact.
//
// Layout: distances for the batch are stored source-minor, D[v][0..7] as eight u16 in
// 16 bytes, so one ds_read_b128 fetches a neighbour's distance to all 8 sources and
// four v_pk_add_u16 (saturating) + four v_pk_min_u16 relax an arc for all of them.
// Sweeps are pull-based over in-rows (Gauss-Seidel, in place, monotone): no atomics,
// no frontier queues.  Rows longer than KB_SEG arcs are split into segments whose
// partial minima are combined in a second pass ("hubs").
//
// After convergence the same segment walk finds, for each (v, source), the FIRST tight
// arc of v's in-row; in-rows are sorted by (-w, u, eid) so that is argmin (dist[u], u,
// eid), the engine tie rule.  Output: key[i][v] = dist16 << 16 | slot16 rows in HBM,
// consumed by path_attr_kernel (path_attr.hpp).
#include "common.hpp"

namespace shd {

constexpr int KB_SRC = 8;     // sources per workgroup (u16 x 8 = 16 bytes per vertex)
constexpr int KB_SEG = 16;    // max arcs per segment
constexpr int KB_BLOCK = 1024;

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

struct KBSeg {   // one pass-1 work item
    int v;       // head vertex
    int a0, a1;  // in-arc range [a0, a1)
    int p;       // -1: whole row (write D[v] directly); else partial slot index
};
struct KBHub {
    int v, p0, p1, pad;
};

struct DevKB {
    int n, nnz, nseg, nhub, npart;
    int bound;
    const uint32_t* __restrict__ arc;   // in-arcs (u << 16 | w), rows sorted by (-w, u, eid)
    const int* __restrict__ row_in;     // in-CSR offsets (n+1)
    const KBSeg* __restrict__ seg;
    const KBHub* __restrict__ hub;
    unsigned long long* dbg;   // SHD_STAMPS builds: 8 words per workgroup
};
#ifdef SHD_STAMPS
#define KB_STAMP(slot) do { if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + (slot)] += __builtin_amdgcn_s_memtime(); } while (0)
#define KB_COUNT(slot) do { if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + (slot)] += 1; } while (0)
#else
#define KB_STAMP(slot) do { } while (0)
#define KB_COUNT(slot) do { } while (0)
#endif

struct KBLayout {
    size_t arc, D, P, total;
    __host__ __device__ static KBLayout make(int n, int nnz, int npart) {
        KBLayout L;
        size_t o = 0;
        L.arc = o; o += a16(sizeof(uint32_t) * (size_t)nnz);
        L.D = o;   o += a16((size_t)16 * n);
        L.P = o;   o += a16((size_t)16 * npart);
        L.total = o;
        return L;
    }
};
constexpr size_t kKBSmall = 16;

struct u16x8 { us2 h[4]; };

__device__ inline u16x8 ld8(const char* p) {
    const uint4 x = *reinterpret_cast<const uint4*>(p);
    u16x8 r;
    r.h[0] = __builtin_bit_cast(us2, x.x); r.h[1] = __builtin_bit_cast(us2, x.y);
    r.h[2] = __builtin_bit_cast(us2, x.z); r.h[3] = __builtin_bit_cast(us2, x.w);
    return r;
}
__device__ inline void st8(char* p, const u16x8& v) {
    uint4 x;
    x.x = __builtin_bit_cast(uint32_t, v.h[0]); x.y = __builtin_bit_cast(uint32_t, v.h[1]);
    x.z = __builtin_bit_cast(uint32_t, v.h[2]); x.w = __builtin_bit_cast(uint32_t, v.h[3]);
    *reinterpret_cast<uint4*>(p) = x;
}
__device__ inline bool eq8(const u16x8& a, const u16x8& b) {
    return __builtin_bit_cast(uint32_t, a.h[0]) == __builtin_bit_cast(uint32_t, b.h[0]) &&
           __builtin_bit_cast(uint32_t, a.h[1]) == __builtin_bit_cast(uint32_t, b.h[1]) &&
           __builtin_bit_cast(uint32_t, a.h[2]) == __builtin_bit_cast(uint32_t, b.h[2]) &&
           __builtin_bit_cast(uint32_t, a.h[3]) == __builtin_bit_cast(uint32_t, b.h[3]);
}
__device__ inline u16x8 inf8() {
    u16x8 r;
    const us2 f = {0xFFFF, 0xFFFF};
    r.h[0] = r.h[1] = r.h[2] = r.h[3] = f;
    return r;
}
__device__ inline u16x8 min8(const u16x8& a, const u16x8& b) {
    u16x8 r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.h[k] = __builtin_elementwise_min(a.h[k], b.h[k]);
    return r;
}
__device__ inline u16x8 addsat8(const u16x8& a, us2 w) {
    u16x8 r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.h[k] = __builtin_elementwise_add_sat(a.h[k], w);
    return r;
}

__device__ inline us2 wsplat(uint32_t rec) {
    const unsigned short w = (unsigned short)(rec & 0xFFFFu);
    const us2 r = {w, w};
    return r;
}

// min over arcs [a0, a1) of D[u] + w, four independent arc/distance reads in flight.
__device__ inline u16x8 relax_row(const uint32_t* arc, const char* D, int a0, int a1) {
    u16x8 acc = inf8();
    int a = a0;
    for (; a + 4 <= a1; a += 4) {
        const uint32_t r0 = arc[a], r1 = arc[a + 1], r2 = arc[a + 2], r3 = arc[a + 3];
        const u16x8 d0 = ld8(D + (size_t)16 * (r0 >> 16));
        const u16x8 d1 = ld8(D + (size_t)16 * (r1 >> 16));
        const u16x8 d2 = ld8(D + (size_t)16 * (r2 >> 16));
        const u16x8 d3 = ld8(D + (size_t)16 * (r3 >> 16));
        acc = min8(min8(acc, addsat8(d0, wsplat(r0))), addsat8(d1, wsplat(r1)));
        acc = min8(min8(acc, addsat8(d2, wsplat(r2))), addsat8(d3, wsplat(r3)));
    }
    for (; a < a1; a++) {
        const uint32_t r0 = arc[a];
        acc = min8(acc, addsat8(ld8(D + (size_t)16 * (r0 >> 16)), wsplat(r0)));
    }
    return acc;
}

__global__ __launch_bounds__(KB_BLOCK) void sssp_batch_kernel(DevKB g, const int* __restrict__ src, int ns,
                                                              uint32_t* __restrict__ keys, long long kld,
                                                              int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* changed = reinterpret_cast<int*>(smem);
    const KBLayout L = KBLayout::make(g.n, g.nnz, g.npart);
    char* base = smem + kKBSmall;
    uint32_t* arc = reinterpret_cast<uint32_t*>(base + L.arc);
    char* D = base + L.D;
    char* P = base + L.P;
    const int tid = threadIdx.x;
    const int n = g.n;

    if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + 0] = __builtin_amdgcn_s_memtime();
    // stage the in-CSR into LDS once per workgroup (16-byte loads)
    {
        const int nq = (g.nnz + 3) / 4;
        const uint4* s4 = reinterpret_cast<const uint4*>(g.arc);
        uint4* d4 = reinterpret_cast<uint4*>(arc);
        for (int q = tid; q < nq; q += KB_BLOCK) d4[q] = s4[q];
    }

    for (int i0 = blockIdx.x * KB_SRC; i0 < ns; i0 += gridDim.x * KB_SRC) {
        int sb[KB_SRC];
#pragma unroll
        for (int b = 0; b < KB_SRC; b++) {
            const int i = i0 + b;
            int sv = -1;
            if (i < ns) {
                sv = src[i];
                if (sv < 0 || sv >= n) { if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL); sv = -1; }
            }
            sb[b] = sv;
        }
        // init: INF everywhere, 0 at each source's own lane
        for (int v = tid; v < n; v += KB_BLOCK) {
            u16x8 d = inf8();
#pragma unroll
            for (int b = 0; b < KB_SRC; b++)
                if (sb[b] == v) d.h[b >> 1][b & 1] = 0;
            st8(D + (size_t)16 * v, d);
        }
        __syncthreads();

        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + 1] = __builtin_amdgcn_s_memtime();
        // ---- Gauss-Seidel pull sweeps to the fixed point -------------------------
        for (;;) {
            KB_COUNT(4);
            if (tid == 0) *changed = 0;
            __syncthreads();
            int ch = 0;
            for (int k = tid; k < g.nseg; k += KB_BLOCK) {
                const KBSeg sg = g.seg[k];
                const u16x8 acc = relax_row(arc, D, sg.a0, sg.a1);
                if (sg.p < 0) {
                    const u16x8 old = ld8(D + (size_t)16 * sg.v);
                    const u16x8 nw = min8(old, acc);
                    if (!eq8(nw, old)) { st8(D + (size_t)16 * sg.v, nw); ch = 1; }
                } else {
                    st8(P + (size_t)16 * sg.p, acc);
                }
            }
            __syncthreads();
            for (int k = tid; k < g.nhub; k += KB_BLOCK) {
                const KBHub h = g.hub[k];
                u16x8 acc = ld8(D + (size_t)16 * h.v);
                const u16x8 old = acc;
                for (int p = h.p0; p < h.p1; p++) acc = min8(acc, ld8(P + (size_t)16 * p));
                if (!eq8(acc, old)) { st8(D + (size_t)16 * h.v, acc); ch = 1; }
            }
            if (ch) *changed = 1;
            __syncthreads();
            const int again = *changed;
            __syncthreads();
            if (!again) break;
        }

        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + 2] = __builtin_amdgcn_s_memtime();
        // ---- parents: first tight arc of each in-row, per source -----------------
        for (int k = tid; k < g.nseg; k += KB_BLOCK) {
            const KBSeg sg = g.seg[k];
            const u16x8 dv = ld8(D + (size_t)16 * sg.v);
            unsigned short slot[KB_SRC];
#pragma unroll
            for (int b = 0; b < KB_SRC; b++) slot[b] = 0xFFFFu;
            const int r0 = g.row_in[sg.v];
            for (int a = sg.a0; a < sg.a1; a += 4) {
                u16x8 c[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t rec = arc[min(a + q, sg.a1 - 1)];
                    c[q] = addsat8(ld8(D + (size_t)16 * (rec >> 16)), wsplat(rec));
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (a + q >= sg.a1) break;
#pragma unroll
                    for (int b = 0; b < KB_SRC; b++) {
                        const unsigned short cb = c[q].h[b >> 1][b & 1], db = dv.h[b >> 1][b & 1];
                        if (slot[b] == 0xFFFFu && db != 0xFFFFu && cb == db) slot[b] = (unsigned short)(a + q - r0);
                    }
                }
            }
            if (sg.p < 0) {
#pragma unroll
                for (int b = 0; b < KB_SRC; b++) {
                    if (sb[b] < 0) continue;
                    const unsigned short db = dv.h[b >> 1][b & 1];
                    uint32_t kv;
                    if (sg.v == sb[b]) kv = 0u;
                    else if (db == 0xFFFFu) kv = 0xFFFFFFFFu;
                    else kv = ((uint32_t)db << 16) | slot[b];
                    keys[(long long)(i0 + b) * kld + sg.v] = kv;
                }
            } else {
                u16x8 ps;
#pragma unroll
                for (int b = 0; b < KB_SRC; b++) ps.h[b >> 1][b & 1] = slot[b];
                st8(P + (size_t)16 * sg.p, ps);  // earlier segments hold lower slots
            }
        }
        __syncthreads();
        for (int k = tid; k < g.nhub; k += KB_BLOCK) {
            const KBHub h = g.hub[k];
            const u16x8 dv = ld8(D + (size_t)16 * h.v);
            u16x8 acc = inf8();
            for (int p = h.p0; p < h.p1; p++) acc = min8(acc, ld8(P + (size_t)16 * p));
#pragma unroll
            for (int b = 0; b < KB_SRC; b++) {
                if (sb[b] < 0) continue;
                const unsigned short db = dv.h[b >> 1][b & 1];
                uint32_t kv;
                if (h.v == sb[b]) kv = 0u;
                else if (db == 0xFFFFu) kv = 0xFFFFFFFFu;
                else kv = ((uint32_t)db << 16) | acc.h[b >> 1][b & 1];
                keys[(long long)(i0 + b) * kld + h.v] = kv;
            }
        }
        __syncthreads();
        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + 3] = __builtin_amdgcn_s_memtime();
    }
}

}  // namespace shd
