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
constexpr int KB_RIT = 3;     // fused: segments per thread, held in registers
constexpr int KB_CV = 16;     // fused: walk records per thread (KB_SRC * n <= KB_CV * KB_BLOCK)
constexpr int KB_WQ = 4;      // fused: targets per lane walked together
constexpr int KB_MAXD = 32;   // fused: arcs a walk collects in registers (deeper: chunked refolds)
constexpr int KB_ONE = 254;   // fused: rtab slot holding 1.0 (the source's own step)
constexpr int KB_NAN = 255;   // fused: rtab slot holding NaN (unreachable vertices)

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
    // fused path attributes (sssp_batch_kernel<true>): arc = u << 16 | ridx << 8 | w
    const double* __restrict__ rtab;    // distinct 1 - loss values (<= 254), indexed by ridx
    int nrtab;
    const double* __restrict__ vf;
    const double* __restrict__ self_w;
    const double* __restrict__ self_r;
    int tcap;                           // staged targets per chunk
};
#ifdef SHD_STAMPS
#define KB_STAMP(slot) do { if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + (slot)] += __builtin_amdgcn_s_memtime(); } while (0)
#define KB_COUNT(slot) do { if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + (slot)] += 1; } while (0)
// fused rows phase, wave 0 of each workgroup: cycles of walk / fold / output, trips, steps
#define KBT_MARK(v) unsigned long long v = 0; if (g.dbg) v = __builtin_amdgcn_s_memtime()
#define KBT_ACC(slot, val) do { if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 16 + (slot)] += (val); } while (0)
#else
#define KBT_MARK(v) do { } while (0)
#define KBT_ACC(slot, val) do { } while (0)
#define KB_STAMP(slot) do { } while (0)
#define KB_COUNT(slot) do { } while (0)
#endif

// fused: parent slots sl u16[KB_SRC][n] (absolute index of each vertex's first tight
// in-arc, 0xFFFF at the source and at unreached vertices), the reliability table, and the
// staged target list tg i32[tcap]; once the parents are known the arc region holds the
// walk records wrec u32[KB_SRC][n] = parent | rix << 16.
struct KBLayout {
    size_t arc, D, P, sl, rt, tg, total;
    __host__ __device__ static KBLayout make(int n, int nnz, int npart, bool fused = false, int tcap = 0) {
        KBLayout L;
        size_t o = 0;
        size_t arcb = a16(sizeof(uint32_t) * (size_t)nnz);
        if (fused && arcb < a16((size_t)4 * KB_SRC * n)) arcb = a16((size_t)4 * KB_SRC * n);  // walk records
        L.arc = o; o += arcb;
        L.D = o;   o += a16((size_t)16 * n);
        L.P = o;   o += a16((size_t)16 * npart);
        L.sl = o;  o += fused ? a16((size_t)2 * KB_SRC * n) : 0;
        L.rt = o;  o += fused ? (size_t)8 * 256 : 0;
        L.tg = o;  o += fused ? a16((size_t)4 * tcap) : 0;
        L.total = o;
        return L;
    }
};
// small: changed flag, fused unit counter | row minima u64[8] | per-source constants of the
// fused rows phase: source, 1.0 * f_s (or 1.0), self-loop latency and reliability
struct KBSmall {
    int changed, flag1, flag2, units;  // KBF sweeps: changed/flag1/flag2 rotate
    unsigned long long rmin[8];
    int src[8];
    double cs[8], sw[8], sr[8];
};
constexpr size_t kKBSmall = (sizeof(KBSmall) + 15) & ~size_t(15);

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

// min over hub partials [p0, p1): four independent LDS reads in flight (a hub row of
// 11 segments was 11 dependent round trips at the end of every sweep)
__device__ inline u16x8 min_parts(const char* P, int p0, int p1, u16x8 acc) {
    int p = p0;
    for (; p + 4 <= p1; p += 4) {
        const u16x8 x0 = ld8(P + (size_t)16 * p), x1 = ld8(P + (size_t)16 * (p + 1));
        const u16x8 x2 = ld8(P + (size_t)16 * (p + 2)), x3 = ld8(P + (size_t)16 * (p + 3));
        acc = min8(acc, min8(min8(x0, x1), min8(x2, x3)));
    }
    for (; p < p1; p++) acc = min8(acc, ld8(P + (size_t)16 * p));
    return acc;
}

// arc weight as a u16 pair: low 16 bits (u << 16 | w), or the low byte of the fused
// record (u << 16 | ridx << 8 | w)
template <bool kFused>
__device__ inline us2 wsplat(uint32_t rec) {
    const unsigned short w = (unsigned short)(rec & (kFused ? 0xFFu : 0xFFFFu));
    const us2 r = {w, w};
    return r;
}

// min over arcs [a0, a1) of D[u] + w, four independent arc/distance reads in flight.
template <bool kFused>
__device__ inline u16x8 relax_row(const uint32_t* arc, const char* D, int a0, int a1) {
    u16x8 acc = inf8();
    int a = a0;
    for (; a + 4 <= a1; a += 4) {
        const uint32_t r0 = arc[a], r1 = arc[a + 1], r2 = arc[a + 2], r3 = arc[a + 3];
        const u16x8 d0 = ld8(D + (size_t)16 * (r0 >> 16));
        const u16x8 d1 = ld8(D + (size_t)16 * (r1 >> 16));
        const u16x8 d2 = ld8(D + (size_t)16 * (r2 >> 16));
        const u16x8 d3 = ld8(D + (size_t)16 * (r3 >> 16));
        acc = min8(min8(acc, addsat8(d0, wsplat<kFused>(r0))), addsat8(d1, wsplat<kFused>(r1)));
        acc = min8(min8(acc, addsat8(d2, wsplat<kFused>(r2))), addsat8(d3, wsplat<kFused>(r3)));
    }
    for (; a < a1; a++) {
        const uint32_t r0 = arc[a];
        acc = min8(acc, addsat8(ld8(D + (size_t)16 * (r0 >> 16)), wsplat<kFused>(r0)));
    }
    return acc;
}

// first tight arc of in-arcs [a0, a1) for each of the batch's sources: slot (a - r0) or
// 0xFFFF when none (or when the vertex is unreached for that source).  Packed: per arc
// and u16 pair, x = c ^ dv is 0 where tight; min(x, 1) * 0xFFFF is 0 there and 0xFFFF
// elsewhere; max with the arc's slot and a running min keep the first tight slot (arcs
// ascend) -- 5 packed ops per pair instead of 8 scalar compare/selects per arc.
template <bool kFused>
__device__ inline void first_tight(const uint32_t* arc, const char* D, int a0, int a1, int r0,
                                   const u16x8& dv, unsigned short (&slot)[KB_SRC]) {
    u16x8 sl = inf8();
    const us2 one = {1, 1}, ffff = {0xFFFF, 0xFFFF};
    for (int a = a0; a < a1; a += 4) {
        u16x8 c[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t rec = arc[min(a + q, a1 - 1)];
            c[q] = addsat8(ld8(D + (size_t)16 * (rec >> 16)), wsplat<kFused>(rec));
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (a + q >= a1) break;
            const unsigned short idx = (unsigned short)(a + q - r0);
            const us2 iv = {idx, idx};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const us2 x = __builtin_bit_cast(
                    us2, __builtin_bit_cast(uint32_t, c[q].h[k]) ^ __builtin_bit_cast(uint32_t, dv.h[k]));
                const us2 cand = __builtin_elementwise_max(__builtin_elementwise_min(x, one) * ffff, iv);
                sl.h[k] = __builtin_elementwise_min(sl.h[k], cand);
            }
        }
    }
#pragma unroll
    for (int b = 0; b < KB_SRC; b++) {
        const unsigned short db = dv.h[b >> 1][b & 1];
        slot[b] = db == 0xFFFFu ? (unsigned short)0xFFFFu : sl.h[b >> 1][b & 1];
    }
}

// Distances + parents -> key rows (dist16 << 16 | slot16) for K2 (path_attr.hpp).
__global__ __launch_bounds__(KB_BLOCK) void sssp_batch_kernel(DevKB g, const int* __restrict__ src, int ns,
                                                              uint32_t* __restrict__ keys, long long kld,
                                                              int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* flags = reinterpret_cast<int*>(smem);  // three rotating sweep flags (see KBF)
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
        if (tid == 0) flags[0] = 0;
        __syncthreads();

        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + 1] = __builtin_amdgcn_s_memtime();
        // ---- Gauss-Seidel pull sweeps to the fixed point -------------------------
        for (int fi = 0;; fi = fi == 2 ? 0 : fi + 1) {
            KB_COUNT(4);
            if (tid == 0) flags[fi == 2 ? 0 : fi + 1] = 0;
            int* changed = flags + fi;
            int ch = 0;
            for (int k = tid; k < g.nseg; k += KB_BLOCK) {
                const KBSeg sg = g.seg[k];
                const u16x8 acc = relax_row<false>(arc, D, sg.a0, sg.a1);
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
                acc = min_parts(P, h.p0, h.p1, acc);
                if (!eq8(acc, old)) { st8(D + (size_t)16 * h.v, acc); ch = 1; }
            }
            if (ch) *changed = 1;
            __syncthreads();
            if (!*changed) break;
        }

        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + 2] = __builtin_amdgcn_s_memtime();
        // ---- parents: first tight arc of each in-row, per source -----------------
        for (int k = tid; k < g.nseg; k += KB_BLOCK) {
            const KBSeg sg = g.seg[k];
            const u16x8 dv = ld8(D + (size_t)16 * sg.v);
            const int r0 = g.row_in[sg.v];
            unsigned short slot[KB_SRC];
            first_tight<false>(arc, D, sg.a0, sg.a1, r0, dv, slot);
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
            acc = min_parts(P, h.p0, h.p1, acc);
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


// KB with fused path attributes: the whole SOURCE rows of KB_SRC sources in one kernel
// (no key rows, no K2).
//  - each thread's <= KB_RIT segments and <= 1 hub stay in registers for the whole launch
//    (packed, no per-sweep descriptor loads)
//  - the parent pass stores, per (source, vertex), the absolute index of the first tight
//    in-arc (nnz < 2^16 whenever the arcs fit the LDS), so no in-row offsets are read
//  - the target list is staged in LDS once, before the sweeps, when it fits (else chunked)
//  - slots become walk records (parent | rix << 16) over the dead arc region; units of
//    (source, 256 targets) from a workgroup queue write the lat row from D and the rel row
//    by walking each target's tree path in LDS (one ds_read_b32 per arc) and folding the
//    factors source-first: the multiplication order of K2's level sweep
//    (relv[v] = relv[parent] * r), so the bits agree.  Row minima as K2.
__global__ __launch_bounds__(KB_BLOCK) void sssp_batch_rows_kernel(DevKB g, const int* __restrict__ src, int ns,
                                                                   int* __restrict__ err,
                                                                   const int* __restrict__ tgt, int nt, long long ld,
                                                                   double* __restrict__ lat_out,
                                                                   double* __restrict__ rel_out,
                                                                   double* __restrict__ row_min) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    KBSmall* sm = reinterpret_cast<KBSmall*>(smem);
    // three sweep flags in rotation: a sweep resets the next one's flag before its first
    // barrier, when every thread has read the flag of two sweeps ago (2 barriers a sweep)
    int* flags = &sm->changed;  // changed, flag1, flag2
    unsigned long long* rmin = sm->rmin;
    const KBLayout L = KBLayout::make(g.n, g.nnz, g.npart, true, g.tcap);
    char* base = smem + kKBSmall;
    uint32_t* arc = reinterpret_cast<uint32_t*>(base + L.arc);
    char* D = base + L.D;
    char* P = base + L.P;
    uint16_t* sl = reinterpret_cast<uint16_t*>(base + L.sl);
    double* rtl = reinterpret_cast<double*>(base + L.rt);
    int* tg = reinterpret_cast<int*>(base + L.tg);
    const int tid = threadIdx.x;
    const int n = g.n;
    const int tcap = g.tcap;

    if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 16 + 0] = __builtin_amdgcn_s_memtime();
    for (int k = tid; k < 256; k += KB_BLOCK)
        rtl[k] = k < g.nrtab ? g.rtab[k] : k == KB_ONE ? 1.0 : NAN;
    const bool one_chunk = nt <= tcap;
    if (one_chunk)
        for (int j = tid; j < nt; j += KB_BLOCK) tg[j] = tgt[j];
    for (int i0 = blockIdx.x * KB_SRC; i0 < ns; i0 += gridDim.x * KB_SRC) {
        {   // the in-CSR into LDS (16-byte loads); the previous batch's walk records overwrote it
            const int nq = (g.nnz + 3) / 4;
            const uint4* s4 = reinterpret_cast<const uint4*>(g.arc);
            uint4* d4 = reinterpret_cast<uint4*>(arc);
            for (int q = tid; q < nq; q += KB_BLOCK) d4[q] = s4[q];
        }
        // this thread's segments (reloaded per batch: nothing lives across the walk)
        // (a0 | len << 16, v | p << 16; p = 0xFFFF: whole row) and hub
        // (host guarantees nseg <= KB_RIT * KB_BLOCK, nhub <= KB_BLOCK, n and npart < 2^16)
        uint32_t sa[KB_RIT], sv[KB_RIT];
#pragma unroll
        for (int it = 0; it < KB_RIT; it++) {
            const int k = tid + it * KB_BLOCK;
            sa[it] = 0u; sv[it] = 0xFFFFFFFFu;
            if (k < g.nseg) {
                const KBSeg sg = g.seg[k];
                sa[it] = (uint32_t)sg.a0 | ((uint32_t)(sg.a1 - sg.a0) << 16);
                sv[it] = (uint32_t)sg.v | ((uint32_t)(sg.p < 0 ? 0xFFFF : sg.p) << 16);
            }
        }
        int hv = -1;
        uint32_t hp = 0u;
        if (tid < g.nhub) {
            const KBHub h = g.hub[tid];
            hv = h.v;
            hp = (uint32_t)h.p0 | ((uint32_t)h.p1 << 16);
        }
        int sb[KB_SRC];
#pragma unroll
        for (int b = 0; b < KB_SRC; b++) {
            const int i = i0 + b;
            int s = -1;
            if (i < ns) {
                s = src[i];
                if (s < 0 || s >= n) { if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL); s = -1; }
            }
            sb[b] = s;
        }
        for (int v = tid; v < n; v += KB_BLOCK) {
            u16x8 d = inf8();
#pragma unroll
            for (int b = 0; b < KB_SRC; b++)
                if (sb[b] == v) d.h[b >> 1][b & 1] = 0;
            st8(D + (size_t)16 * v, d);
        }
        if (tid < KB_SRC) {  // rows-phase constants (their loads overlap the sweeps)
            rmin[tid] = kInfBits;
            const int s = sb[tid];
            sm->src[tid] = s;
            const double fs = s >= 0 ? g.vf[s] : NAN;
            sm->cs[tid] = isnan(fs) ? 1.0 : 1.0 * fs;
            sm->sw[tid] = s >= 0 ? g.self_w[s] : NAN;
            sm->sr[tid] = s >= 0 ? g.self_r[s] : NAN;
        }
        if (tid == 0) { sm->units = 0; sm->changed = 0; }
        __syncthreads();

        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 16 + 1] = __builtin_amdgcn_s_memtime();
        // ---- Gauss-Seidel pull sweeps to the fixed point -------------------------
        for (int fi = 0;; fi = fi == 2 ? 0 : fi + 1) {
            if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 16 + 4] += 1;
            if (tid == 0) flags[fi == 2 ? 0 : fi + 1] = 0;
            int* changed = flags + fi;
            int ch = 0;
#pragma unroll
            for (int it = 0; it < KB_RIT; it++) {
                if (sv[it] == 0xFFFFFFFFu) continue;
                const int a0 = (int)(sa[it] & 0xFFFFu), a1 = a0 + (int)(sa[it] >> 16);
                const int v = (int)(sv[it] & 0xFFFFu), p = (int)(sv[it] >> 16);
                const u16x8 acc = relax_row<true>(arc, D, a0, a1);
                if (p == 0xFFFF) {
                    const u16x8 old = ld8(D + (size_t)16 * v);
                    const u16x8 nw = min8(old, acc);
                    if (!eq8(nw, old)) { st8(D + (size_t)16 * v, nw); ch = 1; }
                } else {
                    st8(P + (size_t)16 * p, acc);
                }
            }
            __syncthreads();
            if (hv >= 0) {
                u16x8 acc = ld8(D + (size_t)16 * hv);
                const u16x8 old = acc;
                acc = min_parts(P, (int)(hp & 0xFFFFu), (int)(hp >> 16), acc);
                if (!eq8(acc, old)) { st8(D + (size_t)16 * hv, acc); ch = 1; }
            }
            if (ch) *changed = 1;
            __syncthreads();
            if (!*changed) break;
        }

        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 16 + 2] = __builtin_amdgcn_s_memtime();
        // ---- parents: absolute index of the first tight in-arc, per source --------
#pragma unroll
        for (int it = 0; it < KB_RIT; it++) {
            if (sv[it] == 0xFFFFFFFFu) continue;
            const int a0 = (int)(sa[it] & 0xFFFFu), a1 = a0 + (int)(sa[it] >> 16);
            const int v = (int)(sv[it] & 0xFFFFu), p = (int)(sv[it] >> 16);
            const u16x8 dv = ld8(D + (size_t)16 * v);
            unsigned short slot[KB_SRC];
            first_tight<true>(arc, D, a0, a1, 0, dv, slot);  // 0xFFFF at the source / unreached
            if (p == 0xFFFF) {
#pragma unroll
                for (int b = 0; b < KB_SRC; b++) sl[b * n + v] = slot[b];
            } else {
                u16x8 ps;
#pragma unroll
                for (int b = 0; b < KB_SRC; b++) ps.h[b >> 1][b & 1] = slot[b];
                st8(P + (size_t)16 * p, ps);  // earlier segments hold lower arc indices
            }
        }
        __syncthreads();
        if (hv >= 0) {
            u16x8 acc = inf8();
            acc = min_parts(P, (int)(hp & 0xFFFFu), (int)(hp >> 16), acc);
#pragma unroll
            for (int b = 0; b < KB_SRC; b++) sl[b * n + hv] = acc.h[b >> 1][b & 1];
        }
        __syncthreads();
        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 16 + 5] = __builtin_amdgcn_s_memtime();

        // ---- slots -> walk records wrec u32[KB_SRC][n] = parent | rix << 16 over the dead
        // arc region (the source and unreached vertices point at themselves, factor 1.0);
        // held in registers across the barrier after which no arc is read
        {
            uint32_t cv[KB_CV];
#pragma unroll
            for (int k = 0; k < KB_CV; k++) {
                const int x = tid + k * KB_BLOCK;
                cv[k] = 0u;
                if (x < KB_SRC * n) {
                    const uint32_t a = sl[x];
                    const uint32_t rec = arc[a == 0xFFFFu ? 0u : a];
                    cv[k] = a == 0xFFFFu ? ((uint32_t)(x % n) | ((uint32_t)KB_ONE << 16))
                                         : ((rec >> 16) | (((rec >> 8) & 0xFFu) << 16));
                }
            }
            __syncthreads();  // every arc read done
#pragma unroll
            for (int k = 0; k < KB_CV; k++) {
                const int x = tid + k * KB_BLOCK;
                if (x < KB_SRC * n) arc[x] = cv[k];
            }
            __syncthreads();
        }
        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 16 + 6] = __builtin_amdgcn_s_memtime();

        // ---- rows: a work queue of (source, KB_WQ * 64 targets) units over all waves, so
        // a source with a deep tree does not hold up the workgroup -------------------------
        const int lane = tid & 63;
        constexpr int UT = KB_WQ * 64;  // targets per unit
        for (int c0 = 0; c0 < nt; c0 += tcap) {
            const int cn = min(tcap, nt - c0);
            if (!one_chunk) {
                __syncthreads();  // the previous chunk's units are done
                for (int j = tid; j < cn; j += KB_BLOCK) tg[j] = tgt[c0 + j];
                if (tid == 0) sm->units = 0;
                __syncthreads();
            }
            const int nch = (cn + UT - 1) / UT;
            for (;;) {
                int u = 0;
                if (lane == 0) u = atomicAdd(&sm->units, 1);
                u = __builtin_amdgcn_readfirstlane(__shfl(u, 0, 64));
                if (u >= KB_SRC * nch) break;
                const int b = u % KB_SRC, j0 = (u / KB_SRC) * UT + lane;
                const int s = sm->src[b];
                if (s < 0) continue;
                constexpr int STEP = 64;
                const double cs = sm->cs[b], s_w = sm->sw[b], s_r = sm->sr[b];
                const uint32_t* wb = arc + b * n;  // walk records of source b
                double* lrow = lat_out ? lat_out + (long long)(i0 + b) * ld : nullptr;
                double* rrow = rel_out ? rel_out + (long long)(i0 + b) * ld : nullptr;
                double lmin = INFINITY;
                int tq[KB_WQ], cur[KB_WQ];
                double ft[KB_WQ];
                uint32_t pk[KB_WQ][KB_MAXD / 4];  // rix of the arcs walked, 4 per word
#pragma unroll
                for (int q = 0; q < KB_WQ; q++) {
                    const int j = j0 + q * STEP;
                    tq[q] = j < cn ? tg[j] : -1;
                    const bool ok = tq[q] >= 0 && tq[q] < n;
                    ft[q] = g.vf[ok ? tq[q] : s];  // in flight during the walk
                    cur[q] = ok && *reinterpret_cast<const unsigned short*>(D + (size_t)16 * tq[q] + 2 * b) != 0xFFFFu
                                 ? tq[q] : s;
#pragma unroll
                    for (int k = 0; k < KB_MAXD / 4; k++) pk[q][k] = 0u;
                }
                KBT_MARK(t_a);
                // walk in blocks of 4 arcs (a chain that reaches the source stays there: parent
                // s, factor exactly 1.0, so the block padding is harmless); one packed word of
                // reliability indices per chain and block
                int nb = 0;  // blocks walked, wave-uniform
#pragma unroll 1
                for (; nb < KB_MAXD / 4; nb++) {
                    bool any = false;
#pragma unroll
                    for (int q = 0; q < KB_WQ; q++) any = any || cur[q] != s;
                    if (!__any(any)) break;
                    uint32_t acc[KB_WQ];
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        uint32_t pr[KB_WQ];
#pragma unroll
                        for (int q = 0; q < KB_WQ; q++) pr[q] = wb[cur[q]];
#pragma unroll
                        for (int q = 0; q < KB_WQ; q++) {
                            acc[q] = e == 0 ? (pr[q] >> 16) : (acc[q] | ((pr[q] >> 16) << (8 * e)));
                            cur[q] = (int)(pr[q] & 0xFFFFu);
                        }
                    }
#pragma unroll
                    for (int q = 0; q < KB_WQ; q++) pk[q][nb] = acc[q];
                }
                KBT_MARK(t_b);
                [[maybe_unused]] const int kmax = 4 * nb;  // stamps only
                // fold source-first: the last arc walked is the first factor.  The fold starts
                // from (1.0 * f_s) * f_t, the reference's order (topology.c:1443-1462 multiplies
                // both vertex factors before the first arc, :1499), so vertex loss is bit-exact
                double c0t[KB_WQ], rr[KB_WQ];
#pragma unroll
                for (int q = 0; q < KB_WQ; q++) {
                    c0t[q] = isnan(ft[q]) ? cs : cs * ft[q];
                    rr[q] = c0t[q];
                }
#pragma unroll 1
                for (int k4 = nb - 1; k4 >= 0; k4--) {
                    uint32_t wq[KB_WQ];
#pragma unroll
                    for (int q = 0; q < KB_WQ; q++) wq[q] = pk[q][k4];
#pragma unroll
                    for (int e = 3; e >= 0; e--) {
                        double x[KB_WQ];
#pragma unroll
                        for (int q = 0; q < KB_WQ; q++) x[q] = rtl[(wq[q] >> (8 * e)) & 0xFFu];
#pragma unroll
                        for (int q = 0; q < KB_WQ; q++) rr[q] *= x[q];
                    }
                }
#pragma unroll
                for (int q = 0; q < KB_WQ; q++) {
                    if (cur[q] == s) continue;
                    // deeper than KB_MAXD arcs: depth L, then chunks of KB_MAXD factors from the
                    // source side, each collected by re-walking from t (O(L^2 / KB_MAXD) steps)
                    const int t = tq[q];
                    int depth = 0;
                    for (int c = t; c != s && depth <= n; c = (int)(wb[c] & 0xFFFFu)) depth++;
                    double r = c0t[q];
                    for (int lo = 1; lo <= depth && lo <= n; lo += 16) {
                        const int hi = min(depth, lo + 15);
                        int c = t;
                        for (int k = 0; k < depth - hi; k++) c = (int)(wb[c] & 0xFFFFu);
                        unsigned long long f0 = 0ull, f1 = 0ull;  // factors of depths hi .. lo
                        for (int k = 0; k <= hi - lo; k++) {
                            const unsigned long long x = wb[c] >> 16;
                            if (k < 8) f0 |= x << (8 * k);
                            else f1 |= x << (8 * (k - 8));
                            c = (int)(wb[c] & 0xFFFFu);
                        }
                        for (int k = hi - lo; k >= 0; k--)
                            r *= rtl[(k < 8 ? f0 >> (8 * k) : f1 >> (8 * (k - 8))) & 0xFFu];
                    }
                    rr[q] = r;
                }
                KBT_MARK(t_c);
#pragma unroll
                for (int q = 0; q < KB_WQ; q++) {
                    const int j = j0 + q * STEP;
                    if (j >= cn) continue;
                    const int t = tq[q];
                    double Lv, Rv;
                    if (t < 0 || t >= n) {
                        raise_err(err, SHD_ROUTE_EINVAL);
                        Lv = Rv = NAN;
                    } else if (t == s) {  // batch path [s]: one self-loop hop (topology.c:1471-1499)
                        if (isnan(s_w)) { raise_err(err, SHD_ROUTE_ENOEDGE); Lv = Rv = NAN; }
                        else { Lv = 0.0 + s_w; Rv = cs * s_r; }
                    } else {
                        const unsigned short dt = *reinterpret_cast<const unsigned short*>(D + (size_t)16 * t + 2 * b);
                        if (dt == 0xFFFFu) {
                            raise_err(err, SHD_ROUTE_EUNREACH);
                            Lv = Rv = NAN;
                        } else {
                            Lv = (double)dt;
                            Rv = rr[q];
                        }
                    }
                    if (lrow) __builtin_nontemporal_store(Lv, lrow + c0 + j);
                    if (rrow) __builtin_nontemporal_store(Rv, rrow + c0 + j);
                    lmin = fmin(lmin, Lv);
                }
                KBT_MARK(t_d);
                KBT_ACC(8, t_b - t_a); KBT_ACC(9, t_c - t_b); KBT_ACC(10, t_d - t_c); KBT_ACC(11, 1); KBT_ACC(12, kmax);
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
                if (lane == 0 && lmin < INFINITY) atomicMin(&rmin[b], as_u(lmin));
            }
        }
        __syncthreads();
        if (tid < KB_SRC && i0 + tid < ns && row_min) row_min[i0 + tid] = as_d(rmin[tid]);
        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 16 + 3] = __builtin_amdgcn_s_memtime();
    }
}

}  // namespace shd
