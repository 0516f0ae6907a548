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
constexpr int KB_RIT = 3;     // fused: segments per thread whose parent records stay in registers
constexpr int KB_WQ = 4;      // fused: targets per lane walked together
constexpr int KB_MAXD = 32;   // fused: arcs a walk collects in registers (deeper: slow path)
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
};
#ifdef SHD_STAMPS
#define KB_STAMP(slot) do { if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + (slot)] += __builtin_amdgcn_s_memtime(); } while (0)
#define KB_COUNT(slot) do { if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + (slot)] += 1; } while (0)
#else
#define KB_STAMP(slot) do { } while (0)
#define KB_COUNT(slot) do { } while (0)
#endif

// fused: once the parents are known the arc region is dead and holds the walk arrays
// par u16[KB_SRC][n] and rix u8[KB_SRC][n]; the reliability table follows P.
struct KBLayout {
    size_t arc, par, rix, D, P, rt, total;
    __host__ __device__ static KBLayout make(int n, int nnz, int npart, bool fused = false) {
        KBLayout L;
        size_t o = 0;
        L.arc = o;
        L.par = o;
        L.rix = o + a16((size_t)2 * KB_SRC * n);
        size_t arcb = a16(sizeof(uint32_t) * (size_t)nnz);
        if (fused) arcb = arcb > L.rix + a16((size_t)KB_SRC * n) ? arcb : L.rix + a16((size_t)KB_SRC * n);
        o += arcb;
        L.D = o;   o += a16((size_t)16 * n);
        L.P = o;   o += a16((size_t)16 * npart);
        L.rt = o;  o += fused ? (size_t)8 * 256 : 0;
        L.total = o;
        return L;
    }
};
constexpr size_t kKBSmall = 80;  // changed flag + fused row minima (u64 x 8)

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
// 0xFFFF when none (or when the vertex is unreached for that source)
template <bool kFused>
__device__ inline void first_tight(const uint32_t* arc, const char* D, int a0, int a1, int r0,
                                   const u16x8& dv, unsigned short (&slot)[KB_SRC]) {
#pragma unroll
    for (int b = 0; b < KB_SRC; b++) slot[b] = 0xFFFFu;
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
#pragma unroll
            for (int b = 0; b < KB_SRC; b++) {
                const unsigned short cb = c[q].h[b >> 1][b & 1], db = dv.h[b >> 1][b & 1];
                if (slot[b] == 0xFFFFu && db != 0xFFFFu && cb == db) slot[b] = (unsigned short)(a + q - r0);
            }
        }
    }
}

// fused walk record of (v, source b): parent | rix << 16
__device__ inline uint32_t kb_record(const uint32_t* arc, int v, int s, unsigned short db, int r0,
                                     unsigned short slot) {
    if (v == s) return (uint32_t)v | ((uint32_t)KB_ONE << 16);
    if (db == 0xFFFFu || slot == 0xFFFFu) return (uint32_t)(s < 0 ? v : s) | ((uint32_t)KB_NAN << 16);
    const uint32_t rec = arc[r0 + slot];
    return (rec >> 16) | (((rec >> 8) & 0xFFu) << 16);
}

// kFused = false: distances + parents -> key rows (dist16 << 16 | slot16) for K2.
// kFused = true : the whole row in one kernel.  Parent records stay in registers until the
// arcs are dead, then become par u16 / rix u8 arrays in the arc region; two waves per
// source write the lat row from D and the rel row by walking each target's tree path in
// LDS and folding the factors source-first -- the multiplication order of K2's level
// sweep (relv[v] = relv[parent] * r), so the bits agree.  Row minima as K2.
template <bool kFused>
__global__ __launch_bounds__(KB_BLOCK) void sssp_batch_kernel(DevKB g, const int* __restrict__ src, int ns,
                                                              uint32_t* __restrict__ keys, long long kld,
                                                              int* __restrict__ err,
                                                              const int* __restrict__ tgt, int nt, long long ld,
                                                              double* __restrict__ lat_out,
                                                              double* __restrict__ rel_out,
                                                              double* __restrict__ row_min) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* changed = reinterpret_cast<int*>(smem);
    unsigned long long* rmin = reinterpret_cast<unsigned long long*>(smem + 16);
    const KBLayout L = KBLayout::make(g.n, g.nnz, g.npart, kFused);
    char* base = smem + kKBSmall;
    uint32_t* arc = reinterpret_cast<uint32_t*>(base + L.arc);
    char* D = base + L.D;
    char* P = base + L.P;
    const int tid = threadIdx.x;
    const int n = g.n;

    if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + 0] = __builtin_amdgcn_s_memtime();
    double* rtl = reinterpret_cast<double*>(base + L.rt);
    if constexpr (kFused) {
        for (int k = tid; k < 256; k += KB_BLOCK)
            rtl[k] = k < g.nrtab ? g.rtab[k] : k == KB_ONE ? 1.0 : NAN;
    }
    auto stage = [&]() {  // the in-CSR into LDS (16-byte loads)
        const int nq = (g.nnz + 3) / 4;
        const uint4* s4 = reinterpret_cast<const uint4*>(g.arc);
        uint4* d4 = reinterpret_cast<uint4*>(arc);
        for (int q = tid; q < nq; q += KB_BLOCK) d4[q] = s4[q];
    };
    if constexpr (!kFused) stage();

    for (int i0 = blockIdx.x * KB_SRC; i0 < ns; i0 += gridDim.x * KB_SRC) {
        if constexpr (kFused) stage();  // the previous batch's walk arrays overwrote it
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
        if (kFused && tid < KB_SRC) rmin[tid] = kInfBits;
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
                const u16x8 acc = relax_row<kFused>(arc, D, sg.a0, sg.a1);
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
        if constexpr (!kFused) {
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
        } else {
        // ---- parents -> walk records, held in registers while the arcs are live ----
        // (host guarantees nseg <= KB_RIT * KB_BLOCK and nhub <= KB_BLOCK)
        uint32_t prec[KB_RIT][KB_SRC];
        int pv[KB_RIT];
#pragma unroll
        for (int it = 0; it < KB_RIT; it++) {
            const int k = tid + it * KB_BLOCK;
            pv[it] = -1;
            if (k >= g.nseg) continue;
            const KBSeg sg = g.seg[k];
            const u16x8 dv = ld8(D + (size_t)16 * sg.v);
            const int r0 = g.row_in[sg.v];
            unsigned short slot[KB_SRC];
            first_tight<true>(arc, D, sg.a0, sg.a1, r0, dv, slot);
            if (sg.p < 0) {
                pv[it] = sg.v;
#pragma unroll
                for (int b = 0; b < KB_SRC; b++)
                    prec[it][b] = kb_record(arc, sg.v, sb[b], dv.h[b >> 1][b & 1], r0, slot[b]);
            } else {
                u16x8 ps;
#pragma unroll
                for (int b = 0; b < KB_SRC; b++) ps.h[b >> 1][b & 1] = slot[b];
                st8(P + (size_t)16 * sg.p, ps);  // earlier segments hold lower slots
            }
        }
        __syncthreads();
        uint32_t hrec[KB_SRC];
        int hv = -1;
        if (tid < g.nhub) {
            const KBHub h = g.hub[tid];
            hv = h.v;
            const u16x8 dv = ld8(D + (size_t)16 * h.v);
            const int r0 = g.row_in[h.v];
            u16x8 acc = inf8();
            for (int p = h.p0; p < h.p1; p++) acc = min8(acc, ld8(P + (size_t)16 * p));
#pragma unroll
            for (int b = 0; b < KB_SRC; b++)
                hrec[b] = kb_record(arc, h.v, sb[b], dv.h[b >> 1][b & 1], r0, acc.h[b >> 1][b & 1]);
        }
        __syncthreads();  // every arc read done: the region becomes par / rix
        uint16_t* par = reinterpret_cast<uint16_t*>(base + L.par);
        uint8_t* rix = reinterpret_cast<uint8_t*>(base + L.rix);
#pragma unroll
        for (int it = 0; it < KB_RIT; it++) {
            if (pv[it] < 0) continue;
#pragma unroll
            for (int b = 0; b < KB_SRC; b++) {
                par[b * n + pv[it]] = (uint16_t)(prec[it][b] & 0xFFFFu);
                rix[b * n + pv[it]] = (uint8_t)(prec[it][b] >> 16);
            }
        }
        if (hv >= 0) {
#pragma unroll
            for (int b = 0; b < KB_SRC; b++) {
                par[b * n + hv] = (uint16_t)(hrec[b] & 0xFFFFu);
                rix[b * n + hv] = (uint8_t)(hrec[b] >> 16);
            }
        }
        __syncthreads();
        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + 5] = __builtin_amdgcn_s_memtime();

        // ---- rows: KB_BLOCK / 64 / KB_SRC waves per source ----------------------
        constexpr int WPS = KB_BLOCK / 64 / KB_SRC;
        const int wv = tid >> 6, lane = tid & 63;
        const int b = wv % KB_SRC;
        const int i = i0 + b;
        int s = -1;
        if (i < ns) {
            s = src[i];
            if (s < 0 || s >= n) s = -1;
        }
        if (s >= 0) {
            const double fs = g.vf[s];
            const double cs = isnan(fs) ? 1.0 : 1.0 * fs;
            const uint16_t* pb = par + b * n;
            const uint8_t* xb = rix + b * n;
            double* lrow = lat_out ? lat_out + (long long)i * ld : nullptr;
            double* rrow = rel_out ? rel_out + (long long)i * ld : nullptr;
            double lmin = INFINITY;
            constexpr int STEP = WPS * 64;
            for (int j0 = (wv / KB_SRC) * 64 + lane; j0 - lane < nt; j0 += STEP * KB_WQ) {
                int tq[KB_WQ], cur[KB_WQ];
                uint32_t pk[KB_WQ][KB_MAXD / 4];
#pragma unroll
                for (int q = 0; q < KB_WQ; q++) {
                    const int j = j0 + q * STEP;
                    tq[q] = j < nt ? tgt[j] : -1;
                    cur[q] = tq[q] >= 0 && tq[q] < n ? tq[q] : s;
#pragma unroll
                    for (int k = 0; k < KB_MAXD / 4; k++) pk[q][k] = 0u;
                }
                // walk: a chain that reaches the source stays there (par[s] = s, factor 1.0)
                int kmax = 0;  // wave-uniform
#pragma unroll
                for (int k = 0; k < KB_MAXD; k++) {
                    bool any = false;
#pragma unroll
                    for (int q = 0; q < KB_WQ; q++) any = any || cur[q] != s;
                    if (!__any(any)) break;
                    kmax = k + 1;
                    uint32_t p[KB_WQ], rx[KB_WQ];
#pragma unroll
                    for (int q = 0; q < KB_WQ; q++) { p[q] = pb[cur[q]]; rx[q] = xb[cur[q]]; }
#pragma unroll
                    for (int q = 0; q < KB_WQ; q++) {
                        pk[q][k >> 2] |= rx[q] << ((k & 3) * 8);
                        cur[q] = (int)p[q];
                    }
                }
                double rr[KB_WQ];
#pragma unroll
                for (int q = 0; q < KB_WQ; q++) rr[q] = cs;
#pragma unroll
                for (int k = KB_MAXD - 1; k >= 0; k--) {
                    if (k >= kmax) continue;
                    double x[KB_WQ];
#pragma unroll
                    for (int q = 0; q < KB_WQ; q++) x[q] = rtl[(pk[q][k >> 2] >> ((k & 3) * 8)) & 0xFFu];
#pragma unroll
                    for (int q = 0; q < KB_WQ; q++) rr[q] *= x[q];
                }
#pragma unroll
                for (int q = 0; q < KB_WQ; q++) {
                    if (cur[q] == s) continue;
                    // deeper than KB_MAXD arcs (rare): fold depth by depth, re-walking from t
                    const int t = tq[q];
                    int depth = 0;
                    for (int c = t; c != s && depth <= n; c = pb[c]) depth++;
                    double r = cs;
                    for (int d = 1; d <= depth && d <= n; d++) {
                        int c = t;
                        for (int k = 0; k < depth - d; k++) c = pb[c];
                        r *= rtl[xb[c]];
                    }
                    rr[q] = r;
                }
                double ft[KB_WQ];
#pragma unroll
                for (int q = 0; q < KB_WQ; q++) ft[q] = g.vf[tq[q] >= 0 && tq[q] < n ? tq[q] : s];
#pragma unroll
                for (int q = 0; q < KB_WQ; q++) {
                    const int j = j0 + q * STEP;
                    if (j >= nt) continue;
                    const int t = tq[q];
                    double Lv, Rv;
                    if (t < 0 || t >= n) {
                        raise_err(err, SHD_ROUTE_EINVAL);
                        Lv = Rv = NAN;
                    } else if (t == s) {  // batch path [s]: one self-loop hop (topology.c:1471-1499)
                        const double w = g.self_w[s];
                        if (isnan(w)) { raise_err(err, SHD_ROUTE_ENOEDGE); Lv = Rv = NAN; }
                        else { Lv = 0.0 + w; Rv = cs * g.self_r[s]; }
                    } else {
                        const unsigned short dt = *reinterpret_cast<const unsigned short*>(D + (size_t)16 * t + 2 * b);
                        if (dt == 0xFFFFu) {
                            raise_err(err, SHD_ROUTE_EUNREACH);
                            Lv = Rv = NAN;
                        } else {
                            Lv = (double)dt;
                            Rv = isnan(ft[q]) ? rr[q] : rr[q] * ft[q];
                        }
                    }
                    if (lrow) __builtin_nontemporal_store(Lv, lrow + j);
                    if (rrow) __builtin_nontemporal_store(Rv, rrow + j);
                    lmin = fmin(lmin, Lv);
                }
            }
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
            if (lane == 0 && lmin < INFINITY) atomicMin(&rmin[b], as_u(lmin));
        }
        __syncthreads();
        if (tid < KB_SRC && i0 + tid < ns && row_min) row_min[i0 + tid] = as_d(rmin[tid]);
        }  // kFused
        if (tid == 0 && g.dbg) g.dbg[(size_t)blockIdx.x * 8 + 3] = __builtin_amdgcn_s_memtime();
    }
}

}  // namespace shd
