#pragma once
// "KD": SOURCE rows for mid/large integer-latency topologies (C3/C4-class, n <= 65535),
// one workgroup per source, u16 distances in LDS (2 B/vertex: 100 KB at n = 50k).
//
// Replaces igraph_get_shortest_paths_dijkstra (topology.c:1756) +
// _topology_computePathProperties (topology.c:1407-1523) for these graphs.
//
// A  Delta-stepping.  Bucket k holds pending vertices with dist in [k*D, (k+1)*D).
//    Pending vertices are a bitmask (u64 word per 64 vertices) plus, per word, a
//    conservative lower bound of the pending distances (wmin), so a sweep opens only
//    words that can hold bucket work.  Each sweep: (1) gather -- one thread per word
//    moves the pending vertices with dist < T into a dense LDS queue (no atomics:
//    nothing else runs), (2) expand -- each wave takes 64 queued vertices and walks
//    their out-arcs with a wave-level load-balanced scan, 64 arcs per step, P steps of
//    arc loads in flight; an improvement is a 32-bit CAS on the word holding two u16
//    distances (there is no 16-bit LDS atomic) followed by set-pending + wmin update.
//    On BA topologies with U[1,250] ms edges D = 16 expands each vertex ~1.03 times
//    (frontier Bellman-Ford: 5.7 times) in ~45 sweeps.
//
//    Fused parents (undirected graphs): when u is expanded, its out-arcs are its in-arcs,
//    so the same dist[v] reads find the tight in-arcs (dist[v] + w == dist[u]).  The
//    engine tie rule takes the tight arc with the largest w, then smallest (u, eid).  A
//    tight HEAVY arc (w >= D) comes from an earlier bucket, which is final when u's last
//    expansion runs, so a heavy winner seen at the last expansion is the final parent:
//    no light arc can beat it and no heavy arc can appear later.  Only vertices whose
//    winner is light (or absent) are marked for a pull fix-up over the light tail of
//    their (-w, u, eid)-sorted in-row (phase B).  Directed graphs fix up every vertex.
//
// B  lat row out (dist is exact: integer latencies, bound < 0xFFFF) + fix-ups.
// C  reliability down the tree, level-synchronous, relv f64 in a per-workgroup HBM slice
//    (8n bytes do not fit LDS at this size), parents u16 in LDS over the dead distances.
// D  rel row out, row min.
#include "common.hpp"

namespace shd {

constexpr int KD_P = 8;  // arc steps (64 arcs each) with loads in flight per wave

struct DevDelta {
    int n, nw;
    int bound;
    int delta;                          // bucket width; arcs with w >= delta are heavy
    int fused;                          // undirected: parents found during expansion
    int qcap;                           // LDS queue capacity (vertices)
    const int* __restrict__ row;        // out-CSR offsets (n+1)
    const uint32_t* __restrict__ oarc;  // out-arcs (v << 16 | w), rows sorted by (v, eid)
    const double* __restrict__ r_out;   // 1 - loss per out-arc
    const int* __restrict__ row_in;     // in-CSR offsets (n+1), rows sorted by (-w, u, eid)
    const int* __restrict__ lstart;     // first light in-arc of each row (directed: row start)
    const uint32_t* __restrict__ iarc;  // in-arcs (u << 16 | w)
    const double* __restrict__ r_in;    // 1 - loss per in-arc
    const double* __restrict__ vf;
    const double* __restrict__ self_w;
    const double* __restrict__ self_r;
    unsigned long long* dbg;            // SHD_STAMPS builds: 8 words per source
};

#ifdef SHD_STAMPS
#define KD_STAMP(slot) do { if (tid == 0 && g.dbg) g.dbg[(size_t)i * 8 + (slot)] = __builtin_amdgcn_s_memtime(); } while (0)
#define KD_COUNT(slot, x) do { if (g.dbg && lane == 0) atomicAdd(&g.dbg[(size_t)i * 8 + (slot)], (unsigned long long)(x)); } while (0)
#else
#define KD_STAMP(slot) do { } while (0)
#define KD_COUNT(slot, x) do { } while (0)
#endif

struct KDSmall {
    unsigned gmin[2];   // min pending distance seen at the start of a sweep (by parity)
    int qtail[2];       // queue length
    int qcur[2];        // next queue slice to expand
    int flag;
    int pad;
    unsigned long long rmin;
};

template <int B>
struct KDLayout {
    size_t wflag, wkey, dist, pend, wmin, fix, queue, total;
    __host__ __device__ static KDLayout make(int n, int qcap) {
        KDLayout L;
        const size_t nw = (size_t)(n + 63) / 64;
        size_t o = a16(sizeof(KDSmall));
        L.wflag = o; o += (size_t)(B / 64) * 64;
        L.wkey = o;  o += (size_t)(B / 64) * 64 * 8;
        L.dist = o;  o += a16(sizeof(uint16_t) * (size_t)(n + 1));
        L.pend = o;  o += a16(8 * nw);
        L.wmin = o;  o += a16(4 * nw);
        L.fix = o;   o += a16(8 * nw);
        L.queue = o; o += a16(sizeof(uint16_t) * (size_t)qcap);
        L.total = o;
        return L;
    }
};

// per-workgroup HBM slice: relv f64[n] | parent u16[n]
__host__ __device__ inline size_t kd_ws_stride(int n) { return a16(sizeof(double) * n) + a16(sizeof(uint16_t) * n) + 256; }

// LDS-only workgroup barrier: outstanding global stores (output rows) stay in flight.
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ inline void wait_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// lower the u16 at d[v] to nd if smaller; true if this call lowered it
__device__ inline bool kd_lower(uint16_t* d, int v, unsigned nd) {
    uint32_t* wp = reinterpret_cast<uint32_t*>(d) + (v >> 1);
    const int sh = (v & 1) * 16;
    uint32_t old = *wp;
    for (;;) {
        const unsigned cur = (old >> sh) & 0xFFFFu;
        if (nd >= cur) return false;
        const uint32_t nw = (old & ~(0xFFFFu << sh)) | (nd << sh);
        const uint32_t prev = atomicCAS(wp, old, nw);
        if (prev == old) return true;
        old = prev;
    }
}

__device__ inline unsigned kd_wave_min(unsigned x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x = min(x, (unsigned)__shfl_xor((int)x, d, 64));
    return x;
}

template <int B>
__global__ __launch_bounds__(B) void sssp_delta_kernel(DevDelta g, const int* __restrict__ src, int ns,
                                                       const int* __restrict__ tgt, int nt, long long ld,
                                                       double* __restrict__ lat_out, double* __restrict__ rel_out,
                                                       double* __restrict__ row_min, int* __restrict__ err,
                                                       char* __restrict__ ws, size_t ws_stride) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int n = g.n, nw = g.nw;
    const KDLayout<B> L = KDLayout<B>::make(n, g.qcap);
    KDSmall* sm = reinterpret_cast<KDSmall*>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned char* wflag = reinterpret_cast<unsigned char*>(smem + L.wflag) + wid * 64;
    unsigned long long* wkey = reinterpret_cast<unsigned long long*>(smem + L.wkey) + wid * 64;
    uint16_t* dist = reinterpret_cast<uint16_t*>(smem + L.dist);
    unsigned long long* pend = reinterpret_cast<unsigned long long*>(smem + L.pend);
    unsigned* wmin = reinterpret_cast<unsigned*>(smem + L.wmin);
    unsigned long long* fix = reinterpret_cast<unsigned long long*>(smem + L.fix);
    uint16_t* queue = reinterpret_cast<uint16_t*>(smem + L.queue);
    const unsigned bound = (unsigned)g.bound;
    const unsigned delta = (unsigned)g.delta;
    double* relv = reinterpret_cast<double*>(ws + (size_t)blockIdx.x * ws_stride);
    uint16_t* wpar = reinterpret_cast<uint16_t*>(ws + (size_t)blockIdx.x * ws_stride + a16(sizeof(double) * n));
    wflag[lane] = 0;

    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (s < 0 || s >= n) {
            if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL);
            continue;
        }
        KD_STAMP(0);
        const double fs = g.vf[s];
        const double cs = isnan(fs) ? 1.0 : 1.0 * fs;
        for (int v = tid; v < (n + 2) / 2; v += B) reinterpret_cast<uint32_t*>(dist)[v] = 0xFFFFFFFFu;
        for (int k = tid; k < nw; k += B) { pend[k] = 0ull; wmin[k] = 0xFFFFFFFFu; fix[k] = 0ull; }
        if (tid == 0) {
            sm->gmin[0] = sm->gmin[1] = 0xFFFFFFFFu;
            sm->qtail[0] = sm->qtail[1] = 0;
            sm->qcur[0] = sm->qcur[1] = 0;
            wpar[s] = (uint16_t)s;
            relv[s] = cs;
        }
        lds_barrier();
        if (tid == 0) {
            dist[s] = 0;
            pend[s >> 6] = 1ull << (s & 63);
            wmin[s >> 6] = 0;
        }
        lds_barrier();

        // ---- A: delta-stepping ----------------------------------------------------
        unsigned T = delta;
        int par = 0;
        for (;;) {
            KD_COUNT(5, tid == 0 ? 1 : 0);
            {
                unsigned m0 = 0xFFFFFFFFu;
                for (int k = tid; k < nw; k += B) m0 = min(m0, wmin[k]);
                const unsigned wm = kd_wave_min(m0);
                if (lane == 0 && wm != 0xFFFFFFFFu) atomicMin(&sm->gmin[par], wm);
            }
            lds_barrier();
            const unsigned m = sm->gmin[par];
            if (m == 0xFFFFFFFFu) break;
            if (m >= T) T = (m / delta + 1) * delta;
            if (tid == 0) { sm->gmin[par ^ 1] = 0xFFFFFFFFu; sm->qtail[par ^ 1] = 0; sm->qcur[par ^ 1] = 0; }
            // gather: move pending vertices with dist < T into the queue (one thread per word)
            for (int k0 = 0; k0 < nw; k0 += B) {
                const int k = k0 + tid;
                unsigned long long bits = 0ull, take = 0ull;
                unsigned rest = 0xFFFFFFFFu;
                const bool act = k < nw && wmin[k] < T;
                if (act) {
                    bits = pend[k];
                    unsigned long long b = bits;
                    while (b) {
                        const int bi = __ffsll((long long)b) - 1;
                        b &= b - 1;
                        const unsigned du = dist[(k << 6) + bi];
                        if (du < T) take |= 1ull << bi;
                        else rest = min(rest, du);
                    }
                }
                const int cnt = __popcll(take);
                int incl = cnt;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int y = __shfl_up(incl, d, 64);
                    if (lane >= d) incl += y;
                }
                int base = 0;
                if (lane == 63 && incl) base = atomicAdd(&sm->qtail[par], incl);
                base = __shfl(base, 63, 64);
                int pos = base + incl - cnt;
                if (act) {
                    unsigned long long b = take;
                    while (b) {
                        const int bi = __ffsll((long long)b) - 1;
                        b &= b - 1;
                        const int u = (k << 6) + bi;
                        if (pos < g.qcap) queue[pos] = (uint16_t)u;
                        else { take &= ~(1ull << bi); rest = min(rest, (unsigned)dist[u]); }
                        pos++;
                    }
                    pend[k] = bits & ~take;
                    wmin[k] = rest;
                }
            }
            lds_barrier();
            const int qn = min(sm->qtail[par], g.qcap);
            KD_COUNT(6, tid == 0 ? qn : 0);
            bool stored = false;
            // expand: waves take 64-vertex slices of the queue
            for (;;) {
                int sl = 0;
                if (lane == 0) sl = atomicAdd(&sm->qcur[par], 1);
                sl = __shfl(sl, 0, 64);
                const int nsl = (qn + 63) >> 6;
                if (sl >= nsl) break;
                const int j = sl + nsl * lane;  // strided: the hubs (low ids, gathered first) spread over slices
                const bool act = j < qn;
                const int u = act ? (int)queue[j] : 0;
                const unsigned du = act ? (unsigned)dist[u] : 0u;
                int beg = 0, deg = 0;
                if (act) { beg = g.row[u]; deg = g.row[u + 1] - beg; }
                int incl = deg;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int y = __shfl_up(incl, d, 64);
                    if (lane >= d) incl += y;
                }
                const int total = __shfl(incl, 63, 64);
                const int excl = incl - deg;
                const int boff = beg - excl;
                if (g.fused) wkey[lane] = ~0ull;
                const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
                for (int base0 = 0; base0 < total; base0 += 64 * KD_P) {
                    uint32_t rec[KD_P];
                    unsigned od[KD_P];
                    int oo[KD_P], aa[KD_P];
#pragma unroll
                    for (int p = 0; p < KD_P; p++) {
                        const int base = base0 + 64 * p;
                        rec[p] = 0u; od[p] = 0u; oo[p] = 0; aa[p] = -1;
                        if (base < total) {
                            // owner of arc position base+lane = last lane starting at or before it
                            const int pos = excl - base;
                            if (deg > 0 && pos >= 0 && pos < 64) wflag[pos] = (unsigned char)(lane + 1);
                            __builtin_amdgcn_wave_barrier();
                            const int fl = wflag[lane];
                            const unsigned long long M = __ballot(fl != 0);
                            wflag[lane] = 0;
                            const unsigned long long carry_m = __ballot(deg > 0 && excl < base && incl > base);
                            const unsigned long long below = M & upto;
                            const int pp = below ? 63 - __clzll((long long)below) : 0;
                            const int via = __shfl(fl, pp, 64) - 1;
                            const int o = below ? via : (carry_m ? __ffsll((long long)carry_m) - 1 : 0);
                            const int ob = __shfl(boff, o, 64);
                            od[p] = (unsigned)__shfl((int)du, o, 64);
                            oo[p] = o;
                            const int e = base + lane;
                            if (e < total) { aa[p] = ob + e; rec[p] = g.oarc[ob + e]; }
                        }
                    }
#pragma unroll
                    for (int p = 0; p < KD_P; p++) {
                        if (aa[p] < 0) continue;
                        const int v = (int)(rec[p] >> 16);
                        const unsigned w = rec[p] & 0xFFFFu;
                        const unsigned nd = od[p] + w;
                        const unsigned dv = dist[v];
                        if (nd < dv && nd <= bound && kd_lower(dist, v, nd)) {
                            atomicOr(&pend[v >> 6], 1ull << (v & 63));
                            atomicMin(&wmin[v >> 6], nd);
                        }
                        if (g.fused && dv + w == od[p])
                            atomicMin(&wkey[oo[p]], ((unsigned long long)(0xFFFFu - w) << 32) | (unsigned)aa[p]);
                    }
                }
                KD_COUNT(7, lane == 0 ? total : 0);
                __builtin_amdgcn_wave_barrier();
                if (act && u != s) {
                    bool heavy = false;
                    if (g.fused) {
                        const unsigned long long kk = wkey[lane];
                        if (kk != ~0ull && (0xFFFFu - (unsigned)(kk >> 32)) >= delta) {
                            heavy = true;
                            const int a = (int)(kk & 0xFFFFFFFFull);
                            wpar[u] = (uint16_t)(g.oarc[a] >> 16);
                            relv[u] = -g.r_out[a];
                            stored = true;
                        }
                    }
                    if (heavy) atomicAnd(&fix[u >> 6], ~(1ull << (u & 63)));
                    else atomicOr(&fix[u >> 6], 1ull << (u & 63));
                }
            }
            // a later expansion of the same vertex (next sweeps, another wave) must land after this one
            if (stored) wait_stores();
            par ^= 1;
            lds_barrier();
        }
        KD_STAMP(1);

        // ---- B: fix-ups (parents over light in-arcs) + lat row --------------------
        for (int v = tid; v < n; v += B) {
            if (v == s || !((fix[v >> 6] >> (v & 63)) & 1ull)) continue;
            const unsigned dv = dist[v];
            const int r1 = g.row_in[v + 1];
            int found = -1;
            for (int a = g.lstart[v]; a < r1; a++) {
                const uint32_t rec = g.iarc[a];
                if ((unsigned)dist[rec >> 16] + (rec & 0xFFFFu) == dv) { found = a; break; }
            }
            if (found < 0) { raise_err(err, SHD_ROUTE_EUNREACH); wpar[v] = 0xFFFFu; relv[v] = -1.0; }
            else { wpar[v] = (uint16_t)(g.iarc[found] >> 16); relv[v] = -g.r_in[found]; }
        }
        KD_STAMP(2);
        wait_stores();
        __syncthreads();
        double* lrow = lat_out ? lat_out + (long long)i * ld : nullptr;
        double* rrow = rel_out ? rel_out + (long long)i * ld : nullptr;
        double lmin = INFINITY;
        for (int j = tid; j < nt; j += B) {
            const int t = tgt[j];
            double Lv;
            if (t < 0 || t >= n) { raise_err(err, SHD_ROUTE_EINVAL); Lv = NAN; }
            else if (t == s) {
                const double sw = g.self_w[s];
                if (isnan(sw)) { raise_err(err, SHD_ROUTE_ENOEDGE); Lv = NAN; }
                else { Lv = 0.0 + sw; lmin = fmin(lmin, Lv); }
            } else if (dist[t] == 0xFFFFu) { raise_err(err, SHD_ROUTE_EUNREACH); Lv = NAN; }
            else { Lv = (double)dist[t]; lmin = fmin(lmin, Lv); }
            if (lrow) __builtin_nontemporal_store(Lv, lrow + j);
        }
        lds_barrier();
        // dist is dead: its LDS becomes the parent array
        uint16_t* parv = dist;
        for (int v = tid; v < n; v += B) parv[v] = wpar[v];
        __syncthreads();

        // ---- C: reliability down the tree (relv in the HBM slice) -----------------
        for (;;) {
            if (tid == 0) sm->flag = 0;
            __syncthreads();
            int progressed = 0;
            for (int v0 = tid; v0 < n; v0 += B * 4) {
                double x[4], rp[4];
                uint16_t p[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int v = v0 + q * B;
                    x[q] = v < n ? relv[v] : 0.0;
                    p[q] = v < n ? parv[v] : (uint16_t)0xFFFFu;
                }
#pragma unroll
                for (int q = 0; q < 4; q++)
                    rp[q] = (signbit(x[q]) && p[q] != 0xFFFFu) ? relv[p[q]] : -1.0;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (!signbit(rp[q])) { relv[v0 + q * B] = rp[q] * (-x[q]); progressed = 1; }
            }
            if (progressed) sm->flag = 1;
            __syncthreads();
            const int again = sm->flag;
            __syncthreads();
            if (!again) break;
        }
        wait_stores();  // relv must land before phase D reads it and the next source rewrites it
        KD_STAMP(3);

        // ---- D: rel row out + row min ----------------------------------------------
        if (tid == 0) sm->rmin = kInfBits;
        __syncthreads();
        if (rrow) {
            for (int j = tid; j < nt; j += B) {
                const int t = tgt[j];
                double Rv = NAN;
                if (t >= 0 && t < n) {
                    if (t == s) Rv = isnan(g.self_w[s]) ? NAN : cs * g.self_r[s];
                    else {
                        const double ft = g.vf[t];
                        Rv = isnan(ft) ? relv[t] : relv[t] * ft;
                    }
                }
                __builtin_nontemporal_store(Rv, rrow + j);
            }
        }
        if (row_min) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
            if (lane == 0 && lmin < INFINITY) atomicMin(&sm->rmin, as_u(lmin));
            __syncthreads();
            if (tid == 0) row_min[i] = as_d(sm->rmin);
        }
        lds_barrier();
        KD_STAMP(4);
    }
}

template <int B>
inline size_t kd_lds_bytes(int n, int qcap) { return KDLayout<B>::make(n, qcap).total; }

}  // namespace shd
