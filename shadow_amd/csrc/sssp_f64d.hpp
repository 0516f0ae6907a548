#pragma once
// "KF": SOURCE rows for fractional-latency topologies (any positive double latencies) whose
// per-source state fits LDS (n up to ~12k at 1024 threads, ~3k at four 256-thread workgroups
// per CU).  One workgroup per source.  "KFH" (H = true): the same kernel for n up to 65535
// (C4f: 50k) with the per-vertex state -- f64 distances / relv, u16 parents, u8 reliability
// indices, 11 B per vertex -- in a per-workgroup HBM slice (most of it lives in L2 / MALL),
// while the bucket ring, the pending / queued bitmasks and their word minima stay in LDS
// (2.4 B per vertex), so the rounds' queue work is still LDS work.
//
// Replaces igraph_get_shortest_paths_dijkstra (topology.c:1756) +
// _topology_computePathProperties (topology.c:1407-1523) where the integer kernels (KBF, KD,
// K32) do not apply: latencies like the reference's own 2293.85 ms (resource/topology.graphml).
//
// A  Delta-stepping on f64 distances held as IEEE bits (non-negative doubles order like u64)
//    in LDS: a bucket round gathers the pending vertices below the bucket bound T into an LDS
//    queue, expands their out-arcs load-balanced over the workgroup (block scan of degrees,
//    owner by binary search), relaxes with ds_min_u64 and marks improved vertices pending.
//    fl(d[u] + w) is monotone in d[u], so any relaxation order reaches the same left-fold
//    minimum: the distances are bit-identical to a heap Dijkstra's.
// B  parents by the engine tie rule: the tight in-arc (fl(d[u] + w) == d[v]) with the
//    smallest (d[u], u), the first such arc in in-row order (eid) -- exactly the generic f64
//    kernel's phase B (sssp_f64.hpp); stored as u16 parent + u8 reliability index in LDS.
// C  lat row out; dist's LDS becomes relv (f64); reliability down the tree by level passes
//    (a vertex is computed once its parent is done: relv[v] = relv[p] * r, the source-first
//    left fold); rel row out, f_t last; row min.
// Measured beside the generic kernel in DESIGN.md (fractional C2/C3 variants).
#include "common.hpp"
#include "sssp_delta.hpp"  // (wave scans)

namespace shd {

struct DevF64D {
    int n, nw;
    double delta;                        // bucket width (the 40th percentile of arc latencies)
    const int* __restrict__ row;         // out-CSR (n+1), arcs by (u, v, eid)
    const int* __restrict__ col;
    const double* __restrict__ w;
    const int* __restrict__ row_in;      // in-CSR (undirected: the out-CSR), arcs by (v, u, eid)
    const int* __restrict__ col_in;
    const double* __restrict__ w_in;
    const uint8_t* __restrict__ rix_in;  // index of each in-arc's 1 - loss in rtab
    const double* __restrict__ rtab;     // distinct 1 - loss values (<= 254)
    int nrtab;
    int hring;                           // KFH: ring entries cap (0: what LDS holds; tests)
    // packed arcs (kernels with PK): head | k << 16 per out- / in-arc, weight = k / wscale,
    // exact (every arc checked when the context is made: decimal latencies, k < 65536)
    const uint32_t* __restrict__ opk;
    const uint32_t* __restrict__ ipk;
    double wscale;
    const double* __restrict__ vf;
    const double* __restrict__ self_w;
    const double* __restrict__ self_r;
    unsigned long long* dbg;             // SHD_STAMPS builds: 16 words per source
};
#ifdef SHD_STAMPS
#define KF_STAMP(k) do { if (tid == 0 && g.dbg) g.dbg[(size_t)i * 16 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#define KF_COUNT(k) do { if (tid == 0 && g.dbg) g.dbg[(size_t)i * 16 + (k)] += 1; } while (0)
#define KF_ADD(k, x) do { if (tid == 0 && g.dbg) g.dbg[(size_t)i * 16 + (k)] += (x); } while (0)
#define KF_MARK() unsigned long long kf_t = __builtin_amdgcn_s_memtime()
#define KF_ACC(k) do { if (tid == 0 && g.dbg) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); g.dbg[(size_t)i * 16 + (k)] += t_ - kf_t; kf_t = t_; } } while (0)
#else
#define KF_MARK() do { } while (0)
#define KF_ACC(k) do { } while (0)
#define KF_STAMP(k) do { } while (0)
#define KF_COUNT(k) do { } while (0)
#define KF_ADD(k, x) do { } while (0)
#endif

constexpr int KF_HUB = 24;  // phase B: vertices of more in-arcs are done by a whole wave
#ifndef KFH_SDIV
#define KFH_SDIV 32  // KFH phase A: slice = max(KFH_SMIN, min(64, entries left / KFH_SDIV)) (0: 64)
#endif
#ifndef KFH_SMIN
#define KFH_SMIN 8
#endif
#ifndef KF_SDIV
#define KF_SDIV 16  // the same for the 1024-thread LDS kernel (0: 64-entry slices)
#endif
#ifndef KF_SMIN
#define KF_SMIN 8
#endif
#ifndef KF_SDIV4
#define KF_SDIV4 4  // ... and for 256-thread workgroups
#endif
#ifndef KF_SMIN4
#define KF_SMIN4 16
#endif
#ifndef KFH_WQ
#define KFH_WQ 4  // KFH reliability walks: targets per lane in flight (C4f 506.9 / 505.4 / 506.5 ms at 2 / 4 / 8)
#endif
#ifndef KFH_HUB
#define KFH_HUB KF_HUB  // (KFH's threshold; C4f 12 / 24 / 48 / 96: 830 / 814 / 860 / 905 ms)
#endif

template <int B>
struct KFSmall {
    int qtail;     // ring entries queued (mod n); phase B: hub list length
    int rhead;     // slices of the round taken
    int flag;
    int pflag[3];  // level passes: pass r raises slot r % 3 and clears slot (r + 1) % 3
    int ovf;       // a push of this round found no free ring slot (the ring is dropped after it); 256-thread
                   // workgroups: bit p for a round of parity p
    unsigned long long wmark[B / 64][4];  // per wave: start marks of a trip's four windows
    unsigned long long mpend[2];  // lower bound of the pending distances (bits), by gather parity
    unsigned long long rmin;
};

// LDS: small | dist u64[n] (relv f64 in phase C) | pend u64[nw] | overlay | rtab f64[256], where
// the overlay holds the out-CSR offsets (i32, n + 1) and the bucket queue (u16 x n) in phase
// A, the parents (u16 x n) and their reliability indices (u8 x n) afterwards
template <int B>
struct KFLayout {
    size_t small, dist, pend, wmin, inq, rowl, queue, par, rix, rtab, total;
    __host__ __device__ static KFLayout make(int n) {
        KFLayout L;
        const size_t nw = (size_t)(n + 63) / 64;
        size_t o = 0;
        L.small = o; o += a16(sizeof(KFSmall<B>));
        L.dist = o;  o += a16(8 * (size_t)n);
        L.pend = o;  o += a16(8 * nw);
        L.wmin = o;  o += a16(8 * nw);
        L.inq = o;   o += a16(8 * nw);
        const size_t ov = o;
        L.rowl = ov;
        L.queue = ov + a16(4 * ((size_t)n + 1));
        L.par = ov;
        L.rix = ov + a16(2 * (size_t)n);
        o = ov + std::max(a16(4 * ((size_t)n + 1)) + a16(2 * (size_t)n), a16(2 * (size_t)n) + a16((size_t)n));
        L.rtab = o;  o += 8 * 256;
        L.total = o;
        return L;
    }
};
template <int B>
inline size_t kf_lds_bytes(int n) { return KFLayout<B>::make(n).total; }

// KFH: LDS = small | pend | wmin | inq | key u16[n] | ring u16[R] | rtab, the ring taking
// what LDS is left (R <= n; C4f: 19.6k entries); HBM slice = dist u64[n] (relv) | par u16[n]
// | rix u8[n]
template <int B>
struct KFHLayout {
    size_t small, pend, wmin, inq, key, queue, rtab, total;
    unsigned ring;  // ring entries
    size_t ws_dist, ws_par, ws_rix, ws_total;
    __host__ __device__ static KFHLayout make(int n) {
        KFHLayout L;
        const size_t nw = (size_t)(n + 63) / 64;
        size_t o = 0;
        L.small = o; o += a16(sizeof(KFSmall<B>));
        L.pend = o;  o += a16(8 * nw);
        L.wmin = o;  o += a16(8 * nw);
        L.inq = o;   o += a16(8 * nw);
        L.key = o;   o += a16(2 * (size_t)n + 2);
        L.queue = o;
        const size_t room = o + 8 * 256 + 64 * 2 <= kLdsBudget ? (kLdsBudget - o - 8 * 256) / 2 : 64;
        L.ring = (unsigned)(room < (size_t)n ? room & ~(size_t)63 : (size_t)n);
        // (at least the 512 B per wave phase B's candidate slots take: small graphs' rings
        // are shorter)
        o += a16(std::max(2 * (size_t)L.ring, (size_t)(B / 64) * 512));
        L.rtab = o;  o += 8 * 256;
        L.total = o;
        L.ws_dist = 0;
        L.ws_par = a16(8 * (size_t)n);
        L.ws_rix = L.ws_par + a16(2 * (size_t)n);
        L.ws_total = (L.ws_rix + a16((size_t)n) + 255) & ~(size_t)255;
        return L;
    }
};
template <int B>
inline size_t kfh_lds_bytes(int n) { return KFHLayout<B>::make(n).total; }
template <int B>
inline size_t kfh_ws_stride(int n) { return KFHLayout<B>::make(n).ws_total; }

// KFH distance keys: a u16 per vertex in LDS, monotone in the f64 distance (0 below 1 ms,
// then 12 mantissa bits per binade up to ~65 s, 65535 above and for +inf), kept equal to
// key(dist) by an LDS min after every improving atomicMin.  Keys only fall, so a stale key
// is larger than the true one, and key(nd) > key[v] proves nd > dist[v]: a relaxation is
// dropped there without touching HBM.  Phase B bounds a neighbour's distance by its key's
// interval [lo, hi) and loads it only when fl(lo + w) <= d[v] <= fl(hi + w) can hold.
__device__ inline unsigned kf_key(unsigned long long b) {
    constexpr unsigned long long one = 0x3FF0000000000000ull;
    return b < one ? 0u : (unsigned)min((b - one) >> 40, 65534ull) + 1u;
}
__device__ inline double kf_key_lo(unsigned k) {
    return k == 0 ? 0.0 : as_d(0x3FF0000000000000ull + ((unsigned long long)(k - 1) << 40));
}
__device__ inline double kf_key_hi(unsigned k) {
    return k == 0 ? 1.0 : k >= 65535 ? (double)INFINITY : as_d(0x3FF0000000000000ull + ((unsigned long long)k << 40));
}
__device__ inline void kf_key_min(uint16_t* keyl, int v, unsigned k) {
    unsigned* w = reinterpret_cast<unsigned*>(keyl) + (v >> 1);
    const int sh = (v & 1) * 16;
    unsigned old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (;;) {
        if (((old >> sh) & 0xFFFFu) <= k) return;
        const unsigned nw = (old & ~(0xFFFFu << sh)) | (k << sh);
        const unsigned prev = atomicCAS(w, old, nw);
        if (prev == old) return;
        old = prev;
    }
}

// KFH phase C level passes: a thread's vertices v = tid + k B (k < 64, n <= 64 B) pending
// as bits; per pass each pending vertex reads its parent and factor index and the parent's
// relv, eight vertices' loads in flight, and is written once its parent is done (the
// source-first left fold, as the LDS passes).  A value written in a pass may be read in
// the same pass (every workgroup thread shares the CU's L1, and 64-bit stores are not torn).
template <int B>
__device__ __attribute__((always_inline)) int kfh_levels(int n, int s, int tid, int lane, double* relv, const uint16_t* par,
                                                     const uint8_t* rix, const double* rtl, KFSmall<B>* sm) {
    unsigned long long rem = 0ull;
#pragma unroll 1
    for (int k = 0; k < 64; k++) {
        const int v = tid + k * B;
        if (v < n && relv[v] == -1.0) rem |= 1ull << k;
    }
    if (tid < 3) sm->pflag[tid] = 0;
    __syncthreads();
    for (int pass = 1;; pass++) {
        int prog = 0;
#pragma unroll 1
        for (int k0 = 0; k0 < 64; k0 += 8) {
            if (!((rem >> k0) & 0xFFull)) continue;
            int pq[8];
            double rp[8], rf[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int v = tid + (k0 + k) * B;
                const bool live = (rem >> (k0 + k)) & 1ull;
                pq[k] = live ? (int)par[v] : s;
                rf[k] = live ? rtl[rix[v]] : 1.0;
            }
#pragma unroll
            for (int k = 0; k < 8; k++) rp[k] = ((rem >> (k0 + k)) & 1ull) ? relv[pq[k]] : -1.0;
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (((rem >> (k0 + k)) & 1ull) && rp[k] != -1.0) {
                    relv[tid + (k0 + k) * B] = rp[k] * rf[k];
                    rem &= ~(1ull << (k0 + k));
                    prog = 1;
                }
        }
        // (parity-indexed: the slot cleared here was last read before the previous barrier,
        // so no wave of the next pass can have its raise overwritten)
        if (__any(prog) && lane == 0) sm->pflag[pass % 3] = 1;
        if (tid == 0) sm->pflag[(pass + 1) % 3] = 0;
        __syncthreads();
        const int again = sm->pflag[pass % 3];
        if (!again) return pass;
    }
}

template <int B, bool H = false, bool PK = false>
// (amdgpu_waves_per_eu(4): four 256-thread workgroups per CU need 128 VGPRs or fewer; the
// 256-thread build came out at 129, three waves per SIMD, so only three workgroups per CU)
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(4))) void sssp_f64d_kernel(DevF64D g, const int* __restrict__ src, int ns,
                                                      const int* __restrict__ tgt, int nt, long long ld,
                                                      double* __restrict__ lat_out, double* __restrict__ rel_out,
                                                      double* __restrict__ row_min, int* __restrict__ err,
                                                      char* __restrict__ ws, size_t ws_stride) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int n = g.n, nw = g.nw;
    const KFLayout<B> L = KFLayout<B>::make(n);
    const KFHLayout<B> LH = KFHLayout<B>::make(n);
    char* const wsb = H ? ws + (size_t)blockIdx.x * ws_stride : nullptr;  // KFH: this workgroup's slice
    KFSmall<B>* sm = reinterpret_cast<KFSmall<B>*>(smem + (H ? LH.small : L.small));
    unsigned long long* dist = reinterpret_cast<unsigned long long*>(H ? wsb + LH.ws_dist : smem + L.dist);
    double* relv = reinterpret_cast<double*>(dist);  // phase C, in place of dist
    unsigned long long* pend = reinterpret_cast<unsigned long long*>(smem + (H ? LH.pend : L.pend));
    // per word a lower bound of its pending distances (bits): a gather opens only the words
    // that can hold work below T
    unsigned long long* wmin = reinterpret_cast<unsigned long long*>(smem + (H ? LH.wmin : L.wmin));
    uint16_t* par = reinterpret_cast<uint16_t*>(H ? wsb + LH.ws_par : smem + L.par);
    uint8_t* rix = reinterpret_cast<uint8_t*>(H ? wsb + LH.ws_rix : smem + L.rix);
    uint16_t* ring = reinterpret_cast<uint16_t*>(smem + (H ? LH.queue : L.queue));
    unsigned long long* inq = reinterpret_cast<unsigned long long*>(smem + (H ? LH.inq : L.inq));  // vertex in the ring
    int* rowc = reinterpret_cast<int*>(smem + L.rowl);  // (LDS copy of the out-CSR offsets; KFH reads g.row)
    const int* rowl = H ? g.row : rowc;
    double* rtl = reinterpret_cast<double*>(smem + (H ? LH.rtab : L.rtab));
    uint16_t* keyl = reinterpret_cast<uint16_t*>(smem + LH.key);  // (KFH only)
    const unsigned R = H ? (g.hring > 0 ? min(LH.ring, (unsigned)g.hring) : LH.ring) : (unsigned)n;  // ring entries
    const int tid = threadIdx.x, lane = tid & 63;
    // ring-overflow flag by round parity (no barrier to reset it): 256-thread rows (KFH
    // with it measured slower: C4f 541.4 against 534.2 ms)
    constexpr bool kPar = B < 1024;
    for (int k = tid; k < 256; k += B) rtl[k] = k < g.nrtab ? g.rtab[k] : NAN;

    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (s < 0 || s >= n) {
            if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL);
            continue;
        }
        for (int v = tid; v < n; v += B) dist[v] = kInfBits;
        if (H)
            for (int v = tid; v < (n + 1) / 2; v += B) reinterpret_cast<unsigned*>(keyl)[v] = 0xFFFFFFFFu;
        for (int k = tid; k < nw; k += B) { pend[k] = 0ull; wmin[k] = kInfBits; inq[k] = 0ull; }
        if (tid == 0) { sm->qtail = 0; sm->rhead = 0; sm->ovf = 0; sm->mpend[0] = sm->mpend[1] = kInfBits; }
        int gpar = 0;  // gather parity
        if (!H)
            for (int v = tid; v <= n; v += B) rowc[v] = g.row[v];  // (phase B reuses this LDS)
        __syncthreads();
        if (tid == 0) {
            dist[s] = 0ull;
            pend[s >> 6] = 1ull << (s & 63);
            wmin[s >> 6] = 0ull;
            if (H) keyl[s] = 0;
        }
        double T = g.delta;
        __syncthreads();
        KF_STAMP(0);

        // ---- A: delta-stepping ------------------------------------------------------
        // The queue is a ring (u16 x n; a vertex is in it at most once, by its inq bit): a
        // round expands the entries queued before it, and a relaxation that brings a vertex
        // below T queues it straight back, so a bucket's rounds need no gather.  Vertices
        // improved to T or above wait in the pending bitmask with per-word lower bounds;
        // only an empty ring (the bucket done) opens the next bucket by one gather.
        unsigned qhead = 0;  // ring entries [qhead, sm->qtail) are queued (mod R)
        bool exactg = false;  // KFH: the next gather compares exact distances
        int rpar = 0;        // round parity (the overflow flag of the round)
        for (;;) {
            KF_MARK();
            if (qhead == (unsigned)sm->qtail) {
                // bucket done: T of the next from the words' lower bounds, then one gather
                for (int k = tid; k < nw; k += B) {
                    const unsigned long long wm = wmin[k];
                    if (wm != kInfBits) atomicMin(&sm->mpend[gpar], wm);
                }
                if (tid == 0) sm->mpend[gpar ^ 1] = kInfBits;  // (the next gather's; last read a gather ago)
                __syncthreads();
                const unsigned long long m = sm->mpend[gpar];
                gpar ^= 1;
                if (m == kInfBits) break;                        // nothing pending: done
                T = (floor(as_d(m) / g.delta) + 1.0) * g.delta;   // the next non-empty bucket
                if (!(as_d(m) < T)) T = as_d(m) * 2.0 + g.delta;  // (guard: rounding at huge m)
                // KFH: the pending vertices sorted against T by their LDS keys (key < key(T):
                // below, key > key(T): above, with the key's interval floor as the word's
                // bound), loading a distance only on an equal key; a gather that takes nothing
                // makes the next one exact (the floors could hold T below every true distance)
                const unsigned kT = kf_key(as_u(T));
                const bool bykey = H && !exactg;  // (C4f 505.0 -> 491.9 ms)
                for (int k0 = 0; k0 < nw; k0 += B) {
                    const int k = k0 + tid;
                    unsigned long long take = 0ull, bits = 0ull, rest = kInfBits;
                    const unsigned long long wm = k < nw ? wmin[k] : kInfBits;
                    if (as_d(wm) < T) {
                        bits = pend[k];
                        for (unsigned long long b = bits; b;) {  // four bits per trip: reads in flight
                            int vq[4];
                            unsigned long long dq[4];
#pragma unroll
                            for (int h = 0; h < 4; h++) {
                                vq[h] = b ? (k << 6) + __ffsll((long long)b) - 1 : -1;
                                b &= b - 1;
                            }
                            if (bykey) {
                                unsigned kq[4];
#pragma unroll
                                for (int h = 0; h < 4; h++) kq[h] = vq[h] >= 0 ? (unsigned)keyl[vq[h]] : 0u;
#pragma unroll
                                for (int h = 0; h < 4; h++) {
                                    if (vq[h] < 0) continue;
                                    if (kq[h] < kT) take |= 1ull << (vq[h] & 63);
                                    else if (kq[h] > kT) rest = min(rest, as_u(kf_key_lo(kq[h])));
                                    else {
                                        const unsigned long long d = dist[vq[h]];
                                        if (as_d(d) < T) take |= 1ull << (vq[h] & 63);
                                        else rest = min(rest, d);
                                    }
                                }
                                continue;
                            }
#pragma unroll
                            for (int h = 0; h < 4; h++) dq[h] = dist[vq[h] >= 0 ? vq[h] : 0];
#pragma unroll
                            for (int h = 0; h < 4; h++) {
                                if (vq[h] < 0) continue;
                                if (as_d(dq[h]) < T) take |= 1ull << (vq[h] & 63);
                                else rest = min(rest, dq[h]);
                            }
                        }
                        pend[k] = bits & ~take;
                        wmin[k] = rest;
                        if (take) atomicOr(&inq[k], take);
                    }
                    const int cnt = __popcll(take);
                    const int incl = kd_wave_incl_sum(cnt);
                    int base = 0;
                    if (lane == 63 && incl) base = atomicAdd(&sm->qtail, incl);
                    base = __builtin_amdgcn_readlane(base, 63);
                    unsigned pos = (unsigned)(base + incl - cnt);
                    for (unsigned long long b = take; b;) {
                        const int bi = __ffsll((long long)b) - 1;
                        b &= b - 1;
                        if (!H || pos - qhead < R) {
                            ring[pos % R] = (uint16_t)((k << 6) + bi);
                        } else {  // (KFH: the ring is full; the vertex stays pending, its word's
                                  // bound 0 until the next gather recomputes it)
                            pend[k] |= 1ull << bi;
                            atomicAnd(&inq[k], ~(1ull << bi));
                            wmin[k] = 0ull;
                        }
                        pos++;
                    }
                }
                __syncthreads();
                if (H && tid == 0 && (unsigned)sm->qtail - qhead > R) sm->qtail = (int)(qhead + R);
                if (H) __syncthreads();
                if (H) exactg = (unsigned)sm->qtail == qhead;  // (uniform: after the barrier)
                KF_COUNT(10);
                KF_ACC(8);
                continue;  // (an empty gather -- a loose lower bound -- recomputes T)
            }
            // one round: the entries queued so far, B at a time, arcs load-balanced over the
            // workgroup: each thread takes 4 arc positions per trip, owners by binary search
            // over the entries' offsets, the 8 arc loads of a trip issued together
            const unsigned qend = (unsigned)sm->qtail;
            KF_COUNT(6);
            const int qn = (int)(qend - qhead);
            __syncthreads();  // every wave has read the round's end before any wave queues more
            // (the other parity's flag was read by every thread before this barrier)
            // (an atomic and: waves already in this round may be setting this parity's bit)
            if (kPar && tid == 0) atomicAnd(&sm->ovf, ~(1 << (rpar ^ 1)));
            // waves pull 64-entry slices of the round's entries (no block barrier inside a
            // round); a slice's arcs are spread over its lanes, 4 positions per lane and trip,
            // owners by a binary search over the slice's lane offsets (ds_bpermute), the 8
            // arc loads of a trip issued together
            for (;;) {
                int c = 0, nn = 64;
                if (lane == 0) {
                    constexpr int sdiv = H ? KFH_SDIV : B >= 1024 ? KF_SDIV : KF_SDIV4,
                                  smin = H ? KFH_SMIN : B >= 1024 ? KF_SMIN : KF_SMIN4;
                    if constexpr (sdiv > 0) {
                        // a round's entries in smaller slices as they run out, so the waves
                        // finish the round together (it ends at a barrier): KFH C4f 570.8 ->
                        // 534.5 ms at 32 / 8 (16 / 16: 542.9, 8 / 32: 556.3, 64 / 8: 540.2,
                        // 32 / 4: 536.5, 128 / 4: 569.1); LDS kernels, 1024 threads: C3f 10.42 ->
                        // 9.47 ms at 16 / 8 (32 / 8: 9.80, 8 / 16: 9.75, 16 / 4: 9.51, 24 / 8: 9.69);
                        // 256 threads: C2f 0.449 -> 0.436 ms at 4 / 16 (8 / 16: 0.444, 16 / 8:
                        // 0.488, 32 / 8: 0.522)
                        const int left = qn - __hip_atomic_load(&sm->rhead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        nn = max(smin, min(64, (left + sdiv - 1) / sdiv));
                    }
                    c = atomicAdd(&sm->rhead, nn);
                }
                c = __builtin_amdgcn_readfirstlane(c);
                nn = __builtin_amdgcn_readfirstlane(nn);
                if (c >= qn) break;
                KF_COUNT(11);
                KF_ACC(9);
                const int q = c + lane;
                int u = 0, beg = 0, deg = 0;
                double dun = 0.0;  // (KFH: the entry's distance, one HBM load per entry)
                if (lane < nn && q < qn) {
                    u = ring[(qhead + (unsigned)q) % R];
                    atomicAnd(&inq[u >> 6], ~(1ull << (u & 63)));  // (may be queued again below)
                    beg = rowl[u];
                    deg = rowl[u + 1] - beg;
                    if (H) dun = as_d(dist[u]);
                }
                const int incl = kd_wave_incl_sum(deg);
                const int total = __builtin_amdgcn_readlane(incl, 63);
                const int excl = incl - deg;
                KF_ACC(12);
                // (every queued vertex has an out-arc -- the graph is strongly connected -- so
                // the slice's non-empty entries are lanes 0 .. R-1)
                const bool valid = lane < nn && q < qn;
                unsigned long long* wm4 = sm->wmark[tid >> 6];
                // one trip: owners, then the trip's arc loads issued (not waited on).  owners:
                // each entry marks its start in the window (of 64 positions) that holds it; the
                // owner of position p is the entries starting before the window plus the marks at
                // or below p, minus one
                auto stage = [&](int p0, int (&aq)[4], int (&uq)[4], int (&vq)[4], double (&wq)[4],
                                 double (&duq)[4]) __attribute__((always_inline)) {
                    if (lane < 4) wm4[lane] = 0ull;
                    __builtin_amdgcn_wave_barrier();
                    const int rel = excl - p0;
                    if (valid && rel >= 0 && rel < 4 * 64) atomicOr(&wm4[rel >> 6], 1ull << (rel & 63));
                    __builtin_amdgcn_wave_barrier();
                    int lo[4];
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const unsigned long long before = __ballot(valid && excl < p0 + r * 64);
                        const unsigned long long mk = wm4[r];
                        const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
                        lo[r] = max(0, __popcll(before) + __popcll(mk & upto) - 1);
                    }
                    __builtin_amdgcn_wave_barrier();  // (the marks are read before the next trip clears them)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int p = p0 + r * 64 + lane;
                        const int ob = __shfl(beg, lo[r], 64), oe = __shfl(excl, lo[r], 64);
                        uq[r] = __shfl(u, lo[r], 64);
                        if (H) duq[r] = __shfl(dun, lo[r], 64);
                        aq[r] = p < total ? ob + (p - oe) : -1;
                    }
                    KF_ACC(13);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int a = aq[r] >= 0 ? aq[r] : 0;
                        if constexpr (PK) vq[r] = (int)g.opk[a];  // (decoded when used: the load stays in flight)
                        else { vq[r] = g.col[a]; wq[r] = g.w[a]; }
                    }
                };
                // packed arcs: head and weight out of the loaded word
                auto decode = [&](int (&vq)[4], double (&wq)[4]) __attribute__((always_inline)) {
                    if constexpr (PK) {
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const uint32_t x = (uint32_t)vq[r];
                            vq[r] = (int)(x & 0xFFFFu);
                            wq[r] = (double)(x >> 16) / g.wscale;
                        }
                    }
                };
                // a trip's relaxations (KFH: hold = the candidates' HBM atomicMin results)
                auto relax = [&](const int (&aq)[4], const int (&uq)[4], const int (&vq)[4], const double (&wq)[4],
                                 const double (&duq)[4], const unsigned long long (&hold)[4]) __attribute__((always_inline)) {
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        if (aq[r] < 0) continue;
                        const int v = vq[r];
                        const double nd = (H ? duq[r] : as_d(dist[uq[r]])) + wq[r];
                        const unsigned long long nb = as_u(nd);
                        if (H || nb < dist[v]) {
                            const unsigned long long old = H ? hold[r] : atomicMin(&dist[v], nb);
                            if (nb < old) {
                                if (H) kf_key_min(keyl, v, kf_key(nb));
                                const unsigned long long bit = 1ull << (v & 63);
                                if (nd < T) {  // this bucket: straight back into the ring
                                    if (!(atomicOr(&inq[v >> 6], bit) & bit)) {
                                        // slots [qhead, qhead + n) may still hold this round's
                                        // unread entries (a wave can take its slice and read it
                                        // late): a push past them is dropped and flagged, and the
                                        // round's end moves the whole ring to the pending bitmask
                                        const unsigned at = (unsigned)atomicAdd(&sm->qtail, 1);
                                        if (at - qhead < R) ring[at % R] = (uint16_t)v;
                                        else if (kPar) atomicOr(&sm->ovf, 1 << rpar);
                                        else sm->ovf = 1;
                                    }
                                } else {
                                    atomicOr(&pend[v >> 6], bit);
                                    atomicMin(&wmin[v >> 6], nb);
                                }
                            }
                        }
                    }
                };
                // (eight arc positions per lane and trip with one trip of atomics in flight
                // measured slower than this: C4f 620.9 against 572.1 ms)
                if constexpr (H && PK) {
                    // KFH with packed arcs, two trips of atomics in flight (C4f 765 -> 733 ms
                    // against the one-trip pipeline below): iteration t issues
                    // trip t + 1's arc loads, then trip t's filter and atomics, then trip t - 1's
                    // relaxations -- the loads return in issue order, so trip t's filter waits
                    // for its own loads only, and trip t - 1's results are waited for with trip
                    // t's atomics still out.  A trip between stage and filter is its loaded arc
                    // words and its owner lanes (8 bits each, 0xFF: no arc); past the filter its
                    // candidate heads, distances and atomic results.
                    auto stage2 = [&](int p0, int (&xq)[4], unsigned& lop) __attribute__((always_inline)) {
                        if (lane < 4) wm4[lane] = 0ull;
                        __builtin_amdgcn_wave_barrier();
                        const int rel = excl - p0;
                        if (valid && rel >= 0 && rel < 4 * 64) atomicOr(&wm4[rel >> 6], 1ull << (rel & 63));
                        __builtin_amdgcn_wave_barrier();
                        lop = 0u;
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const unsigned long long before = __ballot(valid && excl < p0 + r * 64);
                            const unsigned long long mk = wm4[r];
                            const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
                            const int lo = max(0, __popcll(before) + __popcll(mk & upto) - 1);
                            const int p = p0 + r * 64 + lane;
                            const int ob = __shfl(beg, lo, 64), oe = __shfl(excl, lo, 64);
                            const bool ok = p < total;
                            xq[r] = (int)g.opk[ok ? ob + (p - oe) : 0];
                            lop |= (unsigned)(ok ? lo : 0xFF) << (8 * r);
                        }
                        __builtin_amdgcn_wave_barrier();  // (the marks are read before the next trip clears them)
                    };
                    auto filter2 = [&](const int (&xq)[4], const unsigned lop, int (&vc)[4], unsigned long long (&nbq)[4],
                                       unsigned long long (&hold)[4]) __attribute__((always_inline)) {
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const unsigned lo = (lop >> (8 * r)) & 0xFFu;
                            const double du = __shfl(dun, (int)(lo & 63u), 64);
                            const uint32_t x = (uint32_t)xq[r];
                            const int v = (int)(x & 0xFFFFu);
                            nbq[r] = as_u(du + (double)(x >> 16) / g.wscale);
                            const bool cand = lo != 0xFFu && kf_key(nbq[r]) <= keyl[v];
                            vc[r] = cand ? v : -1;
                            hold[r] = cand ? atomicMin(&dist[v], nbq[r]) : 0ull;
                        }
                    };
                    auto relax2 = [&](const int (&vc)[4], const unsigned long long (&nbq)[4],
                                      const unsigned long long (&hold)[4]) __attribute__((always_inline)) {
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const int v = vc[r];
                            const unsigned long long nb = nbq[r];
                            if (v >= 0 && nb < hold[r]) {
                                kf_key_min(keyl, v, kf_key(nb));
                                const unsigned long long bit = 1ull << (v & 63);
                                if (as_d(nb) < T) {
                                    if (!(atomicOr(&inq[v >> 6], bit) & bit)) {
                                        const unsigned at = (unsigned)atomicAdd(&sm->qtail, 1);
                                        if (at - qhead < R) ring[at % R] = (uint16_t)v;
                                        else if (kPar) atomicOr(&sm->ovf, 1 << rpar);
                                        else sm->ovf = 1;
                                    }
                                } else {
                                    atomicOr(&pend[v >> 6], bit);
                                    atomicMin(&wmin[v >> 6], nb);
                                }
                            }
                        }
                    };
                    int xa[4], vp[4];
                    unsigned la;
                    unsigned long long np_[4], hp[4];
                    stage2(0, xa, la);
                    bool prev = false;
                    for (int p0 = 0;; p0 += 4 * 64) {
                        const bool more = p0 + 4 * 64 < total;  // (wave-uniform)
                        int xb[4];
                        unsigned lb = 0u;
                        if (more) stage2(p0 + 4 * 64, xb, lb);
                        int vc[4];
                        unsigned long long nbq[4], hold[4];
                        filter2(xa, la, vc, nbq, hold);
                        if (prev) relax2(vp, np_, hp);
#pragma unroll
                        for (int r = 0; r < 4; r++) { vp[r] = vc[r]; np_[r] = nbq[r]; hp[r] = hold[r]; }
                        prev = true;
                        if (!more) break;
#pragma unroll
                        for (int r = 0; r < 4; r++) xa[r] = xb[r];
                        la = lb;
                    }
                    relax2(vp, np_, hp);
                } else if constexpr (H) {
                    // KFH, software-pipelined: a trip's HBM atomics are in flight while the next
                    // trip's owners are found and its arc loads issued; its relaxations (which
                    // wait for the atomics' results) come after.  Past the filter a trip keeps
                    // only v, its candidate distance nb and the atomic's result.
                    int aq[4], uq[4], vq[4];
                    double wq[4], duq[4];
                    stage(0, aq, uq, vq, wq, duq);
                    for (int p0 = 0;; p0 += 4 * 64) {
#ifdef SHD_STAMPS
                        if (tid == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        KF_ACC(14);
#endif
                        decode(vq, wq);
                        // the key filter, then the candidates' HBM atomics issued together
                        unsigned long long hold[4], nbq[4];
                        int vc[4];
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            nbq[r] = as_u(duq[r] + wq[r]);
                            const bool cand = aq[r] >= 0 && kf_key(nbq[r]) <= keyl[vq[r]];
                            vc[r] = cand ? vq[r] : -1;
                            hold[r] = cand ? atomicMin(&dist[vq[r]], nbq[r]) : 0ull;
                        }
                        const bool more = p0 + 4 * 64 < total;  // (wave-uniform)
                        if (more) stage(p0 + 4 * 64, aq, uq, vq, wq, duq);
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            const int v = vc[r];
                            const unsigned long long nb = nbq[r];
                            if (v >= 0 && nb < hold[r]) {
                                kf_key_min(keyl, v, kf_key(nb));
                                const unsigned long long bit = 1ull << (v & 63);
                                if (as_d(nb) < T) {  // this bucket: straight back into the ring
                                    if (!(atomicOr(&inq[v >> 6], bit) & bit)) {
                                        const unsigned at = (unsigned)atomicAdd(&sm->qtail, 1);
                                        if (at - qhead < R) ring[at % R] = (uint16_t)v;
                                        else if (kPar) atomicOr(&sm->ovf, 1 << rpar);
                                        else sm->ovf = 1;  // (a dropped push: see the relax above)
                                    }
                                } else {
                                    atomicOr(&pend[v >> 6], bit);
                                    atomicMin(&wmin[v >> 6], nb);
                                }
                            }
                        }
                        if (!more) break;
                    }
                } else {
                    for (int p0 = 0; p0 < total; p0 += 4 * 64) {
                        int aq[4], uq[4], vq[4];
                        double wq[4], duq[4];
                        stage(p0, aq, uq, vq, wq, duq);
                        decode(vq, wq);
                        if (tid == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        KF_ACC(14);
                        const unsigned long long hold[4] = {0ull, 0ull, 0ull, 0ull};
                        relax(aq, uq, vq, wq, duq, hold);
                    }
                }
            }
            __syncthreads();
            if (tid == 0) sm->rhead = 0;  // (every wave has left the loop above)
            qhead = qend;
            if (kPar ? (sm->ovf >> rpar) & 1 : sm->ovf) {  // (uniform) ring overflow: its vertices (inq) become pending, the ring empty
                for (int k = tid; k < nw; k += B) {
                    const unsigned long long b = inq[k];
                    if (b) { pend[k] |= b; wmin[k] = 0ull; inq[k] = 0ull; }  // (0: a valid lower bound)
                }
                qhead = (unsigned)sm->qtail;
                KF_COUNT(15);
            }
            // (the flag's reset: 256-thread rows clear the other parity's bit at the next
            // round's start, which spares a barrier per round: C2f 0.72 -> 0.45 ms; 1024-thread
            // rows keep the barrier, measured faster there: C3f 10.4 against 10.6-10.7 ms)
            rpar ^= 1;
            if (!kPar) {
                __syncthreads();
                if (tid == 0) sm->ovf = 0;  // (every thread has read it)
            }
            KF_ACC(9);
        }

        KF_STAMP(1);
        // ---- B: parents (tight in-arc with min (d[u], u), first in in-row order) ------
        // two vertices per trip, four in-arcs of each: eight arc loads in flight.  Vertices
        // of more than KF_HUB in-arcs (the BA hubs: one would hold its thread, and the
        // workgroup, for hundreds of trips) are listed and done by whole waves below.
        if (tid == 0) sm->qtail = 0;  // (hub list length; the ring is free now)
        __syncthreads();
        // a neighbour's distance for the tightness test (KFH: INFINITY -- never tight -- when
        // its key interval rules the arc out, so most in-arcs cost no HBM load)
        auto dnb = [&](int u, double w, double dv) __attribute__((always_inline)) {
            if constexpr (H) {
                const unsigned ku = keyl[u];
                if (!(kf_key_lo(ku) + w <= dv && dv <= kf_key_hi(ku) + w)) return (double)INFINITY;
            }
            return as_d(dist[u]);
        };
        if constexpr (H) {
        // KFH, coalesced: a wave takes 64 consecutive vertices at a time (a counter), walks their
        // contiguous in-arc range 256 arcs per trip (lane = arc, four positions per lane: the
        // heads and weights are coalesced loads), finds each arc's vertex by a binary search
        // over the lanes' row starts (row_in is ascending over the lanes), and hands the
        // trip's candidate arcs (few) to their vertices' lanes one by one, in arc order (see
        // the candidates below).  (The per-vertex scan below reads each
        // vertex's arcs in its own lane, 64 lines per load instruction: KFH C4f 799 -> 779 ms
        // with this walk, and its register peak went, 68 B/lane of scratch -> none; the LDS
        // kernels keep the scan: C3f 10.4 against 13.5 ms, C2f 0.45 against 0.62 ms, and with
        // the counted candidates below and the exact LDS test, 9.42 against 9.48 and 0.463
        // against 0.439 ms.)
        (void)dnb;
        if (tid == 0) sm->rhead = 0;
        __syncthreads();
        // the next chunk is taken, and its row starts and distances loaded, before this one's
        // arcs are walked (its setup round trip under this chunk's: C4f 506.2 -> 504.6 ms)
        auto grab = [&]() __attribute__((always_inline)) {
            int c = 0;
            if (lane == 0) c = atomicAdd(&sm->rhead, 64);
            return __builtin_amdgcn_readfirstlane(c);
        };
        int cn = grab(), a0n = 0x7fffffff, aendn = 0;
        unsigned long long dvn = kInfBits;
        auto setup = [&](int c) __attribute__((always_inline)) {
            if (c < n) {
                const int vv = c + lane;
                a0n = vv < n ? g.row_in[vv] : 0x7fffffff;
                aendn = g.row_in[min(c + 64, n)];
                dvn = vv < n ? dist[vv] : kInfBits;
            }
        };
        setup(cn);
        for (;;) {
            const int c0 = cn;
            if (c0 >= n) break;
            const int v = c0 + lane;
            const bool vok = v < n;
            const int a0 = a0n, aend = aendn;
            const double dvr = as_d(dvn);
            cn = grab();
            setup(cn);
            const bool scan = vok && v != s && dvr < INFINITY;
            const double dvt = scan ? dvr : -1.0;  // (-1: never tight -- the source, unreachable)
            // Candidates: the in-arcs whose key interval admits fl(d[u] + w) == d[v] -- every
            // tight arc among them (keys are conservative), and v has at least one tight arc.
            // A vertex with exactly one candidate takes it without loading d[u]; only vertices
            // with two or more (ties, or a near miss inside the key interval) load their
            // candidates' distances and apply the tie rule in a second scan of their arcs
            // (each candidate's d[u] was an HBM load per trip: C4f phase B ~3.1 M cycles/row).
            int cnt = 0, bu = 0x7fffffff, ba = -1;
            const int A0 = __builtin_amdgcn_readfirstlane(a0);
            // candidates counted per vertex by LDS atomics in the wave's 64-vertex slot array
            // (count, first arc); a serial hand-off of each trip's candidates over the ballot
            // (readlanes to the vertex's lane) took longer: C4f 535.2 -> 506.6 ms
            uint32_t* pbs = reinterpret_cast<uint32_t*>(smem + LH.queue) + (tid >> 6) * 128;
            pbs[lane] = 0u;
            pbs[64 + lane] = 0xFFFFFFFFu;
            __builtin_amdgcn_wave_barrier();
            // (the next trip's words loaded under this one, or eight positions per lane: C4f
            // 570.8 / 577.3 ms against 570.9)
            constexpr int BW = 4;  // arc positions per lane and trip
            for (int base = A0; base < aend; base += BW * 64) {
                int uq[BW];
                double wq[BW];
#pragma unroll
                for (int r = 0; r < BW; r++) {
                    const int a = min(base + r * 64 + lane, aend - 1);
                    if constexpr (PK) uq[r] = (int)g.ipk[a];
                    else { uq[r] = g.col_in[a]; wq[r] = g.w_in[a]; }
                }
                int jq[BW];
                bool cq[BW];
#pragma unroll
                for (int r = 0; r < BW; r++) {
                    const int a = base + r * 64 + lane;
                    int j = 0;
#pragma unroll
                    for (int st = 32; st >= 1; st >>= 1)
                        if (__shfl(a0, j + st, 64) <= a) j += st;
                    jq[r] = j;
                    if constexpr (PK) {
                        const uint32_t x = (uint32_t)uq[r];
                        uq[r] = (int)(x & 0xFFFFu);
                        wq[r] = (double)(x >> 16) / g.wscale;
                    }
                    const double dvo = __shfl(dvt, j, 64);
                    cq[r] = false;
                    if (a < aend && dvo >= 0.0) {
                        const unsigned ku = keyl[uq[r]];
                        cq[r] = kf_key_lo(ku) + wq[r] <= dvo && dvo <= kf_key_hi(ku) + wq[r];
                    }
                }
#pragma unroll
                for (int r = 0; r < BW; r++)
                    if (cq[r]) {
                        atomicAdd(&pbs[jq[r]], 1u);
                        atomicMin(&pbs[64 + jq[r]], (uint32_t)(base + r * 64 + lane));
                    }
            }
            __builtin_amdgcn_wave_barrier();
            cnt = (int)pbs[lane];
            if (cnt == 1) {
                ba = (int)pbs[64 + lane];
                if constexpr (PK) bu = (int)(g.ipk[ba] & 0xFFFFu);
                else bu = g.col_in[ba];
            }
            __builtin_amdgcn_wave_barrier();  // (the slots are read before the next chunk clears them)
            if (scan && cnt >= 2) {
                // the exact rule over this vertex's arcs: tight (fl(d[u] + w) == d[v], d[u]
                // loaded for candidates only), minimum (d[u], u), the first arc on a full tie
                double bd = INFINITY;
                bu = 0x7fffffff; ba = -1;
                const int a1v = g.row_in[v + 1];
                for (int a = a0; a < a1v; a++) {
                    int u;
                    double w;
                    if constexpr (PK) {
                        const uint32_t x = g.ipk[a];
                        u = (int)(x & 0xFFFFu);
                        w = (double)(x >> 16) / g.wscale;
                    } else { u = g.col_in[a]; w = g.w_in[a]; }
                    const unsigned ku = keyl[u];
                    if (!(kf_key_lo(ku) + w <= dvr && dvr <= kf_key_hi(ku) + w)) continue;
                    const double du = as_d(dist[u]);
                    if (du + w == dvr && (du < bd || (du == bd && u < bu))) { bd = du; bu = u; ba = a; }
                }
            }
            if (vok) {
                int pu = v, pr = 255;
                if (ba >= 0) { pu = bu; pr = g.rix_in[ba]; }
                else if (scan) raise_err(err, SHD_ROUTE_EUNREACH);  // (cannot happen)
                par[v] = (uint16_t)pu;
                rix[v] = (uint8_t)pr;
            }
        }
        __syncthreads();
        } else {
        for (int v0 = tid; v0 < n; v0 += 2 * B) {
            int vv[2], a0[2], a1[2], bu[2], ba[2];
            double dv[2], bd[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                vv[h] = v0 + h * B;
                const bool ok = vv[h] < n;
                dv[h] = ok ? as_d(dist[vv[h]]) : INFINITY;
                const bool scan = ok && vv[h] != s && dv[h] < INFINITY;
                a0[h] = scan ? g.row_in[vv[h]] : 0;
                a1[h] = scan ? g.row_in[vv[h] + 1] : 0;
                if (a1[h] - a0[h] > (H ? KFH_HUB : KF_HUB)) {
                    const int hs = atomicAdd(&sm->qtail, 1);
                    if (!H || hs < (int)R) {  // (KFH: a full list leaves the hub to its thread)
                        ring[hs] = (uint16_t)vv[h];
                        a1[h] = a0[h];
                        vv[h] = -1 - vv[h];  // (written by the wave below)
                    }
                }
                bd[h] = INFINITY; bu[h] = 0x7fffffff; ba[h] = -1;
            }
            constexpr int KBW = H ? 8 : 4;  // in-arcs per vertex and step (KFH: more HBM loads in flight)
            for (int t0 = 0; t0 < max(a1[0] - a0[0], a1[1] - a0[1]); t0 += KBW) {
                int uq[2][KBW];
                double wq[2][KBW];
#pragma unroll
                for (int h = 0; h < 2; h++)
#pragma unroll
                    for (int q = 0; q < KBW; q++) {
                        const int a = min(a0[h] + t0 + q, max(a1[h] - 1, 0));
                        if constexpr (PK) uq[h][q] = (int)g.ipk[a];
                        else { uq[h][q] = g.col_in[a]; wq[h][q] = g.w_in[a]; }
                    }
                if constexpr (PK) {
#pragma unroll
                    for (int h = 0; h < 2; h++)
#pragma unroll
                        for (int q = 0; q < KBW; q++) {
                            const uint32_t x = (uint32_t)uq[h][q];
                            uq[h][q] = (int)(x & 0xFFFFu);
                            wq[h][q] = (double)(x >> 16) / g.wscale;
                        }
                }
#pragma unroll
                for (int h = 0; h < 2; h++)
#pragma unroll
                    for (int q = 0; q < KBW; q++) {
                        if (a0[h] + t0 + q >= a1[h]) continue;
                        const double du = dnb(uq[h][q], wq[h][q], dv[h]);
                        if (du + wq[h][q] == dv[h] && (du < bd[h] || (du == bd[h] && uq[h][q] < bu[h]))) {
                            bd[h] = du; bu[h] = uq[h][q]; ba[h] = a0[h] + t0 + q;
                        }
                    }
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int v = vv[h];
                if (v < 0 || v >= n) continue;
                int pu = v, pr = 255;
                if (ba[h] >= 0) { pu = bu[h]; pr = g.rix_in[ba[h]]; }
                else if (v != s && dv[h] < INFINITY) raise_err(err, SHD_ROUTE_EUNREACH);  // (cannot happen)
                par[v] = (uint16_t)pu;
                rix[v] = (uint8_t)pr;
            }
        }
        __syncthreads();
        {
            // hubs: 16 lanes per hub (four hubs per wave at a time), 4 in-arcs per lane and
            // step with the loads in flight, then the lexicographic (d[u], u, arc) minimum
            // over the hub's 16 lanes
            const int nhub = min(sm->qtail, (int)R);
            const int sub = lane >> 4, sl = lane & 15;
            for (int h0 = (tid >> 6) * 4; h0 < nhub; h0 += (B / 64) * 4) {
                const int h = h0 + sub;
                const bool hv = h < nhub;
                const int v = hv ? ring[h] : 0;
                const double dv = as_d(dist[v]);
                const int a0 = hv ? g.row_in[v] : 0, a1 = hv ? g.row_in[v + 1] : 0;
                double bd = INFINITY;
                int bu = 0x7fffffff, ba = 0x7fffffff;
                for (int t = a0 + sl; __any(t < a1); t += 64) {
                    int uq[4];
                    double wq[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int a = min(t + 16 * q, max(a1 - 1, 0));
                        if constexpr (PK) {
                            const uint32_t x = g.ipk[a];
                            uq[q] = (int)(x & 0xFFFFu);
                            wq[q] = (double)(x >> 16) / g.wscale;
                        } else { uq[q] = g.col_in[a]; wq[q] = g.w_in[a]; }
                    }
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int a = t + 16 * q;
                        if (a >= a1) continue;
                        const double du = dnb(uq[q], wq[q], dv);
                        if (du + wq[q] == dv && (du < bd || (du == bd && (uq[q] < bu || (uq[q] == bu && a < ba))))) {
                            bd = du; bu = uq[q]; ba = a;
                        }
                    }
                }
#pragma unroll
                for (int d = 8; d >= 1; d >>= 1) {  // within the 16 lanes of the hub
                    const double od = __shfl_xor(bd, d, 64);
                    const int ou = __shfl_xor(bu, d, 64), oa = __shfl_xor(ba, d, 64);
                    if (od < bd || (od == bd && (ou < bu || (ou == bu && oa < ba)))) { bd = od; bu = ou; ba = oa; }
                }
                if (hv && sl == 0) {
                    if (ba != 0x7fffffff) { par[v] = (uint16_t)bu; rix[v] = g.rix_in[ba]; }
                    else { par[v] = (uint16_t)v; rix[v] = 255; raise_err(err, SHD_ROUTE_EUNREACH); }
                }
            }
        }
        __syncthreads();

        }
        KF_STAMP(2);
        // ---- C: lat row, then reliability down the tree ------------------------------
        const double fs = g.vf[s];
        const double cs = isnan(fs) ? 1.0 : 1.0 * fs;
        const double sw_s = g.self_w[s], sr_s = g.self_r[s];
        double* lrow = lat_out ? lat_out + (long long)i * ld : nullptr;
        double* rrow = rel_out ? rel_out + (long long)i * ld : nullptr;
        double lmin = INFINITY;
        for (int j = tid; j < nt; j += B) {
            const int t = tgt[j];
            double Lv;
            if (t < 0 || t >= n) { raise_err(err, SHD_ROUTE_EINVAL); Lv = NAN; }
            else if (t == s) {
                if (isnan(sw_s)) { raise_err(err, SHD_ROUTE_ENOEDGE); Lv = NAN; }
                else Lv = 0.0 + sw_s;  // the batch path [s]: one self-loop hop (topology.c:1471-1499)
            } else {
                Lv = as_d(dist[t]);
                if (!(Lv < INFINITY)) { raise_err(err, SHD_ROUTE_EUNREACH); Lv = NAN; }
                else if (Lv == 0.0) Lv = 1.0;  // topology.c:1848-1852
            }
            if (lrow) lrow[j] = Lv;
            if (!isnan(Lv)) lmin = fmin(lmin, Lv);
        }
        __syncthreads();
        KF_STAMP(3);
        // KFH (round 5): reliability by walks in LDS.  Phase A/B's LDS is dead now; the
        // parents (u16) and factor indices (u8) come in from the slice (150 KB at C4f), and
        // each target walks its tree path to the source, keeping the indices of the lossy arcs
        // (a lossless arc's exact 1.0 leaves every product unchanged) and folds them
        // source-first: the products of the level passes below, bit for bit.  Two targets per
        // lane in turn.  A path with more than 16 lossy arcs sends the whole row to the level
        // passes (rare: ~2 lossy arcs per C4f path).
        bool walked = false;
        if constexpr (H) {
            const size_t po = LH.pend, ro = LH.pend + a16(2 * (size_t)n);
            if (rrow && ro + a16((size_t)n) <= LH.rtab) {
                uint16_t* parl = reinterpret_cast<uint16_t*>(smem + po);
                uint8_t* rixl = reinterpret_cast<uint8_t*>(smem + ro);
                for (int v = tid; v < n; v += B) { parl[v] = par[v]; rixl[v] = rix[v]; }
                if (tid == 0) sm->flag = 0;
                __syncthreads();
                int deep = 0;
                for (int j0 = tid; j0 < nt; j0 += KFH_WQ * B) {
                    int t2[KFH_WQ], v2[KFH_WQ], ns2[KFH_WQ];
                    unsigned long long lo2[KFH_WQ], hi2[KFH_WQ];
                    bool go2[KFH_WQ];
                    double R2[KFH_WQ];
#pragma unroll
                    for (int h = 0; h < KFH_WQ; h++) {
                        const int j = j0 + h * B;
                        const int t = j < nt ? tgt[j] : -1;
                        t2[h] = t; v2[h] = t; ns2[h] = 0; lo2[h] = hi2[h] = 0ull; go2[h] = false; R2[h] = NAN;
                        if (j >= nt) continue;
                        if (t < 0 || t >= n) continue;  // (the lat row raised EINVAL)
                        if (t == s) R2[h] = isnan(sw_s) ? (double)NAN : cs * sr_s;
                        else if (rixl[t] != 255) go2[h] = true;  // (255: unreachable, NaN)
                    }
                    auto anygo = [&]() __attribute__((always_inline)) {
                        bool a = false;
#pragma unroll
                        for (int h = 0; h < KFH_WQ; h++) a = a || go2[h];
                        return a;
                    };
                    for (int step = 0; anygo() && step < n; step++) {
#pragma unroll
                        for (int h = 0; h < KFH_WQ; h++) {
                            if (!go2[h]) continue;
                            const int v = v2[h];
                            const unsigned r = rixl[v];
                            const int pv = parl[v];
                            if (rtl[r] != 1.0) {
                                const int k = ns2[h]++;
                                if (k < 8) lo2[h] |= (unsigned long long)r << (8 * k);
                                else if (k < 16) hi2[h] |= (unsigned long long)r << (8 * (k - 8));
                                else deep = 1;
                            }
                            v2[h] = pv;
                            if (pv == s) go2[h] = false;
                        }
                    }
                    if (anygo()) deep = 1;  // (a parent cycle: cannot happen)
#pragma unroll
                    for (int h = 0; h < KFH_WQ; h++) {
                        const int j = j0 + h * B;
                        if (j >= nt) continue;
                        const int t = t2[h];
                        if (t >= 0 && t < n && t != s && rixl[t] != 255) {
                            // from (1.0 * f_s) * f_t, the reference's order (topology.c:1443-1462,
                            // then :1499): bit-exact under vertex loss
                            const double ft = g.vf[t];
                            double x = isnan(ft) ? cs : cs * ft;
                            for (int k = min(ns2[h], 16) - 1; k >= 0; k--) {
                                const unsigned r = (unsigned)((k < 8 ? lo2[h] >> (8 * k) : hi2[h] >> (8 * (k - 8))) & 0xFFull);
                                x *= rtl[r];
                            }
                            R2[h] = x;
                        }
                        rrow[j] = R2[h];
                    }
                }
                if (deep) sm->flag = 1;
                __syncthreads();
                walked = sm->flag == 0;
                __syncthreads();  // (every thread has read the flag)
            }
        }
        if (!walked) {
        // relv over dist's LDS: the source cs, unreachable NaN, the rest pending (-1)
        for (int v = tid; v < n; v += B) {
            const bool unr = v != s && !(as_d(dist[v]) < INFINITY);
            relv[v] = v == s ? cs : unr ? (double)NAN : -1.0;
        }
        __syncthreads();
        // level passes: a vertex whose parent is done takes relv[p] * r(p, v); every vertex is
        // written once, after its parent, so the products are the source-first left folds.
        // A thread keeps its vertices' parents and factors in registers and reads all their
        // parents' values at once per pass; a value written during a pass may be read in the
        // same pass (64-bit LDS accesses are not torn), which only finishes chains sooner
        // (parents and factor indices packed: 2 x u16 and 4 x u8 per register)
        if constexpr (H) {
            [[maybe_unused]] const int passes = kfh_levels<B>(n, s, tid, lane, relv, par, rix, rtl, sm);
            KF_ADD(7, passes);
        } else {
        uint32_t pk2[8], rx4[4];
        unsigned rem = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) pk2[k] = (uint32_t)s | ((uint32_t)s << 16);
#pragma unroll
        for (int k = 0; k < 4; k++) rx4[k] = 0u;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int v = tid + k * B;
            if (v < n) {
                pk2[k >> 1] = (pk2[k >> 1] & ~(0xFFFFu << (16 * (k & 1)))) | ((uint32_t)par[v] << (16 * (k & 1)));
                rx4[k >> 2] |= (uint32_t)rix[v] << (8 * (k & 3));
                if (relv[v] == -1.0) rem |= 1u << k;
            }
        }
        if (tid < 3) sm->pflag[tid] = 0;
        __syncthreads();
        for (int pass = 1;; pass++) {
            int prog = 0;
#pragma unroll
            for (int k0 = 0; k0 < 16; k0 += 8) {
                if (!((rem >> k0) & 0xFFu)) continue;
                double rp[8], rf[8];
#pragma unroll
                for (int k = k0; k < k0 + 8; k++) {
                    const bool live = (rem >> k) & 1u;
                    rp[k - k0] = live ? relv[(pk2[k >> 1] >> (16 * (k & 1))) & 0xFFFFu] : -1.0;
                    rf[k - k0] = rtl[(rx4[k >> 2] >> (8 * (k & 3))) & 0xFFu];
                }
#pragma unroll
                for (int k = k0; k < k0 + 8; k++)
                    if (((rem >> k) & 1u) && rp[k - k0] != -1.0) {
                        relv[tid + k * B] = rp[k - k0] * rf[k - k0];
                        rem &= ~(1u << k);
                        prog = 1;
                    }
            }
            // (parity-indexed flags, as kfh_levels: one barrier per pass, no lost raise)
            if (__any(prog) && lane == 0) sm->pflag[pass % 3] = 1;
            if (tid == 0) sm->pflag[(pass + 1) % 3] = 0;
            __syncthreads();
            const int again = sm->pflag[pass % 3];
            KF_COUNT(7);
            if (!again) break;
        }
        }
        }  // (!walked)
        KF_STAMP(4);
        for (int j = tid; j < (walked ? 0 : nt); j += B) {
            const int t = tgt[j];
            double Rv = NAN;
            if (t >= 0 && t < n) {
                if (t == s) Rv = isnan(sw_s) ? NAN : cs * sr_s;
                else {
                    const double x = relv[t];
                    const double ft = g.vf[t];
                    Rv = isnan(ft) ? x : x * ft;
                }
            }
            if (rrow) rrow[j] = Rv;
        }
        if (row_min) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
            if (tid == 0) sm->rmin = kInfBits;
            __syncthreads();
            if (lane == 0 && lmin < INFINITY) atomicMin(&sm->rmin, as_u(lmin));
            __syncthreads();
            if (tid == 0) row_min[i] = as_d(sm->rmin);
        }
        KF_STAMP(5);
        __syncthreads();
    }
}

}  // namespace shd
