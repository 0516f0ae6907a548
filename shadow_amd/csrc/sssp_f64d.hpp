#pragma once
// "KF": SOURCE rows for fractional-latency topologies (any positive double latencies) whose
// per-source state fits LDS (n up to ~12k at 1024 threads, ~3k at four 256-thread workgroups
// per CU).  One workgroup per source.
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
    double delta;                        // bucket width (the 12th percentile of arc latencies)
    const int* __restrict__ row;         // out-CSR (n+1), arcs by (u, v, eid)
    const int* __restrict__ col;
    const double* __restrict__ w;
    const int* __restrict__ row_in;      // in-CSR (undirected: the out-CSR), arcs by (v, u, eid)
    const int* __restrict__ col_in;
    const double* __restrict__ w_in;
    const uint8_t* __restrict__ rix_in;  // index of each in-arc's 1 - loss in rtab
    const double* __restrict__ rtab;     // distinct 1 - loss values (<= 254)
    int nrtab;
    const double* __restrict__ vf;
    const double* __restrict__ self_w;
    const double* __restrict__ self_r;
    unsigned long long* dbg;             // SHD_STAMPS builds: 8 words per source
};
#ifdef SHD_STAMPS
#define KF_STAMP(k) do { if (tid == 0 && g.dbg) g.dbg[(size_t)i * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#define KF_COUNT(k) do { if (tid == 0 && g.dbg) g.dbg[(size_t)i * 8 + (k)] += 1; } while (0)
#else
#define KF_STAMP(k) do { } while (0)
#define KF_COUNT(k) do { } while (0)
#endif

template <int B>
struct KFSmall {
    int off[B + 1];   // block scan of the queue slice's degrees
    int u[B];
    int beg[B];
    int wsum[B / 64];
    int qtail;
    int flag;
    unsigned long long mpend;  // min distance (bits) over pending vertices left at or above T
    unsigned long long rmin;
};

// LDS: small | dist u64[n] (relv f64 in phase C) | pend u64[nw] | overlay | rtab f64[256], where
// the overlay holds the out-CSR offsets (i32, n + 1) and the bucket queue (u16 x n) in phase
// A, the parents (u16 x n) and their reliability indices (u8 x n) afterwards
template <int B>
struct KFLayout {
    size_t small, dist, pend, rowl, queue, par, rix, rtab, total;
    __host__ __device__ static KFLayout make(int n) {
        KFLayout L;
        const size_t nw = (size_t)(n + 63) / 64;
        size_t o = 0;
        L.small = o; o += a16(sizeof(KFSmall<B>));
        L.dist = o;  o += a16(8 * (size_t)n);
        L.pend = o;  o += a16(8 * nw);
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

template <int B>
__device__ inline int kf_block_excl_scan(int x, KFSmall<B>* sm, int* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) sm->wsum[wv] = incl;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < B / 64; k++) {
        const int s = sm->wsum[k];
        pre += (k < wv) ? s : 0;
        tot += s;
    }
    *total = tot;
    return pre + incl - x;
}

template <int B>
__global__ __launch_bounds__(B) void sssp_f64d_kernel(DevF64D g, const int* __restrict__ src, int ns,
                                                      const int* __restrict__ tgt, int nt, long long ld,
                                                      double* __restrict__ lat_out, double* __restrict__ rel_out,
                                                      double* __restrict__ row_min, int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int n = g.n, nw = g.nw;
    const KFLayout<B> L = KFLayout<B>::make(n);
    KFSmall<B>* sm = reinterpret_cast<KFSmall<B>*>(smem + L.small);
    unsigned long long* dist = reinterpret_cast<unsigned long long*>(smem + L.dist);
    double* relv = reinterpret_cast<double*>(smem + L.dist);  // phase C, in place of dist
    unsigned long long* pend = reinterpret_cast<unsigned long long*>(smem + L.pend);
    uint16_t* par = reinterpret_cast<uint16_t*>(smem + L.par);
    uint8_t* rix = reinterpret_cast<uint8_t*>(smem + L.rix);
    uint16_t* queue = reinterpret_cast<uint16_t*>(smem + L.queue);
    int* rowl = reinterpret_cast<int*>(smem + L.rowl);
    double* rtl = reinterpret_cast<double*>(smem + L.rtab);
    const int tid = threadIdx.x, lane = tid & 63;
    for (int k = tid; k < 256; k += B) rtl[k] = k < g.nrtab ? g.rtab[k] : NAN;

    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (s < 0 || s >= n) {
            if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL);
            continue;
        }
        for (int v = tid; v < n; v += B) dist[v] = kInfBits;
        for (int k = tid; k < nw; k += B) pend[k] = 0ull;
        for (int v = tid; v <= n; v += B) rowl[v] = g.row[v];  // (phase B reuses this LDS)
        __syncthreads();
        if (tid == 0) {
            dist[s] = 0ull;
            pend[s >> 6] = 1ull << (s & 63);
        }
        double T = g.delta;
        __syncthreads();
        KF_STAMP(0);

        // ---- A: delta-stepping ------------------------------------------------------
        for (;;) {
            if (tid == 0) { sm->qtail = 0; sm->mpend = kInfBits; }
            __syncthreads();
            // gather: pending vertices below T into the queue (one thread per word)
            for (int k0 = 0; k0 < nw; k0 += B) {
                const int k = k0 + tid;
                unsigned long long bits = k < nw ? pend[k] : 0ull, take = 0ull;
                unsigned long long rest = kInfBits;
                for (unsigned long long b = bits; b;) {
                    const int bi = __ffsll((long long)b) - 1;
                    b &= b - 1;
                    const unsigned long long dv = dist[(k << 6) + bi];
                    if (as_d(dv) < T) take |= 1ull << bi;
                    else rest = min(rest, dv);
                }
                if (rest != kInfBits) atomicMin(&sm->mpend, rest);
                const int cnt = __popcll(take);
                const int incl = kd_wave_incl_sum(cnt);
                int base = 0;
                if (lane == 63 && incl) base = atomicAdd(&sm->qtail, incl);
                base = __builtin_amdgcn_readlane(base, 63);
                int pos = base + incl - cnt;
                for (unsigned long long b = take; b;) {
                    const int bi = __ffsll((long long)b) - 1;
                    b &= b - 1;
                    queue[pos++] = (uint16_t)((k << 6) + bi);
                }
                if (take) pend[k] = bits & ~take;
            }
            __syncthreads();
            const int qn = sm->qtail;
            KF_COUNT(6);
            if (qn == 0) {
                const unsigned long long m = sm->mpend;
                if (m == kInfBits) break;                       // nothing pending: done
                T = (floor(as_d(m) / g.delta) + 1.0) * g.delta;  // the next non-empty bucket
                if (!(as_d(m) < T)) T = as_d(m) * 2.0 + g.delta; // (guard: rounding at huge m)
                __syncthreads();
                continue;
            }
            // expand the queue, B entries at a time, arcs load-balanced over the workgroup:
            // each thread takes 4 arc positions per trip, owners by binary search over the
            // entries' offsets, the 8 arc loads of a trip issued together
            for (int c0 = 0; c0 < qn; c0 += B) {
                const int q = c0 + tid;
                int u = 0, beg = 0, deg = 0;
                if (q < qn) {
                    u = queue[q];
                    beg = rowl[u];
                    deg = rowl[u + 1] - beg;
                }
                int total;
                const int off = kf_block_excl_scan<B>(deg, sm, &total);
                const int cnt = min(B, qn - c0);
                sm->off[tid] = off;
                sm->u[tid] = u;
                sm->beg[tid] = beg;
                __syncthreads();
                for (int e0 = 0; e0 < total; e0 += 4 * B) {
                    int aq[4], uq[4];
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int e = e0 + r * B + tid;
                        int lo = 0, hi = cnt;  // last entry with off <= e
                        while (hi - lo > 1) {
                            const int mid = (lo + hi) >> 1;
                            if (sm->off[mid] <= e) lo = mid; else hi = mid;
                        }
                        aq[r] = e < total ? sm->beg[lo] + (e - sm->off[lo]) : -1;
                        uq[r] = sm->u[lo];
                    }
                    int vq[4];
                    double wq[4];
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int a = aq[r] >= 0 ? aq[r] : 0;
                        vq[r] = g.col[a];
                        wq[r] = g.w[a];
                    }
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        if (aq[r] < 0) continue;
                        const int v = vq[r];
                        const unsigned long long nb = as_u(as_d(dist[uq[r]]) + wq[r]);
                        if (nb < dist[v]) {
                            const unsigned long long old = atomicMin(&dist[v], nb);
                            if (nb < old) atomicOr(&pend[v >> 6], 1ull << (v & 63));
                        }
                    }
                }
                __syncthreads();
            }
        }

        KF_STAMP(1);
        // ---- B: parents (tight in-arc with min (d[u], u), first in in-row order) ------
        for (int v = tid; v < n; v += B) {
            const double dv = as_d(dist[v]);
            int pu = v, pr = 255;
            if (v != s && dv < INFINITY) {
                double bd = INFINITY;
                int bu = 0x7fffffff, ba = -1;
                const int a1 = g.row_in[v + 1];
                for (int a0 = g.row_in[v]; a0 < a1; a0 += 4) {
                    int uq[4];
                    double wq[4];
#pragma unroll
                    for (int h = 0; h < 4; h++) {
                        const int a = min(a0 + h, a1 - 1);
                        uq[h] = g.col_in[a];
                        wq[h] = g.w_in[a];
                    }
#pragma unroll
                    for (int h = 0; h < 4; h++) {
                        if (a0 + h >= a1) continue;
                        const double du = as_d(dist[uq[h]]);
                        if (du + wq[h] == dv && (du < bd || (du == bd && uq[h] < bu))) { bd = du; bu = uq[h]; ba = a0 + h; }
                    }
                }
                if (ba >= 0) { pu = bu; pr = g.rix_in[ba]; }
                else raise_err(err, SHD_ROUTE_EUNREACH);  // (a finite distance always has a tight arc)
            }
            par[v] = (uint16_t)pu;
            rix[v] = (uint8_t)pr;
        }
        __syncthreads();

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
        // relv over dist's LDS: the source cs, unreachable NaN, the rest pending (-1)
        for (int v = tid; v < n; v += B) {
            const bool unr = v != s && !(as_d(dist[v]) < INFINITY);
            relv[v] = v == s ? cs : unr ? (double)NAN : -1.0;
        }
        __syncthreads();
        // level passes: a vertex whose parent is done takes relv[p] * r(p, v); every vertex is
        // written once, after its parent, so the products are the source-first left folds
        if (tid == 0) sm->flag = 0;
        __syncthreads();
        for (;;) {
            int prog = 0;
            double nv[16];
            unsigned todo = 0;
            int k = 0;
            for (int v = tid; v < n; v += B, k++) {
                if (k >= 16) break;
                if (relv[v] == -1.0) {
                    const double rp = relv[par[v]];
                    if (rp != -1.0) { nv[k] = rp * rtl[rix[v]]; todo |= 1u << k; }
                }
            }
            __syncthreads();
            k = 0;
            for (int v = tid; v < n; v += B, k++) {
                if (k >= 16) break;
                if ((todo >> k) & 1u) { relv[v] = nv[k]; prog = 1; }
            }
            if (__any(prog) && lane == 0) sm->flag = 1;
            __syncthreads();
            const int again = sm->flag;
            __syncthreads();  // every thread has read the flag before it is cleared
            if (tid == 0) sm->flag = 0;
            KF_COUNT(7);
            if (!again) break;
        }
        KF_STAMP(4);
        for (int j = tid; j < nt; j += B) {
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
