#pragma once
// "K16": SOURCE rows for large integer-latency topologies (C3/C4-class, n <= 65535,
// e.g. 50k vertices / 1M arcs), one 1024-thread workgroup per source, fused:
//   A  frontier Bellman-Ford with u16 distances in LDS (2 B/vertex: 100 KB at n=50k).
//      There is no 16-bit LDS atomic, so an improvement is a 32-bit CAS on the word
//      holding two neighbouring distances.  Frontiers are bitmasks (u64 words = 64
//      vertices); each wave takes one word at a time and expands the set bits with
//      the wave-level load-balanced scheme of sssp_k32.hpp.
//   B  lat row out (dist is exact: integer latencies, bound < 0xFFFF); parent slot =
//      first tight arc of the (-w, u, eid)-sorted in-row (= argmin (dist[u], u, eid)).
//   C  reliability down the tree, level-synchronous, relv in a per-workgroup HBM slice
//      (8n bytes do not fit LDS at this size), parents u16 in LDS.
//   D  rel row out, row min.
// Replaces igraph_get_shortest_paths_dijkstra (topology.c:1756) +
// _topology_computePathProperties (topology.c:1407-1523) for these graphs.
#include "common.hpp"

namespace shd {

constexpr int K16_BLOCK = 1024;

struct DevK16 {
    int n;
    int bound;
    const int* __restrict__ row;        // out-CSR offsets
    const uint32_t* __restrict__ oarc;  // out-arcs (v << 16 | w)
    const int* __restrict__ row_in;     // in-CSR offsets, rows sorted by (-w, u, eid)
    const uint32_t* __restrict__ iarc;  // in-arcs (u << 16 | w)
    const double* __restrict__ r_in;    // 1 - loss per in-arc
    const double* __restrict__ vf;
    const double* __restrict__ self_w;
    const double* __restrict__ self_r;
};

struct K16Layout {
    size_t dist, cur, nxt, total;
    __host__ __device__ static K16Layout make(int n) {
        K16Layout L;
        size_t o = 64;  // small: cursor, any, flag, rmin
        const size_t nw = (size_t)(n + 63) / 64;
        L.dist = o; o += a16(sizeof(uint16_t) * (size_t)(n + 1));
        L.cur = o;  o += a16(sizeof(unsigned long long) * nw);
        L.nxt = o;  o += a16(sizeof(unsigned long long) * nw);
        L.total = o;
        return L;
    }
};

// relv (f64 n) + parent slots (u16 n) per workgroup, in HBM
__host__ __device__ inline size_t k16_ws_stride(int n) { return a16(sizeof(double) * n) + a16(sizeof(uint16_t) * n) + 256; }

__device__ inline unsigned dist16(const uint16_t* d, int v) { return d[v]; }

// lower the u16 at d[v] to nd if smaller; true if this call lowered it
__device__ inline bool lower16(uint16_t* d, int v, unsigned nd) {
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

__global__ __launch_bounds__(K16_BLOCK) void sssp_k16_kernel(DevK16 g, const int* __restrict__ src, int ns,
                                                             const int* __restrict__ tgt, int nt, long long ld,
                                                             double* __restrict__ lat_out, double* __restrict__ rel_out,
                                                             double* __restrict__ row_min, int* __restrict__ err,
                                                             char* __restrict__ ws, size_t ws_stride) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* cursor = reinterpret_cast<int*>(smem);
    int* anyflag = reinterpret_cast<int*>(smem + 4);
    int* flag = reinterpret_cast<int*>(smem + 8);
    unsigned long long* rmin = reinterpret_cast<unsigned long long*>(smem + 16);
    unsigned char* wflag_all = reinterpret_cast<unsigned char*>(smem + 64);  // 16 waves x 64 B after layout
    const int n = g.n;
    const K16Layout L = K16Layout::make(n);
    uint16_t* dist = reinterpret_cast<uint16_t*>(smem + L.dist);
    unsigned long long* cur = reinterpret_cast<unsigned long long*>(smem + L.cur);
    unsigned long long* nxt = reinterpret_cast<unsigned long long*>(smem + L.nxt);
    unsigned char* wflag = reinterpret_cast<unsigned char*>(smem + L.total) + (threadIdx.x >> 6) * 64;
    (void)wflag_all;
    const int tid = threadIdx.x, lane = tid & 63;
    const int nw = (n + 63) >> 6;
    const unsigned bound = (unsigned)g.bound;
    double* relv = reinterpret_cast<double*>(ws + (size_t)blockIdx.x * ws_stride);
    uint16_t* pslot = reinterpret_cast<uint16_t*>(ws + (size_t)blockIdx.x * ws_stride + a16(sizeof(double) * n));
    wflag[lane] = 0;

    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (s < 0 || s >= n) {
            if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL);
            continue;
        }
        for (int v = tid; v < n + 1; v += K16_BLOCK) dist[v] = 0xFFFFu;
        for (int k = tid; k < nw; k += K16_BLOCK) { cur[k] = 0ull; nxt[k] = 0ull; }
        __syncthreads();
        if (tid == 0) { dist[s] = 0; cur[s >> 6] = 1ull << (s & 63); }
        __syncthreads();

        // ---- A: frontier Bellman-Ford ------------------------------------------
        for (;;) {
            if (tid == 0) { *cursor = 0; *anyflag = 0; }
            __syncthreads();
            bool any = false;
            for (;;) {
                int w = 0;
                if (lane == 0) w = atomicAdd(cursor, 1);
                w = __shfl(w, 0, 64);
                if (w >= nw) break;
                const unsigned long long m = cur[w];
                if (!m) continue;
                if (lane == 0) cur[w] = 0ull;
                const int u = (w << 6) + lane;
                const bool act = (m >> lane) & 1ull;
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
                const unsigned du = act ? dist[u] : 0xFFFFu;
                const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
                for (int base = 0; base < total; base += 64) {
                    // inactive (degree-0) lanes sit between active ones: record WHICH lane
                    // starts at each arc position, owner = last start at or before j
                    const int pos = excl - base;
                    if (deg > 0 && pos >= 0 && pos < 64) wflag[pos] = (unsigned char)(lane + 1);
                    __builtin_amdgcn_wave_barrier();
                    const int fl = wflag[lane];
                    const unsigned long long M = __ballot(fl != 0);
                    wflag[lane] = 0;
                    const unsigned long long carry_m = __ballot(deg > 0 && excl < base && incl > base);
                    const unsigned long long below = M & upto;
                    const int p = below ? 63 - __clzll((long long)below) : 0;
                    const int via = __shfl(fl, p, 64) - 1;
                    const int o = below ? via : (carry_m ? __ffsll((long long)carry_m) - 1 : 0);
                    const int ob = __shfl(boff, o, 64);
                    const unsigned od = __shfl((int)du, o, 64);
                    const int e = base + lane;
                    if (e < total) {
                        const uint32_t rec = g.oarc[ob + e];
                        const int v = (int)(rec >> 16);
                        const unsigned nd = od + (rec & 0xFFFFu);
                        if (nd <= bound && nd < dist16(dist, v) && lower16(dist, v, nd)) {
                            atomicOr(&nxt[v >> 6], 1ull << (v & 63));
                            any = true;
                        }
                    }
                }
            }
            if (any) *anyflag = 1;
            __syncthreads();
            const int again = *anyflag;
            unsigned long long* t = cur; cur = nxt; nxt = t;  // nxt (old cur) is all zero again
            __syncthreads();
            if (!again) break;
        }

        // ---- B: lat row out + parent slots (first tight in-arc) ------------------
        const double fs = g.vf[s];
        const double cs = isnan(fs) ? 1.0 : 1.0 * fs;
        double* lrow = lat_out ? lat_out + (long long)i * ld : nullptr;
        double* rrow = rel_out ? rel_out + (long long)i * ld : nullptr;
        for (int v = tid; v < n; v += K16_BLOCK) {
            const unsigned dv = dist[v];
            uint16_t slot = 0xFFFFu;
            double rv = -1.0;
            if (v == s) { slot = 0; rv = cs; }
            else if (dv != 0xFFFFu) {
                const int r0 = g.row_in[v], r1 = g.row_in[v + 1];
                for (int a = r0; a < r1; a++) {
                    const uint32_t rec = g.iarc[a];
                    if (dist[rec >> 16] + (rec & 0xFFFFu) == dv) { slot = (uint16_t)(a - r0); break; }
                }
                rv = slot != 0xFFFFu ? -g.r_in[r0 + slot] : -1.0;
            }
            pslot[v] = slot;
            relv[v] = rv;  // sign bit set = pending, holds -r of the parent arc
        }
        if (lrow) {
            for (int j = tid; j < nt; j += K16_BLOCK) {
                const int t = tgt[j];
                double Lv;
                if (t < 0 || t >= n) { raise_err(err, SHD_ROUTE_EINVAL); Lv = NAN; }
                else if (t == s) Lv = isnan(g.self_w[s]) ? NAN : 0.0 + g.self_w[s];
                else Lv = dist[t] == 0xFFFFu ? NAN : (double)dist[t];
                lrow[j] = Lv;
            }
        }
        double lmin = INFINITY;
        for (int j = tid; j < nt; j += K16_BLOCK) {
            const int t = tgt[j];
            if (t < 0 || t >= n) continue;
            if (t == s) { if (isnan(g.self_w[s])) raise_err(err, SHD_ROUTE_ENOEDGE); else lmin = fmin(lmin, 0.0 + g.self_w[s]); }
            else if (dist[t] == 0xFFFFu) raise_err(err, SHD_ROUTE_EUNREACH);
            else lmin = fmin(lmin, (double)dist[t]);
        }
        __syncthreads();
        // dist is dead: its LDS becomes parent vertex ids
        uint16_t* par = dist;
        for (int v = tid; v < n; v += K16_BLOCK) {
            const uint16_t sl = pslot[v];
            par[v] = (v == s) ? (uint16_t)s : (sl == 0xFFFFu ? (uint16_t)0xFFFFu
                                                             : (uint16_t)(g.iarc[g.row_in[v] + sl] >> 16));
        }
        __syncthreads();

        // ---- C: reliability down the tree (relv in HBM, workgroup-private) -----------
        for (;;) {
            if (tid == 0) *flag = 0;
            __syncthreads();
            int progressed = 0;
            for (int v0 = tid; v0 < n; v0 += K16_BLOCK * 4) {
                double x[4], rp[4];
                uint16_t p[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int v = v0 + q * K16_BLOCK;
                    x[q] = v < n ? relv[v] : 0.0;
                    p[q] = v < n ? par[v] : (uint16_t)0xFFFFu;
                }
#pragma unroll
                for (int q = 0; q < 4; q++)
                    rp[q] = (signbit(x[q]) && p[q] != 0xFFFFu) ? relv[p[q]] : -1.0;
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (!signbit(rp[q])) { relv[v0 + q * K16_BLOCK] = rp[q] * (-x[q]); progressed = 1; }
            }
            if (progressed) *flag = 1;
            __syncthreads();
            const int again = *flag;
            __syncthreads();
            if (!again) break;
        }

        // ---- D: rel row out + row min ------------------------------------------
        if (tid == 0) *rmin = kInfBits;
        __syncthreads();
        if (rrow) {
            for (int j = tid; j < nt; j += K16_BLOCK) {
                const int t = tgt[j];
                double Rv = NAN;
                if (t >= 0 && t < n) {
                    if (t == s) Rv = isnan(g.self_w[s]) ? NAN : cs * g.self_r[s];
                    else {
                        const double ft = g.vf[t];
                        Rv = isnan(ft) ? relv[t] : relv[t] * ft;
                    }
                }
                rrow[j] = Rv;
            }
        }
        if (row_min) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
            if (lane == 0 && lmin < INFINITY) atomicMin(rmin, as_u(lmin));
            __syncthreads();
            if (tid == 0) row_min[i] = as_d(*rmin);
        }
        __syncthreads();
    }
}

inline size_t k16_lds_bytes(int n) { return K16Layout::make(n).total + (K16_BLOCK / 64) * 64; }

}  // namespace shd
