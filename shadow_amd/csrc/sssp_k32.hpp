#pragma once
// Integer-latency SOURCE-rows kernel ("K32"), one workgroup per source, all per-source
// state in LDS.  Exact replacement for igraph_get_shortest_paths_dijkstra
// (topology.c:1756) + _topology_computePathProperties (topology.c:1407-1523) when
// every edge latency is an integer and every shortest-path latency is < 2^16 ms:
// then the reference's double left-fold sums are exact integers and u32 arithmetic
// reproduces them bit for bit.
//
// Key idea: key[v] = dist16 << 16 | slot16 where slot is the position of the relaxing
// arc in v's in-row, and in-rows are sorted by (-w, u, eid).  For tight arcs
// dist[u] = dist[v] - w, so the smallest slot among tight arcs is the engine tie rule
// argmin (dist[u], u, eid), and ONE ds_min_u32 per relaxation resolves distance and
// deterministic parent together -- no separate parent pass.
//
// LDS per source: key u32[n] | relv f64[n] (frontier queues u16[2n] overlay it during
// phase A) | par u16[n] | dedup bits u32[n/32]  =  ~14.1 n bytes.
#include "common.hpp"

namespace shd {

struct ArcRec {      // one out-arc u->v, 8 bytes, one global_load_dwordx2
    uint16_t col;    // v
    uint16_t w;      // integer latency
    uint16_t rslot;  // position of this arc in v's in-row (sorted by -w, u, eid)
    uint16_t pad;
};

struct DevK32 {
    int n;
    int bound;                           // all shortest-path latencies <= bound < 0xFFFF
    const int* __restrict__ row;         // out-CSR offsets (n+1)
    const ArcRec* __restrict__ arc;      // out-arcs
    const int* __restrict__ row_in;      // in-CSR offsets (n+1)
    const uint16_t* __restrict__ col_in; // in-row neighbour u, rows sorted by (-w, u, eid)
    const double* __restrict__ r_in;     // 1 - loss of that in-arc
    const double* __restrict__ vf;
    const double* __restrict__ self_w;
    const double* __restrict__ self_r;
    unsigned long long* dbg;             // SHD_STAMPS diagnostic builds only: 8 words per source
};

#ifdef SHD_STAMPS
#define K32_STAMP(slot) do { if (tid == 0 && g.dbg) { g.dbg[(size_t)i * 8 + (slot)] = __builtin_amdgcn_s_memtime(); } } while (0)
#define K32_COUNT(slot, x) do { if (g.dbg) atomicAdd(&g.dbg[(size_t)i * 8 + (slot)], (unsigned long long)(x)); } while (0)
#else
#define K32_STAMP(slot) do { } while (0)
#define K32_COUNT(slot, x) do { } while (0)
#endif

struct K32Layout {
    size_t key, relv, par, bits, total;
    __host__ __device__ static K32Layout make(int n) {
        K32Layout L;
        size_t o = 0;
        L.key = o;  o += a16(sizeof(uint32_t) * n);
        L.relv = o; o += a16(sizeof(double) * n);   // q0,q1 (u16 n each) overlay this
        L.par = o;  o += a16(sizeof(uint16_t) * n);
        L.bits = o; o += a16(sizeof(uint32_t) * ((n + 31) / 32));
        L.total = o;
        return L;
    }
};

template <int B>
struct K32Small {
    unsigned char wflag[B / 64][64];  // per-wave arc-window start flags
    int qnext;
    int cursor;
    int flag;
    unsigned long long rmin;
};

template <int B>
__global__ __launch_bounds__(B) void sssp_k32_kernel(DevK32 g, const int* __restrict__ src, int ns,
                                                     const int* __restrict__ tgt, int nt, long long ld,
                                                     double* __restrict__ lat_out, double* __restrict__ rel_out,
                                                     double* __restrict__ row_min, int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr size_t kSm = (sizeof(K32Small<B>) + 15) & ~size_t(15);
    K32Small<B>* sm = reinterpret_cast<K32Small<B>*>(smem);
    const int n = g.n;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    unsigned char* wflag = sm->wflag[tid >> 6];
    wflag[lane] = 0;
    const K32Layout L = K32Layout::make(n);
    char* base = smem + kSm;
    uint32_t* key = reinterpret_cast<uint32_t*>(base + L.key);
    double* relv = reinterpret_cast<double*>(base + L.relv);
    uint16_t* q0 = reinterpret_cast<uint16_t*>(base + L.relv);
    uint16_t* q1 = q0 + n;
    uint16_t* par = reinterpret_cast<uint16_t*>(base + L.par);
    uint32_t* bits = reinterpret_cast<uint32_t*>(base + L.bits);
    const int nwords = (n + 31) >> 5;
    const uint32_t bound = (uint32_t)g.bound;

    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (s < 0 || s >= n) {
            if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL);
            continue;
        }
        for (int v = tid; v < n; v += B) key[v] = 0xFFFFFFFFu;
        for (int k = tid; k < nwords; k += B) bits[k] = 0u;
        __syncthreads();
        if (tid == 0) {
            key[s] = 0u;
            q0[0] = (uint16_t)s;
        }
        uint16_t* qc = q0;
        uint16_t* qn = q1;
        int qlen = 1;
        __syncthreads();
        K32_STAMP(0);

        // ---- phase A: frontier Bellman-Ford on packed (dist, slot) keys ----------
        // Each wave grabs 64 frontier vertices at a time (LDS cursor) and expands their
        // arcs 64 at a time, load-balanced with no block barrier: wave scan of the
        // degrees, then each arc lane finds its owner vertex from the window's
        // start-position mask (ballot of LDS flags) and two popcounts.
        while (qlen > 0) {
            if (tid == 0) { sm->qnext = 0; sm->cursor = 0; }
            __syncthreads();
            for (;;) {
                int start = 0;
                if (lane == 0) start = atomicAdd(&sm->cursor, 64);
                start = __shfl(start, 0, 64);
                if (start >= qlen) break;
                const int k = start + lane;
                int u = 0, beg = 0, deg = 0;
                if (k < qlen) {
                    u = qc[k];
                    atomicAnd(&bits[u >> 5], ~(1u << (u & 31)));
                    beg = g.row[u];
                    deg = g.row[u + 1] - beg;
                }
                int incl = deg;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int y = __shfl_up(incl, d, 64);
                    if (lane >= d) incl += y;
                }
                const int total = __shfl(incl, 63, 64);
                if (lane == 0) K32_COUNT(5, total);
                const int excl = incl - deg;
                const int boff = beg - excl;
                const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
                for (int base = 0; base < total; base += 64) {
                    const int pos = excl - base;
                    if (deg > 0 && pos >= 0 && pos < 64) wflag[pos] = 1;
                    __builtin_amdgcn_wave_barrier();
                    const unsigned long long M = __ballot(wflag[lane] != 0);
                    wflag[lane] = 0;
                    const int l0 = __popcll(__ballot(incl <= base));
                    const int o = (l0 + __popcll(M & upto) - (int)(M & 1ull)) & 63;
                    const int ob = __shfl(boff, o, 64);
                    const int ou = __shfl(u, o, 64);
                    const int e = base + lane;
                    bool push = false;
                    int v = 0;
                    if (e < total) {
                        const ArcRec rec = g.arc[ob + e];
                        const uint32_t nd = (key[ou] >> 16) + rec.w;
                        v = rec.col;
                        const uint32_t cand = (nd << 16) | rec.rslot;
                        if (nd <= bound && cand < key[v]) {  // nd > bound can never be final
                            const uint32_t old = atomicMin(&key[v], cand);
                            if (nd < (old >> 16)) {  // distance improved: (re)expand v
                                const uint32_t m = 1u << (v & 31);
                                push = !(atomicOr(&bits[v >> 5], m) & m);
                            }
                        }
                    }
                    // wave-aggregated enqueue
                    const unsigned long long pm = __ballot(push);
                    if (pm) {
                        int qb = 0;
                        const int leader = __ffsll((long long)pm) - 1;
                        if (lane == leader) qb = atomicAdd(&sm->qnext, __popcll(pm));
                        qb = __shfl(qb, leader, 64);
                        if (push) qn[qb + __popcll(pm & ((1ull << lane) - 1ull))] = (uint16_t)v;
                    }
                }
            }
            __syncthreads();
            qlen = sm->qnext;
            uint16_t* t = qc; qc = qn; qn = t;
            if (tid == 0) K32_COUNT(6, 1);
            __syncthreads();
        }
        K32_STAMP(1);

        // ---- phase B: parent vertex from the slot; relv init (queues are dead) ----
        const double fs = g.vf[s];
        const double cs = isnan(fs) ? 1.0 : 1.0 * fs;
        for (int v = tid; v < n; v += B) {
            const uint32_t kv = key[v];
            uint16_t p = 0xFFFFu;
            if (v == s) p = (uint16_t)s;
            else if (kv != 0xFFFFFFFFu) p = g.col_in[g.row_in[v] + (kv & 0xFFFFu)];
            par[v] = p;
            relv[v] = (v == s) ? cs : -1.0;
        }
        __syncthreads();
        K32_STAMP(2);

        // ---- phase C: reliability down the tree, level-synchronous, LDS only ------
        for (;;) {
            if (tid == 0) sm->flag = 0;
            __syncthreads();
            int progressed = 0;
            for (int v = tid; v < n; v += B) {
                if (relv[v] >= 0.0) continue;
                const uint16_t p = par[v];
                if (p == 0xFFFFu) continue;
                const double ru = relv[p];
                if (ru >= 0.0) {
                    relv[v] = ru * g.r_in[g.row_in[v] + (key[v] & 0xFFFFu)];
                    progressed = 1;
                }
            }
            if (progressed) sm->flag = 1;
            __syncthreads();
            const int again = sm->flag;
            __syncthreads();
            if (!again) break;
            if (tid == 0) K32_COUNT(7, 1);
        }
        K32_STAMP(3);

        // ---- phase D: row output + row min -----------------------------------
        if (tid == 0) sm->rmin = kInfBits;
        __syncthreads();
        double lmin = INFINITY;
        double* lrow = lat_out ? lat_out + (long long)i * ld : nullptr;
        double* rrow = rel_out ? rel_out + (long long)i * ld : nullptr;
        for (int j = tid; j < nt; j += B) {
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
                } else {
                    Lv = 0.0 + ws_;
                    Rv = cs * g.self_r[s];
                }
            } else {
                const uint32_t kt = key[t];
                if (kt == 0xFFFFFFFFu) {
                    raise_err(err, SHD_ROUTE_EUNREACH);
                    Lv = Rv = NAN;
                } else {
                    Lv = (double)(kt >> 16);
                    const double ft = g.vf[t];
                    Rv = isnan(ft) ? relv[t] : relv[t] * ft;
                }
            }
            if (lrow) lrow[j] = Lv;
            if (rrow) rrow[j] = Rv;
            lmin = fmin(lmin, Lv);
        }
        if (row_min) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
            if ((tid & 63) == 0 && lmin < INFINITY) atomicMin(&sm->rmin, as_u(lmin));
            __syncthreads();
            if (tid == 0) row_min[i] = as_d(sm->rmin);
        }
        __syncthreads();
        K32_STAMP(4);
    }
}

template <int B>
constexpr size_t k32_small_bytes() { return (sizeof(K32Small<B>) + 15) & ~size_t(15); }

}  // namespace shd
