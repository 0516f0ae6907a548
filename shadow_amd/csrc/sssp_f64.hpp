#pragma once
// Generic f64 SOURCE-rows kernel (any positive double latencies).
#include "common.hpp"
namespace shd {
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

}  // namespace shd
