#pragma once
// "K2": path attributes from (dist16 | parent-slot16) key rows -- the per-target part
// of _topology_computeSourcePaths (topology.c:1805-1864) and
// _topology_computePathProperties (topology.c:1407-1523):
//   lat = dist (exact integer sum), rel = ((1*f_s) * r_1 * ... * r_L) * f_t, multiplied
//   in path order from the source down the deterministic shortest-path tree,
//   the self entry = the self-loop hop, the 0 -> 1 ms fix, and the row minimum.
// One workgroup per source; relv f64[n] and parent u16[n] in LDS (10 n bytes).
#include "common.hpp"

namespace shd {

constexpr int AT_ILP = 8;  // independent elements per thread per loop trip

struct DevAttr {
    int n;
    const int* __restrict__ row_in;      // in-CSR offsets, rows sorted by (-w, u, eid)
    const uint16_t* __restrict__ col_in; // in-row neighbour u
    const double* __restrict__ r_in;     // 1 - loss of that in-arc
    const double* __restrict__ vf;
    const double* __restrict__ self_w;
    const double* __restrict__ self_r;
    unsigned long long* dbg;   // SHD_STAMPS builds: 8 words per source
};

struct AttrLayout {
    size_t relv, par, total;
    __host__ __device__ static AttrLayout make(int n) {
        AttrLayout L;
        size_t o = 32;  // small: flag, rmin
        L.relv = o; o += a16(sizeof(double) * n);
        L.par = o;  o += a16(sizeof(uint16_t) * n);
        L.total = o;
        return L;
    }
};

template <int B>
__global__ __launch_bounds__(B) void path_attr_kernel(DevAttr g, const uint32_t* __restrict__ keys, long long kld,
                                                      const int* __restrict__ src, int ns,
                                                      const int* __restrict__ tgt, int nt, long long ld,
                                                      double* __restrict__ lat_out, double* __restrict__ rel_out,
                                                      double* __restrict__ row_min, int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* flag = reinterpret_cast<int*>(smem);
    unsigned long long* rmin = reinterpret_cast<unsigned long long*>(smem + 16);
    const AttrLayout L = AttrLayout::make(g.n);
    double* relv = reinterpret_cast<double*>(smem + L.relv);
    uint16_t* par = reinterpret_cast<uint16_t*>(smem + L.par);
    const int n = g.n;
    const int tid = threadIdx.x;

    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (s < 0 || s >= n) {
            if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL);
            continue;
        }
        const uint32_t* krow = keys + (long long)i * kld;
        if (tid == 0 && g.dbg) g.dbg[(size_t)i * 8 + 0] = __builtin_amdgcn_s_memtime();
        const double fs = g.vf[s];
        const double cs = isnan(fs) ? 1.0 : 1.0 * fs;
        // parent vertex + parent-arc reliability (stored negated: sign bit = pending)
        // blocked by AT_ILP vertices per thread so the dependent global gathers overlap
        for (int v0 = tid; v0 < n; v0 += B * AT_ILP) {
            uint32_t kv[AT_ILP];
            int a[AT_ILP];
#pragma unroll
            for (int q = 0; q < AT_ILP; q++) {
                const int v = v0 + q * B;
                kv[q] = v < n ? krow[v] : 0xFFFFFFFFu;
                a[q] = v < n ? g.row_in[v] : 0;
            }
            uint16_t pu[AT_ILP];
            double pr[AT_ILP];
#pragma unroll
            for (int q = 0; q < AT_ILP; q++) {
                const bool ok = kv[q] != 0xFFFFFFFFu;
                const int aa = a[q] + (int)(kv[q] & 0xFFFFu);
                pu[q] = ok ? g.col_in[aa] : (uint16_t)0xFFFFu;
                pr[q] = ok ? g.r_in[aa] : 1.0;
            }
#pragma unroll
            for (int q = 0; q < AT_ILP; q++) {
                const int v = v0 + q * B;
                if (v >= n) break;
                if (v == s) { par[v] = (uint16_t)s; relv[v] = cs; }
                else if (kv[q] == 0xFFFFFFFFu) { par[v] = 0xFFFFu; relv[v] = -1.0; }
                else { par[v] = pu[q]; relv[v] = -pr[q]; }
            }
        }
        __syncthreads();
        if (tid == 0 && g.dbg) g.dbg[(size_t)i * 8 + 1] = __builtin_amdgcn_s_memtime();
        // level-synchronous propagation down the tree (LDS only)
        for (;;) {
            if (tid == 0 && g.dbg) g.dbg[(size_t)i * 8 + 5] += 1;
            if (tid == 0) *flag = 0;
            __syncthreads();
            int progressed = 0;
            for (int v0 = tid; v0 < n; v0 += B * AT_ILP) {
                double x[AT_ILP], rp[AT_ILP];
                uint16_t p[AT_ILP];
#pragma unroll
                for (int q = 0; q < AT_ILP; q++) {
                    const int v = v0 + q * B;
                    x[q] = v < n ? relv[v] : 0.0;
                    p[q] = v < n ? par[v] : (uint16_t)0xFFFFu;
                }
#pragma unroll
                for (int q = 0; q < AT_ILP; q++)
                    rp[q] = (signbit(x[q]) && p[q] != 0xFFFFu) ? relv[p[q]] : -1.0;
#pragma unroll
                for (int q = 0; q < AT_ILP; q++)
                    if (!signbit(rp[q])) { relv[v0 + q * B] = rp[q] * (-x[q]); progressed = 1; }
            }
            if (progressed) *flag = 1;
            __syncthreads();
            const int again = *flag;
            __syncthreads();
            if (!again) break;
        }
        if (tid == 0) *rmin = kInfBits;
        __syncthreads();
        if (tid == 0 && g.dbg) g.dbg[(size_t)i * 8 + 2] = __builtin_amdgcn_s_memtime();
        double lmin = INFINITY;
        double* lrow = lat_out ? lat_out + (long long)i * ld : nullptr;
        double* rrow = rel_out ? rel_out + (long long)i * ld : nullptr;
        for (int j0 = tid; j0 < nt; j0 += B * AT_ILP) {
            int tq[AT_ILP];
            uint32_t kt[AT_ILP];
            double ft[AT_ILP];
#pragma unroll
            for (int q = 0; q < AT_ILP; q++) {
                const int j = j0 + q * B;
                tq[q] = j < nt ? tgt[j] : s;
            }
#pragma unroll
            for (int q = 0; q < AT_ILP; q++) {
                const bool ok = tq[q] >= 0 && tq[q] < n;
                kt[q] = ok ? krow[tq[q]] : 0xFFFFFFFFu;
                ft[q] = ok ? g.vf[tq[q]] : NAN;
            }
#pragma unroll
            for (int q = 0; q < AT_ILP; q++) {
                const int j = j0 + q * B;
                if (j >= nt) break;
                const int t = tq[q];
                double Lv, Rv;
                if (t < 0 || t >= n) {
                    raise_err(err, SHD_ROUTE_EINVAL);
                    Lv = Rv = NAN;
                } else if (t == s) {  // batch path [s]: one self-loop hop (topology.c:1471-1499)
                    const double w = g.self_w[s];
                    if (isnan(w)) { raise_err(err, SHD_ROUTE_ENOEDGE); Lv = Rv = NAN; }
                    else { Lv = 0.0 + w; Rv = cs * g.self_r[s]; }
                } else if (kt[q] == 0xFFFFFFFFu) {
                    raise_err(err, SHD_ROUTE_EUNREACH);
                    Lv = Rv = NAN;
                } else {
                    Lv = (double)(kt[q] >> 16);
                    Rv = isnan(ft[q]) ? relv[t] : relv[t] * ft[q];
                }
                if (lrow) lrow[j] = Lv;
                if (rrow) rrow[j] = Rv;
                lmin = fmin(lmin, Lv);
            }
        }
        if (row_min) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
            if ((tid & 63) == 0 && lmin < INFINITY) atomicMin(rmin, as_u(lmin));
            __syncthreads();
            if (tid == 0) row_min[i] = as_d(*rmin);
        }
        __syncthreads();
        if (tid == 0 && g.dbg) g.dbg[(size_t)i * 8 + 3] = __builtin_amdgcn_s_memtime();
    }
}

}  // namespace shd
