#pragma once
// K3 direct paths, self paths, K5 min reduce, K4 blocked min-plus Floyd-Warshall.
#include "common.hpp"
namespace shd {
// K3: direct paths from dense per-pair latency / reliability (complete graphs).
// One workgroup per source row; each lane takes two adjacent targets per step, so a sorted
// contiguous target list (the attached set of a complete graph) streams W, R and the
// outputs as 16-byte accesses (loads streamed once: nontemporal), two steps in flight;
// any other list falls back to 8-byte accesses per target.
typedef double k3_d2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(kBlock) void direct_rows_kernel(
    int n, const double* __restrict__ W, const double* __restrict__ R, const double* __restrict__ vf,
    const int* __restrict__ src, int ns, const int* __restrict__ tgt, int nt, long long ld,
    double* __restrict__ lat_out, double* __restrict__ rel_out, double* __restrict__ row_min,
    int* __restrict__ err) {
    __shared__ unsigned long long rmin;
    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (threadIdx.x == 0) rmin = kInfBits;
        __syncthreads();
        double lmin = INFINITY;
        const bool sok = s >= 0 && s < n;
        const double fs = sok ? vf[s] : NAN;
        const long long sb = (long long)(sok ? s : 0) * n;
        double* lrow = lat_out ? lat_out + (long long)i * ld : nullptr;
        double* rrow = rel_out ? rel_out + (long long)i * ld : nullptr;
        // (lat, rel) of target t from its w, r and vertex factor (topology.c:1877-1927)
        auto entry = [&](int t, double w, double r, double ft, double& Lv, double& Rv) __attribute__((always_inline)) {
            Lv = NAN; Rv = NAN;
            if (!sok || t < 0 || t >= n) raise_err(err, SHD_ROUTE_EINVAL);
            else if (isnan(w)) raise_err(err, SHD_ROUTE_ENOEDGE);
            else {
                double Rr = 1.0;
                if (!isnan(fs)) Rr *= fs;
                if (!isnan(ft)) Rr *= ft;
                Lv = 0.0 + w;
                Rv = Rr * r;
            }
            lmin = fmin(lmin, Lv);
        };
        const bool out_even = !(((uintptr_t)lrow | (uintptr_t)rrow) & 8);
#pragma unroll 2
        for (int j0 = 2 * (int)threadIdx.x; j0 < nt; j0 += 2 * kBlock) {
            const bool two = j0 + 1 < nt;
            const int t0 = tgt[j0], t1 = two ? tgt[j0 + 1] : -1;
            double w0 = NAN, w1 = NAN, r0 = NAN, r1 = NAN, f0 = NAN, f1 = NAN;
            if (sok && two && t1 == t0 + 1 && t0 >= 0 && t1 < n && !((sb + t0) & 1) && !(t0 & 1)) {
                const k3_d2 w = __builtin_nontemporal_load(reinterpret_cast<const k3_d2*>(W + sb + t0));
                const k3_d2 r = __builtin_nontemporal_load(reinterpret_cast<const k3_d2*>(R + sb + t0));
                const k3_d2 f = *reinterpret_cast<const k3_d2*>(vf + t0);
                w0 = w.x; w1 = w.y; r0 = r.x; r1 = r.y; f0 = f.x; f1 = f.y;
            } else {
                if (sok && t0 >= 0 && t0 < n) { w0 = W[sb + t0]; r0 = R[sb + t0]; f0 = vf[t0]; }
                if (sok && t1 >= 0 && t1 < n) { w1 = W[sb + t1]; r1 = R[sb + t1]; f1 = vf[t1]; }
            }
            double L0, R0, L1 = NAN, R1 = NAN;
            entry(t0, w0, r0, f0, L0, R0);
            if (two) entry(t1, w1, r1, f1, L1, R1);
            if (two && out_even) {  // (j0 is even: the pair is 16-byte aligned with the row)
                if (lrow) __builtin_nontemporal_store(k3_d2{L0, L1}, reinterpret_cast<k3_d2*>(lrow + j0));
                if (rrow) __builtin_nontemporal_store(k3_d2{R0, R1}, reinterpret_cast<k3_d2*>(rrow + j0));
            } else {
                if (lrow) { __builtin_nontemporal_store(L0, lrow + j0); if (two) __builtin_nontemporal_store(L1, lrow + j0 + 1); }
                if (rrow) { __builtin_nontemporal_store(R0, rrow + j0); if (two) __builtin_nontemporal_store(R1, rrow + j0 + 1); }
            }
        }
        if (row_min) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
            if ((threadIdx.x & 63) == 0 && lmin < INFINITY) atomicMin(&rmin, as_u(lmin));
            __syncthreads();
            if (threadIdx.x == 0) row_min[i] = as_d(rmin);
        }
        __syncthreads();
    }
}

// Self path: first minimum-latency incident edge in igraph incident order
// (ascending neighbour, the self-loop at its own position), used twice.
__global__ void self_kernel(DevGraph g, const int* __restrict__ vs, int nv, double* __restrict__ lat,
                            double* __restrict__ rel, int* __restrict__ err) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nv) return;
    const int v = vs[k];
    if (v < 0 || v >= g.n) { raise_err(err, SHD_ROUTE_EINVAL); lat[k] = rel[k] = NAN; return; }
    double mn = 0.0, rm = 0.0;
    bool any = false;
    const double sw = g.self_w[v];
    bool self_done = isnan(sw);
    const int e1 = g.row[v + 1];
    for (int a = g.row[v]; a <= e1; a++) {
        // interleave the self-loop before the first neighbour > v
        if (!self_done && (a == e1 || g.col[a] > v)) {
            if (mn == 0 || sw < mn) { mn = sw; rm = g.self_r[v]; }
            self_done = true; any = true;
        }
        if (a == e1) break;
        const double w = g.w[a];
        if (mn == 0 || w < mn) { mn = w; rm = g.r[a]; }
        any = true;
    }
    if (!any) { raise_err(err, SHD_ROUTE_ENOEDGE); lat[k] = rel[k] = NAN; return; }
    lat[k] = 2.0f * mn;
    rel[k] = rm * rm;
}

// K5: device-wide min of non-negative doubles; *out must hold +inf/0xFF.. bits first.
__global__ __launch_bounds__(kBlock) void min_reduce_kernel(const double* __restrict__ vals, long long count,
                                                            unsigned long long* __restrict__ out) {
    double m = INFINITY;
    for (long long k = blockIdx.x * (long long)kBlock + threadIdx.x; k < count;
         k += (long long)gridDim.x * kBlock)
        m = fmin(m, vals[k]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = fmin(m, __shfl_xor(m, d, 64));
    if ((threadIdx.x & 63) == 0 && m < INFINITY) atomicMin(out, as_u(m));
}

// K5 for up to kMinOneBlock values: one workgroup reduces and stores the result itself
// (no clearing memset, no atomics): the same bits as min_reduce_kernel after a 0xFF fill.
constexpr long long kMinOneBlock = 1 << 20;
__global__ __launch_bounds__(1024) void min_reduce_block_kernel(const double* __restrict__ vals, long long count,
                                                                unsigned long long* __restrict__ out) {
    __shared__ double wm[16];
    double m = INFINITY;
    for (long long k = threadIdx.x; k < count; k += 1024) m = fmin(m, vals[k]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = fmin(m, __shfl_xor(m, d, 64));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = wm[0];
        for (int k = 1; k < 16; k++) r = fmin(r, wm[k]);
        *out = r < INFINITY ? as_u(r) : ~0ull;
    }
}

// Blocked min-plus Floyd-Warshall (K4), 32x32 tiles of doubles in LDS.
constexpr int kT = 32;
__global__ __launch_bounds__(kT * 8) void fw_diag_kernel(double* d, int n, int k0) {
    __shared__ double t[kT][kT + 1];
    const int tx = threadIdx.x & (kT - 1), ty0 = threadIdx.x / kT;
    for (int y = ty0; y < kT; y += 8) {
        int gi = k0 + y, gj = k0 + tx;
        t[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
    }
    __syncthreads();
    for (int k = 0; k < kT; k++) {
        for (int y = ty0; y < kT; y += 8) {
            double c = t[y][k] + t[k][tx];
            if (c < t[y][tx]) t[y][tx] = c;
        }
        __syncthreads();
    }
    for (int y = ty0; y < kT; y += 8) {
        int gi = k0 + y, gj = k0 + tx;
        if (gi < n && gj < n) d[(long long)gi * n + gj] = t[y][tx];
    }
}
__global__ __launch_bounds__(kT * 8) void fw_panel_kernel(double* d, int n, int k0) {
    // blockIdx.x = other tile index b (skip diagonal), blockIdx.y = 0 row panel, 1 col panel
    __shared__ double dg[kT][kT + 1];
    __shared__ double t[kT][kT + 1];
    const int nb = (n + kT - 1) / kT;
    int b = blockIdx.x;
    const int kb = k0 / kT;
    if (b >= kb) b++;
    if (b >= nb) return;
    const int tx = threadIdx.x & (kT - 1), ty0 = threadIdx.x / kT;
    const bool rowp = blockIdx.y == 0;  // tile (kb, b)
    const int bi = rowp ? k0 : b * kT, bj = rowp ? b * kT : k0;
    for (int y = ty0; y < kT; y += 8) {
        int gi = k0 + y, gj = k0 + tx;
        dg[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
        gi = bi + y; gj = bj + tx;
        t[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
    }
    __syncthreads();
    for (int k = 0; k < kT; k++) {
        for (int y = ty0; y < kT; y += 8) {
            double c = rowp ? dg[y][k] + t[k][tx] : t[y][k] + dg[k][tx];
            if (c < t[y][tx]) t[y][tx] = c;
        }
        __syncthreads();
    }
    for (int y = ty0; y < kT; y += 8) {
        int gi = bi + y, gj = bj + tx;
        if (gi < n && gj < n) d[(long long)gi * n + gj] = t[y][tx];
    }
}
__global__ __launch_bounds__(kT * 8) void fw_rest_kernel(double* d, int n, int k0) {
    __shared__ double rp[kT][kT + 1];  // row panel tile (k, bj)
    __shared__ double cp[kT][kT + 1];  // col panel tile (bi, k)
    const int bi = blockIdx.y * kT, bj = blockIdx.x * kT;
    if (bi == k0 || bj == k0) return;
    const int tx = threadIdx.x & (kT - 1), ty0 = threadIdx.x / kT;
    double acc[kT / 8];
    for (int q = 0; q < kT / 8; q++) {
        int y = ty0 + 8 * q;
        int gi = k0 + y, gj = bj + tx;
        rp[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
        gi = bi + y; gj = k0 + tx;
        cp[y][tx] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
        gi = bi + y; gj = bj + tx;
        acc[q] = (gi < n && gj < n) ? d[(long long)gi * n + gj] : INFINITY;
    }
    __syncthreads();
    for (int k = 0; k < kT; k++) {
        const double b = rp[k][tx];
#pragma unroll
        for (int q = 0; q < kT / 8; q++) {
            double c = cp[ty0 + 8 * q][k] + b;
            acc[q] = c < acc[q] ? c : acc[q];
        }
    }
    for (int q = 0; q < kT / 8; q++) {
        int gi = bi + ty0 + 8 * q, gj = bj + tx;
        if (gi < n && gj < n) d[(long long)gi * n + gj] = acc[q];
    }
}

}  // namespace shd
