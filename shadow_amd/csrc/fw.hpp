#pragma once
// K4: blocked min-plus Floyd-Warshall for dense all-pairs tables,
// and the SOURCE-row latency / reliability of the path it implies.
//
// No reference equivalent in Shadow 1.14: a complete graph never takes shortest paths
// there (topology.c:1321-1323, 2019-2021: direct mode, K3).  K4 is the dense
// alternative to per-source SSSP; its rows follow the same SOURCE(s,.) semantics as
// shd_route_rows (topology.c:1407-1523, 1655-1875): lat is the left-fold path sum,
// rel the source-first product along the engine tie rule's shortest-path tree.
//
// Integer latencies only (FW adds two subpath sums, so it is not a left fold: exact only
// when every sum is an exact integer).  Distances are u16 (bound < 0xFFFF), two per
// 32-bit lane, so a relaxation of two pairs is one v_pk_add_u16 (clamped: 0xFFFF stays
// "no path") + one v_pk_min_u16.  VALU-bound by design: min-plus is not a multiply-add
// contraction, so MFMA does not apply.
//
//  fw_init     D[i][j] = w(i,j) (0 on the diagonal, 0xFFFF = no edge), padded to 64
//  fw_diag     the first pivot tile: 64 dependent steps in LDS (one workgroup); every later
//              pivot tile is closed by its own workgroup inside the previous fw_rest launch
//  fw_panel    row / column panel tiles: D* (x) P and P (x) D* with the closed pivot
//              tile D* -- one tropical product each, no dependent steps
//  fw_rest     every other tile: C = min(C, colpanel (x) rowpanel)
//  The tropical product of two 64x64 u16 tiles: 256 threads, 4 rows x 4 columns each,
//  A stored transposed in LDS so a thread's 4 rows at step k are one 8-byte read.
//
//  fw_inlist   once per graph: every vertex's in-arcs sorted by the tie-rule key
//              (0xFFFF - w) << 16 | u, with a start index per small threshold
//  fw_parent   per (source s, vertex v): the tie-rule parent among the tight in-arcs
//              (D[s][u] + w(u,v) == D[s][v]): largest w, then smallest u -- the first
//              tight arc of v's sorted in-list, scanned from the first arc with w <= D[s][v]
//  fw_rows     per source: reliability top-down in distance order (parents have smaller
//              distance: w >= 1), rel[v] = rel[p] * r(p,v), f_t last; lat / rel rows out
#include "common.hpp"

namespace shd {

#ifndef FW_TILE
#define FW_TILE 64  // (128 with 8 x 8 blocks measured 5.5 ms against 3.9: 2 waves per SIMD, 128-step pivots)
#endif
constexpr int FW_T = FW_TILE;  // tile edge (64: 4 x 4 per thread, 128: 8 x 8)

typedef unsigned short fw_us2 __attribute__((ext_vector_type(2)));

__device__ inline uint32_t fw_pkadd(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(__builtin_bit_cast(fw_us2, a),
                                                                      __builtin_bit_cast(fw_us2, b)));
}
__device__ inline uint32_t fw_pkmin(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(fw_us2, a),
                                                                  __builtin_bit_cast(fw_us2, b)));
}

// D (Np x Np u16) from the dense W (n x n f64, NaN = no edge)
__global__ void fw_init_kernel(const double* __restrict__ W, int n, int np, uint16_t* __restrict__ D) {
    const long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (k >= (long long)np * np) return;
    const int i = (int)(k / np), j = (int)(k % np);
    uint16_t d = 0xFFFFu;
    if (i == j) d = 0;
    else if (i < n && j < n) {
        const double w = W[(long long)i * n + j];
        if (!isnan(w)) d = w < 65535.0 ? (uint16_t)w : (uint16_t)0xFFFFu;  // >= the bound: never on a path
    }
    D[k] = d;
}

// R consecutive u16 as R/2 packed words (8 or 16 bytes: one LDS or global access)
template <int H>
__device__ inline void fw_ld(const uint16_t* p, uint32_t (&v)[H]) {
    if constexpr (H == 2) {
        const uint2 x = *reinterpret_cast<const uint2*>(p);
        v[0] = x.x; v[1] = x.y;
    } else {
        static_assert(H == 4, "4 or 8 columns per thread");
        const uint4 x = *reinterpret_cast<const uint4*>(p);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
}
template <int H>
__device__ inline void fw_st(uint16_t* p, const uint32_t (&v)[H]) {
    if constexpr (H == 2) *reinterpret_cast<uint2*>(p) = make_uint2(v[0], v[1]);
    else *reinterpret_cast<uint4*>(p) = make_uint4(v[0], v[1], v[2], v[3]);
}

// One T x T tile product C = min(C, A (x) B); At is A transposed ([k][i]), B is [k][j].
// 256 threads as 16 x 16, each an R x R block (R = T / 16: rows R r.., columns R c..) held
// as R x R/2 packed column pairs.  Per k: one R-wide read of A's column and of B's row
// (8- or 16-byte LDS reads) for R^2 relaxations.
#ifndef FW_PIPE
#define FW_PIPE 0  // (round 6, FW_PIPE 1 / 2 / 3: C5 table 2.88 / 2.88 / 2.88 ms against 2.80-2.84 off)
#endif
// one step k of the product: per row the adds into temporaries before the mins (an op_sel'd
// add followed directly by its dependent min costs an s_nop)
template <int R, int H>
__device__ inline void fw_step(const uint32_t (&av)[H], const uint32_t (&bv)[H], uint32_t (&acc)[R][H]) {
#pragma unroll
    for (int i = 0; i < R; i++) {
        // a row value broadcast to both halves is a shuffle the packed add takes as an
        // op_sel modifier: no instruction of its own
        const fw_us2 x = __builtin_bit_cast(fw_us2, av[i >> 1]);
        const fw_us2 a2 = (i & 1) ? __builtin_shufflevector(x, x, 1, 1) : __builtin_shufflevector(x, x, 0, 0);
        uint32_t t[H];
#pragma unroll
        for (int h = 0; h < H; h++)
            t[h] = __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(a2, __builtin_bit_cast(fw_us2, bv[h])));
#pragma unroll
        for (int h = 0; h < H; h++) acc[i][h] = fw_pkmin(acc[i][h], t[h]);
    }
}
template <int T>
__device__ inline void fw_tile_product(const uint16_t* At, const uint16_t* Bt, uint32_t (&acc)[T / 16][T / 32], int r, int c) {
    constexpr int R = T / 16, H = R / 2;
    if constexpr (FW_PIPE > 0) {
        // (round 6, measured and off) LDS reads FW_PIPE steps ahead in a ring of FW_PIPE + 1
        // register sets, the loop unrolled in full, and a scheduling barrier between a step's
        // reads and its compute: the compiler's own schedule of the loop below merges two
        // steps' reads into one ds_read2 right before an lgkmcnt(0) wait and its use, but the
        // other three waves of the SIMD already cover that latency: no gain
        constexpr int P = FW_PIPE, NB = FW_PIPE + 1;
        uint32_t av[NB][H], bv[NB][H];
#pragma unroll
        for (int k = 0; k < P; k++) {
            fw_ld<H>(At + k * T + R * r, av[k]);
            fw_ld<H>(Bt + k * T + R * c, bv[k]);
        }
#pragma unroll
        for (int k = 0; k < T; k++) {
            if (k + P < T) {
                fw_ld<H>(At + (k + P) * T + R * r, av[(k + P) % NB]);
                fw_ld<H>(Bt + (k + P) * T + R * c, bv[(k + P) % NB]);
            }
            __builtin_amdgcn_sched_barrier(0);
            fw_step<R, H>(av[k % NB], bv[k % NB], acc);
        }
        return;
    }
    // software-pipelined LDS reads (step k + 1's in flight while step k computes), and per
    // row the adds into temporaries before the mins (an op_sel'd add followed directly by
    // its dependent min costs an s_nop)
    uint32_t av[H], bv[H];
    fw_ld<H>(At + R * r, av);
    fw_ld<H>(Bt + R * c, bv);
#pragma unroll 4
    for (int k = 0; k < T; k++) {
        const int kn = k + 1 < T ? k + 1 : k;
        uint32_t an[H], bn[H];
        fw_ld<H>(At + kn * T + R * r, an);
        fw_ld<H>(Bt + kn * T + R * c, bn);
        // a row value broadcast to both halves is a shuffle the packed add takes as an
        // op_sel modifier: no instruction of its own
#pragma unroll
        for (int i = 0; i < R; i++) {
            const fw_us2 x = __builtin_bit_cast(fw_us2, av[i >> 1]);
            const fw_us2 a2 = (i & 1) ? __builtin_shufflevector(x, x, 1, 1) : __builtin_shufflevector(x, x, 0, 0);
            uint32_t t[H];
#pragma unroll
            for (int h = 0; h < H; h++)
                t[h] = __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(a2, __builtin_bit_cast(fw_us2, bv[h])));
#pragma unroll
            for (int h = 0; h < H; h++) acc[i][h] = fw_pkmin(acc[i][h], t[h]);
        }
#pragma unroll
        for (int h = 0; h < H; h++) { av[h] = an[h]; bv[h] = bn[h]; }
    }
}

// tile (ti, tj) of D <-> registers of the thread's R x R block
template <int T>
__device__ inline void fw_load_block(const uint16_t* D, int np, int ti, int tj, int r, int c, uint32_t (&acc)[T / 16][T / 32]) {
    constexpr int R = T / 16;
#pragma unroll
    for (int i = 0; i < R; i++) fw_ld<R / 2>(D + (long long)(ti * T + R * r + i) * np + tj * T + R * c, acc[i]);
}
template <int T>
__device__ inline void fw_store_block(uint16_t* D, int np, int ti, int tj, int r, int c, const uint32_t (&acc)[T / 16][T / 32]) {
    constexpr int R = T / 16;
#pragma unroll
    for (int i = 0; i < R; i++) fw_st<R / 2>(D + (long long)(ti * T + R * r + i) * np + tj * T + R * c, acc[i]);
}
// a global tile into LDS, [row][col] (transpose = false) or [col][row]
template <int T>
__device__ inline void fw_stage(const uint16_t* D, int np, int ti, int tj, uint16_t* L, bool transpose) {
    if (!transpose) {
        for (int q = threadIdx.x; q < T * T / 4; q += 256) {
            const int row = q / (T / 4), c4 = (q % (T / 4)) * 4;
            *reinterpret_cast<uint2*>(L + row * T + c4) =
                *reinterpret_cast<const uint2*>(D + (long long)(ti * T + row) * np + tj * T + c4);
        }
        return;
    }
    // transposed: a wave's lanes take 64 consecutive rows of one 4-column strip, so the
    // 2-byte LDS writes of a wave land on consecutive addresses (lanes of one row would all
    // write one bank: 16-way conflicts)
    for (int q = threadIdx.x; q < T * T / 4; q += 256) {
        const int row = q % T, c4 = (q / T) * 4;
        const uint2 v = *reinterpret_cast<const uint2*>(D + (long long)(ti * T + row) * np + tj * T + c4);
        L[(c4 + 0) * T + row] = (uint16_t)(v.x & 0xFFFFu);
        L[(c4 + 1) * T + row] = (uint16_t)(v.x >> 16);
        L[(c4 + 2) * T + row] = (uint16_t)(v.y & 0xFFFFu);
        L[(c4 + 3) * T + row] = (uint16_t)(v.y >> 16);
    }
}

// Closing a pivot tile: T dependent steps D[i][j] = min(D[i][j], D[i][k] + D[k][j]) on the
// thread blocks x (registers) with the tile mirrored in L (row-major, staged and synced).
// Step k reads row k and column k, which step k leaves unchanged (D[k][k] = 0:
// min(D[i][k], D[i][k] + 0) = D[i][k]), so its writes need no barrier before them: one
// barrier per step (writes of step k before the reads of step k + 1).  The thread's own
// block lives in registers across the steps; LDS carries its updates for the other
// threads' column-k / row-k reads.
template <int T>
__device__ inline void fw_close(uint16_t* L, uint32_t (&x)[T / 16][T / 32], int r, int c) {
    constexpr int R = T / 16, H = R / 2;
    for (int k = 0; k < T; k++) {
        fw_us2 col[R];
#pragma unroll
        for (int i = 0; i < R; i++) {
            const unsigned short y = L[(R * r + i) * T + k];
            col[i] = fw_us2{y, y};
        }
        uint32_t rowk[H];
        fw_ld<H>(L + k * T + R * c, rowk);
#pragma unroll
        for (int i = 0; i < R; i++) {
#pragma unroll
            for (int h = 0; h < H; h++)
                x[i][h] = fw_pkmin(x[i][h], __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(
                                                                            col[i], __builtin_bit_cast(fw_us2, rowk[h]))));
            fw_st<H>(L + (R * r + i) * T + R * c, x[i]);
        }
        __syncthreads();
    }
}

// pivot tile kb on its own (the first pivot; later pivots are closed inside fw_rest)
template <int T>
__global__ __launch_bounds__(256) void fw_diag_kernel(uint16_t* __restrict__ D, int np, int kb) {
    constexpr int R = T / 16, H = R / 2;
    __shared__ __attribute__((aligned(16))) uint16_t L[T * T];
    const int r = threadIdx.x / 16, c = threadIdx.x % 16;
    fw_stage<T>(D, np, kb, kb, L, false);
    __syncthreads();
    uint32_t x[R][H];
#pragma unroll
    for (int i = 0; i < R; i++) fw_ld<H>(L + (R * r + i) * T + R * c, x[i]);
    fw_close<T>(L, x, r, c);
    fw_store_block<T>(D, np, kb, kb, r, c, x);
}

// panels of pivot kb: blockIdx.y = 0 row panel (kb, b), 1 column panel (b, kb), b != kb
template <int T>
__global__ __launch_bounds__(256) void fw_panel_kernel(uint16_t* __restrict__ D, int np, int kb) {
    __shared__ __attribute__((aligned(16))) uint16_t At[T * T];
    __shared__ __attribute__((aligned(16))) uint16_t Bt[T * T];
    const int nb = np / T;
    int b = blockIdx.x;
    if (b >= kb) b++;
    if (b >= nb) return;
    const int r = threadIdx.x / 16, c = threadIdx.x % 16;
    const bool rowp = blockIdx.y == 0;
    const int ti = rowp ? kb : b, tj = rowp ? b : kb;
    uint32_t acc[T / 16][T / 32];
    fw_load_block<T>(D, np, ti, tj, r, c, acc);
    // row panel: C = D* (x) C (A = pivot, B = the panel); column panel: C = C (x) D*
    fw_stage<T>(D, np, rowp ? kb : ti, rowp ? kb : tj, At, true);
    fw_stage<T>(D, np, rowp ? ti : kb, rowp ? tj : kb, Bt, false);
    __syncthreads();
    fw_tile_product<T>(At, Bt, acc, r, c);
    fw_store_block<T>(D, np, ti, tj, r, c, acc);
}

// every tile (i, j), i, j != kb: C = min(C, D[i][kb] (x) D[kb][j]).  The workgroup of tile
// (kb + 1, kb + 1) -- dispatched first -- then closes it as the next pivot tile while the
// other tiles of this launch run, so the serial pivot steps leave the critical path
template <int T>
__global__ __launch_bounds__(256) void fw_rest_kernel(uint16_t* __restrict__ D, int np, int kb) {
    constexpr int R = T / 16, H = R / 2;
    __shared__ __attribute__((aligned(16))) uint16_t At[T * T];
    __shared__ __attribute__((aligned(16))) uint16_t Bt[T * T];
    const int nb = np / T;
    int by = blockIdx.y, bx = blockIdx.x;
    // swap block (0, 0) with the next pivot's block (kb, kb) (tile (kb + 1, kb + 1))
    if (kb + 1 < nb) {
        if (bx == 0 && by == 0) bx = by = kb;
        else if (bx == kb && by == kb) bx = by = 0;
    }
    int ti = by, tj = bx;
    if (ti >= kb) ti++;
    if (tj >= kb) tj++;
    if (ti >= nb || tj >= nb) return;
    const int r = threadIdx.x / 16, c = threadIdx.x % 16;
    // C's loads are issued first: their latency overlaps the panel staging and its barrier
    uint32_t acc[T / 16][T / 32];
    fw_load_block<T>(D, np, ti, tj, r, c, acc);
    fw_stage<T>(D, np, ti, kb, At, true);
    fw_stage<T>(D, np, kb, tj, Bt, false);
    __syncthreads();
    fw_tile_product<T>(At, Bt, acc, r, c);
    if (ti == kb + 1 && tj == kb + 1) {
        __syncthreads();  // every thread's product is done with At
#pragma unroll
        for (int i = 0; i < R; i++) fw_st<H>(At + (R * r + i) * T + R * c, acc[i]);
        __syncthreads();
        fw_close<T>(At, acc, r, c);
    }
    fw_store_block<T>(D, np, ti, tj, r, c, acc);
}

// fw_rest with the next pivot's panels fused in (one launch per pivot instead of a panel and
// a rest launch).  1-D grid of (nb - 1)^2 workgroups: workgroup 0 takes the next pivot tile
// (pn, pn) = (kb + 1, kb + 1), applies pivot kb, closes it and publishes it (stores drained,
// agent release, flag[pn]); the next (nb - 2)^2 take the tiles outside rows and columns kb, pn;
// the next 2 (nb - 2) take row pn and column pn: pivot kb's update, then -- once flag[pn] is
// up (agent acquire) -- the panel product with the closed pivot (row: C = D* (x) C, column:
// C = C (x) D*), exactly fw_panel_kernel's work for pivot pn; the last two take tiles
// (pn, kb) and (kb, pn), pivot kb's own panels, which pivot kb leaves as they are: the panel
// product only.  These are dispatched last, so the pivot's closing workgroup (dispatched
// first) has long finished when they wait.  The last pivot (pn = nb) has no next pivot:
// (nb - 1)^2 plain rest tiles only.
// one tile of fw_restp: role 0 plain, 1 the next pivot, 2 / 3 row / column panel of pn
// after pivot kb's update, 4 / 5 the same without it (tiles of pivot kb's own panels)
template <int T>
__device__ inline void fw_restp_tile(uint16_t* __restrict__ D, int np, int kb, int* __restrict__ flag, int ti, int tj,
                                     int role, uint16_t* At, uint16_t* Bt, int* __restrict__ err) {
    constexpr int R = T / 16, H = R / 2;
    const int pn = kb + 1;
    const int tid = threadIdx.x, r = tid / 16, c = tid % 16;
    uint32_t acc[R][H];
    fw_load_block<T>(D, np, ti, tj, r, c, acc);
    if (role < 4) {
        fw_stage<T>(D, np, ti, kb, At, true);
        fw_stage<T>(D, np, kb, tj, Bt, false);
        __syncthreads();
        fw_tile_product<T>(At, Bt, acc, r, c);
    } else {
        role -= 2;  // the panel product alone
    }
    if (role == 1) {
        __syncthreads();  // every thread's product is done with At
#pragma unroll
        for (int i = 0; i < R; i++) fw_st<H>(At + (R * r + i) * T + R * c, acc[i]);
        __syncthreads();
        fw_close<T>(At, acc, r, c);
        fw_store_block<T>(D, np, ti, tj, r, c, acc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores drained
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&flag[pn], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (role >= 2) {
        // the closed pivot pn: one relaxed poll loop, one agent acquire, then plain loads
        __shared__ int s_open;
        if (tid == 0) {
            int spin = 0;
            while (__hip_atomic_load(&flag[pn], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 && spin < (1 << 24)) {
                __builtin_amdgcn_s_sleep(2);
                spin++;
            }
            // a pivot never published (a lost or stalled closing workgroup): the product
            // would read an open tile, so the launch reports a device error and this tile
            // keeps its values (the flag is read once more: it may have been published
            // between the last poll and the loop's exit)
            const bool open = spin >= (1 << 24) &&
                              __hip_atomic_load(&flag[pn], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
            if (open) raise_err(err, SHD_ROUTE_EDEVICE);
            s_open = open ? 1 : 0;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // (also: every thread's product is done with At / Bt)
        if (s_open) {
            fw_store_block<T>(D, np, ti, tj, r, c, acc);
            return;
        }
        if (role == 2) {
            // row panel: C = D* (x) C -- A = D* transposed, B = C as it now stands
            fw_stage<T>(D, np, pn, pn, At, true);
#pragma unroll
            for (int i = 0; i < R; i++) fw_st<H>(Bt + (R * r + i) * T + R * c, acc[i]);
        } else {
            // column panel: C = C (x) D* -- A = C transposed, B = D*
#pragma unroll
            for (int i = 0; i < R; i++)
#pragma unroll
                for (int h = 0; h < H; h++) {
                    At[(R * c + 2 * h) * T + R * r + i] = (uint16_t)(acc[i][h] & 0xFFFFu);
                    At[(R * c + 2 * h + 1) * T + R * r + i] = (uint16_t)(acc[i][h] >> 16);
                }
            fw_stage<T>(D, np, pn, pn, Bt, false);
        }
        __syncthreads();
        fw_tile_product<T>(At, Bt, acc, r, c);
    }
    fw_store_block<T>(D, np, ti, tj, r, c, acc);
}

// tile w of a pivot's fw_restp grid ((nb - 1)^2 + 2 when a next pivot exists): role and
// coordinates (see fw_restp_kernel)
__device__ inline void fw_restp_map(int w, int nb, int kb, int& ti, int& tj, int& role) {
    const int pn = kb + 1;
    auto skip = [&](int a, int x0, int x1) {  // a-th index of [0, nb) without x0 < x1
        if (a >= x0) a++;
        if (a >= x1) a++;
        return a;
    };
    role = 0;
    if (pn < nb) {
        const int m = nb - 2;
        if (w == 0) { ti = tj = pn; role = 1; }
        else if (w - 1 < m * m) { ti = skip((w - 1) / max(m, 1), kb, pn); tj = skip((w - 1) % max(m, 1), kb, pn); }
        else if (w - 1 - m * m < m) { ti = pn; tj = skip(w - 1 - m * m, kb, pn); role = 2; }
        else if (w - 1 - m * m < 2 * m) { ti = skip(w - 1 - m * m - m, kb, pn); tj = pn; role = 3; }
        else if (w - 1 - m * m == 2 * m) { ti = pn; tj = kb; role = 4; }  // row panel, no rest product
        else { ti = kb; tj = pn; role = 5; }                              // column panel, no rest product
    } else {
        const int m = nb - 1;
        ti = w / m; tj = w % m;
        if (ti >= kb) ti++;
        if (tj >= kb) tj++;
    }
}

template <int T>
__global__ __launch_bounds__(256) void fw_restp_kernel(uint16_t* __restrict__ D, int np, int kb, int* __restrict__ flag,
                                                       int* __restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint16_t At[T * T];
    __shared__ __attribute__((aligned(16))) uint16_t Bt[T * T];
    const int nb = np / T;
    int ti, tj, role;
    fw_restp_map(blockIdx.x, nb, kb, ti, tj, role);
    if (ti >= nb || tj >= nb) return;
    fw_restp_tile<T>(D, np, kb, flag, ti, tj, role, At, Bt, err);
}

// fw_restp with persistent plain workgroups (SHD_ROUTE_FWREST=3): workgroup 0 the next
// pivot, workgroups 1 .. P loop over the plain tiles (t = w - 1 + k P) with the next tile's
// C block and panel tiles loaded into registers while the current product runs (its
// staging latency off the critical path), the rest the panel roles as in fw_restp.
template <int T>
__global__ __launch_bounds__(256) void fw_restpp_kernel(uint16_t* __restrict__ D, int np, int kb, int* __restrict__ flag,
                                                        int P, int* __restrict__ err) {
    static_assert(T == 64, "4 x 4 blocks, 4 staging loads per panel and thread");
    constexpr int R = T / 16, H = R / 2;
    __shared__ __attribute__((aligned(16))) uint16_t At[T * T];
    __shared__ __attribute__((aligned(16))) uint16_t Bt[T * T];
    const int nb = np / T, pn = kb + 1;
    const int w = blockIdx.x;
    const int m = pn < nb ? nb - 2 : nb - 1, nplain = m * m;
    const int base = pn < nb ? 1 : 0;  // first plain tile index in fw_restp_map order
    int ti, tj, role;
    if (pn < nb && w == 0) {
        fw_restp_map(0, nb, kb, ti, tj, role);
        fw_restp_tile<T>(D, np, kb, flag, ti, tj, role, At, Bt, err);
        return;
    }
    if (w >= base + P) {  // panel roles
        fw_restp_map(w - P + nplain, nb, kb, ti, tj, role);
        if (ti < nb && tj < nb) fw_restp_tile<T>(D, np, kb, flag, ti, tj, role, At, Bt, err);
        return;
    }
    const int tid = threadIdx.x, r = tid / 16, c = tid % 16;
    struct Pre { uint2 a[4], b[4], c[R]; };
    auto load = [&](int t, Pre& x) __attribute__((always_inline)) {
        int i, j, ro;
        fw_restp_map(base + t, nb, kb, i, j, ro);
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const int q = tid + 256 * h;
            const int rowa = q % T, c4a = (q / T) * 4;            // column panel (i, kb), transposed
            x.a[h] = *reinterpret_cast<const uint2*>(D + (long long)(i * T + rowa) * np + kb * T + c4a);
            const int rowb = q / (T / 4), c4b = (q % (T / 4)) * 4;  // row panel (kb, j)
            x.b[h] = *reinterpret_cast<const uint2*>(D + (long long)(kb * T + rowb) * np + j * T + c4b);
        }
#pragma unroll
        for (int k = 0; k < R; k++) x.c[k] = *reinterpret_cast<const uint2*>(D + (long long)(i * T + R * r + k) * np + j * T + R * c);
    };
    Pre cur;
    int t = w - base;
    if (t >= nplain) return;
    load(t, cur);
    for (;;) {
        __syncthreads();  // the previous product is done with At / Bt
#pragma unroll
        for (int h = 0; h < 4; h++) {
            const int q = tid + 256 * h;
            const int rowa = q % T, c4a = (q / T) * 4;
            At[(c4a + 0) * T + rowa] = (uint16_t)(cur.a[h].x & 0xFFFFu);
            At[(c4a + 1) * T + rowa] = (uint16_t)(cur.a[h].x >> 16);
            At[(c4a + 2) * T + rowa] = (uint16_t)(cur.a[h].y & 0xFFFFu);
            At[(c4a + 3) * T + rowa] = (uint16_t)(cur.a[h].y >> 16);
            const int rowb = q / (T / 4), c4b = (q % (T / 4)) * 4;
            *reinterpret_cast<uint2*>(Bt + rowb * T + c4b) = cur.b[h];
        }
        uint32_t acc[R][H];
#pragma unroll
        for (int k = 0; k < R; k++) { acc[k][0] = cur.c[k].x; acc[k][1] = cur.c[k].y; }
        int i, j, ro;
        fw_restp_map(base + t, nb, kb, i, j, ro);
        __syncthreads();
        const int tn = t + P;
        if (tn < nplain) load(tn, cur);  // in flight during the product
        fw_tile_product<T>(At, Bt, acc, r, c);
        fw_store_block<T>(D, np, i, j, r, c, acc);
        if (tn >= nplain) break;
        t = tn;
    }
}

// The rest update of pivot kb over 128 x 128 regions (2 x 2 tiles of 64) with 8 x 8
// register blocks: 256 threads as 16 x 16, thread (r, c) holds rows 8r.. and columns 8c..
// of the region.  Per k step one 16-byte LDS read of the column panel (transposed: the
// thread's 8 rows) and one of the row panel (its 8 columns) feed 64 relaxations (32
// v_pk_add_u16 + 32 v_pk_min_u16): half the LDS bytes per relaxation of the 4 x 4 form,
// which shared the LDS and VALU evenly and ran at 0.27 of the packed-u16 VALU rate.
// Regions are fixed in absolute tile coordinates and the 1-D grid maps region w to
// workgroup w every pivot, so a region stays on XCD w % 8 and its tiles in that XCD's L2
// across pivots.  Tiles in pivot row or column kb (the panels), or past the matrix, are
// not written.  The region holding the next pivot tile (kb + 1, kb + 1) is dispatched
// first (its workgroup id swapped with 0) and closes that tile after its product, as the
// 64 x 64 kernel did.
constexpr int FW_RG = 2 * FW_T;  // region edge
__global__ __launch_bounds__(256) void fw_rest2_kernel(uint16_t* __restrict__ D, int np, int kb) {
    static_assert(FW_T == 64, "regions of 2 x 2 tiles of 64");
    __shared__ __attribute__((aligned(16))) uint16_t At[FW_T * FW_RG];  // [k][i], i < 128
    __shared__ __attribute__((aligned(16))) uint16_t Bt[FW_T * FW_RG];  // [k][j], j < 128
    const int nb = np / FW_T, nr = (nb + 1) / 2;
    const int pn = kb + 1;
    int w = blockIdx.x;
    if (pn < nb) {
        const int wp = (pn / 2) * nr + pn / 2;
        if (w == 0) w = wp;
        else if (w == wp) w = 0;
    }
    const int I = w / nr, J = w % nr;
    if (I >= nr) return;
    const int tid = threadIdx.x, r = tid >> 4, c = tid & 15;
    // valid tile rows / columns of the region (not the pivot's, not past the matrix)
    const bool row_ok[2] = {2 * I < nb && 2 * I != kb, 2 * I + 1 < nb && 2 * I + 1 != kb};
    const bool col_ok[2] = {2 * J < nb && 2 * J != kb, 2 * J + 1 < nb && 2 * J + 1 != kb};
    if (!((row_ok[0] || row_ok[1]) && (col_ok[0] || col_ok[1]))) return;  // (uniform)
    const int ti = 2 * I + (r >> 3), tj = 2 * J + (c >> 3);
    const bool mine = row_ok[r >> 3] && col_ok[c >> 3];
    const long long row0 = (long long)ti * FW_T + 8 * (r & 7);
    const int col0 = tj * FW_T + 8 * (c & 7);
    // C first: its loads overlap the panel staging
    uint32_t acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        if (mine) {
            const uint4 x = *reinterpret_cast<const uint4*>(D + (row0 + i) * np + col0);
            acc[i][0] = x.x; acc[i][1] = x.y; acc[i][2] = x.z; acc[i][3] = x.w;
        } else {
            acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0xFFFFFFFFu;
        }
    }
    // column panel D[region rows][kb cols] transposed into At: a wave's lanes take 64
    // consecutive rows of one 4-column strip (consecutive 2-byte LDS writes); rows of a
    // tile past the matrix read as "no path"
    for (int q = tid; q < FW_RG * FW_T / 4; q += 256) {
        const int row = q % FW_RG, c4 = (q / FW_RG) * 4;
        const int gt = 2 * I + (row >> 6);
        uint2 v = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
        if (gt < nb) v = *reinterpret_cast<const uint2*>(D + ((long long)2 * I * FW_T + row) * np + kb * FW_T + c4);
        At[(c4 + 0) * FW_RG + row] = (uint16_t)(v.x & 0xFFFFu);
        At[(c4 + 1) * FW_RG + row] = (uint16_t)(v.x >> 16);
        At[(c4 + 2) * FW_RG + row] = (uint16_t)(v.y & 0xFFFFu);
        At[(c4 + 3) * FW_RG + row] = (uint16_t)(v.y >> 16);
    }
    // row panel D[kb rows][region cols] into Bt as is
    for (int q = tid; q < FW_T * FW_RG / 8; q += 256) {
        const int k = q / (FW_RG / 8), c8 = (q % (FW_RG / 8)) * 8;
        const int gt = 2 * J + (c8 >> 6);
        uint4 v = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (gt < nb) v = *reinterpret_cast<const uint4*>(D + ((long long)kb * FW_T + k) * np + 2 * J * FW_T + c8);
        *reinterpret_cast<uint4*>(Bt + k * FW_RG + c8) = v;
    }
    __syncthreads();
    // software-pipelined: step k + 1's two LDS reads are in flight while step k computes;
    // per row the four packed adds go to their own temporaries before the four mins, so
    // no add is followed directly by its dependent min (which costs an s_nop after an
    // op_sel'd add)
    uint4 av = *reinterpret_cast<const uint4*>(At + 8 * r);
    uint4 bv = *reinterpret_cast<const uint4*>(Bt + 8 * c);
#pragma unroll 2
    for (int k = 0; k < FW_T; k++) {
        const int kn = k + 1 < FW_T ? k + 1 : k;
        const uint4 an = *reinterpret_cast<const uint4*>(At + kn * FW_RG + 8 * r);
        const uint4 bn = *reinterpret_cast<const uint4*>(Bt + kn * FW_RG + 8 * c);
        const uint32_t aw[4] = {av.x, av.y, av.z, av.w}, bw[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const fw_us2 x = __builtin_bit_cast(fw_us2, aw[i >> 1]);
            const fw_us2 a2 = (i & 1) ? __builtin_shufflevector(x, x, 1, 1) : __builtin_shufflevector(x, x, 0, 0);
            uint32_t t[4];
#pragma unroll
            for (int h = 0; h < 4; h++)
                t[h] = __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(a2, __builtin_bit_cast(fw_us2, bw[h])));
#pragma unroll
            for (int h = 0; h < 4; h++) acc[i][h] = fw_pkmin(acc[i][h], t[h]);
        }
        av = an;
        bv = bn;
    }
    const bool pivot_region = pn < nb && (pn >> 1) == I && (pn >> 1) == J;
    const bool pivot_mine = pivot_region && ti == pn && tj == pn;
    if (pivot_region) {
        // the next pivot tile: its 64 owner threads hand it over in LDS, the whole
        // workgroup closes it in the 4 x 4 layout, and stores it
        __syncthreads();  // every thread's product is done with At
        if (pivot_mine)
#pragma unroll
            for (int i = 0; i < 8; i++)
                *reinterpret_cast<uint4*>(At + (8 * (r & 7) + i) * FW_T + 8 * (c & 7)) =
                    make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
        __syncthreads();
        const int r4 = tid / 16, c4 = tid % 16;
        uint32_t x[4][2];
#pragma unroll
        for (int i = 0; i < 4; i++) fw_ld<2>(At + (4 * r4 + i) * FW_T + 4 * c4, x[i]);
        fw_close<FW_T>(At, x, r4, c4);
        fw_store_block<FW_T>(D, np, pn, pn, r4, c4, x);
    }
    if (mine && !pivot_mine)
#pragma unroll
        for (int i = 0; i < 8; i++)
            *reinterpret_cast<uint4*>(D + (row0 + i) * np + col0) = make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
}

// In-arc lists for the parent search, built once per graph: row v holds the keys
// (0xFFFF - w) << 16 | u of every in-arc u -> v (u != v, w < 0xFFFF) in increasing order,
// i.e. the engine tie rule's preference order (largest w, then smallest u), then FW_END
// padding; pos[v][x] (x < FW_X) is the first index whose arc has w <= x.  One workgroup
// per vertex: the column of the dense W, a bitonic sort of sp (power of two >= np) keys
// in LDS, and a lower bound per threshold.
constexpr int FW_X = 256;
#ifndef FW_SCAN
#define FW_SCAN 8  // in-arcs per parent-scan trip (4 or 8)
#endif
constexpr uint32_t FW_END = 0xFFFFFFFFu;
// Keys (pk = 0): (0xFFFF - w) << 16 | u.  Packed (pk = 1, round 6: every w <= 255 and the
// reliability indices rix present): (255 - w) << 24 | u << 8 | rix(u, v) -- the same order
// (largest w, then smallest u), and the parent arc's reliability index comes out of
// fw_parent with the parent, so fw_rows no longer gathers it from the dense n x n rix
// matrix (one 64-byte line per (p, v) pair: ~1 GB per C5 rows launch)
__device__ inline uint32_t fw_key_u(uint32_t e, int pk) { return pk ? (e >> 8) & 0xFFFFu : e & 0xFFFFu; }
__device__ inline uint32_t fw_key_w(uint32_t e, int pk) { return pk ? 0xFFu - (e >> 24) : 0xFFFFu - (e >> 16); }
__global__ __launch_bounds__(1024) void fw_inlist_kernel(const double* __restrict__ W, int n, int np, int sp,
                                                         uint32_t* __restrict__ inl, uint16_t* __restrict__ pos,
                                                         const uint8_t* __restrict__ rix, int pk) {
    extern __shared__ __attribute__((aligned(16))) uint32_t fkeys[];
    const int v = blockIdx.x, tid = threadIdx.x, B = blockDim.x;
    for (int k = tid; k < sp; k += B) {
        uint32_t key = FW_END;
        if (k < n && k != v) {
            const double w = W[(long long)k * n + v];
            if (!isnan(w) && w < 65535.0)
                key = pk ? ((0xFFu - (uint32_t)w) << 24) | ((uint32_t)k << 8) | (uint32_t)rix[(long long)k * n + v]
                         : ((0xFFFFu - (uint32_t)w) << 16) | (uint32_t)k;
        }
        fkeys[k] = key;
    }
    __syncthreads();
    for (int size = 2; size <= sp; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < sp / 2; t += B) {
                const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const uint32_t a = fkeys[lo], b = fkeys[hi];
                if ((a > b) == up) { fkeys[lo] = b; fkeys[hi] = a; }
            }
            __syncthreads();
        }
    }
    for (int k = tid; k < np; k += B) inl[(long long)v * np + k] = fkeys[k];
    for (int x = tid; x < FW_X; x += B) {
        // w <= x  <=>  key >= thr
        const uint32_t thr = pk ? (x >= 255 ? 0u : (0xFFu - (uint32_t)x) << 24) : (0xFFFFu - (uint32_t)x) << 16;
        int lo = 0, hi = sp;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (fkeys[mid] < thr) lo = mid + 1; else hi = mid;
        }
        pos[(long long)v * FW_X + x] = (uint16_t)lo;
    }
}

// parents: key[s][v] = min over u != v with D[s][u] + w(u,v) == D[s][v] of
// (0xFFFF - w) << 16 | u (largest w, then smallest u: the engine tie rule), FW_END for the
// source and unreachable vertices.  One workgroup per source with D[s][.] in LDS; a thread
// scans its targets' in-arc lists in key order from the first arc with w <= D[s][v] (pos
// table, or a binary search past FW_X) and stops at the first tight arc, which is the
// minimum key.  A scan visits only the arcs with w in (w*, D[s][v]]: on K4000 with
// U[1,250] latencies ~20 trips of 8 arcs, each a dependent global load.  Round 5: a thread
// keeps FW_PQ scans in flight (a slot whose scan ends takes the thread's next target in the
// same trip), so a trip's loads cover FW_PQ targets (0.90 ms for C5's 16 M pairs with one).
// The scan starts at the 8-arc boundary below the first candidate: the arcs before it
// have w > D[s][v], never tight (D[s][u] + w > D[s][v]), so they cost a compare, not a
// result.  In-arc lists hold np entries padded with FW_END, so a scan always ends.
#ifndef FW_PQ
// (round 6, with the packed keys: C5 rows 0.640 ms at 2, 0.655 at 4, 0.733 at 6 and 8; two
// runs each, spread 0.005)
#define FW_PQ 2
#endif
// (round 6) The key form is a template parameter and a trip's 8 arcs are checked without
// branches: the hits (tight arcs, and the FW_END padding that ends a list) are folded by a
// min, which is the first hit since a list ascends and its padding comes last.  The SQ
// counters had the lane-per-target scan VALU-bound (255 M VALU instructions per C5 launch,
// ~88% issue), not memory-bound: the runtime key form doubled every decode into a select.
template <bool PK>
__global__ __launch_bounds__(1024) void fw_parent_kernel(const uint16_t* __restrict__ D, const uint32_t* __restrict__ inl,
                                                         const uint16_t* __restrict__ pos, int n, int np,
                                                         const int* __restrict__ src, int ns,
                                                         uint32_t* __restrict__ key) {
    extern __shared__ __attribute__((aligned(16))) uint16_t drow[];
    static_assert(FW_SCAN == 8, "two 16-byte loads per scan trip");
    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (s < 0 || s >= n) continue;  // fw_rows raises the error for this row
        __syncthreads();
        const uint16_t* Ds = D + (long long)s * np;
        for (int q = threadIdx.x; q < np / 8; q += blockDim.x)
            reinterpret_cast<uint4*>(drow)[q] = reinterpret_cast<const uint4*>(Ds)[q];
        __syncthreads();
        uint32_t* const krow = key + (long long)i * np;
        // slots: target v (-1 idle), its distance, scan position (-1: not yet located)
        int sv[FW_PQ], sk[FW_PQ];
        unsigned sd[FW_PQ];
        int vnext = threadIdx.x;
        // the next target that needs a scan (the source and unreachable vertices are written
        // here; a target at distance >= FW_X is located by its binary search at once)
        auto take = [&](int q) __attribute__((always_inline)) {
            sv[q] = -1;
            while (vnext < n) {
                const int v = vnext;
                vnext += blockDim.x;
                const unsigned d = drow[v];
                if (v == s || d == 0xFFFFu) { krow[v] = FW_END; continue; }
                sv[q] = v; sd[q] = d; sk[q] = -1;
                if (d >= (unsigned)FW_X) {
                    const uint32_t* lv = inl + (long long)v * np;
                    const uint32_t thr = PK ? 0u : (0xFFFFu - d) << 16;  // (packed: every w <= 255 < d)
                    int lo = 0, hi = pos[(long long)v * FW_X + FW_X - 1];
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (lv[mid] < thr) lo = mid + 1; else hi = mid;
                    }
                    sk[q] = lo & ~(FW_SCAN - 1);
                }
                return;
            }
        };
#pragma unroll
        for (int q = 0; q < FW_PQ; q++) take(q);
        for (;;) {
            bool any = false;
#pragma unroll
            for (int q = 0; q < FW_PQ; q++) any = any || sv[q] >= 0;
            if (!any) break;
            // one trip: every slot's loads first (a located slot's next 8 arcs, an unlocated
            // one's pos entry), then the checks
            uint4 ea[FW_PQ], eb[FW_PQ];
            unsigned pk[FW_PQ];
#pragma unroll
            for (int q = 0; q < FW_PQ; q++) {
                ea[q] = eb[q] = make_uint4(FW_END, FW_END, FW_END, FW_END);
                pk[q] = 0u;
                if (sv[q] < 0) continue;
                if (sk[q] >= 0) {
                    const uint32_t* lv = inl + (long long)sv[q] * np + sk[q];
                    ea[q] = *reinterpret_cast<const uint4*>(lv);
                    eb[q] = *reinterpret_cast<const uint4*>(lv + 4);
                } else {
                    pk[q] = pos[(long long)sv[q] * FW_X + sd[q]];
                }
            }
#pragma unroll
            for (int q = 0; q < FW_PQ; q++) {
                if (sv[q] < 0) continue;
                if (sk[q] < 0) { sk[q] = (int)pk[q] & ~(FW_SCAN - 1); continue; }
                const uint32_t e[FW_SCAN] = {ea[q].x, ea[q].y, ea[q].z, ea[q].w, eb[q].x, eb[q].y, eb[q].z, eb[q].w};
                unsigned dd[FW_SCAN];
#pragma unroll
                for (int h = 0; h < FW_SCAN; h++) dd[h] = drow[e[h] == FW_END ? 0u : fw_key_u(e[h], PK)];
                uint32_t best = FW_END;
                bool done = false;
#pragma unroll
                for (int h = 0; h < FW_SCAN; h++) {
                    const bool end = e[h] == FW_END;
                    const bool tight = !end && dd[h] + fw_key_w(e[h], PK) == sd[q];
                    best = min(best, tight ? e[h] : FW_END);
                    done = done || end || tight;
                }
                sk[q] += FW_SCAN;
                if (!done && sk[q] >= np) done = true;  // (np: a multiple of 64; lists end in FW_END)
                if (done) {
                    krow[sv[q]] = best;
                    take(q);
                }
            }
        }
    }
}

// parents for 8 sources at once (round 6): D[s][.] of 8 sources interleaved in LDS as u16 x 8
// per vertex, so one 16-byte LDS read gives D[s_b][u] for all 8 and one pass over v's in-list
// serves the 8 scans: the arc loads (one cache line per lane and 8 arcs, the bound of the
// per-source kernel) are shared by 8 sources, and the 8 tightness tests are 4 packed adds and
// compares.  A lane scans from the start of the largest distance among its 8 (pos table:
// the earliest start) until every source has its first tight arc (or the list's padding):
// an arc before a source's own start is never tight for it (w > d), so the union scan finds
// the same first hit per source.  Needs 16 np bytes of LDS.  (C5: fw_parent 0.48 -> ~0.27 ms.)
template <bool PK>
__global__ __launch_bounds__(1024) void fw_parent8_kernel(const uint16_t* __restrict__ D, const uint32_t* __restrict__ inl,
                                                          const uint16_t* __restrict__ pos, int n, int np,
                                                          const int* __restrict__ src, int ns,
                                                          uint32_t* __restrict__ key) {
    extern __shared__ __attribute__((aligned(16))) uint16_t dl[];  // [np][8]
    for (int i0 = blockIdx.x * 8; i0 < ns; i0 += gridDim.x * 8) {
        int sb[8];
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const int i = i0 + b;
            int s = i < ns ? src[i] : -1;
            sb[b] = s >= 0 && s < n ? s : -1;  // (fw_rows raises the error for a bad source)
        }
        __syncthreads();  // the previous batch is done with dl
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint16_t* Ds = sb[b] >= 0 ? D + (long long)sb[b] * np : nullptr;
            for (int u = threadIdx.x; u < np; u += blockDim.x) dl[8 * u + b] = Ds ? Ds[u] : (uint16_t)0xFFFFu;
        }
        __syncthreads();
        for (int v = threadIdx.x; v < n; v += blockDim.x) {
            const uint4 dq = *reinterpret_cast<const uint4*>(dl + 8 * v);
            const uint32_t dw[4] = {dq.x, dq.y, dq.z, dq.w};
            unsigned pend = 0u;
            int dmax = -1;
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const int db = (int)((dw[b >> 1] >> (16 * (b & 1))) & 0xFFFFu);
                if (sb[b] >= 0 && v != sb[b] && db != 0xFFFF) { pend |= 1u << b; dmax = max(dmax, db); }
            }
            uint32_t best[8];
#pragma unroll
            for (int b = 0; b < 8; b++) best[b] = FW_END;
            if (pend) {
                const uint32_t* lv = inl + (long long)v * np;
                int lo = 0;
                if (dmax < FW_X) lo = pos[(long long)v * FW_X + dmax];
                else if (!PK) {  // (packed: every w <= 255 < dmax, the whole list)
                    const uint32_t thr = (0xFFFFu - (uint32_t)dmax) << 16;
                    int hi = pos[(long long)v * FW_X + FW_X - 1];
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (lv[mid] < thr) lo = mid + 1; else hi = mid;
                    }
                }
                int a = lo & ~7;
                uint4 ea = *reinterpret_cast<const uint4*>(lv + a), eb = *reinterpret_cast<const uint4*>(lv + a + 4);
                while (pend) {
                    const uint32_t e[8] = {ea.x, ea.y, ea.z, ea.w, eb.x, eb.y, eb.z, eb.w};
                    const int an = a + 8;
                    if (an < np) {  // the next trip's arcs in flight during this one's checks
                        ea = *reinterpret_cast<const uint4*>(lv + an);
                        eb = *reinterpret_cast<const uint4*>(lv + an + 4);
                    }
#pragma unroll
                    for (int h = 0; h < 8; h++) {
                        const uint32_t x = e[h];
                        if (x == FW_END) pend = 0u;  // (the padding follows every arc)
                        if (!pend) continue;
                        const uint32_t u = fw_key_u(x, PK), w = fw_key_w(x, PK);
                        const fw_us2 w2 = {(unsigned short)w, (unsigned short)w};
                        const uint4 uq = *reinterpret_cast<const uint4*>(dl + 8 * u);
                        const uint32_t uw[4] = {uq.x, uq.y, uq.z, uq.w};
                        uint32_t y = 0u;
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            // halves of z are 0 exactly where D[s][u] + w == D[s][v] (an
                            // unreachable u saturates at 0xFFFF, never a reached distance)
                            const uint32_t z = __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(
                                                   __builtin_bit_cast(fw_us2, uw[k]), w2)) ^ dw[k];
                            const fw_us2 zm = __builtin_bit_cast(fw_us2, z) - fw_us2{1, 1};
                            const uint32_t t = __builtin_bit_cast(uint32_t, zm) & ~z & 0x80008000u;  // bit 15 / 31: half == 0
                            y |= t >> (15 - 2 * k);
                        }
                        const unsigned hit = ((y | (y >> 15)) & 0xFFu) & pend;
#pragma unroll
                        for (int b = 0; b < 8; b++) best[b] = ((hit >> b) & 1u) ? x : best[b];
                        pend &= ~hit;
                    }
                    a = an;
                    if (a >= np) pend = 0u;  // (unreached: every list ends in FW_END)
                }
            }
#pragma unroll
            for (int b = 0; b < 8; b++)
                if (sb[b] >= 0) key[(long long)(i0 + b) * np + v] = best[b];
        }
    }
}

// rows: per source (one workgroup), rel down the parent tree in distance order (LDS
// buckets by distance), then the lat / rel rows for the targets; the self entry is the
// batch self-loop (lat = w_ss, rel = (1*f_s)*r_ss) as in every SOURCE row
struct FWRowsArgs {
    int n, np, bound;
    const uint16_t* D;
    const uint32_t* key;     // [ns][np]
    const double* R;         // dense 1 - loss, n x n (NaN = no edge)
    // (round 5) the same as indices into a table of the distinct reliabilities (<= 255 of
    // them, nrtab > 0): a random (p, v) read of 1 byte from a 16 MB matrix (C5) instead of 8
    // from a 128 MB one, the factor from the table in LDS
    const uint8_t* rix;
    const double* rtab;
    int nrtab;
    const double* vf;
    const double* self_w;
    const double* self_r;
    int pk;                  // packed keys: parent << 8 | rix in the key (fw_inlist_kernel)
};
__global__ __launch_bounds__(1024) void fw_rows_kernel(FWRowsArgs a, const int* __restrict__ src, int ns,
                                                       const int* __restrict__ tgt, int nt, long long ld,
                                                       double* __restrict__ lat_out, double* __restrict__ rel_out,
                                                       double* __restrict__ row_min, int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // rel f64[n] | order u16[n] | bucket starts int[bound + 2] (u16 order since round 6:
    // 40 KB per workgroup on C5's 4000 vertices, so four 512-thread workgroups fit a CU)
    double* rel = reinterpret_cast<double*>(smem);
    uint16_t* order = reinterpret_cast<uint16_t*>(smem + a16(sizeof(double) * a.n));
    int* bstart = reinterpret_cast<int*>(smem + a16(sizeof(double) * a.n) + a16(sizeof(uint16_t) * a.n));
    __shared__ unsigned long long rmin;
    __shared__ double rtl[256];
    for (int k = threadIdx.x; k < a.nrtab; k += blockDim.x) rtl[k] = a.rtab[k];
    const int nbk = a.bound + 2;
    for (int i = blockIdx.x; i < ns; i += gridDim.x) {
        const int s = src[i];
        if (s < 0 || s >= a.n) { if (threadIdx.x == 0) raise_err(err, SHD_ROUTE_EINVAL); continue; }
        const uint16_t* Ds = a.D + (long long)s * a.np;
        const uint32_t* Ks = a.key + (long long)i * a.np;
        for (int b = threadIdx.x; b < nbk; b += blockDim.x) bstart[b] = 0;
        if (threadIdx.x == 0) rmin = kInfBits;
        __syncthreads();
        // counting sort of the vertices by distance
        for (int v = threadIdx.x; v < a.n; v += blockDim.x) {
            const unsigned d = Ds[v];
            if (d <= (unsigned)a.bound) atomicAdd(&bstart[d + 1], 1);
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int b = 1; b < nbk; b++) bstart[b] += bstart[b - 1];
        __syncthreads();
        for (int v = threadIdx.x; v < a.n; v += blockDim.x) {
            const unsigned d = Ds[v];
            if (d <= (unsigned)a.bound) order[atomicAdd(&bstart[d], 1)] = (uint16_t)v;
        }
        __syncthreads();
        // bstart[d] now holds the end of bucket d; buckets in increasing distance
        const double fs = a.vf[s];
        const double cs = isnan(fs) ? 1.0 : 1.0 * fs;
        if (threadIdx.x == 0) rel[s] = cs;
        __syncthreads();
        for (int d = 1; d <= a.bound; d++) {
            const int b0 = bstart[d - 1], b1 = bstart[d];
            if (b0 == b1) continue;
            for (int q = b0 + (int)threadIdx.x; q < b1; q += blockDim.x) {
                const int v = order[q];
                const uint32_t k = Ks[v];
                if (k == 0xFFFFFFFFu) { raise_err(err, SHD_ROUTE_EUNREACH); rel[v] = NAN; continue; }
                const int p = (int)fw_key_u(k, a.pk);
                rel[v] = rel[p] * (a.pk ? rtl[k & 0xFFu]
                                        : a.nrtab > 0 ? rtl[a.rix[(long long)p * a.n + v]] : a.R[(long long)p * a.n + v]);
            }
            __syncthreads();
        }
        double lmin = INFINITY;
        double* lrow = lat_out ? lat_out + (long long)i * ld : nullptr;
        double* rrow = rel_out ? rel_out + (long long)i * ld : nullptr;
        for (int j = threadIdx.x; j < nt; j += blockDim.x) {
            const int t = tgt[j];
            double L = NAN, Rv = NAN;
            if (t < 0 || t >= a.n) raise_err(err, SHD_ROUTE_EINVAL);
            else if (t == s) {
                if (isnan(a.self_w[s])) raise_err(err, SHD_ROUTE_ENOEDGE);
                else { L = 0.0 + a.self_w[s]; Rv = cs * a.self_r[s]; }
            } else if (Ds[t] == 0xFFFFu) raise_err(err, SHD_ROUTE_EUNREACH);
            else {
                L = (double)Ds[t];
                const double ft = a.vf[t];
                Rv = isnan(ft) ? rel[t] : rel[t] * ft;
            }
            if (!isnan(L)) lmin = fmin(lmin, L);
            if (lrow) __builtin_nontemporal_store(L, lrow + j);
            if (rrow) __builtin_nontemporal_store(Rv, rrow + j);
        }
        if (row_min) {
#pragma unroll
            for (int dd = 32; dd >= 1; dd >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, dd, 64));
            if ((threadIdx.x & 63) == 0 && lmin < INFINITY) atomicMin(&rmin, as_u(lmin));
            __syncthreads();
            if (threadIdx.x == 0) row_min[i] = as_d(rmin);
        }
        __syncthreads();
    }
}

}  // namespace shd
