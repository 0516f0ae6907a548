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
//    words that can hold bucket work.  Each sweep:
//      gather  one thread per word moves the pending vertices with dist < T into a
//              dense LDS queue (no atomics: nothing else runs);
//      prep    one thread per queue entry loads its CSR row bounds (all loads in
//              flight at once, so a sweep pays one global latency for them);
//      expand  each wave takes a 64-entry slice (strided over the queue, so the BA
//              hubs -- low ids, gathered first -- spread over all slices) and walks the
//              slice's out-arcs with a wave-level load-balanced scan: KD_P steps of 64
//              arcs at a time, owners found for all steps with one marker write, all
//              arc loads in flight together, all dist reads batched.
//    An improvement is a 32-bit CAS on the word holding two u16 distances (there is no
//    16-bit LDS atomic), then set-pending + wmin update.  On BA topologies with
//    U[1,250] ms edges D = 15 expands each vertex ~1.03 times (frontier Bellman-Ford:
//    5.7 times).
//
//    Fused parents (undirected graphs): when u is expanded, its out-arcs are its in-arcs,
//    so the same dist[v] reads find the tight in-arcs (dist[v] + w == dist[u]).  The
//    engine tie rule takes the tight arc with the largest w, then smallest (u, eid).  A
//    tight HEAVY arc (w >= D) comes from an earlier bucket, which is final when u's last
//    expansion runs, so a heavy winner seen at the last expansion is the final parent:
//    no light arc can beat it and no heavy arc can appear later.  Vertices whose winner
//    is light or absent (45% on C4: shortest-path trees favour short arcs) are marked
//    for a pull fix-up over the light tail of their (-w, u, eid)-sorted in-row (phase
//    B, ~12% of the arcs).  Directed graphs fix up every vertex over its whole in-row.
//
// B  fix-ups (four vertices and four tail arcs each in flight per thread; long tails one
//    wave per vertex), lat row out (dist is exact: integer latencies, bound < 0xFFFF).
// C  reliability down the tree: parents u16 in LDS over the dead distances, relv f64 in
//    a per-workgroup HBM slice (8n bytes do not fit LDS at this size).  Level sweeps
//    over a pending bitmask: a vertex is ready when its parent left the pending set in
//    an earlier sweep; ready vertices load relv[parent] and their own -r together.
// D  rel row out, row min.  Output rows are non-temporal stores (written once, never
//    re-read here) so they do not evict the CSR from L2.
//
// Measured on MI355X under a full-chip load (tools/micro/lat_probe.hip): a dependent
// L2 gather costs ~2.4k cycles, a random 4-8 B gather into a 16-64 MB array is line-
// traffic bound at ~0.3-0.5 per CU-cycle, and because gfx9 counts loads and stores in ONE
// in-order vmcnt, a load consumed after a store waits ~5-15k cycles for that store.  So:
//  * arc records carry everything a parent needs: out-arcs {v | w << 16, ridx} where
//    ridx indexes the table of distinct reliabilities (101 entries on C4), so the winning
//    parent (vertex, ridx) comes out of the expansion itself, no gather;
//  * fix-ups read a compact light in-CSR (12% of the arcs, L2-resident);
//  * loads are straight-line (clamped addresses, no branches around them) and stores are
//    deferred: a slice records each winner in LDS, the next sweep flushes the records
//    (wpr, one u32 per vertex) before its only global loads.
#include "common.hpp"

namespace shd {

constexpr int KD_P = 8;  // arc steps (64 arcs each) with loads in flight per wave
static_assert(KD_P == 8, "owner markers are read as one u64 per lane");
constexpr int KD_TAIL = 4;  // light-tail arcs per fix-up vertex loaded speculatively
constexpr int KD_W = 8;      // bitmask words per wave step in the gather / readiness scans
constexpr int KD_IMP = 192;  // per-wave list of improving arcs (v | nd << 16), flushed past 128
constexpr uint32_t KD_NONE = 0xFFFFFFFFu;      // no parent recorded
constexpr uint32_t KD_SRC_MARK = 0xFFFFFFFEu;  // parent record of the source itself

// Seeded rows (planned launches, engine.hip shd_route_plan_*).  A source s whose
// neighbour u already has its row (dist d_u and parent records p_u, kept in a row
// store) starts from D0(v) = w(s,u) + d_u(v) instead of infinity.  D0 is a set of
// path lengths that is already consistent (d_u(x) <= d_u(v) + w(v,x) for every arc),
// so only s and the vertices that improve on D0 are ever expanded: on the BA
// topologies 15-18% of them (C3/C4) instead of all.  Parents of the vertices that do
// not improve: their tight in-arcs are exactly u's tight in-arcs (all of whose tails
// also kept D0) plus tight arcs from improved vertices, so the parent is the better
// (engine tie rule) of p_u(v) and the tight improved in-neighbours, which the
// expansion reports as tie events (dist[x] + w == dist[v], found by the same reads).
// Up to KD_SEEDS seeds per row: D0(v) = min_j w(s,u_j) + d_{u_j}(v) is still consistent
// (a min of consistent labellings), and a vertex keeping D0 takes the best (tie rule) of
// the parents p_{u_j}(v) of the seeds that attain the min, and of its tie events.  Two
// seeds leave 3-4% of the vertices to improve on C3/C4 (one seed: 14-20%).
// global (address space 1) pointers for non-inlined helpers: flat accesses would count in
// lgkmcnt too, so every LDS wait would also wait for the output stores
#define KD_GLOBAL __attribute__((address_space(1)))

#ifndef KD_NSEEDS
#define KD_NSEEDS 3  // seeds per row at most (KDJob holds up to 3; the planner's default: engine.hip)
#endif
constexpr int KD_SEEDS = KD_NSEEDS;
#ifndef KD_NTLOAD
#define KD_NTLOAD 1  // 1024-thread rows: streaming loads of the seed rows and phase C's parent records
#endif
#ifndef KD_JUMPS
#define KD_JUMPS 1  // phase C pointer-jumping rounds before the walks (C4: 0: 50.5 ms, 1: 48.6, 2: 49.3, 3: 51.5, to convergence: 54.2)
#endif
struct __attribute__((aligned(64))) KDJob {  // padded to 64 bytes (copied as 16 ints)
    int row;               // output row
    int s;                 // source vertex
    int store;             // row-store slot this row is kept in for later seeds, -1 = not kept
    int nseed;             // seeds used (0 = unseeded: a root)
    int seed[KD_SEEDS];    // row-store slots of the seeds' rows
    int u[KD_SEEDS];       // seed vertices: neighbours of s, or two hops away (s -> x -> u)
    int wr[KD_SEEDS];      // offset: the length of the s -> u path the seed's row is shifted by
    int rec[KD_SEEDS];     // parent record of u itself if it keeps D0: s | ridx(s,u) << 16 |
                           // w(s,u) << 24 for a neighbour, x | ridx(x,u) << 16 | w(x,u) << 24
                           // for a two-hop seed (arc (x,u) is tight whenever u keeps D0)
};
static_assert(sizeof(KDJob) == 64, "one 64-byte job record");
constexpr uint32_t KD_EVTAG = 0xFFFF0000u;  // ring record y of a tie event: v | KD_EVTAG
typedef unsigned short kd_us2 __attribute__((ext_vector_type(2)));
typedef double kd_d2 __attribute__((ext_vector_type(2)));
typedef unsigned kd_u4 __attribute__((ext_vector_type(4)));
typedef unsigned kd_u2 __attribute__((ext_vector_type(2)));

struct DevDelta {
    int* next;                          // source queue counter (zeroed before each launch)
    const KDJob* __restrict__ jobs;     // planned launch: job j instead of src[j] / row j
    const uint16_t* __restrict__ drow;  // row store: dist u16 [slot * rstride + v]
    uint16_t* drow_out;                 // (the same store, written)
    uint32_t* prow;                     // row store: parent records [slot * rstride + v]
    long long rstride;
    int evcap;                          // tie events per source held in the workgroup slice
    int* done;                          // per row-store slot: 1 once the kept row is complete
    int n, nw;
    int nlight;                         // light in-arcs
    int nnz;                            // out-arcs
    int bound;
    int delta;                          // bucket width; arcs with w >= delta are heavy
    int fused;                          // undirected + packed records: parents found during expansion
    int rc;                             // LDS work-queue capacity per bucket round (vertices)
    const int* __restrict__ row;        // out-CSR offsets (n+1)
    const uint32_t* __restrict__ orec;  // out-arcs v | w << 16, rows sorted by (v, eid)
    const uint16_t* __restrict__ oridx; // rtab index of each out-arc
    const int* __restrict__ lrow;       // light in-CSR offsets (n+1)
    const uint2* __restrict__ lrec;     // light in-arcs {u | w << 16, ridx}, rows by (-w, u, eid)
                                        // (directed graphs: every in-arc)
    const double* __restrict__ rtab;    // distinct 1 - loss values, indexed by ridx
    int nrtab;
    int rone;                           // index of exactly 1.0 in rtab (-1: none)
    int walk;                           // phase C by path walks in LDS (nrtab <= 256, fits)
    int packed;                         // orec = v | w << 16 | ridx << 24 (w < 256, nrtab <= 256)
    const double* __restrict__ vf;
    const double* __restrict__ self_w;
    const double* __restrict__ self_r;
    int has_vf;                         // some vertex factor other than 1.0 (else every f_v is 1.0 or
                                        // absent, a no-op in every product: vf is not read)
    int dflags;                         // diagnostic builds: 1 = skip the output-row stores
    int seed_drop;                      // tests (SHD_ROUTE_SEEDDROP): bit q drops seed q >= 1 of every
                                        // seeded job, as an unready seed is dropped (KD_SEEDSPIN)
    unsigned long long* dbg;            // SHD_STAMPS builds: KD_NACC words per source
    unsigned long long* stats;          // liveness: the longest single wait (s_sleep rounds) of [0] a compute
                                        // wave for writer-ring space, [1] the writer on a reserved record
                                        // not yet written, [2] a slice on a queue entry not yet written
};

constexpr int KD_NACC = 40;
#ifdef SHD_STAMPS
// KD_NACC words per source (32-35: pre-init: walk cycles of wave 0, barrier wait, pre-init
// cycles of its first wave, rows pre-initialised): 0-4 phase stamps, 5 sweeps, 6 queued, 7 arcs, 8-11 summed sweep
// parts, 12-15 phase C (sweeps, compute, store drain, barriers), 16-19 phase B parts
// accumulated in LDS (sm->acc) and written out once per source: a global read-modify-
// write inside the timed regions would drain the wave's vmcnt and distort them
#define KD_ACCP (sm->acc)
#define KD_OUT (!(dflags & 1))
#define KD_DFLAGS g.dflags
#define KD_STAMP(slot) do { if (tid == 0) sm->acc[slot] = __builtin_amdgcn_s_memtime(); } while (0)
#define KD_COUNT(slot, x) do { if (lane == 0 && (x)) atomicAdd(&sm->acc[slot], (unsigned long long)(x)); } while (0)
#define KD_MARK() do { if (tid == 0) kd_t = __builtin_amdgcn_s_memtime(); } while (0)
#define KD_ACC(slot) do { if (tid == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); sm->acc[slot] += t_ - kd_t; kd_t = t_; } } while (0)
#define KD_FLUSH() do { lds_barrier(); if (g.dbg && i >= 0) for (int q_ = tid; q_ < KD_NACC; q_ += B) g.dbg[(size_t)i * KD_NACC + q_] = sm->acc[q_]; lds_barrier(); if (tid < KD_NACC) sm->acc[tid] = 0; lds_barrier(); } while (0)
#else
#define KD_ACCP nullptr
#define KD_OUT true
#define KD_DFLAGS 0
#define KD_STAMP(slot) do { } while (0)
#define KD_COUNT(slot, x) do { } while (0)
#define KD_MARK() do { } while (0)
#define KD_ACC(slot) do { } while (0)
#define KD_FLUSH() do { } while (0)
#endif

// the output phases' launch-invariant arguments, staged in LDS once per launch: kd_output
// takes only its row's values (its ~26 arguments used to overflow the 32 argument VGPRs of
// the call ABI, and every row stored the rest to the stack: scratch traffic per row)
struct KDOut {
    const KD_GLOBAL int* tgt;
    KD_GLOBAL double* lat_out;
    KD_GLOBAL double* rel_out;
    KD_GLOBAL double* row_min;
    int* err;
    KD_GLOBAL double* relv;      // this workgroup's HBM slice
    const KD_GLOBAL double* rtab;
    const KD_GLOBAL double* vf;
    long long ld;
    int n, nw, nt, tsorted;
    unsigned rmask;
    int rc, walk, nrtab, rone, has_vf, dflags;
};

struct KDSmall {
    unsigned gmin[2];   // min pending distance at the start of a bucket round (by parity)
    int head, tail;     // work queue of this bucket round: grabbed / reserved
    int busy;           // compute waves holding a grabbed slice
    int nexit;          // compute waves that left the async loop
    int rtail, rdone;   // parent-record ring: reserved / consumed by the writer wave
    int qtail[2];       // phase B/C list lengths (by parity)
    int qcur[2];        // phase B long-tail list lengths
    unsigned long long rmin;
    int deep;           // phase C path walk: some target deeper than KD_MAXD
    int next;           // the workgroup's next source index
    int nev;            // seeded: tie events the writer wave stored
    int evovf;          // seeded: more tie events than the slice holds (rerun unseeded)
    int tsorted;        // the target list is strictly increasing: positions from tmask/tpre
    int jflag[3];       // phase C pointer jumping: "some pointer moved" per round (mod 3)
    int wnext;          // phase C walks (wdyn): the next block of targets
    int wnext2, novf;   // phase C capped walks (KD_WCAP): next block of the second pass, chains listed
    KDJob job;          // the current job (kept in LDS: read where needed, not held in
                        // registers across phase A, whose expansion needs all of them)
    // planned launches: the next job is taken at the start of this row's output phases
    KDJob njob;         // the next job (valid when njb >= 0)
    int njb;            // its queue index (-1: not taken; the loop takes one as usual)
    int wpar;           // which of the two per-workgroup record slices the current row uses
    const KDJob* jobs;  // (the launch's job list, queue counter, row store and flags, for the
    int* qnext;         //  non-inlined output phases)
    const uint16_t* drow;
    uint32_t* prow;
    long long rstride;
    int* done;
    uint32_t* wsl[2];   // the two record slices of this workgroup
    int ns;
    KDOut out;          // kd_output's launch-invariant arguments
#ifdef SHD_STAMPS
    unsigned long long acc[KD_NACC];
#endif
};

// LDS: per-wave scratch | dist u16[n+1] | pend, fix u64[nw] | wmin u32[nw] | work.
// work holds the bucket work queue (u16 x rc) + the parent-record ring (uint2 x rr) in
// phase A, and the phase B/C vertex lists (u16 x qcap + i32 x qcap) afterwards.
template <int B>
struct KDLayout {
    size_t tmask, tpre, wmark, wkey, wimp, dist, pend, fix, wmin, work, ring, rrec, qv, qbeg, rix, rtabl, total;
    int qcap;
    __host__ __device__ static KDLayout make(int n, int rc, int rr) {
        KDLayout L;
        const size_t nw = (size_t)(n + 63) / 64;
        size_t o = a16(sizeof(KDSmall));
        // target set of the launch (kept for every source): a bit per vertex and the
        // exclusive popcount prefix per word, so an output position is rank(v) with no
        // global load (output loops never wait behind their own stores: one vmcnt)
        L.tmask = o; o += a16(8 * nw);
        L.tpre = o;  o += a16(4 * nw);
        L.dist = o;  o += a16(sizeof(uint16_t) * (size_t)(n + 1));
        // everything after dist is re-initialised per source or written before it is read:
        // the path walk of phase C reuses it for the parent-arc reliability indices (u8 x n)
        // and the reliability table
        L.rix = o;
        L.wmark = o; o += (size_t)(B / 64) * 8 * KD_P;
        L.wkey = o;  o += (size_t)(B / 64) * 64 * 4;
        L.wimp = o;  o += (size_t)(B / 64) * KD_IMP * 4;
        L.pend = o;  o += a16(8 * nw);
        L.fix = o;   o += a16(8 * nw);
        L.wmin = o;  o += a16(4 * nw);
        L.work = o;
        const size_t wbytes = a16(2 * (size_t)rc) + 8 * (size_t)rr;
        L.ring = o;
        L.rrec = o + a16(2 * (size_t)rc);
        L.qcap = (int)((wbytes - 16) / 6) & ~7;
        L.qv = o;
        L.qbeg = o + a16(2 * (size_t)L.qcap);
        o += wbytes;
        L.total = o;
        L.rtabl = a16(L.rix + (size_t)n);
        return L;
    }
};
constexpr int KD_MAXD = 32;           // phase C path walk: arcs held in registers
// build-time variants (A/B builds, tools/build_var.sh; the defaults are the shipped kernel:
// round 4, C4 45.8 -> 44.2 ms with SDIV 8 + WDYN + WCAP 2 against all three off, C3 2.74 ->
// 2.76 ms; the losing variants -- lat row fused into the parent copy or the walks, records
// loaded only where a seed attains D0, pre-init of the next row under the walks -- measured
// 44.9-50.1 ms and were removed in round 5)
#ifndef KD_SDIV
#define KD_SDIV 8   // phase A (1024-thread workgroups): a grab takes max(KD_SMIN, queued / KD_SDIV) entries, at most 64 (0: min(64, queued))
#endif
#ifndef KD_SMIN
#define KD_SMIN 16
#endif
#ifndef KD_WDYN
#define KD_WDYN 1   // phase C: waves take 128-target walk blocks from a counter (0: static blocks)
#endif
#ifndef KD_WCAP
#define KD_WCAP 2   // phase C: first-pass walks capped at KD_WCAP blocks of 4 arcs, the rest in a second pass (0: one pass)
#endif
#ifndef KD_SEEDSPIN
#define KD_SEEDSPIN 8  // seeded init: polls (s_sleep 8 each) of a second or third seed's flag before it is dropped (0: wait; round 4: C3 2.68 -> 2.53 ms, C4 44.7 -> 44.4)
#endif
#ifndef KD_WQ_N
#define KD_WQ_N 2
#endif
constexpr int KD_WQ = KD_WQ_N;        // phase C path walk: targets per thread (4 measured 1% slower at C4: its registers put 39 VGPRs of the output function in callee-saved ranges, saved to scratch and restored around every row; 2: 13)
constexpr int KD_ONE = 254;           // phase C: rtab slot holding 1.0 (the source's own step)
constexpr int KD_NAN = 255;           // phase C: rtab slot holding NaN (unreachable vertices)
constexpr int KD_RR = 512;  // parent-record ring slots (1024-thread workgroups; smaller ones use 256)
template <int B>
constexpr int kd_rr() { return B >= 1024 ? KD_RR : 256; }

// per-workgroup HBM slice: relv f64[n] | wpr u32[n + 8], the parent record of every vertex:
// parent | ridx << 16 (| w << 24, packed arcs) of the parent arc (KD_SRC_MARK for the source)
// | tie events
// {p | ridx << 16 | w << 24, v} x n (seeded rows) | a second record slice u32[n + 8] (rows
// alternate between the two).  Seeded rows use relv as u32 keys.
__host__ __device__ inline size_t kd_ws_stride(int n) {
    return a16(sizeof(double) * n) + a16(sizeof(uint32_t) * (n + 8)) + a16(8 * (size_t)n) + 256 +
           a16(sizeof(uint32_t) * (n + 8));
}
// the second record slice, after relv | wpr | events
__host__ __device__ inline size_t kd_ws_wpr1(int n) {
    return a16(sizeof(double) * n) + a16(sizeof(uint32_t) * (n + 8)) + a16(8 * (size_t)n) + 256;
}
__host__ __device__ inline long long kd_row_stride(int n) { return ((long long)n + 2 + 7) & ~7ll; }

// LDS-only workgroup barrier: outstanding global stores (output rows) stay in flight.
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ inline void wait_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ inline unsigned kd_wave_min(unsigned x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x = min(x, (unsigned)__shfl_xor((int)x, d, 64));
    return x;
}

// wave-wide min of a u32 with DPP row shifts/broadcasts (VALU only, no LDS round trips)
__device__ inline unsigned kd_wave_min_dpp(unsigned x) {
    int v = (int)x;
    const int inf = (int)0xFFFFFFFFu;
    v = (int)min((unsigned)v, (unsigned)__builtin_amdgcn_update_dpp(inf, v, 0x111, 0xF, 0xF, false));  // row_shr:1
    v = (int)min((unsigned)v, (unsigned)__builtin_amdgcn_update_dpp(inf, v, 0x112, 0xF, 0xF, false));  // row_shr:2
    v = (int)min((unsigned)v, (unsigned)__builtin_amdgcn_update_dpp(inf, v, 0x114, 0xF, 0xF, false));  // row_shr:4
    v = (int)min((unsigned)v, (unsigned)__builtin_amdgcn_update_dpp(inf, v, 0x118, 0xF, 0xF, false));  // row_shr:8
    v = (int)min((unsigned)v, (unsigned)__builtin_amdgcn_update_dpp(inf, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = (int)min((unsigned)v, (unsigned)__builtin_amdgcn_update_dpp(inf, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return (unsigned)__builtin_amdgcn_readlane(v, 63);
}

// wave-wide inclusive prefix sum with DPP row shifts/broadcasts: VALU only (a __shfl_up
// scan is six dependent ds_bpermute round trips through the LDS crossbar)
__device__ inline int kd_wave_incl_sum(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return x;
}

// wave-wide inclusive prefix max of non-negative ints, as kd_wave_incl_sum
__device__ inline int kd_wave_incl_max(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false));
    return x;
}

// ob[p] = x of lane own[p], od[p] = y of lane own[p] for the KD_P steps: all 16 crossbar
// reads issued back to back with one wait (left to the compiler, register pressure makes
// it wait after every pair, i.e. eight LDS round trips in a row)
__device__ inline void kd_bpermute16(const int own[8], int x, int y, int ob[8], uint32_t od[8]) {
    int a[8];
#pragma unroll
    for (int p = 0; p < 8; p++) a[p] = own[p] << 2;
    asm volatile(
        "ds_bpermute_b32 %0, %16, %24\n\t"
        "ds_bpermute_b32 %1, %16, %25\n\t"
        "ds_bpermute_b32 %2, %17, %24\n\t"
        "ds_bpermute_b32 %3, %17, %25\n\t"
        "ds_bpermute_b32 %4, %18, %24\n\t"
        "ds_bpermute_b32 %5, %18, %25\n\t"
        "ds_bpermute_b32 %6, %19, %24\n\t"
        "ds_bpermute_b32 %7, %19, %25\n\t"
        "ds_bpermute_b32 %8, %20, %24\n\t"
        "ds_bpermute_b32 %9, %20, %25\n\t"
        "ds_bpermute_b32 %10, %21, %24\n\t"
        "ds_bpermute_b32 %11, %21, %25\n\t"
        "ds_bpermute_b32 %12, %22, %24\n\t"
        "ds_bpermute_b32 %13, %22, %25\n\t"
        "ds_bpermute_b32 %14, %23, %24\n\t"
        "ds_bpermute_b32 %15, %23, %25\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(ob[0]), "=&v"(od[0]), "=&v"(ob[1]), "=&v"(od[1]), "=&v"(ob[2]), "=&v"(od[2]),
          "=&v"(ob[3]), "=&v"(od[3]), "=&v"(ob[4]), "=&v"(od[4]), "=&v"(ob[5]), "=&v"(od[5]),
          "=&v"(ob[6]), "=&v"(od[6]), "=&v"(ob[7]), "=&v"(od[7])
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
          "v"(x), "v"(y));
}

__device__ inline unsigned ld16(const uint16_t* d, int v) { return d[v]; }
// component k (a constant after unrolling) of a uint4 without taking its address (an
// address-taken register array lands in scratch memory)
__device__ inline uint32_t kd_comp(const uint4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// pop up to four set bits of *b (lowest first) into v[] as vertex ids of word k (-1 = none)
__device__ inline void pop4(unsigned long long* b, int k, int v[4]) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const unsigned long long x = *b;
        v[q] = x ? (k << 6) + __ffsll((long long)x) - 1 : -1;
        *b = x & (x - 1);
    }
}

// Relax the wave's list of improving arcs {v | nd << 16}: a CAS on the u32 word holding
// dist[v] (retry while still an improvement), then below T -> work queue (one reservation
// for the whole pass), else -> pending bitmask.  Entries may repeat a vertex; the CAS sorts
// them out.  Called by a whole wave (ballots); `cnt` is wave-uniform.
__device__ inline void kd_relax_list(const uint32_t* wimp, int cnt, int lane, unsigned long long upto,
                                     uint32_t* dist32, unsigned long long* pend, unsigned* wmin, uint16_t* ring,
                                     int* tail, int rc, unsigned T, unsigned long long* sm_acc) {
    __builtin_amdgcn_wave_barrier();
    for (int b0 = 0; b0 < cnt; b0 += 64) {
        const bool act = b0 + lane < cnt;
        const uint32_t e = act ? wimp[b0 + lane] : 0u;
        const unsigned v = e & 0xFFFFu, nd = e >> 16, sh = (v & 1u) << 4;
        bool won = false;
        if (act) {
            uint32_t old = dist32[v >> 1];
            for (;;) {
                if (nd >= ((old >> sh) & 0xFFFFu)) break;
                const uint32_t got = atomicCAS(&dist32[v >> 1], old, (old & ~(0xFFFFu << sh)) | (nd << sh));
                if (got == old) { won = true; break; }
                old = got;
            }
        }
        const bool push = won && nd < T;
        if (won && nd >= T) { atomicOr(&pend[v >> 6], 1ull << (v & 63)); atomicMin(&wmin[v >> 6], nd); }
        const unsigned long long pm = __ballot(push);
        if (pm) {
            const int ctot = __popcll(pm);
            // reservation: tail may run past rc; readers clamp it, entries past rc stay pending
            int qb = 0;
            if (lane == 0) qb = atomicAdd(tail, ctot);
            qb = __builtin_amdgcn_readfirstlane(qb);
            const int qk = max(0, min(ctot, rc - qb));
            const int rk = __popcll(pm & (upto >> 1));
            // one copy of the vertex: the queue's (else the pending bitmask)
            if (push && rk < qk) { ring[qb + rk] = (uint16_t)v; atomicAnd(&pend[v >> 6], ~(1ull << (v & 63))); }
            if (push && rk >= qk) { atomicOr(&pend[v >> 6], 1ull << (v & 63)); atomicMin(&wmin[v >> 6], nd); }
#ifdef SHD_STAMPS
            if (lane == 0 && ctot > qk) atomicAdd(&sm_acc[14], (unsigned long long)(ctot - qk));
#endif
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// planned launches (jobs): every job from the queue, in queue order, so a job a workgroup
// waits on (its seed) was taken earlier by a running workgroup: no residency assumption

// the current job's seeds, from its LDS copy (wave-uniform: scalar registers)
#define SEED_VIEW()                                                                                   \
    const int nseed = __builtin_amdgcn_readfirstlane(sm->job.nseed);                                   \
    int su[KD_SEEDS], sslot[KD_SEEDS];                                                                 \
    unsigned wsu[KD_SEEDS], rsu[KD_SEEDS];                                                             \
    const uint16_t* sdrow[KD_SEEDS];                                                                   \
    const uint32_t* sprow[KD_SEEDS];                                                                   \
    _Pragma("unroll") for (int q_ = 0; q_ < KD_SEEDS; q_++) {                                          \
        const int sl_ = __builtin_amdgcn_readfirstlane(q_ < nseed ? sm->job.seed[q_] : 0);             \
        const unsigned wr_ = (unsigned)__builtin_amdgcn_readfirstlane(q_ < nseed ? sm->job.wr[q_] : 0); \
        su[q_] = __builtin_amdgcn_readfirstlane(q_ < nseed ? sm->job.u[q_] : -1);                      \
        sslot[q_] = sl_; wsu[q_] = wr_ & 0xFFFFu;                                                      \
        rsu[q_] = (unsigned)__builtin_amdgcn_readfirstlane(q_ < nseed ? sm->job.rec[q_] : 0);          \
        sdrow[q_] = g.drow + (size_t)sl_ * g.rstride;                                                  \
        sprow[q_] = g.prow + (size_t)sl_ * g.rstride;                                                  \
    }                                                                                                  \
    (void)sslot; (void)rsu; (void)sprow; (void)su

__device__ inline int kd_next_source(int* ctr, int* slot, int tid, bool all_queued = false) {
    if (tid == 0) *slot = (all_queued ? 0 : (int)gridDim.x) + atomicAdd(ctr, 1);
    __syncthreads();
    const int i = *slot;
    __syncthreads();  // every thread has read it before thread 0 writes the next one
    return i;
}

// Phases C/D of one row (lat row, parent copy, reliability by walks or level sweeps, rel
// row, row min), called once per row.  Not inlined, on purpose: see the call site.
template <int B>
__device__ __attribute__((noinline)) void kd_output(const int i, const int s, const double cs, const double sw_s,
                                                    const double sr_s, const KD_GLOBAL uint32_t* __restrict__ wpr) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int RR = kd_rr<B>();
    KDSmall* sm = reinterpret_cast<KDSmall*>(smem);
    // the launch-invariant arguments out of LDS, as wave-uniform (scalar) values
    auto uni = [](auto x) __attribute__((always_inline)) {
        using T = decltype(x);
        if constexpr (sizeof(T) == 8) {
            unsigned long long b;
            __builtin_memcpy(&b, &x, 8);
            b = (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b) |
                ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32)) << 32);
            T y;
            __builtin_memcpy(&y, &b, 8);
            return y;
        } else {
            return (T)__builtin_amdgcn_readfirstlane((int)x);
        }
    };
    const KDOut& O = sm->out;
    const KD_GLOBAL int* __restrict__ const tgt = uni(O.tgt);
    KD_GLOBAL double* __restrict__ const lat_out = uni(O.lat_out);
    KD_GLOBAL double* __restrict__ const rel_out = uni(O.rel_out);
    KD_GLOBAL double* __restrict__ const row_min = uni(O.row_min);
    int* __restrict__ const err = uni(O.err);
    KD_GLOBAL double* __restrict__ const relv = uni(O.relv);
    const KD_GLOBAL double* __restrict__ const rtab = uni(O.rtab);
    const KD_GLOBAL double* __restrict__ const vf = uni(O.vf);
    const long long ld = uni(O.ld);
    const int n = uni(O.n), nw = uni(O.nw), nt = uni(O.nt), tsorted = uni(O.tsorted);
    const unsigned rmask = uni(O.rmask);
    const int rc = uni(O.rc), walk = uni(O.walk), nrtab = uni(O.nrtab), rone = uni(O.rone);
    const int has_vf = uni(O.has_vf), dflags = uni(O.dflags);
    const KDLayout<B> L = KDLayout<B>::make(n, rc, RR);
    const int tid = threadIdx.x, lane = tid & 63;
    uint16_t* dist = reinterpret_cast<uint16_t*>(smem + L.dist);
    unsigned long long* pend = reinterpret_cast<unsigned long long*>(smem + L.pend);
    unsigned long long* fix = reinterpret_cast<unsigned long long*>(smem + L.fix);
    uint16_t* qv = reinterpret_cast<uint16_t*>(smem + L.qv);
    const unsigned long long* tmask = reinterpret_cast<const unsigned long long*>(smem + L.tmask);
    const unsigned* tpre = reinterpret_cast<const unsigned*>(smem + L.tpre);
    const int qcap = L.qcap;
    auto tpos = [&](int v) __attribute__((always_inline)) {
        const unsigned long long wd = tmask[v >> 6], bit = 1ull << (v & 63);
        return (wd & bit) ? (int)tpre[v >> 6] + __popcll(wd & (bit - 1ull)) : -1;
    };
    struct { int walk; const KD_GLOBAL double* rtab; int nrtab; const KD_GLOBAL double* vf; int has_vf; } g = {walk, rtab, nrtab, vf, has_vf};
#ifdef SHD_STAMPS
    unsigned long long kd_t = __builtin_amdgcn_s_memtime();
#endif
    (void)lane; (void)dflags;
    // helper rows (i < 0, multi-GPU plans) only seed others: no output, no phase C
    KD_GLOBAL double* lrow = lat_out && i >= 0 ? lat_out + (long long)i * ld : nullptr;
    KD_GLOBAL double* rrow = rel_out && i >= 0 ? rel_out + (long long)i * ld : nullptr;
    double lmin = INFINITY;
    auto lat_of = [&](int t) __attribute__((always_inline)) {
        double Lv;
        if (t < 0 || t >= n) { raise_err(err, SHD_ROUTE_EINVAL); Lv = NAN; }
        else if (t == s) {
            if (isnan(sw_s)) { raise_err(err, SHD_ROUTE_ENOEDGE); Lv = NAN; }
            else { Lv = 0.0 + sw_s; lmin = fmin(lmin, Lv); }
        } else if (dist[t] == 0xFFFFu) { raise_err(err, SHD_ROUTE_EUNREACH); Lv = NAN; }
        else { Lv = (double)dist[t]; lmin = fmin(lmin, Lv); }
        return Lv;
    };
    // phase B's parent records (wpr) visible to every wave (loading the parent copy's first
    // trip here, under the lat row, measured slower: its registers cost callee saves, 41.5 ->
    // 41.8 ms at C4)
    const bool walks = g.walk && rrow;
    // (a kept row's lat row written last, from its row store, so that the parent copy's loads
    // do not queue behind the lat row's stores, measured slower: C4 41.69 against 41.30 ms)
    wait_stores();
    __syncthreads();
    if (tsorted) {
        // two vertex pairs per lane, 128 vertices apart, so that each of the wave's two 16-B
        // store instructions covers 1 KB of consecutive positions: full lines (four adjacent
        // vertices per lane, round 5's first form, split every line over two instructions and
        // each half went to HBM on its own: C4 writes 75.6 -> 58.7 GB per launch, 41.9 -> 41.5 ms)
        const int lpar = (int)(((uintptr_t)lrow >> 3) & 1);
        const int wv = tid >> 6;
        for (int b0 = 256 * wv; b0 < (i >= 0 ? n : 0); b0 += 256 * (B / 64)) {
#pragma unroll
            for (int p = 0; p < 2; p++) {
                const int v = b0 + 128 * p + 2 * lane;
                if (v >= n) continue;
                const unsigned long long wd = tmask[v >> 6];
                const int sh = v & 63;
                const int j = (int)tpre[v >> 6] + __popcll(wd & ((1ull << sh) - 1ull));
                const uint32_t d2 = *reinterpret_cast<const uint32_t*>(dist + v);
                int jq[2];
                double Lq[2];
                int jn = j;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int vv = v + h;
                    const bool tg = vv < n && ((wd >> (sh + h)) & 1ull);
                    jq[h] = tg ? jn++ : -1;
                    const unsigned d = (d2 >> (16 * h)) & 0xFFFFu;
                    double Lv = 0.0;
                    if (tg) {
                        if (vv == s) {
                            if (isnan(sw_s)) { raise_err(err, SHD_ROUTE_ENOEDGE); Lv = NAN; }
                            else { Lv = 0.0 + sw_s; lmin = fmin(lmin, Lv); }
                        } else if (d == 0xFFFFu) { raise_err(err, SHD_ROUTE_EUNREACH); Lv = NAN; }
                        else { Lv = (double)d; lmin = fmin(lmin, Lv); }
                    }
                    Lq[h] = Lv;
                }
                if (!lrow || !KD_OUT) continue;
                const int ja = jq[0], jb = jq[1];
                if (ja >= 0 && jb == ja + 1 && !((ja + lpar) & 1))
                    __builtin_nontemporal_store(kd_d2{Lq[0], Lq[1]}, reinterpret_cast<KD_GLOBAL kd_d2*>(lrow + ja));
                else {
                    if (ja >= 0) __builtin_nontemporal_store(Lq[0], lrow + ja);
                    if (jb >= 0) __builtin_nontemporal_store(Lq[1], lrow + jb);
                }
            }
        }
    } else {
        for (int j = tid; j < (i >= 0 ? nt : 0); j += B) {
            const double Lv = lat_of(tgt[j]);
            if (lrow && KD_OUT) __builtin_nontemporal_store(Lv, lrow + j);
        }
    }
    // planned launches: the next job is taken here (queue order is unchanged: a job is still
    // taken after every job it seeds from)
    const bool queued = sm->jobs != nullptr;
    if (tid == 0) {
        sm->deep = 0; sm->rmin = kInfBits; sm->wnext = 0; sm->wnext2 = 0; sm->novf = 0;
        if (queued) sm->njb = atomicAdd(sm->qnext, 1);
    }
    __syncthreads();
    const int njb = queued ? __builtin_amdgcn_readfirstlane(sm->njb) : -1;
    if (tid < 16 && njb >= 0) {
        const int x = njb < sm->ns ? ((const KD_GLOBAL int*)(sm->jobs + njb))[tid] : (tid == 3 ? 0 : -1);
        reinterpret_cast<int*>(&sm->njob)[tid] = x;  // (past the end: nseed = 0)
    }

    KD_ACC(18);
    // dist is dead: its LDS becomes the parent array
    uint16_t* parv = dist;
    if (walks) {
        // ---- C': reliability by walking each target's tree path in LDS -------------
        // parv u16 + rix u8 (index of the parent arc's reliability) + rtab in LDS; each
        // target walks <= KD_MAXD arcs to the source, then folds the product source-first
        // (the order the level sweep multiplies in, so the bits agree)
        // rtl[KD_ONE] = 1.0 is the source's own "arc" (a walk parked at the source keeps
        // multiplying by an exact 1.0) and rtl[KD_NAN] marks unreachable vertices
        uint8_t* rixl = reinterpret_cast<uint8_t*>(smem + L.rix);
        double* rtl = reinterpret_cast<double*>(smem + L.rtabl);
        for (int k = tid; k < 256; k += B)
            rtl[k] = k < g.nrtab ? g.rtab[k] : k == KD_ONE ? 1.0 : NAN;
        // 4 consecutive vertices per 16-B record load, 2 loads per half-trip and thread (8 K
        // vertices), the next half-trip's loads issued before this one's copy
        // (wpr rows hold n + 8 records, dist n + 1 entries padded to 16 B: the last group's
        // reads stay inside; its writes past n are dropped)
        auto copy_trip = [&](const int v0, const auto& pr) __attribute__((always_inline)) {
            constexpr int NQ = sizeof(pr) / sizeof(pr[0]);
            uint2 dv[NQ];
#pragma unroll
            for (int q = 0; q < NQ; q++) dv[q] = *reinterpret_cast<const uint2*>(dist + min(v0 + q * 4 * B, (n - 1) & ~3));
            // (each thread overwrites only the dist entries it read itself)
#pragma unroll
            for (int q = 0; q < NQ; q++) {
                const int vb = v0 + q * 4 * B;
                if (vb >= n) continue;
                uint32_t pw[2] = {0u, 0u}, rw = 0u;
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    const int v = vb + h;
                    const uint32_t p = h == 0 ? pr[q].x : h == 1 ? pr[q].y : h == 2 ? pr[q].z : pr[q].w;
                    const uint32_t d = ((h < 2 ? dv[q].x : dv[q].y) >> (16 * (h & 1))) & 0xFFFFu;
                    const bool src_v = v == s, unr = !src_v && d == 0xFFFFu;
                    const uint32_t pv = src_v || unr ? (uint32_t)s : (p & 0xFFFFu);
                    // an arc of reliability exactly 1.0 folds as the KD_ONE slot (same factor)
                    const uint32_t ri = min((p >> 16) & rmask, (uint32_t)(g.nrtab - 1));
                    const uint32_t rx = src_v ? (uint32_t)KD_ONE : unr ? (uint32_t)KD_NAN
                                        : ri == (uint32_t)rone ? (uint32_t)KD_ONE : ri;
                    pw[h >> 1] |= pv << (16 * (h & 1));
                    rw |= rx << (8 * h);
                }
                if (vb + 4 <= n) {
                    *reinterpret_cast<uint2*>(parv + vb) = make_uint2(pw[0], pw[1]);
                    *reinterpret_cast<uint32_t*>(rixl + vb) = rw;
                } else {
                    for (int h = 0; h < n - vb; h++) {
                        parv[vb + h] = (uint16_t)((pw[h >> 1] >> (16 * (h & 1))) & 0xFFFFu);
                        rixl[vb + h] = (uint8_t)((rw >> (8 * h)) & 0xFFu);
                    }
                }
            }
        };
        auto load_trip = [&](const int v0, auto& pr) __attribute__((always_inline)) {
            constexpr int NQ = sizeof(pr) / sizeof(pr[0]);
#pragma unroll
            for (int q = 0; q < NQ; q++)
                if constexpr (B >= 1024 && KD_NTLOAD)  // (streamed, as the seeded init's loads: C4 41.23 -> 41.13 ms)
                    pr[q] = __builtin_nontemporal_load(reinterpret_cast<const KD_GLOBAL kd_u4*>(wpr + min(v0 + q * 4 * B, (n - 1) & ~3)));
                else
                    pr[q] = *reinterpret_cast<const KD_GLOBAL kd_u4*>(wpr + min(v0 + q * 4 * B, (n - 1) & ~3));
        };
        {
            // the next half-trip's records in flight while this one is copied (two 16-B
            // records per lane and half-trip: four, or one-trip lookahead at four, raised the
            // callee saves, kernel scratch 152 -> 260 B/lane; C3 2.09 -> 2.02 ms, C4 the same)
            constexpr int PQ = 2;
            kd_u4 pa[PQ], pb[PQ];
            int v0 = 4 * tid;
            if (v0 < n) load_trip(v0, pa);
            for (; v0 < n; v0 += 8 * PQ * B) {
                const int v1 = v0 + 4 * PQ * B;
                if (v1 < n) load_trip(v1, pb);
                copy_trip(v0, pa);
                if (v1 >= n) break;
                if (v1 + 4 * PQ * B < n) load_trip(v1 + 4 * PQ * B, pa);
                copy_trip(v1, pb);
            }
        }
        __syncthreads();
        // Lossless arcs (slot KD_ONE: exactly 1.0) multiply as exact no-ops, so a chain only
        // needs the lossy ones (20% of the arcs on the BASELINE topologies): parv[v] becomes the
        // nearest proper ancestor whose own arc is lossy (or s) by pointer jumping, each round
        // doubling the lossless runs skipped (4-6 rounds).  A jump reads a pointer that may be
        // mid-update in another thread; the old and the new value both skip only lossless
        // vertices, so any interleaving gives the same products.  Run to convergence the
        // walks below would take ~2.2 arcs per target instead of ~9.5 (wave maxima 6-7 vs ~18),
        // but every round is a full pass of two LDS gathers per vertex, bank-conflict bound
        // like the walk steps it saves: one round pays (KD_JUMPS).  (Path halving inside the
        // walks instead, writing the skip back, measured the same as one round; both together
        // slower.)
        {
            const int per = (n + B - 1) / B;  // vertices per thread: v = tid + k * B
            unsigned long long live = per >= 64 ? ~0ull : ((1ull << per) - 1ull);
            if (tid < 3) sm->jflag[tid] = 0;
            __syncthreads();
            // (round r raises slot r % 3 and clears slot (r + 1) % 3 before its barrier: the
            // slot of round r - 1 may still be read after that barrier)
            for (int rnd = 0; rnd < KD_JUMPS; rnd++) {
                int any = 0;
                for (int k0 = 0; k0 < per; k0 += 4) {
                    const unsigned lb = k0 < 64 ? (unsigned)((live >> k0) & 0xFull) : 0xFu;
                    if (!lb) continue;
                    int vq[4], jq[4];
                    bool act[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        vq[q] = tid + (k0 + q) * B;
                        act[q] = ((lb >> q) & 1u) && vq[q] < n;
                        jq[q] = act[q] ? (int)parv[vq[q]] : s;
                    }
                    unsigned rq[4], jj[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) { rq[q] = rixl[jq[q]]; jj[q] = parv[jq[q]]; }
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        if (!act[q]) {
                            if (k0 + q < 64) live &= ~(1ull << (k0 + q));
                        } else if (jq[q] == s || rq[q] != (unsigned)KD_ONE) {
                            if (k0 + q < 64) live &= ~(1ull << (k0 + q));
                        } else {
                            parv[vq[q]] = (uint16_t)jj[q];
                            any = 1;
                        }
                    }
                }
                if (any) sm->jflag[rnd % 3] = 1;
                if (tid == 0) sm->jflag[(rnd + 1) % 3] = 0;
                __syncthreads();
                if (!sm->jflag[rnd % 3]) break;
            }
        }
        KD_ACC(19);
        // sorted targets: one pass over the vertices, positions from the LDS mask (no
        // global load behind the previous group's stores); else over the target list
        const int lim = tsorted ? n : nt;
        const int rpar = (int)(((uintptr_t)rrow >> 3) & 1);
        // one set of KD_WQ chains per thread: walk <= NB blocks of 4 arcs, fold source-first,
        // store.  In a capped first pass (ovl != nullptr) a chain still short of the source
        // after NB blocks is listed in ovl (v | j << 16) instead of stored, and the second pass
        // walks the listed chains again in dense waves: a wave then runs for its deepest
        // ordinary chain, not for the deepest chain of any 128 targets (KD_WCAP)
        auto walk_set = [&](auto NBC, int (&t2)[KD_WQ], int (&jq)[KD_WQ], KD_GLOBAL uint32_t* ovl) __attribute__((always_inline)) {
            constexpr int NB = decltype(NBC)::value;
            int cur[KD_WQ];
            uint32_t pk[KD_WQ][NB];
#pragma unroll
            for (int q = 0; q < KD_WQ; q++) {
                cur[q] = t2[q] >= 0 && t2[q] < n ? t2[q] : s;
#pragma unroll
                for (int k = 0; k < NB; k++) pk[q][k] = 0u;
            }
            // blocks of 4 arcs (parked chains multiply an exact 1.0, so the padding is
            // harmless): one packed word per chain and block keeps the loop off the VALU
            int nb = 0;  // blocks walked, wave-uniform (unrolled: pk stays in registers)
#pragma unroll
            for (int b = 0; b < NB; b++) {
                bool any = false;
#pragma unroll
                for (int q = 0; q < KD_WQ; q++) any = any || cur[q] != s;
                if (!__any(any)) break;
                uint32_t acc[KD_WQ];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    uint32_t p[KD_WQ], rx[KD_WQ];
#pragma unroll
                    for (int q = 0; q < KD_WQ; q++) { p[q] = parv[cur[q]]; rx[q] = rixl[cur[q]]; }
#pragma unroll
                    for (int q = 0; q < KD_WQ; q++) {
                        acc[q] = e == 0 ? rx[q] : (acc[q] | (rx[q] << (8 * e)));
                        cur[q] = (int)p[q];
                    }
                }
#pragma unroll
                for (int q = 0; q < KD_WQ; q++) pk[q][b] = acc[q];
                nb = b + 1;
            }
            if (ovl) {
#pragma unroll
                for (int q = 0; q < KD_WQ; q++) {
                    const bool more = cur[q] != s;  // (t2 >= 0: parked chains sit at s)
                    const unsigned long long m = __ballot(more);
                    if (m) {
                        int base = 0;
                        if (lane == 0) base = atomicAdd(&sm->novf, __popcll(m));
                        base = __builtin_amdgcn_readfirstlane(base);
                        if (more) {
                            const int at = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                            // sorted targets: vertex | position << 16 (both < n <= 65535);
                            // a caller's list: the full 32-bit position (the vertex is
                            // tgt[position]), since such a list may exceed 65535 entries
                            ovl[at] = tsorted ? (uint32_t)t2[q] | ((uint32_t)jq[q] << 16) : (uint32_t)jq[q];
                            jq[q] = -1;  // stored by the second pass
                        }
                    }
                }
            } else {
                bool any = false;
#pragma unroll
                for (int q = 0; q < KD_WQ; q++) any = any || cur[q] != s;
                if (any) sm->deep = 1;  // the level sweep below redoes the row
            }
            // the fold starts from (1.0 * f_s) * f_t: the reference multiplies both vertex
            // factors before the first arc (topology.c:1443-1462, then :1499), so a walked
            // row is bit-exact under vertex loss too (the level sweep below multiplies f_t
            // last: within 1e-12)
            double f2[KD_WQ];
#pragma unroll
            for (int q = 0; q < KD_WQ; q++) f2[q] = g.has_vf ? g.vf[(t2[q] >= 0 && t2[q] < n) ? t2[q] : s] : (double)NAN;
            double rr[KD_WQ];
#pragma unroll
            for (int q = 0; q < KD_WQ; q++) rr[q] = isnan(f2[q]) ? cs : cs * f2[q];
#pragma unroll
            for (int k4 = NB - 1; k4 >= 0; k4--) {  // source-first: the last arc walked first
                if (k4 >= nb) continue;  // (uniform)
                uint32_t wq[KD_WQ];
#pragma unroll
                for (int q = 0; q < KD_WQ; q++) wq[q] = pk[q][k4];
#pragma unroll
                for (int e = 3; e >= 0; e--) {
                    // (arcs of reliability exactly 1.0 read the KD_ONE slot, as parked chains
                    // do: one shared address, a broadcast)
                    double x[KD_WQ];
#pragma unroll
                    for (int q = 0; q < KD_WQ; q++) x[q] = rtl[(wq[q] >> (8 * e)) & 0xFFu];
#pragma unroll
                    for (int q = 0; q < KD_WQ; q++) rr[q] *= x[q];
                }
            }
            double Rv[KD_WQ];
#pragma unroll
            for (int q = 0; q < KD_WQ; q++) {
                const int t = t2[q];
                Rv[q] = NAN;
                if (t >= 0 && t < n) {
                    if (t == s) Rv[q] = isnan(sw_s) ? NAN : cs * sr_s;
                    else Rv[q] = rr[q];
                }
            }
            if (KD_OUT) {
#pragma unroll
                for (int q = 0; q < KD_WQ; q += 2) {
                    const int ja = jq[q], jb = jq[q + 1];
                    if (tsorted && ja >= 0 && jb == ja + 1 && !((ja + rpar) & 1))
                        __builtin_nontemporal_store(kd_d2{Rv[q], Rv[q + 1]}, reinterpret_cast<KD_GLOBAL kd_d2*>(rrow + ja));
                    else {
                        if (ja >= 0) __builtin_nontemporal_store(Rv[q], rrow + ja);
                        if (jb >= 0) __builtin_nontemporal_store(Rv[q + 1], rrow + jb);
                    }
                }
            }
        };
        // blocks of KD_WQ x WB targets: the whole workgroup's threads share a block in turn
        // (static), or each wave takes the next block of KD_WQ x 64 from a counter (wdyn: a
        // wave of shallow chains takes more blocks, no wave waits at the barrier for another)
        constexpr bool wdyn = KD_WDYN != 0;
        const int WB = wdyn ? 64 : B;
        const int li = wdyn ? lane : tid;  // this thread's place in its block
        // (capped first pass: its list over relv's HBM slice, unused by the walks; the slice
        // holds 2n entries, and a list gets at most one per target position, so a caller's
        // unsorted list longer than 2n (duplicates) walks uncapped in one pass instead)
        KD_GLOBAL uint32_t* const ovl =
            KD_WCAP > 0 && (tsorted || nt <= 2 * n) ? reinterpret_cast<KD_GLOBAL uint32_t*>(relv) : nullptr;
        auto grab = [&]() __attribute__((always_inline)) {
            int c = 0;
            if (lane == 0) c = atomicAdd(&sm->wnext, 1);
            return __builtin_amdgcn_readfirstlane(c) * (KD_WQ * 64);
        };
        for (int blk = 0;; blk++) {
            int jbase;
            if constexpr (wdyn) jbase = grab();
            else jbase = blk * (KD_WQ * B);
            if (jbase >= lim) break;
            const int j0 = jbase + li;
            // KD_WQ targets per thread: independent parent chains in flight.  A chain that
            // reaches the source stays there (parv[s] = s, factor 1.0), so a step is two LDS
            // reads and a byte insert, and the wave stops when every chain is parked.
            int t2[KD_WQ], jq[KD_WQ];
#pragma unroll
            for (int q = 0; q < KD_WQ; q++) {
                const int j = j0 + q * WB;
                if (tsorted) {
                    // chains (0, 1) and (2, 3) are adjacent vertices: paired 16-B stores
                    const int v = jbase + (q >> 1) * 2 * WB + 2 * li + (q & 1);
                    jq[q] = v < n ? tpos(v) : -1;
                    t2[q] = jq[q] >= 0 ? v : -1;
                } else {
                    jq[q] = j < nt ? j : -1;
                    t2[q] = j < nt ? tgt[j] : -1;
                }
            }
            if (KD_WCAP > 0 && ovl) walk_set(std::integral_constant<int, (KD_WCAP > 0 ? KD_WCAP : 1)>{}, t2, jq, ovl);
            else walk_set(std::integral_constant<int, KD_MAXD / 4>{}, t2, jq, nullptr);
        }
        if (KD_WCAP > 0 && ovl) {
            // second pass: the listed chains, 128 per wave-block, walked in full
            wait_stores();  // (the list, in HBM, visible to every wave)
            __syncthreads();
            const int novf = sm->novf;
            for (;;) {
                int c = 0;
                if (lane == 0) c = atomicAdd(&sm->wnext2, 1);
                const int e0 = __builtin_amdgcn_readfirstlane(c) * (KD_WQ * 64);
                if (e0 >= novf) break;
                int t2[KD_WQ], jq[KD_WQ];
#pragma unroll
                for (int q = 0; q < KD_WQ; q++) {
                    const int e = e0 + q * 64 + lane;
                    const uint32_t x = e < novf ? ovl[e] : 0xFFFFFFFFu;
                    if (tsorted) {
                        t2[q] = e < novf ? (int)(x & 0xFFFFu) : -1;
                        jq[q] = e < novf ? (int)(x >> 16) : -1;
                    } else {
                        jq[q] = e < novf ? (int)x : -1;
                        t2[q] = e < novf ? tgt[x] : -1;
                    }
                }
                walk_set(std::integral_constant<int, KD_MAXD / 4>{}, t2, jq, nullptr);
            }
        }
#ifdef SHD_STAMPS
        if (tid == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); sm->acc[32] += t_ - kd_t; kd_t = t_; }
#endif
        __syncthreads();
#ifdef SHD_STAMPS
        if (tid == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); sm->acc[33] += t_ - kd_t; kd_t = t_; }
#endif
        KD_ACC(13);
        KD_STAMP(3);
    }
    const bool sweep = i >= 0 && (!(g.walk && rrow) || sm->deep);
    if (sweep) {
    // parent records: parent | ridx << 16 (writer wave and phase B), KD_SRC_MARK at s
    for (int v0 = tid; v0 < n; v0 += B * 8) {
        uint32_t pr[8];
#pragma unroll
        for (int q = 0; q < 8; q++) pr[q] = wpr[min(v0 + q * B, n - 1)];
        double rr[8];
#pragma unroll
        for (int q = 0; q < 8; q++) rr[q] = g.rtab[min((int)((pr[q] >> 16) & rmask), g.nrtab - 1)];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int v = v0 + q * B;
            if (v >= n) continue;
            const bool src_v = pr[q] == KD_SRC_MARK;
            parv[v] = src_v ? (uint16_t)v : (uint16_t)(pr[q] & 0xFFFFu);
            relv[v] = src_v ? cs : -rr[q];
        }
    }
    for (int k = tid; k < nw; k += B) {
        unsigned long long mk = (k == nw - 1 && (n & 63)) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
        if (k == (s >> 6)) mk &= ~(1ull << (s & 63));
        pend[k] = mk;
        fix[k] = 0ull;
    }
    wait_stores();
    __syncthreads();
    KD_ACC(19);

    if (tid == 0) sm->qtail[0] = sm->qtail[1] = 0;
    lds_barrier();
    // ---- C: reliability down the tree ------------------------------------------
    // per level: pending vertices whose parent is done are compacted into qv, then one
    // thread per listed vertex loads relv[parent] and its own -r and stores the product
    for (int c = 0;; c ^= 1) {
        KD_COUNT(12, tid == 0 ? 1 : 0);
        if (tid == 0) sm->qtail[c ^ 1] = 0;
        for (int k0 = 0; k0 < nw; k0 += B) {
            const int k = k0 + tid;
            unsigned long long b = k < nw ? pend[k] : 0ull, ready = 0ull;
            while (b) {  // ready = pending vertices whose parent is done (LDS only)
                int v4[4];
                pop4(&b, k, v4);
                int p4[4];
#pragma unroll
                for (int q = 0; q < 4; q++) p4[q] = (int)parv[v4[q] >= 0 ? v4[q] : 0];
                unsigned long long pw[4];
#pragma unroll
                for (int q = 0; q < 4; q++) pw[q] = pend[p4[q] >> 6];
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (v4[q] >= 0 && !((pw[q] >> (p4[q] & 63)) & 1ull)) ready |= 1ull << (v4[q] & 63);
            }
            const int cnt = __popcll(ready);
            int incl = kd_wave_incl_sum(cnt);
            int base = 0;
            if (lane == 63 && incl) base = atomicAdd(&sm->qtail[c], incl);
            base = __builtin_amdgcn_readlane(base, 63);
            int pos = base + incl - cnt;
            unsigned long long listed = 0ull;
            b = ready;
            while (b && pos < qcap) {
                const int bi = __ffsll((long long)b) - 1;
                b &= b - 1;
                qv[pos++] = (uint16_t)((k << 6) + bi);
                listed |= 1ull << bi;
            }
            if (k < nw) fix[k] = listed;
        }
        lds_barrier();
        KD_ACC(13);
        const int cnt = min(sm->qtail[c], qcap);
        if (cnt == 0) break;
        for (int j0 = 0; j0 < cnt; j0 += B * 4) {
            int v4[4], p4[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int j = j0 + q * B + tid;
                v4[q] = j < cnt ? (int)qv[j] : -1;
                p4[q] = (int)parv[v4[q] >= 0 ? v4[q] : 0];
            }
            double xp[4], xv[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                xp[q] = relv[p4[q]];
                xv[q] = relv[v4[q] >= 0 ? v4[q] : 0];
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (v4[q] >= 0) relv[v4[q]] = xp[q] * (-xv[q]);
        }
        wait_stores();  // this level's relv visible before its vertices count as done
        KD_ACC(14);
        lds_barrier();
        for (int k = tid; k < nw; k += B) {
            const unsigned long long r = fix[k];
            if (r) pend[k] &= ~r;
        }
        lds_barrier();
        KD_ACC(15);
    }
    KD_STAMP(3);

    // ---- D: rel row out + row min ----------------------------------------------
    if (rrow) {
        for (int j0 = tid; j0 < nt; j0 += B * 4) {
            int t4[4];
            double x4[4], f4[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int j = j0 + q * B;
                t4[q] = j < nt ? tgt[j] : s;
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int t = (t4[q] >= 0 && t4[q] < n) ? t4[q] : s;
                x4[q] = relv[t];
                f4[q] = g.has_vf ? g.vf[t] : (double)NAN;
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int j = j0 + q * B;
                if (j >= nt) continue;
                const int t = t4[q];
                double Rv = NAN;
                if (t >= 0 && t < n) {
                    if (t == s) Rv = isnan(sw_s) ? NAN : cs * sr_s;
                    else Rv = isnan(f4[q]) ? x4[q] : x4[q] * f4[q];
                }
                if (KD_OUT) __builtin_nontemporal_store(Rv, rrow + j);
            }
        }
    }
    }  // sweep
    if (row_min && i >= 0) {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) lmin = fmin(lmin, __shfl_xor(lmin, d, 64));
        if (lane == 0 && lmin < INFINITY) atomicMin(&sm->rmin, as_u(lmin));
        __syncthreads();
        if (tid == 0) row_min[i] = as_d(sm->rmin);
    }
}

#define KD_KERNEL_PARAMS                                                                                   \
    DevDelta g, const int* __restrict__ src, int ns, const int* __restrict__ tgt, int nt, long long ld,     \
        double* __restrict__ lat_out, double* __restrict__ rel_out, double* __restrict__ row_min,          \
        int* __restrict__ err, char* __restrict__ ws, size_t ws_stride
template <int B>
__device__ __attribute__((always_inline)) inline void kd_rows_body(KD_KERNEL_PARAMS) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int n = g.n, nw = g.nw;
    constexpr int RR = kd_rr<B>();
    const KDLayout<B> L = KDLayout<B>::make(n, g.rc, RR);
    KDSmall* sm = reinterpret_cast<KDSmall*>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint32_t* wkey = reinterpret_cast<uint32_t*>(smem + L.wkey) + wid * 64;
    uint32_t* wimp = reinterpret_cast<uint32_t*>(smem + L.wimp) + wid * KD_IMP;
    uint16_t* dist = reinterpret_cast<uint16_t*>(smem + L.dist);
    uint32_t* wmark = reinterpret_cast<uint32_t*>(smem + L.wmark) + wid * 2 * KD_P;  // 64 x KD_P start bits
    unsigned long long* pend = reinterpret_cast<unsigned long long*>(smem + L.pend);
    unsigned* wmin = reinterpret_cast<unsigned*>(smem + L.wmin);
    unsigned long long* fix = reinterpret_cast<unsigned long long*>(smem + L.fix);
    uint16_t* ring = reinterpret_cast<uint16_t*>(smem + L.ring);
    uint2* rrec = reinterpret_cast<uint2*>(smem + L.rrec);
    uint16_t* qv = reinterpret_cast<uint16_t*>(smem + L.qv);
    int* qbeg = reinterpret_cast<int*>(smem + L.qbeg);
    unsigned long long* tmask = reinterpret_cast<unsigned long long*>(smem + L.tmask);
    unsigned* tpre = reinterpret_cast<unsigned*>(smem + L.tpre);
    const unsigned delta = (unsigned)g.delta;
    const int qcap = L.qcap;
    const unsigned wmask = g.packed ? 0xFFu : 0xFFFFu;
    // parent records: parent | ridx << 16 (| w << 24 with packed arcs: the tie-rule key of
    // a record is then a byte permutation of it)
    const unsigned rmask = g.packed ? 0xFFu : 0xFFFFu;
    const __amdgpu_buffer_rsrc_t orsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(g.orec), (short)0, g.nnz * 4, 0x00020000);
    const int rc = g.rc;
    constexpr int NW = B / 64;
    const bool writer = wid == NW - 1;  // drains parent records; never waits on a global load
    double* relv = reinterpret_cast<double*>(ws + (size_t)blockIdx.x * ws_stride);
    uint32_t* const wslice = reinterpret_cast<uint32_t*>(ws + (size_t)blockIdx.x * ws_stride + a16(sizeof(double) * n));
    uint2* const evl = reinterpret_cast<uint2*>(ws + (size_t)blockIdx.x * ws_stride + a16(sizeof(double) * n) +
                                                a16(sizeof(uint32_t) * (n + 8)));
#ifdef SHD_STAMPS
    if (tid < KD_NACC) sm->acc[tid] = 0;
    __syncthreads();
#endif
    const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);

    // the launch's target set, once per workgroup: a strictly increasing list (every
    // caller here passes the sorted attached set) becomes a bitmask + word prefix in LDS,
    // so the output loops find a target's position without a global load; any other list
    // takes the general loops (tgt[j] loads)
    for (int k = tid; k < nw; k += B) tmask[k] = 0ull;
    if (tid == 0) sm->tsorted = 1;
    __syncthreads();
    for (int j = tid; j < nt; j += B) {
        const int t = tgt[j];
        const bool ok = t >= 0 && t < n && (j == 0 || tgt[j - 1] < t);
        if (!ok) sm->tsorted = 0;  // (every writer stores 0)
        else atomicOr(&tmask[t >> 6], 1ull << (t & 63));
    }
    __syncthreads();
    if (wid == 0) {
        int run = 0;
        for (int k0 = 0; k0 < nw; k0 += 64) {
            const int k = k0 + lane;
            const int c = k < nw ? __popcll(tmask[k]) : 0;
            const int incl = kd_wave_incl_sum(c);
            if (k < nw) tpre[k] = (unsigned)(run + incl - c);
            run += __builtin_amdgcn_readlane(incl, 63);
        }
    }
    __syncthreads();
    const bool tsorted = __builtin_amdgcn_readfirstlane(sm->tsorted) != 0;

    // sources: one each to start, then from a queue, so workgroups that drew cheap
    // sources take more and the launch ends within about one source of the mean
    // (a static stride ended with the workgroups holding ceil(ns / grid) sources)
    const bool queued = g.jobs != nullptr;
    if (tid == 0) {
        sm->njb = -1; sm->wpar = 0;
        sm->jobs = g.jobs; sm->qnext = g.next; sm->drow = g.drow; sm->prow = g.prow; sm->rstride = g.rstride;
        sm->done = g.done; sm->ns = ns;
        sm->wsl[0] = wslice;
        sm->wsl[1] = reinterpret_cast<uint32_t*>(ws + (size_t)blockIdx.x * ws_stride + kd_ws_wpr1(n));
        KDOut& o = sm->out;
        o.tgt = (const KD_GLOBAL int*)tgt; o.lat_out = (KD_GLOBAL double*)lat_out; o.rel_out = (KD_GLOBAL double*)rel_out;
        o.row_min = (KD_GLOBAL double*)row_min; o.err = err; o.relv = (KD_GLOBAL double*)relv;
        o.rtab = (const KD_GLOBAL double*)g.rtab; o.vf = (const KD_GLOBAL double*)g.vf; o.ld = ld;
        o.n = n; o.nw = nw; o.nt = nt; o.tsorted = tsorted ? 1 : 0; o.rmask = rmask; o.rc = g.rc; o.walk = g.walk;
        o.nrtab = g.nrtab; o.rone = g.rone; o.has_vf = g.has_vf; o.dflags = KD_DFLAGS;
    }
    // (the barriers of kd_next_source publish these)
    // the next job: taken in the previous row's output phases (planned launches), else here
    for (int jb = queued ? kd_next_source(g.next, &sm->next, tid, true) : (int)blockIdx.x; jb < ns;
         jb = sm->njb >= 0 ? sm->njb : kd_next_source(g.next, &sm->next, tid, queued)) {
        if (tid < 16) {
            int x;
            if (sm->njb >= 0) x = reinterpret_cast<const int*>(&sm->njob)[tid];
            else if (g.jobs) x = reinterpret_cast<const int*>(g.jobs + jb)[tid];
            else x = tid == 0 ? jb : tid == 1 ? src[jb] : tid == 2 ? -1 : 0;  // row, s, store = -1, nseed = 0
            reinterpret_cast<int*>(&sm->job)[tid] = x;
        }
        if (tid == 0) sm->wpar ^= 1;  // rows alternate between the two record slices
        __syncthreads();
        if (tid == 0) sm->njb = -1;   // (every thread has read it: the increment above)
        const int i = sm->job.row, s = sm->job.s;
        {
            bool bad = s < 0 || s >= n || sm->job.nseed < 0 || sm->job.nseed > KD_SEEDS;
            for (int q = 0; q < KD_SEEDS; q++)
                if (q < sm->job.nseed) bad = bad || sm->job.u[q] < 0 || sm->job.u[q] >= n || sm->job.seed[q] < 0;
            if (bad) {  // (uniform: every thread read the same job)
                if (tid == 0) raise_err(err, SHD_ROUTE_EINVAL);
                // njb = -1 (thread 0, above) visible to every thread before the loop
                // increment reads it: all take the next job from kd_next_source together
                __syncthreads();
                continue;
            }
        }
        // parent records: the row kept for later seeds is this source's own array
        auto wpr_of = [&]() __attribute__((always_inline)) {
            const int st = __builtin_amdgcn_readfirstlane(sm->job.store);
            return st >= 0 ? g.prow + (size_t)st * g.rstride : sm->wsl[__builtin_amdgcn_readfirstlane(sm->wpar)];
        };
        const double fs = g.vf[s];
        const double cs = isnan(fs) ? 1.0 : 1.0 * fs;
        // the (s, s) entry's self-loop, loaded before this source's first store
        const double sw_s = g.self_w[s], sr_s = g.self_r[s];
    kd_restart:
#ifdef SHD_STAMPS
        unsigned long long kd_t = 0;
#endif
        KD_MARK();
#ifdef SHD_STAMPS
        wait_stores();  // diagnostic: the previous row's output stores, drained here
        KD_ACC(9);
#endif
        const bool seeded = __builtin_amdgcn_readfirstlane(sm->job.nseed) > 0;
        if (seeded) {
            uint32_t* const wpr = wpr_of();
            // the seeds' rows are ready: one relaxed poll of each flag, one agent-scope
            // acquire (this CU's L1 invalidated), then every wave reads them with plain loads.
            // With KD_SEEDSPIN > 0 a seed after the first that is not ready within that many
            // polls is dropped from the job (any subset of the seeds gives exact rows: the
            // fix-up phases start from whichever upper bounds D0 holds)
            if (tid == 0) {
#ifdef SHD_STAMPS
                const unsigned long long w0 = __builtin_amdgcn_s_memtime();
#endif
                const int ns0 = sm->job.nseed;
                int kept = 0;
                for (int q = 0; q < ns0; q++) {
                    const int* const flag = &g.done[sm->job.seed[q]];
                    const int cap = (q == 0 || KD_SEEDSPIN == 0) ? (1 << 22) : KD_SEEDSPIN;
                    int spin = 0;
                    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 && spin < cap) {
                        __builtin_amdgcn_s_sleep(8);
                        spin++;
                    }
                    if (spin >= (1 << 22)) raise_err(err, SHD_ROUTE_EDEVICE);
                    if (spin >= cap && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
                        continue;  // (KD_SEEDSPIN: dropped)
                    if (q > 0 && ((g.seed_drop >> q) & 1)) continue;  // (tests: a chosen subset)
                    if (kept != q) {
                        sm->job.seed[kept] = sm->job.seed[q];
                        sm->job.u[kept] = sm->job.u[q];
                        sm->job.wr[kept] = sm->job.wr[q];
                        sm->job.rec[kept] = sm->job.rec[q];
                    }
                    kept++;
                }
                sm->job.nseed = kept;
#ifdef SHD_STAMPS
                sm->acc[31] += __builtin_amdgcn_s_memtime() - w0;
                sm->acc[36] += ns0 - kept;
#endif
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            SEED_VIEW();
            // one streaming pass, 8 vertices per lane (16-B loads of every seed's distances
            // and parent records): D0(v) = min_j w(s,u_j) + d_{u_j}(v), saturating at 0xFFFF
            // (= unreached), into LDS; and the parent record a vertex keeps if it never
            // improves on D0: the best (tie rule: largest w, then smallest parent) of the
            // parents of the seeds attaining D0(v), u_j's own vertex having parent s.  Phase
            // A's records overwrite the vertices that do improve.
            // 4 vertices per lane: 8-B distance and 16-B parent-record loads of every seed
            // (loading a seed's records only where it attains D0 measured slower: round 4,
            // DESIGN.md 4.3)
            for (int v0 = 4 * tid; v0 <= n; v0 += 4 * B) {
                const int vl = min(v0, n & ~3);
                uint2 dq[KD_SEEDS];
                uint4 pq[KD_SEEDS];
#pragma unroll
                for (int q = 0; q < KD_SEEDS; q++) {
                    if (q < nseed) {
                        if constexpr (B >= 1024 && KD_NTLOAD) {
                            // streaming loads: a neighbour seed's row is read by few rows, and
                            // passes through L2 without pushing out the CSR (C4 41.50 -> 41.23
                            // ms); 256-thread rows keep them cached (C3's landmark rows seed
                            // ~27 rows each: 2.03 -> 2.17 ms streamed)
                            typedef unsigned u2v __attribute__((ext_vector_type(2)));
                            const u2v d2 = __builtin_nontemporal_load(reinterpret_cast<const u2v*>(sdrow[q] + vl));
                            const kd_u4 p4 = __builtin_nontemporal_load(reinterpret_cast<const kd_u4*>(sprow[q] + vl));
                            dq[q] = make_uint2(d2.x, d2.y);
                            pq[q] = make_uint4(p4.x, p4.y, p4.z, p4.w);
                        } else {
                            dq[q] = *reinterpret_cast<const uint2*>(sdrow[q] + vl);
                            pq[q] = *reinterpret_cast<const uint4*>(sprow[q] + vl);
                        }
                    } else {
                        dq[q] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
                        pq[q] = make_uint4(KD_NONE, KD_NONE, KD_NONE, KD_NONE);
                    }
                }
                uint32_t dw[2], rw[4];
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    const int v = v0 + h;
                    unsigned dbest = 0xFFFFu, kbest = 0xFFFFFFFFu;
                    uint32_t rbest = KD_NONE;
#pragma unroll
                    for (int q = 0; q < KD_SEEDS; q++) {
                        const uint32_t d2 = (h < 2) ? dq[q].x : dq[q].y;
                        const unsigned d = (h & 1) ? (d2 >> 16) : (d2 & 0xFFFFu);
                        const unsigned c = q < nseed ? min(0xFFFFu, wsu[q] + d) : 0xFFFFFu;
                        const uint32_t p = kd_comp(pq[q], h);
                        const uint32_t r = v == su[q] ? rsu[q] : p;  // (rsu: the seed vertex's record)
                        const uint32_t k = __builtin_amdgcn_perm(~r, r, 0x07010002u);  // (255-w) | p | ridx
                        if (c < dbest || (c == dbest && k < kbest)) { dbest = c; kbest = k; rbest = r; }
                    }
                    if (v >= n) dbest = 0xFFFFu;
                    if (v == s) rbest = KD_SRC_MARK;
                    if (h & 1) dw[h >> 1] |= dbest << 16;
                    else dw[h >> 1] = dbest;
                    rw[h] = rbest;
                }
                *reinterpret_cast<uint2*>(dist + v0) = make_uint2(dw[0], dw[1]);
                *reinterpret_cast<uint4*>(wpr + v0) = make_uint4(rw[0], rw[1], rw[2], rw[3]);
            }
            wait_stores();  // before phase A's writer overwrites improved vertices
        } else {
            for (int v = tid; v < (n + 2) / 2; v += B) reinterpret_cast<uint32_t*>(dist)[v] = 0xFFFFFFFFu;
        }
        for (int k = tid; k < nw; k += B) { pend[k] = 0ull; wmin[k] = 0xFFFFFFFFu; fix[k] = 0ull; }
        for (int q = tid; q < RR; q += B) rrec[q] = make_uint2(0u, 0xFFFFFFFFu);  // phases B/C reuse the area
        if (lane < 2 * KD_P) wmark[lane] = 0u;  // phase C reuses it
        if (tid == 0) {
            sm->gmin[0] = sm->gmin[1] = 0xFFFFFFFFu;
            sm->rtail = sm->rdone = 0;
            sm->nev = 0; sm->evovf = 0;
            wpr_of()[s] = KD_SRC_MARK;
        }
        lds_barrier();
        KD_ACC(29);
        KD_STAMP(0);  // after the seed wait and the distance init
        if (tid == 0) {
            dist[s] = 0;
            pend[s >> 6] = 1ull << (s & 63);
            wmin[s >> 6] = 0;
        }
        lds_barrier();

        // ---- A: delta-stepping, asynchronous inside a bucket ------------------------
        // Bucket round: (1) T from the min pending distance; (2) gather the pending vertices
        // with dist < T into the work queue; (3) compute waves pull 64-entry slices from the
        // queue and push every vertex they improve below T straight back, so a bucket's
        // light-arc chains need no barriers; far improvements
        // and queue overflow go to the pending bitmask.  The last wave is the writer: it
        // drains the slices' parent records into wpr (HBM) so compute waves never wait on a
        // store.  A round ends when no wave holds a slice and the queue is empty.
        unsigned T = delta;
        int par = 0;
        const int ncomp = NW - 1;
        int wnev = 0;  // writer wave: tie events stored so far
        KD_MARK();
        for (;;) {
            KD_COUNT(5, tid == 0 ? 1 : 0);
            {
                unsigned m0 = 0xFFFFFFFFu;
                for (int k = tid; k < nw; k += B) m0 = min(m0, wmin[k]);
                const unsigned wm = kd_wave_min_dpp(m0);
                if (lane == 0 && wm != 0xFFFFFFFFu) atomicMin(&sm->gmin[par], wm);
            }
            for (int q = tid; q < rc; q += B) ring[q] = 0xFFFFu;
            if (tid == 0) { sm->gmin[par ^ 1] = 0xFFFFFFFFu; sm->head = sm->tail = 0; sm->busy = 0; sm->nexit = 0; }
            lds_barrier();
            const unsigned m = sm->gmin[par];
            if (m == 0xFFFFFFFFu) break;
            if (m >= T) T = (m / delta + 1) * delta;
            KD_ACC(11);
            // gather: pending vertices with dist < T into the queue (one thread per word)
            for (int k0 = 0; k0 < nw; k0 += B) {
                const int k = k0 + tid;
                unsigned long long bits = 0ull, take = 0ull;
                unsigned rest = 0xFFFFFFFFu;
                const bool act = k < nw && wmin[k] < T;
                if (act) {
                    bits = pend[k];
                    unsigned long long b = bits;
                    while (b) {  // four bits per trip: independent LDS reads in flight
                        int v4[4];
                        pop4(&b, k, v4);
                        unsigned d4[4];
#pragma unroll
                        for (int q = 0; q < 4; q++) d4[q] = ld16(dist, v4[q] >= 0 ? v4[q] : n);
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            if (v4[q] < 0) continue;
                            if (d4[q] < T) take |= 1ull << (v4[q] & 63);
                            else rest = min(rest, d4[q]);
                        }
                    }
                }
                const int cnt = __popcll(take);
                int incl = kd_wave_incl_sum(cnt);
                int base = 0;
                if (lane == 63 && incl) base = atomicAdd(&sm->tail, incl);
                base = __builtin_amdgcn_readlane(base, 63);
                int pos = base + incl - cnt;
                if (act) {
                    unsigned long long b = take;
                    while (b) {
                        const int bi = __ffsll((long long)b) - 1;
                        b &= b - 1;
                        const int u = (k << 6) + bi;
                        if (pos < rc) ring[pos] = (uint16_t)u;
                        else {
                            take &= ~(1ull << bi);
                            rest = min(rest, (unsigned)dist[u]);
#ifdef SHD_STAMPS
                            atomicAdd(&sm->acc[15], 1ull);
#endif
                        }
                        pos++;
                    }
                    pend[k] = bits & ~take;
                    wmin[k] = rest;
                }
            }
            lds_barrier();
            if (tid == 0) sm->tail = min(sm->tail, rc);
            lds_barrier();
            KD_ACC(8);
            if (!writer) {
                // ---- compute wave: pull slices until the round drains ----------------
                // records {x, y} for the writer's ring from the lanes in `m` (wave-uniform
                // call): one reservation, then one 64-bit LDS write per record, so the
                // writer never sees half a record
                auto push_rec = [&](unsigned long long m, bool mine, uint32_t x, uint32_t y) __attribute__((always_inline)) {
                    const int nr = __popcll(m);
                    int rb = 0;
                    if (lane == 0) {
                        rb = atomicAdd(&sm->rtail, nr);
                        int w8 = 0;
                        for (; rb + nr - __hip_atomic_load(&sm->rdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > RR
                               && w8 < (1 << 22); w8++)
                            __builtin_amdgcn_s_sleep(1);
                        if (w8 >= (1 << 22)) raise_err(err, SHD_ROUTE_EDEVICE);
                        if (w8 && g.stats) atomicMax(&g.stats[0], (unsigned long long)w8);
                    }
                    rb = __builtin_amdgcn_readfirstlane(rb);
                    if (mine) {
                        const int slot = (rb + __popcll(m & (upto >> 1))) & (RR - 1);
                        *reinterpret_cast<volatile unsigned long long*>(&rrec[slot]) =
                            (unsigned long long)x | ((unsigned long long)y << 32);
                    }
                };
                int spins = 0;
                for (;;) {
                    int h = 0, nn = 0;
                    if (lane == 0) {
                        // idle waves only read: busy is raised just around a real grab, so an
                        // idle wave never hides the all-idle state from the others
                        if (min(__hip_atomic_load(&sm->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), rc) >
                            __hip_atomic_load(&sm->head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                            atomicAdd(&sm->busy, 1);
                            h = __hip_atomic_load(&sm->head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            const int t = min(__hip_atomic_load(&sm->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), rc);
                            nn = min(64, t - h);
                            // a short queue spread over more waves (each slice pays the same
                            // two global-load latencies, whatever its size)
                            if (KD_SDIV > 0 && B >= 1024) nn = min(nn, max(KD_SMIN, (t - h + KD_SDIV - 1) / max(KD_SDIV, 1)));
                            // (256-thread rows keep 64-entry grabs: queued / 3, 6 or 12 with 16, 8, 8
                            // at least measured C3 2.17 / 2.51 / 2.85 ms against 2.01)
                            if (nn > 0 && atomicCAS(&sm->head, h, h + nn) != h) nn = 0;
                            if (nn <= 0) { nn = 0; atomicSub(&sm->busy, 1); }
                        }
                    }
                    nn = __builtin_amdgcn_readfirstlane(nn);
                    h = __builtin_amdgcn_readfirstlane(h);
                    if (nn == 0) {
                        int fin = 0;
                        if (lane == 0) {
                            const int bz = __hip_atomic_load(&sm->busy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            const int t = min(__hip_atomic_load(&sm->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), rc);
                            const int hh = __hip_atomic_load(&sm->head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            fin = bz == 0 && hh == t;
                        }
                        if (__builtin_amdgcn_readfirstlane(fin)) break;
                        KD_COUNT(21, 1);
                        if (++spins > (1 << 22)) { if (lane == 0) raise_err(err, SHD_ROUTE_EDEVICE); break; }
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    spins = 0;
#ifdef SHD_STAMPS
                    unsigned long long ks0 = __builtin_amdgcn_s_memtime();
#endif
                    // the slice: queue entries [h, h+nn), written right after reservation
                    const bool act = lane < nn;
                    int u = 0;
                    if (act) {
                        volatile uint16_t* slot = ring + h + lane;
                        unsigned x = *slot;
                        int w8 = 0;
                        for (; x == 0xFFFFu && w8 < (1 << 22); w8++) { __builtin_amdgcn_s_sleep(1); x = *slot; }
                        if (x == 0xFFFFu) raise_err(err, SHD_ROUTE_EDEVICE);
                        if (w8 && g.stats) atomicMax(&g.stats[2], (unsigned long long)w8);
                        u = x == 0xFFFFu ? s : (int)x;
                    }
                    const unsigned du0 = act ? ld16(dist, u) : 0u;
                    int beg = 0, deg = 0;
                    {
                        const int r0 = g.row[u], r1 = g.row[u + 1];
                        if (act) { beg = r0; deg = r1 - r0; }
                    }
                    // the expansion needs the non-empty rows on lanes 0..R-1 (owner = running
                    // row count + mbcnt); a slice with an empty row among them (directed graphs)
                    // is compacted through the wave's list area, which is free at this point
                    const unsigned long long nonempty = __ballot(deg > 0);
                    const int crank = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(nonempty >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((unsigned)nonempty, 0u));
                    unsigned du = du0;
                    const int deg0 = deg;
                    if ((nonempty & (nonempty + 1ull)) != 0ull) {  // not a prefix of the lanes
                        if (deg > 0) { wimp[crank] = (uint32_t)beg; wimp[64 + crank] = (uint32_t)deg; wimp[128 + crank] = du0; }
                        __builtin_amdgcn_wave_barrier();
                        const int R = __popcll(nonempty);
                        beg = lane < R ? (int)wimp[lane] : 0;
                        deg = lane < R ? (int)wimp[64 + lane] : 0;
                        du = lane < R ? wimp[128 + lane] : 0u;
                        __builtin_amdgcn_wave_barrier();
                    }
                    int incl = kd_wave_incl_sum(deg);
                    const int total = __builtin_amdgcn_readlane(incl, 63);
                    const int excl = incl - deg;
                    const int boff = beg - excl;
                    if (g.fused) wkey[lane] = ~0u;
                    // owner of arc position q = (#rows starting at or before q) - 1: a running
                    // row count plus one mbcnt per step
                    int rows_before = 0;  // rows starting before the current step
#ifdef SHD_STAMPS
                    if (tid == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); sm->acc[22] += t_ - ks0; ks0 = t_; }
#endif
                    int nimp = 0;  // improving arcs listed, relaxed when the list fills or the slice ends
                    // Windows of KD_P steps x 64 arcs, software-pipelined: the owners and out-arc
                    // loads of window k+1 are issued before window k is processed, so the L2/HBM
                    // latency of the records overlaps the dist reads and relaxations.
                    struct Win {
                        uint32_t rx[KD_P];   // out-arc records v | w << 16
                        uint32_t odo[KD_P];  // owner's du | owner lane << 16
                        int obv[KD_P];       // owner's arc offset: arc of step p = obv + b0 + lane + 64 p
                    };
                    Win wa, wb;
                    const int dul = (int)(du | ((unsigned)lane << 16));
                    // owners: each lane whose row starts inside the window marks its start (lane + 1;
                    // marker of position q at byte (q % 64) * 8 + q / 64, so one ds_read_b64 per lane
                    // fetches its position in all KD_P steps).  Dense slices: owner = running row
                    // count + mbcnt of the step's start mask; else a DPP prefix max over the marks,
                    // seeded at position 0 with the row covering the step's first arc.  The loads
                    // are issued even for a window past the slice's arcs (range-checked no-ops), so
                    // the load counter the next window waits on is static.
                    auto issue = [&](Win& W, const int b0) __attribute__((always_inline)) {
                        const bool live = b0 < total;
                        if (live) {
                            // start bits of the window's rows (u64 per step), one atomic OR per
                            // row start; lane p < KD_P reads step p's word, readlane hands it out
                            const int pos = excl - b0;
                            const bool mark = deg > 0 && pos >= 0 && pos < 64 * KD_P;
                            if (mark) atomicOr(&wmark[pos >> 5], 1u << (pos & 31));
                            __builtin_amdgcn_wave_barrier();
                            const unsigned long long mw = reinterpret_cast<const unsigned long long*>(wmark)[lane & (KD_P - 1)];
                            int oo[KD_P];
#pragma unroll
                            for (int p = 0; p < KD_P; p++) {
                                const unsigned long long st =
                                    ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(mw >> 32), p) << 32) |
                                    (unsigned)__builtin_amdgcn_readlane((int)(unsigned)mw, p);
                                const unsigned long long sh = st >> 1;
                                oo[p] = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(sh >> 32),
                                            __builtin_amdgcn_mbcnt_lo((unsigned)sh, (unsigned)(rows_before + (int)(st & 1ull) - 1)));
                                rows_before += __popcll(st);
                            }
                            kd_bpermute16(oo, boff, dul, W.obv, W.odo);
                            if (lane < KD_P) reinterpret_cast<unsigned long long*>(wmark)[lane] = 0ull;
                        } else {
#pragma unroll
                            for (int p = 0; p < KD_P; p++) { W.obv[p] = 0; W.odo[p] = 0u; }
                        }
                        const int lbw = b0 + lane;
                        const int soff = live ? 0 : 0x40000000;  // past every record: no-op loads
#pragma unroll
                        for (int p = 0; p < KD_P; p++)
                            W.rx[p] = __builtin_amdgcn_raw_buffer_load_b32(orsrc, ((uint32_t)(W.obv[p] + lbw) << 2) + 256u * p, soff, 0);
                    };
                    // one window: read dist[v], compare, and append the improving lanes (~5% of
                    // arcs) to the wave's list; the tight check for fused parents is one exec-masked
                    // ds_min_u64 per step
                    auto process = [&](const Win& W, const int b0) __attribute__((always_inline)) {
                        const int lb = b0 + lane;
                        // all KD_P dist reads in flight before the first LDS store of the steps
                        // (the compiler cannot move a read above a store that may alias it)
                        unsigned dvs[KD_P];
#pragma unroll
                        for (int p = 0; p < KD_P; p++) dvs[p] = ld16(dist, (int)(W.rx[p] & 0xFFFFu));
                        // one step; FULL: every lane holds an arc (all but the slice's last window)
                        auto step = [&](const int p, auto full) __attribute__((always_inline)) {
                            const unsigned v = W.rx[p] & 0xFFFFu, w = (W.rx[p] >> 16) & wmask;
                            const unsigned odu = W.odo[p] & 0xFFFFu;
                            const unsigned dv = dvs[p], nd = odu + w;
                            bool valid = true;
                            if constexpr (!decltype(full)::value) valid = lb + 64 * p < total;
                            const bool imp = valid && nd < dv;  // nd < dv <= 0xFFFF: fits u16
                            const unsigned long long im = __ballot(imp);
                            if (imp) {
                                const unsigned r = __builtin_amdgcn_mbcnt_hi((unsigned)(im >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((unsigned)im, (unsigned)nimp));
                                wimp[r] = v | (nd << 16);
                            }
                            nimp += __popcll(im);
                            // tie rule: largest w, then smallest (parent, eid) = smallest v (simple
                            // graph, rows sorted by (v, eid)).  Packed records: the key
                            // (255 - w) << 24 | v << 8 | ridx is one byte permutation of ~rec / rec
                            if (g.fused && valid && dv + w == odu)
                                atomicMin(&wkey[W.odo[p] >> 16], __builtin_amdgcn_perm(~W.rx[p], W.rx[p], 0x06010003u));
                            if (seeded) {
                                // tie event: the owner x is a tight in-neighbour of v (x improved:
                                // only improved vertices are expanded); v's parent is settled
                                // after phase A if v keeps its seeded distance
                                const bool tie = valid && nd == dv;
                                const unsigned long long tm = __ballot(tie);
                                if (tm) {
                                    const int pv = __shfl(u, (int)(W.odo[p] >> 16), 64);
                                    push_rec(tm, tie, (uint32_t)pv | ((W.rx[p] >> 24) << 16) | (w << 24), v | KD_EVTAG);
                                }
                            }
                        };
                        // the list holds KD_IMP >= 3 x 64 entries: a flush check every second step
                        static_assert(KD_IMP >= 192, "two steps between flush checks");
                        auto flush = [&]() __attribute__((always_inline)) {
                            kd_relax_list(wimp, nimp, lane, upto, reinterpret_cast<uint32_t*>(dist), pend, wmin, ring,
                                          &sm->tail, rc, T, KD_ACCP);
                            nimp = 0;
                        };
                        if (b0 + 64 * KD_P <= total) {
#pragma unroll
                            for (int p = 0; p < KD_P; p += 2) {
                                step(p, std::true_type{});
                                step(p + 1, std::true_type{});
                                if (nimp > KD_IMP - 128) flush();
                            }
                        } else {
                            const int nstep = (total - b0 + 63) >> 6;  // steps holding arcs (< KD_P)
#pragma unroll
                            for (int p = 0; p < KD_P; p += 2) {
                                if (p >= nstep) break;
                                step(p, std::false_type{});
                                if (p + 1 < nstep) step(p + 1, std::false_type{});
                                if (nimp > KD_IMP - 128) flush();
                            }
                        }
                    };
                    issue(wa, 0);
                    for (int b0 = 0; b0 < total;) {
                        issue(wb, b0 + 64 * KD_P);
                        process(wa, b0);
                        b0 += 64 * KD_P;
                        if (b0 >= total) break;
                        issue(wa, b0 + 64 * KD_P);
                        process(wb, b0);
                        b0 += 64 * KD_P;
                    }
                    if (nimp) kd_relax_list(wimp, nimp, lane, upto, reinterpret_cast<uint32_t*>(dist), pend, wmin, ring, &sm->tail, rc, T, KD_ACCP);
#ifdef SHD_STAMPS
                    if (tid == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); sm->acc[23] += t_ - ks0; ks0 = t_; sm->acc[25] += (total + 64 * KD_P - 1) / (64 * KD_P); }
#endif
                    KD_COUNT(7, total);
                    KD_COUNT(6, nn);
                    KD_COUNT(20, 1);
                    __builtin_amdgcn_wave_barrier();
                    // parent records {winner, u | du << 16} to the writer's ring
                    const bool hasrec = act && u != s;
                    uint32_t prec = KD_NONE;
                    if (g.fused && hasrec) {
                        const uint32_t kk = deg0 > 0 ? wkey[crank] : ~0u;
                        if (kk != ~0u && (0xFFu - (kk >> 24)) >= delta)  // heavy winner: parent | ridx << 16
                            prec = ((kk >> 8) & 0xFFFFu) | ((kk & 0xFFu) << 16) | ((0xFFu - (kk >> 24)) << 24);
                    }
                    const unsigned long long rm = __ballot(hasrec);
                    if (rm) push_rec(rm, hasrec, prec, (uint32_t)u | (du0 << 16));
                    if (lane == 0) atomicSub(&sm->busy, 1);
#ifdef SHD_STAMPS
                    if (tid == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); sm->acc[24] += t_ - ks0; sm->acc[26] += 1; }
#endif
                }
                if (lane == 0) atomicAdd(&sm->nexit, 1);
            } else {
                // ---- writer wave: parent records -> wpr (HBM) + fix bits -------------
                uint32_t* const wpr = wpr_of();
                int rd = __hip_atomic_load(&sm->rdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                int spins = 0;
                for (;;) {
                    const int rt = __hip_atomic_load(&sm->rtail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (rt > rd) {
                        // up to 4 x 64 records per pass, and at most RR - 64: a compute wave whose
                        // reservation (<= 64 slots) starts inside the pass then never waits for ring
                        // space the pass has not released (with RR = 256 a full pass could hold the
                        // first slots of a reservation whose owner was still waiting to write them:
                        // both sides spun to their caps, a ~110 ms stall per occurrence on C3)
                        const int k = min(min(4 * 64, RR - 64), rt - rd);
                        int uu[4], ev[4];
                        uint32_t xx[4];
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            uu[q] = -1;
                            ev[q] = -1;
                            xx[q] = KD_NONE;
                            if (q * 64 + lane < k) {
                                const int slot = (rd + q * 64 + lane) & (RR - 1);
                                volatile unsigned long long* sp = reinterpret_cast<volatile unsigned long long*>(&rrec[slot]);
                                unsigned long long rv = *sp;
                                int w8 = 0;
                                for (; (rv >> 32) == 0xFFFFFFFFull && w8 < (1 << 22); w8++) {
                                    __builtin_amdgcn_s_sleep(1);
                                    rv = *sp;
                                }
                                if (w8 >= (1 << 22)) raise_err(err, SHD_ROUTE_EDEVICE);
                                if (w8 && g.stats) atomicMax(&g.stats[1], (unsigned long long)w8);
                                const uint32_t x = (uint32_t)rv, y = (uint32_t)(rv >> 32);
                                *sp = 0xFFFFFFFF00000000ull;
                                const int u = (int)(y & 0xFFFFu);
                                if (y != 0xFFFFFFFFu && (y & KD_EVTAG) == KD_EVTAG) {  // tie event (seeded rows)
                                    ev[q] = u; xx[q] = x;
                                } else if (y != 0xFFFFFFFFu && ld16(dist, u) == (y >> 16)) {  // from u's latest expansion
                                    const unsigned long long bit = 1ull << (u & 63);
                                    if (x != KD_NONE) { uu[q] = u; xx[q] = x; atomicAnd(&fix[u >> 6], ~bit); }
                                    else atomicOr(&fix[u >> 6], bit);
                                }
                            }
                        }
#pragma unroll
                        for (int q = 0; q < 4; q++)  // records are parent | ridx << 16
                            if (uu[q] >= 0) wpr[uu[q]] = xx[q];
#pragma unroll
                        for (int q = 0; q < 4; q++) {  // tie events -> the slice's event list
                            const unsigned long long em = __ballot(ev[q] >= 0);
                            if (em) {
                                const int at = wnev + __popcll(em & (upto >> 1));
                                if (ev[q] >= 0 && at < g.evcap) evl[at] = make_uint2(xx[q], (uint32_t)ev[q]);
                                wnev += __popcll(em);
                            }
                        }
                        rd += k;
                        __builtin_amdgcn_wave_barrier();
                        if (lane == 0) __hip_atomic_store(&sm->rdone, rd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        spins = 0;
                        continue;
                    }
                    if (__hip_atomic_load(&sm->nexit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == ncomp &&
                        __hip_atomic_load(&sm->rtail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == rd) {
                        if (lane == 0) sm->nev = wnev;
                        break;
                    }
                    if (++spins > (1 << 22)) { if (lane == 0) raise_err(err, SHD_ROUTE_EDEVICE); break; }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            par ^= 1;
            lds_barrier();
            KD_ACC(10);
        }
        wait_stores();  // the writer's records land before phase B rewrites fixed-up vertices
        lds_barrier();
        if (seeded) {
            // ---- A': parents of the vertices that kept D0 ------------------------------
            KD_MARK();
            const int nev = sm->nev;
            if (nev > g.evcap) {  // (uniform) the slice lost events: this row again, unseeded
                lds_barrier();
                if (tid == 0) sm->job.nseed = 0;
                lds_barrier();
                goto kd_restart;
            }
            uint32_t* const wpr = wpr_of();
            SEED_VIEW();
            auto d0 = [&](int v) __attribute__((always_inline)) {
                unsigned x = 0xFFFFu;
#pragma unroll
                for (int q = 0; q < KD_SEEDS; q++)
                    if (q < nseed) x = min(x, min(0xFFFFu, wsu[q] + (unsigned)sdrow[q][v]));
                return x;
            };
            KD_ACC(27);
            // a vertex that kept D0 holds the seed-derived parent from the init pass; a tight
            // improved in-neighbour reported as a tie event may beat it (tie rule: largest w,
            // then smallest parent): keys (255 - w) << 24 | parent << 8 | ridx, min over
            // that parent and every valid event, through u32 keys in the slice (relv is free)
            uint32_t* key = reinterpret_cast<uint32_t*>(relv);
            // event e -> v (-1 if invalid: v improved on D0, or the arc is not tight) + key
            auto event = [&](int e, int& v, uint32_t& ke) __attribute__((always_inline)) {
                const uint2 r = evl[e];
                v = (int)r.y;
                const int p = (int)(r.x & 0xFFFFu);
                const unsigned w = r.x >> 24, dv = ld16(dist, v);
                if (dv != d0(v) || ld16(dist, p) + w != dv) { v = -1; return; }
                ke = ((0xFFu - w) << 24) | ((uint32_t)p << 8) | ((r.x >> 16) & 0xFFu);
            };
            for (int e = tid; e < nev; e += B) {
                int v; uint32_t ke = 0;
                event(e, v, ke);
                if (v >= 0) {  // u's parent (from the copy above) as the starting key
                    const uint32_t b = wpr[v];
                    const unsigned pb = b & 0xFFFFu, wb = ld16(dist, v) - ld16(dist, (int)pb);
                    key[v] = ((0xFFu - wb) << 24) | (pb << 8) | ((b >> 16) & 0xFFu);
                }
            }
            wait_stores();
            lds_barrier();
            for (int e = tid; e < nev; e += B) {
                int v; uint32_t ke = 0;
                event(e, v, ke);
                if (v >= 0) atomicMin(&key[v], ke);
            }
            wait_stores();
            lds_barrier();
            for (int e = tid; e < nev; e += B) {
                int v; uint32_t ke = 0;
                event(e, v, ke);
                if (v >= 0) {
                    const uint32_t k = __hip_atomic_load(&key[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    wpr[v] = ((k >> 8) & 0xFFFFu) | ((k & 0xFFu) << 16) | ((0xFFu - (k >> 24)) << 24);
                }
            }
            wait_stores();
            lds_barrier();
            KD_ACC(28);
        }
        KD_STAMP(1);
        KD_MARK();

        // ---- B: fix-ups (first tight arc of the light in-row tail) ---------------------
        // rounds over a compacted list (qv) so all threads share the work evenly; per entry
        // the row bounds and KD_TAIL tail arcs are loaded straight-line, long tails are
        // re-queued (qbeg) for one wave per vertex
        const int last_arc = g.nlight > 0 ? g.nlight - 1 : 0;
        uint32_t* const wpr = wpr_of();  // (phases B and C)
        if (tid == 0) {
            fix[s >> 6] &= ~(1ull << (s & 63));
            sm->qtail[0] = sm->qtail[1] = 0;
            sm->qcur[0] = sm->qcur[1] = 0;
        }
        for (int rnd = 0;; rnd ^= 1) {
            if (tid == 0) { sm->qtail[rnd ^ 1] = 0; sm->qcur[rnd ^ 1] = 0; }
            lds_barrier();
            for (int k0 = 0; k0 < nw; k0 += B) {
                const int k = k0 + tid;
                unsigned long long bits = k < nw ? fix[k] : 0ull;
                const int cnt = __popcll(bits);
                int incl = kd_wave_incl_sum(cnt);
                int base = 0;
                if (lane == 63 && incl) base = atomicAdd(&sm->qtail[rnd], incl);
                base = __builtin_amdgcn_readlane(base, 63);
                int pos = base + incl - cnt;
                unsigned long long b = bits, listed = 0ull;
                while (b && pos < qcap) {
                    const int bi = __ffsll((long long)b) - 1;
                    b &= b - 1;
                    qv[pos++] = (uint16_t)((k << 6) + bi);
                    listed |= 1ull << bi;
                }
                if (listed) fix[k] = bits & ~listed;
            }
            lds_barrier();
            const int cnt = min(sm->qtail[rnd], qcap);
            if (cnt == 0) break;
            for (int j0 = 0; j0 < cnt; j0 += B * 4) {
                int v4[4], a4[4], r4[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int j = j0 + q * B + tid;
                    v4[q] = j < cnt ? (int)qv[j] : -1;
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int vv = v4[q] >= 0 ? v4[q] : 0;
                    a4[q] = g.lrow[vv];
                    r4[q] = g.lrow[vv + 1];
                }
                uint2 rc[4][KD_TAIL];
#pragma unroll
                for (int q = 0; q < 4; q++)
#pragma unroll
                    for (int e = 0; e < KD_TAIL; e++) rc[q][e] = g.lrec[min(a4[q] + e, last_arc)];
                unsigned dt[4][KD_TAIL], d4[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    d4[q] = ld16(dist, v4[q] >= 0 ? v4[q] : 0);
#pragma unroll
                    for (int e = 0; e < KD_TAIL; e++) dt[q][e] = ld16(dist, (int)(rc[q][e].x & 0xFFFFu));
                }
                uint32_t out_a[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    int f = -1;
                    uint32_t rec = KD_NONE;  // parent | ridx << 16 of the first tight arc
#pragma unroll
                    for (int e = KD_TAIL - 1; e >= 0; e--)
                        if (a4[q] + e < r4[q] && dt[q][e] + (rc[q][e].x >> 16) == d4[q]) {
                            f = e;
                            rec = (rc[q][e].x & 0xFFFFu) | (rc[q][e].y << 16) | (g.packed ? (rc[q][e].x >> 16) << 24 : 0u);
                        }
                    out_a[q] = rec;
                    if (v4[q] >= 0 && f < 0) {
                        if (r4[q] - a4[q] > KD_TAIL) {  // long tail: one wave per vertex below
                            const int at = atomicAdd(&sm->qcur[rnd], 1);
                            qbeg[at] = v4[q];  // at < cnt <= qcap
                            v4[q] = -1;
                        } else raise_err(err, SHD_ROUTE_EUNREACH);
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (v4[q] >= 0) wpr[v4[q]] = out_a[q];
            }
            lds_barrier();
            const int nlong = sm->qcur[rnd];
            for (int j = wid; j < nlong; j += B / 64) {
                const int v = qbeg[j];
                const unsigned dv = ld16(dist, v);
                const int r1 = g.lrow[v + 1];
                uint32_t fr = KD_NONE;
                for (int a0 = g.lrow[v] + KD_TAIL; a0 < r1 && fr == KD_NONE; a0 += 64) {
                    const int a = a0 + lane;
                    const uint2 rc = g.lrec[min(a, last_arc)];
                    const bool tight = a < r1 && ld16(dist, (int)(rc.x & 0xFFFFu)) + (rc.x >> 16) == dv;
                    const unsigned long long tm = __ballot(tight);
                    if (tm) fr = (uint32_t)__builtin_amdgcn_readlane((int)((rc.x & 0xFFFFu) | (rc.y << 16) | (g.packed ? (rc.x >> 16) << 24 : 0u)),
                                                                  __ffsll((long long)tm) - 1);
                }
                if (lane == 0) {
                    if (fr == KD_NONE) raise_err(err, SHD_ROUTE_EUNREACH);
                    wpr[v] = fr;
                }
            }
        }
        KD_ACC(16);
        KD_ACC(17);
        const int store = __builtin_amdgcn_readfirstlane(sm->job.store);
        if (store >= 0) {
            // this row seeds later ones: its parent records are final (wpr), keep its
            // distances (u16, incl. the pad); once every wave's stores have drained, the
            // flag (agent-scope release first) lets the rows it seeds start, before this
            // row's own output
            uint16_t* dr = g.drow_out + (size_t)store * g.rstride;
            // (streaming stores here and for the init's records measured the same: C4 41.87 / 41.91
            // against 41.93 / 41.89 ms)
            for (int v0 = 8 * tid; v0 <= n; v0 += 8 * B)
                *reinterpret_cast<uint4*>(dr + v0) = *reinterpret_cast<const uint4*>(dist + v0);
            wait_stores();
            __syncthreads();
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&g.done[store], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        KD_STAMP(2);
        // output phases in their own function: its registers are allocated for these loops
        // alone (inlined, phase A's pressure spilled the values they use to scratch, and
        // every reload waited behind the row's output stores: one in-order vmcnt)
        kd_output<B>(i, s, cs, sw_s, sr_s, (const KD_GLOBAL uint32_t*)wpr);
        lds_barrier();
        KD_STAMP(4);
        KD_FLUSH();
    }
}

// The table's rows (every planned or plain rows launch) ...
template <int B>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(4))) void sssp_delta_kernel(KD_KERNEL_PARAMS) {
    kd_rows_body<B>(g, src, ns, tgt, nt, ld, lat_out, rel_out, row_min, err, ws, ws_stride);
}
// ... and the planner's own rows (closeness and landmark rows, kept in a store, no output):
// the same code under its own name, so kernel statistics of a rows launch are not averaged
// with the planner's small launches
template <int B>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(4))) void kd_plan_rows_kernel(KD_KERNEL_PARAMS) {
    kd_rows_body<B>(g, src, ns, tgt, nt, ld, lat_out, rel_out, row_min, err, ws, ws_stride);
}

template <int B>
inline size_t kd_lds_bytes(int n, int rc) { return KDLayout<B>::make(n, rc, kd_rr<B>()).total; }

// phase C by path walks: u8 reliability index per vertex + the table itself in LDS
template <int B>
inline bool kd_walk_fits(int n, int rc, int nrtab) {
    const KDLayout<B> L = KDLayout<B>::make(n, rc, kd_rr<B>());
    return nrtab <= KD_ONE && L.rtabl + 8 * 256 <= L.total;
}

}  // namespace shd
