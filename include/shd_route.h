/*
 * shd_route.h -- C-ABI of the MI355X-native topology routing engine.
 *
 * This is the boundary that replaces the igraph-backed path computation inside
 * Shadow 1.14's src/main/routing/topology.c (mckerrigan/shadow).  Shadow keeps
 * its public routing API unchanged (topology.h:17-28); its topology.c front end
 * calls this module instead of igraph for every number that ends up in a Path
 * (path.c:13-21: latency, reliability).  Plain C types only; no HIP/torch types
 * in any signature.  One context per GPU; contexts are not re-entrant, and a context
 * (with its plans) runs one rows launch at a time: the launches of shd_route_rows_async
 * and shd_route_rows_planned_async share the context's work-queue counter and
 * per-workgroup scratch, so two of them must not be in flight together (enqueue them
 * on one stream, or synchronise in between).
 *
 * Reference interface each entry point replaces (file:line in the reference):
 *   shd_route_create   <- _topology_loadGraph/_topology_checkGraph/_topology_extractEdgeWeights
 *                         (topology.c:371-399, 1187-1246): graph in, validated, resident
 *   shd_route_rows     <- _topology_computeSourcePaths (topology.c:1655-1875) =
 *                         igraph_get_shortest_paths_dijkstra (topology.c:1756) +
 *                         _topology_computePathProperties (topology.c:1407-1523),
 *                         batched over many sources; with SHD_ROUTE_DISPATCH also the
 *                         direct-path dispatch of _topology_getPathEntry (topology.c:2019-2031)
 *                         and _topology_lookupDirectPath (topology.c:1877-1927)
 *   shd_route_direct   <- _topology_lookupDirectPath (topology.c:1877-1927) for many pairs
 *   shd_route_self     <- _topology_computeShortestPathToSelf (topology.c:1545-1653)
 *   shd_route_min_reduce <- minimumPathLatency tracking (topology.c:1374-1385)
 *   shd_route_fw       <- (no reference equivalent; dense all-pairs alternative)
 *
 * Semantics of one (s,t) entry are exactly the Path the reference would cache:
 *   t != s : lat = 0.0 + sum of edge latencies along the chosen shortest path, summed
 *            from s (bit-exact: any relaxation order reaches the same left-fold minimum);
 *            rel = ((1.0*f_s)*f_t) * prod(1 - loss_e) with absent vertex factors skipped.
 *            The engine multiplies f_t last, so rel is bit-exact whenever f_t is absent
 *            or 1.0 and within a few ulp otherwise.
 *   t == s : the batch self-loop entry (path [s]): lat = w_ss, rel = (1.0*f_s)*r_ss;
 *            SHD_ROUTE_ENOEDGE if s has no self-loop (topology.c:1488-1495).
 * Ties between equal-latency paths are broken deterministically: the parent of v is
 * the tight in-arc (u->v) with the smallest (dist[u], u, edge id).  Latency never
 * depends on ties; reliability matches igraph wherever the shortest path is unique.
 */
#ifndef SHD_ROUTE_H
#define SHD_ROUTE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes: 0 = success, negative = failure (topology.c maps them to critical()) */
#define SHD_ROUTE_OK 0
#define SHD_ROUTE_EINVAL (-1)       /* bad argument / graph fails topology.c validation */
#define SHD_ROUTE_ENOMEM (-2)       /* host or device allocation failed */
#define SHD_ROUTE_EDEVICE (-3)      /* HIP runtime error */
#define SHD_ROUTE_ENOEDGE (-4)      /* a hop has no edge (missing self-loop; topology.c:1488) */
#define SHD_ROUTE_EUNREACH (-5)     /* a target is unreachable (graph not strongly connected) */
#define SHD_ROUTE_EUNSUPPORTED (-6) /* request outside what this build supports */

/* flags for shd_route_rows */
#define SHD_ROUTE_DISPATCH 0x1u /* apply topology.c:2019 dispatch: complete graph -> direct,
                                   prefer-direct && adjacent -> direct, else source paths */

typedef struct shd_route shd_route_t;

/* A topology as igraph holds it after igraph_read_graph_graphml: vertices and edges
 * numbered in graphml document order.  Arrays are read during shd_route_create only. */
typedef struct shd_graph {
    int32_t n_vertices;
    int32_t n_edges;
    const int32_t* edge_src;          /* [n_edges] */
    const int32_t* edge_dst;          /* [n_edges] */
    const double* edge_latency;       /* [n_edges] ms, > 0        (topology.c:1070) */
    const double* edge_packetloss;    /* [n_edges] in [0,1]       (topology.c:1090) */
    const double* vertex_packetloss;  /* [n_vertices] or NULL; NaN = absent (topology.c:330-347) */
    int32_t directed;                 /* graphml edgedefault="directed" */
    int32_t prefer_direct;            /* graph attribute preferdirectpaths (topology.c:761-790) */
} shd_graph_t;

typedef struct shd_route_info {
    int32_t n_vertices;
    int32_t n_edges;
    int32_t n_arcs;          /* CSR arcs used by SSSP (self-loops excluded) */
    int32_t is_complete;     /* topology.c:450-552 */
    int32_t directed;
    int32_t prefer_direct;
    int32_t integer_weights; /* every latency integral and path sums exact in u32 */
    int32_t multigraph;      /* parallel edges present (SURVEY hazard H3) */
    int32_t device;
    int32_t lds_resident;    /* per-source state fits the 160 KiB LDS (KF above ~12k vertices: 0, KFH) */
    uint64_t device_bytes;   /* resident graph bytes */
    double min_edge_latency;
    int32_t kernel;          /* SSSP kernel: 0 = generic f64, 1 = integer K32 (LDS keys), 2 = KB/KBF
                              * (8 sources per workgroup, C2-class), 4 = KD (delta-stepping, u16
                              * distances, seeded plans), 5 = KF (f64 delta-stepping in LDS: the
                              * fractional-latency path; with lds_resident 0 its KFH form, vertex
                              * state in HBM, up to 65535 vertices); 3 = K16 in diagnostic builds only */
    int32_t dist_bound;      /* K32: proven bound on every shortest-path latency (ms) */
    int32_t block;           /* threads per workgroup of the SSSP kernel */
    int32_t reserved;        /* KD: bucket width delta; KB: 1 when path attributes are fused; KF:
                              * the packed arcs' decimal scale (latency = k / scale, 4 bytes per
                              * arc; 0 = f64 arcs) */
    int32_t lat16;           /* 1 when every table latency, the self-loop diagonal included, is an
                              * integer below 0xFFFF: the SHD_ROUTE_PAYLOAD_LAT16 eligibility */
} shd_route_info_t;

int shd_route_create(shd_route_t** out, const shd_graph_t* graph, int device);
void shd_route_destroy(shd_route_t* ctx);
int shd_route_get_info(const shd_route_t* ctx, shd_route_info_t* info);
const char* shd_route_strerror(int code);

/* Eager batch of SOURCE(s,.) rows: for i < ns, j < nt,
 *   lat_out[i*nt + j], rel_out[i*nt + j] = Path(src[i] -> tgt[j]);
 *   row_min_out[i] = min_j lat_out[i*nt + j]   (any of the three outputs may be NULL).
 * Host pointers; the call blocks.  SHD_ROUTE_ENOEDGE / SHD_ROUTE_EUNREACH are per-entry
 * failures: every row is still written, the failed entries are NaN (the reference skips
 * storing those targets, topology.c:1812-1870) and the code is returned at the end. */
int shd_route_rows(shd_route_t* ctx, const int32_t* src, int32_t ns, const int32_t* tgt,
                   int32_t nt, uint32_t flags, double* lat_out, double* rel_out,
                   double* row_min_out);

/* Same, all pointers device pointers (inputs already resident in HBM, outputs written
 * in HBM with row stride ld >= nt); enqueued on `stream` (a hipStream_t, NULL =
 * default stream); returns after enqueueing.  Errors detected on the device are
 * reported by the next shd_route_sync(). */
int shd_route_rows_async(shd_route_t* ctx, const int32_t* d_src, int32_t ns,
                         const int32_t* d_tgt, int32_t nt, int64_t ld, uint32_t flags,
                         double* d_lat, double* d_rel, double* d_row_min, void* stream);

/* Wait for `stream` and return the first device-side error raised since the last sync. */
int shd_route_sync(shd_route_t* ctx, void* stream);

/* Direct-path pairs (topology.c:1877-1927) for the full src x tgt block. */
int shd_route_direct(shd_route_t* ctx, const int32_t* src, int32_t ns, const int32_t* tgt,
                     int32_t nt, double* lat_out, double* rel_out, double* row_min_out);

/* Self paths (topology.c:1545-1653) for a list of vertices. */
int shd_route_self(shd_route_t* ctx, const int32_t* v, int32_t nv, double* lat_out,
                   double* rel_out);

/* Device-wide min over `count` non-negative doubles (runahead, topology.c:1374-1385).
 * Device pointers; result written to *d_out. */
int shd_route_min_reduce_async(shd_route_t* ctx, const double* d_vals, int64_t count,
                               double* d_out, void* stream);

/* ---- planned (seeded) rows: the eager fill of many sources at once -----------------
 * Replaces the same reference work as shd_route_rows (one SOURCE(s,.) row per source,
 * topology.c:1655-1875), planned over the whole source list.  A row whose source s has
 * a neighbour u among the planned sources may start from u's finished row: distances
 * w(s,u) + d_u(v) are path lengths that already satisfy every arc, so only the vertices
 * that improve on them are expanded, and the rows come out bit-identical to unseeded
 * rows (same distances, same engine tie rule for parents, same source-first products).
 * Up to three seeds per row; a row short of neighbour seeds takes rows two hops away,
 * and the first rows of the launch take landmark rows (the most central vertices' rows,
 * computed on the host when the plan is built).  The plan orders the rows into one
 * launch, where a row waits for its seeds' ready flags, and keeps the seeding rows (u16
 * distances + parent records per vertex) in a device row store.
 * Rows of a multi-GPU job: with world > 1 this rank's output rows are whole subtrees of
 * the seed forest (shd_route_plan_rows gives their positions in the caller's list), the
 * forest's top rows recomputed on every rank as helper rows.  Plans need the KD kernel
 * on an undirected integer-latency topology (else the plan falls back to plain rows);
 * SHD_ROUTE_SEED=0 in the environment disables seeding. */
typedef struct shd_route_plan shd_route_plan_t;

typedef struct shd_route_plan_info {
    int32_t rows;          /* output rows of this rank */
    int32_t seeded;        /* 1 = seeded launches, 0 = plain rows */
    int32_t launches;      /* kernel launches per shd_route_rows_planned_async */
    int32_t levels;        /* depth of the seed forest (longest chain of seeded rows) */
    int32_t roots;         /* rows computed from scratch (no neighbour, two-hop or landmark seed) */
    int32_t helpers;       /* rows computed only to seed others (no output) */
    int32_t stored_rows;   /* rows kept in the row store */
    int32_t world, rank;
    uint64_t store_bytes;  /* device bytes of the row store */
    int32_t delta;         /* the rows' bucket width (ms; at most the context's, info.reserved) */
    int32_t pad_;
} shd_route_plan_info_t;

int shd_route_plan_create(shd_route_t* ctx, const int32_t* src, int32_t ns, int32_t world, int32_t rank,
                          shd_route_plan_t** out);
void shd_route_plan_destroy(shd_route_plan_t* plan);  /* before its context's shd_route_destroy */
int shd_route_plan_get_info(const shd_route_plan_t* plan, shd_route_plan_info_t* info);
/* positions (in the caller's source list) of this rank's output rows, in row order */
int shd_route_plan_rows(const shd_route_plan_t* plan, int32_t* pos_out);
/* this rank's rows of the plan: row r of d_lat / d_rel / d_row_min = source
 * src[pos[r]]; device pointers as shd_route_rows_async.  A landmark-only plan built on the
 * device (256-thread contexts, and ranks with few rows per workgroup slot; info.launches 4)
 * seeds every row from its nearest landmark rows (the highest-degree vertices' exact rows),
 * and this call computes those landmark rows too, on the stream, before the rows: the
 * landmark rows and the job records derived from them (each row's nearest landmarks, its
 * offsets and seed records) are recomputed in every call, so every SSSP behind the table
 * runs inside it; the queue order is the plan's, fixed when it is made.  SHD_ROUTE_PLAN_REUSE skips that and reuses the
 * last computation (the plan's creation, or shd_route_plan_refresh_async), which a caller
 * may run separately to time the rows launch alone; other plans ignore the flag. */
#define SHD_ROUTE_PLAN_REUSE 0x200u
int shd_route_rows_planned_async(shd_route_t* ctx, const shd_route_plan_t* plan, const int32_t* d_tgt,
                                 int32_t nt, int64_t ld, uint32_t flags, double* d_lat, double* d_rel,
                                 double* d_row_min, void* stream);
/* the landmark rows, queue order and job records of a device-built landmark-only plan,
 * enqueued on the stream; SHD_ROUTE_OK and nothing enqueued for other plans.  `what`:
 * SHD_ROUTE_REFRESH_ALL computes every landmark row into the plan's store,
 * SHD_ROUTE_REFRESH_MINE only this rank's share (shd_route_plan_landmarks), and
 * SHD_ROUTE_REFRESH_JOBS derives the job records from the store as it stands; 0 = ALL | JOBS, what shd_route_rows_planned_async runs first without
 * SHD_ROUTE_PLAN_REUSE.  A multi-GPU rank runs MINE, exchanges the store slots with the
 * other ranks (an all-gather of equal shares), then JOBS and the rows with
 * SHD_ROUTE_PLAN_REUSE: each landmark row is computed once per job instead of once per rank.
 * No reference equivalent (Shadow 1.14 has no multi-process path, master.c:414-416). */
#define SHD_ROUTE_REFRESH_ALL 0x1u
#define SHD_ROUTE_REFRESH_MINE 0x2u
#define SHD_ROUTE_REFRESH_JOBS 0x4u
int shd_route_plan_refresh_async(shd_route_t* ctx, const shd_route_plan_t* plan, uint32_t what, void* stream);
/* the landmark store of such a plan: nland rows of row_stride u16 distances (d_drow) and as
 * many u32 parent records (d_prow), slot k = landmark k; this rank's share is the slots
 * [first, first + count).  SHD_ROUTE_EUNSUPPORTED for other plans. */
int shd_route_plan_landmarks(const shd_route_plan_t* plan, int32_t* nland, int32_t* first, int32_t* count,
                             int64_t* row_stride);
/* moves the plan's landmark store into caller memory (nland * row_stride elements each,
 * device, kept alive by the caller for the plan's lifetime), e.g. buffers a collective
 * library can all-gather into; the current contents are copied.  Blocks. */
int shd_route_plan_bind_store(shd_route_t* ctx, shd_route_plan_t* plan, uint16_t* d_drow, uint32_t* d_prow);

/* ---- the eager fill of a dense Path cache ------------------------------------------
 * The front end's cache (shd_topology.h) replaces topology.c's hash of Paths
 * (topology.c:1284-1386) with an upper triangle over the attached vertices A (sorted):
 * pair {A[i], A[j]}, i <= j, holds the Path of row i (first writer wins over both
 * directions under ascending sources, topology.c:1307-1336) as interleaved (lat, rel)
 * doubles at lr_out + 2 * (i * na - i * (i - 1) / 2 + (j - i)).  This fills the rows this
 * rank owns (world/rank: the plan's partition; world 1: all) with one seeded plan: rows
 * on the device, packed into the triangle layout and copied out in 512 MiB chunks on a
 * second stream while the next chunk packs.  lr_out is host memory, pinned for full
 * PCIe rate when it comes from shd_route_host_alloc.  *min_out = the smallest latency
 * written (topology.c:1374-1385), *seconds_out = the wall time (nullable).  Flags as
 * shd_route_rows (SHD_ROUTE_DISPATCH for the topology.c:2019 dispatch).  The rank's rows
 * are held whole in HBM (2 x 8 x rows x na bytes + 2 GiB; C4 on one GPU: 41 GB): a
 * larger request is SHD_ROUTE_ENOMEM (shard it over more devices).
 *
 * With SHD_ROUTE_FILL_LAT16 in flags the triangle is the compact layout instead (10.7 B per
 * pair against 16): row i starts a 64-byte line at line shd_route_tri16_line(na, i), and
 * its pairs j >= i go six to a line, pair e = j - i in line row_start + e / 6 at slot
 * e % 6 -- the line holds rel as 6 doubles (bytes 0-47), then lat as 6 u16 (bytes 48-59,
 * 0xFFFF = NaN), 4 pad bytes; a lookup is still one cache line.  Exact only when every
 * latency written is an integer below 0xFFFF (info.lat16, and the caller's direct-path
 * and self-path latencies): else SHD_ROUTE_EUNSUPPORTED.  lr_out then points at
 * 64 * shd_route_tri16_line(na, na) bytes (16-byte aligned). */
#define SHD_ROUTE_FILL_LAT16 0x100u
int shd_route_fill_triangle(shd_route_t* ctx, const int32_t* A, int32_t na, int32_t world, int32_t rank,
                            uint32_t flags, double* lr_out, double* min_out, double* seconds_out);

/* first 64-byte line of row i in the SHD_ROUTE_FILL_LAT16 triangle (i = na: the line count):
 * sum over r < i of ceil((na - r) / 6) */
static inline int64_t shd_route_tri16_line(int32_t na, int32_t i) {
    /* sum of (na - r) over r < i, plus the pads (6 - (na - r) % 6) % 6: period 6, sum 15 */
    int64_t pairs = (int64_t)i * na - (int64_t)i * (i - 1) / 2;
    int64_t pad = (int64_t)(i / 6) * 15;
    for (int32_t t = 0; t < i % 6; t++) pad += (6 - ((na - t) % 6 + 6) % 6) % 6;
    return (pairs + pad) / 6;
}
/* ---- multi-GPU table assembly payload (no reference equivalent: Shadow 1.14 is one
 * process, master.c:414-416).  The Path cache needs each unordered pair once
 * (topology.c:1307-1336: the first writer stores both directions), so the rows a rank
 * sends to the others are their upper triangles: row r of d_lat / d_rel (row stride ld,
 * na targets = the sorted attached list) is the row of attached position d_pos[r] and
 * keeps the targets j >= d_pos[r], packed at element offset d_off[r] - d_off[0] of
 * d_out_lat / d_out_rel (d_off: int64 per row, the caller's prefix sums of na - pos).
 * With SHD_ROUTE_PAYLOAD_LAT16 latencies go out as u16 (exact: integer latencies whose
 * shortest paths are below 65535 ms, proven at create, and integer self-loops below 65535
 * ms -- info.lat16; NaN -> 0xFFFF, which no latency takes; else SHD_ROUTE_EUNSUPPORTED),
 * otherwise as f64; rel always as f64.  C4 over 8 GPUs: 10 B
 * per pair of the triangle instead of 16 B per pair of the square (0.31x the bytes). */
#define SHD_ROUTE_PAYLOAD_LAT16 0x1u
int shd_route_tri_payload_async(shd_route_t* ctx, const double* d_lat, const double* d_rel, int64_t ld,
                                const int32_t* d_pos, const int64_t* d_off, int32_t nrows, int32_t na, uint32_t flags,
                                void* d_out_lat, double* d_out_rel, void* stream);

/* Pinned host memory (NULL on failure), for lr_out above: huge-page-advised anonymous
 * memory first-touched in 256 MiB chunks by background threads.  shd_route_host_alloc
 * returns once the whole buffer is touched and registered with HIP as ONE registration
 * (any copy may span it; hipHostMalloc if the registration fails).
 * shd_route_host_alloc_lazy returns at once and registers each 256 MiB chunk separately:
 * until shd_route_host_wait(p) returns, the memory may be used only as
 * shd_route_fill_triangle's lr_out (no CPU reads or writes: the workers first-touch each
 * chunk), whose copies wait for each chunk they land in -- so the fill's D2H overlaps the
 * pinning of the rest (C4's 13.3 GB triangle) instead of following it.  A caller's own
 * hipMemcpy into lazy memory must not span a 256 MiB chunk boundary (the runtime fails a
 * copy across two registrations).  shd_route_host_wait returns SHD_ROUTE_OK once every
 * chunk is settled, including a chunk the runtime refused to register (it stays pageable:
 * the fill's copies into it still complete, slower); shd_route_host_unpinned(p) waits the
 * same way and returns how many bytes of p stayed pageable (0 = all pinned; for memory not
 * from these allocators, 0).  shd_route_host_free takes either. */
void* shd_route_host_alloc(size_t bytes);
void* shd_route_host_alloc_lazy(size_t bytes);
int shd_route_host_wait(void* p);
int64_t shd_route_host_unpinned(void* p);
void shd_route_host_free(void* p);

/* KD liveness counters since the last reset (no reference equivalent): the longest single
 * wait, in s_sleep rounds, of the delta-stepping kernel's waves on each other -- out[0] a
 * compute wave for space in the parent-record ring, out[1] the writer wave on a reserved
 * record not yet written, out[2] a wave on a work-queue entry not yet written; out[3] 0.  A
 * stall (both sides of the ring spinning to their caps) shows as 2^22; healthy waits are
 * hundreds.  Synchronises the device; reset != 0 zeroes the counters. */
int shd_route_kd_stats(shd_route_t* ctx, uint64_t* out, int32_t reset);

/* K4: all-pairs shortest latencies by blocked min-plus
 * Floyd-Warshall over all vertices, u16 on the device (kept in the context).  Integer
 * latencies with every shortest path below 65535 ms, n <= 12000, simple graphs; else
 * SHD_ROUTE_EUNSUPPORTED.  No reference equivalent: Shadow 1.14 never takes shortest
 * paths on a complete graph (topology.c:1321-1323, 2019-2021); this is the dense
 * alternative to per-source SSSP. */
int shd_route_fw_table_async(shd_route_t* ctx, void* stream);

/* SOURCE(s,.) rows (as shd_route_rows_async without dispatch: topology.c:1407-1523)
 * from the resident K4 table: lat from the table, the parent of each vertex by the
 * engine tie rule among its tight in-arcs, rel the source-first product down that
 * tree.  Same entries as shd_route_rows_async bit for bit (integer latencies).  Device
 * pointers; call shd_route_fw_table_async first (same stream or synchronised). */
int shd_route_fw_rows_async(shd_route_t* ctx, const int32_t* d_src, int32_t ns, const int32_t* d_tgt,
                            int32_t nt, int64_t ld, double* d_lat, double* d_rel, double* d_row_min,
                            void* stream);

/* Dense all-pairs shortest latencies by blocked min-plus Floyd-Warshall over all
 * vertices: d_dist is n x n (device, row-major).  Bit-exact against Dijkstra only
 * for integer-valued latencies (fl sums of subpaths are not left folds otherwise). */
int shd_route_fw_async(shd_route_t* ctx, double* d_dist, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SHD_ROUTE_H */
