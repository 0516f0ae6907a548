/*
 * oracle.h -- CPU restatement of Shadow 1.14's topology path computation.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (shadow_amd/, include/)
 * links, loads or calls this code.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * Parity status: the reference (mckerrigan/shadow src/main/routing/topology.c)
 * cannot be compiled here: its arithmetic lives in igraph 0.7.1 (not vendored,
 * not installed, no network).  This file restates
 *   - topology.c:402-444   _topology_getEdgeHelper   (get_eid, r_e = 1 - loss_e)
 *   - topology.c:450-552   _topology_isComplete
 *   - topology.c:1307-1386 _topology_shouldStorePath / _topology_storePathInCache
 *   - topology.c:1407-1523 _topology_computePathProperties
 *   - topology.c:1545-1653 _topology_computeShortestPathToSelf
 *   - topology.c:1655-1875 _topology_computeSourcePaths
 *   - topology.c:1877-1927 _topology_lookupDirectPath
 *   - topology.c:1969-2051 _topology_getPathEntry (eager, ascending-source order)
 *   - master.c:148-159     runahead truncation
 * plus igraph 0.7.1's igraph_get_shortest_paths_dijkstra, 2-way indexed heap
 * and igraph_incident order (published algorithm, restated from the 0.7.1
 * sources' documented behaviour).
 * It is pinned by the reference's own fixtures (1-vertex configs under
 * src/test/ and resource/examples, the bundled 183-vertex complete topology)
 * and cross-checked against networkx for latency (tests/test_oracle.py).
 * Multi-vertex Dijkstra-mode reliability on tied shortest paths depends on
 * the recalled igraph heap order and is therefore only "pinned" by that
 * restatement; unique-shortest-path pairs are order independent.
 */
#ifndef SHD_ORACLE_H
#define SHD_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_graph orc_graph;

/* Tie-break rules for the shortest-path tree. */
enum {
    ORC_TIE_IGRAPH = 0, /* igraph 0.7.1 2-way-heap pop order (the reference) */
    ORC_TIE_MINKEY = 1  /* engine rule: parent = argmin (dist[u], u, eid) over tight in-arcs */
};

/* Build the igraph-like indexed edge list. vloss may be NULL (attribute absent);
 * NaN entries mean "absent" (topology.c:330-347). Returns NULL on bad input. */
orc_graph* orc_graph_new(int32_t n, int32_t m, const int32_t* from, const int32_t* to,
                         const double* latency, const double* packetloss,
                         const double* vertex_packetloss, int32_t directed);
void orc_graph_free(orc_graph* g);

int32_t orc_is_complete(const orc_graph* g);                    /* topology.c:450-552 */
int64_t orc_get_eid(const orc_graph* g, int32_t from, int32_t to); /* -1 if none */

/* One single-source Dijkstra. dist[n] (-1.0 = unreached), parent_eid[n] (-1 = none). */
int32_t orc_dijkstra(const orc_graph* g, int32_t src, int32_t tiebreak,
                     double* dist, int64_t* parent_eid);

/* SOURCE(s, .) raw row (topology.c:1655-1875 batch semantics, no store filter):
 * lat/rel for each target; unique[j] = 1 iff the shortest s->t path is unique
 * (nullable); hops[j] = edges on the chosen path (nullable).
 * Returns 0, or -1 if a hop has no edge (missing self-loop, topology.c:1488-1495). */
int32_t orc_source_row(const orc_graph* g, int32_t src, const int32_t* tgt, int32_t nt,
                       int32_t tiebreak, double* lat, double* rel, uint8_t* unique,
                       int32_t* hops);

/* DIRECT(s,t) (topology.c:1877-1927). Returns 0, or -1 if no edge. */
int32_t orc_direct(const orc_graph* g, int32_t s, int32_t t, double* lat, double* rel);

/* SELF(s) (topology.c:1545-1653): twice the first min-latency incident edge. */
int32_t orc_self_path(const orc_graph* g, int32_t s, double* lat, double* rel);

/* Eager path cache: attached set A (ascending vertex ids),
 * dense |A|x|A| answer to lookup(A[i], A[j]) after an ascending-source fill,
 * is_direct flags (nullable), unique flags (nullable), min stored latency.
 * prefer_direct is the graph's 'preferdirectpaths' flag. */
int32_t orc_eager_table(const orc_graph* g, const int32_t* A, int32_t na, int32_t prefer_direct,
                        int32_t tiebreak, double* lat, double* rel, uint8_t* is_direct,
                        uint8_t* unique, double* min_latency);

/* master.c:148-159: (SimulationTime)minPathLatency * 1e6 ns; 10 ms default if unset/0. */
uint64_t orc_runahead_ns(double min_latency);

/* CPU baselines (bench.py cpu_baseline).  Both return elapsed seconds.
 * faithful: 1 thread, per source igraph-order Dijkstra + per-target path walk with
 *   get_eid per hop and the unconditional path/log string formatting of
 *   topology.c:1449,1502,1831 (the reference serialises Dijkstra under graphLock).
 * parallel: OpenMP over sources, no formatting; threads<=0 means all cores. */
double orc_bench_faithful(const orc_graph* g, const int32_t* src, int32_t ns,
                          const int32_t* tgt, int32_t nt, double* checksum);
double orc_bench_parallel(const orc_graph* g, const int32_t* src, int32_t ns,
                          const int32_t* tgt, int32_t nt, int32_t threads,
                          double* checksum, int32_t* threads_used);
/* C5 (complete graph): the direct fill of every pair of A (topology.c:1877-1927), rows
 * over OpenMP threads; and nk k-phases of f64 Floyd-Warshall from k0 over n x n d
 * (extrapolate x n/nk).  Both return elapsed seconds. */
double orc_bench_direct(const orc_graph* g, const int32_t* A, int32_t na, int32_t threads,
                        double* checksum, int32_t* threads_used);
double orc_bench_fw_phases(int32_t n, double* d, int32_t k0, int32_t nk, int32_t threads,
                           int32_t* threads_used);

/* Blocked-free reference Floyd-Warshall over dense n x n (for K4 parity),
 * d is n*n row-major with +inf for no edge; in-place. */
void orc_floyd_warshall(int32_t n, double* d);

#ifdef __cplusplus
}
#endif
#endif
