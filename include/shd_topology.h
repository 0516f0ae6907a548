/*
 * shd_topology.h -- C front end with the semantics of Shadow 1.14's
 * src/main/routing/topology.c (mckerrigan/shadow), keyed by vertex index.
 *
 * Shadow's own topology.c keeps its public API (topology.h:17-28) and its
 * Address->vertex map (virtualIP, topology.c:1388-1405); each public function then
 * becomes a one-line call into this module.  Behind it:
 *   - graphml loading with igraph_read_graph_graphml numbering (document order,
 *     missing numeric attribute = NaN) and the validation of topology.c:565-1185;
 *   - the Path cache as dense upper-triangle arrays over the attached vertices,
 *     filled eagerly (ascending sources, first writer wins over both directions,
 *     topology.c:1307-1336) by the HIP engine (include/shd_route.h) on the first
 *     cache miss, optionally sharded over several GPUs;
 *   - minimumPathLatency and the runahead it implies (topology.c:1374-1385,
 *     master.c:148-159).
 * Functions returning int use SHD_ROUTE_* codes; getters return -1 on error like
 * topology_getLatency / topology_getReliability (topology.c:2065-2087).
 */
#ifndef SHD_TOPOLOGY_H
#define SHD_TOPOLOGY_H

#include <stdint.h>
#include <stdio.h>

#include "shd_route.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct shd_topology shd_topology_t;

/* graphml -> igraph-numbered arrays (plain or .xz/.gz file).  On success the caller
 * owns *out (release with shd_graphml_free). Validation as topology.c:565-1185;
 * returns SHD_ROUTE_EINVAL with a message in errbuf on failure. */
enum { SHD_VATTR_IP, SHD_VATTR_CITYCODE, SHD_VATTR_COUNTRYCODE, SHD_VATTR_GEOCODE, SHD_VATTR_TYPE, SHD_VATTR_N };
typedef struct shd_graphml {
    shd_graph_t graph;         /* arrays owned by this struct */
    char** vertex_ids;         /* graphml node id of each vertex */
    double* bandwidth_down;    /* vertex attributes Shadow reads at attach time */
    double* bandwidth_up;
    int32_t has_vertex_packetloss;
    /* string vertex attributes ip, citycode, countrycode, geocode, type (SHD_VATTR_*):
     * has = the key is declared for nodes; values as igraph holds them (key default or
     * "" where a node has no <data>); NULL arrays when the key is not declared */
    int32_t has_vertex_str[SHD_VATTR_N];
    char** vertex_str[SHD_VATTR_N];
} shd_graphml_t;
int shd_graphml_load(const char* path, shd_graphml_t* out, char* errbuf, size_t errlen);
void shd_graphml_free(shd_graphml_t* g);

/* topology_new (topology.c:2486-2510): load, validate, make one engine context per
 * device in `devices` (NULL/0 -> device 0).  NULL on failure. */
shd_topology_t* shd_topology_new(const char* graph_path, const int* devices, int ndev);
shd_topology_t* shd_topology_new_from_graph(const shd_graph_t* g, const int* devices, int ndev);
void shd_topology_free(shd_topology_t* top);  /* topology_free (topology.c:2441) */

int32_t shd_topology_vertex_count(const shd_topology_t* top);
int32_t shd_topology_find_vertex(const shd_topology_t* top, const char* graphml_id);

/* topology_attach's effect on routing (topology.c:2371-2439): the vertex joins
 * verticesWithAttachedHosts; detach never shrinks it (topology.c:2437). */
int shd_topology_attach_vertex(shd_topology_t* top, int32_t vertex);
int32_t shd_topology_attached_count(const shd_topology_t* top);

/* Host attachment: _topology_findAttachmentVertex (topology.c:2245-2366) with its
 * per-vertex filter hook (topology.c:2094-2216) and longest-prefix match
 * (topology.c:2218-2243).  The index interns each vertex's parsed IP and case-folded
 * codes once, with posting lists per code and sorted IPs, so a lookup touches only the
 * candidates of the chosen list instead of making 5 igraph string-attribute lookups
 * per vertex.  Hints may be NULL.
 * next_double(ctx) is called exactly where the reference calls
 * random_nextDouble(randomSourcePool) (one draw, only when no longest-prefix match is
 * used), so a caller passing Shadow's Random keeps its stream bit for bit.
 * Returns the vertex index, or -1 (no vertices / bad arguments). */
typedef struct shd_attach shd_attach_t;
typedef double (*shd_next_double_fn)(void* ctx);
int shd_attach_create(shd_attach_t** out, const shd_graphml_t* g);
int32_t shd_attach_find_vertex(const shd_attach_t* a, shd_next_double_fn next_double, void* ctx,
                               const char* ip_hint, const char* citycode_hint, const char* countrycode_hint,
                               const char* geocode_hint, const char* type_hint);
void shd_attach_destroy(shd_attach_t* a);

/* topology_attach (topology.c:2371-2439) for a topology loaded from graphml: pick the
 * vertex as above, attach it, return the vertex (-1 on error) and, when the out
 * pointers are non-NULL, its bandwidths truncated to integers like (guint64) casts. */
int32_t shd_topology_attach(shd_topology_t* top, shd_next_double_fn next_double, void* ctx,
                            const char* ip_hint, const char* citycode_hint, const char* countrycode_hint,
                            const char* geocode_hint, const char* type_hint,
                            uint64_t* bw_down_out, uint64_t* bw_up_out);

/* Public accessors (topology.c:2053-2092); fill the cache on the first miss. */
double shd_topology_get_latency(shd_topology_t* top, int32_t src, int32_t dst);
double shd_topology_get_reliability(shd_topology_t* top, int32_t src, int32_t dst);
int shd_topology_is_routable(shd_topology_t* top, int32_t src, int32_t dst);
void shd_topology_increment_path_packet_counter(shd_topology_t* top, int32_t src, int32_t dst);
uint64_t shd_topology_get_path_packet_count(shd_topology_t* top, int32_t src, int32_t dst);
int shd_topology_is_direct_path(shd_topology_t* top, int32_t src, int32_t dst);

/* minimumPathLatency over all cached Paths and the runahead it sets (ns). */
double shd_topology_min_path_latency(shd_topology_t* top);
uint64_t shd_topology_runahead_ns(shd_topology_t* top);

/* Explicit eager fill (otherwise done by the first accessor); seconds spent in
 * *elapsed_s (nullable), like shortestPathTotalTime (topology.c:1751-1788). */
int shd_topology_fill(shd_topology_t* top, double* elapsed_s);
/* Host bytes of the current fill's triangle (0 before the first fill): 16 per pair
 * (interleaved lat/rel doubles) or the compact layout of shd_route_fill_triangle
 * (SHD_ROUTE_FILL_LAT16, 64 bytes per six pairs of a row), chosen at creation when every
 * stored latency is an integer below 0xFFFF (env SHD_TOPOLOGY_LAT16=0 keeps the doubles). */
uint64_t shd_topology_triangle_bytes(shd_topology_t* top);

/* _topology_logAllCachedPaths (topology.c:1929-1967): one line per cached Path. */
int shd_topology_dump_paths(shd_topology_t* top, FILE* out);

#ifdef __cplusplus
}
#endif
#endif /* SHD_TOPOLOGY_H */
