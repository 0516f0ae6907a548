/*
 * topology.c -- Shadow 1.14's src/main/routing/topology.c with the MI355X engine behind
 * it: the drop-in this repo proposes, compiled and run here
 * against shadow_env.h.  Every public function keeps its reference signature
 * (topology.h:17-28); the graph, the Path cache, the Dijkstra runs, the locks around
 * them and the runahead bookkeeping move into libshd_topology / libshd_route.  What
 * stays here is Shadow's own Address -> vertex map (virtualIP, topology.c:1388-1405).
 */
#include "topology.h"

#include "../include/shd_topology.h"

struct _Topology {
    shd_topology_t* route;     /* graph, Path cache, GPU fill, runahead (shd_topology.h) */
    GHashTable* virtualIP;     /* IP -> vertex, as topology.c:40-41 */
    GRWLock virtualIPLock;
    gint reportedRunahead;     /* the one worker_updateMinTimeJump call (see below) */
    MAGIC_DECLARE;
};

static int _gpu_count(void) {
    const char* e = getenv("SHD_GPUS");  /* devices the eager fill shards its rows over */
    int n = e ? atoi(e) : 1;
    return n > 0 && n <= 64 ? n : 1;
}

Topology* topology_new(const gchar* graphPath) {               /* topology.c:2486-2510 */
    Topology* top = g_new0(Topology, 1);
    MAGIC_INIT(top);
    int devices[64];
    const int nd = _gpu_count();
    for (int d = 0; d < nd; d++) devices[d] = d;
    top->route = shd_topology_new(graphPath, devices, nd);
    if (!top->route) {
        critical("fatal error loading topology at path '%s'", graphPath);
        MAGIC_CLEAR(top);
        g_free(top);
        return NULL;
    }
    top->virtualIP = g_hash_table_new(g_direct_hash, g_direct_equal);
    g_rw_lock_init(&top->virtualIPLock);
    return top;
}

static gdouble _next_double(void* rnd) { return random_nextDouble((Random*)rnd); }

void topology_attach(Topology* top, Address* address, Random* randomSourcePool, gchar* ipHint,
                     gchar* citycodeHint, gchar* countrycodeHint, gchar* geocodeHint, gchar* typeHint,
                     guint64* bwDownOut, guint64* bwUpOut) {          /* topology.c:2371-2423 */
    MAGIC_ASSERT(top);
    /* _topology_findAttachmentVertex (topology.c:2245-2366) over the front end's index,
     * drawing random_nextDouble exactly where the reference draws */
    gint v = shd_topology_attach(top->route, _next_double, randomSourcePool, ipHint, citycodeHint,
                                 countrycodeHint, geocodeHint, typeHint, bwDownOut, bwUpOut);
    if (v < 0) {
        critical("unable to attach host to the topology");
        return;
    }
    g_rw_lock_writer_lock(&top->virtualIPLock);
    g_hash_table_replace(top->virtualIP, GUINT_TO_POINTER(address_toNetworkIP(address)), GINT_TO_POINTER(v));
    g_rw_lock_writer_unlock(&top->virtualIPLock);
}

void topology_detach(Topology* top, Address* address) {       /* topology.c:2432-2439 */
    MAGIC_ASSERT(top);
    /* the address leaves the map; the vertex stays among the attached ones */
    g_rw_lock_writer_lock(&top->virtualIPLock);
    g_hash_table_remove(top->virtualIP, GUINT_TO_POINTER(address_toNetworkIP(address)));
    g_rw_lock_writer_unlock(&top->virtualIPLock);
}

/* _topology_getConnectedVertexIndex (topology.c:1388-1405): lookup_extended, so vertex 0
 * is found; -1 when the address is not attached */
static gint _vertex(Topology* top, Address* a) {
    gpointer p = NULL;
    g_rw_lock_reader_lock(&top->virtualIPLock);
    const gboolean found =
        g_hash_table_lookup_extended(top->virtualIP, GUINT_TO_POINTER(address_toNetworkIP(a)), NULL, &p);
    g_rw_lock_reader_unlock(&top->virtualIPLock);
    return found ? GPOINTER_TO_INT(p) : -1;
}

/* test hook (not part of topology.h): the vertex an address is attached to, -1 if none */
gint topology_testVertexOf(Topology* top, Address* a) { return _vertex(top, a); }

/* The reference reports a new minimum from _topology_storePathInCache on every decrease
 * (topology.c:1383-1385); the eager fill knows the true minimum at the first lookup, so
 * the glue reports it once, from the first looking-up worker thread */
static void _report_runahead(Topology* top) {
    if (g_atomic_int_get(&top->reportedRunahead)) return;
    const gdouble m = shd_topology_min_path_latency(top->route);
    if (m > 0 && g_atomic_int_compare_and_exchange(&top->reportedRunahead, 0, 1)) worker_updateMinTimeJump(m);
}

gdouble topology_getLatency(Topology* top, Address* s, Address* d) {            /* :2065 */
    MAGIC_ASSERT(top);
    const gdouble v = shd_topology_get_latency(top->route, _vertex(top, s), _vertex(top, d));
    _report_runahead(top);
    return v;
}

gdouble topology_getReliability(Topology* top, Address* s, Address* d) {        /* :2077 */
    MAGIC_ASSERT(top);
    const gdouble v = shd_topology_get_reliability(top->route, _vertex(top, s), _vertex(top, d));
    _report_runahead(top);
    return v;
}

gboolean topology_isRoutable(Topology* top, Address* s, Address* d) {           /* :2089 */
    MAGIC_ASSERT(top);
    return shd_topology_is_routable(top->route, _vertex(top, s), _vertex(top, d)) ? TRUE : FALSE;
}

void topology_incrementPathPacketCounter(Topology* top, Address* s, Address* d) {  /* :2053 */
    MAGIC_ASSERT(top);
    shd_topology_increment_path_packet_counter(top->route, _vertex(top, s), _vertex(top, d));
}

void topology_free(Topology* top) {                            /* topology.c:2441-2484 */
    MAGIC_ASSERT(top);
    const char* dump = getenv("SHD_DUMP_PATHS");  /* _topology_logAllCachedPaths */
    if (dump && *dump) {
        FILE* f = fopen(dump, "w");
        if (f) { shd_topology_dump_paths(top->route, f); fclose(f); }
    }
    shd_topology_free(top->route);
    g_hash_table_destroy(top->virtualIP);
    g_rw_lock_clear(&top->virtualIPLock);
    MAGIC_CLEAR(top);
    g_free(top);
}
