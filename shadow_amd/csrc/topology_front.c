/*
 * topology_front.c -- the Path cache and public accessors of Shadow 1.14's
 * src/main/routing/topology.c, rebuilt over the HIP routing engine (shd_route.h).
 *
 * Reference behaviour kept (file:line in mckerrigan/shadow):
 *   - one Path per unordered pair, first writer wins over both directions
 *     (_topology_shouldStorePath, topology.c:1307-1336); lookups probe (s,d) then
 *     (d,s) (topology.c:1987-1990, 2033-2037).  With the fill running over attached
 *     sources in ascending order, the stored orientation of {s,t} is from min(s,t),
 *     so the cache is one upper triangle over the attached vertices.
 *   - dispatch complete / prefer-direct+adjacent -> direct path, else source paths
 *     (topology.c:2019-2031), self entry = batch self-loop hop;
 *   - minimumPathLatency over every stored Path (topology.c:1374-1385) and the
 *     runahead it implies, truncated to whole ms (master.c:148-159, 10 ms default);
 *   - -1 from the getters when a vertex has no attached host (topology.c:1973-1985);
 *   - verticesWithAttachedHosts never shrinks on detach (topology.c:2437).
 * What changes: the cache is dense (|A|(|A|+1)/2 latency + reliability doubles
 * instead of a glib hash of 48-byte Paths), it is filled eagerly at the first miss
 * by batched GPU rows (instead of one serialised igraph Dijkstra per missing source,
 * topology.c:1747-1781), and the fill can shard sources over several GPUs.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/shd_topology.h"

typedef struct {
    uint64_t key;    /* triangle index + 1, 0 = empty */
    uint64_t val;
} pcslot;
typedef struct {
    pthread_mutex_t lock;
    pcslot* s;       /* key and count in one slot: one cache miss per probe */
    size_t cap, len;
} __attribute__((aligned(64))) pcmap;  /* one stripe per cache line: no false sharing */

#define PC_STRIPES 64
static inline unsigned pc_stripe(uint64_t key) { return (unsigned)((key * 0xD6E8FEB86659FD93ull) >> 58); }

/* One fill of the Path cache over the attached set of its time.  Published to readers
 * with a release store and never changed or freed while the topology lives: a late
 * attach retires it (readers still holding it stay valid) and the next lookup fills a
 * new one, carrying the packet counters over.  Lookups pay one acquire load. */
typedef struct pcache {
    int32_t na;
    int32_t* A;          /* sorted attached vertices */
    int32_t* cid;        /* vertex -> index in A, -1 = not attached */
    double* lr;          /* (lat, rel) pairs: one cache line serves both getters; or, with
                          * l16, the compact layout of shd_route.h (SHD_ROUTE_FILL_LAT16): six
                          * pairs per 64-byte line, rel f64 x 6 then lat u16 x 6 */
    int l16;
    int64_t* row16;      /* l16: first line of each row (na + 1) */
    uint32_t* cnt;       /* packet counters per pair (calloc: pages commit on first touch);
                          * each 2^32 wrap adds 2^32 to the striped spill map pc */
    double min_lat;
    pcmap pc[PC_STRIPES];  /* spill map for counters past 2^32, striped over locks */
    struct pcache* older;  /* retired fills (freed with the topology) */
} pcache;

struct shd_topology {
    shd_graphml_t gml;   /* owns the arrays when loaded from a file */
    shd_graph_t g;       /* view used by the engine */
    int owns_copy;       /* arrays copied by shd_topology_new_from_graph */
    int ndev;
    shd_route_t** eng;
    int32_t n;
    int complete, directed, prefer_direct;
    int lat16;           /* the fill may use the compact layout: every latency it stores is an
                          * integer below 0xFFFF (engine info.lat16; direct and self paths are
                          * edge latencies or twice one: 2 * max edge latency < 0xFFFF) */
    /* host adjacency for the prefer-direct isDirect flags */
    int32_t* arow;
    int32_t* acol;
    /* attached set */
    uint8_t* attached;
    int32_t nattached;
    /* dense cache over A (sorted attached vertices), upper triangle incl. diagonal */
    pcache* cache;       /* current fill (acquire/release), NULL = fill at the next lookup */
    pcache* retired;     /* the fills a late attach replaced */
    double fill_seconds;
    pthread_mutex_t lock;
    shd_attach_t* at;    /* host attachment index (graphml topologies only) */
};

static inline size_t tri(int32_t na, int32_t i, int32_t j) { /* i <= j */
    return (size_t)i * (size_t)na - ((size_t)i * (size_t)(i - 1)) / 2 + (size_t)(j - i);
}

/* the stored Path of pair (i, j), i <= j: latency (NaN = never stored) and reliability,
 * from the interleaved doubles or from the compact line layout (widened exactly) */
static inline double lat_at(const pcache* c, int32_t i, int32_t j) {
    if (c->l16) {
        const int64_t e = j - i;
        const unsigned char* line = (const unsigned char*)c->lr + 64 * (c->row16[i] + e / 6);
        const uint16_t x = ((const uint16_t*)(line + 48))[e % 6];
        return x == 0xFFFFu ? NAN : (double)x;
    }
    return c->lr[2 * tri(c->na, i, j)];
}
static inline double rel_at(const pcache* c, int32_t i, int32_t j) {
    if (c->l16) {
        const int64_t e = j - i;
        return ((const double*)((const unsigned char*)c->lr + 64 * (c->row16[i] + e / 6)))[e % 6];
    }
    return c->lr[2 * tri(c->na, i, j) + 1];
}
static inline void set_at(pcache* c, int32_t i, int32_t j, double lat, double rel) {
    if (c->l16) {
        const int64_t e = j - i;
        unsigned char* line = (unsigned char*)c->lr + 64 * (c->row16[i] + e / 6);
        ((uint16_t*)(line + 48))[e % 6] = isnan(lat) ? (uint16_t)0xFFFFu : (uint16_t)lat;
        ((double*)line)[e % 6] = rel;
        return;
    }
    c->lr[2 * tri(c->na, i, j)] = lat;
    c->lr[2 * tri(c->na, i, j) + 1] = rel;
}

static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return (x > y) - (x < y);
}

static void build_adjacency(shd_topology_t* t) {
    const shd_graph_t* g = &t->g;
    int32_t n = g->n_vertices;
    t->arow = calloc((size_t)n + 1, sizeof(int32_t));
    for (int32_t e = 0; e < g->n_edges; e++) {
        t->arow[g->edge_src[e] + 1]++;
        if (!g->directed && g->edge_src[e] != g->edge_dst[e]) t->arow[g->edge_dst[e] + 1]++;
    }
    for (int32_t v = 0; v < n; v++) t->arow[v + 1] += t->arow[v];
    t->acol = malloc(sizeof(int32_t) * ((size_t)t->arow[n] + 1));
    int32_t* fill = malloc(sizeof(int32_t) * ((size_t)n + 1));
    memcpy(fill, t->arow, sizeof(int32_t) * (size_t)n);
    for (int32_t e = 0; e < g->n_edges; e++) {
        int32_t a = g->edge_src[e], b = g->edge_dst[e];
        t->acol[fill[a]++] = b;
        if (!g->directed && a != b) t->acol[fill[b]++] = a;
    }
    free(fill);
    for (int32_t v = 0; v < n; v++) qsort(t->acol + t->arow[v], (size_t)(t->arow[v + 1] - t->arow[v]), sizeof(int32_t), cmp_i32);
}

/* _topology_verticesAreAdjacent (topology.c:1248-1264) via get_eid semantics */
static int adjacent(const shd_topology_t* t, int32_t s, int32_t d) {
    int32_t lo = t->arow[s], hi = t->arow[s + 1];
    while (lo < hi) {
        int32_t mid = (lo + hi) / 2;
        if (t->acol[mid] < d) lo = mid + 1;
        else if (t->acol[mid] > d) hi = mid;
        else return 1;
    }
    return 0;
}

#define FILL_MAX_DEV 64  /* fill worker threads (one per device context) */

static uint64_t* pc_slot(pcmap* m, uint64_t key);

static void pcache_free(pcache* c) {
    while (c) {
        pcache* o = c->older;
        free(c->A); free(c->cid); shd_route_host_free(c->lr); free(c->cnt); free(c->row16);
        for (int k = 0; k < PC_STRIPES; k++) { pthread_mutex_destroy(&c->pc[k].lock); free(c->pc[k].s); }
        free(c);
        c = o;
    }
}

static shd_topology_t* finish_new(shd_topology_t* t, const int* devices, int ndev) {
    t->n = t->g.n_vertices;
    t->ndev = ndev > 0 ? (ndev < FILL_MAX_DEV ? ndev : FILL_MAX_DEV) : 1;
    t->eng = calloc((size_t)t->ndev, sizeof(shd_route_t*));
    for (int d = 0; d < t->ndev; d++) {
        int dev = (devices && ndev > 0) ? devices[d] : 0;
        if (shd_route_create(&t->eng[d], &t->g, dev) != SHD_ROUTE_OK) {
            shd_topology_free(t);
            return NULL;
        }
    }
    shd_route_info_t info;
    shd_route_get_info(t->eng[0], &info);
    t->complete = info.is_complete;
    t->directed = info.directed;
    t->prefer_direct = info.prefer_direct;
    double maxw = 0;
    for (int32_t e = 0; e < t->g.n_edges; e++)
        if (t->g.edge_latency[e] > maxw) maxw = t->g.edge_latency[e];
    const char* e16 = getenv("SHD_TOPOLOGY_LAT16");  /* "0": keep the interleaved doubles (A/B) */
    t->lat16 = info.lat16 && 2.0 * maxw < 65535.0 && !(e16 && atoi(e16) == 0);
    t->attached = calloc((size_t)t->n, 1);
    build_adjacency(t);
    pthread_mutex_init(&t->lock, NULL);
    return t;
}

/* the counter stripes are cache-line aligned: allocate the struct that way */
static shd_topology_t* alloc_top(void) {
    const size_t sz = (sizeof(shd_topology_t) + 63) & ~(size_t)63;
    shd_topology_t* t = aligned_alloc(64, sz);
    if (t) memset(t, 0, sz);
    return t;
}

shd_topology_t* shd_topology_new(const char* graph_path, const int* devices, int ndev) {
    shd_topology_t* t = alloc_top();
    char err[512];
    if (shd_graphml_load(graph_path, &t->gml, err, sizeof(err)) != SHD_ROUTE_OK) {
        fprintf(stderr, "shd_topology_new: %s\n", err);
        free(t);
        return NULL;
    }
    t->g = t->gml.graph;
    if (shd_attach_create(&t->at, &t->gml) != SHD_ROUTE_OK) t->at = NULL;
    return finish_new(t, devices, ndev);
}

shd_topology_t* shd_topology_new_from_graph(const shd_graph_t* g, const int* devices, int ndev) {
    if (!g || g->n_vertices <= 0) return NULL;
    shd_topology_t* t = alloc_top();
    t->owns_copy = 1;
    t->g = *g;
    size_t m = (size_t)g->n_edges, n = (size_t)g->n_vertices;
    int32_t* s = malloc(sizeof(int32_t) * (m + 1));
    int32_t* d = malloc(sizeof(int32_t) * (m + 1));
    double* l = malloc(sizeof(double) * (m + 1));
    double* p = malloc(sizeof(double) * (m + 1));
    memcpy(s, g->edge_src, sizeof(int32_t) * m); memcpy(d, g->edge_dst, sizeof(int32_t) * m);
    memcpy(l, g->edge_latency, sizeof(double) * m); memcpy(p, g->edge_packetloss, sizeof(double) * m);
    t->g.edge_src = s; t->g.edge_dst = d; t->g.edge_latency = l; t->g.edge_packetloss = p;
    if (g->vertex_packetloss) {
        double* vl = malloc(sizeof(double) * n);
        memcpy(vl, g->vertex_packetloss, sizeof(double) * n);
        t->g.vertex_packetloss = vl;
    }
    return finish_new(t, devices, ndev);
}

void shd_topology_free(shd_topology_t* t) {
    if (!t) return;
    if (t->eng) for (int d = 0; d < t->ndev; d++) if (t->eng[d]) shd_route_destroy(t->eng[d]);
    free(t->eng);
    if (t->owns_copy) {
        free((void*)t->g.edge_src); free((void*)t->g.edge_dst); free((void*)t->g.edge_latency);
        free((void*)t->g.edge_packetloss); free((void*)t->g.vertex_packetloss);
    }
    shd_attach_destroy(t->at);
    shd_graphml_free(&t->gml);
    free(t->arow); free(t->acol); free(t->attached);
    pcache_free(t->cache);
    pcache_free(t->retired);
    free(t);
}

int32_t shd_topology_vertex_count(const shd_topology_t* t) { return t ? t->n : -1; }

int32_t shd_topology_find_vertex(const shd_topology_t* t, const char* id) {
    if (!t || !id || !t->gml.vertex_ids) return -1;
    for (int32_t v = 0; v < t->n; v++)
        if (!strcmp(t->gml.vertex_ids[v], id)) return v;
    return -1;
}

int shd_topology_attach_vertex(shd_topology_t* t, int32_t v) {
    if (!t || v < 0 || v >= t->n) return SHD_ROUTE_EINVAL;
    pthread_mutex_lock(&t->lock);
    if (!t->attached[v]) {
        t->attached[v] = 1;
        t->nattached++;
        /* the next lookup refills over the grown attached set (paths do not depend on the
         * target set, so pairs already cached keep their values; their counters move over).
         * Readers still holding the old fill keep a valid one: it is retired, not freed */
        pcache* c = t->cache;
        if (c) {
            __atomic_store_n(&t->cache, (pcache*)NULL, __ATOMIC_RELEASE);
            c->older = t->retired;
            t->retired = c;
        }
    }
    pthread_mutex_unlock(&t->lock);
    return SHD_ROUTE_OK;
}

int32_t shd_topology_attach(shd_topology_t* t, shd_next_double_fn next_double, void* ctx,
                            const char* ip_hint, const char* citycode_hint, const char* countrycode_hint,
                            const char* geocode_hint, const char* type_hint,
                            uint64_t* bw_down_out, uint64_t* bw_up_out) {
    if (!t || !t->at) return -1;
    const int32_t v = shd_attach_find_vertex(t->at, next_double, ctx, ip_hint, citycode_hint, countrycode_hint,
                                             geocode_hint, type_hint);
    if (v < 0 || shd_topology_attach_vertex(t, v) != SHD_ROUTE_OK) return -1;
    /* topology.c:2394-2405: default cluster bandwidths, (guint64) casts */
    if (bw_up_out) *bw_up_out = (uint64_t)t->gml.bandwidth_up[v];
    if (bw_down_out) *bw_down_out = (uint64_t)t->gml.bandwidth_down[v];
    return v;
}

int32_t shd_topology_attached_count(const shd_topology_t* t) { return t ? t->nattached : -1; }

typedef struct {
    shd_topology_t* t;
    pcache* c;
    int dev, nd;
    int rc;
    double min_lat;
} fill_job;

/* One thread per device context: the rows its plan share owns (shd_route_fill_triangle:
 * one seeded plan, rows packed into this triangle and copied out on the device), so the
 * eager fill is one call per device instead of a batch per chunk of sources. */
static void* fill_worker(void* arg) {
    fill_job* job = arg;
    pcache* c = job->c;
    double mn = INFINITY;
    int rc = shd_route_fill_triangle(job->t->eng[job->dev], c->A, c->na, job->nd, job->dev,
                                     SHD_ROUTE_DISPATCH | (c->l16 ? SHD_ROUTE_FILL_LAT16 : 0u), c->lr, &mn, NULL);
    /* ENOEDGE: a self pair without a self-loop; that entry stays NaN, i.e. not stored by
     * the batch, as the reference skips the failed target (topology.c:1488-1495,
     * 1812-1870); fill_locked resolves it below.  EUNREACH (not after the
     * strong-connectivity check at load) leaves the pair unstored */
    if (rc && rc != SHD_ROUTE_ENOEDGE && rc != SHD_ROUTE_EUNREACH) job->rc = rc;
    job->min_lat = mn;
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* counters of the pairs the last retired fill held, moved to fill c (after a late
 * attach every old pair is still a pair: the attached set only grows).  A reader that
 * still holds the retired fill may count into it after this pass has read a pair:
 * packet counts are approximate across a late attach (Shadow attaches every host before
 * the simulation starts, so this does not arise there).  The spill maps are read under
 * their locks, as a concurrent wrap may be growing one: every stripe is locked once for
 * the whole pass (a lock round trip per pair was O(na^2) of them). */
static void carry_counters(pcache* o, pcache* c) {
    for (int k = 0; k < PC_STRIPES; k++) pthread_mutex_lock(&o->pc[k].lock);
    for (int32_t i = 0; i < o->na; i++)
        for (int32_t j = i; j < o->na; j++) {
            const size_t ko = tri(o->na, i, j);
            uint64_t v = __atomic_load_n(&o->cnt[ko], __ATOMIC_RELAXED);
            const pcmap* m = &o->pc[pc_stripe((uint64_t)ko + 1)];
            if (m->cap) {
                size_t h = (((uint64_t)ko + 1) * 0x9E3779B97F4A7C15ull) & (m->cap - 1);
                while (m->s[h].key && m->s[h].key != (uint64_t)ko + 1) h = (h + 1) & (m->cap - 1);
                if (m->s[h].key) v += m->s[h].val;
            }
            if (!v) continue;
            int32_t a = c->cid[o->A[i]], b = c->cid[o->A[j]];
            if (a > b) { int32_t x = a; a = b; b = x; }
            const size_t k = tri(c->na, a, b);
            c->cnt[k] = (uint32_t)v;
            if (v >> 32) {
                pcmap* mm = &c->pc[pc_stripe((uint64_t)k + 1)];
                *pc_slot(mm, (uint64_t)k + 1) = v & ~(uint64_t)UINT32_MAX;
            }
        }
    for (int k = PC_STRIPES - 1; k >= 0; k--) pthread_mutex_unlock(&o->pc[k].lock);
}

static int fill_locked(shd_topology_t* t) {
    if (t->cache) return SHD_ROUTE_OK;
    const double t0 = now_s();
    pcache* c = calloc(1, sizeof(pcache));
    if (!c) return SHD_ROUTE_ENOMEM;
    for (int k = 0; k < PC_STRIPES; k++) pthread_mutex_init(&c->pc[k].lock, NULL);
    c->A = malloc(sizeof(int32_t) * ((size_t)t->nattached + 1));
    c->cid = malloc(sizeof(int32_t) * (size_t)t->n);
    if (!c->A || !c->cid) { pcache_free(c); return SHD_ROUTE_ENOMEM; }
    for (int32_t v = 0; v < t->n; v++) {
        c->cid[v] = -1;
        if (t->attached[v]) { c->cid[v] = c->na; c->A[c->na++] = v; }
    }
    const size_t ntri = (size_t)c->na * ((size_t)c->na + 1) / 2;
    c->l16 = t->lat16;
    size_t bytes = 2 * sizeof(double) * ntri;
    if (c->l16) {
        c->row16 = malloc(sizeof(int64_t) * ((size_t)c->na + 1));
        if (!c->row16) { pcache_free(c); return SHD_ROUTE_ENOMEM; }
        c->row16[0] = 0;
        for (int32_t i = 0; i < c->na; i++) c->row16[i + 1] = c->row16[i] + (c->na - i + 5) / 6;
        bytes = 64 * (size_t)c->row16[c->na];
    }
    /* pinned: the device copies its rows straight into the triangle at full PCIe rate; the
     * chunks are registered in the background while the rows run and the first chunks copy */
    c->lr = shd_route_host_alloc_lazy(bytes ? bytes : 16);
    c->cnt = calloc(ntri ? ntri : 1, sizeof(uint32_t));
    if (!c->lr || !c->cnt) { pcache_free(c); return SHD_ROUTE_ENOMEM; }
    int rc = SHD_ROUTE_OK;
    double mn_fill = INFINITY;
    if (c->na) {
        pthread_t th[FILL_MAX_DEV];
        fill_job jobs[FILL_MAX_DEV];
        int started[FILL_MAX_DEV];
        const int nd = t->ndev;  /* <= FILL_MAX_DEV (finish_new) */
        for (int d = 0; d < nd; d++) {
            jobs[d].t = t; jobs[d].c = c; jobs[d].dev = d; jobs[d].nd = nd; jobs[d].rc = 0;
            jobs[d].min_lat = INFINITY;
            started[d] = pthread_create(&th[d], NULL, fill_worker, &jobs[d]) == 0;
        }
        for (int d = 0; d < nd; d++) {
            if (started[d]) pthread_join(th[d], NULL);
            else fill_worker(&jobs[d]);  /* no thread: this device's rows inline */
            if (jobs[d].rc && !rc) rc = jobs[d].rc;
            if (jobs[d].min_lat < mn_fill) mn_fill = jobs[d].min_lat;
        }
    }
    if (!rc) rc = shd_route_host_wait(c->lr);
    if (rc) { pcache_free(c); return rc; }
    /* (s,s) pairs the batch could not store (no self-loop at s): the reference's next
     * (s,s) lookup misses and computes _topology_computeShortestPathToSelf
     * (topology.c:1674-1676, 1545-1653), i.e. 2*w_min and r_min^2 over s's out-edges */
    {
        int32_t nself = 0;
        int32_t* sv = malloc(sizeof(int32_t) * ((size_t)c->na + 1));
        for (int32_t i = 0; i < c->na; i++)
            if (isnan(lat_at(c, i, i))) sv[nself++] = c->A[i];
        if (nself) {
            double* sl = malloc(sizeof(double) * (size_t)nself);
            double* sr = malloc(sizeof(double) * (size_t)nself);
            rc = shd_route_self(t->eng[0], sv, nself, sl, sr);
            if (rc == SHD_ROUTE_ENOEDGE) rc = SHD_ROUTE_OK;  /* no out-edge: stays unstored */
            for (int32_t q = 0; q < nself && !rc; q++) {
                const int32_t ii = c->cid[sv[q]];
                set_at(c, ii, ii, sl[q], sr[q]);
                if (!isnan(sl[q]) && sl[q] < mn_fill) mn_fill = sl[q];
            }
            free(sl); free(sr);
        }
        free(sv);
        if (rc) { pcache_free(c); return rc; }
    }
    /* minimumPathLatency over every stored Path (topology.c:1374-1385; 0 = unset): the
     * fill's per-device minima over the pairs it wrote, and the self pairs above */
    c->min_lat = mn_fill < INFINITY ? mn_fill : 0;
    if (t->retired) carry_counters(t->retired, c);
    t->fill_seconds += now_s() - t0;
    __atomic_store_n(&t->cache, c, __ATOMIC_RELEASE);
    return SHD_ROUTE_OK;
}

uint64_t shd_topology_triangle_bytes(shd_topology_t* t) {
    const pcache* c = t ? __atomic_load_n(&t->cache, __ATOMIC_ACQUIRE) : NULL;
    if (!c) return 0;
    return c->l16 ? 64 * (uint64_t)c->row16[c->na] : 16 * ((uint64_t)c->na * ((uint64_t)c->na + 1) / 2);
}

int shd_topology_fill(shd_topology_t* t, double* elapsed_s) {
    if (!t) return SHD_ROUTE_EINVAL;
    pthread_mutex_lock(&t->lock);
    int rc = fill_locked(t);
    pthread_mutex_unlock(&t->lock);
    if (elapsed_s) *elapsed_s = t->fill_seconds;
    return rc;
}

/* the published fill, filling it first if needed (NULL on failure) */
static pcache* cache_of(shd_topology_t* t) {
    pcache* c = __atomic_load_n(&t->cache, __ATOMIC_ACQUIRE);
    if (c) return c;
    pthread_mutex_lock(&t->lock);
    const int rc = fill_locked(t);
    c = t->cache;
    pthread_mutex_unlock(&t->lock);
    return rc ? NULL : c;
}

/* _topology_getPathEntry (topology.c:1969-2051) -> index into the triangle of *cp, or -1;
 * *ip <= *jp its attached positions */
static int64_t entry_ij(shd_topology_t* t, int32_t s, int32_t d, pcache** cp, int32_t* ip, int32_t* jp) {
    if (!t || s < 0 || d < 0 || s >= t->n || d >= t->n) return -1;
    pcache* c = cache_of(t);
    if (!c) return -1;
    int32_t i = c->cid[s], j = c->cid[d];
    if (i < 0 || j < 0) return -1;  /* address not connected to the topology */
    if (i > j) { const int32_t x = i; i = j; j = x; }
    *cp = c; *ip = i; *jp = j;
    return isnan(lat_at(c, i, j)) ? -1 : (int64_t)tri(c->na, i, j);  /* never stored (topology.c:2040-2046) */
}
static int64_t entry(shd_topology_t* t, int32_t s, int32_t d, pcache** cp) {
    int32_t i, j;
    return entry_ij(t, s, d, cp, &i, &j);
}

double shd_topology_get_latency(shd_topology_t* t, int32_t s, int32_t d) {
    pcache* c;
    int32_t i, j;
    return entry_ij(t, s, d, &c, &i, &j) < 0 ? -1.0 : lat_at(c, i, j);
}

double shd_topology_get_reliability(shd_topology_t* t, int32_t s, int32_t d) {
    pcache* c;
    int32_t i, j;
    return entry_ij(t, s, d, &c, &i, &j) < 0 ? -1.0 : rel_at(c, i, j);
}

int shd_topology_is_routable(shd_topology_t* t, int32_t s, int32_t d) {
    return shd_topology_get_latency(t, s, d) > -1;  /* topology.c:2089-2092 */
}

int shd_topology_is_direct_path(shd_topology_t* t, int32_t s, int32_t d) {
    pcache* c;
    if (entry(t, s, d, &c) < 0) return -1;
    const int32_t a = s < d ? s : d, b = s < d ? d : s;  /* stored orientation: min -> max */
    return t->complete || (t->prefer_direct && adjacent(t, a, b));
}

static uint64_t* pc_slot(pcmap* m, uint64_t key) {
    if (m->len * 2 + 2 > m->cap) {
        size_t nc = m->cap ? m->cap * 2 : 4096;
        pcslot* ns = calloc(nc, sizeof(pcslot));
        for (size_t i = 0; i < m->cap; i++)
            if (m->s[i].key) {
                size_t j = (m->s[i].key * 0x9E3779B97F4A7C15ull) & (nc - 1);
                while (ns[j].key) j = (j + 1) & (nc - 1);
                ns[j] = m->s[i];
            }
        free(m->s);
        m->s = ns; m->cap = nc;
    }
    size_t j = (key * 0x9E3779B97F4A7C15ull) & (m->cap - 1);
    while (m->s[j].key && m->s[j].key != key) j = (j + 1) & (m->cap - 1);
    if (!m->s[j].key) { m->s[j].key = key; m->len++; }
    return &m->s[j].val;
}

/* read without inserting */
static uint64_t pc_get(pcache* c, uint64_t key) {
    const unsigned st = pc_stripe(key);
    uint64_t v = 0;
    pcmap* m = &c->pc[st];
    pthread_mutex_lock(&m->lock);
    if (m->cap) {
        size_t j = (key * 0x9E3779B97F4A7C15ull) & (m->cap - 1);
        while (m->s[j].key && m->s[j].key != key) j = (j + 1) & (m->cap - 1);
        if (m->s[j].key) v = m->s[j].val;
    }
    pthread_mutex_unlock(&m->lock);
    return v;
}

void shd_topology_increment_path_packet_counter(shd_topology_t* t, int32_t s, int32_t d) {
    pcache* c;
    int64_t k = entry(t, s, d, &c);
    if (k < 0) return;
    /* path_incrementPacketCount (path.c:57-60) without its data race: one relaxed
     * atomic add on the pair's own counter, no lock */
    if (__atomic_fetch_add(&c->cnt[k], 1u, __ATOMIC_RELAXED) != UINT32_MAX) return;
    const uint64_t key = (uint64_t)k + 1;
    const unsigned st = pc_stripe(key);
    pthread_mutex_lock(&c->pc[st].lock);
    *pc_slot(&c->pc[st], key) += 1ull << 32;
    pthread_mutex_unlock(&c->pc[st].lock);
}

uint64_t shd_topology_get_path_packet_count(shd_topology_t* t, int32_t s, int32_t d) {
    pcache* c;
    int64_t k = entry(t, s, d, &c);
    if (k < 0) return 0;
    return pc_get(c, (uint64_t)k + 1) + __atomic_load_n(&c->cnt[k], __ATOMIC_RELAXED);
}

double shd_topology_min_path_latency(shd_topology_t* t) {
    if (!t) return -1;
    pcache* c = cache_of(t);
    return c ? c->min_lat : -1;
}

uint64_t shd_topology_runahead_ns(shd_topology_t* t) {
    double m = shd_topology_min_path_latency(t);
    uint64_t ns = m > 0 ? ((uint64_t)m) * 1000000ull : 0;  /* master.c:153 */
    return ns > 0 ? ns : 10ull * 1000000ull;              /* master.c:138 */
}

int shd_topology_dump_paths(shd_topology_t* t, FILE* out) {
    if (!t || !out) return SHD_ROUTE_EINVAL;
    pcache* c = cache_of(t);
    if (!c) return SHD_ROUTE_EDEVICE;
    for (int32_t i = 0; i < c->na; i++)
        for (int32_t j = i; j < c->na; j++) {
            const size_t k = tri(c->na, i, j);
            const int32_t a = c->A[i], b = c->A[j];
            const char* ia = t->gml.vertex_ids ? t->gml.vertex_ids[a] : NULL;
            const char* ib = t->gml.vertex_ids ? t->gml.vertex_ids[b] : NULL;
            char na_[32], nb_[32];
            if (!ia) { snprintf(na_, sizeof na_, "%d", a); ia = na_; }
            if (!ib) { snprintf(nb_, sizeof nb_, "%d", b); ib = nb_; }
            const uint64_t pc = pc_get(c, (uint64_t)k + 1) + __atomic_load_n(&c->cnt[k], __ATOMIC_RELAXED);
            /* path_toString (path.c:62-74) inside _topology_logAllCachedPathsHelper2 */
            fprintf(out, "Found path %s%s%s in cache: SourceIndex=%d DestinationIndex=%d Latency=%f "
                         "Reliability=%f PacketCount=%llu isDirect=%s\n",
                    ia, t->directed ? "->" : "<->", ib, a, b, lat_at(c, i, j), rel_at(c, i, j), (unsigned long long)pc,
                    (t->complete || (t->prefer_direct && adjacent(t, a, b))) ? "True" : "False");
        }
    return SHD_ROUTE_OK;
}
