/*
 * oracle.c -- CPU restatement of Shadow 1.14 topology path semantics + igraph 0.7.1
 * Dijkstra.  TEST INFRASTRUCTURE ONLY (see oracle.h for scope and parity status).
 *
 * Every function cites the reference location it restates.  igraph 0.7.1 pieces
 * (indexed edge list, incident order, 2-way heap, Dijkstra) follow the library's
 * published 0.7.1 algorithm as summarised in SURVEY.md Appendix B.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

struct orc_graph {
    int32_t n, m, directed;
    int32_t* from;   /* igraph storage order: undirected edges keep from = max(a,b) */
    int32_t* to;
    double* lat;     /* edge 'latency' attribute, ms */
    double* rel;     /* 1.0 - packetloss (topology.c:437, 1.0f promoted to double) */
    double* vf;      /* 1.0 - vertex packetloss, NaN = attribute absent (topology.c:330-347) */
    int32_t* oi;     /* edge ids ordered by (from, to, id)  -- igraph 'oi' */
    int32_t* ii;     /* edge ids ordered by (to, from, id)  -- igraph 'ii' */
    int32_t* os;     /* n+1 offsets into oi by from */
    int32_t* is;     /* n+1 offsets into ii by to */
    /* plain CSR for the fast (non-igraph-order) baselines: arcs out of each vertex */
    int32_t* crow;   /* n+1 */
    int32_t* ccol;
    int32_t* ceid;
};

/* ------------------------------------------------------------------------- */
/* igraph 0.7.1 indexed edge list (type_indexededgelist.c: igraph_add_edges,   */
/* igraph_vector_order): undirected edges are stored with from >= to, and oi/ii */
/* are stable radix orders, i.e. ties by ascending edge id.                    */

static const orc_graph* g_sort_ctx;
static int cmp_oi(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    const orc_graph* g = g_sort_ctx;
    if (g->from[x] != g->from[y]) return g->from[x] < g->from[y] ? -1 : 1;
    if (g->to[x] != g->to[y]) return g->to[x] < g->to[y] ? -1 : 1;
    return x < y ? -1 : (x > y);
}
static int cmp_ii(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    const orc_graph* g = g_sort_ctx;
    if (g->to[x] != g->to[y]) return g->to[x] < g->to[y] ? -1 : 1;
    if (g->from[x] != g->from[y]) return g->from[x] < g->from[y] ? -1 : 1;
    return x < y ? -1 : (x > y);
}

orc_graph* orc_graph_new(int32_t n, int32_t m, const int32_t* from, const int32_t* to,
                         const double* latency, const double* packetloss,
                         const double* vloss, int32_t directed) {
    if (n <= 0 || m < 0) return NULL;
    orc_graph* g = (orc_graph*)calloc(1, sizeof(*g));
    g->n = n; g->m = m; g->directed = directed ? 1 : 0;
    g->from = malloc(sizeof(int32_t) * (m ? m : 1));
    g->to = malloc(sizeof(int32_t) * (m ? m : 1));
    g->lat = malloc(sizeof(double) * (m ? m : 1));
    g->rel = malloc(sizeof(double) * (m ? m : 1));
    g->vf = malloc(sizeof(double) * n);
    for (int32_t e = 0; e < m; e++) {
        int32_t a = from[e], b = to[e];
        if (a < 0 || a >= n || b < 0 || b >= n) { orc_graph_free(g); return NULL; }
        if (!g->directed && a < b) { int32_t t = a; a = b; b = t; }
        g->from[e] = a; g->to[e] = b;
        g->lat[e] = latency[e];
        g->rel[e] = (1.0f - packetloss[e]);
    }
    for (int32_t v = 0; v < n; v++) {
        double p = vloss ? vloss[v] : NAN;
        g->vf[v] = isnan(p) ? NAN : (1.0f - p);
    }
    g->oi = malloc(sizeof(int32_t) * (m ? m : 1));
    g->ii = malloc(sizeof(int32_t) * (m ? m : 1));
    for (int32_t e = 0; e < m; e++) g->oi[e] = g->ii[e] = e;
    g_sort_ctx = g;
    qsort(g->oi, m, sizeof(int32_t), cmp_oi);
    qsort(g->ii, m, sizeof(int32_t), cmp_ii);
    g->os = calloc(n + 1, sizeof(int32_t));
    g->is = calloc(n + 1, sizeof(int32_t));
    for (int32_t e = 0; e < m; e++) { g->os[g->from[e] + 1]++; g->is[g->to[e] + 1]++; }
    for (int32_t v = 0; v < n; v++) { g->os[v + 1] += g->os[v]; g->is[v + 1] += g->is[v]; }
    /* CSR of OUT arcs (undirected: both directions), self-loops dropped */
    g->crow = calloc(n + 1, sizeof(int32_t));
    for (int32_t e = 0; e < m; e++) {
        if (g->from[e] == g->to[e]) continue;
        if (g->directed) g->crow[from[e] + 1]++;
        else { g->crow[g->from[e] + 1]++; g->crow[g->to[e] + 1]++; }
    }
    for (int32_t v = 0; v < n; v++) g->crow[v + 1] += g->crow[v];
    int32_t nnz = g->crow[n];
    g->ccol = malloc(sizeof(int32_t) * (nnz ? nnz : 1));
    g->ceid = malloc(sizeof(int32_t) * (nnz ? nnz : 1));
    int32_t* fill = malloc(sizeof(int32_t) * n);
    memcpy(fill, g->crow, sizeof(int32_t) * n);
    for (int32_t e = 0; e < m; e++) {
        if (g->from[e] == g->to[e]) continue;
        if (g->directed) {
            int32_t a = from[e], b = to[e];
            g->ccol[fill[a]] = b; g->ceid[fill[a]++] = e;
        } else {
            int32_t a = g->from[e], b = g->to[e];
            g->ccol[fill[a]] = b; g->ceid[fill[a]++] = e;
            g->ccol[fill[b]] = a; g->ceid[fill[b]++] = e;
        }
    }
    free(fill);
    return g;
}

void orc_graph_free(orc_graph* g) {
    if (!g) return;
    free(g->from); free(g->to); free(g->lat); free(g->rel); free(g->vf);
    free(g->oi); free(g->ii); free(g->os); free(g->is);
    free(g->crow); free(g->ccol); free(g->ceid);
    free(g);
}

/* IGRAPH_OTHER(graph, edge, v) */
static inline int32_t other(const orc_graph* g, int32_t e, int32_t v) {
    return g->to[e] == v ? g->from[e] : g->to[e];
}

/* igraph_incident(graph, eids, v, mode): OUT part (oi by from==v) then, for
 * undirected graphs (mode forced to ALL) the IN part (ii by to==v). A self-loop
 * of an undirected graph therefore appears twice. Returns count, fills buf. */
static int32_t incident(const orc_graph* g, int32_t v, int32_t* buf) {
    int32_t k = 0;
    for (int32_t i = g->os[v]; i < g->os[v + 1]; i++) buf[k++] = g->oi[i];
    if (!g->directed)
        for (int32_t i = g->is[v]; i < g->is[v + 1]; i++) buf[k++] = g->ii[i];
    return k;
}
static int32_t incident_count(const orc_graph* g, int32_t v) {
    int32_t k = g->os[v + 1] - g->os[v];
    if (!g->directed) k += g->is[v + 1] - g->is[v];
    return k;
}

/* igraph 0.7.1 BINSEARCH over one adjacency run. */
static int64_t binsearch(const int32_t* idx, const int32_t* keyof, int32_t lo, int32_t hi, int32_t key) {
    while (lo < hi) {
        int32_t mid = lo + (hi - lo) / 2;
        int32_t e = idx[mid];
        if (keyof[e] < key) lo = mid + 1;
        else if (keyof[e] > key) hi = mid;
        else return e;
    }
    return -1;
}
/* FIND_DIRECTED_EDGE: search the shorter of from's out-run and to's in-run. */
static int64_t find_directed(const orc_graph* g, int32_t xfrom, int32_t xto) {
    int32_t s1 = g->os[xfrom], e1 = g->os[xfrom + 1];
    int32_t s2 = g->is[xto], e2 = g->is[xto + 1];
    if (e1 - s1 < e2 - s2) return binsearch(g->oi, g->to, s1, e1, xto);
    return binsearch(g->ii, g->from, s2, e2, xfrom);
}
/* topology.c:402-444 -> igraph_get_eid(graph, &eid, from, to, directedness, error=FALSE).
 * Undirected graphs use FIND_UNDIRECTED_EDGE (from=max, to=min). */
int64_t orc_get_eid(const orc_graph* g, int32_t from, int32_t to) {
    if (from < 0 || to < 0 || from >= g->n || to >= g->n) return -1;
    if (g->directed) return find_directed(g, from, to);
    int32_t a = from > to ? from : to, b = from > to ? to : from;
    return find_directed(g, a, b);
}

/* topology.c:450-552 _topology_isComplete: every vertex needs >= n incident OUT
 * edges, after subtracting one for an undirected self-loop counted twice. */
int32_t orc_is_complete(const orc_graph* g) {
    for (int32_t v = 0; v < g->n; v++) {
        int64_t ecount = incident_count(g, v);
        if (!g->directed && orc_get_eid(g, v, v) >= 0) ecount -= 1;
        if (ecount < g->n) return 0;
    }
    return 1;
}

/* ------------------------------------------------------------------------- */
/* igraph 0.7.1 indheap.c: igraph_2wheap_t (max-heap with vertex index).       */
typedef struct {
    double* data;
    int32_t* index;   /* heap pos -> vertex */
    int32_t* index2;  /* vertex -> heap pos + 2, 0 = not in heap */
    int32_t size;
} wheap;

#define W_PARENT(x) ((((x) + 1) / 2) - 1)
#define W_LEFT(x) (((x) + 1) * 2 - 1)
#define W_RIGHT(x) (((x) + 1) * 2)

static void wh_switch(wheap* h, int32_t e1, int32_t e2) {
    if (e1 != e2) {
        double t = h->data[e1]; h->data[e1] = h->data[e2]; h->data[e2] = t;
        int32_t t1 = h->index[e1], t2 = h->index[e2];
        h->index2[t1] = e2 + 2;
        h->index2[t2] = e1 + 2;
        h->index[e1] = t2; h->index[e2] = t1;
    }
}
static void wh_shift_up(wheap* h, int32_t elem) {
    while (!(elem == 0 || h->data[elem] < h->data[W_PARENT(elem)])) {
        wh_switch(h, elem, W_PARENT(elem));
        elem = W_PARENT(elem);
    }
}
static void wh_sink(wheap* h, int32_t head) {
    for (;;) {
        int32_t size = h->size;
        if (W_LEFT(head) >= size) return;
        if (W_RIGHT(head) == size || h->data[W_LEFT(head)] >= h->data[W_RIGHT(head)]) {
            if (h->data[head] < h->data[W_LEFT(head)]) {
                wh_switch(h, head, W_LEFT(head));
                head = W_LEFT(head);
            } else return;
        } else {
            if (h->data[head] < h->data[W_RIGHT(head)]) {
                wh_switch(h, head, W_RIGHT(head));
                head = W_RIGHT(head);
            } else return;
        }
    }
}
static void wh_push(wheap* h, int32_t idx, double elem) {
    int32_t size = h->size++;
    h->data[size] = elem;
    h->index[size] = idx;
    h->index2[idx] = size + 2;
    wh_shift_up(h, size);
}
static double wh_delete_max(wheap* h, int32_t* idx_out) {
    double tmp = h->data[0];
    int32_t tmpidx = h->index[0];
    wh_switch(h, 0, h->size - 1);
    h->size--;
    h->index2[tmpidx] = 0;
    wh_sink(h, 0);
    *idx_out = tmpidx;
    return tmp;
}
static void wh_modify(wheap* h, int32_t idx, double elem) {
    int32_t pos = h->index2[idx] - 2;
    h->data[pos] = elem;
    wh_sink(h, pos);
    wh_shift_up(h, pos);
}

/* igraph_get_shortest_paths_dijkstra (0.7.1, structural_properties.c), mode OUT
 * (undirected -> ALL via lazy inclist).  Stops early once every target popped;
 * targets == NULL means all vertices.  parents[] holds eid+1 (0 = none). */
static void dijkstra_igraph(const orc_graph* g, int32_t from, const uint8_t* is_target_in,
                            int32_t to_reach, double* dists, int64_t* parent_eid,
                            int32_t* incbuf, wheap* Q, uint8_t* is_target) {
    int32_t n = g->n;
    for (int32_t v = 0; v < n; v++) { dists[v] = -1.0; parent_eid[v] = -1; Q->index2[v] = 0; }
    if (is_target_in) memcpy(is_target, is_target_in, n);
    else { memset(is_target, 1, n); to_reach = n; }
    Q->size = 0;
    dists[from] = 0.0;
    wh_push(Q, from, 0);
    while (Q->size > 0 && to_reach > 0) {
        int32_t minnei;
        double mindist = -wh_delete_max(Q, &minnei);
        if (is_target[minnei]) { is_target[minnei] = 0; to_reach--; }
        int32_t nlen = incident(g, minnei, incbuf);
        for (int32_t i = 0; i < nlen; i++) {
            int32_t edge = incbuf[i];
            int32_t tto = other(g, edge, minnei);
            double altdist = mindist + g->lat[edge];
            double curdist = dists[tto];
            if (curdist < 0) {
                dists[tto] = altdist;
                parent_eid[tto] = edge;
                wh_push(Q, tto, -altdist);
            } else if (altdist < curdist) {
                dists[tto] = altdist;
                parent_eid[tto] = edge;
                wh_modify(Q, tto, -altdist);
            }
        }
    }
}

/* Engine tie-break: parent(v) = argmin over tight in-edges e=(u->v), u != v, of
 * (dist[u], u, e); tight means fl(dist[u] + w_e) == dist[v] exactly. */
static void parents_minkey(const orc_graph* g, int32_t src, const double* dist, int64_t* parent_eid,
                           int32_t* incbuf) {
    for (int32_t v = 0; v < g->n; v++) {
        parent_eid[v] = -1;
        if (v == src || dist[v] < 0) continue;
        double bd = INFINITY; int32_t bu = -1; int64_t be = -1;
        int32_t k;
        if (g->directed) {
            k = 0;
            for (int32_t i = g->is[v]; i < g->is[v + 1]; i++) incbuf[k++] = g->ii[i];
        } else k = incident(g, v, incbuf);
        for (int32_t i = 0; i < k; i++) {
            int32_t e = incbuf[i];
            int32_t u = g->directed ? g->from[e] : other(g, e, v);
            if (u == v || dist[u] < 0) continue;
            if (dist[u] + g->lat[e] != dist[v]) continue;
            if (dist[u] < bd || (dist[u] == bd && (u < bu || (u == bu && e < be)))) {
                bd = dist[u]; bu = u; be = e;
            }
        }
        parent_eid[v] = be;
    }
}

typedef struct {
    int32_t* incbuf;
    wheap Q;
    uint8_t* is_target;
    uint8_t* tmask;
    double* dist;
    int64_t* peid;
    int32_t* order;
    uint8_t* cnt;
    int32_t* path;
} scratch;

static int32_t max_incident(const orc_graph* g) {
    int32_t mx = 1;
    for (int32_t v = 0; v < g->n; v++) {
        int32_t k = incident_count(g, v);
        if (k > mx) mx = k;
    }
    return mx;
}
static void scratch_init(scratch* s, const orc_graph* g) {
    int32_t n = g->n;
    s->incbuf = malloc(sizeof(int32_t) * (max_incident(g) + 1));
    s->Q.data = malloc(sizeof(double) * (n + 1));
    s->Q.index = malloc(sizeof(int32_t) * (n + 1));
    s->Q.index2 = calloc(n, sizeof(int32_t));
    s->is_target = malloc(n);
    s->tmask = malloc(n);
    s->dist = malloc(sizeof(double) * n);
    s->peid = malloc(sizeof(int64_t) * n);
    s->order = malloc(sizeof(int32_t) * n);
    s->cnt = malloc(n);
    s->path = malloc(sizeof(int32_t) * (n + 1));
}
static void scratch_free(scratch* s) {
    free(s->incbuf); free(s->Q.data); free(s->Q.index); free(s->Q.index2);
    free(s->is_target); free(s->tmask); free(s->dist); free(s->peid); free(s->order);
    free(s->cnt); free(s->path);
}

int32_t orc_dijkstra(const orc_graph* g, int32_t src, int32_t tiebreak, double* dist, int64_t* parent_eid) {
    if (src < 0 || src >= g->n) return -1;
    scratch s; scratch_init(&s, g);
    dijkstra_igraph(g, src, NULL, g->n, dist, parent_eid, s.incbuf, &s.Q, s.is_target);
    if (tiebreak == ORC_TIE_MINKEY) parents_minkey(g, src, dist, parent_eid, s.incbuf);
    scratch_free(&s);
    return 0;
}

/* shortest-path multiplicity over the tight DAG, capped at 2 (1 = unique). */
static const double* g_dist_ctx;
static int cmp_dist(const void* a, const void* b) {
    double x = g_dist_ctx[*(const int32_t*)a], y = g_dist_ctx[*(const int32_t*)b];
    if (x < y) return -1;
    if (x > y) return 1;
    return (*(const int32_t*)a > *(const int32_t*)b) - (*(const int32_t*)a < *(const int32_t*)b);
}
static void path_multiplicity(const orc_graph* g, int32_t src, const double* dist, scratch* s) {
    int32_t n = g->n, k = 0;
    for (int32_t v = 0; v < n; v++) { s->cnt[v] = 0; if (dist[v] >= 0) s->order[k++] = v; }
    g_dist_ctx = dist;
    qsort(s->order, k, sizeof(int32_t), cmp_dist);
    s->cnt[src] = 1;
    for (int32_t i = 0; i < k; i++) {
        int32_t u = s->order[i];
        if (!s->cnt[u]) continue;
        int32_t nl;
        if (g->directed) {
            nl = 0;
            for (int32_t j = g->os[u]; j < g->os[u + 1]; j++) s->incbuf[nl++] = g->oi[j];
        } else nl = incident(g, u, s->incbuf);
        for (int32_t j = 0; j < nl; j++) {
            int32_t e = s->incbuf[j];
            int32_t v = g->directed ? g->to[e] : other(g, e, u);
            if (v == u || v == src) continue;
            if (dist[u] + g->lat[e] != dist[v]) continue;
            int c = s->cnt[v] + s->cnt[u] + (dist[u] == dist[v] ? 2 : 0);
            s->cnt[v] = (uint8_t)(c > 2 ? 2 : c);
        }
    }
}

/* topology.c:1407-1523 _topology_computePathProperties over an igraph vertex path. */
static int32_t path_properties(const orc_graph* g, int32_t src, const int32_t* P, int32_t nV,
                               double* lat_out, double* rel_out) {
    double totalLatency = 0.0, totalReliability = 1.0;
    if (!isnan(g->vf[src])) totalReliability *= g->vf[src];
    int32_t target = P[nV - 1];
    if ((src != target) || (src == target && nV > 2)) {
        if (!isnan(g->vf[target])) totalReliability *= g->vf[target];
    }
    int32_t start = nV == 1 ? 0 : 1;
    int32_t fromV = src;
    for (int32_t i = start; i < nV; i++) {
        int32_t toV = P[i];
        int64_t e = orc_get_eid(g, fromV, toV);
        if (e < 0) return -1;
        totalLatency += g->lat[e];
        totalReliability *= g->rel[e];
        fromV = toV;
    }
    *lat_out = totalLatency;
    *rel_out = totalReliability;
    return 0;
}

/* igraph path reconstruction: walk parents back to the source; source -> [s]. */
static int32_t build_path(const orc_graph* g, int32_t t, const int64_t* peid, int32_t* P) {
    int32_t size = 0, act = t;
    while (peid[act] >= 0) { size++; act = other(g, (int32_t)peid[act], act); }
    P[size] = t;
    act = t;
    int32_t k = size;
    while (peid[act] >= 0) { act = other(g, (int32_t)peid[act], act); P[--k] = act; }
    return size + 1;
}

static int32_t source_row_s(const orc_graph* g, int32_t src, const int32_t* tgt, int32_t nt,
                            int32_t tiebreak, double* lat, double* rel, uint8_t* unique,
                            int32_t* hops, scratch* s) {
    int32_t n = g->n;
    memset(s->tmask, 0, n);
    int32_t to_reach = 0;
    for (int32_t j = 0; j < nt; j++) {
        if (tgt[j] < 0 || tgt[j] >= n) return -1;
        if (!s->tmask[tgt[j]]) { s->tmask[tgt[j]] = 1; to_reach++; }
    }
    dijkstra_igraph(g, src, s->tmask, to_reach, s->dist, s->peid, s->incbuf, &s->Q, s->is_target);
    if (tiebreak == ORC_TIE_MINKEY) parents_minkey(g, src, s->dist, s->peid, s->incbuf);
    if (unique) path_multiplicity(g, src, s->dist, s);
    for (int32_t j = 0; j < nt; j++) {
        int32_t t = tgt[j];
        int32_t nV = build_path(g, t, s->peid, s->path);
        double L, R;
        if (path_properties(g, src, s->path, nV, &L, &R) != 0) return -1;
        if (L == 0) L = 1; /* topology.c:1848-1852 */
        lat[j] = L; rel[j] = R;
        if (hops) hops[j] = nV == 1 ? 1 : nV - 1;
        if (unique) unique[j] = (t == src) ? 1 : (s->cnt[t] == 1);
    }
    return 0;
}

int32_t orc_source_row(const orc_graph* g, int32_t src, const int32_t* tgt, int32_t nt,
                       int32_t tiebreak, double* lat, double* rel, uint8_t* unique, int32_t* hops) {
    if (src < 0 || src >= g->n) return -1;
    scratch s; scratch_init(&s, g);
    int32_t r = source_row_s(g, src, tgt, nt, tiebreak, lat, rel, unique, hops, &s);
    scratch_free(&s);
    return r;
}

/* topology.c:1877-1927 _topology_lookupDirectPath */
int32_t orc_direct(const orc_graph* g, int32_t s, int32_t t, double* lat, double* rel) {
    double totalLatency = 0.0, totalReliability = 1.0;
    if (!isnan(g->vf[s])) totalReliability *= g->vf[s];
    if (!isnan(g->vf[t])) totalReliability *= g->vf[t];
    int64_t e = orc_get_eid(g, s, t);
    if (e < 0) return -1;
    totalLatency += g->lat[e];
    totalReliability *= g->rel[e];
    *lat = totalLatency; *rel = totalReliability;
    return 0;
}

/* topology.c:1545-1653 _topology_computeShortestPathToSelf: first minimum over
 * igraph_es_incident(v, OUT) order, used twice. */
int32_t orc_self_path(const orc_graph* g, int32_t v, double* lat, double* rel) {
    int32_t* buf = malloc(sizeof(int32_t) * (max_incident(g) + 1));
    int32_t k = incident(g, v, buf);
    double minLatency = 0.0, relMin = 0.0;
    for (int32_t i = 0; i < k; i++) {
        int32_t e = buf[i];
        double w = g->lat[e];
        if (minLatency == 0 || w < minLatency) { minLatency = w; relMin = g->rel[e]; }
    }
    free(buf);
    if (k == 0) return -1;
    *lat = 2.0f * minLatency;
    *rel = relMin * relMin;
    return 0;
}

/* Eager cache: ascending sources, first-writer-wins over both
 * directions (topology.c:1307-1336), direct dispatch (topology.c:2019-2031),
 * min latency tracking (topology.c:1374-1385). */
int32_t orc_eager_table(const orc_graph* g, const int32_t* A, int32_t na, int32_t prefer_direct,
                        int32_t tiebreak, double* lat, double* rel, uint8_t* is_direct,
                        uint8_t* unique, double* min_latency) {
    int32_t complete = orc_is_complete(g);
    double minLat = 0;
    double* rl = malloc(sizeof(double) * na);
    double* rr = malloc(sizeof(double) * na);
    uint8_t* ru = malloc(na);
    scratch s; scratch_init(&s, g);
    int32_t ret = 0;
    for (int32_t i = 0; i < na && !ret; i++) {
        int32_t src = A[i];
        if (!complete) {
            if (source_row_s(g, src, A, na, tiebreak, rl, rr, ru, NULL, &s) != 0) { ret = -1; break; }
        }
        for (int32_t j = i; j < na; j++) {
            int32_t t = A[j];
            double L, R; uint8_t d, u;
            if (complete || (prefer_direct && orc_get_eid(g, src, t) >= 0)) {
                if (orc_direct(g, src, t, &L, &R) != 0) { ret = -1; break; }
                d = 1; u = 1;
            } else { L = rl[j]; R = rr[j]; d = 0; u = ru[j]; }
            lat[(int64_t)i * na + j] = lat[(int64_t)j * na + i] = L;
            rel[(int64_t)i * na + j] = rel[(int64_t)j * na + i] = R;
            if (is_direct) is_direct[(int64_t)i * na + j] = is_direct[(int64_t)j * na + i] = d;
            if (unique) unique[(int64_t)i * na + j] = unique[(int64_t)j * na + i] = u;
            if (minLat == 0 || L < minLat) minLat = L;
        }
    }
    scratch_free(&s);
    free(rl); free(rr); free(ru);
    if (min_latency) *min_latency = minLat;
    return ret;
}

uint64_t orc_runahead_ns(double minPathLatency) {
    /* master.c:153 truncates to whole ms; master.c:138 defaults to 10 ms when 0 */
    uint64_t ns = ((uint64_t)minPathLatency) * 1000000ull;
    return ns > 0 ? ns : 10ull * 1000000ull;
}

/* ------------------------------------------------------------------------- */
/* CPU baselines                                                               */
static double now_s(void) {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

double orc_bench_faithful(const orc_graph* g, const int32_t* src, int32_t ns,
                          const int32_t* tgt, int32_t nt, double* checksum) {
    scratch s; scratch_init(&s, g);
    int32_t n = g->n;
    char** ids = malloc(sizeof(char*) * n);
    for (int32_t v = 0; v < n; v++) { ids[v] = malloc(24); snprintf(ids[v], 24, "poi-%d", v); }
    size_t cap = 1 << 16;
    char* pathbuf = malloc(cap);
    char* logbuf = malloc(cap + 256);
    double sum = 0;
    double t0 = now_s();
    for (int32_t i = 0; i < ns; i++) {
        int32_t sv = src[i];
        memset(s.tmask, 0, n);
        int32_t to_reach = 0;
        for (int32_t j = 0; j < nt; j++) if (!s.tmask[tgt[j]]) { s.tmask[tgt[j]] = 1; to_reach++; }
        dijkstra_igraph(g, sv, s.tmask, to_reach, s.dist, s.peid, s.incbuf, &s.Q, s.is_target);
        for (int32_t j = 0; j < nt; j++) {
            int32_t nV = build_path(g, tgt[j], s.peid, s.path);
            /* path walk with per-hop get_eid and formatting, topology.c:1449,1477-1508 */
            double L = 0.0, R = 1.0;
            if (!isnan(g->vf[sv])) R *= g->vf[sv];
            int32_t target = s.path[nV - 1];
            if (sv != target && !isnan(g->vf[target])) R *= g->vf[target];
            size_t off = (size_t)snprintf(pathbuf, cap, "%s", ids[sv]);
            int32_t fromV = sv;
            for (int32_t k = nV == 1 ? 0 : 1; k < nV; k++) {
                int32_t toV = s.path[k];
                int64_t e = orc_get_eid(g, fromV, toV);
                if (e < 0) break;
                L += g->lat[e]; R *= g->rel[e];
                if (off + 96 < cap)
                    off += (size_t)snprintf(pathbuf + off, cap - off, "%s[%f,%f]-->%s",
                                            g->directed ? "--" : "<--", g->lat[e], 1.0f - g->rel[e], ids[toV]);
                fromV = toV;
            }
            /* per-target log string, topology.c:1829-1834 */
            snprintf(logbuf, cap + 256, "shortest path %s%s%s (%i%s%i) is %f ms with %f loss, path: %s",
                     ids[sv], g->directed ? "-->" : "<-->", ids[target], sv,
                     g->directed ? "-->" : "<-->", target, L, 1 - R, pathbuf);
            sum += L + R + (double)(unsigned char)logbuf[0] * 0.0;
        }
    }
    double dt = now_s() - t0;
    for (int32_t v = 0; v < n; v++) free(ids[v]);
    free(ids); free(pathbuf); free(logbuf);
    scratch_free(&s);
    if (checksum) *checksum = sum;
    return dt;
}

/* Fast restatement: lazy binary heap Dijkstra over CSR; rel propagated in settle
 * order (parents settle first), vertex factors as in topology.c:1443-1462. */
typedef struct { double d; int32_t v; } hitem;
static void hpush(hitem* h, int32_t* sz, double d, int32_t v) {
    int32_t i = (*sz)++;
    while (i > 0) {
        int32_t p = (i - 1) >> 1;
        if (h[p].d < d || (h[p].d == d && h[p].v <= v)) break;
        h[i] = h[p]; i = p;
    }
    h[i].d = d; h[i].v = v;
}
static hitem hpop(hitem* h, int32_t* sz) {
    hitem top = h[0], last = h[--(*sz)];
    int32_t i = 0, n = *sz;
    for (;;) {
        int32_t c = 2 * i + 1;
        if (c >= n) break;
        if (c + 1 < n && (h[c + 1].d < h[c].d || (h[c + 1].d == h[c].d && h[c + 1].v < h[c].v))) c++;
        if (last.d < h[c].d || (last.d == h[c].d && last.v <= h[c].v)) break;
        h[i] = h[c]; i = c;
    }
    h[i] = last;
    return top;
}

double orc_bench_parallel(const orc_graph* g, const int32_t* src, int32_t ns,
                          const int32_t* tgt, int32_t nt, int32_t threads,
                          double* checksum, int32_t* threads_used) {
    int32_t n = g->n;
    int32_t nnz = g->crow[n];
    int32_t used = 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    double sum = 0;
    double t0 = now_s();
#pragma omp parallel reduction(+ : sum)
    {
#ifdef _OPENMP
#pragma omp single
        used = omp_get_num_threads();
#endif
        double* dist = malloc(sizeof(double) * n);
        int32_t* par = malloc(sizeof(int32_t) * n);
        int32_t* st = malloc(sizeof(int32_t) * (n + 1));
        uint8_t* done = malloc(n);
        hitem* h = malloc(sizeof(hitem) * (nnz + n + 1));
#pragma omp for schedule(dynamic, 4)
        for (int32_t i = 0; i < ns; i++) {
            int32_t sv = src[i];
            for (int32_t v = 0; v < n; v++) { dist[v] = INFINITY; done[v] = 0; par[v] = -1; }
            int32_t sz = 0;
            dist[sv] = 0.0;
            hpush(h, &sz, 0.0, sv);
            while (sz) {
                hitem it = hpop(h, &sz);
                int32_t u = it.v;
                if (done[u]) continue;
                done[u] = 1;
                for (int32_t a = g->crow[u]; a < g->crow[u + 1]; a++) {
                    int32_t v = g->ccol[a];
                    double nd = it.d + g->lat[g->ceid[a]];
                    if (nd < dist[v]) { dist[v] = nd; par[v] = a; hpush(h, &sz, nd, v); }
                }
            }
            /* rel along settle order: recompute with explicit parent vertex */
            for (int32_t j = 0; j < nt; j++) {
                int32_t t = tgt[j];
                double L, R;
                if (t == sv) {
                    int64_t e = orc_get_eid(g, sv, sv);
                    L = e >= 0 ? 0.0 + g->lat[e] : -1;
                    R = (isnan(g->vf[sv]) ? 1.0 : g->vf[sv]) * (e >= 0 ? g->rel[e] : 0);
                } else {
                    /* walk to the source, then multiply in forward (path) order */
                    double prod;
                    int32_t v = t, hops = 0;
                    while (v != sv && hops <= n) { hops++; int32_t a = par[v]; int32_t e = g->ceid[a];
                        v = g->directed ? g->from[e] : other(g, e, v); }
                    int32_t stackn = hops, k = 0;
                    v = t;
                    while (v != sv && k < stackn) { int32_t e = g->ceid[par[v]]; st[k++] = e;
                        v = g->directed ? g->from[e] : other(g, e, v); }
                    double c = 1.0;
                    if (!isnan(g->vf[sv])) c *= g->vf[sv];
                    if (!isnan(g->vf[t])) c *= g->vf[t];
                    prod = c;
                    for (int32_t q = k - 1; q >= 0; q--) prod *= g->rel[st[q]];
                    L = dist[t]; R = prod;
                }
                sum += L + R;
            }
        }
        free(dist); free(par); free(st); free(done); free(h);
    }
    double dt = now_s() - t0;
    if (checksum) *checksum = sum;
    if (threads_used) *threads_used = used;
    return dt;
}

/* C5 CPU baseline: the reference's fill of a complete graph, every
 * pair by _topology_lookupDirectPath (topology.c:1877-1927: get_eid + factor products),
 * rows spread over `threads` OpenMP threads, each row written to a per-thread buffer
 * as the cache store would. */
double orc_bench_direct(const orc_graph* g, const int32_t* A, int32_t na, int32_t threads,
                        double* checksum, int32_t* threads_used) {
    int32_t used = 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    double sum = 0;
    double t0 = now_s();
#pragma omp parallel reduction(+ : sum)
    {
#ifdef _OPENMP
#pragma omp single
        used = omp_get_num_threads();
#endif
        double* row = malloc(sizeof(double) * 2 * (size_t)na);
#pragma omp for schedule(dynamic, 4)
        for (int32_t i = 0; i < na; i++) {
            for (int32_t j = 0; j < na; j++) {
                double L = -1, R = 0;
                orc_direct(g, A[i], A[j], &L, &R);
                row[2 * j] = L; row[2 * j + 1] = R;
            }
            sum += row[2 * (i % na)] + row[2 * (na - 1) + 1];
        }
        free(row);
    }
    double dt = now_s() - t0;
    if (checksum) *checksum = sum;
    if (threads_used) *threads_used = used;
    return dt;
}

/* C5 CPU baseline for K4: `nk` k-phases (k0 .. k0+nk-1) of f64 Floyd-Warshall over the
 * n x n matrix d, rows of each phase spread over `threads` OpenMP threads (the caller
 * extrapolates x n / nk to the whole table). */
double orc_bench_fw_phases(int32_t n, double* d, int32_t k0, int32_t nk, int32_t threads,
                           int32_t* threads_used) {
    int32_t used = 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    double t0 = now_s();
    for (int32_t k = k0; k < k0 + nk && k < n; k++) {
#pragma omp parallel
        {
#ifdef _OPENMP
#pragma omp single
            used = omp_get_num_threads();
#endif
            const double* dk = d + (int64_t)k * n;
#pragma omp for schedule(static)
            for (int32_t i = 0; i < n; i++) {
                if (i == k) continue;
                double* di = d + (int64_t)i * n;
                double dik = di[k];
                if (isinf(dik)) continue;
                for (int32_t j = 0; j < n; j++) {
                    double c = dik + dk[j];
                    di[j] = c < di[j] ? c : di[j];
                }
            }
        }
    }
    double dt = now_s() - t0;
    if (threads_used) *threads_used = used;
    return dt;
}

void orc_floyd_warshall(int32_t n, double* d) {
    for (int32_t k = 0; k < n; k++)
        for (int32_t i = 0; i < n; i++) {
            double dik = d[(int64_t)i * n + k];
            if (isinf(dik)) continue;
            for (int32_t j = 0; j < n; j++) {
                double c = dik + d[(int64_t)k * n + j];
                if (c < d[(int64_t)i * n + j]) d[(int64_t)i * n + j] = c;
            }
        }
}
