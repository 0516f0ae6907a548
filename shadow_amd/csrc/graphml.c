/*
 * graphml.c -- graphml -> igraph-numbered topology arrays + Shadow's validation.
 *
 * Replaces igraph_read_graph_graphml as used by _topology_loadGraph (topology.c:371-399)
 * for the attributes Shadow reads, and _topology_checkGraphAttributes /
 * _topology_checkGraphVerticesHelperHook / _topology_checkGraphEdgesHelperHook
 * (topology.c:565-722, 811-978, 1041-1124).  Streaming libxml2 reader (the library
 * igraph itself parses graphml with), so .xz/.gz inputs work as they do for Shadow.
 *   - vertices and edges are numbered in document order; an edge endpoint that names
 *     an undeclared node adds that vertex (igraph's id trie);
 *   - numeric attributes missing on an element are NaN (or the <key>'s <default>);
 *   - numeric = attr.type int|long|float|double, string = string (igraph's mapping).
 * Deviation: the reference overwrites isSuccess per attribute check
 * (topology.c:636-700), so only the last type check counts; here any wrong type fails.
 */
#define _GNU_SOURCE
#include <libxml/xmlreader.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "../../include/shd_topology.h"

enum { K_NODE = 1, K_EDGE = 2, K_GRAPH = 4 };
enum { T_NUM = 1, T_STR = 2, T_BOOL = 3 };

typedef struct {
    char* id;
    int for_mask;
    char* name;
    int type;
    char* defval;
} gkey;

typedef struct {
    char** keys;
    int32_t* vals;
    size_t cap, len;
} idmap;

static uint64_t fnv(const char* s) {
    uint64_t h = 1469598103934665603ull;
    for (; *s; s++) h = (h ^ (unsigned char)*s) * 1099511628211ull;
    return h;
}
static int32_t idmap_get(idmap* m, const char* k, int32_t insert_val, int* inserted) {
    if (m->len * 2 + 2 > m->cap) {
        size_t nc = m->cap ? m->cap * 2 : 1024;
        char** nk = calloc(nc, sizeof(char*));
        int32_t* nv = calloc(nc, sizeof(int32_t));
        for (size_t i = 0; i < m->cap; i++)
            if (m->keys[i]) {
                size_t j = fnv(m->keys[i]) & (nc - 1);
                while (nk[j]) j = (j + 1) & (nc - 1);
                nk[j] = m->keys[i];
                nv[j] = m->vals[i];
            }
        free(m->keys); free(m->vals);
        m->keys = nk; m->vals = nv; m->cap = nc;
    }
    size_t j = fnv(k) & (m->cap - 1);
    while (m->keys[j]) {
        if (!strcmp(m->keys[j], k)) { *inserted = 0; return m->vals[j]; }
        j = (j + 1) & (m->cap - 1);
    }
    m->keys[j] = strdup(k);
    m->vals[j] = insert_val;
    m->len++;
    *inserted = 1;
    return insert_val;
}
static void idmap_free(idmap* m) {
    for (size_t i = 0; i < m->cap; i++) free(m->keys[i]);
    free(m->keys); free(m->vals);
}

typedef struct {
    double* a;
    size_t len, cap;
} dvec;
static void dpush(dvec* v, double x) {
    if (v->len == v->cap) { v->cap = v->cap ? 2 * v->cap : 1024; v->a = realloc(v->a, v->cap * sizeof(double)); }
    v->a[v->len++] = x;
}
typedef struct {
    int32_t* a;
    size_t len, cap;
} ivec;
static void ipush(ivec* v, int32_t x) {
    if (v->len == v->cap) { v->cap = v->cap ? 2 * v->cap : 1024; v->a = realloc(v->a, v->cap * sizeof(int32_t)); }
    v->a[v->len++] = x;
}

typedef struct {
    char** a;
    size_t len, cap;
} svec;
static void spush(svec* v, char* x) {
    if (v->len == v->cap) { v->cap = v->cap ? 2 * v->cap : 1024; v->a = realloc(v->a, v->cap * sizeof(char*)); }
    v->a[v->len++] = x;
}
/* string vertex attributes read at attach time (topology.c:2094-2216), by SHD_VATTR_* */
static const char* const kVstrName[SHD_VATTR_N] = {"ip", "citycode", "countrycode", "geocode", "type"};
static int vstr_slot(const char* name) {
    for (int a = 0; a < SHD_VATTR_N; a++) if (!strcmp(name, kVstrName[a])) return a;
    return -1;
}

static double parse_num(const char* s) {
    if (!s) return NAN;
    while (*s == ' ' || *s == '\t' || *s == '\n' || *s == '\r') s++;
    if (!*s) return NAN;
    char* end;
    double x = strtod(s, &end);
    return end == s ? NAN : x;
}

static void seterr(char* buf, size_t len, const char* fmt, ...) {
    if (!buf || !len) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, len, fmt, ap);
    va_end(ap);
}

/* vertex attribute slots Shadow validates */
enum { VA_BWDOWN, VA_BWUP, VA_LOSS, VA_ASN, VA_N };
enum { EA_LAT, EA_LOSS, EA_JITTER, EA_N };

static int type_of(const char* t) {
    if (!t) return T_STR;
    if (!strcmp(t, "int") || !strcmp(t, "long") || !strcmp(t, "float") || !strcmp(t, "double")) return T_NUM;
    if (!strcmp(t, "boolean")) return T_BOOL;
    return T_STR;
}

int shd_graphml_load(const char* path, shd_graphml_t* out, char* errbuf, size_t errlen) {
    if (!path || !out) return SHD_ROUTE_EINVAL;
    memset(out, 0, sizeof(*out));
    xmlTextReaderPtr rd = xmlReaderForFile(path, NULL, XML_PARSE_HUGE | XML_PARSE_NONET);
    if (!rd) { seterr(errbuf, errlen, "cannot open graphml '%s'", path); return SHD_ROUTE_EINVAL; }

    gkey* keys = NULL;
    int nkeys = 0, capk = 0;
    idmap ids = {0};
    char** vid = NULL;
    size_t vcap = 0;
    dvec va[VA_N] = {{0}};
    svec vs[SHD_VATTR_N] = {{0}};
    ivec esrc = {0}, edst = {0};
    dvec ea[EA_N] = {{0}};
    int directed = 1; /* graphml default edgedefault is "directed" */
    char* prefer = NULL;
    int32_t n = 0;
    int cur_kind = 0; /* K_NODE / K_EDGE / K_GRAPH while inside one */
    int64_t cur = -1;
    int in_key = -1;
    int rc = SHD_ROUTE_OK, ret;

    while ((ret = xmlTextReaderRead(rd)) == 1) {
        int type = xmlTextReaderNodeType(rd);
        const char* nm = (const char*)xmlTextReaderConstLocalName(rd);
        if (type == XML_READER_TYPE_ELEMENT) {
            if (!strcmp(nm, "key")) {
                if (nkeys == capk) { capk = capk ? 2 * capk : 32; keys = realloc(keys, capk * sizeof(gkey)); }
                gkey* k = &keys[nkeys];
                memset(k, 0, sizeof(*k));
                char* s;
                k->id = (char*)xmlTextReaderGetAttribute(rd, BAD_CAST "id");
                s = (char*)xmlTextReaderGetAttribute(rd, BAD_CAST "for");
                k->for_mask = !s || !strcmp(s, "all") ? (K_NODE | K_EDGE | K_GRAPH)
                            : !strcmp(s, "node") ? K_NODE : !strcmp(s, "edge") ? K_EDGE
                            : !strcmp(s, "graph") ? K_GRAPH : 0;
                xmlFree(s);
                k->name = (char*)xmlTextReaderGetAttribute(rd, BAD_CAST "attr.name");
                s = (char*)xmlTextReaderGetAttribute(rd, BAD_CAST "attr.type");
                k->type = type_of(s);
                xmlFree(s);
                in_key = nkeys++;
                if (xmlTextReaderIsEmptyElement(rd)) in_key = -1;
            } else if (!strcmp(nm, "default") && in_key >= 0) {
                keys[in_key].defval = (char*)xmlTextReaderReadString(rd);
            } else if (!strcmp(nm, "graph")) {
                char* s = (char*)xmlTextReaderGetAttribute(rd, BAD_CAST "edgedefault");
                directed = !(s && !strcmp(s, "undirected"));
                xmlFree(s);
                cur_kind = K_GRAPH;
                cur = 0;
            } else if (!strcmp(nm, "node") || !strcmp(nm, "edge")) {
                const int isnode = nm[0] == 'n';
                if (isnode) {
                    char* id = (char*)xmlTextReaderGetAttribute(rd, BAD_CAST "id");
                    if (!id) { seterr(errbuf, errlen, "node without id"); rc = SHD_ROUTE_EINVAL; break; }
                    int ins;
                    int32_t v = idmap_get(&ids, id, n, &ins);
                    if (ins) {
                        if ((size_t)n == vcap) { vcap = vcap ? 2 * vcap : 1024; vid = realloc(vid, vcap * sizeof(char*)); }
                        vid[n] = strdup(id);
                        for (int a = 0; a < VA_N; a++) dpush(&va[a], NAN);
                        for (int a = 0; a < SHD_VATTR_N; a++) spush(&vs[a], NULL);
                        n++;
                    }
                    xmlFree(id);
                    cur = v;
                    cur_kind = K_NODE;
                } else {
                    int32_t ends[2];
                    const char* an[2] = {"source", "target"};
                    for (int q = 0; q < 2; q++) {
                        char* id = (char*)xmlTextReaderGetAttribute(rd, BAD_CAST an[q]);
                        if (!id) { seterr(errbuf, errlen, "edge without %s", an[q]); rc = SHD_ROUTE_EINVAL; break; }
                        int ins;
                        ends[q] = idmap_get(&ids, id, n, &ins);
                        if (ins) {
                            if ((size_t)n == vcap) { vcap = vcap ? 2 * vcap : 1024; vid = realloc(vid, vcap * sizeof(char*)); }
                            vid[n] = strdup(id);
                            for (int a = 0; a < VA_N; a++) dpush(&va[a], NAN);
                            for (int a = 0; a < SHD_VATTR_N; a++) spush(&vs[a], NULL);
                            n++;
                        }
                        xmlFree(id);
                    }
                    if (rc) break;
                    ipush(&esrc, ends[0]);
                    ipush(&edst, ends[1]);
                    for (int a = 0; a < EA_N; a++) dpush(&ea[a], NAN);
                    cur = (int64_t)esrc.len - 1;
                    cur_kind = K_EDGE;
                }
                if (xmlTextReaderIsEmptyElement(rd)) cur_kind = K_GRAPH;
            } else if (!strcmp(nm, "data") && cur_kind) {
                char* key = (char*)xmlTextReaderGetAttribute(rd, BAD_CAST "key");
                gkey* k = NULL;
                for (int i = 0; i < nkeys && key; i++)
                    if (keys[i].id && !strcmp(keys[i].id, key)) { k = &keys[i]; break; }
                xmlFree(key);
                char* text = (char*)xmlTextReaderReadString(rd);
                if (k && k->name && (k->for_mask & cur_kind)) {
                    if (cur_kind == K_NODE && k->type == T_NUM) {
                        double x = parse_num(text);
                        if (!strcmp(k->name, "bandwidthdown")) va[VA_BWDOWN].a[cur] = x;
                        else if (!strcmp(k->name, "bandwidthup")) va[VA_BWUP].a[cur] = x;
                        else if (!strcmp(k->name, "packetloss")) va[VA_LOSS].a[cur] = x;
                        else if (!strcmp(k->name, "asn")) va[VA_ASN].a[cur] = x;
                    } else if (cur_kind == K_NODE && k->type == T_STR && vstr_slot(k->name) >= 0) {
                        char** slot = &vs[vstr_slot(k->name)].a[cur];
                        free(*slot);
                        *slot = strdup(text ? text : "");
                    } else if (cur_kind == K_EDGE && k->type == T_NUM) {
                        double x = parse_num(text);
                        if (!strcmp(k->name, "latency")) ea[EA_LAT].a[cur] = x;
                        else if (!strcmp(k->name, "packetloss")) ea[EA_LOSS].a[cur] = x;
                        else if (!strcmp(k->name, "jitter")) ea[EA_JITTER].a[cur] = x;
                    } else if (cur_kind == K_GRAPH && !strcmp(k->name, "preferdirectpaths")) {
                        free(prefer);
                        prefer = text ? strdup(text) : NULL;
                    }
                }
                xmlFree(text);
            }
        } else if (type == XML_READER_TYPE_END_ELEMENT) {
            if (!strcmp(nm, "key")) in_key = -1;
            else if (!strcmp(nm, "node") || !strcmp(nm, "edge")) cur_kind = K_GRAPH;
            else if (!strcmp(nm, "graph")) cur_kind = 0;
        }
    }
    if (ret < 0 && !rc) { seterr(errbuf, errlen, "XML parse error in '%s'", path); rc = SHD_ROUTE_EINVAL; }
    xmlFreeTextReader(rd);

    /* key defaults apply to elements lacking a <data> (igraph); a declared string key
     * without a default leaves "" (igraph), which topology.c treats as absent */
    int has_vs[SHD_VATTR_N] = {0};
    for (int i = 0; i < nkeys && !rc; i++) {
        gkey* k = &keys[i];
        if (!k->name || !(k->for_mask & K_NODE) || k->type != T_STR || vstr_slot(k->name) < 0) continue;
        const int a = vstr_slot(k->name);
        has_vs[a] = 1;
        for (size_t j = 0; j < vs[a].len; j++)
            if (!vs[a].a[j]) vs[a].a[j] = strdup(k->defval ? k->defval : "");
    }
    for (int i = 0; i < nkeys && !rc; i++) {
        gkey* k = &keys[i];
        if (!k->defval || !k->name || k->type != T_NUM) continue;
        double d = parse_num(k->defval);
        dvec* col = NULL;
        if (k->for_mask & K_NODE) {
            if (!strcmp(k->name, "bandwidthdown")) col = &va[VA_BWDOWN];
            else if (!strcmp(k->name, "bandwidthup")) col = &va[VA_BWUP];
            else if (!strcmp(k->name, "packetloss")) col = &va[VA_LOSS];
            else if (!strcmp(k->name, "asn")) col = &va[VA_ASN];
            if (col) for (size_t j = 0; j < col->len; j++) if (isnan(col->a[j])) col->a[j] = d;
        }
        col = NULL;
        if (k->for_mask & K_EDGE) {
            if (!strcmp(k->name, "latency")) col = &ea[EA_LAT];
            else if (!strcmp(k->name, "packetloss")) col = &ea[EA_LOSS];
            else if (!strcmp(k->name, "jitter")) col = &ea[EA_JITTER];
            if (col) for (size_t j = 0; j < col->len; j++) if (isnan(col->a[j])) col->a[j] = d;
        }
    }

    /* _topology_checkGraphAttributes (topology.c:565-722): declared types + required keys */
    int have_bwd = 0, have_bwu = 0, have_lat = 0, have_eloss = 0, have_vloss = 0;
    for (int i = 0; i < nkeys && !rc; i++) {
        gkey* k = &keys[i];
        if (!k->name) continue;
        const char* nmk = k->name;
        if (k->for_mask & K_NODE) {
            int want = 0;
            if (!strcmp(nmk, "bandwidthdown")) { want = T_NUM; have_bwd = 1; }
            else if (!strcmp(nmk, "bandwidthup")) { want = T_NUM; have_bwu = 1; }
            else if (!strcmp(nmk, "packetloss")) { want = T_NUM; have_vloss = 1; }
            else if (!strcmp(nmk, "asn")) want = T_NUM;
            else if (!strcmp(nmk, "ip") || !strcmp(nmk, "citycode") || !strcmp(nmk, "countrycode") ||
                     !strcmp(nmk, "type") || !strcmp(nmk, "geocode") || !strcmp(nmk, "id")) want = T_STR;
            if (want && k->type != want) {
                seterr(errbuf, errlen, "vertex attribute '%s' has an unsupported type", nmk);
                rc = SHD_ROUTE_EINVAL;
            }
        }
        if ((k->for_mask & K_EDGE) && !rc) {
            int want = 0;
            if (!strcmp(nmk, "latency")) { want = T_NUM; have_lat = 1; }
            else if (!strcmp(nmk, "packetloss")) { want = T_NUM; have_eloss = 1; }
            else if (!strcmp(nmk, "jitter")) want = T_NUM;
            if (want && k->type != want) {
                seterr(errbuf, errlen, "edge attribute '%s' has an unsupported type", nmk);
                rc = SHD_ROUTE_EINVAL;
            }
        }
        if ((k->for_mask & K_GRAPH) && !strcmp(nmk, "preferdirectpaths") && k->type != T_STR && !rc) {
            seterr(errbuf, errlen, "graph attribute 'preferdirectpaths' must be a string");
            rc = SHD_ROUTE_EINVAL;
        }
    }
    if (!rc && (!have_bwd || !have_bwu)) { seterr(errbuf, errlen, "required vertex attribute bandwidthdown/bandwidthup missing"); rc = SHD_ROUTE_EINVAL; }
    if (!rc && (!have_lat || !have_eloss)) { seterr(errbuf, errlen, "required edge attribute latency/packetloss missing"); rc = SHD_ROUTE_EINVAL; }
    if (!rc && n == 0) { seterr(errbuf, errlen, "graph has no vertices"); rc = SHD_ROUTE_EINVAL; }
    /* per-vertex (topology.c:811-978) and per-edge (topology.c:1041-1124) values */
    for (int32_t v = 0; v < n && !rc; v++) {
        if (!(va[VA_BWDOWN].a[v] > 0.0) || !(va[VA_BWUP].a[v] > 0.0)) {
            seterr(errbuf, errlen, "vertex %d ('%s'): bandwidth missing, NaN or non-positive", v, vid[v]);
            rc = SHD_ROUTE_EINVAL;
        } else if (!isnan(va[VA_ASN].a[v]) && !(va[VA_ASN].a[v] > 0.0)) {
            seterr(errbuf, errlen, "vertex %d ('%s'): asn non-positive", v, vid[v]);
            rc = SHD_ROUTE_EINVAL;
        } else if (!isnan(va[VA_LOSS].a[v]) && !(va[VA_LOSS].a[v] >= 0.0 && va[VA_LOSS].a[v] <= 1.0)) {
            seterr(errbuf, errlen, "vertex %d ('%s'): packetloss out of [0,1]", v, vid[v]);
            rc = SHD_ROUTE_EINVAL;
        }
    }
    for (size_t e = 0; e < esrc.len && !rc; e++) {
        if (!(ea[EA_LAT].a[e] > 0.0)) {
            seterr(errbuf, errlen, "edge %zu: latency missing, NaN or non-positive", e);
            rc = SHD_ROUTE_EINVAL;
        } else if (!(ea[EA_LOSS].a[e] >= 0.0 && ea[EA_LOSS].a[e] <= 1.0)) {
            seterr(errbuf, errlen, "edge %zu: packetloss missing or out of [0,1]", e);
            rc = SHD_ROUTE_EINVAL;
        } else if (!isnan(ea[EA_JITTER].a[e]) && !(ea[EA_JITTER].a[e] >= 0.0)) {
            seterr(errbuf, errlen, "edge %zu: jitter negative", e);
            rc = SHD_ROUTE_EINVAL;
        }
    }

    if (!rc) {
        shd_graph_t* g = &out->graph;
        g->n_vertices = n;
        g->n_edges = (int32_t)esrc.len;
        g->edge_src = esrc.a; esrc.a = NULL;
        g->edge_dst = edst.a; edst.a = NULL;
        g->edge_latency = ea[EA_LAT].a; ea[EA_LAT].a = NULL;
        g->edge_packetloss = ea[EA_LOSS].a; ea[EA_LOSS].a = NULL;
        out->has_vertex_packetloss = have_vloss;
        if (have_vloss) { g->vertex_packetloss = va[VA_LOSS].a; va[VA_LOSS].a = NULL; }
        g->directed = directed;
        /* topology.c:769-790: prefix true/yes/1, case-insensitive */
        g->prefer_direct = prefer && (!strncasecmp(prefer, "true", 4) || !strncasecmp(prefer, "yes", 3) ||
                                      !strncasecmp(prefer, "1", 1));
        out->vertex_ids = vid; vid = NULL;
        out->bandwidth_down = va[VA_BWDOWN].a; va[VA_BWDOWN].a = NULL;
        out->bandwidth_up = va[VA_BWUP].a; va[VA_BWUP].a = NULL;
        for (int a = 0; a < SHD_VATTR_N; a++) {
            out->has_vertex_str[a] = has_vs[a];
            out->vertex_str[a] = vs[a].a; vs[a].a = NULL;
        }
    }
    if (vid) { for (int32_t v = 0; v < n; v++) free(vid[v]); free(vid); }
    for (int a = 0; a < VA_N; a++) free(va[a].a);
    for (int a = 0; a < SHD_VATTR_N; a++) {
        if (vs[a].a) for (size_t j = 0; j < vs[a].len; j++) free(vs[a].a[j]);
        free(vs[a].a);
    }
    for (int a = 0; a < EA_N; a++) free(ea[a].a);
    free(esrc.a); free(edst.a); free(prefer);
    for (int i = 0; i < nkeys; i++) {
        xmlFree(keys[i].id); xmlFree(keys[i].name); xmlFree(keys[i].defval);
    }
    free(keys);
    idmap_free(&ids);
    return rc;
}

void shd_graphml_free(shd_graphml_t* g) {
    if (!g) return;
    if (g->vertex_ids) {
        for (int32_t v = 0; v < g->graph.n_vertices; v++) free(g->vertex_ids[v]);
        free(g->vertex_ids);
    }
    free((void*)g->graph.edge_src); free((void*)g->graph.edge_dst);
    free((void*)g->graph.edge_latency); free((void*)g->graph.edge_packetloss);
    free((void*)g->graph.vertex_packetloss);
    free(g->bandwidth_down); free(g->bandwidth_up);
    for (int a = 0; a < SHD_VATTR_N; a++) {
        if (g->vertex_str[a]) for (int32_t v = 0; v < g->graph.n_vertices; v++) free(g->vertex_str[a][v]);
        free(g->vertex_str[a]);
    }
    memset(g, 0, sizeof(*g));
}
