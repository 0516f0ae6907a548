/*
 * attach.c -- host attachment of Shadow 1.14's src/main/routing/topology.c
 * (mckerrigan/shadow): which vertex a host joins, given its hints.
 *
 * Reference behaviour kept:
 *   - a string attribute counts only when the key exists and the value is non-empty
 *     (_topology_findVertexAttributeString, topology.c:306-328); codes and types match
 *     case-insensitively in ASCII (g_ascii_strcasecmp, topology.c:2117-2120);
 *   - IPs are inet_pton values in network byte order (address_stringToIP, address.c:
 *     145-152); "usable" excludes INADDR_NONE, INADDR_ANY and the host-order constant
 *     INADDR_LOOPBACK compared against that network-order value (topology.c:2126,
 *     2262), as the reference compares them;
 *   - vertices are visited in index order; the first exact IP match clears every
 *     candidate list and from then on only exact matches are collected (topology.c:
 *     2134-2161); the per-list IP counters are never cleared;
 *   - the first non-empty list of CityAndType, City, CountryAndType, Country,
 *     GeoAndType, Geo, Type, All is used (topology.c:2299-2323); longest-prefix match
 *     over it when the requested IP is usable (for All: when an ip hint was given) and
 *     the list holds a usable IP, unless an exact match was found (topology.c:2330);
 *     the match is ~(ip_v ^ ip) on the network-order values, the first candidate or any
 *     later one with a larger value, or any when the best is still 0 (topology.c:
 *     2218-2243), over every candidate including those without an IP (INADDR_NONE);
 *   - otherwise one random_nextDouble draw picks element round((len-1) * d) in list
 *     order (topology.c:2333-2339).
 * What changes: the per-vertex strings are parsed and interned case-folded once into
 * integers (IP values, dictionary ids per attribute), with posting lists per id and the
 * usable IPs sorted by (ip, vertex).  A host then costs a binary search for exact IP
 * matches, O(1) list sizes (a walk of one posting list for the *AndType lists) and the
 * chosen member by index, instead of 8 GQueues filled through 5 igraph attribute
 * lookups per vertex per host under the graph lock.  Only a longest-prefix match still
 * walks its whole list.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <math.h>
#include <netinet/in.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/shd_topology.h"

enum { L_CITY_TYPE, L_CITY, L_COUNTRY_TYPE, L_COUNTRY, L_GEO_TYPE, L_GEO, L_TYPE, L_ALL, L_N };

struct shd_attach {
    int32_t n;
    int has_ip;
    uint32_t* ip;        /* inet_pton value (network order) of the ip string, INADDR_NONE if none */
    uint8_t* ip_usable;  /* found and not NONE / ANY / LOOPBACK (as compared at topology.c:2126) */
    /* citycode, countrycode, geocode, type interned case-folded: id[k][v] in 1..nid[k],
     * 0 = not found / empty; dictionary str[k][id] (folded) with hashes hs[k][id] */
    uint32_t* id[4];
    uint32_t nid[4];
    char** str[4];
    uint64_t* hs[4];
    uint32_t* tab[4];    /* open-addressing table hash -> id (0 = empty), tmask + 1 slots */
    uint32_t tmask;
    /* posting lists: vertices holding id i of attribute k are post[k][off[k][i] ..
     * off[k][i+1]) in index order, nipc[k][i] of them with a usable IP */
    int32_t* off[4];
    int32_t* post[4];
    int32_t* nipc[4];
    int32_t nusable;
    /* usable IPs sorted by (ip, vertex): exact matches are one equal range */
    int32_t nex;
    uint32_t* exip;
    int32_t* exv;
};

static int fold(int c) { return (c >= 'A' && c <= 'Z') ? c + ('a' - 'A') : c; }
static uint64_t fold_hash(const char* s) {
    uint64_t h = 1469598103934665603ull;
    for (; *s; s++) h = (h ^ (uint64_t)(unsigned char)fold((unsigned char)*s)) * 1099511628211ull;
    return h | 1ull;  /* never 0: 0 marks "not found" */
}
static int ascii_caseeq(const char* a, const char* b) {
    for (;; a++, b++) {
        const int x = fold((unsigned char)*a), y = fold((unsigned char)*b);
        if (x != y) return 0;
        if (!x) return 1;
    }
}
static uint32_t str_to_ip(const char* s) {
    struct in_addr in;
    return (s && inet_pton(AF_INET, s, &in) == 1) ? (uint32_t)in.s_addr : (uint32_t)INADDR_NONE;
}
static int ip_usable(uint32_t ip) {
    return ip != (uint32_t)INADDR_NONE && ip != (uint32_t)INADDR_ANY && ip != (uint32_t)INADDR_LOOPBACK;
}

static int cmp_u64(const void* x, const void* y) {
    const uint64_t p = *(const uint64_t*)x, q = *(const uint64_t*)y;
    return (p > q) - (p < q);
}

/* id of the case-folded string x among attribute k's values, 0 if absent */
static uint32_t intern_find(const shd_attach_t* a, int k, const char* x) {
    const uint64_t h = fold_hash(x);
    for (uint32_t j = (uint32_t)(h >> 17) & a->tmask;; j = (j + 1) & a->tmask) {
        const uint32_t i = a->tab[k][j];
        if (!i) return 0;
        if (a->hs[k][i] == h && ascii_caseeq(a->str[k][i], x)) return i;
    }
}
static void intern_add(shd_attach_t* a, int k, uint32_t i) {
    uint32_t j = (uint32_t)(a->hs[k][i] >> 17) & a->tmask;
    while (a->tab[k][j]) j = (j + 1) & a->tmask;
    a->tab[k][j] = i;
}

int shd_attach_create(shd_attach_t** out, const shd_graphml_t* g) {
    if (!out || !g || g->graph.n_vertices <= 0) return SHD_ROUTE_EINVAL;
    shd_attach_t* a = calloc(1, sizeof(*a));
    const int32_t n = g->graph.n_vertices;
    a->n = n;
    a->ip = malloc(sizeof(uint32_t) * (size_t)n);
    a->ip_usable = calloc((size_t)n, 1);
    a->has_ip = g->has_vertex_str[SHD_VATTR_IP] && g->vertex_str[SHD_VATTR_IP];
    for (int32_t v = 0; v < n; v++) {
        const char* s = a->has_ip ? g->vertex_str[SHD_VATTR_IP][v] : NULL;
        a->ip[v] = str_to_ip(s);
        a->ip_usable[v] = (s && s[0]) ? (uint8_t)ip_usable(a->ip[v]) : 0;
    }
    const int slot[4] = {SHD_VATTR_CITYCODE, SHD_VATTR_COUNTRYCODE, SHD_VATTR_GEOCODE, SHD_VATTR_TYPE};
    uint32_t cap = 16;
    while (cap < 2u * (uint32_t)n + 2u) cap <<= 1;
    a->tmask = cap - 1;
    for (int k = 0; k < 4; k++) {
        a->tab[k] = calloc(cap, sizeof(uint32_t));
        a->id[k] = calloc((size_t)n, sizeof(uint32_t));
        a->str[k] = calloc((size_t)n + 1, sizeof(char*));
        a->hs[k] = calloc((size_t)n + 1, sizeof(uint64_t));
        const int has = g->has_vertex_str[slot[k]] && g->vertex_str[slot[k]];
        for (int32_t v = 0; v < n && has; v++) {
            const char* x = g->vertex_str[slot[k]][v];
            if (x && x[0]) {
                uint32_t i = intern_find(a, k, x);
                if (!i) {
                    i = ++a->nid[k];
                    a->str[k][i] = strdup(x);
                    for (char* c = a->str[k][i]; *c; c++) *c = (char)fold((unsigned char)*c);
                    a->hs[k][i] = fold_hash(x);
                    intern_add(a, k, i);
                }
                a->id[k][v] = i;
            }
        }
    }
    for (int k = 0; k < 4; k++) {
        const uint32_t m = a->nid[k];
        a->off[k] = calloc((size_t)m + 2, sizeof(int32_t));
        a->nipc[k] = calloc((size_t)m + 1, sizeof(int32_t));
        a->post[k] = malloc(sizeof(int32_t) * ((size_t)n + 1));
        for (int32_t v = 0; v < n; v++) {
            a->off[k][a->id[k][v] + 1]++;
            a->nipc[k][a->id[k][v]] += a->ip_usable[v];
        }
        for (uint32_t i = 0; i <= m; i++) a->off[k][i + 1] += a->off[k][i];
        int32_t* fill = malloc(sizeof(int32_t) * ((size_t)m + 1));
        memcpy(fill, a->off[k], sizeof(int32_t) * ((size_t)m + 1));
        for (int32_t v = 0; v < n; v++) a->post[k][fill[a->id[k][v]]++] = v;
        free(fill);
    }
    a->exip = malloc(sizeof(uint32_t) * ((size_t)n + 1));
    a->exv = malloc(sizeof(int32_t) * ((size_t)n + 1));
    uint64_t* keys = malloc(sizeof(uint64_t) * ((size_t)n + 1));
    for (int32_t v = 0; v < n; v++)
        if (a->ip_usable[v]) keys[a->nex++] = ((uint64_t)a->ip[v] << 32) | (uint32_t)v;
    a->nusable = a->nex;
    qsort(keys, (size_t)a->nex, sizeof(uint64_t), cmp_u64);
    for (int32_t i = 0; i < a->nex; i++) { a->exip[i] = (uint32_t)(keys[i] >> 32); a->exv[i] = (int32_t)(uint32_t)keys[i]; }
    free(keys);
    *out = a;
    return SHD_ROUTE_OK;
}

void shd_attach_destroy(shd_attach_t* a) {
    if (!a) return;
    for (int k = 0; k < 4; k++) {
        if (a->str[k]) for (uint32_t i = 1; i <= a->nid[k]; i++) free(a->str[k][i]);
        free(a->str[k]);
        free(a->hs[k]);
        free(a->id[k]);
        free(a->off[k]); free(a->post[k]); free(a->nipc[k]); free(a->tab[k]);
    }
    free(a->exip); free(a->exv);
    free(a->ip);
    free(a->ip_usable);
    free(a);
}

/* candidate list L (topology.c:2299-2323) as a view: members are base[0..len) (base NULL:
 * every vertex 0..len), keeping only those of type `filt` when filt != 0 */
typedef struct {
    const int32_t* base;
    int32_t len;
    uint32_t filt;
} view_t;

static view_t list_view(const shd_attach_t* a, int list, const uint32_t hid[4]) {
    view_t w = {NULL, 0, 0};
    if (list == L_ALL) { w.len = a->n; return w; }
    static const int attr[L_ALL] = {0, 0, 1, 1, 2, 2, 3};
    const int k = attr[list];
    const uint32_t h = hid[k];
    if (h == UINT32_MAX || (list != L_TYPE && (list & 1) == 0 && hid[3] == UINT32_MAX)) return w;
    w.base = a->post[k] + a->off[k][h];
    w.len = a->off[k][h + 1] - a->off[k][h];
    w.filt = (list == L_CITY_TYPE || list == L_COUNTRY_TYPE || list == L_GEO_TYPE) ? hid[3] : 0;
    return w;
}

/* members and usable-IP members of a view */
static void view_count(const shd_attach_t* a, const view_t* w, int list, const uint32_t hid[4], int32_t* cnt,
                       int32_t* nip) {
    if (!w->filt) {
        *cnt = w->len;
        if (list == L_ALL) *nip = a->nusable;
        else {
            static const int attr[L_ALL] = {0, 0, 1, 1, 2, 2, 3};
            *nip = a->nipc[attr[list]][hid[attr[list]]];
        }
        return;
    }
    int32_t c = 0, u = 0;
    const uint32_t* ty = a->id[3];
    for (int32_t i = 0; i < w->len; i++) {
        const int32_t v = w->base[i];
        const int32_t in = ty[v] == w->filt;
        c += in;
        u += in & a->ip_usable[v];
    }
    *cnt = c;
    *nip = u;
}

int32_t shd_attach_find_vertex(const shd_attach_t* a, shd_next_double_fn next_double, void* ctx,
                               const char* ip_hint, const char* citycode_hint, const char* countrycode_hint,
                               const char* geocode_hint, const char* type_hint) {
    if (!a || a->n <= 0) return -1;
    /* requested IP (topology.c:2258-2264); requestedIP stays 0 when unusable (g_new0) */
    uint32_t req = 0;
    int req_usable = 0;
    if (ip_hint) {
        const uint32_t ip = str_to_ip(ip_hint);
        if (ip_usable(ip)) { req = ip; req_usable = 1; }
    }
    /* a hint matches the vertices holding its interned id; an absent, empty or unknown
     * hint matches none (UINT32_MAX is never an id) */
    const char* hint[4] = {citycode_hint, countrycode_hint, geocode_hint, type_hint};
    uint32_t hid[4];
    for (int k = 0; k < 4; k++) {
        const uint32_t i = (hint[k] && hint[k][0]) ? intern_find(a, k, hint[k]) : 0;
        hid[k] = i ? i : UINT32_MAX;
    }

    /* exact IP matches (topology.c:2134-2161): an equal range of the sorted IPs, in
     * vertex order; they replace every list and are chosen from at random */
    int32_t lo = 0, hi = 0;
    if (req_usable) {
        int32_t l = 0, r = a->nex;
        while (l < r) { const int32_t m = (l + r) / 2; if (a->exip[m] < req) l = m + 1; else r = m; }
        lo = hi = l;
        while (hi < a->nex && a->exip[hi] == req) hi++;
    }
    if (hi > lo) {
        const double d = next_double ? next_double(ctx) : 0.0;
        const int32_t range = hi - lo - 1;
        int32_t k = (int32_t)round((double)(range * d));
        if (k < 0) k = 0;
        if (k > range) k = range;
        return a->exv[lo + k];
    }

    /* the first non-empty list (topology.c:2299-2323) */
    int list = 0;
    view_t w;
    int32_t len = 0, nip = 0;
    for (; list <= L_ALL; list++) {
        w = list_view(a, list, hid);
        if (w.len == 0) continue;
        view_count(a, &w, list, hid, &len, &nip);
        if (len > 0) break;
    }
    if (len <= 0) return -1;
    const int lpm = list == L_ALL ? (ip_hint != NULL && nip > 0) : (req_usable && nip > 0);

    int32_t pick = -1;
    if (lpm) {
        /* _topology_getLongestPrefixMatch over the list in order (topology.c:2218-2243) */
        uint32_t best = 0;
        for (int32_t i = 0; i < w.len; i++) {
            const int32_t v = w.base ? w.base[i] : i;
            if (w.filt && a->id[3][v] != w.filt) continue;
            const uint32_t match = ~(a->ip[v] ^ req);
            if (match > best || best == 0) { best = match; pick = v; }
        }
        return pick;
    }
    /* one random_nextDouble draw, element round((len-1) * d) in list order */
    const double d = next_double ? next_double(ctx) : 0.0;
    const int32_t range = len - 1;
    int32_t k = (int32_t)round((double)(range * d));
    if (k < 0) k = 0;
    if (k > range) k = range;
    if (!w.filt) return w.base ? w.base[k] : k;
    for (int32_t i = 0, seen = 0; i < w.len; i++) {
        const int32_t v = w.base[i];
        if (a->id[3][v] == w.filt && seen++ == k) return v;
    }
    return pick;
}
