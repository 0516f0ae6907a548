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
 * integers (IP values, dictionary ids per attribute), and the lists are counted
 * in one pass and materialised for the chosen list only, instead of 8 GQueues filled
 * through 5 igraph attribute lookups per vertex per host under the graph lock.
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

/* id of the case-folded string x among attribute k's values, 0 if absent (the
 * dictionaries are small: a few hundred codes) */
static uint32_t intern_find(const shd_attach_t* a, int k, const char* x) {
    const uint64_t h = fold_hash(x);
    for (uint32_t i = 1; i <= a->nid[k]; i++)
        if (a->hs[k][i] == h && ascii_caseeq(a->str[k][i], x)) return i;
    return 0;
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
    for (int k = 0; k < 4; k++) {
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
                }
                a->id[k][v] = i;
            }
        }
    }
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
    }
    free(a->ip);
    free(a->ip_usable);
    free(a);
}

/* list membership bits of vertex v (bit L_*) for the interned hint ids */
static inline unsigned lists_of(const shd_attach_t* a, int32_t v, const uint32_t hid[4]) {
    const unsigned city = a->id[0][v] == hid[0], country = a->id[1][v] == hid[1];
    const unsigned geo = a->id[2][v] == hid[2], type = a->id[3][v] == hid[3];
    return ((city & type) << L_CITY_TYPE) | (city << L_CITY) | ((country & type) << L_COUNTRY_TYPE) |
           (country << L_COUNTRY) | ((geo & type) << L_GEO_TYPE) | (geo << L_GEO) | (type << L_TYPE) |
           (1u << L_ALL);
}

int32_t shd_attach_find_vertex(const shd_attach_t* a, shd_next_double_fn next_double, void* ctx,
                               const char* ip_hint, const char* citycode_hint, const char* countrycode_hint,
                               const char* geocode_hint, const char* type_hint) {
    if (!a || a->n <= 0) return -1;
    const int32_t n = a->n;
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

    /* pass 1: exact IP matches, else per-list sizes and usable-IP counts */
    int32_t cnt[L_N] = {0}, nip[L_N] = {0}, nexact = 0;
    for (int32_t v = 0; v < n; v++) {
        if (req_usable && a->ip_usable[v] && a->ip[v] == req) { nexact++; continue; }
        if (nexact) continue;  /* after the first exact match only exact matches count */
        const unsigned m = lists_of(a, v, hid);
        const int32_t u = a->ip_usable[v];
        for (int l = 0; l < L_N; l++) {
            const int32_t in = (int32_t)((m >> l) & 1u);
            cnt[l] += in;
            nip[l] += in & u;
        }
    }
    int list = L_ALL, lpm = 0;
    int32_t len;
    if (nexact) {
        len = nexact;  /* candidatesAll holds the exact matches; random choice among them */
    } else {
        for (list = 0; list < L_ALL && cnt[list] == 0; list++) {}
        len = cnt[list];
        lpm = list == L_ALL ? (ip_hint != NULL && nip[L_ALL] > 0) : (req_usable && nip[list] > 0);
    }
    if (len <= 0) return -1;

    int32_t pick = -1;
    if (lpm) {
        /* _topology_getLongestPrefixMatch over the list in order (topology.c:2218-2243) */
        uint32_t best = 0;
        for (int32_t v = 0; v < n; v++) {
            if (!(lists_of(a, v, hid) & (1u << list))) continue;
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
    for (int32_t v = 0, seen = 0; v < n; v++) {
        const int in = nexact ? (req_usable && a->ip_usable[v] && a->ip[v] == req)
                              : ((lists_of(a, v, hid) >> list) & 1u);
        if (in && seen++ == k) { pick = v; break; }
    }
    return pick;
}
