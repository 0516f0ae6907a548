/*
 * glue_main.c -- drives integration/topology.c the way Shadow does (master.c:224
 * topology_new, host.c:181 topology_attach per host, worker.c:267-279 per packet:
 * isRoutable, getLatency, getReliability, incrementPathPacketCounter; host.c:243
 * topology_detach; master.c:115 topology_free) and prints one JSON line.
 * usage: glue_test <graphml[.xz]> <hosts> <packets> [seed]
 */
#include <arpa/inet.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "topology.h"

static gdouble g_runahead = -1;
gint topology_testVertexOf(Topology* top, Address* a);  /* test hook in topology.c */
void worker_updateMinTimeJump(gdouble minPathLatency) { g_runahead = minPathLatency; }

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s graphml hosts packets [seed]\n", argv[0]); return 2; }
    const int H = atoi(argv[2]);
    const long P = atol(argv[3]);
    Random rnd = {.seed = argc > 4 ? (guint)atoi(argv[4]) : 1u};
    double t0 = now_s();
    Topology* top = topology_new(argv[1]);
    if (!top) return 1;
    Address* a = g_new0(Address, H);
    guint64 bw_down = 0, bw_up = 0, bw_sum = 0;
    for (int h = 0; h < H; h++) {
        a[h].ip = htonl(0x0B000001u + (guint32)h);  /* 11.0.0.1, ... */
        topology_attach(top, &a[h], &rnd, NULL, NULL, NULL, NULL, NULL, &bw_down, &bw_up);
        bw_sum += bw_down + bw_up;
    }
    const double t_attach = now_s() - t0;
    double lat_sum = 0, rel_min = 2, rel_max = -1, lat_min = 1e300;
    long routable = 0;
    t0 = now_s();
    guint seed2 = 7;
    /* SHD_GLUE_TRACE=<file>: the first SHD_GLUE_TRACE_N (1000) routable packets as
     * "src_vertex dst_vertex latency reliability" lines, exact (%.17g) */
    FILE* trace = getenv("SHD_GLUE_TRACE") ? fopen(getenv("SHD_GLUE_TRACE"), "w") : NULL;
    const long trace_n = getenv("SHD_GLUE_TRACE_N") ? atol(getenv("SHD_GLUE_TRACE_N")) : 1000;
    for (long k = 0; k < P; k++) {
        Address* s = &a[rand_r(&seed2) % H];
        Address* d = &a[rand_r(&seed2) % H];
        if (!topology_isRoutable(top, s, d)) continue;          /* worker.c:267 */
        const gdouble L = topology_getLatency(top, s, d);       /* worker.c:275 */
        const gdouble R = topology_getReliability(top, s, d);   /* worker.c:279 */
        topology_incrementPathPacketCounter(top, s, d);
        if (trace && routable < trace_n)
            fprintf(trace, "%d %d %.17g %.17g\n", topology_testVertexOf(top, s), topology_testVertexOf(top, d), L, R);
        routable++;
        lat_sum += L;
        if (L < lat_min) lat_min = L;
        if (R < rel_min) rel_min = R;
        if (R > rel_max) rel_max = R;
    }
    const double t_packets = now_s() - t0;
    if (trace) fclose(trace);
    /* host.c:243: a detached address has no vertex any more -> -1 (topology.c:1973-1985) */
    topology_detach(top, &a[0]);
    const gdouble after = topology_getLatency(top, &a[0], &a[H > 1 ? 1 : 0]);
    const gboolean after_r = topology_isRoutable(top, &a[H > 1 ? 1 : 0], &a[0]);
    printf("{\"hosts\": %d, \"packets\": %ld, \"routable\": %ld, \"lat_sum\": %.17g, \"lat_min\": %.17g, "
           "\"rel_min\": %.17g, \"rel_max\": %.17g, \"runahead_reported_ms\": %.17g, \"detached_latency\": %.17g, "
           "\"detached_routable\": %d, \"bw_sum\": %llu, \"attach_s\": %.6f, \"packets_s\": %.6f}\n",
           H, P, routable, lat_sum, lat_min, rel_min, rel_max, g_runahead, after, after_r ? 1 : 0,
           (unsigned long long)bw_sum, t_attach, t_packets);
    topology_free(top);
    g_free(a);
    return 0;
}
