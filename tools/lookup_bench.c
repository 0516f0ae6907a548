/* Per-packet lookup path: worker_sendPacket (worker.c:243-304) makes
 * three topology calls per packet -- topology_isRoutable / getLatency,
 * getReliability and incrementPathPacketCounter (topology.c:2053-2092) -- each of
 * which in the reference takes the pathCache RW lock and two glib hash lookups
 * (topology.c:1284-1305).  Here they index the dense triangle (no lock after the
 * fill) plus a striped counter map.  This driver loads a graphml, attaches every
 * vertex, fills on the GPU, then times T threads x M packets of the three calls over
 * seeded random (src, dst) pairs and prints one JSON line.
 *
 *   gcc -O2 -pthread -Iinclude tools/lookup_bench.c -Lshadow_amd -lshd_topology \
 *       -Wl,-rpath,$PWD/shadow_amd -o gpurun_out/lookup_bench
 *   gpurun_out/lookup_bench graph.xml threads packets_per_thread
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "shd_topology.h"

typedef struct {
    shd_topology_t* top;
    int32_t n;
    long packets;
    uint64_t seed;
    double checksum;
} job_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static inline uint64_t xorshift(uint64_t* s) {
    uint64_t x = *s;
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    return *s = x;
}

static void* worker(void* arg) {
    job_t* j = arg;
    uint64_t s = j->seed;
    double acc = 0;
    for (long p = 0; p < j->packets; p++) {
        const uint64_t r = xorshift(&s);
        const int32_t a = (int32_t)((r & 0xFFFFFFFFu) % (uint32_t)j->n);
        const int32_t b = (int32_t)((r >> 32) % (uint32_t)j->n);
        if (!shd_topology_is_routable(j->top, a, b)) continue;   /* worker.c:267 */
        acc += shd_topology_get_latency(j->top, a, b);            /* worker.c:275 */
        acc += shd_topology_get_reliability(j->top, a, b);        /* worker.c:279 */
        shd_topology_increment_path_packet_counter(j->top, a, b);
    }
    j->checksum = acc;
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s graph.xml threads packets_per_thread\n", argv[0]); return 2; }
    const int T = atoi(argv[2]);
    const long M = atol(argv[3]);
    shd_topology_t* top = shd_topology_new(argv[1], NULL, 0);
    if (!top) return 1;
    const int32_t n = shd_topology_vertex_count(top);
    for (int32_t v = 0; v < n; v++) shd_topology_attach_vertex(top, v);
    double fill_s = 0;
    if (shd_topology_fill(top, &fill_s)) { fprintf(stderr, "fill failed\n"); return 1; }
    pthread_t th[256];
    job_t jobs[256];
    const int nt = T < 256 ? T : 256;
    const double t0 = now_s();
    for (int i = 0; i < nt; i++) {
        jobs[i] = (job_t){top, n, M, 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1), 0};
        pthread_create(&th[i], NULL, worker, &jobs[i]);
    }
    double chk = 0;
    for (int i = 0; i < nt; i++) { pthread_join(th[i], NULL); chk += jobs[i].checksum; }
    const double dt = now_s() - t0;
    const double pkts = (double)nt * (double)M;
    /* every counted packet must be visible exactly once in the counters */
    uint64_t counted = 0;
    for (int32_t a = 0; a < n; a++)
        for (int32_t b = a; b < n; b++) counted += shd_topology_get_path_packet_count(top, a, b);
    printf("{\"metric\": \"packet_lookups_per_s\", \"value\": %.1f, \"threads\": %d, \"packets\": %.0f, "
           "\"ns_per_packet_per_thread\": %.2f, \"calls_per_packet\": 4, \"n_vertices\": %d, "
           "\"fill_s\": %.4f, \"counted\": %llu, \"checksum\": %.6e}\n",
           pkts / dt, nt, pkts, 1e9 * dt * nt / pkts, n, fill_s, (unsigned long long)counted, chk);
    shd_topology_free(top);
    return counted == (uint64_t)pkts ? 0 : 3;
}
