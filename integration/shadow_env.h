/*
 * shadow_env.h -- stand-ins for the few pieces of Shadow 1.14 that the topology.c glue
 * touches (Address, Random, logging, the runahead upcall), so that the glue in
 * integration/topology.c compiles and runs outside the simulator.  In Shadow these come
 * from main/routing/address.h, main/utility/random.h, support/logger and main/core/worker.h;
 * only their interfaces matter here.  Test harness, not product.
 */
#ifndef SHD_GLUE_SHADOW_ENV_H
#define SHD_GLUE_SHADOW_ENV_H

#include <glib.h>
#include <netinet/in.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct _Address {
    in_addr_t ip;  /* network order, as address_toNetworkIP returns it */
} Address;
static inline in_addr_t address_toNetworkIP(Address* a) { return a->ip; }

/* random.c:29-40: rand_r over a per-pool seed, scaled to [0, 1] */
typedef struct _Random {
    guint seed;
} Random;
static inline gdouble random_nextDouble(Random* r) { return ((gdouble)rand_r(&r->seed)) / ((gdouble)RAND_MAX); }

#define critical(...) (fprintf(stderr, "critical: " __VA_ARGS__), fputc('\n', stderr))
#define MAGIC_DECLARE guint magic
#define MAGIC_INIT(o) ((o)->magic = 0xAABBCCDDu)
#define MAGIC_ASSERT(o) g_assert((o) && (o)->magic == 0xAABBCCDDu)
#define MAGIC_CLEAR(o) ((o)->magic = 0)

/* worker.c:412 (-> slave.c:381 -> master.c:148): the runahead upcall */
void worker_updateMinTimeJump(gdouble minPathLatency);

#endif
