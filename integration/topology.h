/* Shadow 1.14's public routing API (reference src/main/routing/topology.h:17-28),
 * unchanged; the stand-in environment replaces main/routing/address.h and
 * main/utility/random.h outside the simulator. */
#ifndef SHD_TOPOLOGY_H_
#define SHD_TOPOLOGY_H_

#include <glib.h>

#include "shadow_env.h"

typedef struct _Topology Topology;

Topology* topology_new(const gchar* graphPath);
void topology_free(Topology* top);

void topology_attach(Topology* top, Address* address, Random* randomSourcePool,
        gchar* ipHint, gchar* citycodeHint, gchar* countrycodeHint, gchar* geocodeHint, gchar* typeHint,
        guint64* bwDownOut, guint64* bwUpOut);
void topology_detach(Topology* top, Address* address);

gboolean topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress);
gdouble topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress);
gdouble topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress);
void topology_incrementPathPacketCounter(Topology* top, Address* srcAddress, Address* dstAddress);

#endif
