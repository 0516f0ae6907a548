"""CPU restatement of Shadow 1.14's host attachment (mckerrigan/shadow
src/main/routing/topology.c) -- TEST INFRASTRUCTURE ONLY: imported by tests/, never
by the product (shadow_amd/).  It follows the reference's own structure (eight
GQueues filled by a per-vertex hook, cleared on the first exact IP match) so that it
checks the product's count-then-materialise implementation (shadow_amd/csrc/attach.c)
independently.

Random draws: Shadow's Random is glibc rand_r over a per-pool seed state
(src/main/utility/random.c:29-43); ShadowRandom calls the same libc rand_r.
"""
from __future__ import annotations

import ctypes as C
import math
import socket
import struct

INADDR_NONE = 0xFFFFFFFF
INADDR_ANY = 0x00000000
INADDR_LOOPBACK = 0x7F000001  # host-order constant, compared against network-order values
RAND_MAX = 2147483647


class ShadowRandom:
    """random_nextDouble (random.c:39-43): rand_r(&seedState) / RAND_MAX."""

    def __init__(self, seed: int):
        self._libc = C.CDLL(None)
        self._libc.rand_r.argtypes = [C.POINTER(C.c_uint)]
        self._libc.rand_r.restype = C.c_int
        self._state = C.c_uint(seed)
        self.draws = 0

    def next_double(self) -> float:
        self.draws += 1
        return float(self._libc.rand_r(C.byref(self._state))) / float(RAND_MAX)


def string_to_ip(s):
    """address_stringToIP (address.c:145-152): inet_pton -> s_addr (network order),
    read as the native little-endian u32 the reference compares; INADDR_NONE on failure."""
    if s is None:
        return INADDR_NONE
    try:
        packed = socket.inet_pton(socket.AF_INET, s)
    except (OSError, ValueError):
        return INADDR_NONE
    return struct.unpack("<I", packed)[0]


def _found(attrs, name, v):
    """_topology_findVertexAttributeString (topology.c:306-328): key exists, value non-empty."""
    col = attrs.get(name)
    if col is None:
        return None
    val = col[v]
    return val if val else None


def _caseeq(a, b):
    """g_ascii_strcasecmp(a, b) == 0."""
    return a.translate(_FOLD) == b.translate(_FOLD)


_FOLD = {c: c + 32 for c in range(ord("A"), ord("Z") + 1)}


def find_attachment_vertex(attrs, n, rnd, ip_hint=None, citycode_hint=None, countrycode_hint=None,
                           geocode_hint=None, type_hint=None):
    """_topology_findAttachmentVertex (topology.c:2245-2366) with the hook of
    topology.c:2094-2216 and the longest-prefix match of topology.c:2218-2243."""
    req_usable, req_ip = False, 0
    if ip_hint is not None:  # topology.c:2258-2264
        ip = string_to_ip(ip_hint)
        if ip not in (INADDR_NONE, INADDR_ANY, INADDR_LOOPBACK):
            req_usable, req_ip = True, ip
    names = ("city_type", "city", "country_type", "country", "geo_type", "geo", "type", "all")
    q = {k: [] for k in names}
    nip = {k: 0 for k in names}
    found_exact = False
    for v in range(n):  # _topology_iterateAllVertices
        city = _found(attrs, "citycode", v)
        country = _found(attrs, "countrycode", v)
        geo = _found(attrs, "geocode", v)
        typ = _found(attrs, "type", v)
        ipstr = _found(attrs, "ip", v)
        city_m = city is not None and citycode_hint is not None and _caseeq(city, citycode_hint)
        country_m = country is not None and countrycode_hint is not None and _caseeq(country, countrycode_hint)
        geo_m = geo is not None and geocode_hint is not None and _caseeq(geo, geocode_hint)
        type_m = typ is not None and type_hint is not None and _caseeq(typ, type_hint)
        usable, vip = False, INADDR_NONE
        if ipstr is not None:
            ip = string_to_ip(ipstr)
            if ip not in (INADDR_NONE, INADDR_ANY, INADDR_LOOPBACK):
                usable, vip = True, ip
        if req_usable and usable and vip == req_ip:  # topology.c:2134-2155
            if not found_exact:
                for k in names:
                    q[k].clear()
            found_exact = True
            q["all"].append(v)
            nip["all"] += 1
        if found_exact:
            continue
        q["all"].append(v)
        nip["all"] += usable
        for k, cond in (("city_type", city_m and type_m), ("city", city_m), ("country_type", country_m and type_m),
                        ("country", country_m), ("geo_type", geo_m and type_m), ("geo", geo_m), ("type", type_m)):
            if cond:
                q[k].append(v)
                nip[k] += usable
    cand, lpm = None, False
    for k in names[:-1]:  # topology.c:2299-2323
        if q[k]:
            cand, lpm = q[k], req_usable and nip[k] > 0
            break
    if cand is None:
        cand, lpm = q["all"], ip_hint is not None and nip["all"] > 0
    assert cand
    if lpm and not found_exact:  # _topology_getLongestPrefixMatch
        best_match, best = 0, -1
        for v in cand:
            ipstr = attrs["ip"][v] if attrs.get("ip") is not None else None
            vip = string_to_ip(ipstr if ipstr else "")
            match = (~(vip ^ req_ip)) & 0xFFFFFFFF
            if match > best_match or best_match == 0:
                best_match, best = match, v
        return best
    d = rnd.next_double()  # topology.c:2333-2339
    x = float((len(cand) - 1) * d)
    chosen = math.floor(x) + (1 if x - math.floor(x) >= 0.5 else 0)  # C round(): half away from zero
    return cand[chosen]
