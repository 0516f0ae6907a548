// engine.hip -- host side of the routing engine (C-ABI in include/shd_route.h).
#include "common.hpp"

#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <sys/mman.h>

#include <thread>
#include "sssp_f64.hpp"
#include "sssp_f64d.hpp"
#include "sssp_k32.hpp"
#include "sssp_batch.hpp"
#include "path_attr.hpp"
#include "sssp_delta.hpp"
#include "direct_fw.hpp"
#include "fw.hpp"

using namespace shd;

// =============================================================================
// Host side
// =============================================================================
// The planner's host workers: one process-wide set, created with the first context that plans
// (KD) and parked on a condition variable between plans, so a plan does not pay ~15 thread
// creations (~0.5 ms).  run(f) starts f on every worker; wait() returns once all of them have
// returned from it.  A plan that finds the set in use (plans on several devices at once)
// starts its own.
struct HostPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, cv_done;
    std::function<void()> fn;
    uint64_t gen = 0;
    int busy = 0;
    bool stop = false;
    explicit HostPool(int n) {
        for (int i = 0; i < n; i++) th.emplace_back([this] { loop(); });
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> l(m);
                cv.wait(l, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
                f = fn;
            }
            f();
            std::lock_guard<std::mutex> l(m);
            if (--busy == 0) cv_done.notify_all();
        }
    }
    void run(std::function<void()> f) {
        std::lock_guard<std::mutex> l(m);
        fn = std::move(f);
        busy = (int)th.size();
        gen++;
        cv.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> l(m);
        cv_done.wait(l, [&] { return busy == 0; });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> l(m);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
};

struct shd_route {
    int device = 0;
    int n = 0, m = 0, nnz = 0;
    int directed = 0, prefer_direct = 0, complete = 0, integer_w = 0, multigraph = 0;
    int self16 = 1;  // every self-loop latency (the table's diagonal) is an integer below 0xFFFF
    double min_w = 0, max_w = 0;
    // device graph
    int* d_row = nullptr; int* d_col = nullptr; double* d_w = nullptr; double* d_r = nullptr;
    int* d_row_in = nullptr; int* d_col_in = nullptr; double* d_w_in = nullptr; double* d_r_in = nullptr;
    double* d_vf = nullptr; double* d_self_w = nullptr; double* d_self_r = nullptr;
    double* d_W = nullptr; double* d_R = nullptr;  // dense direct tables (complete graphs, lazy)
    int* d_err = nullptr;
    char* d_ws = nullptr; size_t ws_stride = 0; int ws_slots = 0;
    bool lds = false;
    size_t lds_bytes = 0;
    // K32 integer fast path (sssp_k32.hpp)
    int k32 = 0, k32_block = 256, k32_bound = 0;
    size_t k32_lds = 0;
    int* d_k32_row_in = nullptr;
    ArcRec* d_arc = nullptr;
    uint16_t* d_k32_col_in = nullptr;
    double* d_k32_r_in = nullptr;
    unsigned long long* d_dbg = nullptr;  // SHD_STAMPS builds: per-source phase stamps
    // KB batched kernel (sssp_batch.hpp) + K2 path attributes (path_attr.hpp)
    int kb = 0, attr = 0, kb_nseg = 0, kb_nhub = 0, kb_npart = 0;
    size_t kb_lds = 0, attr_lds = 0;
    uint32_t* d_kb_arc = nullptr;
    KBSeg* d_kb_seg = nullptr;
    KBHub* d_kb_hub = nullptr;
    int kb_fused = 0, kbf_nrtab = 0, kb_grid_cap = 0, kbf_tcap = 0;  // sssp_batch_kernel<true>: rows in one kernel
    size_t kbf_lds = 0;
    uint32_t* d_kbf_arc = nullptr;    // in-arcs u << 16 | ridx << 8 | w
    double* d_kbf_rtab = nullptr;     // distinct reliabilities
    uint32_t* d_keys = nullptr;     // key rows scratch (ns x n u32), grown on demand
    size_t keys_cap = 0;
    // KD delta-stepping kernel (sssp_delta.hpp)
    int kd = 0, kd_block = 1024, kd_slots = 0, kd_delta = 1, kd_qcap = 0;
    size_t kd_lds = 0, kd_stride = 0;
    // the planner's unseeded hub rows on 256-thread contexts (C3): 1024-thread workgroups,
    // one row per CU, cut the latency of that launch (each row is unseeded and alone)
    int kd_hub_block = 0, kd_hub_qcap = 0, kd_hub_delta = 1;
    size_t kd_hub_lds = 0;
    int* d_kd_lstart = nullptr;   // light in-CSR offsets (n+1)
    uint32_t* d_kd_orec = nullptr;  // out-arc records v | w << 16
    uint16_t* d_kd_oridx = nullptr; // rtab index per out-arc
    uint32_t* d_kd_lrec = nullptr;  // light in-arc records (2 x u32 per arc)
    double* d_kd_rtab = nullptr;    // distinct reliabilities
    int kd_nlight = 0, kd_nrtab = 1, kd_walk = 0, kd_packed = 0, kd_fused = 0;
    int has_vf = 0;  // some vertex has a packet-loss factor (else f_v is absent everywhere)
    int vf_lossy = 0;  // some vertex factor is not exactly 1.0 (else every present f_v is a no-op)
    int kd_rone = -1;  // rtab index of exactly 1.0 (-1: none)
    char* d_kd_ws = nullptr;
    int* d_fwflag = nullptr;  // K4: per pivot, its closed tile is published (fw_restp_kernel)
    unsigned long long* d_kd_stats = nullptr;  // KD liveness counters (shd_route_kd_stats)
    int* d_kd_next = nullptr;  // KD source queue counter
    // host copies for seeded planning (shd_route_plan_*): out-CSR, rtab index per arc and
    // the landmark closeness of every vertex (computed on the first plan)
    std::vector<int> h_row, h_col;
    std::vector<double> h_w;
    std::vector<uint16_t> h_ridx;
    std::vector<double> close;
    // landmark rows (planner): the most central vertices' distances and tie-rule parent
    // records computed on the host, uploaded as seed rows for the plan's roots
    std::vector<int> lm_v;
    std::vector<uint16_t> lm_hd;  // landmark l's u16 distance of v at [l * lm_rs + v] (0xFFFF: unreached)
    std::vector<uint32_t> lm_hp;  // and its parent record
    long long lm_rs = 0;
    uint16_t* d_lm_drow = nullptr;  // the landmark rows in the row-store format (device)
    uint32_t* d_lm_prow = nullptr;
    char* d_hub_ws = nullptr;       // the planner's hub-row launch scratch (kept: a free costs a sync)
    size_t hub_ws_bytes = 0;
    int sel = 0;  // selected SSSP kernel: 0 f64, 1 K32, 2 KB+K2, 4 KD, 5 KF (3: the retired K16)
    // KF (fractional latencies, LDS-resident f64 delta-stepping)
    int kf_block = 0, kf_slots = 0;
    size_t kf_lds = 0;
    double kf_delta = 1.0;
    int kf_nrtab = 0;
    int kf_h = 0;             // KFH: the per-vertex state in a per-workgroup HBM slice (n > ~12k)
    char* d_kf_ws = nullptr;
    size_t kf_ws_stride = 0;
    uint8_t* d_kf_rix = nullptr;
    uint32_t* d_kf_opk = nullptr;  // KF packed arcs (head | k << 16, weight k / kf_wscale), or null
    uint32_t* d_kf_ipk = nullptr;
    double kf_wscale = 0.0;
    double* d_kf_rtab = nullptr;
    // K4 (fw.hpp): u16 all-pairs table + dense u16 weights, Np x Np (Np = n rounded to 64)
    uint16_t* d_fwD = nullptr;
    uint32_t* d_fwinl = nullptr;  // K4 parent search: sorted in-arc keys per vertex (np x np)
    uint16_t* d_fwpos = nullptr;  // and the start index per small threshold (n x FW_X)
    uint32_t* d_fwkey = nullptr;
    uint8_t* d_fwrix = nullptr;  // K4 rows: reliability index of each arc (dense n x n u8)
    double* d_fwrtab = nullptr;  // and the distinct reliabilities (fw_nrtab <= 255; 0: dense R reads)
    int fw_pk = 0;               // K4 in-list keys carry the parent arc's reliability index
    int fw_nrtab = 0;
    size_t fwkey_cap = 0;
    int fw_np = 0, fw_ready = 0;
    uint64_t device_bytes = 0;
    // host copies needed for lazy dense build
    std::vector<int32_t> e_src, e_dst;
    std::vector<double> e_lat, e_rel;
    std::vector<void*> allocs;
};

namespace {

HostPool* host_pool();
int plan_threads();
std::mutex g_pool_mu, g_pool_use;
std::unique_ptr<HostPool> g_pool;

// KD workgroup sizes: f(std::integral_constant<int, B>) for the runtime block size
template <typename F>
auto kd_dispatch(int blk, F f) {
    switch (blk) {
        case 1024: return f(std::integral_constant<int, 1024>{});
        case 768: return f(std::integral_constant<int, 768>{});
        case 512: return f(std::integral_constant<int, 512>{});
        default: return f(std::integral_constant<int, 256>{});
    }
}

int hip_check(hipError_t e) { return e == hipSuccess ? SHD_ROUTE_OK : SHD_ROUTE_EDEVICE; }

template <typename T>
int upload(shd_route* c, T** dptr, const std::vector<T>& h) {
    size_t bytes = sizeof(T) * (h.empty() ? 1 : h.size());
    if (hipMalloc((void**)dptr, bytes) != hipSuccess) return SHD_ROUTE_ENOMEM;
    c->allocs.push_back(*dptr);
    c->device_bytes += bytes;
    if (!h.empty() && hipMemcpy(*dptr, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    return SHD_ROUTE_OK;
}

DevGraph dev_graph(const shd_route* c) {
    DevGraph g;
    g.n = c->n; g.prefer_direct = c->prefer_direct;
    g.row = c->d_row; g.col = c->d_col; g.w = c->d_w; g.r = c->d_r;
    g.row_in = c->d_row_in; g.col_in = c->d_col_in; g.w_in = c->d_w_in; g.r_in = c->d_r_in;
    g.vf = c->d_vf; g.self_w = c->d_self_w; g.self_r = c->d_self_r;
    return g;
}

// Build a CSR (rows by `key`, columns by `other`), arcs sorted by (row, col, eid).
void build_csr(int n, const std::vector<int32_t>& rows, const std::vector<int32_t>& cols,
               const std::vector<int32_t>& eids, const std::vector<double>& lat,
               const std::vector<double>& rel, std::vector<int>& row, std::vector<int>& col,
               std::vector<double>& w, std::vector<double>& r, std::vector<int>* eid_out = nullptr) {
    const size_t k = rows.size();
    std::vector<size_t> idx(k);
    std::iota(idx.begin(), idx.end(), 0);
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
        if (rows[a] != rows[b]) return rows[a] < rows[b];
        if (cols[a] != cols[b]) return cols[a] < cols[b];
        return eids[a] < eids[b];
    });
    row.assign(n + 1, 0);
    col.resize(k); w.resize(k); r.resize(k);
    for (size_t q = 0; q < k; q++) {
        size_t a = idx[q];
        row[rows[a] + 1]++;
        col[q] = cols[a];
        w[q] = lat[eids[a]];
        r[q] = rel[eids[a]];
    }
    if (eid_out) {
        eid_out->resize(k);
        for (size_t q = 0; q < k; q++) (*eid_out)[q] = eids[idx[q]];
    }
    for (int v = 0; v < n; v++) row[v + 1] += row[v];
}

bool strongly_connected(int n, const std::vector<int>& row, const std::vector<int>& col,
                        const std::vector<int>& row_in, const std::vector<int>& col_in) {
    auto reach_all = [&](const std::vector<int>& R, const std::vector<int>& Cc) {
        std::vector<char> seen(n, 0);
        std::vector<int> st{0};
        seen[0] = 1;
        int cnt = 1;
        while (!st.empty()) {
            int u = st.back(); st.pop_back();
            for (int a = R[u]; a < R[u + 1]; a++)
                if (!seen[Cc[a]]) { seen[Cc[a]] = 1; cnt++; st.push_back(Cc[a]); }
        }
        return cnt == n;
    };
    return reach_all(row, col) && reach_all(row_in, col_in);
}

int alloc_ws(shd_route* c) {
    // per-source state in HBM when it cannot live in LDS
    StateLayout L = StateLayout::make(c->n);
    c->ws_stride = a16(L.total) + 256;
    c->ws_slots = 1024;  // 256 CUs x 4 workgroups
    size_t bytes = c->ws_stride * (size_t)c->ws_slots;
    if (hipMalloc((void**)&c->d_ws, bytes) != hipSuccess) return SHD_ROUTE_ENOMEM;
    c->allocs.push_back(c->d_ws);
    return SHD_ROUTE_OK;
}

int ensure_dense(shd_route* c) {
    if (c->d_W) return SHD_ROUTE_OK;
    const size_t nn = (size_t)c->n * c->n;
    std::vector<double> W(nn, NAN), R(nn, NAN);
    // igraph_get_eid on a simple graph returns the unique edge; for parallel edges we
    // keep the lowest edge id (documented deviation, SURVEY hazard H3).
    for (int e = c->m - 1; e >= 0; e--) {
        int a = c->e_src[e], b = c->e_dst[e];
        W[(size_t)a * c->n + b] = c->e_lat[e];
        R[(size_t)a * c->n + b] = c->e_rel[e];
        if (!c->directed) {
            W[(size_t)b * c->n + a] = c->e_lat[e];
            R[(size_t)b * c->n + a] = c->e_rel[e];
        }
    }
    int rc = upload(c, &c->d_W, W);
    if (rc) return rc;
    return upload(c, &c->d_R, R);
}

// Host Dijkstra (exact for integer weights) -> eccentricity of vertex 0.
double ecc0(int n, const std::vector<int>& row, const std::vector<int>& col, const std::vector<double>& w) {
    std::vector<double> d(n, INFINITY);
    std::vector<std::pair<double, int>> h;
    d[0] = 0;
    h.push_back({0.0, 0});
    auto cmp = [](const std::pair<double, int>& a, const std::pair<double, int>& b) { return a.first > b.first; };
    while (!h.empty()) {
        std::pop_heap(h.begin(), h.end(), cmp);
        auto [du, u] = h.back();
        h.pop_back();
        if (du > d[u]) continue;
        for (int a = row[u]; a < row[u + 1]; a++) {
            double nd = du + w[a];
            if (nd < d[col[a]]) { d[col[a]] = nd; h.push_back({nd, col[a]}); std::push_heap(h.begin(), h.end(), cmp); }
        }
    }
    double mx = 0;
    for (double x : d) mx = std::max(mx, x);
    return mx;
}

// K32 eligibility + device arrays: in-rows sorted by (-w, u, eid); out-arc records carry
// the slot of the same arc in its head's in-row.
int prepare_k32(shd_route* c, const std::vector<int>& row, const std::vector<int>& col,
                const std::vector<double>& w, const std::vector<int>& eid, const std::vector<int>& row_in,
                const std::vector<int>& col_in, const std::vector<double>& w_in) {
    const int n = c->n;
    const char* force = getenv("SHD_ROUTE_KERNEL");
    if (force && (!strcmp(force, "f64") || !strcmp(force, "kf"))) return SHD_ROUTE_OK;
    if (force && !*force) force = nullptr;
    if (!c->integer_w || n > 65535 || c->multigraph) return SHD_ROUTE_OK;
    for (int a = 0; a < c->nnz; a++) if (w[a] > 65535.0) return SHD_ROUTE_OK;
    std::vector<int> indeg(n, 0);
    for (int a = 0; a < c->nnz; a++) indeg[col[a]]++;
    for (int v = 0; v < n; v++) if (indeg[v] > 65535) return SHD_ROUTE_OK;
    const double bound = ecc0(n, row, col, w) + ecc0(n, row_in, col_in, w_in);
    if (!(bound < 65535.0)) return SHD_ROUTE_OK;
    const K32Layout L = K32Layout::make(n);
    size_t lds = 0;
    int block = 0;
    for (int b : {256, 512, 1024}) {
        size_t sm = b == 256 ? k32_small_bytes<256>() : b == 512 ? k32_small_bytes<512>() : k32_small_bytes<1024>();
        size_t tot = sm + L.total;
        if (tot > kLdsBudget) continue;
        int per_cu = (int)(kLdsBudget / tot);
        if (per_cu * (b / 64) >= 16 || b == 1024) { block = b; lds = tot; break; }
    }
    // in-rows: every out-arc a = (u -> v) appears in v's in-row
    std::vector<int> irow(n + 1, 0);
    for (int a = 0; a < c->nnz; a++) irow[col[a] + 1]++;
    for (int v = 0; v < n; v++) irow[v + 1] += irow[v];
    std::vector<int> order(c->nnz), fill(irow.begin(), irow.end() - 1), src_of(c->nnz);
    for (int u = 0; u < n; u++)
        for (int a = row[u]; a < row[u + 1]; a++) { src_of[a] = u; order[fill[col[a]]++] = a; }
    for (int v = 0; v < n; v++)
        std::sort(order.begin() + irow[v], order.begin() + irow[v + 1], [&](int x, int y) {
            if (w[x] != w[y]) return w[x] > w[y];
            if (src_of[x] != src_of[y]) return src_of[x] < src_of[y];
            return eid[x] < eid[y];
        });
    std::vector<ArcRec> arcs(c->nnz);
    std::vector<uint16_t> cin(c->nnz);
    std::vector<double> rin(c->nnz);
    for (int v = 0; v < n; v++)
        for (int q = irow[v]; q < irow[v + 1]; q++) {
            int a = order[q];
            arcs[a].rslot = (uint16_t)(q - irow[v]);
            cin[q] = (uint16_t)src_of[a];
            rin[q] = c->e_rel[eid[a]];
        }
    for (int a = 0; a < c->nnz; a++) {
        arcs[a].col = (uint16_t)col[a];
        arcs[a].w = (uint16_t)w[a];
        arcs[a].pad = 0;
    }
    int rc = upload(c, &c->d_k32_row_in, irow);
    if (!rc) rc = upload(c, &c->d_arc, arcs);
    if (!rc) rc = upload(c, &c->d_k32_col_in, cin);
    if (!rc) rc = upload(c, &c->d_k32_r_in, rin);
    if (rc) return rc;
    c->k32_bound = (int)bound;
    const bool want_k32 = !force || !strcmp(force, "k32") || !strcmp(force, "auto");
    (void)0;
    const bool want_kb = !force || !strcmp(force, "kb") || !strcmp(force, "auto");
    if (block && want_k32) {
        const void* fn = block == 256 ? (const void*)sssp_k32_kernel<256>
                       : block == 512 ? (const void*)sssp_k32_kernel<512> : (const void*)sssp_k32_kernel<1024>;
        rc = hip_check(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        if (rc) return rc;
        c->k32 = 1; c->k32_block = block; c->k32_lds = lds;
    }
    // K2 path attributes: relv f64 + parent u16 per vertex in LDS
    const AttrLayout AL = AttrLayout::make(n);
    if (AL.total <= kLdsBudget) {
        c->attr = 1;
        c->attr_lds = AL.total;
        rc = hip_check(hipFuncSetAttribute((const void*)path_attr_kernel<256>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)AL.total));
        if (rc) return rc;
    }
    // packed in-arcs (u << 16 | w), rows sorted by (-w, u, eid): KB
    {
        std::vector<uint32_t> packed(((size_t)c->nnz + 3) / 4 * 4, 0u);
        for (int q = 0; q < c->nnz; q++) packed[q] = ((uint32_t)cin[q] << 16) | (uint32_t)w[order[q]];
        rc = upload(c, &c->d_kb_arc, packed);
        if (rc) return rc;
    }
    // KD delta-stepping: bucket width ~ the 15th (22nd) percentile of arc latencies (>= 1),
    // so ~15% (22%) of arcs are light; light in-arcs are the tail of each (-w)-sorted in-row
    const bool want_kd = !force || !strcmp(force, "kd") || !strcmp(force, "auto");
    if (want_kd && c->nnz > 0) {
        // one 1024-thread workgroup per CU when dist fills the LDS; smaller graphs run several
        // 256-thread workgroups (sources) per CU
        int blk = n > 16384 ? 1024 : 256;
        if (const char* e = getenv("SHD_ROUTE_KDBLOCK")) {
            const int b = atoi(e);
            if (b == 256 || b == 1024) blk = b;  // (512/768: the phase-A ring sizing assumes 256 or 1024)
        }
        int delta = 1;
        if (const char* e = getenv("SHD_ROUTE_DELTA")) delta = std::max(1, atoi(e));
        else {
            // 1024-thread rows: the 15th percentile (38 on C4; seeded rows expand few vertices
            // per bucket, so fewer, wider buckets pay: C4 57 -> 53 ms from the 6th percentile's
            // 15.  Round-5 sweep, two reps each: 30/35/38-40/50/60 = 41.23-41.55/41.05/
            // 41.04-41.40/41.90/42.92 ms).  256-thread rows (three compute waves) take the
            // 22nd (55 on C3: 1.986 ms; 45/65/80 = 2.004-2.017/1.991/2.012-2.017 ms)
            std::vector<int> ws(c->nnz);
            for (int a = 0; a < c->nnz; a++) ws[a] = (int)w[a];
            const size_t k = (size_t)c->nnz * (blk >= 1024 ? 15 : 22) / 100;
            std::nth_element(ws.begin(), ws.begin() + k, ws.end());
            delta = std::max(1, ws[k]);
        }
        const size_t base = kd_dispatch(blk, [&](auto B) { return kd_lds_bytes<decltype(B)::value>(n, 0); });
        if (base + 2 * 512 <= kLdsBudget) {
            // work queue: the rest of the CU's LDS at one workgroup per CU (large n), else
            // enough for a few workgroups per CU
            int qcap;
            if (blk < 768) {
                // four 256-thread workgroups per CU: the queue takes what is left of a quarter
                const size_t quarter = kLdsBudget / 4;
                qcap = base + 64 + 2 * 512 <= quarter ? (int)std::min<size_t>((size_t)n, (quarter - base - 64) / 2)
                                                      : std::min(n, std::max(1024, n / 2));
            } else qcap = (int)std::min<size_t>((size_t)n, (kLdsBudget - base - 64) / 2);
            if (const char* e = getenv("SHD_ROUTE_QCAP")) qcap = std::min(qcap, std::max(64, atoi(e)));
            qcap &= ~7;
            const size_t lds = kd_dispatch(blk, [&](auto B) { return kd_lds_bytes<decltype(B)::value>(n, qcap); });
            int maxdeg = 0;
            for (int v = 0; v < n; v++) maxdeg = std::max(maxdeg, row[v + 1] - row[v]);
            // reliability table: every distinct 1-loss value (exact bits), indexed by u16
            std::vector<double> rtab;
            std::vector<uint16_t> ridx_out(c->nnz);
            bool rtab_ok = true;
            {
                std::vector<std::pair<uint64_t, int>> keyed(c->nnz);
                for (int a = 0; a < c->nnz; a++) {
                    uint64_t bits;
                    std::memcpy(&bits, &c->e_rel[eid[a]], 8);
                    keyed[a] = {bits, a};
                }
                std::sort(keyed.begin(), keyed.end());
                for (int q = 0; q < c->nnz && rtab_ok; q++) {
                    if (q == 0 || keyed[q].first != keyed[q - 1].first) {
                        double x;
                        std::memcpy(&x, &keyed[q].first, 8);
                        rtab.push_back(x);
                        if (rtab.size() > 65535) rtab_ok = false;
                    }
                    ridx_out[keyed[q].second] = (uint16_t)(rtab.size() - 1);
                }
            }
            if (lds <= kLdsBudget && maxdeg <= 65535 && rtab_ok) {
                // out-arc records v | w << 16 (| ridx << 24 when packed); light in-CSR records
                // {u | w << 16, ridx}, light = w < delta.  Fused parents (found during the
                // expansion, 32-bit tie keys) need an undirected graph and packed records
                // (w < 256, <= 256 reliabilities); otherwise the in-CSR holds every in-arc and
                // phase B finds every parent.
                std::vector<uint32_t> orec(c->nnz);
                int maxw = 0;
                for (int a = 0; a < c->nnz; a++) maxw = std::max(maxw, (int)w[a]);
                bool packed = maxw < 256 && rtab.size() <= 256;
                if (const char* e = getenv("SHD_ROUTE_KDPACK")) packed = packed && atoi(e) != 0;
                for (int a = 0; a < c->nnz; a++)
                    orec[a] = (uint32_t)col[a] | ((uint32_t)w[a] << 16) | (packed ? (uint32_t)ridx_out[a] << 24 : 0u);
                c->kd_packed = packed ? 1 : 0;
                const bool fused = !c->directed && packed;
                c->kd_fused = fused ? 1 : 0;
                std::vector<int> lrow(n + 1, 0);
                std::vector<uint32_t> lrec;
                for (int v = 0; v < n; v++) {
                    for (int q = irow[v]; q < irow[v + 1]; q++) {
                        const int a = order[q];
                        if (fused && (int)w[a] >= delta) continue;
                        lrec.push_back((uint32_t)cin[q] | ((uint32_t)w[a] << 16));
                        lrec.push_back(ridx_out[a]);
                    }
                    lrow[v + 1] = (int)(lrec.size() / 2);
                }
                if (lrec.empty()) lrec.assign(2, 0u);
                c->h_row = row; c->h_col = col; c->h_w = w; c->h_ridx = ridx_out;
                rc = upload(c, &c->d_kd_lstart, lrow);
                if (!rc) rc = upload(c, &c->d_kd_orec, orec);
                if (!rc) rc = upload(c, &c->d_kd_oridx, ridx_out);
                if (!rc) rc = upload(c, &c->d_kd_lrec, lrec);
                if (!rc) rc = upload(c, &c->d_kd_rtab, rtab);
                if (rc) return rc;
                c->kd_nlight = lrow[n];
                c->kd_nrtab = std::max<int>(1, (int)rtab.size());
                for (int q = 0; q < (int)rtab.size(); q++)
                    if (rtab[q] == 1.0) c->kd_rone = q;
                // 16 waves per CU: 4 per SIMD at <= 128 VGPRs (amdgpu_waves_per_eu(4))
                const int per_cu = std::max(1, std::min((int)(kLdsBudget / lds), 1024 / blk));
                c->kd_slots = 256 * per_cu;
                // tests cap the grid so that every workgroup runs many sources in turn
                if (const char* e = getenv("SHD_ROUTE_KDGRID")) c->kd_slots = std::max(1, std::min(c->kd_slots, atoi(e)));
                c->kd_stride = kd_ws_stride(n);
                if (hipMalloc((void**)&c->d_kd_ws, c->kd_stride * (size_t)c->kd_slots) != hipSuccess)
                    return SHD_ROUTE_ENOMEM;
                c->allocs.push_back(c->d_kd_ws);
                if (hipMalloc((void**)&c->d_kd_next, sizeof(int)) != hipSuccess) return SHD_ROUTE_ENOMEM;
                c->allocs.push_back(c->d_kd_next);
                if (hipMalloc((void**)&c->d_kd_stats, sizeof(unsigned long long) * 4) != hipSuccess ||
                    hipMemset(c->d_kd_stats, 0, sizeof(unsigned long long) * 4) != hipSuccess)
                    return SHD_ROUTE_ENOMEM;
                c->allocs.push_back(c->d_kd_stats);
                for (int pk = 0; pk < 2 && !rc; pk++) {
                    const void* fn = kd_dispatch(blk, [&](auto B) {
                        return pk ? (const void*)kd_plan_rows_kernel<decltype(B)::value>
                                  : (const void*)sssp_delta_kernel<decltype(B)::value>;
                    });
                    rc = hip_check(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                }
                if (rc) return rc;
                c->kd = 1; c->kd_block = blk; c->kd_lds = lds; c->kd_delta = delta; c->kd_qcap = qcap;
                if (blk < 1024 && !getenv("SHD_ROUTE_DELTA") && !getenv("SHD_ROUTE_QCAP")) {
                    // hub rows in 1024-thread workgroups: that block's queue and bucket width
                    const size_t hb = kd_lds_bytes<1024>(n, 0);
                    if (hb + 2 * 512 <= kLdsBudget) {
                        const int hq = (int)std::min<size_t>((size_t)n, (kLdsBudget - hb - 64) / 2) & ~7;
                        const size_t hl = kd_lds_bytes<1024>(n, hq);
                        std::vector<int> ws2(c->nnz);
                        for (int a = 0; a < c->nnz; a++) ws2[a] = (int)w[a];
                        const size_t k12 = (size_t)c->nnz * 12 / 100;
                        std::nth_element(ws2.begin(), ws2.begin() + k12, ws2.end());
                        if (hl <= kLdsBudget &&
                            hipFuncSetAttribute((const void*)kd_plan_rows_kernel<1024>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)hl) == hipSuccess) {
                            c->kd_hub_block = 1024; c->kd_hub_qcap = hq; c->kd_hub_lds = hl;
                            // (the light in-CSR above holds the in-arcs with w < delta, and a
                            // row's fused parents are exact only if its bucket width is at most
                            // that: the hub rows' 12th percentile never exceeds the context's)
                            c->kd_hub_delta = std::min(delta, std::max(1, ws2[k12]));
                        }
                    }
                    if (const char* e = getenv("SHD_ROUTE_HUB1024")) if (atoi(e) == 0) c->kd_hub_block = 0;
                }
                c->kd_walk = kd_dispatch(blk, [&](auto B) { return kd_walk_fits<decltype(B)::value>(n, qcap, c->kd_nrtab); }) ? 1 : 0;
                if (const char* e = getenv("SHD_ROUTE_KDWALK")) c->kd_walk = c->kd_walk && atoi(e) != 0;
            }
        }
    }
    // KB batched kernel: segments of <= KB_SEG in-arcs, hub rows split
    if (c->attr && want_kb) {
        std::vector<KBSeg> segs;
        std::vector<KBHub> hubs;
        int npart = 0;
        for (int v = 0; v < n; v++) {
            const int a0 = irow[v], a1 = irow[v + 1];
            if (a1 - a0 <= KB_SEG) { segs.push_back({v, a0, a1, -1}); continue; }
            KBHub h{v, npart, 0, 0};
            for (int a = a0; a < a1; a += KB_SEG) segs.push_back({v, a, std::min(a1, a + KB_SEG), npart++});
            h.p1 = npart;
            hubs.push_back(h);
        }
        // equal-length segments side by side: a wave's lanes finish their rows together
        std::stable_sort(segs.begin(), segs.end(),
                         [](const KBSeg& x, const KBSeg& y) { return (x.a1 - x.a0) > (y.a1 - y.a0); });
        // thread t takes segments t, t + KB_BLOCK, ...: a sweep lasts as long as the wave
        // whose lanes' longest segments add up most.  Each block of KB_BLOCK segments may
        // run long->short or short->long over the threads; pick the directions with the
        // smallest such wave time (C2: 29 -> 22 arc steps; the mean is 20)
        {
            const int nb = ((int)segs.size() + KB_BLOCK - 1) / KB_BLOCK;
            constexpr int kWaves = KB_BLOCK / 64;
            auto cost = [&](unsigned dirs) {
                int wt[kWaves] = {0};
                for (int b = 0; b < nb; b++) {
                    const int k0 = b * KB_BLOCK, cnt = std::min((int)segs.size() - k0, KB_BLOCK);
                    for (int w = 0; w < kWaves; w++) {
                        int mx = 0;
                        for (int l = w * 64; l < std::min(cnt, w * 64 + 64); l++) {
                            const KBSeg& sg = segs[k0 + (((dirs >> b) & 1u) ? cnt - 1 - l : l)];
                            mx = std::max(mx, sg.a1 - sg.a0);
                        }
                        wt[w] += mx;
                    }
                }
                return *std::max_element(wt, wt + kWaves);
            };
            unsigned best = 0;
            if (nb <= 12) {
                int bc = cost(0);
                for (unsigned d = 1; d < (1u << nb); d++) {
                    const int c2 = cost(d);
                    if (c2 < bc) { bc = c2; best = d; }
                }
            }
            for (int b = 0; b < nb; b++)
                if ((best >> b) & 1u) {
                    const int k0 = b * KB_BLOCK, cnt = std::min((int)segs.size() - k0, KB_BLOCK);
                    std::reverse(segs.begin() + k0, segs.begin() + k0 + cnt);
                }
        }
        const KBLayout KL = KBLayout::make(n, c->nnz, npart);
        const size_t kbl = kKBSmall + KL.total;
        if (kbl <= kLdsBudget) {
            rc = upload(c, &c->d_kb_seg, segs);
            if (!rc && !hubs.empty()) rc = upload(c, &c->d_kb_hub, hubs);
            if (!rc) rc = hip_check(hipFuncSetAttribute((const void*)sssp_batch_kernel,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kbl));
            if (rc) return rc;
            c->kb = 1; c->kb_lds = kbl; c->kb_nseg = (int)segs.size(); c->kb_nhub = (int)hubs.size();
            c->kb_npart = npart;
            // fused rows (no key rows, no K2): records u << 16 | ridx << 8 | w need w < 256 and
            // <= 254 distinct reliabilities; parent records of <= KB_RIT segments per thread
            int maxw = 0;
            for (int a = 0; a < c->nnz; a++) maxw = std::max(maxw, (int)w[a]);
            std::map<uint64_t, int> rix;
            for (int q = 0; q < c->nnz; q++) {
                uint64_t bits;
                std::memcpy(&bits, &rin[q], 8);
                rix.emplace(bits, 0);
            }
            // staged targets: as many as the rest of the LDS holds (one chunk when nt <= n)
            const size_t fb0 = kKBSmall + KBLayout::make(n, c->nnz, npart, true, 0).total;
            int tcap = fb0 < kLdsBudget ? (int)std::min<size_t>((size_t)n, (kLdsBudget - fb0 - 64) / 4) : 0;
            tcap = tcap >= 64 ? (tcap & ~63) : 0;
            const size_t fbl = kKBSmall + KBLayout::make(n, c->nnz, npart, true, tcap).total;
            bool fuse = maxw < 256 && rix.size() <= (size_t)KB_ONE && (int)segs.size() <= KB_RIT * KB_BLOCK &&
                        (int)hubs.size() <= KB_BLOCK && c->nnz < 0xFFFF && KB_SRC * n <= KB_CV * KB_BLOCK && npart < 0xFFFF && tcap >= 64 &&
                        fbl <= kLdsBudget;
            if (const char* e = getenv("SHD_ROUTE_KBTCAP")) tcap = std::max(64, std::min(tcap, atoi(e)) & ~63);
            if (const char* e = getenv("SHD_ROUTE_KBFUSE")) fuse = fuse && atoi(e) != 0;
            if (fuse) {
                std::vector<double> rtab;
                for (auto& kv : rix) {
                    kv.second = (int)rtab.size();
                    double x;
                    std::memcpy(&x, &kv.first, 8);
                    rtab.push_back(x);
                }
                std::vector<uint32_t> farc(((size_t)c->nnz + 3) / 4 * 4, 0u);
                for (int q = 0; q < c->nnz; q++) {
                    uint64_t bits;
                    std::memcpy(&bits, &rin[q], 8);
                    farc[q] = ((uint32_t)cin[q] << 16) | ((uint32_t)rix[bits] << 8) | (uint32_t)w[order[q]];
                }
                rc = upload(c, &c->d_kbf_arc, farc);
                if (!rc) rc = upload(c, &c->d_kbf_rtab, rtab);
                if (!rc) rc = hip_check(hipFuncSetAttribute((const void*)sssp_batch_rows_kernel,
                                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)fbl));
                if (rc) return rc;
                c->kb_fused = 1; c->kbf_lds = fbl; c->kbf_nrtab = (int)rtab.size(); c->kbf_tcap = tcap;
            }
            // tests cap the grid so that every workgroup runs several batches in turn
            if (const char* e = getenv("SHD_ROUTE_KBGRID")) c->kb_grid_cap = std::max(1, atoi(e));
        }
    }
    c->sel = c->kb ? 2 : c->kd ? 4 : c->k32 ? 1 : 0;  // KB (C2-class), else KD (C3/C4-class)
    return SHD_ROUTE_OK;
}

DevDelta kd_args(const shd_route* c) {
    DevDelta k;
    k.n = c->n; k.nw = (c->n + 63) / 64; k.bound = c->k32_bound; k.delta = c->kd_delta;
    k.fused = c->kd_fused; k.rc = c->kd_qcap;
    k.row = c->d_row; k.orec = c->d_kd_orec; k.oridx = c->d_kd_oridx;
    k.nnz = c->nnz; k.lrow = c->d_kd_lstart; k.lrec = reinterpret_cast<const uint2*>(c->d_kd_lrec); k.nlight = c->kd_nlight;
    k.rtab = c->d_kd_rtab; k.nrtab = c->kd_nrtab; k.rone = c->kd_rone; k.walk = c->kd_walk; k.packed = c->kd_packed;
    k.vf = c->d_vf; k.self_w = c->d_self_w; k.self_r = c->d_self_r; k.dbg = c->d_dbg; k.dflags = 0;
    // a factor of exactly 1.0 multiplies as a no-op: KD reads vf only where one is not
    k.has_vf = c->vf_lossy;
#ifdef SHD_STAMPS
    if (const char* e = getenv("SHD_ROUTE_DFLAGS")) k.dflags = atoi(e);
#endif
    k.seed_drop = 0;
    if (const char* e = getenv("SHD_ROUTE_SEEDDROP")) k.seed_drop = atoi(e) & ~1;

    k.jobs = nullptr; k.drow = nullptr; k.drow_out = nullptr; k.prow = nullptr; k.rstride = 0; k.evcap = c->n;
    k.done = nullptr;
    // tests shrink the tie-event list to force the unseeded rerun of overflowing rows
    if (const char* e = getenv("SHD_ROUTE_EVCAP")) k.evcap = std::max(0, std::min(c->n, atoi(e)));
    k.next = nullptr;
    k.stats = c->d_kd_stats;
    return k;
}

// one KD launch of ns sources (k.jobs: planned jobs, else d_src); `next` is zeroed
int kd_launch(shd_route* c, DevDelta k, int* next, const int32_t* d_src, int ns, const int32_t* d_tgt, int nt,
              int64_t ld, double* d_lat, double* d_rel, double* d_row_min, hipStream_t st, bool planner = false,
              char* ws = nullptr, int max_grid = 0, bool hub = false) {
    if (ns <= 0) return SHD_ROUTE_OK;
    k.next = next;
    if (!ws) ws = c->d_kd_ws;
    const int grid = std::min(ns, max_grid > 0 ? std::min(max_grid, c->kd_slots) : c->kd_slots);
    // (hub: the planner's rows in 1024-thread workgroups where the context's are smaller)
    const bool big = hub && planner && c->kd_hub_block > 0;
    size_t lds = c->kd_lds;
    if (big) { k.rc = c->kd_hub_qcap; k.delta = c->kd_hub_delta; lds = c->kd_hub_lds; }
    kd_dispatch(big ? c->kd_hub_block : c->kd_block, [&](auto B) {
        constexpr int b = decltype(B)::value;
        if (planner)
            hipLaunchKernelGGL(kd_plan_rows_kernel<b>, dim3(grid), dim3(b), lds, st, k, d_src, ns, d_tgt,
                               nt, (long long)ld, d_lat, d_rel, d_row_min, c->d_err, ws, c->kd_stride);
        else
            hipLaunchKernelGGL(sssp_delta_kernel<b>, dim3(grid), dim3(b), c->kd_lds, st, k, d_src, ns, d_tgt,
                               nt, (long long)ld, d_lat, d_rel, d_row_min, c->d_err, ws, c->kd_stride);
        return 0;
    });
    return hip_check(hipGetLastError());
}

int take_err(shd_route* c) {
    int h = 0;
    if (hipMemcpy(&h, c->d_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (h) {
        int z = 0;
        if (hipMemcpy(c->d_err, &z, sizeof(int), hipMemcpyHostToDevice) != hipSuccess) return SHD_ROUTE_EDEVICE;
    }
    return h;
}

}  // namespace

extern "C" {

const char* shd_route_strerror(int code) {
    switch (code) {
        case SHD_ROUTE_OK: return "success";
        case SHD_ROUTE_EINVAL: return "invalid argument or topology failed validation";
        case SHD_ROUTE_ENOMEM: return "out of memory";
        case SHD_ROUTE_EDEVICE: return "HIP device error";
        case SHD_ROUTE_ENOEDGE: return "path hop without an edge (missing self-loop?)";
        case SHD_ROUTE_EUNREACH: return "target unreachable";
        case SHD_ROUTE_EUNSUPPORTED: return "unsupported request";
        default: return "unknown error";
    }
}

// KF eligibility + device arrays (graphs the integer kernels do not take): per in-arc index
// of its 1 - loss in a table of the distinct values, bucket width, block size.  Fits when
// the per-source LDS state does and every thread holds at most 16 vertices in the level
// passes (n <= 16 B); above that KFH (n <= 65535: the ring is u16), one 1024-thread
// workgroup per CU with its vertex state in an HBM slice (C4f: 550 KB per slice).
int prepare_kf(shd_route* c, const std::vector<int>& col, const std::vector<double>& w, const std::vector<int>& row_in,
               const std::vector<int>& col_in, const std::vector<double>& w_in, const std::vector<double>& r_in) {
    const int n = c->n;
    const char* force = getenv("SHD_ROUTE_KERNEL");
    if (force && *force && strcmp(force, "kf") && strcmp(force, "auto")) return SHD_ROUTE_OK;
    if (c->nnz == 0 || n > 65535) return SHD_ROUTE_OK;
    std::vector<double> rtab;
    std::vector<uint8_t> rix(c->nnz);
    {
        std::vector<std::pair<uint64_t, int>> keyed(c->nnz);
        for (int a = 0; a < c->nnz; a++) {
            uint64_t bits;
            std::memcpy(&bits, &r_in[a], 8);
            keyed[a] = {bits, a};
        }
        std::sort(keyed.begin(), keyed.end());
        for (int q = 0; q < c->nnz; q++) {
            if (q == 0 || keyed[q].first != keyed[q - 1].first) {
                if ((int)rtab.size() == 254) return SHD_ROUTE_OK;  // (255 marks unreachable)
                double x;
                std::memcpy(&x, &keyed[q].first, 8);
                rtab.push_back(x);
            }
            rix[keyed[q].second] = (uint8_t)(rtab.size() - 1);
        }
    }
    int blk = 0;
    size_t lds = 0;
    bool hbm = false;
    if (n <= 16 * 256 && kf_lds_bytes<256>(n) <= kLdsBudget / 4) { blk = 256; lds = kf_lds_bytes<256>(n); }
    else if (n <= 16 * 1024 && kf_lds_bytes<1024>(n) <= kLdsBudget) { blk = 1024; lds = kf_lds_bytes<1024>(n); }
    else if (n <= 64 * 1024 && kfh_lds_bytes<1024>(n) <= kLdsBudget) { blk = 1024; lds = kfh_lds_bytes<1024>(n); hbm = true; }
    if (const char* e = getenv("SHD_ROUTE_KFH"))  // (tests: KFH on graphs KF takes)
        if (atoi(e) && n <= 64 * 1024 && kfh_lds_bytes<1024>(n) <= kLdsBudget) { blk = 1024; lds = kfh_lds_bytes<1024>(n); hbm = true; }
    if (!blk) return SHD_ROUTE_OK;
    // bucket width: the 40th percentile of arc latencies (KF rounds cost far more than the
    // re-expansions wider buckets bring: C3f 15.0 / 13.4 / 13.1 ms at the 12th / 25th / 50th,
    // C2f 0.60 / 0.55 / 0.57 ms); KFH the 10th, where a re-expansion is HBM traffic (C4f, the
    // width in ms: 15 / 25 / 35 / 50 / 70 / ~100 (40th) / 200: 822 / 815 / 822 / 835 / 842 /
    // 886 / 1061 ms)
    std::vector<double> ws(w_in.begin(), w_in.end());
    const size_t k = ws.size() * (hbm ? 10 : 40) / 100;
    std::nth_element(ws.begin(), ws.begin() + k, ws.end());
    double delta = ws[k];
    if (const char* e = getenv("SHD_ROUTE_KFDELTA")) delta = atof(e);
    if (!(delta > 0.0) || std::isinf(delta)) delta = c->min_w > 0 ? c->min_w : 1.0;
    int rc = upload(c, &c->d_kf_rix, rix);
    if (!rc) rc = upload(c, &c->d_kf_rtab, rtab);
    // Packed arcs (KFH): when every latency is a decimal k / scale (scale 1, 10, 100 or 1000)
    // with k < 65536, an arc is one u32, head | k << 16, and the kernel divides k by the scale
    // -- IEEE division of two exact integers is the correctly rounded k / scale, the double the
    // decimal parses to, and each arc is checked here (C4f's latencies have two decimals: 4
    // bytes per arc read instead of 12; C4f 780 -> 764 ms).  The LDS kernels keep f64 arcs:
    // there the division costs more than the bytes (C3f 10.39 -> 10.59, C2f 0.45 -> 0.49 ms)
    double wscale = 0.0;
    if (hbm && !(getenv("SHD_ROUTE_KFPK") && atoi(getenv("SHD_ROUTE_KFPK")) == 0)) {
        for (const double sc : {1.0, 10.0, 100.0, 1000.0}) {
            auto fits = [&](const std::vector<double>& ws) {
                for (const double x : ws) {
                    const double k = std::nearbyint(x * sc);
                    if (!(k >= 1.0 && k <= 65535.0) || k / sc != x) return false;
                }
                return true;
            };
            if (fits(w) && (c->directed ? fits(w_in) : true)) { wscale = sc; break; }
        }
    }
    if (!rc && wscale > 0.0) {
        auto pack = [&](const std::vector<int>& cc, const std::vector<double>& ws) {
            std::vector<uint32_t> pk(cc.size());
            for (size_t a = 0; a < cc.size(); a++)
                pk[a] = (uint32_t)cc[a] | ((uint32_t)std::nearbyint(ws[a] * wscale) << 16);
            return pk;
        };
        rc = upload(c, &c->d_kf_opk, pack(col, w));
        if (!rc) {
            if (c->directed) rc = upload(c, &c->d_kf_ipk, pack(col_in, w_in));
            else c->d_kf_ipk = c->d_kf_opk;
        }
        c->kf_wscale = wscale;
    }
    const bool pk = wscale > 0.0;
    const void* kfn = hbm ? (pk ? (const void*)sssp_f64d_kernel<1024, true, true> : (const void*)sssp_f64d_kernel<1024, true>)
                    : blk == 256 ? (pk ? (const void*)sssp_f64d_kernel<256, false, true> : (const void*)sssp_f64d_kernel<256>)
                                 : (pk ? (const void*)sssp_f64d_kernel<1024, false, true> : (const void*)sssp_f64d_kernel<1024>);
    if (!rc) rc = hip_check(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (rc) return rc;
    c->kf_block = blk; c->kf_lds = lds; c->kf_delta = delta; c->kf_nrtab = (int)rtab.size();
    c->kf_slots = 256 * std::max(1, std::min((int)(kLdsBudget / lds), 1024 / blk));
    if (hbm) {
        c->kf_h = 1;
        c->kf_ws_stride = kfh_ws_stride<1024>(n);
        if (hipMalloc((void**)&c->d_kf_ws, c->kf_ws_stride * (size_t)c->kf_slots) != hipSuccess) return SHD_ROUTE_ENOMEM;
        c->allocs.push_back(c->d_kf_ws);
    }
    c->sel = 5;
    return SHD_ROUTE_OK;
}

int shd_route_create(shd_route_t** out, const shd_graph_t* g, int device) {
    if (!out || !g) return SHD_ROUTE_EINVAL;
    *out = nullptr;
    const int n = g->n_vertices, m = g->n_edges;
    if (n <= 0 || m < 0 || (m > 0 && (!g->edge_src || !g->edge_dst || !g->edge_latency || !g->edge_packetloss)))
        return SHD_ROUTE_EINVAL;
    // validation as topology.c:1041-1124 (edges) and 811-978 (vertex packetloss)
    for (int e = 0; e < m; e++) {
        int a = g->edge_src[e], b = g->edge_dst[e];
        double w = g->edge_latency[e], p = g->edge_packetloss[e];
        if (a < 0 || a >= n || b < 0 || b >= n) return SHD_ROUTE_EINVAL;
        if (!(w > 0.0) || std::isinf(w)) return SHD_ROUTE_EINVAL;
        if (!(p >= 0.0 && p <= 1.0)) return SHD_ROUTE_EINVAL;
    }
    if (g->vertex_packetloss)
        for (int v = 0; v < n; v++) {
            double p = g->vertex_packetloss[v];
            if (!std::isnan(p) && !(p >= 0.0 && p <= 1.0)) return SHD_ROUTE_EINVAL;
        }
    if (hipSetDevice(device) != hipSuccess) return SHD_ROUTE_EDEVICE;

    shd_route* c = new (std::nothrow) shd_route();
    if (!c) return SHD_ROUTE_ENOMEM;
    c->device = device; c->n = n; c->m = m;
    c->directed = g->directed ? 1 : 0;
    c->prefer_direct = g->prefer_direct ? 1 : 0;
    c->e_src.assign(g->edge_src, g->edge_src + m);
    c->e_dst.assign(g->edge_dst, g->edge_dst + m);
    c->e_lat.assign(g->edge_latency, g->edge_latency + m);
    c->e_rel.resize(m);
    for (int e = 0; e < m; e++) c->e_rel[e] = (1.0f - g->edge_packetloss[e]);  // topology.c:437

    // arcs for SSSP (self-loops excluded: w > 0 never relaxes them)
    std::vector<int32_t> ar, ac, ae, ir, ic, ie;
    std::vector<double> self_w(n, NAN), self_r(n, NAN);
    std::vector<int> loops(n, 0), degm(n, 0);
    double maxw = 0;
    c->min_w = m ? INFINITY : 0;
    bool integral = true;
    for (int e = 0; e < m; e++) {
        int a = g->edge_src[e], b = g->edge_dst[e];
        double w = g->edge_latency[e];
        maxw = std::max(maxw, w);
        c->min_w = std::min(c->min_w, w);
        if (w != std::floor(w) || w > 1048576.0) integral = false;
        if (a == b) {
            if (std::isnan(self_w[a])) { self_w[a] = w; self_r[a] = c->e_rel[e]; }
            loops[a]++;
            continue;
        }
        ar.push_back(a); ac.push_back(b); ae.push_back(e);
        degm[a]++;
        if (!c->directed) { ar.push_back(b); ac.push_back(a); ae.push_back(e); degm[b]++; }
        else { ir.push_back(b); ic.push_back(a); ie.push_back(e); }
    }
    c->integer_w = integral && (double)n * maxw < 2147483647.0;
    c->max_w = maxw;
    for (int v = 0; v < n; v++)
        if (!std::isnan(self_w[v]) && !(self_w[v] == std::floor(self_w[v]) && self_w[v] < 65535.0)) c->self16 = 0;
    std::vector<int> row, col, row_in, col_in, eid;
    std::vector<double> w, r, w_in, r_in;
    build_csr(n, ar, ac, ae, c->e_lat, c->e_rel, row, col, w, r, &eid);
    if (c->directed) build_csr(n, ir, ic, ie, c->e_lat, c->e_rel, row_in, col_in, w_in, r_in);
    c->nnz = (int)col.size();
    for (int v = 0; v < n && !c->multigraph; v++)
        for (int a = row[v] + 1; a < row[v + 1]; a++)
            if (col[a] == col[a - 1]) { c->multigraph = 1; break; }
    for (int v = 0; v < n; v++) if (loops[v] > 1) c->multigraph = 1;

    // topology.c:738-806: strongly connected, one cluster
    if (!strongly_connected(n, row, col, c->directed ? row_in : row, c->directed ? col_in : col)) {
        delete c;
        return SHD_ROUTE_EINVAL;
    }
    // topology.c:450-552 isComplete: OUT-incident count (undirected: loops twice, minus one)
    c->complete = 1;
    for (int v = 0; v < n; v++) {
        long long ecount;
        if (c->directed) ecount = (row[v + 1] - row[v]) + loops[v];
        else ecount = (row[v + 1] - row[v]) + 2LL * loops[v] - (loops[v] > 0 ? 1 : 0);
        if (ecount < n) { c->complete = 0; break; }
    }

    std::vector<double> vf(n, NAN);
    if (g->vertex_packetloss)
        for (int v = 0; v < n; v++)
            if (!std::isnan(g->vertex_packetloss[v])) {
                vf[v] = (1.0f - g->vertex_packetloss[v]);
                c->has_vf = 1;
                if (vf[v] != 1.0) c->vf_lossy = 1;
            }

    int rc = SHD_ROUTE_OK;
    if (!rc) rc = upload(c, &c->d_row, row);
    if (!rc) rc = upload(c, &c->d_col, col);
    if (!rc) rc = upload(c, &c->d_w, w);
    if (!rc) rc = upload(c, &c->d_r, r);
    if (c->directed) {
        if (!rc) rc = upload(c, &c->d_row_in, row_in);
        if (!rc) rc = upload(c, &c->d_col_in, col_in);
        if (!rc) rc = upload(c, &c->d_w_in, w_in);
        if (!rc) rc = upload(c, &c->d_r_in, r_in);
    } else {
        c->d_row_in = c->d_row; c->d_col_in = c->d_col; c->d_w_in = c->d_w; c->d_r_in = c->d_r;
    }
    if (!rc) rc = upload(c, &c->d_vf, vf);
    if (!rc) rc = upload(c, &c->d_self_w, self_w);
    if (!rc) rc = upload(c, &c->d_self_r, self_r);
    if (!rc) {
        std::vector<int> z(1, 0);
        rc = upload(c, &c->d_err, z);
    }
    StateLayout L = StateLayout::make(n);
    c->lds_bytes = kSmallBytes + L.total;
    c->lds = c->lds_bytes <= kLdsBudget;
    if (!rc) {
        if (c->lds) {
            rc = hip_check(hipFuncSetAttribute((const void*)sssp_rows_kernel<true>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds_bytes));
        } else {
            rc = alloc_ws(c);
        }
    }
    if (!rc) rc = prepare_k32(c, row, col, w, eid, c->directed ? row_in : row, c->directed ? col_in : col,
                              c->directed ? w_in : w);
    if (!rc && c->sel == 0)
        rc = prepare_kf(c, col, w, c->directed ? row_in : row, c->directed ? col_in : col, c->directed ? w_in : w,
                        c->directed ? r_in : r);
    if (rc) {
        shd_route_destroy(c);
        return rc;
    }
    if (c->sel == 4 && c->kd_fused) host_pool();  // the planner's workers, parked until a plan
    *out = c;
    return SHD_ROUTE_OK;
}

void shd_route_destroy(shd_route_t* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->d_keys) (void)hipFree(c->d_keys);
    if (c->d_fwkey) (void)hipFree(c->d_fwkey);
    if (c->d_lm_drow) (void)hipFree(c->d_lm_drow);
    if (c->d_lm_prow) (void)hipFree(c->d_lm_prow);
    if (c->d_hub_ws) (void)hipFree(c->d_hub_ws);
    for (void* p : c->allocs) (void)hipFree(p);
    delete c;
}

// u16 latency payloads are exact: integer latencies whose shortest paths are proven below
// 0xFFFF and integer self-loops (the diagonal, kept out of the CSR and its bound) below it
static bool lat16_ok(const shd_route* c) {
    return c->integer_w && c->self16 && c->k32_bound > 0 && c->k32_bound < 0xFFFF;
}

int shd_route_get_info(const shd_route_t* c, shd_route_info_t* info) {
    if (!c || !info) return SHD_ROUTE_EINVAL;
    info->n_vertices = c->n;
    info->n_edges = c->m;
    info->n_arcs = c->nnz;
    info->is_complete = c->complete;
    info->directed = c->directed;
    info->prefer_direct = c->prefer_direct;
    info->integer_weights = c->integer_w;
    info->multigraph = c->multigraph;
    info->device = c->device;
    info->lds_resident = ((c->lds || c->sel) && !c->kf_h) ? 1 : 0;  // (KFH: vertex state in HBM)
    info->kernel = c->sel;
    info->dist_bound = c->k32_bound;
    info->block = c->sel == 2 ? KB_BLOCK : c->sel == 3 ? 1024 : c->sel == 4 ? c->kd_block
                : c->sel == 1 ? c->k32_block : c->sel == 5 ? c->kf_block : kBlock;
    info->reserved = c->sel == 4 ? c->kd_delta : c->sel == 2 ? c->kb_fused : c->sel == 5 ? (int)c->kf_wscale : 0;
    info->lat16 = lat16_ok(c) ? 1 : 0;
    info->device_bytes = c->device_bytes;
    info->min_edge_latency = c->min_w;
    return SHD_ROUTE_OK;
}

int shd_route_rows_async(shd_route_t* c, const int32_t* d_src, int32_t ns, const int32_t* d_tgt,
                         int32_t nt, int64_t ld, uint32_t flags, double* d_lat, double* d_rel,
                         double* d_row_min, void* stream) {
    if (!c || ns < 0 || nt < 0 || (ns && !d_src) || (nt && !d_tgt) || ld < nt) return SHD_ROUTE_EINVAL;
    if (ns == 0) return SHD_ROUTE_OK;
    hipStream_t st = (hipStream_t)stream;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if ((flags & SHD_ROUTE_DISPATCH) && c->complete) {
        int rc = ensure_dense(c);
        if (rc) return rc;
        int grid = std::min(ns, 65535);
        hipLaunchKernelGGL(direct_rows_kernel, dim3(grid), dim3(kBlock), 0, st, c->n, c->d_W, c->d_R,
                           c->d_vf, d_src, ns, d_tgt, nt, (long long)ld, d_lat, d_rel, d_row_min, c->d_err);
        return hip_check(hipGetLastError());
    }
    const int dispatch = (flags & SHD_ROUTE_DISPATCH) ? 1 : 0;
    if (c->sel == 2 && !(dispatch && c->prefer_direct)) {
        DevKB kb;
        kb.n = c->n; kb.nnz = c->nnz; kb.nseg = c->kb_nseg; kb.nhub = c->kb_nhub; kb.npart = c->kb_npart;
        kb.bound = c->k32_bound; kb.arc = c->d_kb_arc; kb.row_in = c->d_k32_row_in; kb.seg = c->d_kb_seg;
        kb.hub = c->d_kb_hub;
        kb.rtab = c->d_kbf_rtab; kb.nrtab = c->kbf_nrtab;
        kb.vf = c->d_vf; kb.self_w = c->d_self_w; kb.self_r = c->d_self_r;
        int gridb = std::min((ns + KB_SRC - 1) / KB_SRC, 1 << 20);
        if (c->kb_grid_cap > 0) gridb = std::min(gridb, c->kb_grid_cap);
        if (c->kb_fused) {
            // KB with fused path attributes: the rows in one kernel
            kb.arc = c->d_kbf_arc;
            kb.dbg = c->d_dbg ? c->d_dbg + (size_t)ns * 8 : nullptr;
            kb.tcap = c->kbf_tcap;
            hipLaunchKernelGGL(sssp_batch_rows_kernel, dim3(gridb), dim3(KB_BLOCK), c->kbf_lds, st, kb, d_src, ns,
                               c->d_err, d_tgt, nt, (long long)ld, d_lat, d_rel, d_row_min);
            return hip_check(hipGetLastError());
        }
        // KB distances+parents for KB_SRC sources per workgroup -> key rows -> K2
        const size_t need = (size_t)ns * c->n;
        if (need > c->keys_cap) {
            if (c->d_keys) (void)hipFree(c->d_keys);
            c->d_keys = nullptr;
            c->keys_cap = 0;
            if (hipMalloc((void**)&c->d_keys, need * sizeof(uint32_t)) != hipSuccess) return SHD_ROUTE_ENOMEM;
            c->keys_cap = need;
        }
        kb.dbg = c->d_dbg ? c->d_dbg + (size_t)ns * 8 : nullptr;
        hipLaunchKernelGGL(sssp_batch_kernel, dim3(gridb), dim3(KB_BLOCK), c->kb_lds, st, kb, d_src, ns,
                           c->d_keys, (long long)c->n, c->d_err);
        int rc = hip_check(hipGetLastError());
        if (rc) return rc;
        DevAttr at;
        at.n = c->n; at.row_in = c->d_k32_row_in; at.col_in = c->d_k32_col_in; at.r_in = c->d_k32_r_in;
        at.vf = c->d_vf; at.self_w = c->d_self_w; at.self_r = c->d_self_r;
        at.dbg = c->d_dbg;
        const int grida = std::min(ns, 1 << 20);
        hipLaunchKernelGGL(path_attr_kernel<256>, dim3(grida), dim3(256), c->attr_lds, st, at, c->d_keys,
                           (long long)c->n, d_src, ns, d_tgt, nt, (long long)ld, d_lat, d_rel, d_row_min, c->d_err);
        return hip_check(hipGetLastError());
    }
    if (c->sel == 4 && !(dispatch && c->prefer_direct)) {
        DevDelta k = kd_args(c);
        if (hipMemsetAsync(c->d_kd_next, 0, sizeof(int), st) != hipSuccess) return SHD_ROUTE_EDEVICE;
        return kd_launch(c, k, c->d_kd_next, d_src, ns, d_tgt, nt, ld, d_lat, d_rel, d_row_min, st);
    }
    if (c->sel == 1 && !(dispatch && c->prefer_direct)) {
        DevK32 k;
        k.n = c->n; k.bound = c->k32_bound; k.row = c->d_row; k.arc = c->d_arc; k.row_in = c->d_k32_row_in;
        k.col_in = c->d_k32_col_in; k.r_in = c->d_k32_r_in; k.vf = c->d_vf; k.self_w = c->d_self_w;
        k.self_r = c->d_self_r;
        k.dbg = c->d_dbg;
        const int grid = std::min(ns, 1 << 20);
        if (c->k32_block == 256)
            hipLaunchKernelGGL(sssp_k32_kernel<256>, dim3(grid), dim3(256), c->k32_lds, st, k, d_src, ns, d_tgt, nt,
                               (long long)ld, d_lat, d_rel, d_row_min, c->d_err);
        else if (c->k32_block == 512)
            hipLaunchKernelGGL(sssp_k32_kernel<512>, dim3(grid), dim3(512), c->k32_lds, st, k, d_src, ns, d_tgt, nt,
                               (long long)ld, d_lat, d_rel, d_row_min, c->d_err);
        else
            hipLaunchKernelGGL(sssp_k32_kernel<1024>, dim3(grid), dim3(1024), c->k32_lds, st, k, d_src, ns, d_tgt, nt,
                               (long long)ld, d_lat, d_rel, d_row_min, c->d_err);
        return hip_check(hipGetLastError());
    }
    if (c->sel == 5 && !(dispatch && c->prefer_direct)) {
        DevF64D k;
        k.n = c->n; k.nw = (c->n + 63) / 64; k.delta = c->kf_delta;
        k.row = c->d_row; k.col = c->d_col; k.w = c->d_w;
        k.row_in = c->d_row_in; k.col_in = c->d_col_in; k.w_in = c->d_w_in;
        k.rix_in = c->d_kf_rix; k.rtab = c->d_kf_rtab; k.nrtab = c->kf_nrtab;
        k.hring = 0;
        if (const char* e = getenv("SHD_ROUTE_KFH_RING")) k.hring = std::max(0, atoi(e));  // (tests: a small ring)
        k.vf = c->d_vf; k.self_w = c->d_self_w; k.self_r = c->d_self_r; k.dbg = c->d_dbg;
        k.opk = c->d_kf_opk; k.ipk = c->d_kf_ipk; k.wscale = c->kf_wscale;
        const int grid = std::min(ns, c->kf_slots);
        auto go = [&](auto kern, int blk, char* ws, size_t wst) {
            hipLaunchKernelGGL(kern, dim3(grid), dim3(blk), c->kf_lds, st, k, d_src, ns, d_tgt, nt, (long long)ld, d_lat,
                               d_rel, d_row_min, c->d_err, ws, wst);
        };
        const bool pk = c->d_kf_opk != nullptr;
        if (c->kf_h) {  // (the slices: one per workgroup slot, grid <= kf_slots)
            if (pk) go(sssp_f64d_kernel<1024, true, true>, 1024, c->d_kf_ws, c->kf_ws_stride);
            else go(sssp_f64d_kernel<1024, true>, 1024, c->d_kf_ws, c->kf_ws_stride);
        } else if (c->kf_block == 256) {
            if (pk) go(sssp_f64d_kernel<256, false, true>, 256, (char*)nullptr, (size_t)0);
            else go(sssp_f64d_kernel<256>, 256, (char*)nullptr, (size_t)0);
        } else {
            if (pk) go(sssp_f64d_kernel<1024, false, true>, 1024, (char*)nullptr, (size_t)0);
            else go(sssp_f64d_kernel<1024>, 1024, (char*)nullptr, (size_t)0);
        }
        return hip_check(hipGetLastError());
    }
    DevGraph g = dev_graph(c);
    if (c->lds) {
        int grid = std::min(ns, 1 << 20);
        hipLaunchKernelGGL(sssp_rows_kernel<true>, dim3(grid), dim3(kBlock), c->lds_bytes, st, g, d_src, ns,
                           d_tgt, nt, (long long)ld, d_lat, d_rel, d_row_min, c->d_err, nullptr, (size_t)0,
                           dispatch);
    } else {
        int grid = std::min(ns, c->ws_slots);
        hipLaunchKernelGGL(sssp_rows_kernel<false>, dim3(grid), dim3(kBlock), kSmallBytes, st, g, d_src, ns,
                           d_tgt, nt, (long long)ld, d_lat, d_rel, d_row_min, c->d_err, c->d_ws, c->ws_stride,
                           dispatch);
    }
    return hip_check(hipGetLastError());
}

int shd_route_sync(shd_route_t* c, void* stream) {
    if (!c) return SHD_ROUTE_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return SHD_ROUTE_EDEVICE;
    return take_err(c);
}

}  // extern "C"

namespace {
// The planner's seed choices on the device (shd_route_plan_create): one thread per source
// row, the same rule as the host's choose() -- the kseeds neighbours u of smaller closeness
// rank (and with a row in the plan) by (w(s,u) + alpha * closeness(u), u), then, if short,
// two-hop rows s -> x -> u (deg x <= hop_deg) by (w(s,x) + w(x,u) + closeness(u), u, record).
// Arcs from the packed out-records (u | w << 16 | ridx << 24).  Entries [0, m) are
// neighbour seeds, [m, m + nh) two-hop seeds (w = w(s,x) + w(x,u), record (x,u)).
// Up to PC_CAND neighbour candidates are listed in order (ncand of them asked for), so
// that the sequential pass, whose usable set is a subset of `avail` (the seed-chain depth
// cap), finds the exact top-kseeds usable ones in the list instead of rescanning the CSR
// row on the host (C3: 928 host recomputations, ~2 ms of the 4.1 ms plan).
constexpr int PC_CAND = 6;
struct PlanChoice {
    int m, nh;
    int u[PC_CAND], w[PC_CAND];
    uint32_t rec[PC_CAND];
    int pad[2];
};
static_assert(KD_SEEDS <= 3 && 2 * KD_SEEDS <= PC_CAND, "PlanChoice holds the candidates");

// A root's landmark seeds on the device (shd_route_plan_create): one wave per root row s, the
// host rule -- the klm landmarks nearest s by (d_L(s), landmark index) (undirected graphs:
// d_L(s) = d(s, L)), each with the record of L's own vertex in s's tree: the last arc (x, L)
// of the s -> L path in L's tree, found by walking L's parent records up from s.
constexpr int LM_DIV_K = 16;  // spread landmark seeds: up to 64 x 16 = 1024 landmarks per row's wave
struct LmChoice {
    int m;
    int l[3], d[3];
    uint32_t rec[3];
    int pad[2];
};
// (bias, device-built landmark-only plans, round 6: a landmark's pick key is d(s, L) + bias[L],
// bias = half L's mean distance to the first 16 landmarks, so that of two landmarks about as
// near to s the more central one seeds the row: its row bounds more of s's paths.  Offline on C3
// (tools/landmark_choice.py, 300 sampled rows, exact distances): the share of vertices a row
// improves on its bound 15.9% -> 13.1%; weights 0.375-0.625 measure the same, 0.25 13.5%, 1.0 15.3%)
__device__ inline LmChoice lm_pick(const uint16_t* __restrict__ drow, const uint32_t* __restrict__ prow, long long rs,
                                   const int* __restrict__ lmv, int nland, int s, int klm, int n, int lane,
                                   const uint16_t* __restrict__ bias = nullptr, int spread = 0) {
    LmChoice o;
    o.m = 0; o.pad[0] = o.pad[1] = 0;
    for (int k = 0; k < 3; k++) { o.l[k] = 0; o.d[k] = 0; o.rec[k] = 0u; }
    // L's own record in s's tree: the last arc (x, L) of L's tree path from s
    auto rec_of = [&](int l) __attribute__((always_inline)) {
        const int L = lmv[l];
        uint32_t rec = KD_SRC_MARK;
        if (L != s) {
            const uint32_t* lp = prow + (long long)l * rs;
            int x = s;
            for (int hop = 0; hop < n && (int)(lp[x] & 0xFFFFu) != L; hop++) x = (int)(lp[x] & 0xFFFFu);
            rec = (uint32_t)x | (lp[x] & 0xFFFF0000u);
        }
        return rec;
    };
    if (bias && spread && nland <= 64 * LM_DIV_K) {
        // Spread seeds (round 6): each next landmark minimises d(s, L) + bias[L] - d(L', L) / 2
        // over the landmarks not picked, L' the nearest already-picked one (its row gives
        // d(L', L) at L's vertex), so the seeds bound s's paths from different sides.  Offline
        // on C3 (tools/landmark_choice.py, 300 rows): improved share 13.5% (central-biased
        // nearest) -> 9.3%; separation weights 3/8-5/8 the same, 3/4 10.6%, 1 14.1%.
        int dl[LM_DIV_K], sc[LM_DIV_K];
#pragma unroll
        for (int j = 0; j < LM_DIV_K; j++) {
            const int l = lane + 64 * j;
            const unsigned d = l < nland ? drow[(long long)l * rs + s] : 0xFFFFu;
            dl[j] = (int)d;
            sc[j] = (l < nland && d != 0xFFFFu) ? (int)d + (int)bias[l] : 0x7FFFFFFF;
        }
        int sep[LM_DIV_K];
#pragma unroll
        for (int j = 0; j < LM_DIV_K; j++) sep[j] = 0x7FFFFFFF;
        for (int k = 0; k < klm && k < 3; k++) {
            // the wave's minimum of (score, l) over the landmarks not yet picked
            unsigned long long best = ~0ull;
#pragma unroll
            for (int j = 0; j < LM_DIV_K; j++) {
                if (sc[j] == 0x7FFFFFFF) continue;
                const int x = k == 0 ? sc[j] : sc[j] - sep[j] / 2;
                const unsigned long long key = ((unsigned long long)(unsigned)(x + 0x40000000) << 32) |
                                               (unsigned)(lane + 64 * j);
                best = min(best, key);
            }
            for (int off = 32; off > 0; off >>= 1) {
                const unsigned long long y = ((unsigned long long)(unsigned)__shfl_xor((int)(best >> 32), off) << 32) |
                                             (unsigned)__shfl_xor((int)(unsigned)best, off);
                best = min(best, y);
            }
            if (best == ~0ull) break;
            const int l = (int)(unsigned)best;
            int dpick = 0;  // (register arrays indexed by unrolled constants only: no scratch)
#pragma unroll
            for (int j = 0; j < LM_DIV_K; j++)
                if (j == (l >> 6)) {
                    if ((l & 63) == lane) sc[j] = 0x7FFFFFFF;  // (picked)
                    dpick = dl[j];
                }
            // separations to the picked landmark: its row at every landmark's vertex
            if (k + 1 < klm) {
                const uint16_t* lr = drow + (long long)l * rs;
#pragma unroll
                for (int j = 0; j < LM_DIV_K; j++) {
                    const int q = lane + 64 * j;
                    if (q < nland) sep[j] = min(sep[j], (int)lr[lmv[q]]);
                }
            }
            o.l[k] = l; o.d[k] = __shfl(dpick, l & 63); o.rec[k] = rec_of(l);
            o.m = k + 1;
        }
        return o;
    }
    // each lane's three smallest keys (d << 16 | l) over its landmarks l = lane + 64 j, read
    // once; the wave's k-th pick is then the minimum over the lanes' lists past the (k-1)-th
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    uint32_t c0 = NONE, c1 = NONE, c2 = NONE;
    for (int l0 = 0; l0 < nland; l0 += 64 * 8) {
        uint32_t d8[8];
#pragma unroll
        for (int h = 0; h < 8; h++) {
            const int l = l0 + 64 * h + lane;
            d8[h] = l < nland ? drow[(long long)l * rs + s] : 0xFFFFu;
        }
        if (bias) {
#pragma unroll
            for (int h = 0; h < 8; h++) {
                const int l = l0 + 64 * h + lane;
                if (l < nland && d8[h] != 0xFFFFu) d8[h] = min(0xFFFEu, d8[h] + (uint32_t)bias[l]);
            }
        }
#pragma unroll
        for (int h = 0; h < 8; h++) {
            const uint32_t key = (d8[h] << 16) | (uint32_t)(l0 + 64 * h + lane);
            if (d8[h] == 0xFFFFu) continue;
            if (key < c2) {
                c2 = key;
                if (c2 < c1) { const uint32_t t = c1; c1 = c2; c2 = t; }
                if (c1 < c0) { const uint32_t t = c0; c0 = c1; c1 = t; }
            }
        }
    }
    for (int k = 0; k < klm && k < 3; k++) {
        uint32_t best = c0;
        for (int off = 32; off > 0; off >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, off));
        if (best == NONE) break;
        if (c0 == best) { c0 = c1; c1 = c2; c2 = NONE; }  // (keys are unique: one lane owns it)
        const int l = (int)(best & 0xFFFFu);
        // (with a bias the key is not the distance: the offset is read back)
        o.l[k] = l; o.d[k] = bias ? (int)drow[(long long)l * rs + s] : (int)(best >> 16); o.rec[k] = rec_of(l);
        o.m = k + 1;
    }
    return o;
}

__global__ void plan_landmark_kernel(const uint16_t* __restrict__ drow, const uint32_t* __restrict__ prow, long long rs,
                                     const int* __restrict__ lmv, int nland, const int* __restrict__ srcq, int nq, int klm,
                                     int n, LmChoice* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (q >= nq) return;  // the whole wave
    const LmChoice o = lm_pick(drow, prow, rs, lmv, nland, srcq[q], klm, n, lane);
    if (lane == 0) out[q] = o;
}

// Landmark-only plans built on the device (round 5): the queue order and the job records
// without a host round trip.  The order is the host rule's: descending (closeness, vertex,
// position), closeness = the sum of the first nclose hub rows' distances (unreached: the
// largest key).  Keys are unique, so a job's queue slot is the number of larger keys (a rank
// sort: every workgroup holds all keys in LDS, nq <= PLAN_DEV_MAXJ; ~20 us at C3, where a
// one-workgroup bitonic sort took ~0.3 ms).
constexpr int PLAN_DEV_MAXJ = 16384;
__global__ void plan_lmall_keys_kernel(const uint16_t* __restrict__ drow, long long rs, int nclose,
                                       const int* __restrict__ srcq, int nq, unsigned long long* __restrict__ keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const int s = srcq[i];
    unsigned sum = 0;
    bool unr = false;
    for (int q = 0; q < nclose; q++) {
        const unsigned d = drow[(long long)q * rs + s];
        unr = unr || d == 0xFFFFu;
        sum += d;
    }
    if (unr) sum = (1u << 20) - 1;  // (16 finite distances sum below it)
    keys[i] = ((unsigned long long)sum << 40) | ((unsigned long long)s << 24) | (unsigned long long)i;
}
__global__ __launch_bounds__(256) void plan_lmall_rank_kernel(const unsigned long long* __restrict__ keys, int nq,
                                                              int* __restrict__ slot) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long rkeys[];
    for (int j = threadIdx.x; j < nq; j += blockDim.x) rkeys[j] = keys[j];
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const unsigned long long k = rkeys[i];
    int r = 0;
    for (int j = 0; j < nq; j++) r += rkeys[j] > k;  // (same j across the wave: an LDS broadcast)
    slot[i] = r;
}

// one wave per job i (jobs in position order, so that a workgroup's waves read neighbouring
// columns of the landmark rows, and consecutive workgroups on one XCD: blockIdx.x % 8 picks
// the XCD, which takes one contiguous eighth of the jobs), the landmark seeds of the row
// (lm_pick) written as its KDJob at its queue slot.  row = the position's index in this
// rank's rows, seeds = landmark slots (the borrowed store holds the landmark rows only).
// nroots counts the jobs left unseeded (no landmark reaches s).
__global__ void plan_lmall_jobs_kernel(const uint16_t* __restrict__ drow, const uint32_t* __restrict__ prow, long long rs,
                                       const int* __restrict__ lmv, int nland, const int* __restrict__ srcq,
                                       const int* __restrict__ slot, int nq, int klm, int n, KDJob* __restrict__ out,
                                       int* __restrict__ nroots, int hub_base = -1,
                                       const uint16_t* __restrict__ bias = nullptr, int spread = 0) {
    const int lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
    const int per = gridDim.x / 8;  // (the grid is a multiple of 8 workgroups)
    const int b = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);  // (XCD-contiguous block order)
    const int i = b * wpb + (threadIdx.x >> 6);
    if (i >= nq) return;  // the whole wave
    const int s = srcq[i];
    const LmChoice o = lm_pick(drow, prow, rs, lmv, nland, s, klm, n, lane, bias, spread);
    if (lane == 0) {
        // (hub_base >= 0: a second-level landmark row of the plan's own hub launch, kept in
        // store slot hub_base + i, no output row)
        KDJob J;
        J.row = hub_base >= 0 ? -1 : i; J.s = s; J.store = hub_base >= 0 ? hub_base + i : -1; J.nseed = o.m;
        for (int k = 0; k < KD_SEEDS; k++) {
            const bool on = k < o.m;
            J.seed[k] = on ? o.l[k] : 0;
            J.u[k] = on ? lmv[o.l[k]] : 0;
            J.wr[k] = on ? o.d[k] : 0;
            J.rec[k] = on ? (int)o.rec[k] : 0;
        }
        out[slot ? slot[i] : i] = J;
        if (o.m == 0 && nroots) atomicAdd(nroots, 1);
    }
}

// each landmark's pick bias (lm_pick): half its mean distance to the first nclose landmarks,
// rounded, from the landmark rows (unreached: the largest bias)
__global__ void plan_lmall_bias_kernel(const uint16_t* __restrict__ drow, long long rs, int nclose,
                                       const int* __restrict__ lmv, int nland, uint16_t* __restrict__ bias) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nland) return;
    const int v = lmv[l];
    unsigned sum = 0;
    bool unr = false;
    for (int q = 0; q < nclose; q++) {
        const unsigned d = drow[(long long)q * rs + v];
        unr = unr || d == 0xFFFFu;
        sum += d;
    }
    bias[l] = unr ? (uint16_t)0x7FFF : (uint16_t)min(0x7FFFu, (sum + (unsigned)nclose) / (2u * (unsigned)nclose));
}

// lexicographic minimum of (x, u, t) over the wave (t: a tie-breaking key, arc or record)
__device__ inline void wave_min3(double& x, int& u, uint32_t& t) {
    for (int o = 32; o > 0; o >>= 1) {
        const double x2 = __shfl_xor(x, o);
        const int u2 = __shfl_xor(u, o);
        const uint32_t t2 = __shfl_xor(t, o);
        if (x2 < x || (x2 == x && (u2 < u || (u2 == u && t2 < t)))) { x = x2; u = u2; t = t2; }
    }
}

// one wave per source row: each pick is the wave's minimum key over the arcs whose head is
// not picked yet, which is the host's top-k of the per-head best keys (duplicate heads of a
// multigraph keep their best arc, the first one on a full tie)
__global__ void plan_choice_kernel(const int* __restrict__ row, const uint32_t* __restrict__ orec,
                                   const double* __restrict__ close, const int* __restrict__ rk,
                                   const uint8_t* __restrict__ avail, const int* __restrict__ srcq, int nq, int kseeds,
                                   int two_hop, int hop_deg, double alpha, int ncand, PlanChoice* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (q >= nq) return;  // the whole wave
    const int s = srcq[q], rks = rk[s], a0 = row[s], a1 = row[s + 1];
    int su[PC_CAND], sw[PC_CAND];
    uint32_t sr[PC_CAND];
#pragma unroll
    for (int k = 0; k < PC_CAND; k++) { su[k] = -1; sw[k] = 0; sr[k] = 0u; }
    auto picked = [&](int u) {
        bool p = false;
#pragma unroll
        for (int k = 0; k < PC_CAND; k++) p = p || u == su[k];
        return p;
    };
    ncand = max(kseeds, min(ncand, PC_CAND));
    int m = 0;
    for (; m < ncand; m++) {
        double bx = INFINITY;
        int bu = INT_MAX;
        uint32_t ba = UINT_MAX;
        for (int a = a0 + lane; a < a1; a += 64) {
            const uint32_t r = orec[a];
            const int u = (int)(r & 0xFFFFu);
            if (u == s || picked(u) || !avail[u] || rk[u] >= rks) continue;
            const double x = (double)((r >> 16) & 0xFFu) + alpha * close[u];
            if (x < bx || (x == bx && (u < bu || (u == bu && (uint32_t)a < ba)))) { bx = x; bu = u; ba = (uint32_t)a; }
        }
        wave_min3(bx, bu, ba);
        if (ba == UINT_MAX) break;
        const uint32_t r = orec[ba];
        su[m] = bu;
        sw[m] = (int)((r >> 16) & 0xFFu);
        sr[m] = (uint32_t)s | ((r >> 24) << 16) | ((r >> 16 & 0xFFu) << 24);
    }
    int nh = 0;
    if (two_hop && m < kseeds) {
        const int need = kseeds - m;
        int hu[3] = {-1, -1, -1};
        for (; nh < need; nh++) {
            double bx = INFINITY;
            int bu = INT_MAX;
            uint32_t br = UINT_MAX;
            int bo = 0;
            for (int a = a0; a < a1; a++) {
                const uint32_t ra = orec[a];
                const int x = (int)(ra & 0xFFFFu);
                if (x == s || row[x + 1] - row[x] > hop_deg) continue;
                const int wa = (int)((ra >> 16) & 0xFFu);
                for (int b = row[x] + lane; b < row[x + 1]; b += 64) {
                    const uint32_t rb = orec[b];
                    const int u = (int)(rb & 0xFFFFu);
                    if (u == s || u == x || rk[u] >= rks || !avail[u]) continue;
                    if (picked(u) || u == hu[0] || u == hu[1] || u == hu[2]) continue;
                    const int wb = (int)((rb >> 16) & 0xFFu);
                    const double cost = (double)wa + (double)wb + close[u];
                    const uint32_t rec = (uint32_t)x | ((rb >> 24) << 16) | ((uint32_t)wb << 24);
                    if (cost < bx || (cost == bx && (u < bu || (u == bu && rec < br)))) { bx = cost; bu = u; br = rec; bo = wa + wb; }
                }
            }
            const double x0 = bx;
            const int u0 = bu;
            const uint32_t r0 = br;
            wave_min3(bx, bu, br);
            if (br == UINT_MAX && bu == INT_MAX) break;
            // the winning lane's w(s,x) + w(x,u)
            const bool mine = x0 == bx && u0 == bu && r0 == br;
            const unsigned long long bal = __ballot(mine);
            bo = __shfl(bo, __ffsll((long long)bal) - 1);
            hu[nh] = bu;
            su[m + nh] = bu;
            sw[m + nh] = bo;
            sr[m + nh] = br;
        }
    }
    if (lane == 0) {
        PlanChoice o;
        o.m = m; o.nh = nh;
        o.pad[0] = o.pad[1] = 0;
        for (int k = 0; k < PC_CAND; k++) {
            const bool v = k < m + nh;
            o.u[k] = v ? su[k] : 0; o.w[k] = v ? sw[k] : 0; o.rec[k] = v ? sr[k] : 0u;
        }
        out[q] = o;
    }
}

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
    int alloc(size_t b) { return hipMalloc(&p, b ? b : 1) == hipSuccess ? SHD_ROUTE_OK : SHD_ROUTE_ENOMEM; }
};

// Host-pointer wrapper: chunks rows so device output stays bounded, copies back.
template <typename Launch>
int host_rows(shd_route* c, const int32_t* src, int32_t ns, const int32_t* tgt, int32_t nt, double* lat_out,
              double* rel_out, double* row_min_out, Launch launch) {
    if (!c || ns < 0 || nt < 0 || (ns && !src) || (nt && !tgt)) return SHD_ROUTE_EINVAL;
    if (ns == 0) return SHD_ROUTE_OK;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    const size_t row_bytes = sizeof(double) * (size_t)std::max(nt, 1);
    int32_t chunk = (int32_t)std::max<size_t>(1, std::min<size_t>(ns, (size_t)(1u << 30) / row_bytes));
    DevBuf dsrc, dtgt, dlat, drel, dmin;
    int rc;
    if ((rc = dsrc.alloc(sizeof(int32_t) * chunk)) || (rc = dtgt.alloc(sizeof(int32_t) * std::max(nt, 1))) ||
        (rc = dlat.alloc(row_bytes * chunk)) || (rc = drel.alloc(row_bytes * chunk)) ||
        (rc = dmin.alloc(sizeof(double) * chunk)))
        return rc;
    if (nt && hipMemcpy(dtgt.p, tgt, sizeof(int32_t) * nt, hipMemcpyHostToDevice) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    int soft = SHD_ROUTE_OK;
    for (int32_t i0 = 0; i0 < ns; i0 += chunk) {
        int32_t k = std::min(chunk, ns - i0);
        if (hipMemcpy(dsrc.p, src + i0, sizeof(int32_t) * k, hipMemcpyHostToDevice) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
        rc = launch((const int32_t*)dsrc.p, k, (const int32_t*)dtgt.p, (double*)dlat.p, (double*)drel.p,
                    (double*)dmin.p);
        if (rc) return rc;
        // per-entry failures (missing self-loop, unreachable target) leave NaN in those
        // entries only: the rows are still copied out and the code returned at the end
        if ((rc = shd_route_sync(c, nullptr)) && rc != SHD_ROUTE_ENOEDGE && rc != SHD_ROUTE_EUNREACH) return rc;
        if (rc && !soft) soft = rc;
        if (lat_out && hipMemcpy(lat_out + (size_t)i0 * nt, dlat.p, row_bytes * k, hipMemcpyDeviceToHost) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
        if (rel_out && hipMemcpy(rel_out + (size_t)i0 * nt, drel.p, row_bytes * k, hipMemcpyDeviceToHost) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
        if (row_min_out && hipMemcpy(row_min_out + i0, dmin.p, sizeof(double) * k, hipMemcpyDeviceToHost) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
    }
    return soft;
}
}  // namespace

namespace {
int planned_host_rows(shd_route* c, const int32_t* src, int32_t ns, const int32_t* tgt, int32_t nt,
                      uint32_t flags, double* lat_out, double* rel_out, double* row_min_out);
}

extern "C" {

int shd_route_rows(shd_route_t* c, const int32_t* src, int32_t ns, const int32_t* tgt, int32_t nt,
                   uint32_t flags, double* lat_out, double* rel_out, double* row_min_out) {
    // many KD rows (at least one per resident workgroup slot, so the plan's landmark rows,
    // row store and table pay off): one seeded plan over all of them when the whole table
    // fits the device; small batches and any device allocation failure take the chunked rows
    if (c && c->sel == 4 && c->kd_fused && ns >= 2 && ns >= c->kd_slots && nt >= 1 && src && tgt &&
        !((flags & SHD_ROUTE_DISPATCH) && (c->complete || c->prefer_direct))) {
        const int rc = planned_host_rows(c, src, ns, tgt, nt, flags, lat_out, rel_out, row_min_out);
        if (rc != SHD_ROUTE_EUNSUPPORTED) return rc;
    }
    return host_rows(c, src, ns, tgt, nt, lat_out, rel_out, row_min_out,
                     [&](const int32_t* ds, int32_t k, const int32_t* dt, double* dl, double* dr, double* dm) {
                         return shd_route_rows_async(c, ds, k, dt, nt, nt, flags, dl, dr, dm, nullptr);
                     });
}

int shd_route_direct(shd_route_t* c, const int32_t* src, int32_t ns, const int32_t* tgt, int32_t nt,
                     double* lat_out, double* rel_out, double* row_min_out) {
    if (!c) return SHD_ROUTE_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    int rc = ensure_dense(c);
    if (rc) return rc;
    return host_rows(c, src, ns, tgt, nt, lat_out, rel_out, row_min_out,
                     [&](const int32_t* ds, int32_t k, const int32_t* dt, double* dl, double* dr, double* dm) {
                         int grid = std::min(k, 65535);
                         hipLaunchKernelGGL(direct_rows_kernel, dim3(grid), dim3(kBlock), 0, nullptr, c->n, c->d_W,
                                            c->d_R, c->d_vf, ds, k, dt, nt, (long long)nt, dl, dr, dm, c->d_err);
                         return hip_check(hipGetLastError());
                     });
}

int shd_route_self(shd_route_t* c, const int32_t* v, int32_t nv, double* lat_out, double* rel_out) {
    if (!c || nv < 0 || (nv && (!v || !lat_out || !rel_out))) return SHD_ROUTE_EINVAL;
    if (nv == 0) return SHD_ROUTE_OK;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    DevBuf dv, dl, dr;
    int rc;
    if ((rc = dv.alloc(sizeof(int32_t) * nv)) || (rc = dl.alloc(sizeof(double) * nv)) ||
        (rc = dr.alloc(sizeof(double) * nv)))
        return rc;
    if (hipMemcpy(dv.p, v, sizeof(int32_t) * nv, hipMemcpyHostToDevice) != hipSuccess) return SHD_ROUTE_EDEVICE;
    DevGraph g = dev_graph(c);
    hipLaunchKernelGGL(self_kernel, dim3((nv + 255) / 256), dim3(256), 0, nullptr, g, (const int*)dv.p, nv,
                       (double*)dl.p, (double*)dr.p, c->d_err);
    if ((rc = hip_check(hipGetLastError()))) return rc;
    if ((rc = shd_route_sync(c, nullptr))) return rc;
    if (hipMemcpy(lat_out, dl.p, sizeof(double) * nv, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(rel_out, dr.p, sizeof(double) * nv, hipMemcpyDeviceToHost) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    return SHD_ROUTE_OK;
}

int shd_route_min_reduce_async(shd_route_t* c, const double* d_vals, int64_t count, double* d_out, void* stream) {
    if (!c || count < 0 || !d_out || (count && !d_vals)) return SHD_ROUTE_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (count <= kMinOneBlock) {  // one launch, no clearing memset
        hipLaunchKernelGGL(min_reduce_block_kernel, dim3(1), dim3(1024), 0, st, d_vals, (long long)count,
                           (unsigned long long*)d_out);
        return hip_check(hipGetLastError());
    }
    if (hipMemsetAsync(d_out, 0xFF, sizeof(double), st) != hipSuccess) return SHD_ROUTE_EDEVICE;
    long long blocks = std::min<long long>((count + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(min_reduce_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, d_vals, (long long)count,
                       (unsigned long long*)d_out);
    return hip_check(hipGetLastError());
}

int shd_route_fw_async(shd_route_t* c, double* d_dist, void* stream) {
    if (!c || !d_dist) return SHD_ROUTE_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    const int n = c->n;
    const int nb = (n + kT - 1) / kT;
    for (int kb = 0; kb < nb; kb++) {
        const int k0 = kb * kT;
        hipLaunchKernelGGL(fw_diag_kernel, dim3(1), dim3(kT * 8), 0, st, d_dist, n, k0);
        if (nb > 1)
            hipLaunchKernelGGL(fw_panel_kernel, dim3(nb - 1, 2), dim3(kT * 8), 0, st, d_dist, n, k0);
        hipLaunchKernelGGL(fw_rest_kernel, dim3(nb, nb), dim3(kT * 8), 0, st, d_dist, n, k0);
    }
    return hip_check(hipGetLastError());
}

}  // extern "C"

// =============================================================================
// Seeded planning (shd_route_plan_*): which row seeds which, and in which launch.
// =============================================================================
struct shd_route_plan {
    shd_route* c = nullptr;
    int world = 1, rank = 0, ns_all = 0;
    int seeded = 0, nroots = 0, nhelpers = 0, nslots = 0;
    int delta = 1;                 // bucket width of the rows (<= the context's kd_delta)
    int nland = 0;                 // landmark seed rows after the kept rows' slots (flags preset)
    std::vector<int32_t> row_pos;  // caller-list position of each output row of this rank
    std::vector<int> lvl_off;      // jobs of launch k: [lvl_off[k], lvl_off[k + 1])
    KDJob* d_jobs = nullptr;
    int* d_next = nullptr;         // the launch's job-queue counter + one ready flag per kept row
    int32_t* d_src = nullptr;      // unseeded plans: the source vertex of each row
    uint16_t* d_drow = nullptr;    // row store
    uint32_t* d_prow = nullptr;
    uint64_t store_bytes = 0;
    // Landmark-only plans built on the device (round 6: their landmark rows are part of every
    // launch): shd_route_rows_planned_async first recomputes the nhub landmark rows into the
    // plan's own store (one hub-row launch, jobs d_hjobs, ready flags d_hdone), then the queue
    // order and the job records from them (plan_lmall_* kernels over d_sq / d_lv / d_key /
    // d_slot), then the rows: every SSSP the table needs runs inside the launch sequence.
    bool lm_step = false;
    int nhub = 0, hub_grid = 0, klm = 0;
    bool hub1024 = false;
    // multi-GPU landmark-only plans: this rank's share of the landmark rows (slots
    // [lm_first, lm_first + lm_count), equal shares), the rest all-gathered from the other
    // ranks by the caller (shd_route_plan_refresh_async with SHD_ROUTE_REFRESH_MINE, then the
    // exchange into the store, then SHD_ROUTE_REFRESH_JOBS)
    int lm_first = 0, lm_count = 0;
    int lm2 = 0;                   // > 0: landmark rows in two levels (SHD_ROUTE_LM2, lm_refresh)
    bool order_fixed = false;      // the queue order (d_slot) is computed; refreshes keep it
    uint16_t* d_bias = nullptr;    // the landmarks' pick biases (lm_pick; null: nearest first)
    int spread = 1;                // seeds picked spread apart (lm_pick; SHD_ROUTE_LMSPREAD=0: nearest-biased)
    KDJob* d_hjobs2 = nullptr;     // (the second level's jobs, written on the device)
    bool store_external = false;   // d_drow / d_prow are the caller's (shd_route_plan_bind_store)
    KDJob* d_hjobs = nullptr;
    int* d_hdone = nullptr;
    int* d_sq = nullptr;
    int* d_lv = nullptr;
    int* d_slot = nullptr;
    unsigned long long* d_key = nullptr;
    ~shd_route_plan() {
        for (void* q : {(void*)d_jobs, (void*)d_next, (void*)d_src, (void*)d_hjobs, (void*)d_hjobs2, (void*)d_bias,
                        (void*)d_hdone, (void*)d_sq, (void*)d_lv, (void*)d_slot, (void*)d_key})
            if (q) (void)hipFree(q);
        if (!store_external)
            for (void* q : {(void*)d_drow, (void*)d_prow})
                if (q) (void)hipFree(q);
    }
};

namespace {

// landmark-only plans: at most this many rows per workgroup slot, and their landmark count
constexpr double PLAN_LMALL_RPS = 1.5;
// (round 5, hub rows outside the step: C3 1 GPU 256 / 512 / 1024 / 2048 landmarks 2.49 / 2.30 /
//  2.18 / 2.07 ms of rows.  Round 6, the landmark rows inside every step: 512 / 768 / 1024 give
//  2.677 / 2.69 / 2.77 ms per step (rows 2.14 / 2.05 / 1.99 + landmark rows and job records
//  0.55 / 0.65 / 0.79), two runs each on one box)
constexpr int PLAN_LMALL_COUNT = 448;

// host threads of a plan (the box's CPU quota is 16)
int plan_threads() {
    int nth = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    if (const char* e = getenv("SHD_ROUTE_PLAN_THREADS")) nth = std::max(1, std::min(64, atoi(e)));
    return nth;
}
// the process-wide planner workers (created once; none when one host thread is asked for)
HostPool* host_pool() {
    std::lock_guard<std::mutex> l(g_pool_mu);
    if (!g_pool && plan_threads() > 1) g_pool.reset(new HostPool(plan_threads() - 1));
    return g_pool.get();
}

// Exact rows of `verts` on the device for the planner: one unplanned KD launch whose jobs
// write no output row (row -1) but keep their row in store slot k, the format seeded rows
// read (u16 distances, 0xFFFF = unreached, and the engine tie-rule parent record
// `parent | ridx << 16 | w << 24` of every vertex).  The store stays in dd / dp (device) and
// is copied back into d_out / p_out.  Blocks: the planner runs once per context, before any
// planned launch.
int device_store_rows(shd_route* c, const std::vector<int>& verts, DevBuf& dd, DevBuf& dp, std::vector<uint16_t>& hd,
                      int ncopy) {
    const int k = (int)verts.size(), n = c->n;
    if (k == 0) return SHD_ROUTE_OK;
    const auto h0 = std::chrono::steady_clock::now();
    auto hs = [&]() { return 1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count(); };
    double h_alloc = 0, h_launch = 0, h_copy = 0;
    const long long rs = kd_row_stride(n);
    std::vector<KDJob> jobs(k);
    for (int q = 0; q < k; q++) {
        std::memset(&jobs[q], 0, sizeof(KDJob));
        jobs[q].row = -1; jobs[q].s = verts[q]; jobs[q].store = q; jobs[q].nseed = 0;
    }
    // one round of workgroups for all k rows (each row is unseeded: k rows on fewer
    // workgroups take k / grid row latencies): up to 256 rows in 1024-thread workgroups, one
    // per CU, and more in the context's own (256-thread contexts: four per CU, each row only
    // ~25% slower: C3's 512 hub rows 1.0 ms in two rounds of 1024-thread rows).  The launch
    // has its own per-workgroup scratch: the context's is left to its rows launches, so none
    // of those can share it even if one is still in flight.
    const bool hub1024 = c->kd_hub_block > 0 && k <= 256;
    const int grid = std::min(k, hub1024 ? 256 : std::max(256, c->kd_slots));
    DevBuf dj, dn;
    if (dj.alloc(sizeof(KDJob) * k) || dd.alloc(sizeof(uint16_t) * (size_t)rs * k) ||
        dp.alloc(sizeof(uint32_t) * (size_t)rs * k) || dn.alloc(sizeof(int) * (1 + (size_t)k)))
        return SHD_ROUTE_ENOMEM;
    const size_t wsb = c->kd_stride * (size_t)grid;
    if (c->hub_ws_bytes < wsb) {
        if (c->d_hub_ws) (void)hipFree(c->d_hub_ws);
        c->d_hub_ws = nullptr; c->hub_ws_bytes = 0;
        if (hipMalloc((void**)&c->d_hub_ws, wsb) != hipSuccess) { c->d_hub_ws = nullptr; return SHD_ROUTE_ENOMEM; }
        c->hub_ws_bytes = wsb;
    }
    // (errors of earlier launches are reported by their own sync, not by this plan)
    if (hipDeviceSynchronize() != hipSuccess) return SHD_ROUTE_EDEVICE;
    int rc = take_err(c);
    if (rc) return rc;
    h_alloc = hs();
    if (hipMemcpy(dj.p, jobs.data(), sizeof(KDJob) * k, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(dn.p, 0, sizeof(int) * (1 + (size_t)k)) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    DevDelta g = kd_args(c);
    g.jobs = (const KDJob*)dj.p;
    g.drow = (const uint16_t*)dd.p; g.drow_out = (uint16_t*)dd.p; g.prow = (uint32_t*)dp.p; g.rstride = rs;
    g.done = (int*)dn.p + 1;
    if ((rc = kd_launch(c, g, (int*)dn.p, nullptr, k, nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr, true,
                        c->d_hub_ws, grid, hub1024)))
        return rc;
    if (hipDeviceSynchronize() != hipSuccess) return SHD_ROUTE_EDEVICE;
    if ((rc = take_err(c))) return rc;
    h_launch = hs();
    // only the rows the host reads (the closeness rows' distances): the landmark rows stay on
    // the device, where the plan's landmark-seed kernel reads them (copying 512 rows of C3 to
    // pageable memory took 6 ms); ensure_lm_host copies them for the host fallback
    ncopy = std::min(ncopy, k);
    hd.resize((size_t)rs * ncopy);
    if (ncopy && hipMemcpy(hd.data(), dd.p, sizeof(uint16_t) * hd.size(), hipMemcpyDeviceToHost) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    h_copy = hs();
    if (getenv("SHD_ROUTE_PLAN_DEBUG"))
        fprintf(stderr, "hub rows (%d): alloc+sync %.2f, launch done %.2f, copies done %.2f ms\n", k, h_alloc, h_launch, h_copy);
    return SHD_ROUTE_OK;
}

// The planner's device rows, once per context, in one launch: the rows of the k highest-degree
// vertices (the hubs of a BA-like topology; ties by id).  The first 16 give every vertex's
// closeness estimate (its mean distance to them); all k are the landmark rows that seed the
// plans' roots, kept on the device in the row-store format (a plan copies them device to
// device).  (Before round 3: 16 pseudo-random closeness rows, then the 16 (64) most central
// vertices' rows in a second launch.)
// the k highest-degree vertices (ties by id): the hub / landmark rows
std::vector<int> hub_vertices(const shd_route* c, int k) {
    const int n = c->n;
    std::vector<int> ord(n);
    std::iota(ord.begin(), ord.end(), 0);
    auto deg = [&](int v) { return c->h_row.empty() ? 0 : c->h_row[v + 1] - c->h_row[v]; };
    std::partial_sort(ord.begin(), ord.begin() + k, ord.end(), [&](int a, int b) {
        return deg(a) != deg(b) ? deg(a) > deg(b) : a < b;
    });
    return std::vector<int>(ord.begin(), ord.begin() + k);
}

int ensure_hub_rows(shd_route* c, int k, bool host_close = true) {
    const int n = c->n;
    k = std::min(n, std::max(k, 16));
    const int L = std::min(n, 16);  // the closeness rows: the first 16 hub rows
    const long long rs = kd_row_stride(n);
    std::vector<uint16_t> hd;
    if ((int)c->lm_v.size() < k) {
        std::vector<int> lv = hub_vertices(c, k);
        DevBuf dd, dp;
        int rc = device_store_rows(c, lv, dd, dp, hd, host_close ? L : 0);
        if (rc) return rc;
        // (no plan keeps a pointer to these rows -- a plan copies them into its own store --
        // so the previous ones are freed; hipFree waits for work still reading them)
        if (c->d_lm_drow) (void)hipFree(c->d_lm_drow);
        if (c->d_lm_prow) (void)hipFree(c->d_lm_prow);
        c->d_lm_drow = (uint16_t*)dd.p; dd.p = nullptr;
        c->d_lm_prow = (uint32_t*)dp.p; dp.p = nullptr;
        c->lm_v = lv;
        c->lm_hd.clear();  // (host copies on demand: ensure_lm_host)
        c->lm_hp.clear();
        c->lm_rs = rs;
        c->close.clear();
        if (!host_close) return SHD_ROUTE_OK;
    } else {
        if (!host_close || (int)c->close.size() == n) return SHD_ROUTE_OK;
        hd.resize((size_t)rs * L);  // (rows computed by a device-built plan: their closeness now)
        if (hipMemcpy(hd.data(), c->d_lm_drow, sizeof(uint16_t) * hd.size(), hipMemcpyDeviceToHost) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
    }
    c->close.assign(n, 0.0);
    for (int v = 0; v < n; v++) {
        double sum = 0;
        for (int q = 0; q < L; q++) {
            const uint16_t x = hd[(size_t)q * rs + v];
            sum += x == 0xFFFFu ? INFINITY : (double)x;
        }
        c->close[v] = sum / L;
    }
    return SHD_ROUTE_OK;
}
int ensure_landmarks(shd_route* c, int k) { return ensure_hub_rows(c, k); }

// the landmark rows on the host (the plan's host fallback for landmark seeds)
int ensure_lm_host(shd_route* c) {
    const size_t cnt = (size_t)c->lm_rs * c->lm_v.size();
    if (c->lm_hd.size() == cnt && c->lm_hp.size() == cnt) return SHD_ROUTE_OK;
    c->lm_hd.resize(cnt);
    c->lm_hp.resize(cnt);
    if (hipMemcpy(c->lm_hd.data(), c->d_lm_drow, sizeof(uint16_t) * cnt, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(c->lm_hp.data(), c->d_lm_prow, sizeof(uint32_t) * cnt, hipMemcpyDeviceToHost) != hipSuccess) {
        c->lm_hd.clear(); c->lm_hp.clear();
        return SHD_ROUTE_EDEVICE;
    }
    return SHD_ROUTE_OK;
}

// A device-built landmark-only plan's in-launch work (shd_route_plan::lm_step), enqueued on
// st: the landmark rows into the plan's store, then the queue order and the job records
// from them.  No host synchronisation: errors surface at the next shd_route_sync.
// the hub-row launch's grid for k rows: up to 256 in 1024-thread workgroups (one per CU) where
// the context's are smaller, more in the context's own
inline bool hub_big(const shd_route* c, int k) { return c->kd_hub_block > 0 && k <= 256; }
inline int hub_grid(const shd_route* c, int k) { return std::min(k, hub_big(c, k) ? 256 : std::max(256, c->kd_slots)); }

int lm_refresh(shd_route* c, const shd_route_plan* P, uint32_t what, hipStream_t st) {
    const int n = c->n, nj = (int)P->row_pos.size();
    const long long rs = kd_row_stride(n);
    if (!what) what = SHD_ROUTE_REFRESH_ALL | SHD_ROUTE_REFRESH_JOBS;
    if ((what & SHD_ROUTE_REFRESH_ALL) && P->lm2 > 0) {
        // two levels: the first lm2 landmark rows unseeded in 1024-thread workgroups (one per
        // CU), then the others seeded from their three nearest of those (the main rows' seeding
        // rule, as the plan_lmall_jobs_kernel writes it), in the context's workgroups
        const int k0 = P->lm2, k1 = P->nhub - P->lm2;
        if (!c->d_hub_ws || c->hub_ws_bytes < c->kd_stride * (size_t)std::max(hub_grid(c, k0), hub_grid(c, k1)))
            return SHD_ROUTE_EINVAL;
        if (hipMemsetAsync(P->d_hdone, 0, sizeof(int) * (1 + (size_t)P->nhub), st) != hipSuccess) return SHD_ROUTE_EDEVICE;
        DevDelta g = kd_args(c);
        g.jobs = P->d_hjobs;
        g.drow = P->d_drow; g.drow_out = P->d_drow; g.prow = P->d_prow; g.rstride = rs;
        g.done = P->d_hdone + 1;
        int rc = kd_launch(c, g, P->d_hdone, nullptr, k0, nullptr, 0, 0, nullptr, nullptr, nullptr, st, true,
                           c->d_hub_ws, hub_grid(c, k0), hub_big(c, k0));
        if (rc) return rc;
        hipLaunchKernelGGL(plan_lmall_jobs_kernel, dim3(8 * (((k1 + 15) / 16 + 7) / 8)), dim3(1024), 0, st, P->d_drow,
                           P->d_prow, rs, P->d_lv, k0, P->d_lv + k0, (const int*)nullptr, k1, P->klm, n, P->d_hjobs2,
                           (int*)nullptr, k0);
        if (hipMemsetAsync(P->d_hdone, 0, sizeof(int), st) != hipSuccess) return SHD_ROUTE_EDEVICE;  // (queue only)
        g.jobs = P->d_hjobs2;
        rc = kd_launch(c, g, P->d_hdone, nullptr, k1, nullptr, 0, 0, nullptr, nullptr, nullptr, st, true,
                       c->d_hub_ws, std::min(k1, c->kd_slots), false);
        if (rc) return rc;
    } else if ((what & SHD_ROUTE_REFRESH_ALL) || (what & SHD_ROUTE_REFRESH_MINE)) {
        const bool all = (what & SHD_ROUTE_REFRESH_ALL) != 0;
        const int q0 = all ? 0 : P->lm_first, k = all ? P->nhub : P->lm_count;
        // (the hub-row launch's scratch: the context's, grown at plan creation to this grid)
        if (!c->d_hub_ws || c->hub_ws_bytes < c->kd_stride * (size_t)hub_grid(c, k)) return SHD_ROUTE_EINVAL;
        if (hipMemsetAsync(P->d_hdone, 0, sizeof(int) * (1 + (size_t)P->nhub), st) != hipSuccess) return SHD_ROUTE_EDEVICE;
        DevDelta g = kd_args(c);
        g.jobs = P->d_hjobs + q0;  // (a job's store slot is its global landmark index)
        g.drow = P->d_drow; g.drow_out = P->d_drow; g.prow = P->d_prow; g.rstride = rs;
        g.done = P->d_hdone + 1;
        const int rc = kd_launch(c, g, P->d_hdone, nullptr, k, nullptr, 0, 0, nullptr, nullptr, nullptr, st, true,
                                 c->d_hub_ws, hub_grid(c, k), hub_big(c, k));
        if (rc) return rc;
    }
    if (!(what & SHD_ROUTE_REFRESH_JOBS)) return SHD_ROUTE_OK;
    // the queue order (peripheral rows first, by the closeness the first 16 landmark rows
    // give) is the plan's schedule: fixed when the plan is made, like a neighbour-seeded
    // plan's list schedule (the rank sort took 0.13 ms of every C3 step); the job records --
    // each row's nearest landmarks, its offsets d(s, L) and L's record in s's tree -- are
    // derived from the landmark rows in every refresh
    if (!P->order_fixed) {
        if (hipMemsetAsync(P->d_next, 0, sizeof(int), st) != hipSuccess) return SHD_ROUTE_EDEVICE;  // (root count)
        const int nb = (nj + 255) / 256;
        hipLaunchKernelGGL(plan_lmall_keys_kernel, dim3(nb), dim3(256), 0, st, P->d_drow, rs, std::min(n, 16), P->d_sq,
                           nj, P->d_key);
        hipLaunchKernelGGL(plan_lmall_rank_kernel, dim3(nb), dim3(256), 8 * nj, st, P->d_key, nj, P->d_slot);
    }
    if (P->d_bias)
        hipLaunchKernelGGL(plan_lmall_bias_kernel, dim3((P->nhub + 255) / 256), dim3(256), 0, st, P->d_drow, rs,
                           std::min(P->nhub, 16), P->d_lv, P->nhub, P->d_bias);
    hipLaunchKernelGGL(plan_lmall_jobs_kernel, dim3(8 * (((nj + 15) / 16 + 7) / 8)), dim3(1024), 0, st, P->d_drow,
                       P->d_prow, rs, P->d_lv, P->nhub, P->d_sq, P->d_slot, nj, P->klm, n, P->d_jobs,
                       P->order_fixed ? (int*)nullptr : P->d_next, -1, (const uint16_t*)P->d_bias, P->spread);
    return hip_check(hipGetLastError());
}

}  // namespace

extern "C" {

int shd_route_plan_create(shd_route_t* c, const int32_t* src, int32_t ns, int32_t world, int32_t rank,
                          shd_route_plan_t** out) {
    if (!c || !out || ns < 0 || (ns && !src) || world < 1 || rank < 0 || rank >= world) return SHD_ROUTE_EINVAL;
    *out = nullptr;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    for (int p = 0; p < ns; p++) if (src[p] < 0 || src[p] >= c->n) return SHD_ROUTE_EINVAL;
    auto P = std::make_unique<shd_route_plan>();
    P->c = c; P->world = world; P->rank = rank; P->ns_all = ns;
    // bucket width of the plan's rows: any width up to the context's is exact (the light
    // in-CSR holds every in-arc below the context's width).  Round 5 read its builds as
    // "split ranks prefer the 12th percentile (30 on C4)"; the direct A/B on one box with
    // this per-plan width says otherwise (C4 8-way emulated, shared context, two runs each:
    // 30 -> 8.95 / 8.97 ms max, 38 -> 8.73 / 8.72 ms), so every plan keeps the context's;
    // SHD_ROUTE_PLAN_DELTA narrows it (tests, A/B runs)
    P->delta = c->kd_delta;
    if (const char* e = getenv("SHD_ROUTE_PLAN_DELTA")) P->delta = std::max(1, std::min(c->kd_delta, atoi(e)));
    const auto t_start = std::chrono::steady_clock::now();
    double t_close = 0, t_land = 0, t_seeds = 0, t_store = 0, t_sched = 0, t_rk = 0, t_order = 0, t_hop = 0, t_loop0 = 0, t_alloc = 0, t_deps = 0;
    int n_recomp = 0;  // SHD_ROUTE_PLAN_DEBUG stage times
    auto since = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
    const int n = c->n;
    const char* env = getenv("SHD_ROUTE_SEED");
    const bool want = (!env || atoi(env) != 0) && c->sel == 4 && c->kd_fused && !c->complete && !c->prefer_direct &&
                      ns >= 2 && !c->h_row.empty();
    // closeness rank of every vertex: a row may only be seeded by rows of smaller rank
    std::vector<int> rk;
    // landmark rows (below): 16 for 1024-thread plans, 64 for 256-thread ones; computed in the
    // same device launch as the closeness rows (ensure_hub_rows)
    int nland = c->multigraph ? 0 : std::min(c->kd_block >= 1024 ? 16 : 64, n);
    // Landmark-only plans (round 5): when a rank has few rows per workgroup slot, seed chains
    // make its time a few serial row latencies (C3 8-way: 1.2 rows per slot, 3-4 levels, 28% of
    // linear); every row then seeds from its 3 nearest of PLAN_LMALL_COUNT landmark rows
    // instead (all at level 0: no waits, no chains).  Multi-GPU ranks with chains take 256
    // landmarks for their roots (C4 8-way 9.08 -> 8.77 ms with 3 landmark seeds each; 256 hub
    // rows cost the plan what 16 do: one unseeded row per CU, in parallel).
    double lmall_rps = PLAN_LMALL_RPS;
    if (const char* e = getenv("SHD_ROUTE_LMALL")) lmall_rps = atof(e);
    // (256-thread contexts, n <= 16384: PLAN_LMALL_COUNT landmarks are >= 3% of the vertices,
    // and the 3 nearest bound a row better than its neighbour rows: C3 1 GPU 2.51 -> 2.30 ms
    // with 512, 8-way 1.12 -> 0.65 ms)
    int lmall_small = 1;
    if (const char* e = getenv("SHD_ROUTE_LMALL_SMALL")) lmall_small = atoi(e);
    const bool lm_all = !c->multigraph && c->kd_slots > 0 &&
                        ((lmall_small && c->kd_block < 1024 && n >= 2048) ||
                         (double)ns / world <= lmall_rps * (double)c->kd_slots);
    if (lm_all) nland = std::min(n, PLAN_LMALL_COUNT);
    else if (world > 1 && !c->multigraph) nland = std::min(n, 256);
    if (const char* e = getenv("SHD_ROUTE_LANDMARKS")) nland = c->multigraph ? 0 : std::max(0, std::min(atoi(e), n));
    // A landmark-only plan is built on the device (round 5): the hub rows without their host
    // closeness, then one kernel for the queue order and one for the job records, and one
    // sync at the end; the plan borrows the context's landmark rows as its row store (no
    // kept rows, no copies).  C3: plan 2.6 -> ~1.3 ms.  The host build below stays for
    // SHD_ROUTE_GPUCHOICE=0 / SHD_ROUTE_LMALL_REV=0 / SHD_ROUTE_PLANDEV=0 and larger ranks.
    auto env_off = [](const char* k) { const char* e = getenv(k); return e && atoi(e) == 0; };
    const int nmine = ns > rank ? (ns - rank + world - 1) / world : 0;
    if (want && lm_all && nland > 0 && nmine >= 2 && nmine <= PLAN_DEV_MAXJ && !env_off("SHD_ROUTE_GPUCHOICE") &&
        !env_off("SHD_ROUTE_LMALL_REV") && !env_off("SHD_ROUTE_PLANDEV")) {
        // Round 6: the landmark rows are computed inside every launch sequence of the plan
        // (lm_refresh), into the plan's own store; creating the plan runs that sequence once
        // (for the root count and to surface errors now), the rows launch reads its results.
        const int nh = std::min(n, std::max(nland, 16));
        const std::vector<int> lv = hub_vertices(c, nh);
        t_close = since();
        std::vector<int> sq;
        sq.reserve(nmine);
        for (int p = rank; p < ns; p += world) { P->row_pos.push_back(p); sq.push_back(src[p]); }
        const int nj = (int)sq.size();
        P->klm = KD_SEEDS;
        if (const char* e = getenv("SHD_ROUTE_LMSEEDS")) P->klm = std::max(1, std::min(KD_SEEDS, atoi(e)));
        const long long rs = kd_row_stride(n);
        P->nhub = nh;
        P->hub1024 = hub_big(c, nh);
        P->hub_grid = hub_grid(c, nh);
        // a rank's share of the landmark rows (equal shares; the last rank's is the rest)
        P->lm_count = (nh + world - 1) / world;
        P->lm_first = std::min(nh, rank * P->lm_count);
        P->lm_count = std::max(0, std::min(nh, P->lm_first + P->lm_count) - P->lm_first);
        std::vector<KDJob> hj(nh);
        for (int q = 0; q < nh; q++) {
            std::memset(&hj[q], 0, sizeof(KDJob));
            hj[q].row = -1; hj[q].s = lv[q]; hj[q].store = q; hj[q].nseed = 0;
        }
        if (const char* e = getenv("SHD_ROUTE_LM2")) {
            const int k0 = atoi(e);
            if (k0 >= 16 && k0 < nh) P->lm2 = k0;
        }
        const bool lmbias = !(getenv("SHD_ROUTE_LMBIAS") && atoi(getenv("SHD_ROUTE_LMBIAS")) == 0);
        if (getenv("SHD_ROUTE_LMSPREAD") && atoi(getenv("SHD_ROUTE_LMSPREAD")) == 0) P->spread = 0;
        if ((lmbias && hipMalloc((void**)&P->d_bias, sizeof(uint16_t) * (size_t)nh) != hipSuccess) ||
            (P->lm2 && hipMalloc((void**)&P->d_hjobs2, sizeof(KDJob) * (size_t)(nh - P->lm2)) != hipSuccess) ||
            hipMalloc((void**)&P->d_sq, sizeof(int) * nj) != hipSuccess ||
            hipMalloc((void**)&P->d_lv, sizeof(int) * nh) != hipSuccess ||
            hipMalloc((void**)&P->d_slot, sizeof(int) * nj) != hipSuccess ||
            hipMalloc((void**)&P->d_key, sizeof(unsigned long long) * nj) != hipSuccess ||
            hipMalloc((void**)&P->d_hjobs, sizeof(KDJob) * nh) != hipSuccess ||
            hipMalloc((void**)&P->d_hdone, sizeof(int) * (1 + (size_t)nh)) != hipSuccess ||
            hipMalloc((void**)&P->d_drow, sizeof(uint16_t) * (size_t)rs * nh) != hipSuccess ||
            hipMalloc((void**)&P->d_prow, sizeof(uint32_t) * (size_t)rs * nh) != hipSuccess ||
            hipMalloc((void**)&P->d_jobs, sizeof(KDJob) * (size_t)nj) != hipSuccess ||
            hipMalloc((void**)&P->d_next, sizeof(int) * (1 + (size_t)nh)) != hipSuccess)
            return SHD_ROUTE_ENOMEM;
        const size_t wsb = c->kd_stride * (size_t)std::max(std::max(P->hub_grid, hub_grid(c, std::max(1, P->lm_count))),
                                                           P->lm2 ? std::max(hub_grid(c, P->lm2), std::min(nh - P->lm2, c->kd_slots)) : 0);
        if (c->hub_ws_bytes < wsb) {
            if (c->d_hub_ws) (void)hipFree(c->d_hub_ws);
            c->d_hub_ws = nullptr; c->hub_ws_bytes = 0;
            if (hipMalloc((void**)&c->d_hub_ws, wsb) != hipSuccess) { c->d_hub_ws = nullptr; return SHD_ROUTE_ENOMEM; }
            c->hub_ws_bytes = wsb;
        }
        if (hipMemcpy(P->d_sq, sq.data(), sizeof(int) * nj, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(P->d_lv, lv.data(), sizeof(int) * nh, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(P->d_hjobs, hj.data(), sizeof(KDJob) * nh, hipMemcpyHostToDevice) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
        int rc;
        if ((rc = hip_check(hipFuncSetAttribute((const void*)plan_lmall_rank_kernel,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, 8 * nj))))
            return rc;
        P->row_pos.shrink_to_fit();
        // (errors of earlier launches are reported by their own sync, not by this plan)
        if (hipDeviceSynchronize() != hipSuccess) return SHD_ROUTE_EDEVICE;
        if ((rc = take_err(c))) return rc;
        if ((rc = lm_refresh(c, P.get(), 0, nullptr))) return rc;
        int nroots = 0;
        if (hipMemcpy(&nroots, P->d_next, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return SHD_ROUTE_EDEVICE;
        if ((rc = take_err(c))) return rc;
        P->lm_step = true;
        P->order_fixed = !(getenv("SHD_ROUTE_LMORDER") && atoi(getenv("SHD_ROUTE_LMORDER")) == 0);
        P->nslots = 0; P->nland = nh; P->store_bytes = (uint64_t)nh * (uint64_t)rs * 6u; P->nroots = nroots;
        P->seeded = 1;
        P->lvl_off = {0, nj};
        if (getenv("SHD_ROUTE_PLAN_DEBUG"))
            fprintf(stderr, "plan world %d rank %d: jobs %d levels 1, device-built landmark-only plan (%d landmarks, "
                    "%d unseeded), landmark rows in every launch: setup %.2f ms, plan total %.2f ms\n", world, rank, nj, nh, nroots,
                    1e3 * t_close, 1e3 * since());
        *out = P.release();
        return SHD_ROUTE_OK;
    }
    if (want) {
        const int rc = ensure_hub_rows(c, nland);
        if (rc) return rc;
        t_close = since();
        // rank by (closeness, vertex).  closeness is a mean of L integer distances, so L times
        // it is an exact integer sum: a counting sort over the sums, vertices ascending within
        // one (an std::sort of (double, int) pairs took ~3 ms at C4)
        rk.resize(n);
        const double L = (double)std::min(n, 16);
        bool integral = true;
        long long smax = 0;
        for (int v = 0; v < n && integral; v++) {
            const double x = c->close[v] * L;
            integral = x >= 0 && x < 1e8 && x == std::floor(x);
            if (integral) smax = std::max(smax, (long long)x);
        }
        if (integral) {
            std::vector<int> cnt((size_t)smax + 2, 0);
            for (int v = 0; v < n; v++) cnt[(size_t)(c->close[v] * L) + 1]++;
            for (long long x = 0; x <= smax; x++) cnt[x + 1] += cnt[x];
            for (int v = 0; v < n; v++) rk[v] = cnt[(size_t)(c->close[v] * L)]++;
        } else {
            std::vector<std::pair<double, int>> ord(n);
            for (int v = 0; v < n; v++) ord[v] = {c->close[v], v};
            std::sort(ord.begin(), ord.end());
            for (int q = 0; q < n; q++) rk[ord[q].second] = q;
        }
        t_rk = since();
    }
    auto by_rank = [&](std::vector<int>& v) {  // positions by (vertex rank, position): counting sort
        std::vector<int> cnt(n + 1, 0), tmp(v.size());
        std::vector<int> sv(v);
        if (!std::is_sorted(sv.begin(), sv.end())) std::sort(sv.begin(), sv.end());
        for (int p : sv) cnt[rk[src[p]] + 1]++;
        for (int x = 0; x < n; x++) cnt[x + 1] += cnt[x];
        for (int p : sv) tmp[cnt[rk[src[p]]]++] = p;
        v.swap(tmp);
    };
    // the best seeds of position p among the positions marked in `avail` (first[v]: the
    // available position of vertex v): neighbours of smaller rank by w(s,u) + closeness(u),
    // then vertex.  One pass keeping the k best in order (what a full sort of the
    // candidates would list first; a multigraph's repeated u keeps its best arc, the first
    // arc on a full tie): hubs have thousands of neighbours, k is at most 3.
    double alpha = 1.0;  // seed score w(s,u) + alpha * closeness(u)
    if (const char* e = getenv("SHD_ROUTE_SEEDALPHA")) alpha = atof(e);
    auto best_seeds = [&](int p, auto avail, int k, int* arc_out) {
        const int s = src[p];
        double sc[KD_SEEDS];
        int m = 0;
        for (int a = c->h_row[s]; a < c->h_row[s + 1]; a++) {
            const int u = c->h_col[a];
            if (u == s || !avail(u) || rk[u] >= rk[s]) continue;
            const double x = c->h_w[a] + alpha * c->close[u];
            int dq = -1;
            for (int q = 0; q < m; q++) if (c->h_col[arc_out[q]] == u) dq = q;
            if (dq >= 0) {
                if (!(x < sc[dq])) continue;
                for (int q = dq; q + 1 < m; q++) { sc[q] = sc[q + 1]; arc_out[q] = arc_out[q + 1]; }
                m--;
            }
            auto before = [&](int q) { return x != sc[q] ? x < sc[q] : u < c->h_col[arc_out[q]]; };
            if (m == k && !before(m - 1)) continue;
            int q = m < k ? m++ : k - 1;
            for (; q > 0 && before(q - 1); q--) { sc[q] = sc[q - 1]; arc_out[q] = arc_out[q - 1]; }
            sc[q] = x;
            arc_out[q] = a;
        }
        return m;
    };
    // ---- which positions this rank computes: output rows + helper rows ----------------
    std::vector<int> job_pos, job_row;
    if (want && world > 1 && lm_all) {
        // landmark-only plans seed from no other row: a rank takes every world-th position
        // (row costs vary with the vertex's place in the graph: a stride spreads them), no
        // helper rows
        for (int p = rank; p < ns; p += world) {
            job_row.push_back((int)P->row_pos.size()); P->row_pos.push_back(p); job_pos.push_back(p);
        }
    } else if (!want || world == 1) {
        // a contiguous block of the caller's list (world 1: all of it)
        const int blk = (ns + world - 1) / world, lo = std::min(ns, rank * blk), hi = std::min(ns, lo + blk);
        for (int p = lo; p < hi; p++) { P->row_pos.push_back(p); job_pos.push_back(p); job_row.push_back(p - lo); }
    } else {
        // Multi-GPU: partition the seed forest (each row's best seed) so that a rank holds
        // whole subtrees: every seed a row needs is then on its own rank.  The forest's
        // top levels (T) are computed on every rank (helper rows where not output there);
        // the subtrees hanging below T go to ranks by size (largest first, least loaded).
        std::vector<int> first(n, -1), pos(ns);
        for (int p = 0; p < ns; p++) if (first[src[p]] < 0) first[src[p]] = p;
        std::iota(pos.begin(), pos.end(), 0);
        by_rank(pos);
        std::vector<int> fpar(ns, -1), flvl(ns, 0), sub(ns, 1);
        // each row's best seed (the forest's parent): on the device, one wave per row (the
        // plan's seed-choice kernel with k = 1: ~1 ms with the copies at C4, against ~6 ms
        // of host CSR scans on every rank); SHD_ROUTE_GPUCHOICE=0 keeps the host scan
        std::vector<int> bu(ns, -1);
        bool dev_forest = !(getenv("SHD_ROUTE_GPUCHOICE") && atoi(getenv("SHD_ROUTE_GPUCHOICE")) == 0) &&
                          c->d_kd_orec != nullptr;
        if (dev_forest) {
            std::vector<uint8_t> av(n);
            for (int v = 0; v < n; v++) av[v] = first[v] >= 0;
            DevBuf dcl, drk, dav, dsq, dout;
            std::vector<PlanChoice> ho(ns);
            dev_forest = !dcl.alloc(sizeof(double) * n) && !drk.alloc(sizeof(int) * n) && !dav.alloc(n) &&
                         !dsq.alloc(sizeof(int) * ns) && !dout.alloc(sizeof(PlanChoice) * ns) &&
                         hipMemcpy(dcl.p, c->close.data(), sizeof(double) * n, hipMemcpyHostToDevice) == hipSuccess &&
                         hipMemcpy(drk.p, rk.data(), sizeof(int) * n, hipMemcpyHostToDevice) == hipSuccess &&
                         hipMemcpy(dav.p, av.data(), n, hipMemcpyHostToDevice) == hipSuccess &&
                         hipMemcpy(dsq.p, src, sizeof(int) * ns, hipMemcpyHostToDevice) == hipSuccess;
            if (dev_forest) {
                hipLaunchKernelGGL(plan_choice_kernel, dim3((ns + 3) / 4), dim3(256), 0, 0, c->d_row, c->d_kd_orec,
                                   (const double*)dcl.p, (const int*)drk.p, (const uint8_t*)dav.p, (const int*)dsq.p, ns,
                                   1, 0, 0, alpha, 1, (PlanChoice*)dout.p);
                dev_forest = hipGetLastError() == hipSuccess &&
                             hipMemcpy(ho.data(), dout.p, sizeof(PlanChoice) * ns, hipMemcpyDeviceToHost) == hipSuccess;
            }
            if (dev_forest)
                for (int p = 0; p < ns; p++) bu[p] = ho[p].m > 0 ? ho[p].u[0] : -1;
        }
        if (!dev_forest)
            for (int p = 0; p < ns; p++) {
                int a;
                bu[p] = best_seeds(p, [&](int u) { return first[u] >= 0; }, 1, &a) ? c->h_col[a] : -1;
            }
        int maxl = 0;
        for (int p : pos) {
            if (bu[p] >= 0) {
                fpar[p] = first[bu[p]];
                flvl[p] = flvl[fpar[p]] + 1;
            }
            maxl = std::max(maxl, flvl[p]);
        }
        for (int q = ns - 1; q >= 0; q--) if (fpar[pos[q]] >= 0) sub[fpar[pos[q]]] += sub[pos[q]];
        // T = the rows whose subtree holds more than a quarter of a rank's share (the
        // forest's skeleton near its roots); every other row hangs in a subtree of at most
        // that size whose head's parent is in T (or which is a whole small tree)
        int capdiv = 4;
        if (const char* e = getenv("SHD_ROUTE_TOPCAP")) capdiv = std::max(1, atoi(e));
        const int cap = std::max(1, ns / (capdiv * world));
        std::vector<int> top, heads;
        for (int p : pos) {
            if (sub[p] > cap) top.push_back(p);
            else if (fpar[p] < 0 || sub[fpar[p]] > cap) heads.push_back(p);
        }
        (void)maxl;
        std::stable_sort(heads.begin(), heads.end(), [&](int a, int b) { return sub[a] > sub[b]; });
        std::vector<int> owner(ns, -1);
        std::vector<long long> load(world, 0);
        auto least = [&]() { return (int)(std::min_element(load.begin(), load.end()) - load.begin()); };
        for (int h : heads) { const int r = least(); owner[h] = r; load[r] += sub[h]; }
        for (int p : top) { const int r = least(); owner[p] = r; load[r] += 1; }
        for (int p : pos) if (owner[p] < 0 && fpar[p] >= 0) owner[p] = owner[fpar[p]];  // (rank order: parent first)
        // rows of this rank: its share of T, then its subtrees, in rank order; helpers: T
        for (int p : pos)
            if (owner[p] == rank) { job_row.push_back((int)P->row_pos.size()); P->row_pos.push_back(p); job_pos.push_back(p); }
        for (int p : top)
            if (owner[p] != rank) { job_pos.push_back(p); job_row.push_back(-1); P->nhelpers++; }
    }
    const int nj = (int)job_pos.size(), nr = (int)P->row_pos.size();
    std::vector<KDJob> jobs;
    if (want && nj >= 2) {
        // jobs renumbered in rank order (a job's seeds, of smaller rank, are settled before
        // it), so that the passes below walk every per-job array in sequence
        {
            std::vector<int> jpos_of(ns, -1);
            for (int j = 0; j < nj; j++) jpos_of[job_pos[j]] = j;
            std::vector<int> order(job_pos);
            by_rank(order);
            std::vector<int> jr(nj);
            for (int q = 0; q < nj; q++) jr[q] = job_row[jpos_of[order[q]]];
            job_pos.swap(order);
            job_row.swap(jr);
            // (landmark-only plans have no seed order to keep: the peripheral rows, the costliest
            // to bound from landmarks, go first, so the launch ends on cheap central ones: C3
            // 2.18 -> 2.12 ms, 8-way 0.63 -> 0.61 ms; SHD_ROUTE_LMALL_REV=0 keeps rank order)
            if (lm_all && !(getenv("SHD_ROUTE_LMALL_REV") && atoi(getenv("SHD_ROUTE_LMALL_REV")) == 0)) {
                std::reverse(job_pos.begin(), job_pos.end());
                std::reverse(job_row.begin(), job_row.end());
            }
        }
        std::vector<int> first(n, -1);  // first job of each source vertex
        for (int j = 0; j < nj; j++) if (first[src[job_pos[j]]] < 0) first[src[job_pos[j]]] = j;
        const std::vector<int>& order = job_pos;
        t_order = since();
        std::vector<int> lvl(nj, 0), slot(nj, -1), nsd(nj, 0);
        std::vector<std::array<int, KD_SEEDS>> seedjob(nj), su(nj), wr(nj);
        // options: seeds per row (1..KD_SEEDS), the `roots` most central rows start
        // unseeded (default: one per workgroup slot, so the launch starts full and the
        // seed chains below them are short: C4 1 GPU 52.9 -> 51.0 ms, an 8-way rank
        // 12.8 -> 10.0 ms, C3 4.0 -> 3.4 ms), and seed chains are at most `depth` rows long
        // default depth cap: about half the rows each workgroup slot runs in turn, so that
        // seed chains are shorter than a slot's queue, and at least 8 (C4: 195 rows per
        // slot, no cap in effect; C3: 9 per slot, cap 8: 3.5 -> 3.1 ms against cap 4)
        // (seeds per row: three, C4 48.6 -> 48.1 ms; on 256-thread rows, whose init pass costs
        // relatively more, two measured better in round 2 (C3 3.00 vs 3.07 ms) and three since
        // the streamed init of round 3 (round 4: C3 2.74 -> 2.67 ms))
        // (multi-GPU ranks: two; a rank's third candidates are mostly two-hop rows, and the
        // extra init pass costs more than they save: 8-way C4 rank 9.6 vs 9.4 ms with three)
        int kseeds = std::min(KD_SEEDS, world == 1 ? 3 : 2), nroot_min = lm_all && nland > 0 ? nj : c->kd_slots;
        int depth = std::max(8, nj / std::max(1, 2 * c->kd_slots));
        if (const char* e = getenv("SHD_ROUTE_SEEDS")) kseeds = std::max(1, std::min(KD_SEEDS, atoi(e)));
        if (const char* e = getenv("SHD_ROUTE_SEED_ROOTS")) nroot_min = std::max(0, atoi(e));
        if (const char* e = getenv("SHD_ROUTE_SEED_DEPTH")) depth = std::max(1, atoi(e));
        // landmark seeds of a root row: three (C4 8-way roots 9.08 -> 8.83 ms with 64
        // landmarks; landmark-only C3 plans 0.79 -> 0.70 ms at 8-way)
        int klm = KD_SEEDS;
        if (const char* e = getenv("SHD_ROUTE_LMSEEDS")) klm = std::max(1, std::min(KD_SEEDS, atoi(e)));
        // seeds of each job: the kseeds neighbours u (jobs of this rank, smaller rank, level
        // below the cap) with the smallest w(s,u) + closeness(u), i.e. the likely gateways
        // of most shortest paths from s
        // A row with fewer such neighbours (a multi-GPU rank holds only its own rows) takes
        // two-hop seeds s -> x -> u (u one of this rank's rows, x any neighbour of degree
        // <= 256): D0 = w(s,x) + w(x,u) + d_u(.) is as consistent as a neighbour's, and u's
        // own record is the arc (x,u), tight whenever u keeps D0.
        bool two_hop = true;
        int hop_deg = 256;  // largest degree of a two-hop row's middle vertex x
        if (const char* e = getenv("SHD_ROUTE_SEED2HOP")) two_hop = atoi(e) != 0;
        if (const char* e = getenv("SHD_ROUTE_HOPDEG")) hop_deg = std::max(1, atoi(e));
        // The roots (the rows that would start unseeded) seed from host-computed landmark
        // rows instead: D0 = d(s, L) + d_L(.) is consistent for any landmark L, and L's own
        // record is the last arc (x, L) of a shortest s -> L path (tight whenever L keeps
        // D0).  C3 roots are a ninth of the rows and cost ~3.4 seeded rows each unseeded.
        // (C3, 1024 roots over 256-thread rows: 16/32/64/256 landmarks 2.90/2.89/2.80/2.76 ms;
        // C4's 256 roots are 0.5% of its rows: 16 and 64 measure the same, and each landmark
        // is a host Dijkstra of the plan (~40 ms at C4))
        if (nland > 0) {
            const double t0 = since();
            const int rc = ensure_landmarks(c, nland);
            if (rc) return rc;
            t_land = since() - t0;
        }
        std::vector<std::array<int, KD_SEEDS>> lmseed(nj);  // landmark index of seed k, or -1
        for (auto& a : lmseed) a.fill(-1);
        std::vector<int> fl(n, -1);  // first job of a vertex, once its level is below the cap
        std::vector<std::array<int, KD_SEEDS>> srec(nj);
        struct Hop { double cost; int u, off; uint32_t rec; };
        // A row's seeds: its best kseeds available neighbour rows, then (if short) its best
        // two-hop rows (s -> x -> u, x of degree <= 256), each list in the order a full sort
        // of the candidates would give.  avail(u): u's row is a usable seed.
        // (the chosen arcs' head, weight and record are kept in the choice: the sequential
        // pass below then reads no CSR array, whose random reads cost ~5 ms at C4)
        struct Choice { int m, nh; int arcs[KD_SEEDS]; int u[KD_SEEDS], w[KD_SEEDS]; uint32_t rec[KD_SEEDS]; Hop hop[KD_SEEDS]; };
        auto choose = [&](int p, auto avail, Choice& C) {
            const int s = src[p];
            C.m = best_seeds(p, avail, kseeds, C.arcs);
            for (int k = 0; k < C.m; k++) {
                const int a = C.arcs[k];
                C.u[k] = c->h_col[a];
                C.w[k] = (int)c->h_w[a];
                C.rec[k] = (uint32_t)s | ((uint32_t)c->h_ridx[a] << 16) | ((uint32_t)c->h_w[a] << 24);
            }
            C.nh = 0;
            if (!two_hop || C.m >= kseeds) return;
            const int need = kseeds - C.m;
            auto before = [](const Hop& x, const Hop& y) {
                return x.cost != y.cost ? x.cost < y.cost : x.u != y.u ? x.u < y.u : x.rec < y.rec;
            };
            for (int a = c->h_row[s]; a < c->h_row[s + 1]; a++) {
                const int x = c->h_col[a];
                if (x == s || c->h_row[x + 1] - c->h_row[x] > hop_deg) continue;
                for (int b = c->h_row[x]; b < c->h_row[x + 1]; b++) {
                    const int u = c->h_col[b];
                    if (u == s || u == x || rk[u] >= rk[s] || !avail(u)) continue;
                    bool dup = false;
                    for (int k = 0; k < C.m; k++) dup = dup || C.u[k] == u;
                    if (dup) continue;
                    const Hop h{c->h_w[a] + c->h_w[b] + c->close[u], u, (int)(c->h_w[a] + c->h_w[b]),
                                (uint32_t)x | ((uint32_t)c->h_ridx[b] << 16) | ((uint32_t)c->h_w[b] << 24)};
                    int dq = -1;
                    for (int q = 0; q < C.nh; q++) if (C.hop[q].u == u) dq = q;
                    if (dq >= 0) {
                        if (!before(h, C.hop[dq])) continue;
                        for (int q = dq; q + 1 < C.nh; q++) C.hop[q] = C.hop[q + 1];
                        C.nh--;
                    }
                    if (C.nh == need && !before(h, C.hop[C.nh - 1])) continue;
                    int q = C.nh < need ? C.nh++ : need - 1;
                    for (; q > 0 && before(h, C.hop[q - 1]); q--) C.hop[q] = C.hop[q - 1];
                    C.hop[q] = h;
                }
            }
        };
        // Choices precomputed on host threads against a superset of the usable rows (every
        // row of an earlier source: the sequential pass below only withholds rows past the
        // seed-chain depth cap); the sequential pass keeps a precomputed choice when every
        // row in it is usable -- then it is exactly the choice over the usable rows -- and
        // recomputes the row otherwise.
        // (not value-initialised: the worker threads first-touch their own pages)
        std::unique_ptr<Choice[]> pre(new Choice[order.size()]);
        // The worker threads take chunks of 256 choices in order and mark each one done; the
        // sequential pass below runs concurrently, consuming the chunks as they complete (and
        // taking a chunk itself while the one it needs is not done), so it hides behind the
        // choices instead of following them (C4: ~1.4 ms).
        const int nq = (int)order.size(), CH = 256;
        const int nchunk = nq > nroot_min ? (nq - nroot_min + CH - 1) / CH : 0;
        std::unique_ptr<std::atomic<int>[]> chunk_done(new std::atomic<int>[std::max(1, nchunk)]);
        for (int k = 0; k < nchunk; k++) chunk_done[k].store(0, std::memory_order_relaxed);
        std::atomic<int> nextq{nroot_min};
        auto take_chunk = [&]() {
            if (nextq.load(std::memory_order_relaxed) >= nq) return false;  // (no unbounded fetch_add)
            const int q0 = nextq.fetch_add(CH);
            if (q0 >= nq) return false;
            const int q1 = std::min(nq, q0 + CH);
            for (int qq = q0; qq < q1; qq++) {
                // the rows come in rank order, i.e. at random places of the CSR: prefetch the
                // row offsets 8 sources ahead and the arcs 4 ahead (choices ~30% faster)
                if (qq + 8 < q1) __builtin_prefetch(&c->h_row[src[order[qq + 8]]]);
                if (qq + 4 < q1) {
                    const int s4 = src[order[qq + 4]], a0 = c->h_row[s4], a1 = c->h_row[s4 + 1];
                    for (int a = a0; a < a1; a += 16) __builtin_prefetch(&c->h_col[a]);
                    for (int a = a0; a < a1; a += 8) __builtin_prefetch(&c->h_w[a]);
                }
                choose(order[qq], [&](int u) { return first[u] >= 0; }, pre[qq]);
            }
            chunk_done[(q0 - nroot_min) / CH].store(1, std::memory_order_release);
            return true;
        };
        // the choices on the device by default (one wave per row, ~1 ms with the copies at C4;
        // on the host workers they took 3.7-8 ms depending on the box's host load: C4 plans
        // 8.5-8.9 against 13.2 ms on one box); SHD_ROUTE_GPUCHOICE=0 keeps them on the host
        const double th0 = since();
        bool dev_choice = nchunk > 0 && !(getenv("SHD_ROUTE_GPUCHOICE") && atoi(getenv("SHD_ROUTE_GPUCHOICE")) == 0);
        std::vector<PlanChoice> dch;  // device candidate lists of the seedable rows, in queue order
        if (dev_choice) {
            auto device_choices = [&]() -> bool {
                const int nqs = nq - nroot_min;
                std::vector<int> sq(nqs);
                for (int i = 0; i < nqs; i++) sq[i] = src[order[nroot_min + i]];
                std::vector<uint8_t> av(n);
                for (int v = 0; v < n; v++) av[v] = first[v] >= 0;
                DevBuf dcl, drk, dav, dsq, dout;
                if (dcl.alloc(sizeof(double) * n) || drk.alloc(sizeof(int) * n) || dav.alloc(n) ||
                    dsq.alloc(sizeof(int) * nqs) || dout.alloc(sizeof(PlanChoice) * nqs))
                    return false;
                if (hipMemcpy(dcl.p, c->close.data(), sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess ||
                    hipMemcpy(drk.p, rk.data(), sizeof(int) * n, hipMemcpyHostToDevice) != hipSuccess ||
                    hipMemcpy(dav.p, av.data(), n, hipMemcpyHostToDevice) != hipSuccess ||
                    hipMemcpy(dsq.p, sq.data(), sizeof(int) * nqs, hipMemcpyHostToDevice) != hipSuccess)
                    return false;
                hipLaunchKernelGGL(plan_choice_kernel, dim3((nqs + 3) / 4), dim3(256), 0, 0, c->d_row, c->d_kd_orec,
                                   (const double*)dcl.p, (const int*)drk.p, (const uint8_t*)dav.p, (const int*)dsq.p, nqs,
                                   kseeds, two_hop ? 1 : 0, hop_deg, alpha, PC_CAND, (PlanChoice*)dout.p);
                dch.resize(nqs);
                if (hipGetLastError() != hipSuccess ||
                    hipMemcpy(dch.data(), dout.p, sizeof(PlanChoice) * nqs, hipMemcpyDeviceToHost) != hipSuccess) {
                    dch.clear();
                    return false;
                }
                return true;
            };
            dev_choice = device_choices();
            if (dev_choice) {
                nextq.store(nq);
                for (int k = 0; k < nchunk; k++) chunk_done[k].store(1, std::memory_order_relaxed);
            }
        }
        // the roots' landmark seeds on the device (a host loop over the landmark rows took
        // ~2 us per root: strided distance reads and a parent walk per landmark seed)
        std::vector<LmChoice> lmc;
        if (nland > 0 && nroot_min > 0 && c->d_lm_drow &&
            !(getenv("SHD_ROUTE_GPUCHOICE") && atoi(getenv("SHD_ROUTE_GPUCHOICE")) == 0)) {
            const int nr0 = std::min(nroot_min, nq);
            std::vector<int> sq(nr0);
            for (int i = 0; i < nr0; i++) sq[i] = src[order[i]];
            std::vector<int> lv(c->lm_v.begin(), c->lm_v.begin() + nland);
            DevBuf dsq, dlv, dout;
            bool ok = !dsq.alloc(sizeof(int) * nr0) && !dlv.alloc(sizeof(int) * nland) && !dout.alloc(sizeof(LmChoice) * nr0) &&
                      hipMemcpy(dsq.p, sq.data(), sizeof(int) * nr0, hipMemcpyHostToDevice) == hipSuccess &&
                      hipMemcpy(dlv.p, lv.data(), sizeof(int) * nland, hipMemcpyHostToDevice) == hipSuccess;
            if (ok) {
                hipLaunchKernelGGL(plan_landmark_kernel, dim3((nr0 + 3) / 4), dim3(256), 0, 0, c->d_lm_drow, c->d_lm_prow,
                                   (long long)c->lm_rs, (const int*)dlv.p, nland, (const int*)dsq.p, nr0, klm, n,
                                   (LmChoice*)dout.p);
                lmc.resize(nr0);
                ok = hipGetLastError() == hipSuccess &&
                     hipMemcpy(lmc.data(), dout.p, sizeof(LmChoice) * nr0, hipMemcpyDeviceToHost) == hipSuccess;
            }
            if (!ok) lmc.clear();
        }
        HostPool* pool = dev_choice ? nullptr : host_pool();
        std::unique_lock<std::mutex> lease(g_pool_use, std::try_to_lock);
        std::unique_ptr<HostPool> own;  // the shared workers are busy with another plan
        if (pool && !lease.owns_lock()) {
            own.reset(new HostPool(plan_threads() - 1));
            pool = own.get();
        }
        struct PoolWait {
            HostPool* p;
            bool on;
            void operator()() { if (on) { p->wait(); on = false; } }
            ~PoolWait() { (*this)(); }
        } pool_wait{pool, pool && nchunk > 0};
        if (pool_wait.on) pool->run([&]() { while (take_chunk()) {} });
        if (getenv("SHD_ROUTE_PIPE") && atoi(getenv("SHD_ROUTE_PIPE")) == 0) {  // A/B: choices first, then the pass
            while (take_chunk()) {}
            pool_wait();
        }
        int nlev = 1, q = 0;
        int n_direct[KD_SEEDS + 1] = {0}, n_twohop = 0;  // SHD_ROUTE_PLAN_DEBUG: seed kinds
        std::unique_ptr<KDJob[]> byjob(new KDJob[nj]);
        t_loop0 = since();
        for (int j = 0; j < nj; j++) {
            const int p = job_pos[j], s = src[p];
            const int qi = q;
            const bool seedable = q++ >= nroot_min;
            if (seedable && (qi - nroot_min) % CH == 0) {
                std::atomic<int>& dn = chunk_done[(qi - nroot_min) / CH];
                while (!dn.load(std::memory_order_acquire))
                    if (!take_chunk()) std::this_thread::yield();
            }
            Choice ch;
            ch.m = ch.nh = 0;
            if (seedable && dev_choice) {
                // the first kseeds usable entries of the device's ordered candidate list are the
                // host rule's choice over the usable rows, when the list held kseeds usable ones
                // or every available neighbour (o.m < PC_CAND); a two-hop fill stands when every
                // listed neighbour was usable (same exclusions, same count) and so are its picks
                const PlanChoice& o = dch[qi - nroot_min];
                int got = 0;
                bool direct_all = true;
                for (int k = 0; k < o.m && got < kseeds; k++) {
                    if (fl[o.u[k]] >= 0) { ch.u[got] = o.u[k]; ch.w[got] = o.w[k]; ch.rec[got] = o.rec[k]; got++; }
                    else direct_all = false;
                }
                ch.m = got;
                bool exact = got == kseeds || o.m < PC_CAND;
                if (exact && got < kseeds && two_hop) {
                    bool hop_ok = o.m < kseeds && direct_all;
                    for (int k = 0; k < o.nh && hop_ok; k++) hop_ok = fl[o.u[o.m + k]] >= 0;
                    if (hop_ok) {
                        ch.nh = o.nh;
                        for (int k = 0; k < o.nh; k++) ch.hop[k] = Hop{0.0, o.u[o.m + k], o.w[o.m + k], o.rec[o.m + k]};
                    } else exact = false;
                }
                if (!exact) { ch.m = ch.nh = 0; choose(p, [&](int u) { return fl[u] >= 0; }, ch); n_recomp++; }
            } else if (seedable) {
                bool ok = true;
                const Choice& pc = pre[qi];
                for (int k = 0; k < pc.m; k++) ok = ok && fl[pc.u[k]] >= 0;
                for (int k = 0; k < pc.nh; k++) ok = ok && fl[pc.hop[k].u] >= 0;
                if (ok) ch = pc;
                else { choose(p, [&](int u) { return fl[u] >= 0; }, ch); n_recomp++; }
            }
            int m = ch.m;
            if (seedable) { n_direct[std::min(ch.m, KD_SEEDS)]++; if (ch.nh) n_twohop++; }
            if (!seedable && nland > 0 && qi < (int)lmc.size()) {
                const LmChoice& o = lmc[qi];
                for (int k = 0; k < o.m; k++) {
                    su[j][k] = c->lm_v[o.l[k]]; wr[j][k] = o.d[k]; srec[j][k] = (int)o.rec[k]; lmseed[j][k] = o.l[k];
                }
                nsd[j] = o.m;
            } else if (!seedable && nland > 0) {
                if (ensure_lm_host(c)) return SHD_ROUTE_EDEVICE;
                // nearest landmarks by d(s, L) (undirected: d_L(s)), up to klm (default kseeds)
                std::vector<std::pair<double, int>> lc;
                for (int l = 0; l < nland; l++) {
                    const uint16_t dls = c->lm_hd[(size_t)l * c->lm_rs + s];
                    if (dls != 0xFFFFu) lc.push_back({(double)dls, l});
                }
                std::sort(lc.begin(), lc.end());
                int mk = 0;
                for (const auto& pr : lc) {
                    if (mk == klm) break;
                    const int l = pr.second, L = c->lm_v[l];
                    uint32_t rec = KD_SRC_MARK;
                    if (L != s) {
                        // the last arc (x, L) of the shortest s -> L path in L's tree
                        int x = s;
                        const uint32_t* lp = c->lm_hp.data() + (size_t)l * c->lm_rs;
                        while ((int)(lp[x] & 0xFFFFu) != L) x = (int)(lp[x] & 0xFFFFu);
                        const uint32_t px = lp[x];  // L | ridx(x,L) << 16 | w << 24
                        rec = (uint32_t)x | (px & 0xFFFF0000u);
                    }
                    su[j][mk] = L; wr[j][mk] = (int)pr.first; srec[j][mk] = (int)rec; lmseed[j][mk] = l;
                    mk++;
                }
                nsd[j] = mk;
            }
            for (int k = 0; k < m; k++) { su[j][k] = ch.u[k]; wr[j][k] = ch.w[k]; srec[j][k] = (int)ch.rec[k]; }
            for (int q2 = 0; q2 < ch.nh; q2++, m++) {
                su[j][m] = ch.hop[q2].u; wr[j][m] = ch.hop[q2].off; srec[j][m] = (int)ch.hop[q2].rec;
            }
            for (int k = 0; k < m; k++) {
                const int sj = first[su[j][k]];
                seedjob[j][k] = sj;
                lvl[j] = std::max(lvl[j], lvl[sj] + 1);
                if (slot[sj] < 0) slot[sj] = P->nslots++;
            }
            if (seedable || nland == 0) nsd[j] = m;
            if (!nsd[j]) P->nroots++;
            nlev = std::max(nlev, lvl[j] + 1);
            if (first[src[p]] == j && lvl[j] + 1 < depth) fl[src[p]] = p;
            {
                // the job record, in job order (the schedule below copies it into queue order:
                // one cache line per job instead of five scattered per-job arrays); its own
                // store slot and landmark slots (-1 - l: after every kept row's slot) are
                // final only after this pass
                KDJob& J = byjob[j];
                std::memset(&J, 0, sizeof(J));
                J.row = job_row[j]; J.s = s; J.store = -1; J.nseed = nsd[j];
                for (int k = 0; k < nsd[j]; k++) {
                    J.seed[k] = lmseed[j][k] >= 0 ? -1 - lmseed[j][k] : slot[seedjob[j][k]];
                    J.u[k] = su[j][k]; J.wr[k] = wr[j][k]; J.rec[k] = srec[j][k];
                }
            }
        }
        pool_wait();
        t_hop = since() - th0;
        t_seeds = since();
        const long long rs = kd_row_stride(n);
        bool uses_lm = false;
        for (int j = 0; j < nj && !uses_lm; j++) uses_lm = nsd[j] > 0 && lmseed[j][0] >= 0;
        P->nland = uses_lm ? nland : 0;
        const int ntot = P->nslots + P->nland;
        P->store_bytes = (uint64_t)ntot * (uint64_t)rs * 6u;
        // the row store's allocation and the landmark rows' device copies run on a second host
        // thread while this one builds the schedule (C4: ~0.5 ms of hipMalloc and copies)
        bool store_ok = false;
        std::thread store_th;
        // (SHD_ROUTE_STORE_SYNC=1: the allocation after the schedule, on this thread -- an A/B
        // of the schedule's time with and without the allocating thread beside it)
        const bool store_sync = getenv("SHD_ROUTE_STORE_SYNC") && atoi(getenv("SHD_ROUTE_STORE_SYNC"));
        auto store_fn = [&]() {
                bool r = hipSetDevice(c->device) == hipSuccess &&
                         hipMalloc((void**)&P->d_drow, sizeof(uint16_t) * (size_t)rs * ntot) == hipSuccess &&
                         hipMalloc((void**)&P->d_prow, sizeof(uint32_t) * (size_t)rs * ntot) == hipSuccess;
                if (r && P->nland)
                    // landmark rows into the slots after the kept rows' (the rows are in the store
                    // format already, pads included)
                    r = hipMemcpy(P->d_drow + (size_t)rs * P->nslots, c->d_lm_drow,
                                  sizeof(uint16_t) * (size_t)rs * P->nland, hipMemcpyDeviceToDevice) == hipSuccess &&
                        hipMemcpy(P->d_prow + (size_t)rs * P->nslots, c->d_lm_prow,
                                  sizeof(uint32_t) * (size_t)rs * P->nland, hipMemcpyDeviceToDevice) == hipSuccess;
                // the job array and the launch's queue counter + ready flags
                r = r && hipMalloc((void**)&P->d_jobs, sizeof(KDJob) * (size_t)nj) == hipSuccess &&
                    hipMalloc((void**)&P->d_next, sizeof(int) * (1 + (size_t)ntot)) == hipSuccess;
                store_ok = r;
            };
        if (ntot > 0 && !store_sync) store_th = std::thread(store_fn);
        struct JoinOne { std::thread& t; ~JoinOne() { if (t.joinable()) t.join(); } } join_store{store_th};
        t_alloc = since();
        if (ntot > 0) {
            std::vector<int> cnt(nlev + 1, 0);
            for (int j = 0; j < nj; j++) cnt[lvl[j] + 1]++;
            for (int k = 0; k < nlev; k++) cnt[k + 1] += cnt[k];
            P->lvl_off = cnt;
            // queue order: list scheduling of the seed DAG over the launch's workgroups with
            // estimated row times (a root ~3.4x a seeded row; a kept row's flag at ~0.7 of
            // it): each workgroup, when free, takes the row whose seeds' flags are estimated
            // earliest.  A row still follows all of its seeds in the queue (no deadlock),
            // but rows no longer wait at every level boundary for seeds just started.
            const int W = std::max(1, c->kd_slots);
            double root_cost = 3.4, flag_at = 0.7, lm_cost = 2.0;  // (landmark-seeded roots)
            if (const char* e = getenv("SHD_ROUTE_LMCOST")) lm_cost = std::max(0.1, atof(e));
            if (const char* e = getenv("SHD_ROUTE_ROOTCOST")) root_cost = std::max(0.1, atof(e));
            if (const char* e = getenv("SHD_ROUTE_FLAGAT")) flag_at = std::max(0.0, std::min(1.0, atof(e)));
            // dependants of each job as one CSR (job j's in [dbeg[j], dbeg[j + 1]))
            std::vector<int> left(nj, 0), dbeg(nj + 1, 0), dep;
            for (int j = 0; j < nj; j++)
                for (int k = 0; k < nsd[j]; k++)
                    if (lmseed[j][k] < 0) { dbeg[seedjob[j][k] + 1]++; left[j]++; }
            for (int j = 0; j < nj; j++) dbeg[j + 1] += dbeg[j];
            dep.resize(dbeg[nj]);
            {
                std::vector<int> fill(dbeg.begin(), dbeg.end() - 1);
                for (int j = 0; j < nj; j++)
                    for (int k = 0; k < nsd[j]; k++)
                        if (lmseed[j][k] < 0) dep[fill[seedjob[j][k]]++] = j;
            }
            t_deps = since();
            // times in integer ticks of 1/100 row: the ready queue is a bucket queue (a row
            // becomes ready strictly after the start of the row that releases it, so the
            // queue's minimum only grows and every bucket is complete when it is reached;
            // within a bucket, rows in job order).  A binary heap of (double, job) pairs took
            // ~6 ms at C4.
            auto tk = [](double x) { return (long long)std::llround(x * 100.0); };
            const long long t_root = tk(root_cost), t_lm = tk(lm_cost), t_one = 100;
            // buckets as singly linked lists through one array (no allocation per bucket): a
            // bucket's rows are sorted by job when it is reached
            std::vector<long long> ready(nj, 0);
            std::vector<int> bhead(1024, -1), bnext(nj, -1), cur_b;
            auto push = [&](long long t, int j) {
                if ((size_t)t >= bhead.size()) bhead.resize(std::max((size_t)t + 1, 2 * bhead.size()), -1);
                bnext[j] = bhead[t];
                bhead[t] = j;
            };
            size_t bq_n = 0;  // rows queued
            for (int j = nj - 1; j >= 0; j--) if (!left[j]) { push(0, j); bq_n++; }
            // free walker slots: a second bucket queue over ticks (a slot frees at its row's
            // start + cost >= the current minimum, so this minimum only grows too); it replaced
            // a binary heap of (tick, slot) pairs, 11.4 -> 7.4 ms for C4's schedule on the host
            std::vector<int> fhead(1024, -1), fnext(W, -1);
            auto fpush = [&](long long t, int w) {
                if ((size_t)t >= fhead.size()) fhead.resize(std::max((size_t)t + 1, 2 * fhead.size()), -1);
                fnext[w] = fhead[t];
                fhead[t] = w;
            };
            for (int w = W - 1; w >= 0; w--) fpush(0, w);
            long long fcur = 0;
            // each job is written into the launch's job array as it is scheduled (queue order)
            jobs.resize(nj);
            const double t_jobs = since();
            int qi = 0;
            auto emit = [&](int j) {
                KDJob& J = jobs[qi++];
                J = byjob[j];
                J.store = slot[j];
                for (int k = 0; k < J.nseed; k++)
                    if (J.seed[k] < 0) J.seed[k] = P->nslots + (-1 - J.seed[k]);
            };
            long long cur = -1;
            size_t pos = 0;
            if (getenv("SHD_ROUTE_SCHED") && atoi(getenv("SHD_ROUTE_SCHED")) == 0) {  // A/B: plain rank order
                for (int j = 0; j < nj; j++) emit(j);
                bq_n = 0;
            }
            while (bq_n) {
                while (pos >= cur_b.size()) {  // next non-empty bucket
                    cur++;
                    cur_b.clear();
                    pos = 0;
                    if ((size_t)cur < bhead.size())
                        for (int j = bhead[cur]; j >= 0; j = bnext[j]) cur_b.push_back(j);
                    if (cur_b.size() > 1) std::sort(cur_b.begin(), cur_b.end());
                }
                const int j = cur_b[pos++];
                bq_n--;
                while (fhead[fcur] < 0) fcur++;
                const int fw = fhead[fcur];
                fhead[fcur] = fnext[fw];
                const long long t = !nsd[j] ? t_root : lmseed[j][0] >= 0 ? t_lm : t_one;
                const long long start = std::max(fcur, cur);
                fpush(start + t, fw);
                emit(j);
                const long long rel = start + std::max(1ll, tk(flag_at * (double)t / 100.0));
                for (int e = dbeg[j]; e < dbeg[j + 1]; e++) {
                    const int d = dep[e];
                    ready[d] = std::max(ready[d], rel);
                    if (--left[d] == 0) { push(ready[d], d); bq_n++; }
                }
            }
            t_sched = since();
            if (getenv("SHD_ROUTE_PLAN_DEBUG")) {
                fprintf(stderr, "  schedule: job array ready %.2f ms (%d jobs, ticks to %lld)\n", 1e3 * t_jobs, nj, cur);
                int hist[KD_SEEDS + 1] = {0};
                for (int j = 0; j < nj; j++) hist[nsd[j]]++;
                fprintf(stderr, "plan world %d rank %d: jobs %d levels %d seeds:", world, rank, nj, nlev);
                for (int k = 0; k <= KD_SEEDS; k++) fprintf(stderr, " %d:%d", k, hist[k]);
                fprintf(stderr, "  closeness rows %.2f ms, rank sort done %.2f, order sort done %.2f, landmark rows %.2f ms, "
                        "seed choices (threads, overlapping the pass) %.2f ms, seeds done %.2f, schedule done %.2f ms\n",
                        1e3 * t_close, 1e3 * t_rk, 1e3 * t_order, 1e3 * t_land, 1e3 * t_hop, 1e3 * t_seeds, 1e3 * t_sched);
                fprintf(stderr, "  seq loop start %.2f (recomputed %d), store thread started %.2f, deps done %.2f\n", 1e3 * t_loop0, n_recomp,
                        1e3 * t_alloc, 1e3 * t_deps);
                int nlm = 0;
                for (int j = 0; j < nj; j++) nlm += nsd[j] > 0 && lmseed[j][0] >= 0;
                fprintf(stderr, "  seed kinds: landmark-seeded roots %d; neighbour-seeded rows by direct seeds:", nlm);
                for (int k = 0; k <= KD_SEEDS; k++) fprintf(stderr, " %d:%d", k, n_direct[k]);
                fprintf(stderr, " (with two-hop seeds %d; at most one direct seed: %.1f%% of the other rows)\n", n_twohop,
                        100.0 * (n_direct[0] + n_direct[1]) / std::max(1, nj - nlm));
            }
        }
        if (store_th.joinable()) store_th.join();
        if (ntot > 0 && store_sync) store_fn();
        t_store = since();
        if (store_ok) {
            P->seeded = 1;
        } else {
            for (void** q : {(void**)&P->d_drow, (void**)&P->d_prow, (void**)&P->d_jobs, (void**)&P->d_next})
                if (*q) { (void)hipFree(*q); *q = nullptr; }
            P->nslots = 0; P->nroots = 0; P->nland = 0; P->store_bytes = 0;
        }
    }
    if (P->seeded) {
        if (hipMemcpy(P->d_jobs, jobs.data(), sizeof(KDJob) * jobs.size(), hipMemcpyHostToDevice) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
    } else {
        // plain rows (the helpers of an unseeded multi-GPU plan are not needed)
        P->nhelpers = 0;
        std::vector<int32_t> sv(std::max(nr, 1), 0);
        for (int r = 0; r < nr; r++) sv[r] = src[P->row_pos[r]];
        if (hipMalloc((void**)&P->d_src, sizeof(int32_t) * sv.size()) != hipSuccess) return SHD_ROUTE_ENOMEM;
        if (hipMemcpy(P->d_src, sv.data(), sizeof(int32_t) * sv.size(), hipMemcpyHostToDevice) != hipSuccess)
            return SHD_ROUTE_EDEVICE;
        P->nroots = nr;
    }
    if (getenv("SHD_ROUTE_PLAN_DEBUG")) fprintf(stderr, "  store thread joined %.2f, plan total %.2f ms\n", 1e3 * t_store, 1e3 * since());
    *out = P.release();
    return SHD_ROUTE_OK;
}

void shd_route_plan_destroy(shd_route_plan_t* P) {
    if (!P) return;
    (void)hipSetDevice(P->c->device);
    delete P;
}

int shd_route_plan_get_info(const shd_route_plan_t* P, shd_route_plan_info_t* info) {
    if (!P || !info) return SHD_ROUTE_EINVAL;
    info->rows = (int32_t)P->row_pos.size();
    info->seeded = P->seeded;
    // (landmark-only: hub rows, [landmark biases,] the job records [+ order keys and ranks], rows)
    info->launches = P->lm_step ? (P->order_fixed ? 3 : 5) + (P->d_bias ? 1 : 0) : 1;
    info->levels = P->seeded ? (int32_t)P->lvl_off.size() - 1 : 1;
    info->roots = P->nroots;
    info->helpers = P->nhelpers;
    info->stored_rows = P->nslots;
    info->world = P->world;
    info->rank = P->rank;
    info->store_bytes = P->store_bytes;
    info->delta = P->seeded ? P->delta : P->c->kd_delta;
    info->pad_ = 0;
    return SHD_ROUTE_OK;
}

int shd_route_plan_rows(const shd_route_plan_t* P, int32_t* pos_out) {
    if (!P || !pos_out) return SHD_ROUTE_EINVAL;
    std::copy(P->row_pos.begin(), P->row_pos.end(), pos_out);
    return SHD_ROUTE_OK;
}

int shd_route_plan_refresh_async(shd_route_t* c, const shd_route_plan_t* P, uint32_t what, void* stream) {
    if (!c || !P || P->c != c || (what & ~(SHD_ROUTE_REFRESH_ALL | SHD_ROUTE_REFRESH_MINE | SHD_ROUTE_REFRESH_JOBS)))
        return SHD_ROUTE_EINVAL;
    if (!P->lm_step) return SHD_ROUTE_OK;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    return lm_refresh(c, P, what, (hipStream_t)stream);
}

int shd_route_plan_landmarks(const shd_route_plan_t* P, int32_t* nland, int32_t* first, int32_t* count,
                             int64_t* row_stride) {
    if (!P || !nland || !first || !count || !row_stride) return SHD_ROUTE_EINVAL;
    if (!P->lm_step) return SHD_ROUTE_EUNSUPPORTED;
    *nland = P->nhub; *first = P->lm_first; *count = P->lm_count;
    *row_stride = kd_row_stride(P->c->n);
    return SHD_ROUTE_OK;
}

int shd_route_plan_bind_store(shd_route_t* c, shd_route_plan_t* P, uint16_t* d_drow, uint32_t* d_prow) {
    if (!c || !P || P->c != c || !d_drow || !d_prow) return SHD_ROUTE_EINVAL;
    if (!P->lm_step) return SHD_ROUTE_EUNSUPPORTED;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    const size_t cells = (size_t)kd_row_stride(c->n) * P->nhub;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(d_drow, P->d_drow, sizeof(uint16_t) * cells, hipMemcpyDeviceToDevice) != hipSuccess ||
        hipMemcpy(d_prow, P->d_prow, sizeof(uint32_t) * cells, hipMemcpyDeviceToDevice) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    if (!P->store_external) {
        (void)hipFree(P->d_drow);
        (void)hipFree(P->d_prow);
    }
    P->d_drow = d_drow; P->d_prow = d_prow; P->store_external = true;
    return SHD_ROUTE_OK;
}

int shd_route_rows_planned_async(shd_route_t* c, const shd_route_plan_t* P, const int32_t* d_tgt, int32_t nt,
                                 int64_t ld, uint32_t flags, double* d_lat, double* d_rel, double* d_row_min,
                                 void* stream) {
    if (!c || !P || P->c != c || nt < 0 || (nt && !d_tgt) || ld < nt) return SHD_ROUTE_EINVAL;
    const int nr = (int)P->row_pos.size();
    if (!P->seeded) return shd_route_rows_async(c, P->d_src, nr, d_tgt, nt, ld, flags, d_lat, d_rel, d_row_min, stream);
    hipStream_t st = (hipStream_t)stream;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (P->lm_step && !(flags & SHD_ROUTE_PLAN_REUSE)) {
        const int rc = lm_refresh(c, P, 0, st);  // the landmark rows and the jobs, on this stream
        if (rc) return rc;
    }
    // one launch: jobs in level order from one queue; a seeded job waits for its seed's
    // ready flag (set once the kept row is complete, before that row's phase C)
    if (hipMemsetAsync(P->d_next, 0, sizeof(int) * (1 + (size_t)P->nslots), st) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (P->nland && hipMemsetD32Async((hipDeviceptr_t)(P->d_next + 1 + P->nslots), 1, (size_t)P->nland, st) != hipSuccess)
        return SHD_ROUTE_EDEVICE;  // landmark rows: complete before the launch
    DevDelta k = kd_args(c);
    k.delta = P->delta;
    k.drow = P->d_drow; k.drow_out = P->d_drow; k.prow = P->d_prow; k.rstride = kd_row_stride(c->n);
    k.jobs = P->d_jobs;
    k.done = P->d_next + 1;
    return kd_launch(c, k, P->d_next, nullptr, P->lvl_off.back(), d_tgt, nt, ld, d_lat, d_rel, d_row_min, st);
}

}  // extern "C"


namespace {
// shd_route_rows through a seeded plan: every row in one device table (EUNSUPPORTED when
// the plan is not seeded or the table does not fit, so the caller takes the chunked path)
int planned_host_rows(shd_route* c, const int32_t* src, int32_t ns, const int32_t* tgt, int32_t nt,
                      uint32_t flags, double* lat_out, double* rel_out, double* row_min_out) {
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    const size_t table = sizeof(double) * (size_t)ns * (size_t)nt;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || 2 * table + ((size_t)ns << 20) > fr / 2) return SHD_ROUTE_EUNSUPPORTED;
    shd_route_plan_t* P = nullptr;
    int rc = shd_route_plan_create(c, src, ns, 1, 0, &P);
    if (rc == SHD_ROUTE_ENOMEM) return SHD_ROUTE_EUNSUPPORTED;  // the chunked rows need far less
    if (rc) return rc;
    std::unique_ptr<shd_route_plan, void (*)(shd_route_plan*)> guard(P, shd_route_plan_destroy);
    if (!P->seeded) return SHD_ROUTE_EUNSUPPORTED;
    DevBuf dtgt, dlat, drel, dmin;
    if (dtgt.alloc(sizeof(int32_t) * nt) || dlat.alloc(table) || drel.alloc(table) || dmin.alloc(sizeof(double) * ns))
        return SHD_ROUTE_EUNSUPPORTED;
    if (hipMemcpy(dtgt.p, tgt, sizeof(int32_t) * nt, hipMemcpyHostToDevice) != hipSuccess) return SHD_ROUTE_EDEVICE;
    // (the plan was made just now: its landmark rows, if any, are current)
    rc = shd_route_rows_planned_async(c, P, (const int32_t*)dtgt.p, nt, nt, flags | SHD_ROUTE_PLAN_REUSE, (double*)dlat.p, (double*)drel.p,
                                      (double*)dmin.p, nullptr);
    if (rc) return rc;
    const int soft = shd_route_sync(c, nullptr);
    if (soft && soft != SHD_ROUTE_ENOEDGE && soft != SHD_ROUTE_EUNREACH) return soft;
    if ((lat_out && hipMemcpy(lat_out, dlat.p, table, hipMemcpyDeviceToHost) != hipSuccess) ||
        (rel_out && hipMemcpy(rel_out, drel.p, table, hipMemcpyDeviceToHost) != hipSuccess) ||
        (row_min_out && hipMemcpy(row_min_out, dmin.p, sizeof(double) * ns, hipMemcpyDeviceToHost) != hipSuccess))
        return SHD_ROUTE_EDEVICE;
    return soft;
}
}  // namespace

// =============================================================================
// K4: blocked min-plus Floyd-Warshall (fw.hpp)
// =============================================================================
namespace {
constexpr int kFwMaxN = 12000;  // fw_rows keeps rel f64 + order u16 per vertex in LDS

// Builds the K4 state once per context: eligibility first (nothing is allocated for an
// ineligible graph, so every call answers EUNSUPPORTED), then the buffers into locals,
// published in the context only when every step has succeeded; the in-list build is
// enqueued on the caller's stream, ahead of the table launches that follow it there.
int fw_prepare(shd_route* c, hipStream_t st) {
    if (c->d_fwD) return SHD_ROUTE_OK;
    if (!c->integer_w || c->multigraph || c->n > kFwMaxN || c->k32_bound <= 0 || c->k32_bound >= 0xFFFF)
        return SHD_ROUTE_EUNSUPPORTED;
    const size_t lds = a16(sizeof(double) * c->n) + a16(sizeof(uint16_t) * c->n) + a16(sizeof(int) * (c->k32_bound + 2));
    if (lds > kLdsBudget) return SHD_ROUTE_EUNSUPPORTED;
    const int np = (c->n + FW_T - 1) / FW_T * FW_T;
    int sp = 1;
    while (sp < np) sp <<= 1;
    if ((size_t)4 * sp > kLdsBudget) return SHD_ROUTE_EUNSUPPORTED;
    int rc = ensure_dense(c);
    if (rc) return rc;
    if ((rc = hip_check(hipFuncSetAttribute((const void*)fw_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)lds))) ||
        (rc = hip_check(hipFuncSetAttribute((const void*)fw_inlist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)(4 * sp)))) ||
        (rc = hip_check(hipFuncSetAttribute((const void*)fw_parent_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)(2 * np)))) ||
        (rc = hip_check(hipFuncSetAttribute((const void*)fw_parent_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)(2 * np)))) ||
        ((size_t)16 * np <= kLdsBudget &&
         ((rc = hip_check(hipFuncSetAttribute((const void*)fw_parent8_kernel<true>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)(16 * np)))) ||
          (rc = hip_check(hipFuncSetAttribute((const void*)fw_parent8_kernel<false>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)(16 * np)))))))
        return rc;
    const size_t cells = (size_t)np * np;
    uint16_t* D = nullptr;
    uint32_t* inl = nullptr;
    uint16_t* pos = nullptr;
    auto undo = [&](int code) {
        if (D) (void)hipFree(D);
        if (inl) (void)hipFree(inl);
        if (pos) (void)hipFree(pos);
        return code;
    };
    if (hipMalloc((void**)&D, 2 * cells) != hipSuccess || hipMalloc((void**)&inl, 4 * cells) != hipSuccess ||
        hipMalloc((void**)&pos, sizeof(uint16_t) * FW_X * (size_t)c->n) != hipSuccess)
        return undo(SHD_ROUTE_ENOMEM);
    // reliability indices (round 5): every distinct 1 - loss (exact bits), at most 255 of them
    // (C5: 101), as a dense u8 matrix: fw_rows reads a parent arc's index and multiplies the
    // table entry in LDS
    std::vector<uint64_t> rbits;
    for (int e = 0; e < c->m; e++) { uint64_t b; std::memcpy(&b, &c->e_rel[e], 8); rbits.push_back(b); }
    std::sort(rbits.begin(), rbits.end());
    rbits.erase(std::unique(rbits.begin(), rbits.end()), rbits.end());
    uint8_t* rixd = nullptr;
    double* rtd = nullptr;
    int nrt = 0;
    if (rbits.size() <= 255 && !getenv("SHD_ROUTE_FWDENSER")) {
        std::vector<double> rt(rbits.size());
        for (size_t q = 0; q < rbits.size(); q++) std::memcpy(&rt[q], &rbits[q], 8);
        std::vector<uint8_t> rix((size_t)c->n * c->n, 0xFF);
        auto idx = [&](double r) {
            uint64_t b; std::memcpy(&b, &r, 8);
            return (uint8_t)(std::lower_bound(rbits.begin(), rbits.end(), b) - rbits.begin());
        };
        // (the same edge ensure_dense keeps: the lowest edge id of a pair)
        for (int e = c->m - 1; e >= 0; e--) {
            const int a = c->e_src[e], b = c->e_dst[e];
            rix[(size_t)a * c->n + b] = idx(c->e_rel[e]);
            if (!c->directed) rix[(size_t)b * c->n + a] = idx(c->e_rel[e]);
        }
        if (hipMalloc((void**)&rixd, rix.size()) != hipSuccess ||
            hipMalloc((void**)&rtd, sizeof(double) * 256) != hipSuccess ||
            hipMemcpy(rixd, rix.data(), rix.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(rtd, rt.data(), sizeof(double) * rt.size(), hipMemcpyHostToDevice) != hipSuccess) {
            for (void* q : {(void*)rixd, (void*)rtd}) if (q) (void)hipFree(q);
            return undo(SHD_ROUTE_ENOMEM);
        }
        nrt = (int)rt.size();
    }
    // packed in-list keys (the parent arc's reliability index inside the key): every latency
    // <= 255 and the u8 index matrix built above (SHD_ROUTE_FWPK=0: the wide keys)
    const int pk = rixd && c->max_w <= 255.0 && !(getenv("SHD_ROUTE_FWPK") && atoi(getenv("SHD_ROUTE_FWPK")) == 0);
    hipLaunchKernelGGL(fw_inlist_kernel, dim3(c->n), dim3(1024), 4 * sp, st, c->d_W, c->n, np, sp, inl, pos, rixd, pk);
    if ((rc = hip_check(hipGetLastError()))) {
        for (void* q : {(void*)rixd, (void*)rtd}) if (q) (void)hipFree(q);
        return undo(rc);
    }
    // (published only now: a failed step above leaves the context as it was, and a retry
    // builds every table again)
    if (rixd) {
        c->d_fwrix = rixd;
        c->d_fwrtab = rtd;
        c->allocs.push_back(c->d_fwrix);
        c->allocs.push_back(c->d_fwrtab);
        c->fw_nrtab = nrt;
    }
    c->d_fwD = D;
    c->fw_pk = pk;
    c->d_fwinl = inl;
    c->d_fwpos = pos;
    c->allocs.push_back(D);
    c->allocs.push_back(inl);
    c->allocs.push_back(pos);
    c->fw_np = np;
    return SHD_ROUTE_OK;
}
}  // namespace

extern "C" {

int shd_route_fw_table_async(shd_route_t* c, void* stream) {
    if (!c) return SHD_ROUTE_EINVAL;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    hipStream_t st = (hipStream_t)stream;
    int rc = fw_prepare(c, st);
    if (rc) return rc;
    const int np = c->fw_np, nb = np / FW_T;
    const unsigned blocks = (unsigned)(((size_t)np * np + 255) / 256);
    hipLaunchKernelGGL(fw_init_kernel, dim3(blocks), dim3(256), 0, st, c->d_W, c->n, np, c->d_fwD);
    // rest kernel: 64 x 64 tiles with 4 x 4 register blocks and the next pivot's panels fused in
    // (default: one launch per pivot); SHD_ROUTE_FWREST=1 the separate panel + rest launches,
    // 2 the 128 x 128-region rest kernel with 8 x 8 blocks (C5 FW table 3.28 ms against 3.06)
    const char* fwr = getenv("SHD_ROUTE_FWREST");
    const int mode = fwr ? atoi(fwr) : 3;
    if ((mode == 0 || mode == 3) && nb > 1) {
        if (!c->d_fwflag) {
            if (hipMalloc((void**)&c->d_fwflag, sizeof(int) * (size_t)(nb + 1)) != hipSuccess) return SHD_ROUTE_ENOMEM;
            c->allocs.push_back(c->d_fwflag);
        }
        if (hipMemsetAsync(c->d_fwflag, 0, sizeof(int) * (size_t)(nb + 1), st) != hipSuccess) return SHD_ROUTE_EDEVICE;
        hipLaunchKernelGGL(fw_diag_kernel<FW_T>, dim3(1), dim3(256), 0, st, c->d_fwD, np, 0);
        hipLaunchKernelGGL(fw_panel_kernel<FW_T>, dim3(nb - 1, 2), dim3(256), 0, st, c->d_fwD, np, 0);
        int P = 1024;  // mode 3: persistent plain-tile workgroups
        if (const char* e = getenv("SHD_ROUTE_FWP")) P = std::max(1, atoi(e));
        for (int kb = 0; kb < nb; kb++) {
            const int nx = kb + 1 < nb ? 2 : 0;  // the next pivot's panel tiles in row / column kb
            if (mode == 0) {
                hipLaunchKernelGGL(fw_restp_kernel<FW_T>, dim3((nb - 1) * (nb - 1) + nx), dim3(256), 0, st, c->d_fwD, np,
                                   kb, c->d_fwflag, c->d_err);
            } else {
                const int m = kb + 1 < nb ? nb - 2 : nb - 1, pp = std::max(1, std::min(P, m * m));
                const int grid = kb + 1 < nb ? 1 + pp + 2 * m + 2 : pp;
                hipLaunchKernelGGL(fw_restpp_kernel<FW_T>, dim3(grid), dim3(256), 0, st, c->d_fwD, np, kb, c->d_fwflag, pp, c->d_err);
            }
        }
        c->fw_ready = 1;
        return hip_check(hipGetLastError());
    }
    const bool rest1 = mode != 2;
    const int nr = (nb + 1) / 2;
    for (int kb = 0; kb < nb; kb++) {
        // pivot tiles after the first are closed inside the previous fw_rest launch
        if (kb == 0) hipLaunchKernelGGL(fw_diag_kernel<FW_T>, dim3(1), dim3(256), 0, st, c->d_fwD, np, kb);
        if (nb > 1) {
            hipLaunchKernelGGL(fw_panel_kernel<FW_T>, dim3(nb - 1, 2), dim3(256), 0, st, c->d_fwD, np, kb);
            if (rest1)
                hipLaunchKernelGGL(fw_rest_kernel<FW_T>, dim3(nb - 1, nb - 1), dim3(256), 0, st, c->d_fwD, np, kb);
            else
                hipLaunchKernelGGL(fw_rest2_kernel, dim3(nr * nr), dim3(256), 0, st, c->d_fwD, np, kb);
        }
    }
    c->fw_ready = 1;
    return hip_check(hipGetLastError());
}

int shd_route_fw_rows_async(shd_route_t* c, const int32_t* d_src, int32_t ns, const int32_t* d_tgt, int32_t nt,
                            int64_t ld, double* d_lat, double* d_rel, double* d_row_min, void* stream) {
    if (!c || ns < 0 || nt < 0 || (ns && !d_src) || (nt && !d_tgt) || ld < nt) return SHD_ROUTE_EINVAL;
    if (!c->fw_ready) return SHD_ROUTE_EINVAL;  // shd_route_fw_table_async first
    if (ns == 0) return SHD_ROUTE_OK;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    hipStream_t st = (hipStream_t)stream;
    const int np = c->fw_np;
    const size_t need = (size_t)ns * np;
    if (need > c->fwkey_cap) {
        if (c->d_fwkey) (void)hipFree(c->d_fwkey);
        c->d_fwkey = nullptr;
        c->fwkey_cap = 0;
        if (hipMalloc((void**)&c->d_fwkey, need * sizeof(uint32_t)) != hipSuccess) return SHD_ROUTE_ENOMEM;
        c->fwkey_cap = need;
    }
    // (256-thread workgroups: at fw_parent's 70 VGPRs a CU holds seven of them, against one of
    // 1024 threads: C5 rows 1.02 -> 0.94 ms; SHD_ROUTE_FWPBLK=512 / 1024 for the A/B)
    int pblk = 256;
    if (const char* e = getenv("SHD_ROUTE_FWPBLK")) pblk = atoi(e) == 1024 ? 1024 : atoi(e) == 512 ? 512 : 256;
    // eight sources per workgroup where their interleaved rows fit the LDS (C5 rows 0.62 ->
    // 0.41 ms at 1024 threads, 0.44 at 512, 0.50 at 256; SHD_ROUTE_FWP8=0: one source per
    // workgroup, SHD_ROUTE_FWP8BLK=512 / 256 for the A/B)
    const bool p8 = (size_t)16 * np <= kLdsBudget && !(getenv("SHD_ROUTE_FWP8") && atoi(getenv("SHD_ROUTE_FWP8")) == 0);
    int p8blk = 1024;
    if (const char* e = getenv("SHD_ROUTE_FWP8BLK")) p8blk = atoi(e) == 512 ? 512 : atoi(e) == 256 ? 256 : 1024;
    if (p8 && c->fw_pk)
        hipLaunchKernelGGL(fw_parent8_kernel<true>, dim3(std::min((ns + 7) / 8, 2048)), dim3(p8blk), 16 * np, st, c->d_fwD,
                           c->d_fwinl, c->d_fwpos, c->n, np, d_src, ns, c->d_fwkey);
    else if (p8)
        hipLaunchKernelGGL(fw_parent8_kernel<false>, dim3(std::min((ns + 7) / 8, 2048)), dim3(p8blk), 16 * np, st, c->d_fwD,
                           c->d_fwinl, c->d_fwpos, c->n, np, d_src, ns, c->d_fwkey);
    else if (c->fw_pk)
        hipLaunchKernelGGL(fw_parent_kernel<true>, dim3(std::min(ns, 8192)), dim3(pblk), 2 * np, st, c->d_fwD, c->d_fwinl,
                           c->d_fwpos, c->n, np, d_src, ns, c->d_fwkey);
    else
        hipLaunchKernelGGL(fw_parent_kernel<false>, dim3(std::min(ns, 8192)), dim3(pblk), 2 * np, st, c->d_fwD, c->d_fwinl,
                           c->d_fwpos, c->n, np, d_src, ns, c->d_fwkey);
    FWRowsArgs a;
    a.pk = c->fw_pk;
    a.n = c->n; a.np = np; a.bound = c->k32_bound; a.D = c->d_fwD; a.key = c->d_fwkey; a.R = c->d_R;
    a.rix = c->d_fwrix; a.rtab = c->d_fwrtab; a.nrtab = c->d_fwrix ? c->fw_nrtab : 0;
    a.vf = c->d_vf; a.self_w = c->d_self_w; a.self_r = c->d_self_r;
    const size_t lds = a16(sizeof(double) * c->n) + a16(sizeof(uint16_t) * c->n) + a16(sizeof(int) * (c->k32_bound + 2));
    // (512-thread workgroups since the u16 order list: C5 rows 0.92 -> 0.81 ms against 1024,
    // 0.86 at 256; SHD_ROUTE_FWRBLK=1024 / 256 for the A/B)
    int rblk = 512;
    if (const char* e = getenv("SHD_ROUTE_FWRBLK")) rblk = atoi(e) == 1024 ? 1024 : atoi(e) == 256 ? 256 : 512;
    hipLaunchKernelGGL(fw_rows_kernel, dim3(std::min(ns, 2048)), dim3(rblk), lds, st, a, d_src, ns, d_tgt, nt,
                       (long long)ld, d_lat, d_rel, d_row_min, c->d_err);
    return hip_check(hipGetLastError());
}

}  // extern "C"

// =============================================================================
// Eager fill of the front end's dense upper-triangle Path cache
// =============================================================================
namespace {
// pack rows [r0, r1) of the planned table into the triangle layout: row r (source A[i],
// i = pos[r]) keeps targets j >= i, as interleaved (lat, rel) pairs; one workgroup per
// row; row minima over the kept entries (NaN skipped) into *mn (u64 bits)
__global__ __launch_bounds__(256) void tri_pack_kernel(const double* __restrict__ lat, const double* __restrict__ rel,
                                                       long long ld, const int* __restrict__ pos,
                                                       const long long* __restrict__ off, int r0, int r1, int na,
                                                       double* __restrict__ out, unsigned long long* __restrict__ mn) {
    for (int r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
        const int i = pos[r];
        const double* lr = lat + (long long)r * ld;
        const double* rr = rel + (long long)r * ld;
        double* o = out + 2 * (off[r] - off[r0]);
        double m = INFINITY;
        for (int j = i + threadIdx.x; j < na; j += 256) {
            const double L = lr[j];
            o[2 * (j - i)] = L;
            o[2 * (j - i) + 1] = rr[j];
            if (!isnan(L)) m = fmin(m, L);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) m = fmin(m, __shfl_xor(m, d, 64));
        if ((threadIdx.x & 63) == 0 && m < INFINITY) atomicMin(mn, as_u(m));
    }
}

// the same into the compact SHD_ROUTE_FILL_LAT16 layout: row r's pairs six to a 64-byte line
// (rel f64 x 6, lat u16 x 6 with NaN -> 0xFFFF, 4 pad bytes) from line loff[r] - loff[r0]
__global__ __launch_bounds__(256) void tri_pack16_kernel(const double* __restrict__ lat, const double* __restrict__ rel,
                                                         long long ld, const int* __restrict__ pos,
                                                         const long long* __restrict__ loff, int r0, int r1, int na,
                                                         uint4* __restrict__ out, unsigned long long* __restrict__ mn) {
    for (int r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
        const int i = pos[r];
        const double* lr = lat + (long long)r * ld;
        const double* rr = rel + (long long)r * ld;
        uint4* o = out + 4 * (loff[r] - loff[r0]);
        const int nl = (na - i + 5) / 6;
        double m = INFINITY;
        for (int l = threadIdx.x; l < nl; l += 256) {
            double R[6];
            uint32_t L16[3] = {0u, 0u, 0u};
#pragma unroll
            for (int e = 0; e < 6; e++) {
                const int j = i + 6 * l + e;
                const double L = j < na ? lr[j] : NAN;
                R[e] = j < na ? rr[j] : 0.0;
                if (!isnan(L)) m = fmin(m, L);
                const uint32_t x = isnan(L) ? 0xFFFFu : (uint32_t)L;
                L16[e >> 1] |= x << (16 * (e & 1));
            }
            uint4* q = o + 4 * (long long)l;
            q[0] = make_uint4((uint32_t)as_u(R[0]), (uint32_t)(as_u(R[0]) >> 32), (uint32_t)as_u(R[1]), (uint32_t)(as_u(R[1]) >> 32));
            q[1] = make_uint4((uint32_t)as_u(R[2]), (uint32_t)(as_u(R[2]) >> 32), (uint32_t)as_u(R[3]), (uint32_t)(as_u(R[3]) >> 32));
            q[2] = make_uint4((uint32_t)as_u(R[4]), (uint32_t)(as_u(R[4]) >> 32), (uint32_t)as_u(R[5]), (uint32_t)(as_u(R[5]) >> 32));
            q[3] = make_uint4(L16[0], L16[1], L16[2], 0u);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) m = fmin(m, __shfl_xor(m, d, 64));
        if ((threadIdx.x & 63) == 0 && m < INFINITY) atomicMin(mn, as_u(m));
    }
}

// multi-GPU table assembly payload: row r (caller position pos[r] in the attached list)
// keeps its upper-triangle targets j >= pos[r]; lat goes out as u16 (integer latencies
// below 65535, NaN -> 0xFFFF) or f64, rel as f64, each into its own packed array at
// element offset off[r] - off[0]
template <bool L16>
__global__ __launch_bounds__(256) void tri_payload_kernel(const double* __restrict__ lat, const double* __restrict__ rel,
                                                          long long ld, const int* __restrict__ pos,
                                                          const long long* __restrict__ off, int nrows, int na,
                                                          void* __restrict__ out_lat, double* __restrict__ out_rel) {
    const long long base = off[0];
    for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
        const int i = pos[r];
        const double* lr = lat + (long long)r * ld;
        const double* rr = rel + (long long)r * ld;
        const long long o = off[r] - base;
        for (int j = i + threadIdx.x; j < na; j += 256) {
            const double L = __builtin_nontemporal_load(lr + j);
            if (L16) {
                const uint16_t x = isnan(L) ? (uint16_t)0xFFFFu : (uint16_t)L;
                static_cast<uint16_t*>(out_lat)[o + (j - i)] = x;
            } else {
                static_cast<double*>(out_lat)[o + (j - i)] = L;
            }
            out_rel[o + (j - i)] = __builtin_nontemporal_load(rr + j);
        }
    }
}
}  // namespace

// Pinned host memory for the fill's triangle (C4: 13.3 GB compact, 20 GB interleaved).
// hipHostMalloc faults and pins 4 KiB pages one by one (3.4 s for 20 GiB on the box);
// anonymous memory advised as transparent huge pages, populated by several threads and
// registered takes ~0.15 s for the same D2H rate (tools/micro/pin_bench.cpp).  It is
// first-touched and registered in 256 MiB chunks by worker threads, lowest chunk first, so
// that the fill's copies (shd_route_fill_triangle waits for each chunk it copies into)
// overlap the pinning of the chunks after them instead of waiting for the whole triangle.
// On the box (tools/micro/pin_overlap.cpp, 8 GiB): 16-thread first-touch 136 GB/s against
// 30 GB/s for MADV_POPULATE_WRITE, registering touched pages 0.5 GB/ms, and a D2H runs at
// its full 57 GB/s while other threads touch and register.  (A copy must not span two
// registrations: the runtime fails it.)  hipHostMalloc stays the fallback.
namespace {
struct HostMap {
    char* base = nullptr;  // the mapping (munmap)
    size_t maplen = 0;
    char* p = nullptr;     // the caller's pointer (2 MiB aligned)
    size_t len = 0;
    size_t chunk = (size_t)256 << 20;
    int nchunk = 0;
    std::unique_ptr<std::atomic<int>[]> state;  // per chunk: 0 pending, 1 registered, 2 not registered
    bool whole = false;    // eager form: chunks are only first-touched (state 1 = touched), then
                           // the whole range is registered once, so any copy may span it
    bool whole_reg = false;
    std::atomic<int> next{0};
    std::atomic<bool> stop{false};
    int fail_chunk = getenv("SHD_ROUTE_REGFAIL_CHUNK") ? atoi(getenv("SHD_ROUTE_REGFAIL_CHUNK")) : -1;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::thread> th;
    // wait until every chunk overlapping [off, off + n) is settled (registered or failed)
    void wait_range(size_t off, size_t n) {
        if (!n) return;
        const int c0 = (int)(off / chunk), c1 = (int)std::min<size_t>((off + n - 1) / chunk, nchunk - 1);
        auto settled = [&] {
            for (int k = c0; k <= c1; k++)
                if (state[k].load(std::memory_order_acquire) == 0) return false;
            return true;
        };
        if (settled()) return;
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, settled);
    }
    void worker() {
        for (int k; !stop.load(std::memory_order_relaxed) && (k = next.fetch_add(1)) < nchunk;) {
            char* a = p + (size_t)k * chunk;
            const size_t n = std::min(chunk, len - (size_t)k * chunk);
            for (size_t o = 0; o < n; o += 4096) a[o] = 0;  // (nothing else touches a pending chunk)
            // (SHD_ROUTE_REGFAIL_CHUNK=k: chunk k is left unregistered, as when the runtime
            // refuses it -- the non-fatal path's test)
            const bool ok = whole || (k != fail_chunk && hipHostRegister(a, n, hipHostRegisterPortable) == hipSuccess);
            {
                std::lock_guard<std::mutex> lk(mu);
                state[k].store(ok ? 1 : 2, std::memory_order_release);
            }
            cv.notify_all();
        }
    }
    ~HostMap() {
        stop = true;
        for (auto& t : th) t.join();
        if (whole) {
            if (whole_reg) (void)hipHostUnregister(p);
        } else {
            for (int k = 0; k < nchunk; k++)
                if (state[k].load() == 1) (void)hipHostUnregister(p + (size_t)k * chunk);
        }
        if (base) munmap(base, maplen);
    }
};
std::mutex g_host_mu;
std::map<char*, std::shared_ptr<HostMap>> g_host_maps;  // by the caller's pointer

std::shared_ptr<HostMap> host_map_of(const void* q) {
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host_maps.upper_bound((char*)q);
    if (it == g_host_maps.begin()) return nullptr;
    --it;
    return (const char*)q < it->first + it->second->len ? it->second : nullptr;
}

void* host_alloc(size_t bytes, bool lazy) {
    if (!bytes) bytes = 1;
    const size_t huge = (size_t)2 << 20;
    const size_t len = (bytes + huge - 1) & ~(huge - 1);
    auto m = std::make_shared<HostMap>();
    void* b = mmap(nullptr, len + huge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (b != MAP_FAILED) {
        m->base = (char*)b;
        m->maplen = len + huge;
        m->p = (char*)(((uintptr_t)b + huge - 1) & ~(uintptr_t)(huge - 1));  // whole huge pages
        m->len = len;
        (void)madvise(m->p, len, MADV_HUGEPAGE);
        m->nchunk = (int)((len + m->chunk - 1) / m->chunk);
        m->state.reset(new std::atomic<int>[m->nchunk]());
        m->whole = !lazy;
        const int nth = std::min(m->nchunk, 12);
        for (int t = 0; t < nth; t++) m->th.emplace_back([mp = m.get()] { mp->worker(); });
        bool ok = true;
        if (!lazy) {
            // touched in parallel, then one registration (a caller's single large copy into
            // the buffer must not span two registrations); on failure, hipHostMalloc below
            m->wait_range(0, len);
            m->whole_reg = ok = hipHostRegister(m->p, len, hipHostRegisterPortable) == hipSuccess;
        }
        if (ok) {
            std::lock_guard<std::mutex> lk(g_host_mu);
            g_host_maps[m->p] = m;
            return m->p;
        }
        m.reset();  // (joins the touch workers and unmaps)
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) return nullptr;
    return p;
}
}  // namespace

extern "C" {

int shd_route_tri_payload_async(shd_route_t* c, const double* d_lat, const double* d_rel, int64_t ld,
                                const int32_t* d_pos, const int64_t* d_off, int32_t nrows, int32_t na, uint32_t flags,
                                void* d_out_lat, double* d_out_rel, void* stream) {
    if (!c || nrows < 0 || na < 0 || ld < na || (nrows && (!d_lat || !d_rel || !d_pos || !d_off || !d_out_lat || !d_out_rel)))
        return SHD_ROUTE_EINVAL;
    const bool l16 = (flags & SHD_ROUTE_PAYLOAD_LAT16) != 0;
    if (l16 && !lat16_ok(c)) return SHD_ROUTE_EUNSUPPORTED;
    if (nrows == 0) return SHD_ROUTE_OK;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(std::min(nrows, 8192));
    if (l16)
        hipLaunchKernelGGL(tri_payload_kernel<true>, grid, dim3(256), 0, st, d_lat, d_rel, (long long)ld, d_pos,
                           (const long long*)d_off, nrows, na, d_out_lat, d_out_rel);
    else
        hipLaunchKernelGGL(tri_payload_kernel<false>, grid, dim3(256), 0, st, d_lat, d_rel, (long long)ld, d_pos,
                           (const long long*)d_off, nrows, na, d_out_lat, d_out_rel);
    return hip_check(hipGetLastError());
}

void* shd_route_host_alloc(size_t bytes) { return host_alloc(bytes, false); }

void* shd_route_host_alloc_lazy(size_t bytes) { return host_alloc(bytes, true); }

int shd_route_host_wait(void* p) {
    if (!p) return SHD_ROUTE_EINVAL;
    auto m = host_map_of(p);
    if (!m) return SHD_ROUTE_OK;
    m->wait_range(0, m->len);
    // a chunk the runtime refused to register stays pageable: copies into it still work
    // (slower) and the data is complete, so this is not an error; shd_route_host_unpinned
    // counts such chunks
    return SHD_ROUTE_OK;
}

int64_t shd_route_host_unpinned(void* p) {
    if (!p) return SHD_ROUTE_EINVAL;
    auto m = host_map_of(p);
    if (!m) return 0;
    m->wait_range(0, m->len);
    if (m->whole) return m->whole_reg ? 0 : (int64_t)m->len;
    int64_t bytes = 0;
    for (int k = 0; k < m->nchunk; k++)
        if (m->state[k].load(std::memory_order_acquire) == 2)
            bytes += (int64_t)std::min(m->chunk, m->len - (size_t)k * m->chunk);
    return bytes;
}

void shd_route_host_free(void* p) {
    if (!p) return;
    std::shared_ptr<HostMap> m;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        auto it = g_host_maps.find((char*)p);
        if (it != g_host_maps.end()) { m = std::move(it->second); g_host_maps.erase(it); }
    }
    if (!m) (void)hipHostFree(p);
    // (else the last reference -- a fill still copying holds one -- joins, unregisters, unmaps)
}

int shd_route_fill_triangle(shd_route_t* c, const int32_t* A, int32_t na, int32_t world, int32_t rank, uint32_t flags,
                            double* lr_out, double* min_out, double* seconds_out) {
    if (!c || na < 0 || (na && (!A || !lr_out)) || world < 1 || rank < 0 || rank >= world) return SHD_ROUTE_EINVAL;
    if (min_out) *min_out = INFINITY;
    const bool l16 = (flags & SHD_ROUTE_FILL_LAT16) != 0;
    // u16 latencies are exact for the source paths (info.lat16) and, with the dispatch, for
    // the direct paths it writes (edge latencies)
    if (l16 && !(lat16_ok(c) && (!(flags & SHD_ROUTE_DISPATCH) || !(c->complete || c->prefer_direct) ||
                                 c->max_w < 65535.0)))
        return SHD_ROUTE_EUNSUPPORTED;
    flags &= ~SHD_ROUTE_FILL_LAT16;
    if (na == 0) return SHD_ROUTE_OK;
    if (hipSetDevice(c->device) != hipSuccess) return SHD_ROUTE_EDEVICE;
    auto t0 = std::chrono::steady_clock::now();
    shd_route_plan_t* P = nullptr;
    int rc = shd_route_plan_create(c, A, na, world, rank, &P);
    if (rc) return rc;
    std::unique_ptr<shd_route_plan, void (*)(shd_route_plan*)> guard(P, shd_route_plan_destroy);
    const int nr = (int)P->row_pos.size();
    if (nr == 0) return SHD_ROUTE_OK;
    // triangle offsets of this rank's rows (host: pair index of (i, i)), their sizes
    std::vector<long long> off(nr + 1);
    auto tri0 = [&](long long i) { return i * (long long)na - i * (i - 1) / 2; };
    for (int r = 0; r < nr; r++) off[r] = tri0(P->row_pos[r]);
    off[nr] = off[nr - 1] + (na - P->row_pos[nr - 1]);
    std::vector<long long> roff(nr + 1, 0);  // packed offsets (pairs) in plan row order
    for (int r = 0; r < nr; r++) roff[r + 1] = roff[r] + (na - P->row_pos[r]);
    // the compact layout in 64-byte lines: triangle line of each row, packed lines in row order
    std::vector<long long> loff(nr + 1), rline(nr + 1, 0);
    if (l16) {
        for (int r = 0; r < nr; r++) loff[r] = shd_route_tri16_line(na, P->row_pos[r]);
        for (int r = 0; r < nr; r++) rline[r + 1] = rline[r] + (na - P->row_pos[r] + 5) / 6;
    }
    const size_t table = sizeof(double) * (size_t)nr * (size_t)na;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return SHD_ROUTE_EDEVICE;
    const size_t stage_pairs = (size_t)32 << 20;  // 512 MiB of (lat, rel) per staging buffer
    if (2 * table + 4 * stage_pairs * 8 + ((size_t)1 << 30) > fr) return SHD_ROUTE_ENOMEM;
    DevBuf dtgt, dlat, drel, dpos, doff, dstage[2], dmn;
    if ((rc = dtgt.alloc(sizeof(int32_t) * na)) || (rc = dlat.alloc(table)) || (rc = drel.alloc(table)) ||
        (rc = dpos.alloc(sizeof(int) * nr)) || (rc = doff.alloc(sizeof(long long) * (nr + 1))) ||
        (rc = dstage[0].alloc(16 * stage_pairs)) || (rc = dstage[1].alloc(16 * stage_pairs)) ||
        (rc = dmn.alloc(sizeof(unsigned long long))))
        return rc;
    hipStream_t cs = nullptr, xs = nullptr;
    if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&xs, hipStreamNonBlocking) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    std::vector<int> posv(P->row_pos.begin(), P->row_pos.end());
    bool ok = hipMemcpy(dtgt.p, A, sizeof(int32_t) * na, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(dpos.p, posv.data(), sizeof(int) * nr, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(doff.p, roff.data(), sizeof(long long) * (nr + 1), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemsetAsync(dmn.p, 0xFF, sizeof(unsigned long long), cs) == hipSuccess;
    if (ok && l16)
        ok = hipMemcpy(doff.p, rline.data(), sizeof(long long) * (nr + 1), hipMemcpyHostToDevice) == hipSuccess;
    // (the plan was made just now: its landmark rows, if any, are current)
    if (ok) rc = shd_route_rows_planned_async(c, P, (const int32_t*)dtgt.p, na, na, flags | SHD_ROUTE_PLAN_REUSE, (double*)dlat.p,
                                              (double*)drel.p, nullptr, cs);
    else rc = SHD_ROUTE_EDEVICE;
    // pack chunks of rows on the compute stream, copy them out on the copy stream; with
    // rows in triangle order (one rank) a chunk is one contiguous range of the cache
    hipEvent_t packed[2], copied[2];
    for (int b = 0; b < 2; b++) { (void)hipEventCreateWithFlags(&packed[b], hipEventDisableTiming); (void)hipEventCreateWithFlags(&copied[b], hipEventDisableTiming); }
    int buf = 0;
    bool first[2] = {true, true};
    // into memory of shd_route_host_alloc_lazy: a copy waits for the chunks it lands in to be
    // pinned, and never spans two chunks (each is its own registration)
    const std::shared_ptr<HostMap> hm = host_map_of(lr_out);
    auto copy_out = [&](char* dst, const char* src, size_t bytes) {
        while (bytes) {
            size_t nb = bytes;
            if (hm) {
                const size_t o = (size_t)(dst - hm->p);
                nb = std::min(nb, (o / hm->chunk + 1) * hm->chunk - o);
                hm->wait_range(o, nb);
            }
            if (hipMemcpyAsync(dst, src, nb, hipMemcpyDeviceToHost, xs) != hipSuccess) return false;
            dst += nb; src += nb; bytes -= nb;
        }
        return true;
    };
    const std::vector<long long>& pk = l16 ? rline : roff;  // packed units: lines or pairs
    const long long stage_units = l16 ? (long long)(16 * stage_pairs / 64) : (long long)stage_pairs;
    for (int r0 = 0; r0 < nr && !rc; buf ^= 1) {
        int r1 = r0;
        while (r1 < nr && pk[r1 + 1] - pk[r0] <= stage_units) r1++;
        if (r1 == r0) r1 = r0 + 1;  // (a row longer than a stage buffer cannot happen: na < 2^25)
        if (!first[buf] && hipStreamWaitEvent(cs, copied[buf], 0) != hipSuccess) { rc = SHD_ROUTE_EDEVICE; break; }
        first[buf] = false;
        if (l16)
            hipLaunchKernelGGL(tri_pack16_kernel, dim3(std::min(r1 - r0, 4096)), dim3(256), 0, cs, (const double*)dlat.p,
                               (const double*)drel.p, (long long)na, (const int*)dpos.p, (const long long*)doff.p, r0, r1,
                               na, (uint4*)dstage[buf].p, (unsigned long long*)dmn.p);
        else
            hipLaunchKernelGGL(tri_pack_kernel, dim3(std::min(r1 - r0, 4096)), dim3(256), 0, cs, (const double*)dlat.p,
                               (const double*)drel.p, (long long)na, (const int*)dpos.p, (const long long*)doff.p, r0, r1,
                               na, (double*)dstage[buf].p, (unsigned long long*)dmn.p);
        if (hipGetLastError() != hipSuccess || hipEventRecord(packed[buf], cs) != hipSuccess ||
            hipStreamWaitEvent(xs, packed[buf], 0) != hipSuccess) { rc = SHD_ROUTE_EDEVICE; break; }
        // copy: consecutive rows with consecutive triangle offsets go out in one piece
        for (int a = r0; a < r1;) {
            int b = a + 1;
            if (l16) {
                while (b < r1 && loff[b] == loff[b - 1] + (na - P->row_pos[b - 1] + 5) / 6) b++;
                const size_t lines = (size_t)(rline[b] - rline[a]);
                if (!copy_out((char*)lr_out + 64 * loff[a], (char*)dstage[buf].p + 64 * (rline[a] - rline[r0]), 64 * lines)) {
                    rc = SHD_ROUTE_EDEVICE;
                    break;
                }
            } else {
                while (b < r1 && off[b] == off[b - 1] + (na - P->row_pos[b - 1])) b++;
                const size_t pairs = (size_t)(roff[b] - roff[a]);
                if (!copy_out((char*)(lr_out + 2 * off[a]), (char*)((double*)dstage[buf].p + 2 * (roff[a] - roff[r0])),
                              16 * pairs)) {
                    rc = SHD_ROUTE_EDEVICE;
                    break;
                }
            }
            a = b;
        }
        if (hipEventRecord(copied[buf], xs) != hipSuccess) rc = SHD_ROUTE_EDEVICE;
        r0 = r1;
    }
    if (hipStreamSynchronize(cs) != hipSuccess || hipStreamSynchronize(xs) != hipSuccess) rc = rc ? rc : SHD_ROUTE_EDEVICE;
    for (int b = 0; b < 2; b++) { (void)hipEventDestroy(packed[b]); (void)hipEventDestroy(copied[b]); }
    (void)hipStreamDestroy(cs); (void)hipStreamDestroy(xs);
    if (rc) return rc;
    const int soft = take_err(c);
    if (soft && soft != SHD_ROUTE_ENOEDGE && soft != SHD_ROUTE_EUNREACH) return soft;
    unsigned long long mb = 0;
    if (hipMemcpy(&mb, dmn.p, sizeof(mb), hipMemcpyDeviceToHost) != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (min_out) {
        double m;
        std::memcpy(&m, &mb, sizeof(m));
        *min_out = mb == ~0ull ? INFINITY : m;
    }
    if (seconds_out) *seconds_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return soft;
}

}  // extern "C"

extern "C" int shd_route_kd_stats(shd_route_t* c, uint64_t* out, int reset) {
    if (!c || !out) return SHD_ROUTE_EINVAL;
    for (int q = 0; q < 4; q++) out[q] = 0;
    if (!c->d_kd_stats) return SHD_ROUTE_OK;
    if (hipSetDevice(c->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return SHD_ROUTE_EDEVICE;
    if (hipMemcpy(out, c->d_kd_stats, sizeof(uint64_t) * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return SHD_ROUTE_EDEVICE;
    if (reset && hipMemset(c->d_kd_stats, 0, sizeof(uint64_t) * 4) != hipSuccess) return SHD_ROUTE_EDEVICE;
    return SHD_ROUTE_OK;
}

#ifdef SHD_STAMPS
// Diagnostic builds only (not part of include/shd_route.h): per-source phase stamps.
extern "C" int shd_route_debug_buffer(shd_route_t* c, void* d_buf) {
    if (!c) return SHD_ROUTE_EINVAL;
    c->d_dbg = (unsigned long long*)d_buf;
    return SHD_ROUTE_OK;
}
#endif
