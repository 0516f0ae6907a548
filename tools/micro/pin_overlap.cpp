// Can pinning the fill's triangle overlap its D2H?  Times, for a <GiB> buffer:
//  1. populate: 16-thread first-touch stores vs 16-thread MADV_POPULATE_WRITE (THP)
//  2. register: one hipHostRegister of the whole buffer vs 256 MiB chunks (1 thread, 8 threads)
//  3. overlap: D2H into a registered buffer A alone, then while another thread populates +
//     registers a buffer B of the same size
// hipcc -O2 -o tools/micro/pin_overlap tools/micro/pin_overlap.cpp -lpthread ; ./tools/micro/pin_overlap 8
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static char* map_huge(size_t bytes) {
    char* p = (char*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) { printf("mmap failed\n"); exit(1); }
    madvise(p, bytes, MADV_HUGEPAGE);
    return p;
}

static void par(size_t bytes, int nth, void (*f)(char*, size_t), char* p) {
    std::vector<std::thread> th;
    const size_t per = ((bytes + nth - 1) / nth + 4095) & ~(size_t)4095;
    for (int t = 0; t < nth; t++)
        th.emplace_back([=] {
            const size_t a = per * t, b = std::min(bytes, a + per);
            if (a < b) f(p + a, b - a);
        });
    for (auto& x : th) x.join();
}
static void touch(char* p, size_t n) { for (size_t o = 0; o < n; o += 4096) p[o] = 0; }
static void populate(char* p, size_t n) { if (madvise(p, n, MADV_POPULATE_WRITE)) touch(p, n); }

static double d2h(void* host, size_t bytes, void* dev, size_t dbytes, hipStream_t st) {
    (void)hipStreamSynchronize(st);
    const double t0 = now();
    for (size_t o = 0; o < bytes; o += dbytes)
        (void)hipMemcpyAsync((char*)host + o, dev, std::min(dbytes, bytes - o), hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    return bytes / (now() - t0) / 1e9;
}

int main(int argc, char** argv) {
    const size_t gib = argc > 1 ? (size_t)atol(argv[1]) : 8;
    const size_t bytes = gib << 30, chunk = (size_t)256 << 20;
    void* dev = nullptr;
    const size_t dbytes = (size_t)512 << 20;
    if (hipMalloc(&dev, dbytes) != hipSuccess) return 1;
    (void)hipMemset(dev, 1, dbytes);
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (int mode = 0; mode < 2; mode++) {
        char* p = map_huge(bytes);
        const double t0 = now();
        par(bytes, 16, mode ? populate : touch, p);
        const double t1 = now();
        printf("populate %s 16 threads: %.3f s (%.1f GB/s)\n", mode ? "MADV_POPULATE_WRITE" : "touch", t1 - t0, bytes / (t1 - t0) / 1e9);
        munmap(p, bytes);
    }
    for (int mode = 0; mode < 3; mode++) {
        char* p = map_huge(bytes);
        par(bytes, 16, touch, p);
        const double t0 = now();
        if (mode == 0) {
            (void)hipHostRegister(p, bytes, hipHostRegisterPortable);
        } else {
            const int nth = mode == 1 ? 1 : 8;
            std::atomic<size_t> next{0};
            std::vector<std::thread> th;
            for (int t = 0; t < nth; t++)
                th.emplace_back([&] {
                    for (size_t o; (o = next.fetch_add(chunk)) < bytes;) (void)hipHostRegister(p + o, std::min(chunk, bytes - o), hipHostRegisterPortable);
                });
            for (auto& x : th) x.join();
        }
        const double t1 = now();
        const double bw = d2h(p, bytes, dev, dbytes, st);
        printf("register %s: %.3f s, then D2H %.1f GB/s\n", mode == 0 ? "whole" : mode == 1 ? "256 MiB chunks, 1 thread" : "256 MiB chunks, 8 threads", t1 - t0, bw);
        if (mode == 0) (void)hipHostUnregister(p);
        else for (size_t o = 0; o < bytes; o += chunk) (void)hipHostUnregister(p + o);
        munmap(p, bytes);
    }
    {
        char* a = map_huge(bytes);
        par(bytes, 16, touch, a);
        (void)hipHostRegister(a, bytes, hipHostRegisterPortable);
        const double alone = d2h(a, bytes, dev, dbytes, st);
        for (int mode = 0; mode < 3; mode++) {
            char* b = map_huge(bytes);
            std::atomic<int> done{0};
            double tb = 0;
            std::thread bg([&] {
                const double t0 = now();
                if (mode == 0) par(bytes, 8, populate, b);
                else if (mode == 1) { par(bytes, 8, populate, b); (void)hipHostRegister(b, bytes, hipHostRegisterPortable); }
                else for (size_t o = 0; o < bytes; o += chunk) { populate(b + o, std::min(chunk, bytes - o)); (void)hipHostRegister(b + o, std::min(chunk, bytes - o), hipHostRegisterPortable); }
                tb = now() - t0;
                done = 1;
            });
            const double t0 = now();
            const double bw = d2h(a, bytes, dev, dbytes, st);
            const double td = now() - t0;
            bg.join();
            printf("D2H alone %.1f GB/s; during background %s: %.1f GB/s (D2H %.3f s, background %.3f s)\n", alone,
                   mode == 0 ? "populate (8 thr)" : mode == 1 ? "populate (8 thr) + one register" : "chunked populate+register (1 thr)",
                   bw, td, tb);
            if (mode == 1) (void)hipHostUnregister(b);
            if (mode == 2) for (size_t o = 0; o < bytes; o += chunk) (void)hipHostUnregister(b + o);
            munmap(b, bytes);
        }
        (void)hipHostUnregister(a);
        munmap(a, bytes);
    }
    (void)hipFree(dev);
    return 0;
}
