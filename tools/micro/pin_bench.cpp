// Host-memory options for the eager fill's 20 GB triangle (C4): allocation + pinning time
// and D2H rate into the buffer.  hipcc -O2 -o tools/micro/pin_bench tools/micro/pin_bench.cpp -lpthread
//   ./tools/micro/pin_bench <GiB>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void touch(char* p, size_t bytes, int nth) {
    std::vector<std::thread> th;
    const size_t per = (bytes + nth - 1) / nth;
    for (int t = 0; t < nth; t++)
        th.emplace_back([=] {
            const size_t a = per * t, b = std::min(bytes, a + per);
            for (size_t o = a; o < b; o += 4096) p[o] = 0;
        });
    for (auto& x : th) x.join();
}

static double d2h(void* host, size_t bytes, void* dev, size_t dbytes) {
    (void)hipDeviceSynchronize();
    const double t0 = now();
    for (size_t o = 0; o < bytes; o += dbytes)
        (void)hipMemcpyAsync((char*)host + o, dev, std::min(dbytes, bytes - o), hipMemcpyDeviceToHost, nullptr);
    (void)hipDeviceSynchronize();
    return bytes / (now() - t0) / 1e9;
}

int main(int argc, char** argv) {
    const size_t gib = argc > 1 ? (size_t)atol(argv[1]) : 20;
    const size_t bytes = gib << 30;
    const int nth = 16;
    void* dev = nullptr;
    const size_t dbytes = (size_t)1 << 30;
    if (hipMalloc(&dev, dbytes) != hipSuccess) return 1;
    (void)hipMemset(dev, 1, dbytes);
    {
        const double t0 = now();
        void* p = nullptr;
        if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) { printf("hipHostMalloc failed\n"); return 1; }
        const double t1 = now();
        const double bw = d2h(p, bytes, dev, dbytes);
        printf("hipHostMalloc: alloc+pin %.3f s, D2H %.1f GB/s (%.3f s)\n", t1 - t0, bw, bytes / bw / 1e9);
        (void)hipHostFree(p);
    }
    for (int huge = 0; huge < 2; huge++) {
        const double t0 = now();
        char* p = (char*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) { printf("mmap failed\n"); return 1; }
        if (huge) madvise(p, bytes, MADV_HUGEPAGE);
        touch(p, bytes, nth);
        const double t1 = now();
        const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable);
        const double t2 = now();
        if (e != hipSuccess) { printf("hipHostRegister failed (%d)\n", (int)e); munmap(p, bytes); continue; }
        const double bw = d2h(p, bytes, dev, dbytes);
        printf("mmap%s + %d-thread touch %.3f s + hipHostRegister %.3f s = %.3f s, D2H %.1f GB/s\n",
               huge ? "+MADV_HUGEPAGE" : "", nth, t1 - t0, t2 - t1, t2 - t0, bw);
        (void)hipHostUnregister(p);
        munmap(p, bytes);
    }
    {
        // pageable destination: the runtime stages through its own pinned buffers
        const double t0 = now();
        char* p = (char*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        madvise(p, bytes, MADV_HUGEPAGE);
        touch(p, bytes, nth);
        const double t1 = now();
        const double bw = d2h(p, bytes, dev, dbytes);
        printf("pageable (THP, touched %.3f s): D2H %.1f GB/s\n", t1 - t0, bw);
        munmap(p, bytes);
    }
    (void)hipFree(dev);
    return 0;
}
