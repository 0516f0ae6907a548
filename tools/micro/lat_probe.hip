// Latency probe: dependent global gathers / store->load serialization / LDS chains under
// a full-chip load (256 workgroups x 1024 threads, one per CU), as in the KD kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdint>

__global__ __launch_bounds__(1024) void probe(const uint32_t* __restrict__ tab, size_t mask, double* __restrict__ scratch,
                                              unsigned long long* out, int rounds, int mode) {
    __shared__ uint16_t lds[50000];
    const int tid = threadIdx.x;
    for (int v = tid; v < 50000; v += 1024) lds[v] = (uint16_t)((v * 2654435761u) % 50000);
    __syncthreads();
    double* my = scratch + (size_t)blockIdx.x * 50000;
    uint32_t x = (tid * 97u + blockIdx.x * 131u) & mask;
    unsigned acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < rounds; r++) {
        if (mode == 0) {            // dependent global gather chain
            x = tab[x] & mask;
        } else if (mode == 1) {     // gather then store (next gather waits for the store: one vmcnt)
            x = tab[x] & mask;
            my[x % 50000] = (double)x;
        } else if (mode == 2) {     // 8 independent gathers per round
            uint32_t y[8];
#pragma unroll
            for (int q = 0; q < 8; q++) y[q] = tab[(x + q * 4099u) & mask];
#pragma unroll
            for (int q = 0; q < 8; q++) x ^= y[q];
            x &= mask;
        } else if (mode == 3) {     // dependent LDS chain
            x = lds[x % 50000];
        } else if (mode == 4) {     // store-only then gather of the same scratch slot
            my[x % 50000] = (double)r;
            x = (uint32_t)(my[(x * 7u) % 50000]) + tab[x & mask];
            x &= mask;
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    acc += x;
    if (tid == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = acc; }
}

int main() {
    const size_t N = 16u << 20;  // 64 MB table (> L2, < MALL)
    std::vector<uint32_t> h(N);
    uint64_t s = 88172645463325252ull;
    for (size_t i = 0; i < N; i++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = (uint32_t)s; }
    uint32_t* d; double* sc; unsigned long long* o;
    hipMalloc(&d, N * 4); hipMemcpy(d, h.data(), N * 4, hipMemcpyHostToDevice);
    hipMalloc(&sc, (size_t)256 * 50000 * 8); hipMalloc(&o, 256 * 16);
    const char* names[] = {"dep gather", "gather+store", "8 indep gathers", "dep LDS u16", "store->load same buf"};
    for (size_t tabsz : {(size_t)1 << 20, (size_t)4 << 20, (size_t)16 << 20}) {  // entries: 4MB,16MB,64MB
        for (int mode = 0; mode < 5; mode++) {
            const int rounds = 200;
            probe<<<256, 1024>>>(d, tabsz - 1, sc, o, rounds, mode);
            hipDeviceSynchronize();
            probe<<<256, 1024>>>(d, tabsz - 1, sc, o, rounds, mode);
            std::vector<unsigned long long> ho(512);
            hipMemcpy(ho.data(), o, 512 * 8, hipMemcpyDeviceToHost);
            double m = 0; for (int b = 0; b < 256; b++) m += ho[b * 2];
            printf("table %4zu MB  %-22s %8.0f cycles/round\n", tabsz * 4 >> 20, names[mode], m / 256 / rounds);
        }
    }
    return 0;
}
