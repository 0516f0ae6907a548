// Packed-u16 VALU throughput on gfx950: the roof K4's min-plus runs against.
// Each thread runs ITER steps of 8 independent (v_pk_add_u16 saturating + v_pk_min_u16) pairs
// (16 packed instructions, 32 u16 relaxations); reports relaxations/s over the whole chip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;
__global__ __launch_bounds__(256) void pk_kernel(uint32_t* out, uint32_t seed) {
    us2 a[8], b[8];
    for (int i = 0; i < 8; i++) {
        a[i] = __builtin_bit_cast(us2, seed * (threadIdx.x + 7u * i));
        b[i] = __builtin_bit_cast(us2, seed ^ (blockIdx.x + 13u * i));
    }
    const us2 c = __builtin_bit_cast(us2, seed | 0x00010001u);
    for (int k = 0; k < ITER; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const us2 t = __builtin_elementwise_add_sat(a[i], c);
            b[i] = __builtin_elementwise_min(b[i], t);
            a[i] = __builtin_elementwise_add_sat(b[i], c);
        }
    }
    uint32_t x = 0;
    for (int i = 0; i < 8; i++) x ^= __builtin_bit_cast(uint32_t, b[i]) ^ __builtin_bit_cast(uint32_t, a[i]);
    if (x == 0x12345678u) out[0] = x;
}
__global__ __launch_bounds__(256) void u32_kernel(uint32_t* out, uint32_t seed) {
    uint32_t a[8], b[8];
    for (int i = 0; i < 8; i++) { a[i] = seed * (threadIdx.x + 7u * i); b[i] = seed ^ (blockIdx.x + 13u * i); }
    const uint32_t c = seed | 1u;
    for (int k = 0; k < ITER; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) { const uint32_t t = a[i] + c; b[i] = min(b[i], t); a[i] = b[i] + c; }
    }
    uint32_t x = 0;
    for (int i = 0; i < 8; i++) x ^= b[i] ^ a[i];
    if (x == 0x12345678u) out[0] = x;
}
int main() {
    uint32_t* d;
    hipMalloc(&d, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int wg_per_cu : {4, 8}) {
        const int grid = 256 * wg_per_cu;
        for (int kind = 0; kind < 2; kind++) {
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (kind == 0) hipLaunchKernelGGL(pk_kernel, dim3(grid), dim3(256), 0, 0, d, 12345u);
                else hipLaunchKernelGGL(u32_kernel, dim3(grid), dim3(256), 0, 0, d, 12345u);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                // instructions per thread: ITER * 8 * 3 VALU (add, min, add)
                const double instr = (double)grid * 256 * ITER * 8 * 3;
                if (rep == 1)
                    printf("%s waves/SIMD %d: %.3f ms, %.1f T lane-instr/s (%s)\n", kind == 0 ? "pk_u16" : "u32   ",
                           wg_per_cu, ms, instr / (ms * 1e-3) / 1e12,
                           kind == 0 ? "x2 u16 ops each" : "1 op each");
            }
        }
    }
    return 0;
}
