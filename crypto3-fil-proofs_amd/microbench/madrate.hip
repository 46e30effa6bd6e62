// madrate.hip -- v_mad_u64_u32 issue rate on gfx950, three forms of 8 independent 64-bit chains
// per lane: (a) every MAD writes VCC as its carry-out, (b) each chain has its own SGPR-pair carry-out,
// (c) compiler-emitted (plain C, varying multiplicand).  Used to set bench.py's VALU roofline peak.
//   hipcc -O3 --offload-arch=gfx950 madrate.hip -o madrate && ./madrate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

__global__ void k_vcc(uint32_t *out, int iters) {
    uint32_t a = threadIdx.x + 1, b = blockIdx.x + 3;
    uint64_t acc[8];
    for (int i = 0; i < 8; i++) acc[i] = i * 77 + threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "vcc");
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s ^= acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void k_sgpr(uint32_t *out, int iters) {
    uint32_t a = threadIdx.x + 1, b = blockIdx.x + 3;
    uint64_t acc[8], c[8];
    for (int i = 0; i < 8; i++) acc[i] = i * 77 + threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(c[i]) : "v"(a), "v"(b));
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s ^= acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void k_plain(uint32_t *out, int iters) {
    uint32_t b = blockIdx.x + 3;
    uint64_t acc[8];
    for (int i = 0; i < 8; i++) acc[i] = i * 77 + threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) acc[i] = (uint64_t)(uint32_t)acc[i] * b + (acc[i] >> 32);
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s ^= acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

template <class K>
static float timeit(K k, dim3 g, dim3 b, uint32_t *o, int it) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k<<<g, b>>>(o, 10);
    hipEventRecord(e0);
    k<<<g, b>>>(o, it);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    const int threads = 256, blocks = 256 * 16;
    const size_t nt = (size_t)threads * blocks;
    uint32_t *o;
    CHECK(hipMalloc(&o, nt * 4));
    const int it = 4000;
    const double ops = (double)nt * it * 8;
    const char *names[3] = {"vcc carry-out", "per-chain SGPR carry-out", "compiler-emitted"};
    float ms[3] = {timeit(k_vcc, dim3(blocks), dim3(threads), o, it), timeit(k_sgpr, dim3(blocks), dim3(threads), o, it),
                   timeit(k_plain, dim3(blocks), dim3(threads), o, it)};
    for (int i = 0; i < 3; i++)
        printf("v_mad_u64_u32 %-26s: %6.2f T lane-ops/s (%.2f cycles per wave64 instr per SIMD @2.4 GHz)\n", names[i],
               ops / ms[i] / 1e9, 1024.0 * 64 * 2.4e9 / (ops / ms[i] * 1e3));
    return 0;
}
