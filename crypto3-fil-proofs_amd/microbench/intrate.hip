// intrate.hip -- issue rate of the 32-bit integer VALU instructions the SHA-256 kernels are made of
// (v_alignbit_b32, v_bitop3_b32, v_add3_u32, v_add_u32) on gfx950: 8 independent chains per lane, 4 waves
// per SIMD.  Sets the VALU peak of the SDR label / tree D roofline (bench.py VALU_LANE_OPS).
//   hipcc -O3 --offload-arch=gfx950 intrate.hip -o intrate && ./intrate
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

#define KERNEL(name, ASM)                                                              \
    __global__ void __launch_bounds__(256) name(uint32_t *out, int iters) {            \
        uint32_t y = threadIdx.x * 3 + 1, z = blockIdx.x + 5;                          \
        uint32_t x[8];                                                                 \
        for (int i = 0; i < 8; i++) x[i] = i * 77 + threadIdx.x;                       \
        for (int it = 0; it < iters; it++) {                                           \
            _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(ASM : "+v"(x[i]) : "v"(y), "v"(z)); \
        }                                                                              \
        uint32_t s = 0;                                                                \
        for (int i = 0; i < 8; i++) s ^= x[i];                                         \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                \
    }

KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, 7")
KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_add, "v_add_u32_e32 %0, %0, %1")
KERNEL(k_xor, "v_xor_b32_e32 %0, %0, %1")

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount, blocks = cus * 4 * 4, threads = 256, iters = 1 << 14;
    uint32_t *out;
    CHECK(hipMalloc(&out, (size_t)blocks * threads * 4));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    struct K {
        const char *name;
        void (*f)(uint32_t *, int);
    } ks[] = {{"v_alignbit_b32", k_alignbit}, {"v_bitop3_b32", k_bitop3}, {"v_add3_u32", k_add3},
              {"v_add_u32", k_add}, {"v_xor_b32", k_xor}};
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 64);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, iters);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double ops = (double)blocks * threads * iters * 8;
        printf("{\"instr\": \"%s\", \"lane_ops_per_s\": %.4e, \"ms\": %.3f, \"cus\": %d}\n", k.name, ops / (ms * 1e-3),
               ms, cus);
    }
    CHECK(hipFree(out));
    return 0;
}
