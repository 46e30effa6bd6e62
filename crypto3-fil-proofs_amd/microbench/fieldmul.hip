// fieldmul.hip -- microbenchmark: instruction throughput and Montgomery-multiplication variants
// for the 381-bit BLS12-381 base field on gfx950.  Standalone executable (not part of the library).
//
//   raw   : v_mad_u64_u32 and v_add_co/v_addc_co throughput (inline asm, independent chains)
//   v0    : mi::operator* -- 32-bit limbs, no-carry CIOS as the compiler emits it (library today)
//   v1    : 32-bit limbs, product scanning (FIPS), v_mad_u64_u32 accumulating into a 64-bit column
//           register with its hardware carry-out counted by v_addc (inline asm)
//   v2    : 29-bit limbs (14), product scanning; column sums of <= 28 products < 2^58 fit in 64 bits,
//           so each limb product is ONE v_mad_u64_u32 and carries are propagated once per column
// Correctness: v1, v2 results (converted back to canonical) are compared with v0 on random inputs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../csrc/field.h"

using namespace mi;

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s line %d\n", #x, hipGetErrorString(e), __LINE__); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// ------------------------------------------------------------------------------ raw throughput
__global__ void k_raw_mad(uint32_t *out, int iters) {
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
__global__ void k_raw_add(uint32_t *out, int iters) {
    uint32_t a = threadIdx.x + 1;
    uint32_t x[8];
    for (int i = 0; i < 8; i++) x[i] = i * 77 + threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; i++) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_raw_mullo(uint32_t *out, int iters) {
    uint32_t a = threadIdx.x + 1;
    uint32_t x[8];
    for (int i = 0; i < 8; i++) x[i] = i * 77 + threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; i++) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ------------------------------------------------------------------------------ v1: FIPS 32-bit
struct Acc96 {
    uint64_t lo;  // c1:c0
    uint32_t c2;
};
__device__ __forceinline__ void mac(Acc96 &a, uint32_t x, uint32_t y) {
    asm volatile(
        "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(a.lo), "+v"(a.c2)
        : "v"(x), "v"(y)
        : "vcc");
}
__device__ __forceinline__ fq32_t mul_v1(const fq32_t &a, const fq32_t &b) {
    constexpr int N = 12;
    uint32_t m[N], t[N];
    Acc96 acc = {0, 0};
    MI_UNROLL for (int k = 0; k < N; k++) {
        MI_UNROLL for (int i = 0; i < k; i++) {
            mac(acc, a.v[i], b.v[k - i]);
            mac(acc, m[i], FqDesc::MOD[k - i]);
        }
        mac(acc, a.v[k], b.v[0]);
        m[k] = (uint32_t)acc.lo * FqDesc::INV;
        mac(acc, m[k], FqDesc::MOD[0]);
        acc.lo = (acc.lo >> 32) | ((uint64_t)acc.c2 << 32);
        acc.c2 = 0;
    }
    MI_UNROLL for (int k = N; k < 2 * N - 1; k++) {
        MI_UNROLL for (int i = k - N + 1; i < N; i++) {
            mac(acc, a.v[i], b.v[k - i]);
            mac(acc, m[i], FqDesc::MOD[k - i]);
        }
        t[k - N] = (uint32_t)acc.lo;
        acc.lo = (acc.lo >> 32) | ((uint64_t)acc.c2 << 32);
        acc.c2 = 0;
    }
    t[N - 1] = (uint32_t)acc.lo;
    fq32_t r;
    MI_UNROLL for (int i = 0; i < N; i++) r.v[i] = t[i];
    return reduce_once(r);
}

// ------------------------------------------------------------------------------ v2: 29-bit limbs
constexpr int L29 = 14;
constexpr uint32_t M29 = (1u << 29) - 1;
constexpr uint32_t P29[L29] = {0x1fffaaabu, 0x0ff7ffffu, 0x14ffffeeu, 0x17fffd62u, 0x0f6241eau, 0x09507b58u, 0x0afd9cc3u,
                               0x109e70a2u, 0x1764774bu, 0x121a5d66u, 0x12c6e9edu, 0x12ffcd34u, 0x00111ea3u, 0x0000000du};
constexpr uint32_t R2_29[L29] = {0x15bef7aeu, 0x1031cd0eu, 0x02dd93e8u, 0x09226323u, 0x0e6e2cd2u,
                                 0x11684daau, 0x1170e5dbu, 0x088e25b1u, 0x1b366399u, 0x1c536f47u,
                                 0x0d1f9cbcu, 0x0278b67fu, 0x1ea66a2bu, 0x0000000cu};
constexpr uint32_t INV29 = 0x1ffcfffdu;
struct fq29 {
    uint32_t v[L29];
};
// result < 2p for inputs < 2p (R = 2^406 >> 4p): no final subtraction
__device__ __forceinline__ fq29 mul_v2(const fq29 &a, const fq29 &b) {
    uint32_t m[L29];
    fq29 r;
    uint64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L29; k++) {
        MI_UNROLL for (int i = 0; i < k; i++) {
            acc += (uint64_t)a.v[i] * b.v[k - i];
            acc += (uint64_t)m[i] * P29[k - i];
        }
        acc += (uint64_t)a.v[k] * b.v[0];
        m[k] = ((uint32_t)acc * INV29) & M29;
        acc += (uint64_t)m[k] * P29[0];
        acc >>= 29;
    }
    MI_UNROLL for (int k = L29; k < 2 * L29 - 1; k++) {
        MI_UNROLL for (int i = k - L29 + 1; i < L29; i++) {
            acc += (uint64_t)a.v[i] * b.v[k - i];
            acc += (uint64_t)m[i] * P29[k - i];
        }
        r.v[k - L29] = (uint32_t)acc & M29;
        acc >>= 29;
    }
    r.v[L29 - 1] = (uint32_t)acc;
    return r;
}
__device__ fq29 to29(const fq32_t &raw) {  // 12x32 -> 14x29 (raw integer)
    fq29 r;
    MI_UNROLL for (int i = 0; i < L29; i++) {
        int bit = 29 * i, w = bit >> 5, s = bit & 31;
        uint64_t x = raw.v[w];
        if (w + 1 < 12) x |= (uint64_t)raw.v[w + 1] << 32;
        r.v[i] = (uint32_t)(x >> s) & M29;
    }
    return r;
}
__device__ fq32_t from29(const fq29 &a) {  // 14x29 -> 12x32 (assumes normalized, < 2^384)
    fq32_t r = fq32_t::zero();
    MI_UNROLL for (int i = 0; i < L29; i++) {
        int bit = 29 * i, w = bit >> 5, s = bit & 31;
        r.v[w] |= a.v[i] << s;
        if (s > 3 && w + 1 < 12) r.v[w + 1] |= a.v[i] >> (32 - s);
    }
    return r;
}

// ------------------------------------------------------------------------------ v3: 13 x 30-bit balanced
// Signed limbs in [-2^29, 2^29): every limb product is at most 2^58 in magnitude, so a column of 13 a*b plus
// 13 m*p products (plus a carry) stays inside a signed 64-bit accumulator (26 * 2^58 = 2^62.7) -- one
// v_mad_i64_i32 per limb product, 338 per multiplication instead of 392 over 14 x 29-bit limbs.
constexpr int L30 = 13;
constexpr int32_t P30[L30] = {-21845, -402915328, 356515836, -352321620, -252304353, 55215067, 288093811,
                              316751073, -321428361, 517541167, -375082566, -91332614, 1704210};
constexpr int32_t R2_30[L30] = {84936463, -82245875, 20063291, -375672600, -184045713, -75371400, -508475920,
                                172522421, -150322876, 98350284, 415856896, -132992156, 1010031};
constexpr uint32_t INV30 = 0x3ffcfffdu;  // -p^-1 mod 2^30
struct fqs {
    int32_t v[L30];
};
__device__ __forceinline__ int32_t sext30(uint32_t x) { return ((int32_t)(x << 2)) >> 2; }
__device__ __forceinline__ fqs mul_v3(const fqs &a, const fqs &b) {
    int32_t m[L30];
    fqs r;
    int64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L30; k++) {
        MI_UNROLL for (int i = 0; i < k; i++) {
            acc += (int64_t)a.v[i] * b.v[k - i];
            acc += (int64_t)m[i] * P30[k - i];
        }
        acc += (int64_t)a.v[k] * b.v[0];
        m[k] = sext30((uint32_t)acc * INV30);
        acc += (int64_t)m[k] * P30[0];
        acc >>= 30;
    }
    MI_UNROLL for (int k = L30; k < 2 * L30 - 1; k++) {
        MI_UNROLL for (int i = k - L30 + 1; i < L30; i++) {
            acc += (int64_t)a.v[i] * b.v[k - i];
            acc += (int64_t)m[i] * P30[k - i];
        }
        r.v[k - L30] = sext30((uint32_t)acc);
        acc = (acc + (1 << 29)) >> 30;  // == (acc - sext30(acc)) >> 30
    }
    r.v[L30 - 1] = (int32_t)acc;
    return r;
}
__device__ fqs to30(const fq32_t &raw) {  // 12x32 canonical -> balanced 13x30
    fqs r;
    int32_t c = 0;
    MI_UNROLL for (int i = 0; i < L30; i++) {
        int bit = 30 * i, w = bit >> 5, s = bit & 31;
        uint64_t x = raw.v[w];
        if (w + 1 < 12) x |= (uint64_t)raw.v[w + 1] << 32;
        int32_t d = (int32_t)((uint32_t)(x >> s) & ((1u << 30) - 1)) + c;
        if (i < L30 - 1) {
            c = d >= (1 << 29) ? 1 : 0;
            d -= c << 30;
        }
        r.v[i] = d;
    }
    return r;
}
__device__ fq32_t from30(const fqs &a0) {  // balanced, |value| < p -> canonical 12x32
    fqs a = a0;
    int top = 0;
    for (int i = L30 - 1; i >= 0; i--)
        if (a.v[i] != 0) { top = a.v[i] < 0 ? -1 : 1; break; }
    if (top < 0)
        for (int i = 0; i < L30; i++) a.v[i] += P30[i];
    uint32_t u[L30];
    int64_t c = 0;
    for (int i = 0; i < L30; i++) {
        int64_t t = (int64_t)a.v[i] + c;
        u[i] = (uint32_t)(t & ((1 << 30) - 1));
        c = t >> 30;
    }
    fq32_t r = fq32_t::zero();
    for (int i = 0; i < L30; i++) {
        int bit = 30 * i, w = bit >> 5, s = bit & 31;
        r.v[w] |= u[i] << s;
        if (s > 2 && w + 1 < 12) r.v[w + 1] |= u[i] >> (32 - s);
    }
    return r;
}
// ------------------------------------------------------------------------------ v4: v3 + one Karatsuba level
// the 169-MAD schoolbook product of v3 as three sub-products over a = a0 + 2^210 a1 (7 + 6 limbs):
// z0 = a0 b0 (49 MADs), z2 = a1 b1 (36), z1 = (a0 + a1)(b0 + b1) (49; signed limb sums below 2^30, so a column of 7
// products stays below 2^62.8), then column c of the product is z0[c] + (z1 - z0 - z2)[c - 7] + z2[c - 14] (64-bit
// two's complement: the intermediate differences may wrap, the column values are the schoolbook ones, < 2^62).  134
// product MADs instead of 169, paid for with 13 limb sums, 26 64-bit column subtractions and 13 64-bit additions,
// and 25 64-bit column registers live into the reduction.  The Montgomery reduction is v3's (169 MADs).
constexpr int KL = 7, KH = L30 - KL;  // 7 low limbs, 6 high
__device__ __forceinline__ fqs mul_v4(const fqs &a, const fqs &b) {
    int32_t sa[KL], sb[KL];
    MI_UNROLL for (int i = 0; i < KL; i++) {
        sa[i] = a.v[i] + (i < KH ? a.v[KL + i] : 0);
        sb[i] = b.v[i] + (i < KH ? b.v[KL + i] : 0);
    }
    int64_t col[2 * L30 - 1];
    MI_UNROLL for (int k = 0; k < 2 * L30 - 1; k++) col[k] = 0;
    // z0 -> col[0..12], z2 -> col[14..24]; mid = z1 - z0 - z2 added at 7..19
    MI_UNROLL for (int k = 0; k < 2 * KL - 1; k++) {
        int64_t z0 = 0, z1 = 0, z2 = 0;
        MI_UNROLL for (int i = 0; i < KL; i++) {
            const int j = k - i;
            if (j < 0 || j >= KL) continue;
            z0 += (int64_t)a.v[i] * b.v[j];
            z1 += (int64_t)sa[i] * sb[j];
            if (i < KH && j < KH) z2 += (int64_t)a.v[KL + i] * b.v[KL + j];
        }
        col[k] += z0;
        col[k + KL] += z1 - z0 - z2;
        if (k < 2 * KH - 1) col[k + 2 * KL] += z2;
    }
    int32_t m[L30];
    fqs r;
    int64_t acc = 0;
    MI_UNROLL for (int k = 0; k < L30; k++) {
        acc += col[k];
        MI_UNROLL for (int i = 0; i < k; i++) acc += (int64_t)m[i] * P30[k - i];
        m[k] = sext30((uint32_t)acc * INV30);
        acc += (int64_t)m[k] * P30[0];
        acc >>= 30;
    }
    MI_UNROLL for (int k = L30; k < 2 * L30 - 1; k++) {
        acc += col[k];
        MI_UNROLL for (int i = k - L30 + 1; i < L30; i++) acc += (int64_t)m[i] * P30[k - i];
        r.v[k - L30] = sext30((uint32_t)acc);
        acc = (acc + (1 << 29)) >> 30;
    }
    r.v[L30 - 1] = (int32_t)acc;
    return r;
}
__global__ void __launch_bounds__(256) k_v4(fqs *d, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    fqs x = d[i], y = d[i ^ 1];
    for (int it = 0; it < iters; it++) x = mul_v4(x, y);
    d[i] = x;
}

__global__ void __launch_bounds__(256) k_v3(fqs *d, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    fqs x = d[i], y = d[i ^ 1];
    for (int it = 0; it < iters; it++) x = mul_v3(x, y);
    d[i] = x;
}
__global__ void k_check3(const fq32_t *xs, const fq32_t *ys, int n, int *bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fq32_t x = xs[i], y = ys[i];
    fq32_t ref = from_mont(to_mont(x) * to_mont(y));
    fqs R2v, one = {};
    MI_UNROLL for (int k = 0; k < L30; k++) R2v.v[k] = R2_30[k];
    one.v[0] = 1;
    fqs a = mul_v3(to30(x), R2v), b = mul_v3(to30(y), R2v);
    fq32_t v3 = from30(mul_v3(mul_v3(a, b), one));
    if (!(v3 == ref)) atomicAdd(bad + 2, 1);
    fqs a4 = mul_v4(to30(x), R2v), b4 = mul_v4(to30(y), R2v);
    fq32_t v4 = from30(mul_v4(mul_v4(a4, b4), one));
    if (!(v4 == ref)) atomicAdd(bad + 3, 1);
}

// ------------------------------------------------------------------------------ throughput kernels
__global__ void __launch_bounds__(256) k_v0(fq32_t *d, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    fq32_t x = d[i], y = d[i ^ 1];
    for (int it = 0; it < iters; it++) x = x * y;
    d[i] = x;
}
__global__ void __launch_bounds__(256) k_v1(fq32_t *d, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    fq32_t x = d[i], y = d[i ^ 1];
    for (int it = 0; it < iters; it++) x = mul_v1(x, y);
    d[i] = x;
}
__global__ void __launch_bounds__(256) k_v2(fq29 *d, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    fq29 x = d[i], y = d[i ^ 1];
    for (int it = 0; it < iters; it++) x = mul_v2(x, y);
    d[i] = x;
}

// correctness: x*y for random canonical x, y through each variant, compared canonically
__global__ void k_check(const fq32_t *xs, const fq32_t *ys, int n, int *bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fq32_t x = xs[i], y = ys[i];
    fq32_t ref = from_mont(to_mont(x) * to_mont(y));
    fq32_t r2;
    MI_UNROLL for (int k = 0; k < 12; k++) r2.v[k] = FqDesc::R2[k];
    fq32_t one = fq32_t::zero();
    one.v[0] = 1;
    fq32_t v1 = mul_v1(mul_v1(mul_v1(x, r2), mul_v1(y, r2)), one);
    fq29 R2v, one29 = {};
    MI_UNROLL for (int k = 0; k < L29; k++) R2v.v[k] = R2_29[k];
    one29.v[0] = 1;
    fq29 a = mul_v2(to29(x), R2v), b = mul_v2(to29(y), R2v);
    fq29 c = mul_v2(mul_v2(a, b), one29);
    fq32_t v2 = reduce_once(from29(c));
    if (!(v1 == ref)) atomicAdd(bad, 1);
    if (!(v2 == ref)) atomicAdd(bad + 1, 1);
}

template <class K, class... A>
float timeit(K k, dim3 g, dim3 b, A... args) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, g, b, 0, 0, args...);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, g, b, 0, 0, args...);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
}

int main() {
    const int threads = 256, blocks = 256 * 16;  // 16 blocks per CU
    const size_t nt = (size_t)threads * blocks;
    uint32_t *o;
    CHECK(hipMalloc(&o, nt * 4));
    int it = 2000;
    float ms = timeit(k_raw_mad, dim3(blocks), dim3(threads), o, it);
    double ops = (double)nt * it * 8;
    printf("raw v_mad_u64_u32 : %.1f G lane-ops/s  (%.2f cycles/wave-instr/SIMD @2.4GHz)\n", ops / ms / 1e6,
           (1024.0 * 2.4e9 / (ops / ms * 1e3)) * 64);
    ms = timeit(k_raw_add, dim3(blocks), dim3(threads), o, it);
    printf("raw v_add_u32     : %.1f G lane-ops/s  (%.2f cycles/wave-instr/SIMD)\n", ops / ms / 1e6,
           (1024.0 * 2.4e9 / (ops / ms * 1e3)) * 64);
    ms = timeit(k_raw_mullo, dim3(blocks), dim3(threads), o, it);
    printf("raw v_mul_lo_u32  : %.1f G lane-ops/s  (%.2f cycles/wave-instr/SIMD)\n", ops / ms / 1e6,
           (1024.0 * 2.4e9 / (ops / ms * 1e3)) * 64);

    // correctness
    const int nc = 1 << 16;
    fq32_t *hx = (fq32_t *)malloc(sizeof(fq32_t) * nc * 2);
    srand(1);
    for (int i = 0; i < 2 * nc; i++) {
        for (int k = 0; k < 12; k++) hx[i].v[k] = ((uint32_t)rand() << 16) ^ (uint32_t)rand();
        hx[i].v[11] &= 0x0fffffffu;  // < p
    }
    // edge values: 0, 1, p-1
    for (int k = 0; k < 12; k++) {
        hx[0].v[k] = 0;
        hx[1].v[k] = FqDesc::MOD[k];
        hx[nc].v[k] = FqDesc::MOD[k];
    }
    hx[1].v[0] -= 1;
    hx[nc].v[0] -= 1;
    fq32_t *dx;
    int *bad;
    CHECK(hipMalloc(&dx, sizeof(fq32_t) * nc * 2));
    CHECK(hipMalloc(&bad, 16));
    CHECK(hipMemset(bad, 0, 16));
    CHECK(hipMemcpy(dx, hx, sizeof(fq32_t) * nc * 2, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_check, dim3(nc / 256), dim3(256), 0, 0, dx, dx + nc, nc, bad);
    hipLaunchKernelGGL(k_check3, dim3(nc / 256), dim3(256), 0, 0, dx, dx + nc, nc, bad);
    int hb[4];
    CHECK(hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost));
    printf("correctness vs v0 over %d random products: v1 mismatches %d, v2 mismatches %d, v3 mismatches %d, "
           "v4 mismatches %d\n", nc, hb[0], hb[1], hb[2], hb[3]);

    // throughput
    it = 200;
    fq32_t *d0;
    CHECK(hipMalloc(&d0, sizeof(fq32_t) * nt));
    CHECK(hipMemset(d0, 1, sizeof(fq32_t) * nt));
    double muls = (double)nt * it;
    ms = timeit(k_v0, dim3(blocks), dim3(threads), d0, it);
    printf("v0 CIOS (compiler)     : %.2f G Fq-mul/s\n", muls / ms / 1e6);
    ms = timeit(k_v1, dim3(blocks), dim3(threads), d0, it);
    printf("v1 FIPS 32-bit + vcc   : %.2f G Fq-mul/s\n", muls / ms / 1e6);
    fq29 *d2;
    CHECK(hipMalloc(&d2, sizeof(fq29) * nt));
    CHECK(hipMemset(d2, 1, sizeof(fq29) * nt));
    ms = timeit(k_v2, dim3(blocks), dim3(threads), d2, it);
    printf("v2 FIPS 29-bit limbs   : %.2f G Fq-mul/s\n", muls / ms / 1e6);
    fqs *d3;
    CHECK(hipMalloc(&d3, sizeof(fqs) * nt));
    CHECK(hipMemset(d3, 1, sizeof(fqs) * nt));
    for (int rep = 0; rep < 3; rep++) {
        ms = timeit(k_v2, dim3(blocks), dim3(threads), d2, it);
        printf("v2 FIPS 29-bit limbs   : %.2f G Fq-mul/s\n", muls / ms / 1e6);
        ms = timeit(k_v3, dim3(blocks), dim3(threads), d3, it);
        printf("v3 13x30 balanced      : %.2f G Fq-mul/s\n", muls / ms / 1e6);
        ms = timeit(k_v4, dim3(blocks), dim3(threads), d3, it);
        printf("v4 13x30 + Karatsuba   : %.2f G Fq-mul/s\n", muls / ms / 1e6);
    }
    return 0;
}
