// sortbench.hip -- bucket grouping of MSM digit entries: rocPRIM onesweep (the round-5 plan) against counting sorts
// whose blocks never wait on each other (histogram by atomics, scan, scatter by atomic cursors).
//
// One window of a split 2^26 plan: n = 2^28 entries, keys in [0, 2^21), vals = entry index.  Distributions:
// uniform keys, and "hot" ones where a fraction of the keys is 0 (a boolean witness puts half its digits into bucket
// 0 of window 0).  Each variant is timed with HIP events (median of 5) and checked: the output must be grouped by key
// with every value present once.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 sortbench.hip -o sortbench && ./sortbench [log_n]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <vector>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

constexpr unsigned KBITS = 21;
constexpr uint32_t NB = 1u << KBITS;

__global__ void k_gen(uint32_t *keys, uint32_t *vals, uint32_t n, uint32_t hot_per_1024, uint64_t seed) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = seed + i * 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    const bool hot = (uint32_t)(x >> 40) % 1024 < hot_per_1024;
    keys[i] = hot ? 0u : (uint32_t)x & (NB - 1);
    vals[i] = i;
}

// ---- counting sort, plain atomics ----
__global__ void k_hist(const uint32_t *__restrict__ keys, uint32_t n, uint32_t *__restrict__ cnt) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&cnt[keys[i]], 1u);
}
__global__ void k_scatter(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals, uint32_t n,
                          uint32_t *__restrict__ cur, uint32_t *__restrict__ out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[atomicAdd(&cur[keys[i]], 1u)] = vals[i];
}

// ---- wave-aggregated: the lanes sharing the wave's first key take one atomic together, the rest their own ----
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__global__ void k_hist_agg(const uint32_t *__restrict__ keys, uint32_t n, uint32_t *__restrict__ cnt) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < n;
    const uint32_t k = live ? keys[i] : 0xffffffffu;
    const uint32_t k0 = __shfl(k, 0);
    const uint64_t m = __ballot(live && k == k0);
    if (live && k == k0) {
        if (lane_id() == (uint32_t)(__ffsll((long long)m) - 1)) atomicAdd(&cnt[k0], (uint32_t)__popcll(m));
    } else if (live) {
        atomicAdd(&cnt[k], 1u);
    }
}
__global__ void k_scatter_agg(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals, uint32_t n,
                              uint32_t *__restrict__ cur, uint32_t *__restrict__ out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < n;
    const uint32_t k = live ? keys[i] : 0xffffffffu;
    const uint32_t k0 = __shfl(k, 0);
    const uint64_t m = __ballot(live && k == k0);
    const uint32_t leader = (uint32_t)(__ffsll((long long)m) - 1);
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(&cur[k0], (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (!live) return;
    uint32_t pos;
    if (k == k0) pos = base + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1));
    else pos = atomicAdd(&cur[k], 1u);
    out[pos] = vals[i];
}

// ---- MSD by the high bits with block-local ranking (no atomics on global counters for the first level) ----
// pass 1: per-block histogram of the high H bits (LDS), written [bin][block]; scan; scatter by LDS-ranked
// position.  pass 2 (per coarse bin, one block each): fine histogram + LDS cursor scatter inside the bin.
constexpr unsigned HB = 10, LB = KBITS - HB;  // 1024 coarse bins, 2048 fine buckets per bin
constexpr unsigned T1 = 256, IPT1 = 16, TILE1 = T1 * IPT1;
__global__ void __launch_bounds__(T1) k_msd_up(const uint32_t *__restrict__ keys, uint32_t n,
                                               uint32_t *__restrict__ bh, uint32_t nblk) {
    __shared__ uint32_t h[1u << HB];
    for (uint32_t j = threadIdx.x; j < (1u << HB); j += T1) h[j] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * TILE1;
    for (uint32_t j = 0; j < IPT1; j++) {
        const uint32_t i = base + j * T1 + threadIdx.x;
        if (i < n) atomicAdd(&h[keys[i] >> LB], 1u);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < (1u << HB); j += T1) bh[(uint64_t)j * nblk + blockIdx.x] = h[j];
}
__global__ void __launch_bounds__(T1) k_msd_down(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                 uint32_t n, const uint32_t *__restrict__ boff, uint32_t nblk,
                                                 uint2 *__restrict__ out) {
    __shared__ uint32_t cur[1u << HB];
    for (uint32_t j = threadIdx.x; j < (1u << HB); j += T1) cur[j] = boff[(uint64_t)j * nblk + blockIdx.x];
    __syncthreads();
    const uint32_t base = blockIdx.x * TILE1;
    for (uint32_t j = 0; j < IPT1; j++) {
        const uint32_t i = base + j * T1 + threadIdx.x;
        if (i < n) {
            const uint32_t k = keys[i];
            const uint32_t p = atomicAdd(&cur[k >> LB], 1u);  // LDS atomic: order inside a bin is arbitrary
            out[p] = make_uint2(k & ((1u << LB) - 1), vals[i]);
        }
    }
}
// pass 2: bin b holds [off[b], off[b + 1]); fine histogram in LDS, scan, LDS cursors, scatter vals; bucket starts
constexpr unsigned T2 = 1024;
__global__ void __launch_bounds__(T2) k_msd_fine(const uint2 *__restrict__ in, const uint32_t *__restrict__ binoff,
                                                 uint32_t *__restrict__ out, uint32_t *__restrict__ bstart) {
    __shared__ uint32_t h[1u << LB];
    __shared__ uint32_t wsum[T2 / 64];
    const uint32_t b = blockIdx.x, lo = binoff[b], hi = binoff[b + 1];
    for (uint32_t j = threadIdx.x; j < (1u << LB); j += T2) h[j] = 0;
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += T2) atomicAdd(&h[in[i].x], 1u);
    __syncthreads();
    // exclusive scan of 2048 counters by 1024 threads: two per thread
    const uint32_t t = threadIdx.x;
    const uint32_t a0 = h[2 * t], a1 = h[2 * t + 1];
    uint32_t s = a0 + a1, incl = s;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if ((t & 63) >= (unsigned)o) incl += y;
    }
    if ((t & 63) == 63) wsum[t >> 6] = incl;
    __syncthreads();
    uint32_t wb = 0;
    for (uint32_t w = 0; w < (t >> 6); w++) wb += wsum[w];
    const uint32_t ex = lo + wb + incl - s;
    __syncthreads();
    h[2 * t] = ex;
    h[2 * t + 1] = ex + a0;
    bstart[(uint64_t)b * (1u << LB) + 2 * t] = ex;
    bstart[(uint64_t)b * (1u << LB) + 2 * t + 1] = ex + a0;
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += T2) {
        const uint2 e = in[i];
        out[atomicAdd(&h[e.x], 1u)] = e.y;
    }
}

// ---- check: grouped by key, every value once ----
static bool check_grouped(const std::vector<uint32_t> &keys_in, const std::vector<uint32_t> &out, uint32_t n) {
    std::vector<uint32_t> cnt(NB + 1, 0), off(NB + 1, 0);
    for (uint32_t i = 0; i < n; i++) cnt[keys_in[i]]++;
    for (uint32_t b = 0; b < NB; b++) off[b + 1] = off[b] + cnt[b];
    std::vector<uint8_t> seen(n, 0);
    for (uint32_t b = 0; b < NB; b++)
        for (uint32_t p = off[b]; p < off[b + 1]; p++) {
            const uint32_t v = out[p];
            if (v >= n || seen[v] || keys_in[v] != b) return false;
            seen[v] = 1;
        }
    return true;
}

int main(int argc, char **argv) {
    const unsigned lg = argc > 1 ? atoi(argv[1]) : 28;
    const uint32_t n = 1u << lg;
    uint32_t *keys, *vals, *keys_s, *vals_s, *cnt, *cur, *bh, *boff, *binoff, *bstart;
    uint2 *mid;
    CK(hipMalloc(&keys, 4ull * n));
    CK(hipMalloc(&vals, 4ull * n));
    CK(hipMalloc(&keys_s, 4ull * n));
    CK(hipMalloc(&vals_s, 4ull * n));
    CK(hipMalloc(&mid, 8ull * n));
    CK(hipMalloc(&cnt, 4ull * (NB + 1)));
    CK(hipMalloc(&cur, 4ull * (NB + 1)));
    const uint32_t nblk1 = (n + TILE1 - 1) / TILE1;
    CK(hipMalloc(&bh, 4ull * nblk1 * (1u << HB) + 4));
    CK(hipMalloc(&boff, 4ull * nblk1 * (1u << HB) + 4));
    CK(hipMalloc(&binoff, 4ull * ((1u << HB) + 1)));
    CK(hipMalloc(&bstart, 4ull * NB));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    using cfg = rocprim::radix_sort_config<
        rocprim::default_config, rocprim::default_config,
        rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 24>, rocprim::kernel_config<1024, 24>, 11,
                                            rocprim::block_radix_rank_algorithm::match>,
        0>;
    size_t sort_bytes = 0, scan_bytes = 0;
    CK(rocprim::radix_sort_pairs<cfg>(nullptr, sort_bytes, keys, keys_s, vals, vals_s, n, 0, KBITS));
    CK(rocprim::exclusive_scan(nullptr, scan_bytes, cnt, cur, 0u, (size_t)NB, rocprim::plus<uint32_t>()));
    size_t scan2_bytes = 0;
    CK(rocprim::exclusive_scan(nullptr, scan2_bytes, bh, boff, 0u, (size_t)nblk1 << HB, rocprim::plus<uint32_t>()));
    void *tmp;
    CK(hipMalloc(&tmp, std::max(sort_bytes, std::max(scan_bytes, scan2_bytes))));
    const unsigned G = (n + 255) / 256;

    for (uint32_t hot : {0u, 512u, 900u}) {
        k_gen<<<G, 256>>>(keys, vals, n, hot, 12345 + hot);
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> hk(n), hout(n);
        CK(hipMemcpy(hk.data(), keys, 4ull * n, hipMemcpyDeviceToHost));
        auto timeit = [&](const char *name, auto &&body, uint32_t *result) {
            std::vector<float> ts;
            for (int r = 0; r < 6; r++) {
                CK(hipEventRecord(e0));
                body();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            CK(hipMemcpy(hout.data(), result, 4ull * n, hipMemcpyDeviceToHost));
            const bool ok = check_grouped(hk, hout, n);
            printf("{\"n\": %u, \"hot_per_1024\": %u, \"variant\": \"%s\", \"ms\": %.3f, \"Gentries_s\": %.2f, \"ok\": %s}\n",
                   n, hot, name, ts[ts.size() / 2], n / (ts[ts.size() / 2] * 1e6), ok ? "true" : "false");
            fflush(stdout);
        };
        timeit("onesweep_pairs_2x11", [&] {
            size_t b = sort_bytes;
            CK(rocprim::radix_sort_pairs<cfg>(tmp, b, keys, keys_s, vals, vals_s, n, 0, KBITS));
        }, vals_s);
        timeit("count_atomic", [&] {
            CK(hipMemsetAsync(cnt, 0, 4ull * NB));
            k_hist<<<G, 256>>>(keys, n, cnt);
            size_t b = scan_bytes;
            CK(rocprim::exclusive_scan(tmp, b, cnt, cur, 0u, (size_t)NB, rocprim::plus<uint32_t>()));
            k_scatter<<<G, 256>>>(keys, vals, n, cur, vals_s);
        }, vals_s);
        timeit("count_atomic_wave_agg", [&] {
            CK(hipMemsetAsync(cnt, 0, 4ull * NB));
            k_hist_agg<<<G, 256>>>(keys, n, cnt);
            size_t b = scan_bytes;
            CK(rocprim::exclusive_scan(tmp, b, cnt, cur, 0u, (size_t)NB, rocprim::plus<uint32_t>()));
            k_scatter_agg<<<G, 256>>>(keys, vals, n, cur, vals_s);
        }, vals_s);
        if (hot) continue;  // msd_10_11 runs a coarse bin in one block: bin 0 of a hot distribution is half the input
        timeit("msd_10_11", [&] {
            k_msd_up<<<nblk1, T1>>>(keys, n, bh, nblk1);
            size_t b = scan2_bytes;
            CK(rocprim::exclusive_scan(tmp, b, bh, boff, 0u, (size_t)nblk1 << HB, rocprim::plus<uint32_t>()));
            k_msd_down<<<nblk1, T1>>>(keys, vals, n, boff, nblk1, mid);
            // bin offsets = boff[bin * nblk1] (+ n at the end): gathered on the device by a tiny kernel-free copy
            CK(hipMemcpy2DAsync(binoff, 4, boff, 4ull * nblk1, 4, 1u << HB, hipMemcpyDeviceToDevice));
            CK(hipMemcpyAsync(binoff + (1u << HB), &n, 4, hipMemcpyHostToDevice));
            k_msd_fine<<<1u << HB, T2>>>(mid, binoff, vals_s, bstart);
        }, vals_s);
    }
    return 0;
}
