// msm_impl.h -- Pippenger multi-scalar multiplication on BLS12-381 G1 / G2 for CDNA4 (gfx950).
//
// Restates crypto3's multiexp ([NOT IN TREE]: libs/crypto/algebra, used by r1cs_gg_ppzksnark's
// prover for the H, L, A, B_G1 (G1) and B_G2 (G2) queries -- SURVEY.md §8a rows a7/a8).
//
// Pipeline (one MSM):
//   1. k_digits     : every scalar -> ceil(256/c) signed c-bit digits; one (bucket key, point
//                     index | sign) pair per non-zero digit, laid out [window][point] (coalesced).
//   2. radix sort   : rocPRIM onesweep per window over the c window-local key bits.
//   3. k_bounds4    : bucket start / end (and the zero-digit tail of each window) from the sorted keys.
//   4. accumulation : buckets are cut into chunks of <= L sorted entries, one thread per chunk,
//                     chunks length-sorted (6-7 bit radix sort) so a wave runs equal-length chunks
//                     (mixed XYZZ += affine adds, point gathered by index); the chunk partials
//                     of buckets with several chunks are summed in place by a strided tree
//                     (only those buckets take part).  Work per thread is bounded by L whatever
//                     the scalar distribution (boolean-heavy Filecoin witnesses put most entries
//                     in bucket 1 of window 0).
//   5. k_bucket_reduce: running-sum reduction sum_b (b+1) B_b over ~2^20 (G1) / 2^18 (G2) segments,
//      then a second running-sum level over the segment sums (k_bucket_reduce_dense), whose <= 8192
//      segments per window are offset by a short double-and-add (k_seg_fold).
//   6. k_sum_groups : stacked per-window tree sums; host combines W = sum acc + S (V - R).
//   7. host         : Horner over windows (c doublings each) on the CPU, in the 64-bit host field (hostfield.h).
// A plan reads its counts back ONCE (plan_counts / plan_finish: chunk totals, the multi-chunk bucket list and every
// chunk-tree level's size), then the result once.
// Window-table plans (msm_run_wt; a small key's queries, mi_points_precompute): the table holds 2^(c w) P_i for
// every window w, so k_digits_wt / k_digits_wt_c (witness scalars: non-zero digits compacted) put every window's
// digits into ONE bucket set; the one window is reduced by bit rows (reduce_bitsum: k_bitsum_first, k_sum_lds)
// and there is no window combination.
#pragma once
#include <hipcub/hipcub.hpp>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include "ctx.h"
#include "g2pair.h"
#include "glv.h"
#include "hostfield.h"

namespace mi {

namespace {

// At least two waves per SIMD for the G2 group-law kernels: without it the Fq2 instances take all 512
// unified registers (256 VGPR + 256 AGPR) and run one wave per SIMD.  msm_g1.hip defines it empty
// before including this header: the G1 instances pick 96-180 VGPRs on their own, and the cap made
// the compiler spill two of the G1 reduction kernels.
#ifndef MI_WAVES2
#define MI_WAVES2 __attribute__((amdgpu_waves_per_eu(2)))
#endif
#ifndef MI_ACC_PREFETCH
#define MI_ACC_PREFETCH 0
#endif
#ifndef MI_WAVES_ACC
#define MI_WAVES_ACC MI_WAVES2
#endif
#ifndef MI_WAVES_RED
#define MI_WAVES_RED MI_WAVES2  // the reduction kernels keep the two-wave cap (see g2pair.h LaneRed)
#endif

// sorted entries per chunk at level 0 (mixed adds); tune::MSM_L0 overrides.  Plans of >= 2^24 points per window take
// L0_LARGE: round 6, same box, alternating, 128 against 64 took the 32 GiB Window-PoSt partition (128 entries per
// bucket on average) from 1,514.9 to 1,483.7 ms and the config-3 proof (64 per bucket) from 469.5 to 468.4 ms (fewer
// chunk-tree additions).  Smaller, latency-bound plans keep the shorter chains.
constexpr uint32_t L0_DEFAULT = 64, L0_LARGE = 128;
constexpr uint32_t L1_DEFAULT = 16;  // chunk partials summed per thread per tree level (full adds); tune::MSM_L1 overrides
constexpr unsigned TREE_MAXL = 16;   // chunk-tree levels counted with the plan (L1 >= 4: up to 4^16 chunks a bucket)

MI_HD uint32_t word_of(const fr_t &s, unsigned k) {
    uint32_t r = 0;
    MI_UNROLL for (int j = 0; j < 8; j++) r = (k == (unsigned)j) ? s.v[j] : r;
    return r;
}

__global__ void k_digits(const fr_t *__restrict__ scalars, const uint32_t *__restrict__ idx, uint32_t n,
                         unsigned c, unsigned nwin, uint32_t invalid, uint32_t wk, uint32_t *__restrict__ keys,
                         uint32_t *__restrict__ vals) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fr_t s = scalars[idx ? idx[i] : i];
    const uint32_t nbk = 1u << (c - 1);
    const uint32_t mask = (1u << c) - 1;
    uint32_t carry = 0;
    for (unsigned w = 0; w < nwin; w++) {
        unsigned bit = w * c, word = bit >> 5, sh = bit & 31;
        uint32_t d = 0;
        if (word < 8) {
            d = word_of(s, word) >> sh;
            if (sh + c > 32 && word + 1 < 8) d |= word_of(s, word + 1) << (32 - sh);
        }
        d = (d & mask) + carry;
        uint32_t neg = 0;
        if (d > nbk) {
            d = (1u << c) - d;
            neg = 1;
            carry = 1;
        } else {
            carry = 0;
        }
        uint64_t o = (uint64_t)w * n + i;
        // bucket within the window (+ w * wk when all windows are sorted in one call)
        keys[o] = (d ? d - 1 : invalid) + w * wk;
        vals[o] = i | (neg << 31);
    }
}

// Window-table plans (fixed-base precomputation, msm_run_wt): table point w * stride + i is 2^(c w) P_i, so the
// window-w digit of scalar i goes into the ONE bucket set of the plan as an entry over that point.  Entries are
// laid out [window][scalar] like k_digits'; zero digits take the key `invalid` and sort last.
__global__ void k_digits_wt(const fr_t *__restrict__ scalars, const uint32_t *__restrict__ idx, uint32_t n, unsigned c,
                            unsigned nwin, uint32_t stride, uint32_t invalid, uint32_t *__restrict__ keys,
                            uint32_t *__restrict__ vals) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fr_t s = scalars[idx ? idx[i] : i];
    const uint32_t nbk = 1u << (c - 1);
    const uint32_t mask = (1u << c) - 1;
    uint32_t carry = 0;
    for (unsigned w = 0; w < nwin; w++) {
        unsigned bit = w * c, word = bit >> 5, sh = bit & 31;
        uint32_t d = 0;
        if (word < 8) {
            d = word_of(s, word) >> sh;
            if (sh + c > 32 && word + 1 < 8) d |= word_of(s, word + 1) << (32 - sh);
        }
        d = (d & mask) + carry;
        uint32_t neg = 0;
        if (d > nbk) {
            d = (1u << c) - d;
            neg = 1;
            carry = 1;
        } else {
            carry = 0;
        }
        const uint64_t o = (uint64_t)w * n + i;
        keys[o] = d ? d - 1 : invalid;
        vals[o] = (w * stride + i) | (neg << 31);
    }
}

// The compacting digit kernels size their per-wave scratch as DIGITS_BLOCK / 64: gfx950 runs 64-wide waves
// only (this library builds for gfx950 alone), and every launch of them passes DIGITS_BLOCK as its block size.
constexpr unsigned DIGITS_BLOCK = 256;
static_assert(DIGITS_BLOCK % 64 == 0 && DIGITS_BLOCK <= 1024, "whole 64-wide waves per digit block");
// The same for sparse scalars (witness vectors: mostly 0 / 1, so most window digits are zero): only the non-zero
// digits are written, compacted at [0, *count) in arbitrary order (per-thread counts, a wave prefix sum and one
// atomic per wave).  The sort then runs over the entries alone.
__global__ void __launch_bounds__(DIGITS_BLOCK) k_digits_wt_c(const fr_t *__restrict__ scalars, const uint32_t *__restrict__ idx,
                                                     uint32_t n, unsigned c, unsigned nwin, uint32_t stride,
                                                     uint32_t *__restrict__ count, uint32_t *__restrict__ keys,
                                                     uint32_t *__restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned lane = threadIdx.x & 63;
    fr_t s = fr_t::zero();
    if (i < n) s = scalars[idx ? idx[i] : i];
    const uint32_t nbk = 1u << (c - 1), mask = (1u << c) - 1;
    // pass 1: this thread's non-zero digits
    uint32_t mine = 0, carry = 0;
    for (unsigned w = 0; w < nwin; w++) {
        const unsigned bit = w * c, word = bit >> 5, sh = bit & 31;
        uint32_t d = 0;
        if (word < 8) {
            d = word_of(s, word) >> sh;
            if (sh + c > 32 && word + 1 < 8) d |= word_of(s, word + 1) << (32 - sh);
        }
        d = (d & mask) + carry;
        if (d > nbk) d = (1u << c) - d, carry = 1;
        else carry = 0;
        mine += d != 0;
    }
    // exclusive prefix over the wave, then over the block's four waves: one atomic per block (the counter is shared
    // by every block of the launch, so per-wave atomics queued behind each other)
    __shared__ uint32_t wsum[DIGITS_BLOCK / 64], bbase;
    const unsigned wave = threadIdx.x >> 6;
    uint32_t incl = mine;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= (unsigned)o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (unsigned w = 0; w < DIGITS_BLOCK / 64; w++) t += wsum[w];
        bbase = t ? atomicAdd(count, t) : 0u;
    }
    __syncthreads();
    uint32_t base = bbase + incl - mine;
    for (unsigned w = 0; w < wave; w++) base += wsum[w];
    if (!mine) return;
    // pass 2: write them
    carry = 0;
    for (unsigned w = 0; w < nwin; w++) {
        const unsigned bit = w * c, word = bit >> 5, sh = bit & 31;
        uint32_t d = 0;
        if (word < 8) {
            d = word_of(s, word) >> sh;
            if (sh + c > 32 && word + 1 < 8) d |= word_of(s, word + 1) << (32 - sh);
        }
        d = (d & mask) + carry;
        uint32_t neg = 0;
        if (d > nbk) d = (1u << c) - d, neg = 1, carry = 1;
        else carry = 0;
        if (d) {
            keys[base] = d - 1;
            vals[base] = (w * stride + i) | (neg << 31);
            base++;
        }
    }
}

// Large MSMs: the same digits, but only the NON-ZERO ones are written, compacted per window at
// [w * n, w * n + wcount[w]) (wave ballots, one atomic per window per workgroup).  Witness scalars are
// boolean-heavy (0/1 and small values): 43 % of the L/A/B digit slots of the synthetic 2^26 circuit
// are zero, and none of them is sorted any more.  Order inside a window is arbitrary before the sort.
constexpr unsigned MAXW_C = 32;  // c >= 8
// Split mode (nreal != 0, n = 2 nreal): point i < nreal takes bits [0, 128) of scalar i, point
// nreal + i bits [128, 256) of the same scalar (its base is 2^128 times as large).
__global__ void __launch_bounds__(256) k_digits_c(const fr_t *__restrict__ scalars, const uint32_t *__restrict__ idx,
                                                  uint32_t n, unsigned c, unsigned nwin, uint32_t nreal,
                                                  uint32_t *__restrict__ wcount, uint32_t *__restrict__ keys,
                                                  uint32_t *__restrict__ vals) {
    __shared__ uint32_t wc[4][MAXW_C];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    fr_t s = fr_t::zero();
    if (i < n) {
        const bool hi = nreal && i >= nreal;
        const uint32_t src = hi ? i - nreal : i;
        s = scalars[idx ? idx[src] : src];
        if (nreal) {
            MI_UNROLL for (int j = 0; j < 4; j++) {
                s.v[j] = hi ? s.v[j + 4] : s.v[j];
                s.v[j + 4] = 0;
            }
        }
    }
    const uint32_t nbk = 1u << (c - 1);
    const uint32_t mask = (1u << c) - 1;
    uint32_t dg[MAXW_C];  // digit | neg << 31; 0 = zero digit
    uint32_t carry = 0;
    // every loop below is fully unrolled over MAXW_C with `if (w < nwin)` guards (no break/continue),
    // so dg[] and rank[] stay in registers (a data-dependent exit spilled them to scratch: 70x slower)
    MI_UNROLL for (unsigned w = 0; w < MAXW_C; w++) dg[w] = 0;
    MI_UNROLL for (unsigned w = 0; w < MAXW_C; w++) {
        if (w < nwin) {
        unsigned bit = w * c, word = bit >> 5, sh = bit & 31;
        uint32_t d = 0;
        if (word < 8) {
            d = word_of(s, word) >> sh;
            if (sh + c > 32 && word + 1 < 8) d |= word_of(s, word + 1) << (32 - sh);
        }
        d = (d & mask) + carry;
        uint32_t neg = 0;
        if (d > nbk) {
            d = (1u << c) - d;
            neg = 1;
            carry = 1;
        } else {
            carry = 0;
        }
        dg[w] = d ? d | (neg << 31) : 0;
        }
    }
    const uint64_t below = (1ull << lane) - 1;
    uint32_t rank[MAXW_C];
    MI_UNROLL for (unsigned w = 0; w < MAXW_C; w++) {
        rank[w] = 0;
        if (w < nwin) {
            uint64_t m = __ballot(dg[w] != 0);
            rank[w] = (uint32_t)__popcll(m & below);
            if (lane == 0) wc[wave][w] = (uint32_t)__popcll(m);
        }
    }
    __syncthreads();
    if (threadIdx.x < nwin) {
        const unsigned w = threadIdx.x;
        uint32_t c0 = wc[0][w], c1 = wc[1][w], c2 = wc[2][w], c3 = wc[3][w];
        uint32_t base = atomicAdd(&wcount[w], c0 + c1 + c2 + c3);
        wc[0][w] = base;
        wc[1][w] = base + c0;
        wc[2][w] = base + c0 + c1;
        wc[3][w] = base + c0 + c1 + c2;
    }
    __syncthreads();
    MI_UNROLL for (unsigned w = 0; w < MAXW_C; w++) {
        if (w < nwin && dg[w]) {
            uint64_t o = (uint64_t)w * n + wc[wave][w] + rank[w];
            keys[o] = (dg[w] & 0x7fffffffu) - 1;
            vals[o] = i | (dg[w] & 0x80000000u);
        }
    }
}

// Split plans: one thread per INPUT scalar writes the digits of both 128-bit halves -- point i (low half)
// and point nreal + i (high half, 2^128-shifted base) -- so the plan costs the same digit work as the
// plain 12-window one (a thread per half-scalar point measured +2.3 ms per 2^26 MSM).  c >= 9 keeps
// ceil(129 / c) <= MAXW_S windows.
constexpr unsigned MAXW_S = 16;
static_assert(MAXW_S == MSM_PLAN_MAXW, "MsmPlan::wn holds MAXW_S windows");
// Entry values (sorted with the keys) are point index | sign << 31; bit 30 is A_MARK in plans built for
// msm_derive_plan_impl, so every plan keeps its point indices below 2^30.
constexpr uint32_t A_MARK = 1u << 30, IDX_MASK = A_MARK - 1;
MI_HD uint32_t word4_of(const uint32_t *v, unsigned k) {
    uint32_t r = 0;
    MI_UNROLL for (int j = 0; j < 4; j++) r = (k == (unsigned)j) ? v[j] : r;
    return r;
}
// signed c-bit digits (| neg << 31, 0 = zero digit) of the 128-bit value v[0..3]
MI_HD void digits128(const uint32_t *v, unsigned c, unsigned nwin, uint32_t *dg) {
    const uint32_t nbk = 1u << (c - 1), mask = (1u << c) - 1;
    uint32_t carry = 0;
    MI_UNROLL for (unsigned w = 0; w < MAXW_S; w++) {
        dg[w] = 0;
        if (w < nwin) {
            unsigned bit = w * c, word = bit >> 5, sh = bit & 31;
            uint32_t d = 0;
            if (word < 4) {
                d = word4_of(v, word) >> sh;
                if (sh + c > 32 && word + 1 < 4) d |= word4_of(v, word + 1) << (32 - sh);
            }
            d = (d & mask) + carry;
            uint32_t neg = 0;
            if (d > nbk) {
                d = (1u << c) - d;
                neg = 1;
                carry = 1;
            } else {
                carry = 0;
            }
            dg[w] = d ? d | (neg << 31) : 0;
        }
    }
}
// GLV (glv.h): the halves are k1 = k mod lambda (over P_i) and k2 = k div lambda (over phi(P_i)), and the
// key carries the half as its low bit -- sub-bucket 2 (digit - 1) + half -- so the entries over P and over
// phi(P) of one bucket are accumulated apart and phi is applied once per bucket sum (k_glv_merge).
// amark (optional, Circuit::a_rank): entries of scalar i with amark[i] != ~0 carry A_MARK (msm_derive_plan_impl).
template <bool GLV>
__global__ void __launch_bounds__(256) k_digits_split(const fr_t *__restrict__ scalars,
                                                      const uint32_t *__restrict__ idx, uint32_t nreal, unsigned c,
                                                      unsigned nwin, uint32_t *__restrict__ wcount,
                                                      uint32_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                                      const uint32_t *__restrict__ amark) {
    __shared__ uint32_t wc[4][MAXW_S];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t n = 2ull * nreal;  // window stride of keys / vals
    fr_t s = fr_t::zero();
    uint32_t mark = 0;
    if (i < nreal) {
        s = scalars[idx ? idx[i] : i];
        if (amark && amark[i] != 0xffffffffu) mark = A_MARK;
    }
    uint32_t dlo[MAXW_S], dhi[MAXW_S];
    if constexpr (GLV) {
        uint32_t k1[4], k2[4];
        glv_split(s.v, k1, k2);
        digits128(k1, c, nwin, dlo);
        digits128(k2, c, nwin, dhi);
    } else {
        digits128(s.v, c, nwin, dlo);
        digits128(s.v + 4, c, nwin, dhi);
    }
    const uint64_t below = (1ull << lane) - 1;
    uint32_t rlo[MAXW_S], rhi[MAXW_S];
    MI_UNROLL for (unsigned w = 0; w < MAXW_S; w++) {
        rlo[w] = rhi[w] = 0;
        if (w < nwin) {
            uint64_t mlo = __ballot(dlo[w] != 0), mhi = __ballot(dhi[w] != 0);
            uint32_t clo = (uint32_t)__popcll(mlo);
            rlo[w] = (uint32_t)__popcll(mlo & below);
            rhi[w] = clo + (uint32_t)__popcll(mhi & below);
            if (lane == 0) wc[wave][w] = clo + (uint32_t)__popcll(mhi);
        }
    }
    __syncthreads();
    if (threadIdx.x < nwin) {
        const unsigned w = threadIdx.x;
        uint32_t c0 = wc[0][w], c1 = wc[1][w], c2 = wc[2][w], c3 = wc[3][w];
        uint32_t base = atomicAdd(&wcount[w], c0 + c1 + c2 + c3);
        wc[0][w] = base;
        wc[1][w] = base + c0;
        wc[2][w] = base + c0 + c1;
        wc[3][w] = base + c0 + c1 + c2;
    }
    __syncthreads();
    MI_UNROLL for (unsigned w = 0; w < MAXW_S; w++) {
        if (w < nwin) {
            const uint64_t o = (uint64_t)w * n + wc[wave][w];
            if (dlo[w]) {
                keys[o + rlo[w]] = ((dlo[w] & 0x7fffffffu) - 1) << (GLV ? 1 : 0);
                vals[o + rlo[w]] = i | mark | (dlo[w] & 0x80000000u);
            }
            if (dhi[w]) {
                keys[o + rhi[w]] = GLV ? (((dhi[w] & 0x7fffffffu) - 1) << 1) | 1u : (dhi[w] & 0x7fffffffu) - 1;
                vals[o + rhi[w]] = (i + nreal) | mark | (dhi[w] & 0x80000000u);
            }
        }
    }
}

// keys are window-local (sorted per window): global bucket = window * nbk + key.  Four sorted keys
// per thread (one 16-byte load); the neighbours across the group edge are single loads (L2 hits).
// zstart[w] = first sorted position of window w holding a zero digit (key nbk sorts last).
// wcnt (compacted digits, else null): window w holds wcnt[w] valid entries from w * n on.
__global__ void k_bounds4(const uint32_t *__restrict__ keys, uint32_t np, uint32_t n, uint32_t nbk, uint32_t wk,
                          const uint32_t *__restrict__ wcnt, uint32_t *__restrict__ start, uint32_t *__restrict__ cnt,
                          uint32_t *__restrict__ zstart) {
    uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t i0 = q * 4;
    if (i0 >= np) return;
    uint32_t k[6];
    k[0] = i0 ? keys[i0 - 1] : 0xffffffffu;
    if (i0 + 4 <= np) {
        uint4 v = *reinterpret_cast<const uint4 *>(keys + i0);
        k[1] = v.x, k[2] = v.y, k[3] = v.z, k[4] = v.w;
    } else {
        MI_UNROLL for (int j = 0; j < 4; j++) k[1 + j] = i0 + j < np ? keys[i0 + j] : 0xffffffffu;
    }
    k[5] = i0 + 4 < np ? keys[i0 + 4] : 0xffffffffu;
    uint32_t w = i0 / n, lo = w * n;
    MI_UNROLL for (int j = 0; j < 4; j++) {
        uint32_t i = i0 + j;
        if (i >= np) break;
        if (i >= lo + n) {
            w++;
            lo += n;
        }
        const uint32_t lim = wcnt ? wcnt[w] : n;
        if (i - lo >= lim) continue;  // beyond the compacted entries of this window
        uint32_t kk = k[1 + j] - w * wk;  // window-local key
        if (kk == nbk) {  // zero digit: not a bucket entry
            if (i == lo || k[j] != k[1 + j]) zstart[w] = i;
            continue;
        }
        uint32_t g = w * nbk + kk;
        if (i == lo || k[j] != k[1 + j]) start[g] = i;
        if (i + 1 == lo + lim || k[2 + j] != k[1 + j]) cnt[g] = i + 1;  // end; converted to a count below
    }
}

// last index i < n with a[i] <= x (a non-decreasing, a[0] <= x): the owner of slot x of an exclusive scan
MI_HD uint32_t owner_of(const uint32_t *__restrict__ a, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;  // a[lo] <= x < a[hi] (a[n] = infinity)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

// one launch for a plan's bucket arrays: start = cnt = 0 over nb buckets, zstart = ~0 over nz windows
__global__ void k_plan_init(uint32_t *__restrict__ start, uint32_t *__restrict__ cnt, uint32_t nb,
                            uint32_t *__restrict__ zstart, uint32_t nz) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) start[b] = cnt[b] = 0;
    if (b < nz) zstart[b] = 0xffffffffu;
}

__global__ void k_end_to_cnt(const uint32_t *__restrict__ start, uint32_t *__restrict__ cnt, uint32_t nb) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint32_t e = cnt[b];
    cnt[b] = e ? e - start[b] : 0;
}

// chunk counts; also zeroes the plan's per-level tree totals (k_tree_count_l1 adds into them later)
__global__ void k_chunk_count(const uint32_t *__restrict__ cnt, uint32_t nb, uint32_t L, uint32_t *__restrict__ ccnt,
                              uint32_t *__restrict__ totals, uint32_t ntot) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < ntot) totals[b] = 0;
    if (b >= nb) return;
    ccnt[b] = (cnt[b] + L - 1) / L;
}



// Level-0 chunk lengths, keyed so a radix sort puts equal lengths next to each other: a wave then
// runs chunks of (nearly) one length instead of "full chunks + remainders" (~69% lane use for
// Poisson(32) buckets).  key = L0 - len (full chunks first).
__global__ void k_chunk_len_keys(const uint32_t *__restrict__ coff, const uint32_t *__restrict__ cnt, uint32_t nb,
                                 uint32_t total, uint32_t L0, uint32_t *__restrict__ chunk_bucket,
                                 uint32_t *__restrict__ keys, uint32_t *__restrict__ ids) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const uint32_t b = owner_of(coff, nb, t);  // the bucket whose chunks start at or before t
    chunk_bucket[t] = b;
    uint32_t local = t - coff[b];
    uint32_t rest = cnt[b] - local * L0;
    keys[t] = L0 - (rest < L0 ? rest : L0);
    ids[t] = t;
}

template <class F>
__global__ void __launch_bounds__(256) MI_WAVES_ACC k_accum_level0(const uint32_t *__restrict__ order,
                                                      const uint32_t *__restrict__ chunk_bucket,
                                                      const uint32_t *__restrict__ coff,
                                                      const uint32_t *__restrict__ off,
                                                      const uint32_t *__restrict__ cnt, uint32_t total, uint32_t L0,
                                                      const uint32_t *__restrict__ vals,
                                                      const Affine<F> *__restrict__ bases,
                                                      const Affine<F> *__restrict__ bases_hi, uint32_t nreal,
                                                      XYZZ<F> *__restrict__ out) {
    using LP = Lane<F>;
    // point j of the plan: bases[j], or in split mode bases_hi[j - nreal] from j = nreal on
    // (G1 only: split mode has no G2 table, and the select costs the G2 lane-pair kernel registers)
    auto src = [&](uint32_t v) {
        const uint32_t j = v & IDX_MASK;
        if constexpr (sizeof(F) == sizeof(fq_t))
            return j < nreal ? bases + j : bases_hi + (j - nreal);
        else
            return bases + j;
    };
    using R = typename LP::R;
    uint32_t u = (blockIdx.x * blockDim.x + threadIdx.x) / LP::K;  // a lane pair per chunk for G2
    if (u >= total) return;
    uint32_t t = order[u];  // chunk id, length-sorted
    uint32_t b = chunk_bucket[t];
    uint32_t local = t - coff[b];
    uint32_t beg = off[b] + local * L0;
    uint32_t lim = local * L0 + L0 < cnt[b] ? local * L0 + L0 : cnt[b];
    uint32_t end = off[b] + lim;
    XYZZ<R> acc = XYZZ<R>::inf();
#if MI_ACC_PREFETCH
    // Software pipeline: the next point's loads (and the index after it) are issued before this
    // addition, so a wave no longer waits out two dependent HBM round trips (index, then point) at
    // the top of every iteration.
    if (beg < end) {
        uint32_t v = vals[beg];
        uint32_t vn = beg + 1 < end ? vals[beg + 1] : 0u;
        Affine<R> a = LP::lda(src(v));
        for (uint32_t p = beg; p < end; p++) {
            Affine<R> an = a;
            uint32_t vnn = 0;
            if (p + 1 < end) {
                an = LP::lda(src(vn));
                if (p + 2 < end) vnn = vals[p + 2];
            }
            if (v >> 31) a.y = lazy_neg(a.y);
            acc = xyzz_add_affine_inl(acc, a);
            a = an;
            v = vn;
            vn = vnn;
        }
    }
#else
    for (uint32_t p = beg; p < end; p++) {
        uint32_t v = vals[p];
        Affine<R> a = LP::lda(src(v));
        if (v >> 31) a.y = lazy_neg(a.y);
        acc = xyzz_add_affine_inl(acc, a);
    }
#endif
    LP::st(out + t, acc);
}

// Buckets that span several level-0 chunks: their chunk partials P0[coff[b] + j] (j < ccnt[b]) are
// summed in place by a strided tree, L1 partials per thread per level.  Only those buckets take
// part (compacted list), so single-chunk buckets are never copied.
__global__ void k_flag_multi(const uint32_t *__restrict__ ccnt, uint32_t nb, uint8_t *__restrict__ flag) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    flag[b] = ccnt[b] > 1;
}

__global__ void k_tree_count(const uint32_t *__restrict__ mlist, const uint32_t *__restrict__ ccnt, uint32_t m,
                             uint32_t stride, uint32_t L1, uint32_t *__restrict__ qcnt) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint32_t n = ccnt[mlist[i]];
    uint32_t parts = (n + stride - 1) / stride;
    qcnt[i] = (parts + L1 - 1) / L1;
}

// the first tree level's quotas before m is known on the host: over all nb slots, zero from *m_dev on; and every
// level's partial count, totals[l] = sum_i ceil(ceil(n_i / L1^l) / L1) for the levels the largest bucket needs
// (stride L1^l below ceil(*maxcnt / L0)), so the tree runs without a host round trip per level.  L1 is a power of
// two (shifts, no division).  TC_PER buckets per thread and one atomic per block and level: a wave-level atomic
// put ~200 K same-address atomics per level into a 2^27-point plan (4 ms per launch in the Window-PoSt proof).
constexpr unsigned TC_PER = 8;
__global__ void __launch_bounds__(256) k_tree_count_l1(const uint32_t *__restrict__ mlist,
                                                       const uint32_t *__restrict__ ccnt,
                                                       const uint32_t *__restrict__ m_dev,
                                                       const uint32_t *__restrict__ maxcnt, uint32_t L0, uint32_t nb,
                                                       unsigned lg1, uint32_t *__restrict__ qcnt,
                                                       uint32_t *__restrict__ totals) {
    __shared__ uint32_t part[TREE_MAXL][4];
    const uint32_t m = *m_dev;
    const uint32_t mask1 = (1u << lg1) - 1;
    const uint32_t maxchunks = (*maxcnt + L0 - 1) / L0;
    unsigned nlev = 0;  // levels with stride 2^(l lg1) below maxchunks
    for (unsigned s = 0; nlev < TREE_MAXL && s < 32 && (1u << s) < maxchunks; s += lg1) nlev++;
    uint32_t acc[TREE_MAXL];
    MI_UNROLL for (unsigned l = 0; l < TREE_MAXL; l++) acc[l] = 0;
    const uint32_t i0 = blockIdx.x * (256 * TC_PER) + threadIdx.x;
    for (unsigned j = 0; j < TC_PER; j++) {
        const uint32_t i = i0 + j * 256;
        const uint32_t n = i < nb && i < m ? ccnt[mlist[i]] : 0u;
        if (i < nb) qcnt[i] = (n + mask1) >> lg1;
        MI_UNROLL for (unsigned l = 0; l < TREE_MAXL; l++) {
            if (l < nlev) {
                const unsigned s = l * lg1;
                const uint32_t parts = n ? ((n - 1) >> s) + 1 : 0u;
                acc[l] += (parts + mask1) >> lg1;
            }
        }
    }
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    MI_UNROLL for (unsigned l = 0; l < TREE_MAXL; l++) {
        if (l < nlev) {
            uint32_t q = acc[l];
            for (int o = 32; o; o >>= 1) q += __shfl_xor(q, o);
            if (lane == 0) part[l][wave] = q;
        }
    }
    __syncthreads();
    if (threadIdx.x < nlev) {
        const uint32_t t = part[threadIdx.x][0] + part[threadIdx.x][1] + part[threadIdx.x][2] + part[threadIdx.x][3];
        if (t) atomicAdd(&totals[threadIdx.x], t);
    }
}


// the plan's counts into one staging block (one readback): chunk total (coff / ccnt tails), m, the first tree level's
// total (qoff / qcnt tails), every level's total
__global__ void k_plan_gather(const uint32_t *__restrict__ coff, const uint32_t *__restrict__ ccnt, uint32_t nb,
                              const uint32_t *__restrict__ m_dev, const uint32_t *__restrict__ qoff,
                              const uint32_t *__restrict__ qcnt, const uint32_t *__restrict__ totals,
                              uint32_t *__restrict__ stage) {
    const uint32_t t = threadIdx.x;
    if (t == 0) stage[0] = coff[nb - 1];
    if (t == 1) stage[1] = ccnt[nb - 1];
    if (t == 2) stage[2] = *m_dev;
    if (t == 3) stage[3] = qoff[nb - 1];
    if (t == 4) stage[4] = qcnt[nb - 1];
    if (t >= 5 && t < 5 + TREE_MAXL) stage[t] = totals[t - 5];
}

template <class F>
__global__ void __launch_bounds__(256) MI_WAVES_RED k_tree_level(const uint32_t *__restrict__ qoff, uint32_t m,
                                                    const uint32_t *__restrict__ mlist,
                                                    const uint32_t *__restrict__ coff,
                                                    const uint32_t *__restrict__ ccnt, uint32_t total,
                                                    uint32_t stride, uint32_t L1, XYZZ<F> *__restrict__ P) {
    using LP = LaneRed<F>;
    using R = typename LP::R;
    uint32_t u = (blockIdx.x * blockDim.x + threadIdx.x) / LP::K;
    if (u >= total) return;
    uint32_t i = owner_of(qoff, m, u);  // the multi-chunk bucket this partial belongs to
    uint32_t b = mlist[i];
    uint32_t q = u - qoff[i];
    uint32_t n = ccnt[b];
    XYZZ<F> *base = P + coff[b];
    uint64_t first = (uint64_t)q * L1 * stride;
    XYZZ<R> acc = LP::ld(base + first);
    for (uint32_t j = 1; j < L1; j++) {
        uint64_t idx = first + (uint64_t)j * stride;
        if (idx < n) acc = xyzz_add_inl(acc, LP::ld(base + idx));
    }
    LP::st(base + first, acc);
}

// Running-sum reduction over one segment of seg_len buckets (all group-law code inlined):
//   seg_run = sum_j B_j,  seg_acc = sum_j (j + 1) B_j   (j = bucket index inside the segment)
// Bucket b's sum is P[off[b]] when cnt[b] != 0 (level-0 chunk slot of its first chunk).
template <class F>
__global__ void __launch_bounds__(256) MI_WAVES_RED k_bucket_reduce(const uint32_t *__restrict__ off,
                                                       const uint32_t *__restrict__ cnt,
                                                       const XYZZ<F> *__restrict__ P, uint32_t nseg_total,
                                                       unsigned seg_len, XYZZ<F> *__restrict__ seg_acc,
                                                       XYZZ<F> *__restrict__ seg_run) {
    using LP = LaneRed<F>;
    using R = typename LP::R;
    uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) / LP::K;
    if (t >= nseg_total) return;
    uint32_t b0 = t * seg_len;  // buckets of one window are contiguous and nbk % seg_len == 0
    XYZZ<R> run = XYZZ<R>::inf(), acc = XYZZ<R>::inf();
    for (int j = (int)seg_len - 1; j >= 0; j--) {
        uint32_t b = b0 + j;
        if (cnt[b]) run = xyzz_add_inl(run, LP::ld(P + off[b]));
        acc = xyzz_add_inl(acc, run);
    }
    LP::st(seg_acc + t, acc);
    LP::st(seg_run + t, run);
}

// The same over a dense array of points (second level: the first level's segment sums), also
// summing the first level's accumulators over the segment (sum_acc).
template <class F>
__global__ void __launch_bounds__(256) MI_WAVES_RED k_bucket_reduce_dense(const XYZZ<F> *__restrict__ P,
                                                             const XYZZ<F> *__restrict__ A, uint32_t nseg_total,
                                                             unsigned seg_len, XYZZ<F> *__restrict__ seg_acc,
                                                             XYZZ<F> *__restrict__ seg_run,
                                                             XYZZ<F> *__restrict__ sum_acc) {
    using LP = LaneRed<F>;
    using R = typename LP::R;
    uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) / LP::K;
    if (t >= nseg_total) return;
    const XYZZ<F> *p = P + (uint64_t)t * seg_len;
    const XYZZ<F> *a = A + (uint64_t)t * seg_len;
    XYZZ<R> run = XYZZ<R>::inf(), acc = XYZZ<R>::inf(), sa = XYZZ<R>::inf();
    for (int j = (int)seg_len - 1; j >= 0; j--) {
        run = xyzz_add_inl(run, LP::ld(p + j));
        acc = xyzz_add_inl(acc, run);
        sa = xyzz_add_inl(sa, LP::ld(a + j));
    }
    LP::st(seg_acc + t, acc);
    LP::st(seg_run + t, run);
    LP::st(sum_acc + t, sa);
}

// out[t] = seg_acc[t] + (s * seg_len) * seg_run[t], s = segment index inside its window
template <class F>
__global__ void __launch_bounds__(256) MI_WAVES_RED k_seg_fold(const XYZZ<F> *__restrict__ seg_acc,
                                                  const XYZZ<F> *__restrict__ seg_run, uint32_t nseg_total,
                                                  uint32_t nseg, unsigned seg_len, XYZZ<F> *__restrict__ out) {
    using LP = LaneRed<F>;
    using R = typename LP::R;
    uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) / LP::K;
    if (t >= nseg_total) return;
    XYZZ<R> acc = LP::ld(seg_acc + t);
    uint32_t k = (t % nseg) * seg_len;
    XYZZ<R> run = LP::ld(seg_run + t);
    if (k && !run.is_inf()) {
        // k * run, left-to-right double-and-add, group law inlined (no device calls)
        XYZZ<R> m = run;
        int top = 31 - __builtin_clz(k);
        for (int bit = top - 1; bit >= 0; bit--) {
            m = xyzz_dbl_inl(m);
            if ((k >> bit) & 1) m = xyzz_add_inl(m, run);
        }
        acc = xyzz_add_inl(acc, m);
    }
    LP::st(out + t, acc);
}

// GLV plans (G1): bucket g's entries over P_i sit in sub-bucket 2g and those over phi(P_i) -- gathered as
// P_i -- in 2g + 1.  B_g = S_2g + phi(S_2g+1) with phi(X, Y, ZZ, ZZZ) = (beta X, Y, ZZ, ZZZ): one Fq
// multiplication and at most one full addition per bucket instead of a beta multiplication per gathered
// point (or a 2^128 table).  Writes the dense bucket sums Bm, live[g] = non-empty and iota[g] = g, the
// off / cnt view reduce_windows reads.
template <class F>
__global__ void __launch_bounds__(256) MI_WAVES_RED k_glv_merge(const uint32_t *__restrict__ coff,
                                                   const uint32_t *__restrict__ cnt,
                                                   const XYZZ<F> *__restrict__ P0, uint32_t nb, F beta,
                                                   XYZZ<F> *__restrict__ Bm, uint32_t *__restrict__ live,
                                                   uint32_t *__restrict__ iota) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nb) return;
    const uint32_t c0 = cnt[2 * g], c1 = cnt[2 * g + 1];
    XYZZ<F> a = XYZZ<F>::inf();
    if (c0) a = P0[coff[2 * g]];
    if (c1) {
        XYZZ<F> b = P0[coff[2 * g + 1]];
        b.X = b.X * beta;
        a = c0 ? xyzz_add_inl(a, b) : b;
    }
    Bm[g] = a;
    live[g] = (c0 | c1) ? 1u : 0u;
    iota[g] = g;
}

// out[w * (n / G) + g] = sum of in[w * n + g * G ... + G)   (n % G == 0)
template <class F>
__global__ void __launch_bounds__(256) MI_WAVES_RED k_sum_groups(const XYZZ<F> *__restrict__ in, uint32_t total_out,
                                                    unsigned G, XYZZ<F> *__restrict__ out) {
    using LP = LaneRed<F>;
    using R = typename LP::R;
    uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) / LP::K;
    if (t >= total_out) return;
    XYZZ<R> acc = LP::ld(in + (uint64_t)t * G);
    for (unsigned i = 1; i < G; i++) acc = xyzz_add_inl(acc, LP::ld(in + (uint64_t)t * G + i));
    LP::st(out + t, acc);
}

// ---- low-depth bucket reduction of one-window plans (reduce_bitsum) ----
// From the first level's segment sums (acc_s = sum_j (j + 1) B_{s SA + j}, run_s = sum_j B_{s SA + j}, s < nseg
// = 2^lseg per window): W = sum_s acc_s + SA sum_s s run_s, and sum_s s run_s = sum_k 2^k T_k with
// T_k = sum of run_s over the s whose bit k is set.  Row 0 of a window sums acc, row 1 + k gives T_k: plain sums,
// so the device part is a tree of depth ~log2(nseg) instead of running sums over the segments (depth ~2 nseg /
// parallelism) -- the reduction of a one-window plan is latency-bound, not work-bound.  Thread (row, g) sums G
// items of its row; bit rows hold nseg / 2 items, so their upper half of partials is the identity.
// The bit-row kernels run a few waves per SIMD at most (latency-bound trees), so they carry no two-wave register cap:
// the G2 lane-pair full addition then keeps its values in registers instead of ~260 spilled dwords
template <class F>
__global__ void __launch_bounds__(256) k_bitsum_first(const XYZZ<F> *__restrict__ acc,
                                                      const XYZZ<F> *__restrict__ run, uint32_t nwin, uint32_t nseg,
                                                      unsigned lseg, unsigned G, XYZZ<F> *__restrict__ out) {
    using LP = LaneRed<F>;  // a lane pair per element for G2 (g2pair.h)
    using R = typename LP::R;
    // rows of a window: 0 / 1 = the two halves of acc, 2 + k = T_k; every row holds nseg / 2 items
    const uint32_t half = nseg >> 1, per = half / G, rpw = 2 + lseg;
    const uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / LP::K;
    if (t >= (uint64_t)nwin * rpw * per) return;
    const uint32_t g = (uint32_t)(t % per), r = (uint32_t)((t / per) % rpw), w = (uint32_t)(t / ((uint64_t)per * rpw));
    XYZZ<R> s = XYZZ<R>::inf();
    if (r < 2) {
        const XYZZ<F> *p = acc + (uint64_t)w * nseg + (uint64_t)r * half + (uint64_t)g * G;
        for (unsigned j = 0; j < G; j++) s = xyzz_add_inl(s, LP::ld(p + j));
    } else {
        const unsigned k = r - 2;
        const XYZZ<F> *p = run + (uint64_t)w * nseg;
        for (unsigned j = 0; j < G; j++) {
            const uint32_t i = g * G + j;
            s = xyzz_add_inl(s, LP::ld(p + (((i >> k) << (k + 1)) | (1u << k) | (i & ((1u << k) - 1)))));
        }
    }
    LP::st(out + t, s);
}

// out[b] = sum of in[b m, b m + m) (m <= 256 / K, a power of two): one block per output, pairwise tree in LDS
template <class F>
__global__ void __launch_bounds__(256) k_sum_lds(const XYZZ<F> *__restrict__ in, uint32_t m,
                                                 XYZZ<F> *__restrict__ out) {
    using LP = LaneRed<F>;
    __shared__ __align__(16) unsigned char raw[256 / LP::K * sizeof(XYZZ<F>)];
    XYZZ<F> *sh = reinterpret_cast<XYZZ<F> *>(raw);
    const uint32_t b = blockIdx.x, e = threadIdx.x / LP::K;  // element of this thread (both lanes of a pair)
    if (e < m) LP::st(sh + e, LP::ld(in + (uint64_t)b * m + e));
    __syncthreads();
    for (uint32_t h = m >> 1; h; h >>= 1) {
        if (e < h) LP::st(sh + e, xyzz_add_inl(LP::ld(sh + e), LP::ld(sh + e + h)));
        __syncthreads();
    }
    if (e == 0) LP::st(out + b, LP::ld(sh));
}

// ---- G2 second-level bucket reduction (g2_second_level) ----
// Bucket sums -> affine by Montgomery's trick over K consecutive buckets per thread (empty or
// infinite buckets become the affine infinity (0, 0)).
template <class F, int K>
__global__ void __launch_bounds__(256) k_bucket_affine(const uint32_t *__restrict__ coff,
                                                       const uint32_t *__restrict__ cnt,
                                                       const XYZZ<F> *__restrict__ P0, uint32_t nb,
                                                       F *__restrict__ pre, Affine<F> *__restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t beg = t * K;
    if (beg >= nb) return;
    const uint64_t end = beg + K < nb ? beg + K : nb;
    F prod = F::one();
    for (uint64_t i = beg; i < end; i++) {
        pre[i] = prod;
        if (cnt[i]) {
            const XYZZ<F> p = P0[coff[i]];
            if (!p.is_inf()) prod = prod * p.ZZZ;
        }
    }
    F inv = inverse_inl(prod);
    for (uint64_t i = end; i-- > beg;) {
        if (!cnt[i]) {
            out[i] = Affine<F>::inf();
            continue;
        }
        const XYZZ<F> p = P0[coff[i]];
        if (p.is_inf()) {
            out[i] = Affine<F>::inf();
            continue;
        }
        F izzz = inv * pre[i];
        inv = inv * p.ZZZ;
        F izz = sqr(p.ZZ * izzz);
        out[i] = {p.X * izz, p.Y * izzz};
    }
}

// Bucket g = w * 2^jbits + j of a non-empty bucket carries weight s = j + 1 < 2^(2 c2): entries
// (window 2w, digit s mod 2^c2) and (window 2w + 1, digit s >> c2), keys window * 2^c2 + digit - 1.
__global__ void k_l2_digits(const uint32_t *__restrict__ cnt, uint32_t nb, unsigned jbits, unsigned c2,
                            uint32_t invalid, uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nb) return;
    const uint32_t w = g >> jbits, s = (g & ((1u << jbits) - 1)) + 1;
    const uint32_t d0 = s & ((1u << c2) - 1), d1 = s >> c2;
    const bool live = cnt[g] != 0;
    keys[2 * (uint64_t)g] = live && d0 ? ((2 * w) << c2) + d0 - 1 : invalid;
    keys[2 * (uint64_t)g + 1] = live && d1 ? ((2 * w + 1) << c2) + d1 - 1 : invalid;
    vals[2 * (uint64_t)g] = g;
    vals[2 * (uint64_t)g + 1] = g;
}

// bucket start / end of globally keyed sorted entries (invalid keys sort last and are skipped)
__global__ void k_bounds_flat(const uint32_t *__restrict__ keys, uint32_t np, uint32_t invalid,
                              uint32_t *__restrict__ start, uint32_t *__restrict__ endp) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const uint32_t k = keys[i];
    if (k == invalid) return;
    if (i == 0 || keys[i - 1] != k) start[k] = i;
    if (i + 1 == np || keys[i + 1] != k) endp[k] = i + 1;
}

inline unsigned grid_for(uint64_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

// (bucket key, point index) pair sort of one window: rocPRIM onesweep with 11-bit places, so the
// 22-bit keys of a 2^26 MSM take 2 places instead of 3 at the gfx950 default of 8 (-8% sort time).
#ifndef MI_SORT_BLOCK
#define MI_SORT_BLOCK 1024
#endif
#ifndef MI_SORT_IPT
#define MI_SORT_IPT 24  // measured: 20.2 vs 21.3 ms of digits+sort per 2^26 MSM at 16
#endif
#ifndef MI_SORT_RADIX
#define MI_SORT_RADIX 11
#endif
// MergeSortLimit 0: rocPRIM's default sends every sort of <= 2^20 items through block sort + merge passes
// (~19 launches per sort); below 2^20 items onesweep's 1-2 passes are far faster (the Winning-PoSt proof's
// 2^19-point MSMs spent 14.6 of 42 ms in merge passes).  Inputs of one block still take the single-block sort.
using onesweep11_cfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<MI_SORT_BLOCK, MI_SORT_IPT>,
                                        rocprim::kernel_config<MI_SORT_BLOCK, MI_SORT_IPT>, MI_SORT_RADIX,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

inline void sort_pairs_u32(void *tmp, size_t &bytes, const uint32_t *k_in, uint32_t *k_out, const uint32_t *v_in,
                           uint32_t *v_out, uint32_t n, unsigned bits, hipStream_t st) {
    MI_HIP(rocprim::radix_sort_pairs<onesweep11_cfg>(tmp, bytes, k_in, k_out, v_in, v_out, n, 0, bits, st));
}

}  // namespace

// ---- phase 1 (scalars only, shared by every MSM over the same scalars: B_G1 and B_G2) ----
// digits -> per-window sort -> bucket bounds -> level-0 chunking -> length-sorted chunk order.
// Level-0 chunking of a bucketed entry list (bucket b: entries [off[b], off[b] + cnt[b]) of vals_s).
// plan_counts queues everything that needs no host-side count -- chunk counts and offsets, the multi-chunk bucket
// list and the first chunk-tree level's quotas -- and the readback of those counts into pin[0, PLAN_PIN); the
// caller reads them after ITS one synchronisation (with its own bucket maxima) and plan_finish completes the plan:
// chunk -> bucket map, length-sorted chunk order.  false when there is no entry at all.
constexpr unsigned PLAN_PIN = 5 + TREE_MAXL;
// scratch slots of the plan arrays that outlive plan_counts / plan_finish (the rest are temporaries): a plan's own, or
// a derived plan's (msm_derive_plan_impl), which must survive the next plan on the same ctx
struct PlanSlots {
    unsigned mlist = 24, chunk_bucket = 17, order = 16;
};
constexpr PlanSlots DERIVED_SLOTS{31, 32, 33};
inline void plan_counts(Ctx &c, MsmPlan &pl, const uint32_t *cntA, uint32_t *offB, uint32_t *cntB, uint32_t nb,
                        const uint32_t *maxcnt_dev, uint32_t *stage, PlanSlots ps = {}) {
    hipStream_t st = c.stream;
    // tune::MSM_L0 / MSM_L1 (tuning A/B): entries per level-0 chunk, partials per tree-level thread (a power of two)
    const uint32_t l0_auto = pl.n >= (1ull << 24) ? L0_LARGE : L0_DEFAULT;
    const int64_t t0 = tune::get(tune::MSM_L0, l0_auto), t1 = tune::get(tune::MSM_L1, L1_DEFAULT);
    uint32_t L0 = t0 >= 2 && t0 <= 1024 ? (uint32_t)t0 : l0_auto, L1 = t1 >= 4 && t1 <= 64 ? (uint32_t)t1 : L1_DEFAULT;
    if (L1 < 4 || L1 > 64 || (L1 & (L1 - 1))) L1 = L1_DEFAULT;
    unsigned lg1 = 0;
    while ((1u << lg1) < L1) lg1++;
    pl.L0 = L0;
    pl.L1 = L1;
    uint32_t *coff = offB, *ccnt = cntB;
    uint32_t *mlist = c.scratch[ps.mlist].as<uint32_t>(3 * (uint64_t)nb + 1 + TREE_MAXL), *m_dev = mlist + nb;
    uint32_t *qcnt = m_dev + 1, *qoff = qcnt + nb, *totals = qoff + nb;
    // level 0: buckets cut into chunks of <= L0 sorted entries; one mixed-add chain per chunk
    k_chunk_count<<<grid_for(nb > TREE_MAXL ? nb : TREE_MAXL, 256), 256, 0, st>>>(cntA, nb, L0, ccnt, totals, TREE_MAXL);
    MI_LAUNCHED(c, "k_chunk_count");
    size_t tmp_bytes = 0;
    MI_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, ccnt, coff, nb, st));
    void *tmp = c.scratch[4].get(tmp_bytes);
    MI_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, ccnt, coff, nb, st));
    // buckets of several chunks, and the first in-place tree level over their partials
    uint8_t *flag = c.scratch[25].as<uint8_t>(nb);
    k_flag_multi<<<grid_for(nb, 256), 256, 0, st>>>(ccnt, nb, flag);
    MI_LAUNCHED(c, "k_flag_multi");
    size_t tb = 0;
    hipcub::CountingInputIterator<uint32_t> ids(0);
    MI_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, ids, flag, mlist, m_dev, nb, st));
    tmp = c.scratch[4].get(tb);
    MI_HIP(hipcub::DeviceSelect::Flagged(tmp, tb, ids, flag, mlist, m_dev, nb, st));
    k_tree_count_l1<<<grid_for(nb, 256 * TC_PER), 256, 0, st>>>(mlist, ccnt, m_dev, maxcnt_dev, L0, nb, lg1, qcnt,
                                                                 totals);
    MI_LAUNCHED(c, "k_tree_count_l1");
    tb = 0;
    MI_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, qcnt, qoff, nb, st));
    tmp = c.scratch[4].get(tb);
    MI_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, qcnt, qoff, nb, st));
    k_plan_gather<<<1, 64, 0, st>>>(coff, ccnt, nb, m_dev, qoff, qcnt, totals, stage);
    MI_LAUNCHED(c, "k_plan_gather");
    pl.coff = coff;
    pl.ccnt = ccnt;
    pl.mlist = mlist;
    pl.qcnt = qcnt;
    pl.qoff = qoff;
}

inline bool plan_finish(Ctx &c, MsmPlan &pl, const uint32_t *offA, const uint32_t *cntA, uint32_t nb,
                        const uint32_t *vals_s, const uint32_t *pin, PlanSlots ps = {}) {
    hipStream_t st = c.stream;
    const uint32_t L0 = pl.L0;
    unsigned len_bits = 1;
    while ((1u << len_bits) <= L0) len_bits++;
    const uint32_t total = pin[0] + pin[1];
    pl.total = total;
    pl.m = pin[2];
    pl.l1_total = pin[3] + pin[4];
    for (unsigned l = 0; l < TREE_MAXL; l++) pl.level_total[l] = pin[5 + l];
    if (total == 0) return false;  // every scalar is zero
    const uint32_t *coff = pl.coff;
    uint32_t *chunk_bucket = c.scratch[ps.chunk_bucket].as<uint32_t>(total + 1);
    // chunk -> bucket (binary search over the chunk offsets) and the length-sorted chunk order (keys/vals scratch of
    // the main sort are free by now)
    uint32_t *lkeys = c.scratch[0].as<uint32_t>(total), *lids = c.scratch[1].as<uint32_t>(total);
    uint32_t *lkeys_s = c.scratch[2].as<uint32_t>(total), *order = c.scratch[ps.order].as<uint32_t>(total);
    k_chunk_len_keys<<<grid_for(total, 256), 256, 0, st>>>(coff, cntA, nb, total, L0, chunk_bucket, lkeys, lids);
    MI_LAUNCHED(c, "k_chunk_len_keys");
    size_t tb = 0;
    sort_pairs_u32(nullptr, tb, lkeys, lkeys_s, lids, order, total, len_bits, st);
    void *tmp2 = c.scratch[4].get(tb);
    sort_pairs_u32(tmp2, tb, lkeys, lkeys_s, lids, order, total, len_bits, st);
    pl.vals_s = vals_s;
    pl.off = offA;
    pl.cnt = cntA;
    pl.chunk_bucket = chunk_bucket;
    pl.order = order;
    return true;
}

// tune::PLAN_PRIO = 1 (A/B): the plan's kernels run on a high-priority stream of the lane, so that a plan built beside
// the other lane's accumulation gets CUs as they free instead of queueing behind long accumulation workgroups.  RAII:
// the lane's stream is swapped for the plan stream (after an event on it) and back (the lane waits for the plan).
struct PlanStream {
    Ctx &c;
    hipStream_t saved = nullptr;
    explicit PlanStream(Ctx &ctx) : c(ctx) {
        if (tune::get(tune::PLAN_PRIO, 0) != 1) return;
        if (!c.plan_stream) {
            int lo = 0, hi = 0;
            MI_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
            MI_HIP(hipStreamCreateWithPriority(&c.plan_stream, hipStreamNonBlocking, hi));
            MI_HIP(hipEventCreateWithFlags(&c.plan_ev[0], hipEventDisableTiming));
            MI_HIP(hipEventCreateWithFlags(&c.plan_ev[1], hipEventDisableTiming));
        }
        saved = c.stream;
        MI_HIP(hipEventRecord(c.plan_ev[0], saved));
        MI_HIP(hipStreamWaitEvent(c.plan_stream, c.plan_ev[0], 0));
        c.stream = c.plan_stream;
    }
    ~PlanStream() {  // also on unwinding: the lane's stream comes back ordered after the plan's work
        if (!saved) return;
        (void)hipEventRecord(c.plan_ev[1], c.plan_stream);
        (void)hipStreamWaitEvent(saved, c.plan_ev[1], 0);
        c.stream = saved;
    }
};

// The plan's arrays live in scratch slots 3, 5-8, 16, 17 and stay valid until the next prepare on
// this ctx; the accumulation phase only uses the other slots.
inline bool msm_prepare_impl(Ctx &c, const fr_t *scalars, const uint32_t *idx, uint64_t nscal, MsmPlan &pl,
                             bool split = false, bool glv = false, const uint32_t *amark = nullptr) {
    pl = MsmPlan();
    if (nscal == 0) return false;
    PlanStream plan_stream(c);
    split = split || glv;
    pl.glv = glv;
    // split mode: 2 nscal points with 128-bit scalars (+1 carry bit), always on the compacted path
    const uint64_t n = split ? 2 * nscal : nscal;
    const unsigned sbits = split ? 129 : 256;
    pl.n = n;
    pl.nreal = split ? nscal : 0;
    hipStream_t st = c.stream;
    const unsigned cb = msm_window_bits_for(n, sbits, glv);
    const unsigned nwin = (sbits + cb - 1) / cb;
    // plan buckets per window: 2^(c-1), or twice that for GLV (sub-buckets over P and over phi(P))
    const uint32_t nbk = (glv ? 2u : 1u) << (cb - 1);
    const uint64_t nb64 = (uint64_t)nwin * nbk;
    const uint64_t np64 = (uint64_t)nwin * n;
    if (np64 >= 0xffffffffull || nb64 >= A_MARK || n >= A_MARK)
        throw std::runtime_error("msm: instance too large for 32-bit sort indices");
    const uint32_t nb = (uint32_t)nb64, np = (uint32_t)np64, invalid = nbk;  // window-local keys
    unsigned key_bits = 1;
    while ((1ull << key_bits) <= invalid) key_bits++;  // cb bits: one fewer onesweep pass than global keys
    if (glv) {  // compacted GLV keys stay below nbk (no zero-digit sentinel): cb bits, as the 2^128 split
        key_bits = 1;
        while ((1ull << key_bits) < nbk) key_bits++;
    }
    // Small MSMs sort every window in ONE call over keys w * (nbk + 1) + local when that still takes
    // two 11-bit onesweep places (2^20: 2 launches instead of 32); large ones sort window by window.
    unsigned all_bits = 1;
    while ((1ull << all_bits) <= (uint64_t)nwin * (nbk + 1) - 1) all_bits++;
    // tune::MSM_SORT = 1 forces the per-window path (and with it the zero-digit compaction when
    // nwin <= MAXW_C) at any size: tests use it to cover the large-MSM path at 2^20
    const bool force_windowed = tune::get(tune::MSM_SORT, 0) == 1;
    const bool one_sort = !force_windowed && !split && all_bits <= 22 && nwin > 1;
    const uint32_t wk = one_sort ? nbk + 1 : 0;
    pl.cb = cb;
    pl.nwin = nwin;
    pl.nbk = nbk;
    pl.nb = nb;

    uint32_t *keys = c.scratch[0].as<uint32_t>(np);
    uint32_t *vals = c.scratch[1].as<uint32_t>(np);
    uint32_t *keys_s = c.scratch[2].as<uint32_t>(np);
    uint32_t *vals_s = c.scratch[3].as<uint32_t>(np);
    uint32_t *offA = c.scratch[5].as<uint32_t>(nb);
    uint32_t *cntA = c.scratch[6].as<uint32_t>(nb);
    uint32_t *offB = c.scratch[7].as<uint32_t>(nb);
    uint32_t *cntB = c.scratch[8].as<uint32_t>(nb);
    // [max bucket size, pad x 3, zstart[nwin], wcount[nwin], the plan's counts (PLAN_PIN)]: one readback
    uint32_t *dmax = c.scratch[9].as<uint32_t>(4 + 2 * nwin + PLAN_PIN);
    uint32_t *zstart = dmax + 4, *wcount = zstart + nwin;
    const bool compact = !one_sort && nwin <= MAXW_C;  // large MSMs: only non-zero digits are sorted
    if (split && !compact) throw std::logic_error("msm: split mode needs the compacted digit path");
    std::vector<uint32_t> wn(nwin, 0);

    {
        ScopedTimer tsort(c, &c.stats.sort, n);
        size_t tmp_bytes = 0;
        if (compact) {
            MI_HIP(hipMemsetAsync(wcount, 0, sizeof(uint32_t) * nwin, st));
            if (split) {
                if (nwin > MAXW_S) throw std::logic_error("msm: split plan with more than MAXW_S windows");
                if (glv)
                    k_digits_split<true><<<grid_for(nscal, 256), 256, 0, st>>>(scalars, idx, (uint32_t)nscal, cb, nwin,
                                                                                wcount, keys, vals, amark);
                else
                    k_digits_split<false><<<grid_for(nscal, 256), 256, 0, st>>>(scalars, idx, (uint32_t)nscal, cb, nwin,
                                                                                 wcount, keys, vals, amark);
                pl.marked = amark != nullptr;
                MI_LAUNCHED(c, "k_digits_split");
            } else {
                k_digits_c<<<grid_for(n, 256), 256, 0, st>>>(scalars, idx, (uint32_t)n, cb, nwin, 0u, wcount, keys,
                                                              vals);
                MI_LAUNCHED(c, "k_digits_c");
            }
            uint32_t *wn_pin = c.pin.as<uint32_t>(nwin);
            MI_HIP(hipMemcpyAsync(wn_pin, wcount, sizeof(uint32_t) * nwin, hipMemcpyDeviceToHost, st));
            MI_HIP(hipStreamSynchronize(st));
            std::copy(wn_pin, wn_pin + nwin, wn.begin());
            if (nwin <= MAXW_S) std::copy(wn_pin, wn_pin + nwin, pl.wn);
            sort_pairs_u32(nullptr, tmp_bytes, keys, keys_s, vals, vals_s, (uint32_t)n, key_bits, st);
            void *tmp = c.scratch[4].get(tmp_bytes);
            for (unsigned w = 0; w < nwin; w++) {
                uint64_t o = (uint64_t)w * n;
                if (wn[w])
                    sort_pairs_u32(tmp, tmp_bytes, keys + o, keys_s + o, vals + o, vals_s + o, wn[w], key_bits, st);
            }
        } else {
            k_digits<<<grid_for(n, 256), 256, 0, st>>>(scalars, idx, (uint32_t)n, cb, nwin, invalid, wk, keys, vals);
            MI_LAUNCHED(c, "k_digits");
            if (one_sort) {
                sort_pairs_u32(nullptr, tmp_bytes, keys, keys_s, vals, vals_s, np, all_bits, st);
                void *tmp = c.scratch[4].get(tmp_bytes);
                sort_pairs_u32(tmp, tmp_bytes, keys, keys_s, vals, vals_s, np, all_bits, st);
            } else {
                sort_pairs_u32(nullptr, tmp_bytes, keys, keys_s, vals, vals_s, (uint32_t)n, key_bits, st);
                void *tmp = c.scratch[4].get(tmp_bytes);
                for (unsigned w = 0; w < nwin; w++) {
                    uint64_t o = (uint64_t)w * n;
                    sort_pairs_u32(tmp, tmp_bytes, keys + o, keys_s + o, vals + o, vals_s + o, (uint32_t)n, key_bits,
                                   st);
                }
            }
        }
        k_plan_init<<<grid_for(nb > nwin ? nb : nwin, 256), 256, 0, st>>>(offA, cntA, nb, zstart, nwin);
        MI_LAUNCHED(c, "k_plan_init");
        const uint32_t nq = (np + 3) / 4;
        k_bounds4<<<grid_for(nq, 256), 256, 0, st>>>(keys_s, np, (uint32_t)n, nbk, wk, compact ? wcount : nullptr,
                                                      offA, cntA, zstart);
        MI_LAUNCHED(c, "k_bounds4");
        k_end_to_cnt<<<grid_for(nb, 256), 256, 0, st>>>(offA, cntA, nb);
        MI_LAUNCHED(c, "k_end_to_cnt");
    }

    // largest bucket (the number of chunk-tree levels), each window's zero-digit start and the plan's counts: one
    // readback
    const unsigned H = 4 + 2 * nwin;
    uint32_t *pin = c.pin.as<uint32_t>(H + PLAN_PIN);
    {
        size_t tmp_bytes = 0;
        MI_HIP(hipcub::DeviceReduce::Max(nullptr, tmp_bytes, cntA, dmax, nb, st));
        void *tmp = c.scratch[4].get(tmp_bytes);
        MI_HIP(hipcub::DeviceReduce::Max(tmp, tmp_bytes, cntA, dmax, nb, st));
        plan_counts(c, pl, cntA, offB, cntB, nb, dmax, dmax + H);
        MI_HIP(hipMemcpyAsync(pin, dmax, sizeof(uint32_t) * (H + PLAN_PIN), hipMemcpyDeviceToHost, st));
        MI_HIP(hipStreamSynchronize(st));
    }
    pl.maxcnt = pin[0];
    pl.entries = 0;  // non-zero digits = mixed additions of the accumulation
    for (unsigned w = 0; w < nwin; w++)
        pl.entries += compact ? wn[w] : pin[4 + w] == 0xffffffffu ? n : pin[4 + w] - (uint64_t)w * n;

    return plan_finish(c, pl, offA, cntA, nb, vals_s, pin + H);
}

// ---- a plan derived from a marked plan (msm_derive_plan): A's MSM over L's digits ----
// L sums z_aux over l; the aux part of A sums the same z_aux over the A points of the variables with A density.  A
// marked L plan (A_MARK on those entries) already holds A's digits, sorted into the same buckets: keeping the marked
// entries of every bucket in order gives A's plan without a digit pass or a sort.  Three passes over L's entries in
// tiles of DERIVE_T (window by window, only the valid entries): count the marked entries per tile; write them,
// compacted, with their point index moved to A's (the compacted position of every source entry goes to `pref`); the
// new bucket bounds from `pref` at each bucket's first and last entry.  Then the usual chunking (plan_counts,
// plan_finish) into slots of their own.
namespace {
constexpr unsigned DERIVE_T = 2048;  // entries per tile: 256 threads x 8
struct DeriveArgs {
    uint64_t n;                        // window stride of the source entries
    uint32_t nwin, nreal_src, nreal_dst, dst_base;
    uint32_t wn[MAXW_S];               // valid source entries of window w
    uint32_t tile0[MAXW_S + 1];        // first tile of window w
    uint32_t vbase[MAXW_S + 1];        // first entry of window w in the windows' concatenation (pref's index)
};
MI_HD unsigned derive_window(const DeriveArgs &a, uint32_t tile) {
    unsigned w = 0;
    while (w + 1 < a.nwin && a.tile0[w + 1] <= tile) w++;
    return w;
}

// Both passes read a tile as 8 rounds of 256 consecutive entries (one coalesced load per thread and round); a round's
// marked entries keep their order through a ballot prefix within each wave and the waves' counts in LDS.
__global__ void __launch_bounds__(256) k_derive_count(const uint32_t *__restrict__ vals, DeriveArgs a,
                                                      uint32_t *__restrict__ tile_cnt) {
    const uint32_t t = blockIdx.x;
    const unsigned w = derive_window(a, t);
    const uint32_t base = (t - a.tile0[w]) * DERIVE_T + threadIdx.x, lim = a.wn[w];
    const uint32_t *src = vals + (uint64_t)w * a.n;
    uint32_t cnt = 0;
    MI_UNROLL for (int k = 0; k < 8; k++) {
        const uint32_t i = base + 256 * k;
        const bool f = i < lim && (src[i] & A_MARK);
        cnt += (uint32_t)__popcll(__ballot(f));  // the wave's marked entries of this round
    }
    __shared__ uint32_t ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) tile_cnt[t] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ void __launch_bounds__(256) k_derive_scatter(const uint32_t *__restrict__ vals,
                                                        const uint2 *__restrict__ rbits, DeriveArgs a,
                                                        const uint32_t *__restrict__ tile_base,
                                                        uint32_t *__restrict__ out, uint32_t *__restrict__ pref) {
    const uint32_t t = blockIdx.x;
    const unsigned w = derive_window(a, t), lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t base = (t - a.tile0[w]) * DERIVE_T + threadIdx.x, lim = a.wn[w];
    const uint32_t *src = vals + (uint64_t)w * a.n;
    uint32_t *pr = pref + a.vbase[w];
    const uint64_t below = (1ull << lane) - 1;
    __shared__ uint32_t ws[2][4];
    uint32_t run = tile_base[t];
    MI_UNROLL for (int k = 0; k < 8; k++) {
        const uint32_t i = base + 256 * k;
        const bool valid = i < lim;
        const uint32_t v = valid ? src[i] : 0u;
        const bool f = (v & A_MARK) != 0;
        const uint64_t m = __ballot(f);
        if (lane == 0) ws[k & 1][wave] = (uint32_t)__popcll(m);
        __syncthreads();  // double-buffered counts: one barrier a round
        uint32_t off = 0, all = 0;
        MI_UNROLL for (unsigned q = 0; q < 4; q++) {
            const uint32_t c = ws[k & 1][q];
            off += q < wave ? c : 0u;
            all += c;
        }
        const uint32_t pos = run + off + (uint32_t)__popcll(m & below);
        if (valid) pr[i] = pos;
        if (f) {
            const uint32_t j = v & IDX_MASK, hi = j >= a.nreal_src ? 1u : 0u;
            const uint32_t var = hi ? j - a.nreal_src : j;
            const uint2 g = rbits[var >> 5];  // (density bits, A points before them) of var's group of 32
            const uint32_t r = g.y + __popc(g.x & ((1u << (var & 31)) - 1));
            out[pos] = (a.dst_base + r + (hi ? a.nreal_dst : 0u)) | (v & 0x80000000u);
        }
        run += all;
    }
}

// bucket b of the source plan (entries [off, off + cnt) of vals, window b / nbk) -> its marked entries' range
__global__ void k_derive_bounds(const uint32_t *__restrict__ off, const uint32_t *__restrict__ cnt, uint32_t nb,
                                uint32_t nbk, const uint32_t *__restrict__ vals, DeriveArgs a,
                                const uint32_t *__restrict__ pref, uint32_t *__restrict__ off2,
                                uint32_t *__restrict__ cnt2) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const uint32_t c = cnt[b];
    if (!c) {
        off2[b] = cnt2[b] = 0;
        return;
    }
    const uint32_t w = b / nbk, o = off[b];
    const uint64_t v0 = a.vbase[w] + (o - (uint64_t)w * a.n), v1 = v0 + c - 1;
    const uint32_t s = pref[v0], e = pref[v1] + ((vals[o + c - 1] & A_MARK) ? 1u : 0u);
    off2[b] = s;
    cnt2[b] = e - s;
}

}  // namespace

// src: a marked split plan (msm_prepare_impl with amark) of nreal_src = src.nreal scalars; rank_bits = (bits, prefix)
// per 32 variables (Circuit::a_bits): the destination point of marked variable v is dst_base + its rank.  The derived plan (pl) is a split plan of nreal_dst
// points: entry point j < nreal_src -> dst_base + rank[j], j >= nreal_src -> nreal_dst + dst_base + rank[j -
// nreal_src].  src's arrays must still be valid (no prepare on their ctx since); false: no marked entry.
inline bool msm_derive_plan_impl(Ctx &c, const MsmPlan &src, const uint32_t *rank_bits, uint64_t nreal_dst,
                                 uint32_t dst_base, MsmPlan &pl) {
    pl = MsmPlan();
    if (!src.total) return false;
    if (!src.marked || !src.nreal || src.nwin > MAXW_S || 2 * (nreal_dst + dst_base) >= A_MARK)
        throw std::logic_error("msm_derive_plan: the source is not a marked split plan");
    PlanStream plan_stream(c);
    hipStream_t st = c.stream;
    DeriveArgs a{};
    a.n = src.n;
    a.nwin = src.nwin;
    a.nreal_src = (uint32_t)src.nreal;
    a.nreal_dst = (uint32_t)nreal_dst;
    a.dst_base = dst_base;
    uint64_t ntiles = 0, ent = 0;
    for (unsigned w = 0; w < src.nwin; w++) {
        a.wn[w] = src.wn[w];
        a.tile0[w] = (uint32_t)ntiles;
        a.vbase[w] = (uint32_t)ent;
        ntiles += (src.wn[w] + DERIVE_T - 1) / DERIVE_T;
        ent += src.wn[w];
    }
    a.tile0[src.nwin] = (uint32_t)ntiles;
    a.vbase[src.nwin] = (uint32_t)ent;
    if (ent >= 0xffffffffull) throw std::runtime_error("msm_derive_plan: too many entries");
    pl.n = 2 * nreal_dst;
    pl.nreal = nreal_dst;
    pl.cb = src.cb;
    pl.nwin = src.nwin;
    pl.nbk = src.nbk;
    pl.nb = src.nb;
    pl.glv = src.glv;
    const uint32_t nb = src.nb;
    uint32_t *pref = c.scratch[0].as<uint32_t>(ent ? ent : 1);
    uint32_t *tile_cnt = c.scratch[1].as<uint32_t>(2 * (ntiles + 1)), *tile_base = tile_cnt + ntiles + 1;
    uint32_t *vals2 = c.scratch[26].as<uint32_t>(ent ? ent : 1);
    uint32_t *off2 = c.scratch[27].as<uint32_t>(nb), *cnt2 = c.scratch[28].as<uint32_t>(nb);
    uint32_t *coff2 = c.scratch[29].as<uint32_t>(nb), *ccnt2 = c.scratch[30].as<uint32_t>(nb);
    uint32_t *dmax = c.scratch[9].as<uint32_t>(4 + PLAN_PIN);  // [max bucket, marked entries, pad x 2, counts]
    {
        ScopedTimer tsort(c, &c.stats.sort, nreal_dst);
        MI_HIP(hipMemsetAsync(tile_cnt + ntiles, 0, 4, st));
        if (ntiles) {
            k_derive_count<<<(unsigned)ntiles, 256, 0, st>>>(src.vals_s, a, tile_cnt);
            MI_LAUNCHED(c, "k_derive_count");
        }
        size_t tb = 0;
        MI_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, tile_cnt, tile_base, ntiles + 1, st));
        void *tmp = c.scratch[4].get(tb);
        MI_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, tile_cnt, tile_base, ntiles + 1, st));
        if (ntiles) {
            k_derive_scatter<<<(unsigned)ntiles, 256, 0, st>>>(src.vals_s, reinterpret_cast<const uint2 *>(rank_bits), a,
                                                               tile_base, vals2, pref);
            MI_LAUNCHED(c, "k_derive_scatter");
        }
        k_derive_bounds<<<grid_for(nb, 256), 256, 0, st>>>(src.off, src.cnt, nb, src.nbk, src.vals_s, a, pref, off2,
                                                           cnt2);
        MI_LAUNCHED(c, "k_derive_bounds");
        tb = 0;
        MI_HIP(hipcub::DeviceReduce::Max(nullptr, tb, cnt2, dmax, nb, st));
        tmp = c.scratch[4].get(tb);
        MI_HIP(hipcub::DeviceReduce::Max(tmp, tb, cnt2, dmax, nb, st));
        MI_HIP(hipMemcpyAsync(dmax + 1, tile_base + ntiles, 4, hipMemcpyDeviceToDevice, st));
    }
    uint32_t *pin = c.pin.as<uint32_t>(4 + PLAN_PIN);
    plan_counts(c, pl, cnt2, coff2, ccnt2, nb, dmax, dmax + 4, DERIVED_SLOTS);
    MI_HIP(hipMemcpyAsync(pin, dmax, sizeof(uint32_t) * (4 + PLAN_PIN), hipMemcpyDeviceToHost, st));
    MI_HIP(hipStreamSynchronize(st));
    pl.maxcnt = pin[0];
    pl.entries = pin[1];
    return plan_finish(c, pl, off2, cnt2, nb, vals2, pin + 4, DERIVED_SLOTS);
}

// tune::MSM_BITSUM = 0 sends one-window plans through reduce_windows (A/B, tests)
inline bool bitsum_enabled() { return tune::get(tune::MSM_BITSUM, 1) != 0; }

// Window-table plan (msm_run_wt): nscal scalars, nwin windows of cb bits, over the table whose window w starts at
// point w * stride (relative to the bases pointer the accumulation gets).  Every window's digits share one set of
// 2^(cb - 1) buckets, so the plan has ONE window (pl.nwin = 1) of nwin * nscal entries.
// sparse: the scalars are mostly zero digits (a witness): compact the non-zero ones first (one more readback, the
// entry count), so the sort runs over the entries only
inline bool msm_prepare_wt_impl(Ctx &c, const fr_t *scalars, const uint32_t *idx, uint64_t nscal, unsigned cb,
                                unsigned nwin, uint64_t stride, MsmPlan &pl, bool sparse = false) {
    pl = MsmPlan();
    if (nscal == 0) return false;
    PlanStream plan_stream(c);
    const uint64_t np64 = (uint64_t)nwin * nscal;
    if (np64 >= 0xffffffffull || (uint64_t)nwin * stride >= A_MARK || cb < 2 || cb > 24)
        throw std::runtime_error("msm: window-table instance too large for 32-bit sort indices");
    hipStream_t st = c.stream;
    const uint32_t nbk = 1u << (cb - 1), invalid = nbk;
    uint32_t np = (uint32_t)np64;
    pl.cb = cb;
    pl.nwin = 1;
    pl.nbk = nbk;
    pl.nb = nbk;
    uint32_t *keys = c.scratch[0].as<uint32_t>(np), *vals = c.scratch[1].as<uint32_t>(np);
    uint32_t *keys_s = c.scratch[2].as<uint32_t>(np), *vals_s = c.scratch[3].as<uint32_t>(np);
    uint32_t *offA = c.scratch[5].as<uint32_t>(nbk), *cntA = c.scratch[6].as<uint32_t>(nbk);
    uint32_t *offB = c.scratch[7].as<uint32_t>(nbk), *cntB = c.scratch[8].as<uint32_t>(nbk);
    uint32_t *dmax = c.scratch[9].as<uint32_t>(8 + PLAN_PIN), *zstart = dmax + 4;  // [max, pad x 3, zstart, pad x 3, counts]
    {
        ScopedTimer tsort(c, &c.stats.sort, nscal);
        if (sparse) {
            uint32_t *cnt_dev = dmax + 7;
            MI_HIP(hipMemsetAsync(cnt_dev, 0, 4, st));
            k_digits_wt_c<<<grid_for(nscal, DIGITS_BLOCK), DIGITS_BLOCK, 0, st>>>(scalars, idx, (uint32_t)nscal, cb, nwin,
                                                                (uint32_t)stride, cnt_dev, keys, vals);
            MI_LAUNCHED(c, "k_digits_wt_c");
            uint32_t *pc = c.pin.as<uint32_t>(1);
            MI_HIP(hipMemcpyAsync(pc, cnt_dev, 4, hipMemcpyDeviceToHost, st));
            MI_HIP(hipStreamSynchronize(st));
            np = *pc;
            if (np == 0) return false;  // every scalar is zero
        } else {
            k_digits_wt<<<grid_for(nscal, 256), 256, 0, st>>>(scalars, idx, (uint32_t)nscal, cb, nwin, (uint32_t)stride,
                                                              invalid, keys, vals);
            MI_LAUNCHED(c, "k_digits_wt");
        }
        pl.n = np;
        size_t tmp_bytes = 0;
        sort_pairs_u32(nullptr, tmp_bytes, keys, keys_s, vals, vals_s, np, cb, st);
        void *tmp = c.scratch[4].get(tmp_bytes);
        sort_pairs_u32(tmp, tmp_bytes, keys, keys_s, vals, vals_s, np, cb, st);
        k_plan_init<<<grid_for(nbk, 256), 256, 0, st>>>(offA, cntA, nbk, zstart, 1);
        MI_LAUNCHED(c, "k_plan_init");
        k_bounds4<<<grid_for((np + 3) / 4, 256), 256, 0, st>>>(keys_s, np, np, nbk, 0, nullptr, offA, cntA, zstart);
        MI_LAUNCHED(c, "k_bounds4");
        k_end_to_cnt<<<grid_for(nbk, 256), 256, 0, st>>>(offA, cntA, nbk);
        MI_LAUNCHED(c, "k_end_to_cnt");
        size_t tb = 0;
        MI_HIP(hipcub::DeviceReduce::Max(nullptr, tb, cntA, dmax, nbk, st));
        tmp = c.scratch[4].get(tb);
        MI_HIP(hipcub::DeviceReduce::Max(tmp, tb, cntA, dmax, nbk, st));
    }
    uint32_t *pin = c.pin.as<uint32_t>(8 + PLAN_PIN);  // one readback: bucket maximum, zero-digit start, plan counts
    plan_counts(c, pl, cntA, offB, cntB, nbk, dmax, dmax + 8);
    MI_HIP(hipMemcpyAsync(pin, dmax, sizeof(uint32_t) * (8 + PLAN_PIN), hipMemcpyDeviceToHost, st));
    MI_HIP(hipStreamSynchronize(st));
    pl.maxcnt = pin[0];
    pl.entries = pin[4] == 0xffffffffu ? np : pin[4];
    return plan_finish(c, pl, offA, cntA, nbk, vals_s, pin + 8);
}

// ---- phase 2 (per base set): accumulation, chunk tree, bucket reduction, window combination ----
// Level-0 accumulation of the plan's chunks over `bases` and the in-place chunk tree: bucket b's sum
// ends up in P0[coff[b]] (when cnt[b] != 0).  Returns P0 (scratch slot 10).
template <class F>
XYZZ<F> *accumulate_chunks(Ctx &c, const MsmPlan &pl, const Affine<F> *bases, const Affine<F> *bases_hi = nullptr) {
    if (pl.nreal && !bases_hi) throw std::logic_error("msm: split plan without the 2^128 base table");
    hipStream_t st = c.stream;
    const unsigned K = Lane<F>::K;      // threads per element in the accumulation (2 for G2: g2pair.h)
    const unsigned KR = LaneRed<F>::K;  // ... and in the reduction kernels
    const unsigned cb = pl.cb, nwin = pl.nwin;
    const uint32_t nbk = pl.nbk, nb = pl.nb, L0 = pl.L0;
    const uint32_t *coff = pl.coff, *ccnt = pl.ccnt, *offA = pl.off, *cntA = pl.cnt;
    XYZZ<F> *P0 = c.scratch[10].as<XYZZ<F>>(pl.total);
    (sizeof(F) == sizeof(fq_t) ? c.stats.madds_g1 : c.stats.madds_g2) += pl.entries;
    {
        // units = input points (the split plan's 2n half-scalar points are n of them)
        ScopedTimer tacc(c, sizeof(F) == sizeof(fq_t) ? &c.stats.accum_g1 : &c.stats.accum_g2,
                         pl.nreal ? pl.nreal : pl.n);
        k_accum_level0<F><<<grid_for((uint64_t)pl.total * K, 256), 256, 0, st>>>(pl.order, pl.chunk_bucket, coff, offA, cntA,
                                                                    pl.total, L0, pl.vals_s, bases, bases_hi,
                                                                    pl.nreal ? (uint32_t)pl.nreal : 0xffffffffu, P0);
        MI_LAUNCHED(c, "k_accum_level0");
    }

    const uint32_t maxchunks = (pl.maxcnt + L0 - 1) / L0;
    if (maxchunks > 1) {  // in-place strided tree over the chunk partials of multi-chunk buckets only
        const uint32_t m = pl.m, *mlist = pl.mlist, L1 = pl.L1;
        unsigned level = 0;
        for (uint64_t stride = 1; stride < maxchunks; stride *= L1, level++) {
            // the first level's quotas were counted with the plan; deeper levels (buckets of more than L0 L1
            // entries) are counted here, into this accumulation's own scratch (a plan serves B_G1 and B_G2 alike,
            // so its arrays stay as they are); every level's partial count came with the plan's readback
            uint32_t total = pl.l1_total, *qcnt = pl.qcnt, *qoff = pl.qoff;
            if (stride > 1) {
                qcnt = c.scratch[2].as<uint32_t>(m);
                qoff = c.scratch[11].as<uint32_t>(m);
                k_tree_count<<<grid_for(m, 256), 256, 0, st>>>(mlist, ccnt, m, (uint32_t)stride, L1, qcnt);
                MI_LAUNCHED(c, "k_tree_count");
                size_t tb = 0;
                MI_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, qcnt, qoff, m, st));
                void *tmp = c.scratch[4].get(tb);
                MI_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, qcnt, qoff, m, st));
                if (level < TREE_MAXL) {
                    total = pl.level_total[level];
                } else {  // beyond the counted levels (L1 = 4 and > 4^16 chunks in one bucket): read it back
                    uint32_t *tail = c.pin.as<uint32_t>(2);
                    MI_HIP(hipMemcpyAsync(&tail[0], qoff + m - 1, 4, hipMemcpyDeviceToHost, st));
                    MI_HIP(hipMemcpyAsync(&tail[1], qcnt + m - 1, 4, hipMemcpyDeviceToHost, st));
                    MI_HIP(hipStreamSynchronize(st));
                    total = tail[0] + tail[1];
                }
            }
            k_tree_level<F><<<grid_for((uint64_t)total * KR, 256), 256, 0, st>>>(qoff, m, mlist, coff, ccnt, total,
                                                                   (uint32_t)stride, L1, P0);
            MI_LAUNCHED(c, "k_tree_level");
        }
    }
    return P0;
}

// Bucket reduction of every window of the plan: W[w] = sum_b (b + 1) B_{w,b} (window-local b).
template <class F>
void reduce_windows(Ctx &c, const MsmPlan &pl, XYZZ<F> *P0, std::vector<XYZZ<F>> &W) {
    hipStream_t st = c.stream;
    const unsigned KR = LaneRed<F>::K;  // threads per element in the reduction kernels
    const unsigned nwin = pl.nwin;
    const uint32_t nbk = pl.nbk, nb = pl.nb;
    const uint32_t *coff = pl.coff, *cntA = pl.cnt;
    // Bucket reduction, two running-sum levels (no per-segment scalar multiplication on the big level):
    //   W = sum_b (b+1) B_b,  b = s*S + j:  W = sum_s accA_s + S * (V - R),
    //   accA_s = sum_j (j+1) B_{sS+j},  runA_s = sum_j B_{sS+j},  R = sum_s runA_s,  V = sum_s (s+1) runA_s,
    // V by a second running-sum level over runA (segments of SB) whose few segment offsets are folded
    // by double-and-add (k_seg_fold).
    // first-level segment count target (threads of k_bucket_reduce); tune::MSM_SEGA_LOG overrides (tuning)
    const int64_t sega_env = tune::get(tune::MSM_SEGA_LOG, 0);
    // small MSMs (<= 2^20 buckets in all) aim at 2^17 first-level segments: 4 buckets per running sum instead of 1
    // leaves the second level a quarter of the segments (Winning PoSt: 20.8-21.8 -> 20.1-20.2 ms, same box,
    // tools/gpu_round4_r.sh at 78a06f8)
    const uint64_t segA_target = sega_env > 0 && sega_env < 40 ? (1ull << sega_env)
                                 : nb <= (1u << 20)           ? (1u << 17)
                                 : sizeof(F) == sizeof(fq_t)  ? (1u << 20)
                                                              : (1u << 18);
    unsigned SA = 1;
    while (SA < nbk && (uint64_t)nb / (SA * 2) >= segA_target) SA *= 2;
    const uint32_t nsegA = nbk / SA, totA = nwin * nsegA;
    // second-level segments per window: 8192 for large MSMs.  Small ones (<= 2^19 first-level segments in all,
    // Winning PoSt's 2^18-2^19-point MSMs) take 2048: k_seg_fold's double-and-add over ~14-bit offsets per
    // segment was the largest reduction kernel there (thousands of full additions per window for a weighted
    // sum the running sums of k_bucket_reduce_dense do with 2 per segment).  tune::MSM_SEGB_LOG = k forces 2^k.
    const int64_t segb_env = tune::get(tune::MSM_SEGB_LOG, 0);
    const uint32_t segB_cap = segb_env > 0 ? (1u << (segb_env > 13 ? 13 : segb_env))
                                           : totA <= (1u << 19) ? 2048u : 8192u;
    const uint32_t nsegB = nsegA < segB_cap ? nsegA : segB_cap, SB = nsegA / nsegB, totB = nwin * nsegB;
    XYZZ<F> *accA = c.scratch[12].as<XYZZ<F>>(2 * (uint64_t)totA), *runA = accA + totA;
    // [sumAccB | runB | foldB] contiguous (one stacked tree sum over 3 * nwin rows), then accB
    XYZZ<F> *sumB = c.scratch[14].as<XYZZ<F>>(4 * (uint64_t)totB), *runB = sumB + totB, *foldB = runB + totB,
            *accB = foldB + totB;
    k_bucket_reduce<F><<<grid_for((uint64_t)totA * KR, 256), 256, 0, st>>>(coff, cntA, P0, totA, SA, accA, runA);
    MI_LAUNCHED(c, "k_bucket_reduce");
    k_bucket_reduce_dense<F><<<grid_for((uint64_t)totB * KR, 256), 256, 0, st>>>(runA, accA, totB, SB, accB, runB, sumB);
    MI_LAUNCHED(c, "k_bucket_reduce_dense");
    k_seg_fold<F><<<grid_for((uint64_t)totB * KR, 256), 256, 0, st>>>(accB, runB, totB, nsegB, SB, foldB);
    MI_LAUNCHED(c, "k_seg_fold");
    // stacked per-row tree sum of nsegB (a power of two) entries, groups of <= 8 (shallow chains)
    const uint32_t rows = 3 * nwin;
    XYZZ<F> *tsum = c.scratch[11].as<XYZZ<F>>(2 * ((uint64_t)rows * nsegB / 2 + rows));
    XYZZ<F> *bufs[2] = {tsum, tsum + (uint64_t)rows * nsegB / 2 + rows};
    const XYZZ<F> *cur = sumB;
    int k = 0;
    for (uint32_t per = nsegB; per > 1;) {
        unsigned G = per >= 8 ? 8 : per;
        uint32_t outs = rows * (per / G);
        k_sum_groups<F><<<grid_for((uint64_t)outs * KR, 256), 256, 0, st>>>(cur, outs, G, bufs[k]);
        MI_LAUNCHED(c, "k_sum_groups");
        per /= G;
        cur = bufs[k];
        k ^= 1;
    }
    XYZZ<F> *sums_pin = c.pin.as<XYZZ<F>>(rows);
    MI_HIP(hipMemcpyAsync(sums_pin, cur, sizeof(XYZZ<F>) * rows, hipMemcpyDeviceToHost, st));
    MI_HIP(hipStreamSynchronize(st));
    std::vector<XYZZ<F>> sums(sums_pin, sums_pin + rows);
    W.assign(nwin, XYZZ<F>::inf());
    unsigned log_sa = 0;
    while ((1u << log_sa) < SA) log_sa++;
    for (unsigned w = 0; w < nwin; w++)  // W = SumA + SA * (V - R), in the host field (hostfield.h)
        W[w] = host::window_from_sums(sums[w], sums[nwin + w], sums[2 * nwin + w], log_sa);
}

// Bucket reduction of a plan with few windows (window-table plans: one) through k_bitsum_first / k_sum_lds; the host
// folds each window's rows: W = row0 + SA sum_k 2^k row(1 + k) (hostfield.h).
template <class F>
void reduce_bitsum(Ctx &c, const MsmPlan &pl, XYZZ<F> *P0, std::vector<XYZZ<F>> &W) {
    hipStream_t st = c.stream;
    const unsigned nwin = pl.nwin;
    const uint32_t nbk = pl.nbk;
    // first-level segments in all (threads of k_bucket_reduce): >= 2^tune::MSM_BS_SEG_LOG (default 2^16) while a
    // segment holds more than one bucket
    const int64_t bs_seg = tune::get(tune::MSM_BS_SEG_LOG, 16);
    const unsigned seg_log = bs_seg > 0 && bs_seg < 32 ? (unsigned)bs_seg : 16u;
    unsigned SA = 1, log_sa = 0;
    while (SA < nbk && (uint64_t)nbk * nwin / (SA * 2) >= (1ull << seg_log)) SA *= 2, log_sa++;
    const uint32_t nseg = nbk / SA, totA = nwin * nseg;
    unsigned lseg = 0;
    while ((1u << lseg) < nseg) lseg++;
    XYZZ<F> *accA = c.scratch[12].as<XYZZ<F>>(2 * (uint64_t)totA), *runA = accA + totA;
    const unsigned KR = LaneRed<F>::K;
    k_bucket_reduce<F><<<grid_for((uint64_t)totA * KR, 256), 256, 0, st>>>(pl.coff, pl.cnt, P0, totA, SA, accA, runA);
    MI_LAUNCHED(c, "k_bucket_reduce");
    // rows per window: the two halves of sum acc, then T_k; nseg / 2 items each.  Items per thread of the first
    // level: enough that <= 2^15 threads run it (the LDS tree passes after it are latency-bound: fewer, shallower
    // blocks; 2^20 over a c = 20 table, same box: 3.29 / 3.26 / 3.24 ms at 4 / 8 / 16 items), tune::MSM_BS_G0 overrides
    const uint32_t rows = nwin * (2 + lseg), half = nseg / 2 ? nseg / 2 : 1;
    const int64_t g0 = tune::get(tune::MSM_BS_G0, 0);
    unsigned G = 1;
    if (g0 > 0 && g0 <= 1024) {
        G = (unsigned)g0;
    } else {
        while ((uint64_t)rows * half / (G * 2) >= (1u << 15) && G < 64) G *= 2;
    }
    while (G > 1 && G > half) G /= 2;
    uint32_t per = nseg >= 2 ? half / G : 1;
    XYZZ<F> *bufs[2] = {c.scratch[11].as<XYZZ<F>>((uint64_t)rows * per), c.scratch[14].as<XYZZ<F>>((uint64_t)rows * per)};
    if (nseg >= 2) {
        k_bitsum_first<F><<<grid_for((uint64_t)rows * per * KR, 256), 256, 0, st>>>(accA, runA, nwin, nseg, lseg, G,
                                                                                 bufs[0]);
        MI_LAUNCHED(c, "k_bitsum_first");
    } else {  // one segment per window: its acc is row 0, row 1 the identity (all-zero coordinates), no bit rows
        MI_HIP(hipMemsetAsync(bufs[0], 0, sizeof(XYZZ<F>) * rows, st));
        for (unsigned w = 0; w < nwin; w++)
            MI_HIP(hipMemcpyAsync(bufs[0] + 2 * (uint64_t)w, accA + w, sizeof(XYZZ<F>), hipMemcpyDeviceToDevice, st));
    }
    int k = 0;
    while (per > 1) {
        const uint32_t m = per < 256 / KR ? per : 256 / KR;
        k_sum_lds<F><<<rows * (per / m), 256, 0, st>>>(bufs[k], m, bufs[k ^ 1]);
        MI_LAUNCHED(c, "k_sum_lds");
        per /= m;
        k ^= 1;
    }
    XYZZ<F> *sums_pin = c.pin.as<XYZZ<F>>(rows);
    MI_HIP(hipMemcpyAsync(sums_pin, bufs[k], sizeof(XYZZ<F>) * rows, hipMemcpyDeviceToHost, st));
    MI_HIP(hipStreamSynchronize(st));
    W.assign(nwin, XYZZ<F>::inf());
    for (unsigned w = 0; w < nwin; w++) {
        const XYZZ<F> *r = sums_pin + (uint64_t)w * (2 + lseg);
        const std::vector<XYZZ<F>> bits(r + 2, r + 2 + lseg);
        W[w] = host::xyzz_add(host::xyzz_add(r[0], r[1]), host::xyzz_dbl_n(host::combine_windows(bits, 1), log_sa));
    }
}

// G2 bucket reduction as a second-level MSM.  The lane-pair full addition (XYZZ + XYZZ) of the
// running-sum reduction needs more than 256 registers (every measured build either spills or runs one
// wave per SIMD), while the lane-pair MIXED addition runs at the accumulation's rate.  So for large
// G2 instances: bucket sums -> affine (batch inversion), then each window's sum_j (j + 1) B_j is a
// Pippenger over those affine points with the small scalars j + 1 split into two c2-bit digits
// (windows 2w, 2w + 1; about 2 mixed additions per bucket, ~2^c2 second-level buckets per window),
// and W_w = W'_{2w} + 2^c2 W'_{2w+1}.  Reuses the level-1 plan's scratch: the plan is consumed.
// tune::G2_L2 = 0 turns it off (the plain reduction), 2 forces it at any size (tests).
template <class F>
bool g2_second_level(Ctx &c, const MsmPlan &pl, XYZZ<F> *P0, std::vector<XYZZ<F>> &W) {
    if constexpr (sizeof(F) != sizeof(fq2_t)) {
        return false;
    } else {
        // tune::G2_L2: 0 off, 1 (default) from 2^20 level-1 buckets on, 2 always (tests)
        const int64_t mode = tune::get(tune::G2_L2, 1);
        if (mode == 0 || (mode == 1 && pl.nb < (1u << 20))) return false;
        hipStream_t st = c.stream;
        const unsigned nwin = pl.nwin, cb = pl.cb;
        const uint32_t nb = pl.nb;
        const unsigned c2 = (cb + 1) / 2;  // s = j + 1 <= 2^(cb - 1) < 2^(2 c2)
        const uint32_t nbk2 = 1u << c2, nwin2 = 2 * nwin, nb2 = nwin2 * nbk2, invalid2 = nb2;
        // 1. bucket sums -> affine
        Affine<F> *Baff = c.scratch[18].as<Affine<F>>(nb);
        F *pre = c.scratch[19].as<F>(nb);
        // tune::G2_AFF_K buckets per inversion (Montgomery's trick; A/B)
        const int64_t kaff = tune::get(tune::G2_AFF_K, 64);  // same-box: 538.2 (32) vs 535.8 (64) vs 536.1 (128) ms per proof
        if (kaff == 128)
            k_bucket_affine<F, 128><<<grid_for(((uint64_t)nb + 127) / 128, 256), 256, 0, st>>>(pl.coff, pl.cnt, P0, nb,
                                                                                             pre, Baff);
        else if (kaff == 64)
            k_bucket_affine<F, 64><<<grid_for(((uint64_t)nb + 63) / 64, 256), 256, 0, st>>>(pl.coff, pl.cnt, P0, nb,
                                                                                           pre, Baff);
        else
            k_bucket_affine<F, 32><<<grid_for(((uint64_t)nb + 31) / 32, 256), 256, 0, st>>>(pl.coff, pl.cnt, P0, nb,
                                                                                           pre, Baff);
        MI_LAUNCHED(c, "k_bucket_affine");
        // 2. two digit entries per non-empty bucket, one sort over all of them
        const uint32_t np2 = 2 * nb;
        uint32_t *keys = c.scratch[0].as<uint32_t>(np2), *vals = c.scratch[1].as<uint32_t>(np2);
        uint32_t *keys_s = c.scratch[2].as<uint32_t>(np2), *vals_s = c.scratch[3].as<uint32_t>(np2);
        k_l2_digits<<<grid_for(nb, 256), 256, 0, st>>>(pl.cnt, nb, cb - 1, c2, invalid2, keys, vals);
        MI_LAUNCHED(c, "k_l2_digits");
        unsigned bits = 1;
        while ((1ull << bits) <= invalid2) bits++;
        size_t tmp_bytes = 0;
        sort_pairs_u32(nullptr, tmp_bytes, keys, keys_s, vals, vals_s, np2, bits, st);
        void *tmp = c.scratch[4].get(tmp_bytes);
        sort_pairs_u32(tmp, tmp_bytes, keys, keys_s, vals, vals_s, np2, bits, st);
        // 3. buckets of the second level
        uint32_t *off2 = c.scratch[5].as<uint32_t>(nb2), *cnt2 = c.scratch[6].as<uint32_t>(nb2);
        k_plan_init<<<grid_for(nb2, 256), 256, 0, st>>>(off2, cnt2, nb2, nullptr, 0);
        MI_LAUNCHED(c, "k_plan_init");
        k_bounds_flat<<<grid_for(np2, 256), 256, 0, st>>>(keys_s, np2, invalid2, off2, cnt2);
        MI_LAUNCHED(c, "k_bounds_flat");
        k_end_to_cnt<<<grid_for(nb2, 256), 256, 0, st>>>(off2, cnt2, nb2);
        MI_LAUNCHED(c, "k_end_to_cnt");
        uint32_t *dm = c.scratch[9].as<uint32_t>(4 + PLAN_PIN);  // [max, sum, pad x 2, the plan's counts]
        uint32_t *head = c.pin.as<uint32_t>(4 + PLAN_PIN);
        tmp_bytes = 0;
        MI_HIP(hipcub::DeviceReduce::Max(nullptr, tmp_bytes, cnt2, dm, nb2, st));
        size_t tb2 = 0;
        MI_HIP(hipcub::DeviceReduce::Sum(nullptr, tb2, cnt2, dm + 1, nb2, st));
        tmp = c.scratch[4].get(tmp_bytes > tb2 ? tmp_bytes : tb2);
        MI_HIP(hipcub::DeviceReduce::Max(tmp, tmp_bytes, cnt2, dm, nb2, st));
        MI_HIP(hipcub::DeviceReduce::Sum(tmp, tb2, cnt2, dm + 1, nb2, st));
        MsmPlan p2;
        plan_counts(c, p2, cnt2, c.scratch[7].as<uint32_t>(nb2), c.scratch[8].as<uint32_t>(nb2), nb2, dm, dm + 4);
        MI_HIP(hipMemcpyAsync(head, dm, sizeof(uint32_t) * (4 + PLAN_PIN), hipMemcpyDeviceToHost, st));
        MI_HIP(hipStreamSynchronize(st));
        p2.n = head[1];
        p2.cb = c2;
        p2.nwin = nwin2;
        p2.nbk = nbk2;
        p2.nb = nb2;
        p2.maxcnt = head[0];
        p2.entries = head[1];
        W.assign(nwin, XYZZ<F>::inf());
        if (!plan_finish(c, p2, off2, cnt2, nb2, vals_s, head + 4)) return true;  // every bucket empty
        // 4. second-level accumulation over the affine buckets, reduction, recombination
        XYZZ<F> *Q0 = accumulate_chunks<F>(c, p2, Baff);
        std::vector<XYZZ<F>> W2;
        reduce_windows<F>(c, p2, Q0, W2);
        for (unsigned w = 0; w < nwin; w++) W[w] = host::xyzz_add(W2[2 * w], host::xyzz_dbl_n(W2[2 * w + 1], c2));
        return true;
    }
}

template <class F>
void msm_accumulate_impl(Ctx &c, const MsmPlan &pl, const Affine<F> *bases, XYZZ<F> *result,
                         const Affine<F> *bases_hi = nullptr) {
    // GLV plans gather the phi(P_i) half as P_i itself (bases doubles as the "hi" table)
    XYZZ<F> *P0 = accumulate_chunks<F>(c, pl, bases, pl.glv ? bases : bases_hi);
    std::vector<XYZZ<F>> W;
    if constexpr (sizeof(F) == sizeof(fq_t)) {
        if (pl.glv) {  // sub-bucket pairs -> bucket sums (k_glv_merge), then the plain reduction over them
            MsmPlan p2 = pl;
            p2.nbk = pl.nbk / 2;
            p2.nb = pl.nb / 2;
            XYZZ<F> *Bm = c.scratch[18].as<XYZZ<F>>(p2.nb);
            uint32_t *live = c.scratch[19].as<uint32_t>(2 * (uint64_t)p2.nb), *iota = live + p2.nb;
            static const fq_t beta = glv_beta();
            k_glv_merge<F><<<grid_for(p2.nb, 256), 256, 0, c.stream>>>(pl.coff, pl.cnt, P0, p2.nb, beta, Bm, live,
                                                                       iota);
            MI_LAUNCHED(c, "k_glv_merge");
            p2.coff = iota;
            p2.cnt = live;
            reduce_windows<F>(c, p2, Bm, W);
        } else if (pl.nwin <= 2 && bitsum_enabled()) {
            reduce_bitsum<F>(c, pl, P0, W);
        } else {
            reduce_windows<F>(c, pl, P0, W);
        }
    } else if (pl.nwin <= 2 && bitsum_enabled()) {
        reduce_bitsum<F>(c, pl, P0, W);
    } else {
        if (!g2_second_level<F>(c, pl, P0, W)) reduce_windows<F>(c, pl, P0, W);
    }
    *result = host::combine_windows(W, pl.cb);  // Horner over the windows in the host field (hostfield.h)
    c.timer.resolve();
}

// MSM over a window table (WinTable, ctx.h): points [lo, lo + n) of the table's base set
template <class F>
void msm_run_wt(Ctx &c, const WinTable &wt, uint64_t lo, const fr_t *scalars, const uint32_t *idx, uint64_t n,
                XYZZ<F> *result, bool sparse = false) {
    if (lo + n > wt.stride) throw std::invalid_argument("msm: range past the end of the window table");
    ScopedTimer whole(c, sizeof(F) == sizeof(fq_t) ? &c.stats.msm_g1 : &c.stats.msm_g2, n);
    MsmPlan pl;
    (sizeof(F) == sizeof(fq_t) ? c.stats.wt_msms : c.stats.wt_msms_g2) += 1;
    if (!msm_prepare_wt_impl(c, scalars, idx, n, wt.c, wt.nwin, wt.stride, pl, sparse)) {
        *result = XYZZ<F>::inf();
        return;
    }
    msm_accumulate_impl<F>(c, pl, reinterpret_cast<const Affine<F> *>(wt.p) + lo, result);
}

template <class F>
void msm_run(Ctx &c, const Affine<F> *bases, const fr_t *scalars, const uint32_t *idx, uint64_t n,
             XYZZ<F> *result, const Affine<F> *bases_hi = nullptr, bool subgroup = false) {
    ScopedTimer whole(c, sizeof(F) == sizeof(fq_t) ? &c.stats.msm_g1 : &c.stats.msm_g2, n);
    MsmPlan pl;
    // G1 split mode: the GLV endomorphism (no table) when tune::MSM_GLV selects it, else the 2^128 table.
    // phi(P) = lambda P holds only on the r-torsion, so auto mode takes GLV only for bases known to be in
    // the prime-order subgroup (generated / checked keys, mi_points_check_subgroup); other on-curve bases
    // run the plain path, which computes sum k_i P_i exactly like bellman's multiexp.
    const int glv_mode = msm_glv_mode();
    const bool glv = sizeof(F) == sizeof(fq_t) && msm_use_split(n) &&
                     (glv_mode == 1 || (glv_mode == 2 && !bases_hi && subgroup));
    const bool split = !glv && bases_hi && msm_use_split(n);
    if (!msm_prepare_impl(c, scalars, idx, n, pl, split, glv)) {
        *result = XYZZ<F>::inf();
        return;
    }
    msm_accumulate_impl<F>(c, pl, bases, result, split ? bases_hi : nullptr);
}

}  // namespace mi
