// g2pair.h -- G2 group law on lane pairs: an Fq2 coordinate split across two adjacent lanes.
//
// The G2 (Fq2) bucket kernels are register-bound: one XYZZ<Fq2> accumulator is 112 registers, and with
// the temporaries of a mixed addition the one-thread-per-chunk kernel needed all 256 VGPRs plus
// scratch spills (2 waves per SIMD at best).  Here lane 2k holds the c0 halves and lane 2k + 1 the c1
// halves of every Fq2 value of one chunk, so each lane carries Fq-sized state and the pair exchanges
// halves with one DPP quad_perm move per register:
//   mul: c0 = a0 b0 + a1 (-b1) (even lane), c1 = a0 b1 + a1 b0 (odd lane), each ONE fused
//        product-scanning Montgomery pass over two products: 2 x 507 lane-MADs, fewer than a
//        3-multiplication Karatsuba on one lane (3 x 338);
//   sqr: c0 = (a0 + a1)(a0 - a1), c1 = 2 a1 a0: one Fq multiplication per lane;
//   add / sub / neg: component-wise, no exchange;  is_zero: both halves (one exchanged flag).
// Every branch of the group law depends only on pair-combined predicates, so both lanes of a pair
// always take the same path (the DPP partner is active).
#pragma once
#include "curve.h"

namespace mi {

__device__ __forceinline__ uint32_t pair_swap(uint32_t x) {
    // quad_perm [1, 0, 3, 2]: exchange with the adjacent lane
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ fq_t pair_swap(const fq_t &a) {
    fq_t r;
    MI_UNROLL for (int i = 0; i < fq_t::L; i++) r.v[i] = pair_swap(a.v[i]);
    return r;
}
__device__ __forceinline__ bool pair_odd() { return threadIdx.x & 1; }

struct fq2h_t {
    fq_t v;  // c0 on even lanes, c1 on odd lanes
    __device__ static fq2h_t zero() { return {fq_t::zero()}; }
    __device__ static fq2h_t one() { return {pair_odd() ? fq_t::zero() : fq_t::one()}; }
    __device__ bool is_zero() const {
        uint32_t z = v.is_zero() ? 1u : 0u;
        return (z & pair_swap(z)) != 0;
    }
};
__device__ __forceinline__ fq2h_t operator+(const fq2h_t &a, const fq2h_t &b) { return {a.v + b.v}; }
__device__ __forceinline__ fq2h_t operator-(const fq2h_t &a, const fq2h_t &b) { return {a.v - b.v}; }
__device__ __forceinline__ fq2h_t operator-(const fq2h_t &a) { return {-a.v}; }
__device__ __forceinline__ fq2h_t dbl(const fq2h_t &a) { return {a.v + a.v}; }
__device__ __forceinline__ fq2h_t operator*(const fq2h_t &a, const fq2h_t &b) {
    // even: a0 b0 + a1 (-b1)     odd: a0 b1 + a1 b0
    // The odd lane sends -b1 instead of b1 (sender-side negation, limb-wise with signed limbs), so the
    // received halves are pa = a_partner, psb = (odd ? b0 : -b1) and both lanes run mul_add(X1, b, X3, psb)
    // with (X1, X3) = (a, pa) on even lanes and (pa, a) on odd lanes: one fused REDC (field.h mul_add).
    __builtin_amdgcn_sched_barrier(0);  // one pair multiplication at a time (register pressure)
    const bool odd = pair_odd();
    const fq_t nb = -b.v;
    fq_t sb;
    MI_UNROLL for (int i = 0; i < fq_t::L; i++) sb.v[i] = odd ? nb.v[i] : b.v.v[i];
    const fq_t pa = pair_swap(a.v), psb = pair_swap(sb);
    fq_t x1, x3;
    MI_UNROLL for (int i = 0; i < fq_t::L; i++) {
        x1.v[i] = odd ? pa.v[i] : a.v.v[i];
        x3.v[i] = odd ? a.v.v[i] : pa.v[i];
    }
    fq2h_t r = {mul_add(x1, b.v, x3, psb)};
    __builtin_amdgcn_sched_barrier(0);
    return r;
}
__device__ __forceinline__ fq2h_t sqr(const fq2h_t &a) {
    // even: (a0 + a1)(a0 - a1)     odd: (a1 + a1) a0
    const bool odd = pair_odd();
    const fq_t pa = pair_swap(a.v);
    fq_t x = a.v + (odd ? a.v : pa);
    fq_t y = odd ? pa : a.v - pa;
    return {x * y};
}
__device__ __forceinline__ fq2h_t mul_add(const fq2h_t &a, const fq2h_t &b, const fq2h_t &c, const fq2h_t &d) {
    return a * b + c * d;
}

// Per-thread view of the coordinates of group elements stored as XYZZ<F> / Affine<F>.
template <class F>
struct Lane;
template <>
struct Lane<fq_t> {  // G1: one thread per element
    static constexpr unsigned K = 1;
    using R = fq_t;
    __device__ static XYZZ<R> ld(const XYZZ<fq_t> *p) { return *p; }
    __device__ static void st(XYZZ<fq_t> *p, const XYZZ<R> &v) { *p = v; }
    __device__ static Affine<R> lda(const Affine<fq_t> *p) { return *p; }
};
template <>
struct Lane<fq2_t> {  // G2: a lane pair per element, this lane's Fq half of every coordinate
    static constexpr unsigned K = 2;
    using R = fq2h_t;
    __device__ static XYZZ<R> ld(const XYZZ<fq2_t> *p) {
        const fq_t *f = reinterpret_cast<const fq_t *>(p) + (threadIdx.x & 1);
        return {{f[0]}, {f[2]}, {f[4]}, {f[6]}};
    }
    __device__ static void st(XYZZ<fq2_t> *p, const XYZZ<R> &v) {
        fq_t *f = reinterpret_cast<fq_t *>(p) + (threadIdx.x & 1);
        f[0] = v.X.v;
        f[2] = v.Y.v;
        f[4] = v.ZZ.v;
        f[6] = v.ZZZ.v;
    }
    __device__ static Affine<R> lda(const Affine<fq2_t> *p) {
        const fq_t *f = reinterpret_cast<const fq_t *>(p) + (threadIdx.x & 1);
        return {{f[0]}, {f[2]}};
    }
};

// Bucket-reduction kernels (full XYZZ + XYZZ additions, two or three live accumulators) use the same
// lane pairs.  A one-thread-per-G2-element reduction variant existed in round 1 for an A/B; built without
// the two-wave cap it took all 512 unified registers and returned a wrong G2 sum at n = 1 on the GPU
// (tools/g2_variants.sh variant C), while the identical group-law code compiled for the host is correct
// under ASan/UBSan against the oracle (tests/test_cpu_grouplaw.py, G2 sequences).  The fault is in that
// AGPR-heavy device build, not in the arithmetic; the variant lost the A/B anyway, so it was removed.
template <class F>
struct LaneRed : Lane<F> {};

}  // namespace mi
