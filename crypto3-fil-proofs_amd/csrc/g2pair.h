// g2pair.h -- G2 group law on lane pairs: an Fq2 coordinate split across two adjacent lanes.
//
// The G2 (Fq2) bucket kernels are register-bound: one XYZZ<Fq2> accumulator is 112 registers, and with
// the temporaries of a mixed addition the one-thread-per-chunk kernel needed all 256 VGPRs plus
// scratch spills (2 waves per SIMD at best).  Here lane 2k holds the c0 halves and lane 2k + 1 the c1
// halves of every Fq2 value of one chunk, so each lane carries Fq-sized state and the pair exchanges
// halves with one DPP quad_perm move per register:
//   mul: c0 = a0 b0 + a1 (2p - b1) (even lane), c1 = a1 b0 + a0 b1 (odd lane), each ONE fused
//        product-scanning Montgomery pass over two products: 2 x 588 lane-MADs, the same MAD count
//        as a 3-multiplication Karatsuba on one lane;
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
    MI_UNROLL for (int i = 0; i < 14; i++) r.v[i] = pair_swap(a.v[i]);
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
    const bool odd = pair_odd();
    const fq_t pa = pair_swap(a.v), pb = pair_swap(b.v);
    // even: a0 b0 + a1 (2p - b1)     odd: a1 b0 + a0 b1   (pa, pb = the partner's halves); both
    // are one unsigned fused REDC (field.h mul_add: column sums < 2^63.4, result < 2p)
    const fq_t npb = -pb;
    fq_t y1, y2;
    MI_UNROLL for (int i = 0; i < 14; i++) {
        y1.v[i] = odd ? pb.v[i] : b.v.v[i];
        y2.v[i] = odd ? b.v.v[i] : npb.v[i];
    }
    return {mul_add(a.v, y1, pa, y2)};
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

}  // namespace mi
