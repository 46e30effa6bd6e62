// ntt.hip -- radix-2 NTT over the BLS12-381 scalar field for CDNA4.
//
// Restates crypto3's evaluation_domain / basic_radix2_domain ([NOT IN TREE]: libs/crypto/math,
// SURVEY.md §8a row a6) with bellman's conventions: omega_n = ROOT_OF_UNITY^(2^(32 - log n)),
// ROOT_OF_UNITY = 7^((r-1)/2^32), coset generator 7.
//
// Structure (Bailey / four-step, no transposes):
//   DIF (natural in -> bit-reversed out) is a sequence of passes.  Pass p works on contiguous
//   sub-problems of size 2^M; inside one, element i = i1 * S + i2 (S = 2^(M-b)).  A workgroup
//   loads a [2^b x T] tile (T consecutive i2 -> T*32-byte contiguous rows) into LDS, runs b
//   radix-2 DIF stages there with twiddles omega_{2^b}^j, multiplies each element by the
//   inter-pass twiddle omega_{2^M}^(i2 * bitrev_b(i1)) and writes the tile back in place.
//   DIT (bit-reversed in -> natural out) is the exact transpose: passes in reverse order,
//   twiddle first, then the transposed butterflies (u + w v, u - w v) in reverse stage order.
// Every twiddle is omega_{2^32}^e = LO[e & 0xffff] * HI[e >> 16] from two 2 MiB tables, so
// one pair of tables serves all domain sizes up to 2^32; in-tile twiddles need HI only.
// Each pass moves the vector through HBM once (read + write): 3 passes at 2^26.
// Inside a pass elements live in 9 x 29-bit limbs (fr29.h, same Montgomery radix as fr_t) in registers
// and in the LDS tile: products need no limb conversion and no final subtraction, butterfly sums and
// differences are lazy and each radix-4 output is brought back below 2r by at most two conditional
// subtractions; HBM keeps the canonical 8 x 32-bit image (< r).
#include "ctx.h"
#include "fr29.h"

namespace mi {

namespace {

constexpr unsigned TILE_LOG = 10;  // 1024 elements = 32 KiB of LDS per workgroup
constexpr unsigned TILE = 1u << TILE_LOG;
constexpr unsigned NTT_THREADS = 256;
// Occupancy target of the pass kernel (waves per SIMD).  LDS (36 KB per 1024-element tile) allows 4
// workgroups = 4 waves per SIMD; the register count decides whether they fit (<= 128 VGPRs).
#ifndef MI_NTT_WAVES
#define MI_NTT_WAVES 0
#endif
#if MI_NTT_WAVES
#define MI_NTT_OCC __attribute__((amdgpu_waves_per_eu(MI_NTT_WAVES)))
#else
#define MI_NTT_OCC
#endif

__device__ __forceinline__ fr_t tw_full(const fr_t *__restrict__ lo, const fr_t *__restrict__ hi, uint32_t e) {
    uint32_t l = e & 0xffffu, h = e >> 16;
    if (l == 0) return hi[h];
    if (h == 0) return lo[l];
    return lo[l] * hi[h];
}

// the same twiddle in 9 x 29-bit limbs (< 2r)
__device__ __forceinline__ fr29_t tw29(const fr29_t *__restrict__ lo, const fr29_t *__restrict__ hi, uint32_t e) {
    uint32_t l = e & 0xffffu, h = e >> 16;
    if (l == 0) return hi[h];
    if (h == 0) return lo[l];
    return fr29_mul(lo[l], hi[h]);
}

__device__ __forceinline__ uint32_t brev(uint32_t x, unsigned bits) {
    return bits ? (__builtin_bitreverse32(x) >> (32 - bits)) : 0;
}

// LDS tile: four planes of 64-bit words (limb pairs) so every access is a ds_read/write_b64 by
// 32-lane groups; positions are XOR-swizzled inside 32-word rows (worst case 2-way bank conflicts
// for every radix-4 access pattern and conflict-free for the contiguous load/store phases).
struct LdsTile {
    uint64_t p[4][TILE];  // limbs (0,1) (2,3) (4,5) (6,7)
    uint32_t q[TILE];     // limb 8
};
__device__ __forceinline__ unsigned swz(unsigned p) { return p ^ (((p >> 5) * 5u) & 31u); }
__device__ __forceinline__ void lds_put(LdsTile &s, unsigned p, const fr29_t &x) {
    const unsigned q = swz(p);
    MI_UNROLL for (int k = 0; k < 4; k++) s.p[k][q] = (uint64_t)x.v[2 * k] | ((uint64_t)x.v[2 * k + 1] << 32);
    s.q[q] = x.v[8];
}
__device__ __forceinline__ fr29_t lds_get(const LdsTile &s, unsigned p) {
    const unsigned q = swz(p);
    fr29_t x;
    MI_UNROLL for (int k = 0; k < 4; k++) {
        uint64_t w = s.p[k][q];
        x.v[2 * k] = (uint32_t)w;
        x.v[2 * k + 1] = (uint32_t)(w >> 32);
    }
    x.v[8] = s.q[q];
    return x;
}
// 4r in 29-bit limbs (2r is R2X29, r is FrDesc::MOD29)
constexpr uint32_t R4X29[9] = {0x00000004u, 0x1fffffe0u, 0x1e5bfeffu, 0x0d2017ffu, 0x160154efu,
                               0x10101343u, 0x1483339du, 0x0994cebeu, 0x01cfb69du};
// v < 8r -> v < 2r
__device__ __forceinline__ fr29_t red8(const fr29_t &v) { return fr29_sub_if_ge(fr29_sub_if_ge(v, R4X29), R2X29); }
__device__ __forceinline__ fr29_t red4(const fr29_t &v) { return fr29_sub_if_ge(v, R2X29); }  // v < 4r -> < 2r
__device__ __forceinline__ fr29_t f29(const fr_t &x) { return fr29_from_fr(x); }
// value < 2r -> canonical 8 x 32-bit image (< r)
__device__ __forceinline__ fr_t to_fr(const fr29_t &x) { return fr_from_fr29(fr29_sub_if_ge(x, FrDesc::MOD29)); }
// insert zero bits at positions p0 < p1 (p1 = p0 + 1 here) / at position p
__device__ __forceinline__ unsigned ins2(unsigned q, unsigned p0) {
    return (q & ((1u << p0) - 1)) | ((q >> p0) << (p0 + 2));
}
__device__ __forceinline__ unsigned ins1(unsigned q, unsigned p) {
    return (q & ((1u << p) - 1)) | ((q >> p) << (p + 1));
}
// In-tile twiddle omega_{2^b}^j = tw[j << sh], sh = TILE_LOG - b, from the 512-entry omega_1024 table kept
// in 29-bit limbs (no conversion in the rounds).  (An LDS copy of the table measured 11.8 vs 11.7 ms per
// 2^26 transform in round 1 and was dropped.)
__device__ __forceinline__ fr29_t tw_b(const fr29_t *__restrict__ tw, unsigned j, unsigned sh) { return tw[j << sh]; }

// The b stages of one tile: radix-4 register rounds (two stages per LDS round trip) plus one
// radix-2 round when b is odd.  DIF runs rounds in order, DIT the transpose in reverse order.
template <bool DIF>
__device__ __forceinline__ void ntt_rounds(LdsTile &sh, unsigned b, unsigned Tlog, unsigned tile,
                                           const fr29_t *__restrict__ tw10, unsigned tsh) {
    const unsigned T = 1u << Tlog;
    const unsigned nquad = tile >> 2;
    const unsigned nr4 = b >> 1;  // radix-4 rounds: DIF stage pairs (0,1), (2,3), ...
    const bool odd = b & 1;       // + one radix-2 round for stage b - 1
    const unsigned q = threadIdx.x;
    const unsigned bmask = (1u << b) - 1;
    for (unsigned rr = 0; rr < nr4 + (odd ? 1 : 0); rr++) {
        // DIF runs rounds in order; DIT runs them in reverse (the radix-2 round first when b is odd)
        const unsigned r = DIF ? rr : nr4 + (odd ? 1 : 0) - 1 - rr;
        const unsigned s = 2 * r;  // first DIF stage of this round
        if (r < nr4) {
            if (q < nquad) {
                const unsigned hs = b - 1 - s;  // i1 bit of stage s; stage s + 1 uses bit hs - 1
                const unsigned p0 = Tlog + hs - 1;
                const unsigned base = ins2(q, p0);
                const unsigned o1 = 1u << p0, o2 = 2u << p0;
                const unsigned i1 = (base >> Tlog) & bmask;
                const unsigned h = 1u << hs;
                const unsigned j0 = (i1 & (h - 1)) << s;        // stage s, pair (x0, x2)
                const unsigned j1 = j0 + (1u << (b - 2));       // stage s, pair (x1, x3)
                const unsigned jq = (i1 & ((h >> 1) - 1)) << (s + 1);  // stage s + 1, both pairs
                // LDS values < 2r; sums / differences lazy (< 8r), products < 1.1r, outputs back below 2r
                fr29_t x0 = lds_get(sh, base), x1 = lds_get(sh, base + o1);
                fr29_t x2 = lds_get(sh, base + o2), x3 = lds_get(sh, base + o2 + o1);
                if (DIF) {
                    fr29_t a = fr29_add(x0, x2), c = fr29_sub_lazy(x0, x2, R2X29);
                    fr29_t bb = fr29_add(x1, x3), dd = fr29_sub_lazy(x1, x3, R2X29);
                    if (j0) c = fr29_mul(c, tw_b(tw10, j0, tsh));
                    dd = fr29_mul(dd, tw_b(tw10, j1, tsh));
                    x0 = red8(fr29_add(a, bb));
                    x1 = fr29_sub_lazy(a, bb, R4X29);
                    x2 = red8(fr29_add(c, dd));
                    x3 = fr29_sub_lazy(c, dd, R2X29);
                    if (jq) {
                        const fr29_t w = tw_b(tw10, jq, tsh);
                        x1 = fr29_mul(x1, w);
                        x3 = fr29_mul(x3, w);
                    } else {
                        x1 = red8(x1);
                        x3 = red8(x3);
                    }
                } else {
                    if (jq) {
                        const fr29_t w = tw_b(tw10, jq, tsh);
                        x1 = fr29_mul(x1, w);
                        x3 = fr29_mul(x3, w);
                    }
                    fr29_t a = fr29_add(x0, x1), bb = fr29_sub_lazy(x0, x1, R2X29);
                    fr29_t c = fr29_add(x2, x3), dd = fr29_sub_lazy(x2, x3, R2X29);
                    if (j0) c = fr29_mul(c, tw_b(tw10, j0, tsh));
                    dd = fr29_mul(dd, tw_b(tw10, j1, tsh));
                    x0 = red8(fr29_add(a, c));
                    x2 = red8(fr29_sub_lazy(a, c, R4X29));
                    x1 = red8(fr29_add(bb, dd));
                    x3 = red8(fr29_sub_lazy(bb, dd, R2X29));
                }
                lds_put(sh, base, x0);
                lds_put(sh, base + o1, x1);
                lds_put(sh, base + o2, x2);
                lds_put(sh, base + o2 + o1, x3);
            }
        } else {  // radix-2 round: DIF stage b - 1 (pairs at i1 bit 0, twiddle exponent 0)
            for (unsigned u = q; u < (tile >> 1); u += NTT_THREADS) {
                const unsigned base = ins1(u, Tlog);
                const fr29_t x0 = lds_get(sh, base), x1 = lds_get(sh, base + T);
                lds_put(sh, base, red4(fr29_add(x0, x1)));
                lds_put(sh, base + T, red4(fr29_sub_lazy(x0, x1, R2X29)));
            }
        }
        __syncthreads();
    }
}

// One pass.  DIF: load -> b DIF stages -> optional inter-pass twiddle -> [epilogue] -> store.
//            DIT: load -> optional inter-pass twiddle -> b DIT stages (reverse) -> store.
// The b stages run as radix-4 rounds (two stages per LDS round trip: each thread holds the four
// elements x, x + h/2, x + h, x + 3h/2 of one group in registers) plus one radix-2 round when b is
// odd; in-tile twiddles omega_{2^b}^j come from the 512-entry omega_1024 table (L1-resident).
// Epilogue (last DIF pass only): epi = 1 multiplies the element at global position pos by
// G^bitrev_L(pos) * scale (coset shift of the bit-reversed coefficients, fused 1/d); epi = 2 also
// converts to canonical form (icoset: H for the MSM).
template <bool DIF, bool FUSED = false>
__global__ void __launch_bounds__(NTT_THREADS) MI_NTT_OCC k_ntt_pass(fr_t *__restrict__ d, unsigned L, unsigned M, unsigned b,
                                                          unsigned Tlog, unsigned Glog, int twiddle,
                                                          const fr29_t *__restrict__ lo,
                                                          const fr29_t *__restrict__ hi,
                                                          const fr29_t *__restrict__ tw10, int epi,
                                                          const fr29_t *__restrict__ glo,
                                                          const fr29_t *__restrict__ ghi, fr_t scale,
                                                          const fr29_t *__restrict__ tw10b = nullptr) {
    __shared__ LdsTile sh;
    const fr29_t *twA = tw10, *twB = tw10b;
    const unsigned tsh = TILE_LOG - b;
    const fr29_t sc29 = fr29_from_fr(scale);
    const unsigned T = 1u << Tlog;
    const unsigned Slog = M - b;
    const uint64_t S = 1ull << Slog;
    const unsigned tile_log = Glog + b + Tlog;
    const unsigned tile = 1u << tile_log;
    uint64_t sub0, i20;
    if (Glog > 0) {  // several whole sub-problems per workgroup (T == S)
        sub0 = (uint64_t)blockIdx.x << Glog;
        i20 = 0;
    } else {
        uint64_t blocks_per_sub = S >> Tlog;
        sub0 = blockIdx.x / blocks_per_sub;
        i20 = (blockIdx.x % blocks_per_sub) << Tlog;
    }
    const unsigned bmask = (1u << b) - 1;
    // load
    for (unsigned e = threadIdx.x; e < tile; e += NTT_THREADS) {
        unsigned t = e & (T - 1), i1 = (e >> Tlog) & bmask, g = e >> (Tlog + b);
        uint64_t gi = ((sub0 + g) << M) + ((uint64_t)i1 << Slog) + i20 + t;
        fr29_t x = f29(d[gi]);
        if (!DIF && twiddle) {
            uint32_t k1 = brev(i1, b);
            uint32_t ex = (uint32_t)(((uint64_t)(i20 + t) * k1) << (32 - M));
            if (ex) x = fr29_mul(x, tw29(lo, hi, ex));
        }
        lds_put(sh, e, x);
    }
    __syncthreads();
    ntt_rounds<DIF>(sh, b, Tlog, tile, twA, tsh);
    if (FUSED) {  // middle of iNTT -> coset -> NTT: epilogue in LDS, then the DIT rounds of the same tile
        for (unsigned e = threadIdx.x; e < tile; e += NTT_THREADS) {
            unsigned t = e & (T - 1), i1 = (e >> Tlog) & bmask, g = e >> (Tlog + b);
            uint64_t gi = ((sub0 + g) << M) + ((uint64_t)i1 << Slog) + i20 + t;
            fr29_t x = lds_get(sh, e);
            uint32_t ex = brev((uint32_t)gi, L);
            if (ex) x = fr29_mul(x, tw29(glo, ghi, ex));
            lds_put(sh, e, fr29_mul(x, sc29));
        }
        __syncthreads();
        ntt_rounds<false>(sh, b, Tlog, tile, twB, tsh);
    }
    // store
    for (unsigned e = threadIdx.x; e < tile; e += NTT_THREADS) {
        unsigned t = e & (T - 1), i1 = (e >> Tlog) & bmask, g = e >> (Tlog + b);
        uint64_t gi = ((sub0 + g) << M) + ((uint64_t)i1 << Slog) + i20 + t;
        fr29_t x = lds_get(sh, e);
        if (DIF && !FUSED && twiddle) {
            uint32_t k1 = brev(i1, b);
            uint32_t ex = (uint32_t)(((uint64_t)(i20 + t) * k1) << (32 - M));
            if (ex) x = fr29_mul(x, tw29(lo, hi, ex));
        }
        if (DIF && !FUSED && epi) {
            uint32_t ex = brev((uint32_t)gi, L);
            if (ex) x = fr29_mul(x, tw29(glo, ghi, ex));
            x = fr29_mul(x, sc29);
            if (epi == 2) {
                d[gi] = fr_from_fr29(fr29_from_mont(x));
                continue;
            }
        }
        d[gi] = to_fr(x);
    }
}

// The outermost pass of the QAP chain, fused (bellman's prover runs
// coset_fft(c), a = (a b - c) / Z, icoset_fft(a) as separate sweeps): the tile positions of the last DIT
// pass of c's coset transform are exactly those of the first DIF pass of H's inverse coset transform (pass
// 0 of the same plan), so one workgroup loads c's tile, finishes its coset NTT in LDS, reads a and b at
// the same positions (their coset evaluations are final), forms h = (a b - c) zinv, runs the first
// inverse-transform rounds and writes h over a.  One HBM sweep and the separate division pass fewer per
// proof; a is read before it is written by the same workgroup only.
__global__ void __launch_bounds__(NTT_THREADS) MI_NTT_OCC k_ntt_qap(fr_t *__restrict__ ha, const fr_t *__restrict__ bv,
                                                         const fr_t *__restrict__ cv, unsigned L, unsigned b,
                                                         unsigned Tlog, const fr29_t *__restrict__ flo,
                                                         const fr29_t *__restrict__ fhi,
                                                         const fr29_t *__restrict__ ftw10,
                                                         const fr29_t *__restrict__ ilo,
                                                         const fr29_t *__restrict__ ihi,
                                                         const fr29_t *__restrict__ itw10, fr_t zinv) {
    __shared__ LdsTile sh;
    const unsigned tsh = TILE_LOG - b;
    const fr29_t z29 = fr29_from_fr(zinv);
    const unsigned T = 1u << Tlog;
    const unsigned Slog = L - b;  // M = L: one sub-problem, Glog = 0 (plan_passes with two or more passes)
    const unsigned tile = 1u << (b + Tlog);
    const uint64_t i20 = (uint64_t)blockIdx.x << Tlog;
    const unsigned bmask = (1u << b) - 1;
    for (unsigned e = threadIdx.x; e < tile; e += NTT_THREADS) {  // c, DIT inter-pass twiddle
        const unsigned t = e & (T - 1), i1 = (e >> Tlog) & bmask;
        const uint64_t gi = ((uint64_t)i1 << Slog) + i20 + t;
        fr29_t x = f29(cv[gi]);
        const uint32_t ex = (uint32_t)(((i20 + t) * brev(i1, b)) << (32 - L));
        if (ex) x = fr29_mul(x, tw29(flo, fhi, ex));
        lds_put(sh, e, x);
    }
    __syncthreads();
    ntt_rounds<false>(sh, b, Tlog, tile, ftw10, tsh);
    for (unsigned e = threadIdx.x; e < tile; e += NTT_THREADS) {  // h = (a b - c) / Z on the coset
        const unsigned t = e & (T - 1), i1 = (e >> Tlog) & bmask;
        const uint64_t gi = ((uint64_t)i1 << Slog) + i20 + t;
        const fr29_t ab = fr29_mul(f29(ha[gi]), f29(bv[gi]));               // < 2r
        lds_put(sh, e, fr29_mul(fr29_sub_lazy(ab, lds_get(sh, e), R2X29), z29));  // (< 4r) z -> < 2r
    }
    __syncthreads();
    ntt_rounds<true>(sh, b, Tlog, tile, itw10, tsh);
    for (unsigned e = threadIdx.x; e < tile; e += NTT_THREADS) {  // DIF inter-pass twiddle, store over a
        const unsigned t = e & (T - 1), i1 = (e >> Tlog) & bmask;
        const uint64_t gi = ((uint64_t)i1 << Slog) + i20 + t;
        fr29_t x = lds_get(sh, e);
        const uint32_t ex = (uint32_t)(((i20 + t) * brev(i1, b)) << (32 - L));
        if (ex) x = fr29_mul(x, tw29(ilo, ihi, ex));
        ha[gi] = to_fr(x);
    }
}

struct PassPlan {
    unsigned M, b, Tlog, Glog;
    bool twiddle;
    uint64_t blocks;
};

std::vector<PassPlan> plan_passes(unsigned L) {
    std::vector<PassPlan> ps;
    if (L == 0) return ps;
    // innermost pass takes up to TILE_LOG bits; the rest is split evenly into passes of <= 8 bits
    unsigned inner = L < TILE_LOG ? L : TILE_LOG;
    unsigned rest = L - inner;
    unsigned nouter = (rest + 7) / 8;
    std::vector<unsigned> bits;
    for (unsigned i = 0; i < nouter; i++) bits.push_back(rest / nouter + (i < rest % nouter ? 1 : 0));
    bits.push_back(inner);
    unsigned M = L;
    for (size_t p = 0; p < bits.size(); p++) {
        PassPlan pp;
        pp.M = M;
        pp.b = bits[p];
        unsigned Slog = M - pp.b;
        unsigned room = TILE_LOG - pp.b;  // log2 of T*G that fits the tile
        if (Slog >= room) {
            pp.Tlog = room;
            pp.Glog = 0;
            pp.blocks = (1ull << (L - M)) * ((1ull << Slog) >> pp.Tlog);
        } else {
            pp.Tlog = Slog;
            unsigned g = room - Slog;
            unsigned nsub_log = L - M;
            if (g > nsub_log) g = nsub_log;
            pp.Glog = g;
            pp.blocks = 1ull << (nsub_log - g);
        }
        pp.twiddle = (p + 1 < bits.size());
        ps.push_back(pp);
        M -= pp.b;
    }
    return ps;
}

__global__ void k_bitrev_permute(fr_t *__restrict__ d, unsigned L, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t r = L ? (__builtin_bitreverse64(i) >> (64 - L)) : 0;
    if (i < r) {
        fr_t a = d[i], b = d[r];
        d[i] = b;
        d[r] = a;
    }
}

__global__ void k_coset_scale(fr_t *__restrict__ d, unsigned L, uint64_t n, int bitrev_pos,
                              const fr_t *__restrict__ lo, const fr_t *__restrict__ hi, fr_t scale,
                              int use_scale, int to_canonical) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t e = bitrev_pos ? brev((uint32_t)i, L) : (uint32_t)i;
    fr_t x = d[i];
    if (e) x = x * tw_full(lo, hi, e);
    if (use_scale) x = x * scale;
    if (to_canonical) x = from_mont(x);
    d[i] = x;
}

__global__ void k_scale(fr_t *__restrict__ d, uint64_t n, fr_t s) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = d[i] * s;
}
__global__ void k_to_mont(fr_t *__restrict__ d, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = to_mont(d[i]);
}
__global__ void k_from_mont(fr_t *__restrict__ d, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = from_mont(d[i]);
}

inline unsigned grid1(uint64_t n) { return (unsigned)((n + 255) / 256); }

void host_table(std::vector<fr_t> &lo, std::vector<fr_t> &hi, const fr_t &w) {
    lo.resize(65536);
    hi.resize(65536);
    lo[0] = fr_t::one();
    for (int i = 1; i < 65536; i++) lo[i] = lo[i - 1] * w;
    fr_t w16 = lo[65535] * w;
    hi[0] = fr_t::one();
    for (int i = 1; i < 65536; i++) hi[i] = hi[i - 1] * w16;
}

fr_t fr_small(uint32_t v) {
    fr_t r = fr_t::zero();
    r.v[0] = v;
    return to_mont(r);
}

}  // namespace

fr_t fr_root_of_unity_2_32() {
    // 7^((r-1) >> 32): (r - 1) has a zero low word, so the exponent is MOD[1..7]
    uint32_t e[7];
    for (int i = 0; i < 7; i++) e[i] = FrDesc::MOD[i + 1];
    return pow_words(fr_small(7), e, 7);
}

void ntt_init_tables(Ctx &c) {
    fr_t w = fr_root_of_unity_2_32();
    // sanity: w^(2^31) == -1
    fr_t t = w;
    for (int i = 0; i < 31; i++) t = sqr(t);
    if (!(t == -fr_t::one())) throw std::runtime_error("ntt: bad 2^32-th root of unity");
    fr_t wi = inverse(w), g = fr_small(7), gi = inverse(g);
    std::vector<fr_t> lo, hi;
    fr_t **dst[4][2] = {{&c.tw.fw_lo, &c.tw.fw_hi}, {&c.tw.iv_lo, &c.tw.iv_hi}, {&c.tw.g_lo, &c.tw.g_hi},
                        {&c.tw.gi_lo, &c.tw.gi_hi}};
    fr_t bases[4] = {w, wi, g, gi};
    for (int k = 0; k < 4; k++) {
        host_table(lo, hi, bases[k]);
        MI_HIP(hipMalloc(dst[k][0], sizeof(fr_t) * 65536));
        MI_HIP(hipMalloc(dst[k][1], sizeof(fr_t) * 65536));
        MI_HIP(hipMemcpy(*dst[k][0], lo.data(), sizeof(fr_t) * 65536, hipMemcpyHostToDevice));
        MI_HIP(hipMemcpy(*dst[k][1], hi.data(), sizeof(fr_t) * 65536, hipMemcpyHostToDevice));
        {  // the same tables in 29-bit limbs for the NTT passes
            std::vector<fr29_t> l29(65536), h29(65536);
            for (int i = 0; i < 65536; i++) l29[i] = fr29_from_fr(lo[i]), h29[i] = fr29_from_fr(hi[i]);
            MI_HIP(hipMalloc(&c.tw.lo29[k], sizeof(fr29_t) * 65536));
            MI_HIP(hipMalloc(&c.tw.hi29[k], sizeof(fr29_t) * 65536));
            MI_HIP(hipMemcpy(c.tw.lo29[k], l29.data(), sizeof(fr29_t) * 65536, hipMemcpyHostToDevice));
            MI_HIP(hipMemcpy(c.tw.hi29[k], h29.data(), sizeof(fr29_t) * 65536, hipMemcpyHostToDevice));
        }
        if (k < 2) {  // omega_1024^j = HI[j * 64] (HI[h] = omega_{2^16}^h), j < 512, in 29-bit limbs
            std::vector<fr29_t> t10(TILE / 2);
            for (unsigned j = 0; j < TILE / 2; j++) t10[j] = fr29_from_fr(hi[j << (16 - TILE_LOG)]);
            fr29_t **p10 = k == 0 ? &c.tw.fw_1024 : &c.tw.iv_1024;
            MI_HIP(hipMalloc(p10, sizeof(fr29_t) * (TILE / 2)));
            MI_HIP(hipMemcpy(*p10, t10.data(), sizeof(fr29_t) * (TILE / 2), hipMemcpyHostToDevice));
        }
    }
}

void ntt_free_tables(Ctx &c) {
    fr_t *ps[8] = {c.tw.fw_lo, c.tw.fw_hi, c.tw.iv_lo, c.tw.iv_hi, c.tw.g_lo, c.tw.g_hi, c.tw.gi_lo, c.tw.gi_hi};
    for (auto p : ps)
        if (p) hipFree(p);
    for (int k = 0; k < 4; k++) {
        if (c.tw.lo29[k]) hipFree(c.tw.lo29[k]);
        if (c.tw.hi29[k]) hipFree(c.tw.hi29[k]);
    }
    if (c.tw.fw_1024) hipFree(c.tw.fw_1024);
    if (c.tw.iv_1024) hipFree(c.tw.iv_1024);
    c.tw = NttTables();
}

static void ntt_run(Ctx &c, fr_t *d, unsigned L, bool inverse, bool dif, int epi = 0, bool inv_gen = false,
                    const fr_t &scale = fr_t::one(), size_t first_pass = 0) {
    if (L > 32) throw std::runtime_error("ntt: domain larger than 2^32");
    if (L == 0) {
        if (epi) {  // single element: coset factor g^0 = 1
            fr_t one = scale;
            scale_all(c, d, 1, one);
            if (epi == 2) fr_from_mont_inplace(c, d, 1);
        }
        return;
    }
    ScopedTimer tm(c, &c.stats.ntt, 1ull << L);
    const fr29_t *lo = c.tw.lo29[inverse ? 1 : 0], *hi = c.tw.hi29[inverse ? 1 : 0];
    const fr29_t *glo = c.tw.lo29[inv_gen ? 3 : 2], *ghi = c.tw.hi29[inv_gen ? 3 : 2];
    const fr29_t *tw10 = inverse ? c.tw.iv_1024 : c.tw.fw_1024;
    auto plan = plan_passes(L);
    if (dif) {
        for (size_t i = first_pass; i < plan.size(); i++) {
            auto &p = plan[i];
            int e = (i + 1 == plan.size()) ? epi : 0;
            k_ntt_pass<true><<<(unsigned)p.blocks, NTT_THREADS, 0, c.stream>>>(d, L, p.M, p.b, p.Tlog, p.Glog,
                                                                                 p.twiddle, lo, hi, tw10, e, glo,
                                                                                 ghi, scale);
        }
    } else {
        for (int i = (int)plan.size() - 1; i >= 0; i--) {
            auto &p = plan[i];
            k_ntt_pass<false><<<(unsigned)p.blocks, NTT_THREADS, 0, c.stream>>>(d, L, p.M, p.b, p.Tlog, p.Glog,
                                                                                  p.twiddle, lo, hi, tw10, 0, glo,
                                                                                  ghi, scale);
        }
    }
    MI_HIP(hipGetLastError());
}

// iNTT (DIF, natural -> bit-reversed) -> * g^bitrev(pos) * scale -> NTT (DIT, -> natural): the QAP's
// "evaluations on the domain -> evaluations on the coset" for a, b, c.  The innermost DIF pass and the
// first DIT pass work on the same contiguous tiles, so they run as ONE kernel (k_ntt_pass<true, true>):
// one HBM pass fewer per vector than ntt_dif_coset_epilogue + ntt_dit.
void ntt_coset_roundtrip(Ctx &c, fr_t *d, unsigned L, const fr_t &scale) {
    if (L > 32) throw std::runtime_error("ntt: domain larger than 2^32");
    if (L == 0) {
        scale_all(c, d, 1, scale);
        return;
    }
    ScopedTimer tm(c, &c.stats.ntt, 1ull << L);
    auto plan = plan_passes(L);
    const size_t last = plan.size() - 1;
    for (size_t i = 0; i < last; i++) {
        auto &p = plan[i];
        k_ntt_pass<true><<<(unsigned)p.blocks, NTT_THREADS, 0, c.stream>>>(d, L, p.M, p.b, p.Tlog, p.Glog, p.twiddle,
                                                                             c.tw.lo29[1], c.tw.hi29[1], c.tw.iv_1024, 0,
                                                                             c.tw.lo29[2], c.tw.hi29[2], scale);
    }
    {
        auto &p = plan[last];
        k_ntt_pass<true, true><<<(unsigned)p.blocks, NTT_THREADS, 0, c.stream>>>(
            d, L, p.M, p.b, p.Tlog, p.Glog, 0, c.tw.lo29[1], c.tw.hi29[1], c.tw.iv_1024, 1, c.tw.lo29[2], c.tw.hi29[2],
            scale, c.tw.fw_1024);
    }
    for (int i = (int)last - 1; i >= 0; i--) {
        auto &p = plan[i];
        k_ntt_pass<false><<<(unsigned)p.blocks, NTT_THREADS, 0, c.stream>>>(d, L, p.M, p.b, p.Tlog, p.Glog, p.twiddle,
                                                                              c.tw.lo29[0], c.tw.hi29[0], c.tw.fw_1024, 0,
                                                                              c.tw.lo29[2], c.tw.hi29[2], scale);
    }
    MI_HIP(hipGetLastError());
}

bool ntt_coset_qap(Ctx &c, fr_t *a, const fr_t *b, fr_t *cc, unsigned L, const fr_t &scale, const fr_t &zinv) {
    if (L > 32) throw std::runtime_error("ntt: domain larger than 2^32");
    auto plan = plan_passes(L);
    if (plan.size() < 2) return false;  // one pass: the caller runs the unfused chain
    {
        ScopedTimer tm(c, &c.stats.ntt, 1ull << L);
        const size_t last = plan.size() - 1;
        for (size_t i = 0; i < last; i++) {
            auto &p = plan[i];
            k_ntt_pass<true><<<(unsigned)p.blocks, NTT_THREADS, 0, c.stream>>>(cc, L, p.M, p.b, p.Tlog, p.Glog, p.twiddle,
                                                                                 c.tw.lo29[1], c.tw.hi29[1], c.tw.iv_1024,
                                                                                 0, c.tw.lo29[2], c.tw.hi29[2], scale);
        }
        {
            auto &p = plan[last];
            k_ntt_pass<true, true><<<(unsigned)p.blocks, NTT_THREADS, 0, c.stream>>>(
                cc, L, p.M, p.b, p.Tlog, p.Glog, 0, c.tw.lo29[1], c.tw.hi29[1], c.tw.iv_1024, 1, c.tw.lo29[2],
                c.tw.hi29[2], scale, c.tw.fw_1024);
        }
        for (size_t i = last - 1; i >= 1; i--) {
            auto &p = plan[i];
            k_ntt_pass<false><<<(unsigned)p.blocks, NTT_THREADS, 0, c.stream>>>(cc, L, p.M, p.b, p.Tlog, p.Glog,
                                                                                  p.twiddle, c.tw.lo29[0], c.tw.hi29[0],
                                                                                  c.tw.fw_1024, 0, c.tw.lo29[2],
                                                                                  c.tw.hi29[2], scale);
        }
        auto &p0 = plan[0];
        if (p0.M != L || p0.Glog != 0 || !p0.twiddle) throw std::logic_error("ntt: unexpected outer pass shape");
        k_ntt_qap<<<(unsigned)p0.blocks, NTT_THREADS, 0, c.stream>>>(a, b, cc, L, p0.b, p0.Tlog, c.tw.lo29[0],
                                                                     c.tw.hi29[0], c.tw.fw_1024, c.tw.lo29[1],
                                                                     c.tw.hi29[1], c.tw.iv_1024, zinv);
        MI_HIP(hipGetLastError());
    }
    // the rest of H's inverse coset transform: passes 1.. with the icoset epilogue (canonical output)
    ntt_run(c, a, L, true, true, 2, true, scale, 1);
    return true;
}

void ntt_dif_coset_epilogue(Ctx &c, fr_t *d, unsigned log_n, bool inverse, bool inverse_gen, const fr_t &scale,
                            bool to_canonical) {
    ntt_run(c, d, log_n, inverse, true, to_canonical ? 2 : 1, inverse_gen, scale);
}

void ntt_dif(Ctx &c, fr_t *d, unsigned log_n, bool inverse) { ntt_run(c, d, log_n, inverse, true); }
void ntt_dit(Ctx &c, fr_t *d, unsigned log_n, bool inverse) { ntt_run(c, d, log_n, inverse, false); }

void bitrev_permute(Ctx &c, fr_t *d, unsigned log_n) {
    uint64_t n = 1ull << log_n;
    k_bitrev_permute<<<grid1(n), 256, 0, c.stream>>>(d, log_n, n);
    MI_HIP(hipGetLastError());
}

void coset_scale_bitrev(Ctx &c, fr_t *d, unsigned log_n, bool inverse_gen, const fr_t *scale_host,
                        bool to_canonical) {
    uint64_t n = 1ull << log_n;
    k_coset_scale<<<grid1(n), 256, 0, c.stream>>>(d, log_n, n, 1, inverse_gen ? c.tw.gi_lo : c.tw.g_lo,
                                                  inverse_gen ? c.tw.gi_hi : c.tw.g_hi,
                                                  scale_host ? *scale_host : fr_t::one(), scale_host != nullptr,
                                                  to_canonical);
    MI_HIP(hipGetLastError());
}

void coset_scale_natural(Ctx &c, fr_t *d, unsigned log_n, bool inverse_gen, const fr_t *scale_host) {
    uint64_t n = 1ull << log_n;
    k_coset_scale<<<grid1(n), 256, 0, c.stream>>>(d, log_n, n, 0, inverse_gen ? c.tw.gi_lo : c.tw.g_lo,
                                                  inverse_gen ? c.tw.gi_hi : c.tw.g_hi,
                                                  scale_host ? *scale_host : fr_t::one(), scale_host != nullptr, 0);
    MI_HIP(hipGetLastError());
}

void scale_all(Ctx &c, fr_t *d, uint64_t n, const fr_t &s) {
    k_scale<<<grid1(n), 256, 0, c.stream>>>(d, n, s);
    MI_HIP(hipGetLastError());
}
void fr_to_mont_inplace(Ctx &c, fr_t *d, uint64_t n) {
    if (!n) return;
    k_to_mont<<<grid1(n), 256, 0, c.stream>>>(d, n);
    MI_HIP(hipGetLastError());
}
void fr_from_mont_inplace(Ctx &c, fr_t *d, uint64_t n) {
    if (!n) return;
    k_from_mont<<<grid1(n), 256, 0, c.stream>>>(d, n);
    MI_HIP(hipGetLastError());
}

}  // namespace mi
