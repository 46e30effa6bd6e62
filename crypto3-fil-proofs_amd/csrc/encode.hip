// encode.hip -- wire formats <-> device representation.
//
// Boundary formats follow the reference's data contracts:
//   * points: zcash/bellman "uncompressed" big-endian encodings, the layout of the Groth params
//     file the reference mmaps (core/crypto/mapped_scheme_params.hpp:43-84): G1 = x|y (96 B),
//     G2 = x.c1|x.c0|y.c1|y.c0 (192 B); flag bits live in the top 3 bits of byte 0
//     (0x40 = point at infinity).
//   * scalars: Fr as 32-byte little-endian (core/fr32.hpp:36-52).
// On device, coordinates are Montgomery 32-bit-limb little-endian; affine infinity is (0, 0).
#include <stdio.h>
#include <stdlib.h>

#include "ctx.h"

namespace mi {

namespace {

__device__ __forceinline__ uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// 48 big-endian bytes -> Montgomery Fq; returns false when the integer is >= p
__device__ __forceinline__ bool fq_from_be48(const uint8_t *p, bool mask_flags, fq_t &out) {
    fq32_t raw;
    MI_UNROLL for (int i = 0; i < 12; i++) {
        uint32_t w = be32(p + 4 * (11 - i));
        if (i == 11 && mask_flags) w &= 0x1fffffffu;
        raw.v[i] = w;
    }
    out = fq_from_raw(raw);
    return !geq_raw(raw, fq32_t::modulus_raw());
}

// zcash/bellman from_uncompressed flag rules for byte 0 of an uncompressed point: the compression
// bit (0x80) is clear; infinity (0x40) has every other bit of the encoding zero; otherwise the sort
// bit (0x20) is clear.  Returns 0 = finite point, 1 = valid infinity, -1 = malformed.
__device__ __forceinline__ int uncompressed_flags(const uint8_t *p, int len) {
    const uint8_t f = p[0];
    if (f & 0x80) return -1;
    if (f & 0x40) {
        uint32_t any = f & 0x3f;
        for (int k = 1; k < len; k++) any |= p[k];
        return any ? -1 : 1;
    }
    return (f & 0x20) ? -1 : 0;
}

// bad[0]: malformed / non-canonical / off-curve points, bad[1]: infinities when reject_inf (bellman's
// Parameters::read refuses the identity in every query: "point at infinity")
__global__ void k_g1_decode(const uint8_t *__restrict__ in, g1_affine_t *__restrict__ out, uint64_t n,
                            int *__restrict__ bad, int reject_inf) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *p = in + 96 * i;
    const int f = uncompressed_flags(p, 96);
    if (f != 0) {
        if (f < 0) atomicAdd(&bad[0], 1);
        else if (reject_inf) atomicAdd(&bad[1], 1);
        out[i] = g1_affine_t::inf();
        return;
    }
    g1_affine_t a;
    bool ok = fq_from_be48(p, true, a.x) & fq_from_be48(p + 48, false, a.y);
    if (!ok || !g1_on_curve(a)) atomicAdd(&bad[0], 1);
    out[i] = a;
}

__global__ void k_g2_decode(const uint8_t *__restrict__ in, g2_affine_t *__restrict__ out, uint64_t n,
                            int *__restrict__ bad, int reject_inf) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *p = in + 192 * i;
    const int f = uncompressed_flags(p, 192);
    if (f != 0) {
        if (f < 0) atomicAdd(&bad[0], 1);
        else if (reject_inf) atomicAdd(&bad[1], 1);
        out[i] = g2_affine_t::inf();
        return;
    }
    g2_affine_t a;
    bool ok = fq_from_be48(p, true, a.x.c1) & fq_from_be48(p + 48, false, a.x.c0) &
              fq_from_be48(p + 96, false, a.y.c1) & fq_from_be48(p + 144, false, a.y.c0);
    if (!ok || !g2_on_curve(a)) atomicAdd(&bad[0], 1);
    out[i] = a;
}

// prime-order-subgroup membership of every decoded point (the checked load; curve.h in_prime_subgroup_fast, the
// endomorphism tests -- round 6; r P == O before, 4-5x the group operations); bad[2] counts points outside it
template <class F>
__global__ void __launch_bounds__(256) k_subgroup(const Affine<F> *__restrict__ pts, uint64_t n,
                                                  int *__restrict__ bad, const SubgroupConsts sc) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (!in_prime_subgroup_fast(pts[i], sc)) atomicAdd(&bad[2], 1);
}

// entries >= r (not a valid Fr: core/fr32.hpp:36-40) -> *bad += 1
__global__ void k_fr_check(const fr_t *__restrict__ d, uint64_t n, int *__restrict__ bad) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (geq_raw(d[i], fr_t::modulus_raw())) atomicAdd(bad, 1);
}

__device__ __forceinline__ void fq_to_be48_dev(const fq_t &a, uint8_t *out) {
    fq32_t raw = fq_to_raw(a);
    MI_UNROLL for (int i = 0; i < 12; i++) {
        uint32_t w = raw.v[i];
        uint8_t *p = out + 4 * (11 - i);
        p[0] = (uint8_t)(w >> 24);
        p[1] = (uint8_t)(w >> 16);
        p[2] = (uint8_t)(w >> 8);
        p[3] = (uint8_t)w;
    }
}
// device affine -> zcash uncompressed; src index = perm_log ? bitrev(i) : i (h is stored bit-reversed)
__global__ void k_g1_encode(const g1_affine_t *__restrict__ in, uint8_t *__restrict__ out, uint64_t n,
                            unsigned perm_log, uint64_t first) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // natural index first + i; with perm_log the source is stored bit-reversed (the h query)
    uint64_t src = perm_log ? (__builtin_bitreverse64(first + i) >> (64 - perm_log)) : first + i;
    uint8_t *p = out + 96 * i;
    const g1_affine_t a = in[src];
    if (a.is_inf()) {
        for (int k = 0; k < 96; k++) p[k] = 0;
        p[0] = 0x40;
        return;
    }
    fq_to_be48_dev(a.x, p);
    fq_to_be48_dev(a.y, p + 48);
}
__global__ void k_g2_encode(const g2_affine_t *__restrict__ in, uint8_t *__restrict__ out, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t *p = out + 192 * i;
    const g2_affine_t a = in[i];
    if (a.is_inf()) {
        for (int k = 0; k < 192; k++) p[k] = 0;
        p[0] = 0x40;
        return;
    }
    fq_to_be48_dev(a.x.c1, p);
    fq_to_be48_dev(a.x.c0, p + 48);
    fq_to_be48_dev(a.y.c1, p + 96);
    fq_to_be48_dev(a.y.c0, p + 144);
}

// x mod r for x < 2^256 (at most two subtractions: 2^256 < 3r)
__global__ void k_fr_canon(fr_t *__restrict__ d, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fr_t x = d[i];
    fr_t m = fr_t::modulus_raw();
    MI_UNROLL for (int k = 0; k < 2; k++) {
        if (geq_raw(x, m)) {
            uint32_t borrow = 0;
            MI_UNROLL for (int j = 0; j < 8; j++) {
                uint64_t t = (uint64_t)x.v[j] - m.v[j] - borrow;
                x.v[j] = (uint32_t)t;
                borrow = (uint32_t)(t >> 63);
            }
        }
    }
    d[i] = x;
}

inline unsigned grid1(uint64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

void debug_sync(Ctx &c, const char *what) {
    if (tune::get(tune::DEBUG_SYNC, 0) != 1) return;  // tune::DEBUG_SYNC (debugging only)
    hipError_t e = hipStreamSynchronize(c.stream);
    fprintf(stderr, "[mi] %s: %s\n", what, hipGetErrorString(e));
    if (e != hipSuccess) throw hip_error(e, std::string("kernel ") + what + " failed: " + hipGetErrorString(e));
}

void g1_decode_uncompressed(Ctx &c, const uint8_t *dev_bytes, g1_affine_t *out, uint64_t n, int *bad_dev,
                            bool reject_inf) {
    if (!n) return;
    k_g1_decode<<<grid1(n), 256, 0, c.stream>>>(dev_bytes, out, n, bad_dev, reject_inf ? 1 : 0);
    MI_HIP(hipGetLastError());
}
void g2_decode_uncompressed(Ctx &c, const uint8_t *dev_bytes, g2_affine_t *out, uint64_t n, int *bad_dev,
                            bool reject_inf) {
    if (!n) return;
    k_g2_decode<<<grid1(n), 256, 0, c.stream>>>(dev_bytes, out, n, bad_dev, reject_inf ? 1 : 0);
    MI_HIP(hipGetLastError());
}
void g1_subgroup_check(Ctx &c, const g1_affine_t *pts, uint64_t n, int *bad_dev) {
    if (!n) return;
    static const SubgroupConsts sc = subgroup_consts();
    k_subgroup<fq_t><<<grid1(n), 256, 0, c.stream>>>(pts, n, bad_dev, sc);
    MI_HIP(hipGetLastError());
}
void g2_subgroup_check(Ctx &c, const g2_affine_t *pts, uint64_t n, int *bad_dev) {
    if (!n) return;
    static const SubgroupConsts sc = subgroup_consts();
    k_subgroup<fq2_t><<<grid1(n), 256, 0, c.stream>>>(pts, n, bad_dev, sc);
    MI_HIP(hipGetLastError());
}
void fr_count_noncanonical(Ctx &c, const fr_t *d, uint64_t n, int *bad_dev, hipStream_t st) {
    if (!n) return;
    k_fr_check<<<grid1(n), 256, 0, st>>>(d, n, bad_dev);
    MI_HIP(hipGetLastError());
}
void g1_encode_uncompressed(Ctx &c, const g1_affine_t *in, uint8_t *dev_out, uint64_t n, unsigned perm_log,
                            uint64_t first) {
    if (!n) return;
    k_g1_encode<<<grid1(n), 256, 0, c.stream>>>(in, dev_out, n, perm_log, first);
    MI_HIP(hipGetLastError());
}
void g2_encode_uncompressed(Ctx &c, const g2_affine_t *in, uint8_t *dev_out, uint64_t n) {
    if (!n) return;
    k_g2_encode<<<grid1(n), 256, 0, c.stream>>>(in, dev_out, n);
    MI_HIP(hipGetLastError());
}
void fr_canonicalize(Ctx &c, fr_t *d, uint64_t n) {
    if (!n) return;
    k_fr_canon<<<grid1(n), 256, 0, c.stream>>>(d, n);
    MI_HIP(hipGetLastError());
}

}  // namespace mi
