// GPU witness of the stacked-PoRep circuit (stacked.h).
//
// Phase A walks the witness program level by level (one launch per level, one thread per op): data copies,
// bit decompositions, picks, and / nor bits and adds write their variables; a Poseidon op runs the literal
// permutation natively and writes its digest; a SHA-256 op runs its compressions natively, keeps each
// block's input state for phase B, and writes the packed digest.  Phase B then re-derives the internal
// variables of every heavy gadget in parallel: one thread per SHA-256 block emulates bellman's
// sha256_compression_function over (value, constant mask, negation mask) words and writes each allocated
// bit in allocation order; one thread per Poseidon hash writes the S-box chain of every round.  Both use
// exactly the allocation order of the host builder (stacked_build.hip) and of oracle/stacked_circuit.py.
//
// Bound: phase B writes ~1.3e8 32-byte variables per 32 GiB partition (4.2 GB) with ~20 VALU ops each;
// SHA-256 blocks are the bulk (~5,000 blocks x ~26 K variables).
#include <cstring>
#include <stdexcept>

#include "ctx.h"
#include "poseidon.h"
#include "poseidon_math.h"
#include "stacked.h"
#include "stacked_pos.h"

namespace mi {
namespace stacked {

namespace {

struct PosKs {
    PosK k[4];  // arity 2, 4, 8, 11
};

struct DevProg {
    WOp *ops = nullptr;
    uint64_t *pin = nullptr;
    ShaBlock *blocks = nullptr;
    uint64_t *pos_ops = nullptr;  // Poseidon op indices grouped by arity (2, 4, 8, 11)
    uint64_t pos_off[5] = {0, 0, 0, 0, 0};
    uint32_t *states = nullptr;  // 8 words per block: the block's input chaining value
    PosKs pk{};                  // device views of the production Poseidon tables (poseidon_tables, per ctx)
    int device = -1;
    ~DevProg() {
        for (void *p : {(void *)ops, (void *)pin, (void *)blocks, (void *)pos_ops, (void *)states})
            if (p) hipFree(p);
    }
};

__device__ __forceinline__ void zput_u32(fr_t *z, uint64_t k, uint32_t lo, uint32_t hi = 0) {
    uint4 *p = reinterpret_cast<uint4 *>(z + k);
    p[0] = make_uint4(lo, hi, 0, 0);
    p[1] = make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ void zput_fr(fr_t *z, uint64_t k, const fr_t &x) {
    uint4 *p = reinterpret_cast<uint4 *>(z + k);
    p[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    p[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}
__device__ __forceinline__ fr_t zget(const fr_t *z, uint64_t k) {
    const uint4 *p = reinterpret_cast<const uint4 *>(z + k);
    uint4 a = p[0], b = p[1];
    fr_t x;
    x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
    x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
    return x;
}
__device__ __forceinline__ uint64_t slot_u64(const uint8_t *slots, uint64_t s) {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(slots + 32 * s);
    return (uint64_t)p[0] | ((uint64_t)p[1] << 32);
}
__device__ __forceinline__ fr_t slot_fr(const uint8_t *slots, uint64_t s) {
    const uint4 *p = reinterpret_cast<const uint4 *>(slots + 32 * s);
    uint4 a = p[0], b = p[1];
    fr_t x;
    x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
    x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
    return x;
}

// ---------------------------------------------------------------------------------------- SHA-256 (native)
__constant__ uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
__constant__ uint32_t kIV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

__device__ __forceinline__ uint32_t rotr32(uint32_t x, int k) { return (x >> k) | (x << (32 - k)); }

__device__ void sha_native(uint32_t st[8], const uint32_t m[16]) {
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = m[i];
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            uint32_t x = w[(i - 15) & 15], y = w[(i - 2) & 15];
            uint32_t s0 = rotr32(x, 7) ^ rotr32(x, 18) ^ (x >> 3);
            uint32_t s1 = rotr32(y, 17) ^ rotr32(y, 19) ^ (y >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + kK[i] + wi;
        uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// message word value and constant mask from its descriptor (stacked.h WD_*)
__device__ __forceinline__ void word_of(uint64_t desc, const fr_t *z, const uint8_t *slots, uint32_t &v, uint32_t &cm) {
    const uint64_t kind = desc >> 62, pay = desc & ((1ull << 62) - 1);
    if (kind == 0) {
        v = (uint32_t)pay;
        cm = 0xFFFFFFFFu;
    } else if (kind == 1) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(z + (pay >> 3));
        v = __builtin_bswap32(p[pay & 7]);
        cm = (pay & 7) == 7 ? 0x80u : 0u;
    } else {
        const uint64_t x = slot_u64(slots, pay >> 1);
        v = (pay & 1) ? (uint32_t)x : (uint32_t)(x >> 32);
        cm = 0;
    }
}

// ---------------------------------------------------------------------------------------- SHA-256 gadget
struct W3 {  // a bellman UInt32: logical value, constant-bit mask, negated-variable mask
    uint32_t v, c, n;
};
struct B1 {
    uint32_t v, c, n;
};
struct Emit {
    fr_t *z;
    uint64_t k;
    __device__ __forceinline__ void put(uint32_t bit) { zput_u32(z, k++, bit); }
};
__device__ __forceinline__ B1 bit_of(const W3 &w, int i) { return B1{(w.v >> i) & 1u, (w.c >> i) & 1u, (w.n >> i) & 1u}; }
__device__ __forceinline__ void set_bit(W3 &w, int i, const B1 &b) {
    w.v |= b.v << i;
    w.c |= b.c << i;
    w.n |= b.n << i;
}
__device__ __forceinline__ B1 b_not(const B1 &x) { return x.c ? B1{x.v ^ 1u, 1u, 0u} : B1{x.v ^ 1u, 0u, x.n ^ 1u}; }
__device__ __forceinline__ B1 b_xor(Emit &E, const B1 &a, const B1 &b) {
    if (a.c && !a.v) return b;
    if (b.c && !b.v) return a;
    if (a.c) return b_not(b);
    if (b.c) return b_not(a);
    E.put((a.v ^ a.n) ^ (b.v ^ b.n));  // the new variable: xor of the operands' variables
    return B1{a.v ^ b.v, 0u, a.n ^ b.n};
}
__device__ __forceinline__ B1 b_and(Emit &E, const B1 &a, const B1 &b) {
    if ((a.c && !a.v) || (b.c && !b.v)) return B1{0u, 1u, 0u};
    if (a.c) return b;
    if (b.c) return a;
    const uint32_t v = a.v & b.v;  // and / and_not / nor all allocate the logical and
    E.put(v);
    return B1{v, 0u, 0u};
}
__device__ B1 b_ch(Emit &E, const B1 &a, const B1 &b, const B1 &c) {
    const uint32_t val = (a.v & b.v) ^ ((a.v ^ 1u) & c.v);
    if (a.c && b.c && c.c) return B1{val, 1u, 0u};
    if (a.c && !a.v) return c;
    if (b.c && !b.v) return b_and(E, b_not(a), c);
    if (c.c && !c.v) return b_and(E, a, b);
    if (c.c && c.v) return b_not(b_and(E, a, b_not(b)));
    if (b.c && b.v) return b_not(b_and(E, b_not(a), b_not(c)));
    E.put(val);
    return B1{val, 0u, 0u};
}
__device__ B1 b_maj(Emit &E, const B1 &a, const B1 &b, const B1 &c) {
    const uint32_t val = (a.v & b.v) ^ (a.v & c.v) ^ (b.v & c.v);
    if (a.c && b.c && c.c) return B1{val, 1u, 0u};
    if (a.c && !a.v) return b_and(E, b, c);
    if (b.c && !b.v) return b_and(E, a, c);
    if (c.c && !c.v) return b_and(E, a, b);
    if (c.c && c.v) return b_not(b_and(E, b_not(a), b_not(b)));
    if (b.c && b.v) return b_not(b_and(E, b_not(a), b_not(c)));
    if (a.c && a.v) return b_not(b_and(E, b_not(b), b_not(c)));
    E.put(val);         // maj
    b_and(E, b, c);     // then b and c
    return B1{val, 0u, 0u};
}
__device__ W3 w_xor(Emit &E, const W3 &a, const W3 &b) {
    W3 r{0, 0, 0};
    for (int i = 0; i < 32; i++) set_bit(r, i, b_xor(E, bit_of(a, i), bit_of(b, i)));
    return r;
}
__device__ __forceinline__ W3 w_rotr(const W3 &a, int k) { return W3{rotr32(a.v, k), rotr32(a.c, k), rotr32(a.n, k)}; }
__device__ __forceinline__ W3 w_shr(const W3 &a, int k) {
    return W3{a.v >> k, (a.c >> k) | (0xFFFFFFFFu << (32 - k)), a.n >> k};
}
__device__ W3 w_addmany(Emit &E, const W3 *ops, int n) {
    uint64_t sum = 0;
    uint32_t allc = 0xFFFFFFFFu;
    for (int i = 0; i < n; i++) {
        sum += ops[i].v;
        allc &= ops[i].c;
    }
    if (allc == 0xFFFFFFFFu) return W3{(uint32_t)sum, 0xFFFFFFFFu, 0};
    const int nb = 64 - __builtin_clzll((uint64_t)n * 0xFFFFFFFFull);
    for (int i = 0; i < nb; i++) E.put((uint32_t)(sum >> i) & 1u);
    return W3{(uint32_t)sum, 0, 0};
}

// bellman sha256_compression_function over W3 words; schedule words kept in LDS (64 lanes x 64 words)
__device__ void sha_gadget(Emit &E, const W3 msg[16], const W3 H[8], W3 (*w)[64]) {
    const int lane = threadIdx.x;
    for (int i = 0; i < 16; i++) w[i][lane] = msg[i];
    for (int i = 16; i < 64; i++) {
        const W3 x = w[i - 15][lane], y = w[i - 2][lane];
        W3 s0 = w_xor(E, w_rotr(x, 7), w_rotr(x, 18));
        s0 = w_xor(E, s0, w_shr(x, 3));
        W3 s1 = w_xor(E, w_rotr(y, 17), w_rotr(y, 19));
        s1 = w_xor(E, s1, w_shr(y, 10));
        W3 ops[4] = {w[i - 16][lane], s0, w[i - 7][lane], s1};
        w[i][lane] = w_addmany(E, ops, 4);
    }
    // a / e: concrete words (the input state) until the first round defers them
    bool a_con = true, e_con = true;
    W3 a_ops[7], e_ops[6];
    a_ops[0] = H[0];
    e_ops[0] = H[4];
    W3 b = H[1], c = H[2], d = H[3], f = H[5], g = H[6], h = H[7];
    for (int i = 0; i < 64; i++) {
        const W3 ne = e_con ? e_ops[0] : w_addmany(E, e_ops, 6);
        W3 s1 = w_xor(E, w_rotr(ne, 6), w_rotr(ne, 11));
        s1 = w_xor(E, s1, w_rotr(ne, 25));
        W3 chv{0, 0, 0};
        for (int q = 0; q < 32; q++) set_bit(chv, q, b_ch(E, bit_of(ne, q), bit_of(f, q), bit_of(g, q)));
        const W3 kk{kK[i], 0xFFFFFFFFu, 0};
        const W3 wi = w[i][lane];
        const W3 na = a_con ? a_ops[0] : w_addmany(E, a_ops, 7);
        W3 s0 = w_xor(E, w_rotr(na, 2), w_rotr(na, 13));
        s0 = w_xor(E, s0, w_rotr(na, 22));
        W3 mj{0, 0, 0};
        for (int q = 0; q < 32; q++) set_bit(mj, q, b_maj(E, bit_of(na, q), bit_of(b, q), bit_of(c, q)));
        e_ops[0] = h; e_ops[1] = s1; e_ops[2] = chv; e_ops[3] = kk; e_ops[4] = wi; e_ops[5] = d;
        a_ops[0] = h; a_ops[1] = s1; a_ops[2] = chv; a_ops[3] = kk; a_ops[4] = wi; a_ops[5] = s0; a_ops[6] = mj;
        e_con = a_con = false;
        h = g; g = f; f = ne; d = c; c = b; b = na;
    }
    // h0 = a + H0 (deferred, 8 operands), h1 = H1 + b ... h4 = e + H4 (7 operands) ...
    W3 a8[8];
    for (int q = 0; q < 7; q++) a8[q] = a_ops[q];
    a8[7] = H[0];
    w_addmany(E, a8, 8);
    W3 t[2];
    t[0] = H[1]; t[1] = b; w_addmany(E, t, 2);
    t[0] = H[2]; t[1] = c; w_addmany(E, t, 2);
    t[0] = H[3]; t[1] = d; w_addmany(E, t, 2);
    W3 e7[7];
    for (int q = 0; q < 6; q++) e7[q] = e_ops[q];
    e7[6] = H[4];
    w_addmany(E, e7, 7);
    t[0] = H[5]; t[1] = f; w_addmany(E, t, 2);
    t[0] = H[6]; t[1] = g; w_addmany(E, t, 2);
    t[0] = H[7]; t[1] = h; w_addmany(E, t, 2);
}

// ---------------------------------------------------------------------------------------- Poseidon
struct ZSink {  // writes each emitted variable (canonical) to z
    fr_t *z;
    uint64_t k;
    __device__ __forceinline__ void put(const fr29_t &x) { zput_fr(z, k++, fr_from_fr29(fr29_from_mont(x))); }
};

template <int T, bool EXPAND>
__device__ __forceinline__ void pos_op_t(const WOp &op, const uint64_t *pin, const PosK &k, fr_t *z) {
    const fr29_t r2 = k.img[k.off_tag + 1];
    fr29_t s[T];
    MI_UNROLL for (int l = 0; l < 9; l++) s[0].v[l] = k.img[k.off_tag].v[l];  // limb-wise (a struct copy went to scratch)
    sfor<T - 1>([&](auto j) { s[j + 1] = fr29_mul(fr29_from_fr(zget(z, pin[op.a + j])), r2); });
    if (EXPAND) {
        ZSink E{z, op.dst};
        pos_run<T, ZSink>(k, s, &E);
    } else {
        const fr29_t out = pos_run<T, ZSink>(k, s, nullptr);
        zput_fr(z, op.b, fr_from_fr29(fr29_from_mont(out)));
    }
}

// ---------------------------------------------------------------------------------------- kernels
__global__ void __launch_bounds__(64) k_wit_level(const WOp *__restrict__ ops, uint64_t n, const uint8_t *__restrict__ slots,
                                                  const ShaBlock *__restrict__ blocks, uint32_t *__restrict__ states,
                                                  fr_t *__restrict__ z) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const WOp op = ops[i];
    switch (op.type) {
        case W_DATA: zput_fr(z, op.dst, slot_fr(slots, op.a)); break;
        case W_COPY: zput_fr(z, op.dst, zget(z, op.a)); break;
        case W_BITS: {
            const fr_t x = zget(z, op.a);
            for (uint32_t q = 0; q < op.n; q++) zput_u32(z, op.dst + q, (x.v[q >> 5] >> (q & 31)) & 1u);
            break;
        }
        case W_DBITS: {
            const uint64_t x = slot_u64(slots, op.a);
            for (uint32_t q = 0; q < op.n; q++) zput_u32(z, op.dst + q, (uint32_t)(x >> (op.b + q)) & 1u);
            break;
        }
        case W_DPACK: {
            uint64_t x = slot_u64(slots, op.a);
            if (op.n < 64) x &= (1ull << op.n) - 1;
            zput_u32(z, op.dst, (uint32_t)x, (uint32_t)(x >> 32));
            break;
        }
        case W_PICK: zput_fr(z, op.dst, zget(z, zget(z, op.c).v[0] ? op.a : op.b)); break;
        case W_AND: zput_u32(z, op.dst, zget(z, op.a).v[0] & zget(z, op.b).v[0]); break;
        case W_NOR: zput_u32(z, op.dst, (zget(z, op.a).v[0] | zget(z, op.b).v[0]) ^ 1u); break;
        case W_ADD: zput_fr(z, op.dst, zget(z, op.a) + zget(z, op.b)); break;
        case W_SHA: {
            uint32_t st[8];
            for (int q = 0; q < 8; q++) st[q] = kIV[q];
            for (uint32_t k = 0; k < op.n; k++) {
                const ShaBlock &blk = blocks[op.a + k];
                uint32_t m[16];
                for (int q = 0; q < 16; q++) {
                    uint32_t cm;
                    word_of(blk.desc[q], z, slots, m[q], cm);
                }
                for (int q = 0; q < 8; q++) states[8 * (op.a + k) + q] = st[q];
                sha_native(st, m);
            }
            // packed digest: bytes of the big-endian words as a little-endian integer, 254 bits
            fr_t x;
            for (int q = 0; q < 8; q++) x.v[q] = __builtin_bswap32(st[q]);
            x.v[7] &= 0x3FFFFFFFu;
            zput_fr(z, op.b, x);
            break;
        }
        default: break;
    }
}

__global__ void __launch_bounds__(64) k_wit_sha_blocks(const ShaBlock *__restrict__ blocks, uint64_t n,
                                                       const uint32_t *__restrict__ states,
                                                       const uint8_t *__restrict__ slots, fr_t *__restrict__ z) {
    __shared__ W3 wsh[64][64];
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ShaBlock &blk = blocks[i];
    W3 msg[16], H[8];
    for (int q = 0; q < 16; q++) {
        uint32_t v, cm;
        word_of(blk.desc[q], z, slots, v, cm);
        msg[q] = W3{v, cm, 0};
    }
    for (int q = 0; q < 8; q++) H[q] = blk.iv ? W3{kIV[q], 0xFFFFFFFFu, 0} : W3{states[8 * i + q], 0, 0};
    Emit E{z, blk.base};
    sha_gadget(E, msg, H, wsh);
}

// Poseidon ops of one arity: phase A (digest only) over ops[0 .. n) or phase B (all variables) over ops[idx[i]].
// Capped at 256 VGPRs (two waves per SIMD): the state spills to scratch for t = 12 rather than using AGPRs.
template <int T, bool EXPAND>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
k_wit_poseidon(const WOp *__restrict__ ops, const uint64_t *__restrict__ idx, uint64_t n,
               const uint64_t *__restrict__ pin, PosK k, fr_t *__restrict__ z) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    pos_op_t<T, EXPAND>(ops[EXPAND ? idx[i] : i], pin, k, z);
}
// Phase A's Poseidon ops are a latency chain: each tree level holds a few dozen to a few hundred hashes, and one
// thread per hash executes a whole permutation alone (0.9 ms per arity-8 level).  Here one hash takes a 16-lane
// group (4 hashes per wave) and lane j holds state element j:
//   full rounds  every lane its S-box, then the state is gathered across the group (9-word shuffles) and lane j
//                forms row j of the MDS product (fr29_row, as the one-thread form);
//   partial      lane 0 its S-box, s0 broadcast; lane j >= 1 updates s_j += w_j s0 while every lane forms its
//                term row_j s_j of the new s0, summed by a 4-level butterfly (each level reduced below 2r).
// The same field values as pos_run (exact arithmetic, lazy representatives < 4r, canonical digest), ~5x
// shorter per hash.  Phase B (EXPAND) uses the same kernel and writes each S-box's variables from its lane.
__device__ __forceinline__ fr29_t shfl29(const fr29_t &x, int src) {
    fr29_t r;
    MI_UNROLL for (int l = 0; l < 9; l++) r.v[l] = (uint32_t)__shfl((int)x.v[l], src, 16);
    return r;
}
__device__ __forceinline__ fr29_t shfl_xor29(const fr29_t &x, int mask) {
    fr29_t r;
    MI_UNROLL for (int l = 0; l < 9; l++) r.v[l] = (uint32_t)__shfl_xor((int)x.v[l], mask, 16);
    return r;
}
__device__ __forceinline__ fr29_t zero29() {
    fr29_t r;
    MI_UNROLL for (int l = 0; l < 9; l++) r.v[l] = 0;
    return r;
}
// row . state of lane j's row `m + j * T` over the group's state (gathered from lanes 0 .. T - 1)
template <int T>
__device__ __forceinline__ fr29_t group_row(const fr29_t &x, const fr29_t *__restrict__ m, int j) {
    fr29_t all[T];
    sfor<T>([&](auto i) { all[i] = shfl29(x, i); });
    return j < T ? fr29_row<T>(m + j * T, all) : zero29();
}

// EXPAND (phase B): every lane also writes its own S-box variables at their fixed offsets in the gadget's
// allocation order (pos_run's Sink order: first full rounds element by element -- the first round's inputs
// without v, the domain tag's first S-box none --, the partial rounds' element 0, the last full rounds, the
// digest), so the gadget's variables come out as pos_run<ZSink> writes them.
__device__ __forceinline__ void zput29(fr_t *z, uint64_t k, const fr29_t &x) {
    zput_fr(z, k, fr_from_fr29(fr29_from_mont(x)));
}
template <int T, bool EXPAND>
__global__ void __launch_bounds__(64) k_wit_poseidon_lanes(const WOp *__restrict__ ops, const uint64_t *__restrict__ idx,
                                                           uint64_t n, const uint64_t *__restrict__ pin, PosK k,
                                                           fr_t *__restrict__ z) {
    static_assert(T <= 16, "one hash per 16-lane group");
    const uint64_t h = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 4);
    const int j = (int)(threadIdx.x & 15);
    if (h >= n) return;  // whole groups only: shuffles stay inside a group
    const WOp op = ops[EXPAND ? idx[h] : h];
    const fr29_t *img = k.img;
    fr29_t x = zero29();
    if (j == 0) {
        MI_UNROLL for (int l = 0; l < 9; l++) x.v[l] = img[k.off_tag].v[l];
    } else if (j < T) {
        x = fr29_mul(fr29_from_fr(zget(z, pin[op.a + j - 1])), img[k.off_tag + 1]);
    }
    const fr29_t *mds = img + k.off_mds;
    const int half = k.rf / 2;
    // S-box with the gadget's variables written at z[at ..]: (v,) v^2, v^4, v^5
    auto sbox_emit = [&](const fr29_t &v, uint64_t at, bool with_v) -> fr29_t {
        const fr29_t v2 = fr29_sqr(v), v4 = fr29_sqr(v2), v5 = fr29_mul(v4, v);
        if (EXPAND) {
            if (with_v) zput29(z, at++, v);
            zput29(z, at++, v2);
            zput29(z, at++, v4);
            zput29(z, at, v5);
        }
        return v5;
    };
    const uint64_t base = op.dst;
    const uint64_t o_full = 3 * (uint64_t)(T - 1);                      // after round 0's input S-boxes
    const uint64_t o_part = o_full + 4 * (uint64_t)T * (half - 1);       // partial rounds
    const uint64_t o_last = o_part + 4 * (uint64_t)k.rp;                 // last full rounds
#pragma unroll 1
    for (int r = 0; r < half; r++) {
        if (j < T) {
            const fr29_t v = fr29_add(x, img[k.off_rc_first + r * T + j]);
            if (r == 0 && j == 0) x = fr29_sbox(v);  // the domain tag's first S-box: a constant, no variables
            else if (r == 0) x = sbox_emit(v, base + 3 * (uint64_t)(j - 1), false);
            else x = sbox_emit(v, base + o_full + 4 * (uint64_t)T * (r - 1) + 4 * (uint64_t)j, true);
        }
        x = group_row<T>(x, mds, j);
    }
    const fr29_t *sp = img + k.off_sparse;
#pragma unroll 1
    for (int q = 0; q < k.rp - 1; q++, sp += 2 * T - 1) {
        if (j == 0) x = sbox_emit(fr29_add(x, img[k.off_rc_part + q]), base + o_part + 4 * (uint64_t)q, true);
        const fr29_t s0 = shfl29(x, 0);
        fr29_t term = j < T ? fr29_mul(sp[j], x) : zero29();  // row_j s_j (s_0 after its S-box)
        MI_UNROLL for (int m = 1; m < 16; m <<= 1)
            term = fr29_sub_if_ge(fr29_add(term, shfl_xor29(term, m)), R2X29);
        if (j == 0) x = term;
        else if (j < T) x = fr29_sub_if_ge(fr29_add(x, fr29_mul(sp[T + j - 1], s0)), R2X29);
    }
    if (j == 0)
        x = sbox_emit(fr29_add(x, img[k.off_rc_part + k.rp - 1]), base + o_part + 4 * (uint64_t)(k.rp - 1), true);
    x = group_row<T>(x, img + k.off_dense, j);
#pragma unroll 1
    for (int r = 0; r < half; r++) {
        if (j < T)
            x = sbox_emit(fr29_add(x, img[k.off_rc_last + r * T + j]), base + o_last + 4 * (uint64_t)T * r + 4 * (uint64_t)j,
                          true);
        x = group_row<T>(x, mds, j);
    }
    if (j == 1) {
        if (EXPAND) zput29(z, base + o_last + 4 * (uint64_t)T * half, x);
        else zput_fr(z, op.b, fr_from_fr29(fr29_from_mont(x)));
    }
}

template <bool EXPAND>
void launch_poseidon(int kind, hipStream_t st, const WOp *ops, const uint64_t *idx, uint64_t n, const uint64_t *pin,
                     const PosKs &pk, fr_t *z) {
    const unsigned g = (unsigned)((n + 63) / 64);
    // 16 lanes per hash shorten a hash 4-5x but use T of 16 lanes: the form for launches too small to fill the
    // chip with one thread per hash (phase A levels -- 23 K hashes per level of the Window-PoSt partition are 367
    // waves for 1,024 SIMDs --, the stacked partition's 3,151 and the Winning-PoSt proof's 726 phase-B gadgets).
    // The Window-PoSt partition's 237 K phase-B gadgets (3.7 K waves) keep one thread per hash: on lanes they
    // took 17.5 ms instead of 6.  tune::WIT_POS_LANES (A/B): the largest launch on lanes, 0 = never.
    const int64_t lm = tune::get(tune::WIT_POS_LANES, 65536);
    const uint64_t lanes_max = lm < 0 ? 0 : (uint64_t)lm;
    if (n <= lanes_max) {
        const unsigned g4 = (unsigned)((n + 3) / 4);
        switch (kind) {
            case 1: k_wit_poseidon_lanes<3, EXPAND><<<g4, 64, 0, st>>>(ops, idx, n, pin, pk.k[0], z); break;
            case 2: k_wit_poseidon_lanes<5, EXPAND><<<g4, 64, 0, st>>>(ops, idx, n, pin, pk.k[1], z); break;
            case 3: k_wit_poseidon_lanes<9, EXPAND><<<g4, 64, 0, st>>>(ops, idx, n, pin, pk.k[2], z); break;
            default: k_wit_poseidon_lanes<12, EXPAND><<<g4, 64, 0, st>>>(ops, idx, n, pin, pk.k[3], z); break;
        }
        return;
    }
    switch (kind) {
        case 1: k_wit_poseidon<3, EXPAND><<<g, 64, 0, st>>>(ops, idx, n, pin, pk.k[0], z); break;
        case 2: k_wit_poseidon<5, EXPAND><<<g, 64, 0, st>>>(ops, idx, n, pin, pk.k[1], z); break;
        case 3: k_wit_poseidon<9, EXPAND><<<g, 64, 0, st>>>(ops, idx, n, pin, pk.k[2], z); break;
        default: k_wit_poseidon<12, EXPAND><<<g, 64, 0, st>>>(ops, idx, n, pin, pk.k[3], z); break;
    }
}

template <class T>
T *upload(const std::vector<T> &v) {
    T *d = nullptr;
    MI_HIP(hipMalloc(&d, sizeof(T) * (v.empty() ? 1 : v.size())));
    if (!v.empty()) MI_HIP(hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
    return d;
}

// every Built holding device programs, so a context's programs go when the context does (forget_ctx)
std::mutex g_built_mu;
std::vector<Built *> g_built;

DevProg *prog_for(Ctx &c, Built &b) {
    std::lock_guard<std::mutex> lk(b.dev_mu);
    for (auto &e : b.dev_progs)
        if (e.first == c.uid) return (DevProg *)e.second;
    if (b.dev_progs.empty()) {
        std::lock_guard<std::mutex> g(g_built_mu);
        g_built.push_back(&b);
    }
    DevProg *p = new DevProg();
    try {
        p->device = c.device;
        p->ops = upload(b.ops);
        p->pin = upload(b.pin);
        p->blocks = upload(b.blocks);
        std::vector<uint64_t> by;
        const unsigned ar[4] = {2, 4, 8, 11};
        for (int q = 0; q < 4; q++) {
            p->pos_off[q] = by.size();
            for (uint64_t o : b.poseidon_ops)
                if (b.ops[o].n == ar[q]) by.push_back(o);
        }
        p->pos_off[4] = by.size();
        p->pos_ops = upload(by);
        MI_HIP(hipMalloc(&p->states, 32 * (b.blocks.empty() ? 1 : b.blocks.size())));
        for (int q = 0; q < 4; q++) poseidon_tables(c, ar[q], &p->pk.k[q]);
        b.dev_progs.emplace_back(c.uid, p);
    } catch (...) {
        delete p;
        throw;
    }
    return p;
}

unsigned grid64(uint64_t n) { return (unsigned)((n + 63) / 64); }

}  // namespace

Built::~Built() {
    {
        std::lock_guard<std::mutex> g(g_built_mu);
        for (size_t i = 0; i < g_built.size(); i++)
            if (g_built[i] == this) {
                g_built.erase(g_built.begin() + i);
                break;
            }
    }
    for (auto &e : dev_progs) delete (DevProg *)e.second;
}

// A destroyed context's device programs (their ops, pin lists and SHA state scratch, and the views of its
// Poseidon tables, which poseidon_free releases) are dropped from every circuit (long-lived circuits
// with many short-lived contexts used to keep them all).
void forget_ctx(uint64_t uid) {
    std::lock_guard<std::mutex> g(g_built_mu);
    for (size_t i = 0; i < g_built.size();) {
        Built *b = g_built[i];
        std::lock_guard<std::mutex> lk(b->dev_mu);
        for (size_t j = 0; j < b->dev_progs.size();)
            if (b->dev_progs[j].first == uid) {
                delete (DevProg *)b->dev_progs[j].second;
                b->dev_progs.erase(b->dev_progs.begin() + j);
            } else {
                j++;
            }
        if (b->dev_progs.empty()) g_built.erase(g_built.begin() + i);
        else i++;
    }
}

void witness_dev(Ctx &c, Built &b, const uint8_t *slots_dev, fr_t *z_dev) {
    DevProg *p = prog_for(c, b);
    hipStream_t st = c.stream;
    static const fr_t one = [] {
        fr_t x = fr_t::zero();
        x.v[0] = 1;
        return x;
    }();
    MI_HIP(hipMemcpyAsync(z_dev, &one, 32, hipMemcpyHostToDevice, st));
    {
        ScopedTimer tm(c, &c.stats.wit_a, b.ops.size());
        for (size_t L = 0; L + 1 < b.level_off.size(); L++)
            for (int kind = 0; kind < 5; kind++) {
                const uint64_t o = b.seg_off[5 * L + kind], n = b.seg_off[5 * L + kind + 1] - o;
                if (!n) continue;
                if (kind == 0) {
                    k_wit_level<<<grid64(n), 64, 0, st>>>(p->ops + o, n, slots_dev, p->blocks, p->states, z_dev);
                    MI_LAUNCHED(c, "k_wit_level");
                } else {
                    launch_poseidon<false>(kind, st, p->ops + o, nullptr, n, p->pin, p->pk, z_dev);
                    MI_LAUNCHED(c, "k_wit_poseidon (phase A)");
                }
            }
    }
    if (!b.blocks.empty()) {
        ScopedTimer tm(c, &c.stats.wit_sha, b.blocks.size());
        k_wit_sha_blocks<<<grid64(b.blocks.size()), 64, 0, st>>>(p->blocks, b.blocks.size(), p->states, slots_dev, z_dev);
        MI_LAUNCHED(c, "k_wit_sha_blocks");
    }
    if (!b.poseidon_ops.empty()) {
        ScopedTimer tm(c, &c.stats.wit_pos, b.poseidon_ops.size());
        for (int q = 0; q < 4; q++) {
            const uint64_t n = p->pos_off[q + 1] - p->pos_off[q];
            if (!n) continue;
            launch_poseidon<true>(q + 1, st, p->ops, p->pos_ops + p->pos_off[q], n, p->pin, p->pk, z_dev);
            MI_LAUNCHED(c, "k_wit_poseidon (phase B)");
        }
    }
    MI_HIP(hipStreamSynchronize(st));
    c.timer.resolve();
}

}  // namespace stacked
}  // namespace mi
