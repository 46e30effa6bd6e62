// prover.hip -- Groth16 prove (bellman/crypto3 r1cs_gg_ppzksnark semantics) on one MI355X.
//
// The reference boundary is the crypto3 prover call inside compound_proof::circuit_proofs /
// prove (libs/storage/include/nil/filecoin/storage/proofs/core/proof/compound_proof.hpp:89-95,
// 127-137; bodies are stubs in the reference and the prover itself is [NOT IN TREE]).  This file
// restates that prover:
//   witness map (bellman ProvingAssignment / libsnark r1cs_to_qap_witness_map):
//     a_j, b_j, c_j = <A_j,z>, <B_j,z>, <C_j,z> for the n circuit rows, then one row "x_i * 0 = 0"
//     per public input (a = x_i), zero padded to d = 2^ceil(log2(n + n_in));
//     a,b,c <- coset_fft(ifft(.)); h_ev = (a*b - c) / (g^d - 1); H = icoset_fft(h_ev)[0..d-2]
//   multiexps: H (h query), L (aux), A (inputs + aux with A-density), B_G1 / B_G2 (B-density)
//   A = alpha + sum_A + r delta1; B = beta2 + sum_B2 + s delta2;
//   C = rs delta1 + s alpha + r beta1 + s sum_A + r sum_B1 + H + L.
// Proof wire format: compressed A (48) | B (96) | C (48) = 192 bytes (proofs/constants.hpp:93).
#include <hipcub/hipcub.hpp>

#include <string.h>

#include <atomic>
#include <exception>
#include <cstring>
#include <future>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>

#include "prover.h"
#include "hostfield.h"
#include <future>

namespace mi {

namespace {

inline unsigned grid1(uint64_t n) { return (unsigned)((n + 255) / 256); }

fr_t fr_small_mont(uint32_t v) {
    fr_t r = fr_t::zero();
    r.v[0] = v;
    return to_mont(r);
}

// ------------------------------------------------------------------------------ witness map
// (A z)_j, (B z)_j, (C z)_j for j < n, one matrix per launch.  Real circuits mix rows of 1-3 terms with
// rows of hundreds (SHA-256 packing, bit decompositions, the Poseidon gadget's linear combinations): one
// thread per row left most lanes of a wave idle behind its longest row (the stacked circuit's A matrix:
// 23x the useful work).  So a wave takes a block of consecutive rows holding <= EVAL_BLOCK entries (and
// rows): its lanes form the products entry-parallel (coalesced col / cidx loads, coefficient table in L2,
// the multiplication skipped for coefficient 1) into LDS, then sum their rows from LDS.  A row with more
// entries is a block of its own, reduced across the wave.
constexpr unsigned EVAL_BLOCK = 256;  // entries (and rows) per wave block: 4 per lane

__device__ __forceinline__ fr_t eval_term(const uint32_t *__restrict__ col, const uint32_t *__restrict__ cidx,
                                          const fr_t *__restrict__ ctab, const fr_t *__restrict__ zm, uint64_t e) {
    const uint32_t ci = cidx[e];
    const fr_t zv = zm[col[e]];
    return ci == 0 ? zv : ctab[ci] * zv;
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ void __launch_bounds__(256) k_eval_blocks(const uint64_t *__restrict__ rp, const uint32_t *__restrict__ col,
                                                     const uint32_t *__restrict__ cidx, const fr_t *__restrict__ ctab,
                                                     const fr_t *__restrict__ zm, const uint32_t *__restrict__ blk,
                                                     uint64_t nblk, fr_t *__restrict__ out) {
    __shared__ fr_t prod[4][EVAL_BLOCK];
    const unsigned w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t b = (uint64_t)blockIdx.x * 4 + w;
    if (b >= nblk) return;  // whole waves only: no workgroup barrier below
    const uint32_t r0 = blk[b], r1 = blk[b + 1];
    const uint64_t e0 = rp[r0], e1 = rp[r1];
    if (e1 - e0 > EVAL_BLOCK) {  // one long row: lane partial sums, then a butterfly across the wave
        fr_t acc = fr_t::zero();
        for (uint64_t e = e0 + lane; e < e1; e += 64) acc = acc + eval_term(col, cidx, ctab, zm, e);
        MI_UNROLL for (int off = 32; off >= 1; off >>= 1) {
            fr_t o;
            MI_UNROLL for (int i = 0; i < 8; i++) o.v[i] = __shfl_xor(acc.v[i], off, 64);
            acc = acc + o;
        }
        if (lane == 0) out[r0] = acc;
        return;
    }
    fr_t *p = prod[w];
    MI_UNROLL for (unsigned k = 0; k < EVAL_BLOCK / 64; k++) {
        const uint64_t e = e0 + lane + 64 * k;
        if (e < e1) p[lane + 64 * k] = eval_term(col, cidx, ctab, zm, e);
    }
    wave_lds_sync();
    for (uint32_t r = r0 + lane; r < r1; r += 64) {
        const uint32_t lo = (uint32_t)(rp[r] - e0), hi = (uint32_t)(rp[r + 1] - e0);
        fr_t s = fr_t::zero();
        for (uint32_t q = lo; q < hi; q++) s = s + p[q];
        out[r] = s;
    }
}

// rows n .. d - 1: the input rows (A = z_i, bellman's input constraints) and the zero padding
__global__ void k_eval_tail(const fr_t *__restrict__ zm, uint64_t n, uint64_t n_in, uint64_t d, fr_t *__restrict__ a,
                            fr_t *__restrict__ b, fr_t *__restrict__ c) {
    const uint64_t j = n + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d) return;
    a[j] = j < n + n_in ? zm[j - n] : fr_t::zero();
    b[j] = fr_t::zero();
    c[j] = fr_t::zero();
}

void eval_witness_map(Ctx &c, const Circuit &C, const fr_t *zm, fr_t *a, fr_t *b, fr_t *cc) {
    fr_t *outs[3] = {a, b, cc};
    for (int m = 0; m < 3; m++)
        if (C.n_blk[m])
            k_eval_blocks<<<(unsigned)((C.n_blk[m] + 3) / 4), 256, 0, c.stream>>>(
                C.row_ptr[m], C.col[m], C.cidx[m], C.ctab, zm, C.blk[m], C.n_blk[m], outs[m]);
    if (C.d > C.n)
        k_eval_tail<<<(unsigned)((C.d - C.n + 255) / 256), 256, 0, c.stream>>>(zm, C.n, C.n_in, C.d, a, b, cc);
    MI_HIP(hipGetLastError());
}

// R1CS satisfaction: rows j with (A z)_j (B z)_j != (C z)_j counted, the first one kept
__global__ void k_check_rows(const uint64_t *__restrict__ rp0, const uint32_t *__restrict__ c0,
                             const uint32_t *__restrict__ k0, const uint64_t *__restrict__ rp1,
                             const uint32_t *__restrict__ c1, const uint32_t *__restrict__ k1,
                             const uint64_t *__restrict__ rp2, const uint32_t *__restrict__ c2,
                             const uint32_t *__restrict__ k2, const fr_t *__restrict__ ctab,
                             const fr_t *__restrict__ zm, uint64_t n, unsigned long long *__restrict__ out) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    fr_t va = fr_t::zero(), vb = fr_t::zero(), vc = fr_t::zero();
    for (uint64_t e = rp0[j]; e < rp0[j + 1]; e++) va = va + ctab[k0[e]] * zm[c0[e]];
    for (uint64_t e = rp1[j]; e < rp1[j + 1]; e++) vb = vb + ctab[k1[e]] * zm[c1[e]];
    for (uint64_t e = rp2[j]; e < rp2[j + 1]; e++) vc = vc + ctab[k2[e]] * zm[c2[e]];
    if (!(va * vb == vc)) {
        atomicAdd(&out[0], 1ull);
        atomicMin(&out[1], (unsigned long long)j);
    }
}

__global__ void k_qap_divide(fr_t *__restrict__ a, const fr_t *__restrict__ b, const fr_t *__restrict__ c,
                             uint64_t d, fr_t zinv) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d) return;
    a[i] = (a[i] * b[i] - c[i]) * zinv;
}

__global__ void k_copy_to_mont(const fr_t *__restrict__ in, fr_t *__restrict__ out, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = to_mont(in[i]);
}

// h_perm[pos] = h[bitrev(pos)], pos < d - 1
__global__ void k_permute_h(const g1_affine_t *__restrict__ h, g1_affine_t *__restrict__ hp, unsigned L,
                            uint64_t m) {
    uint64_t pos = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= m) return;
    uint64_t r = L ? (__builtin_bitreverse64(pos) >> (64 - L)) : 0;
    hp[pos] = h[r];
}

// ------------------------------------------------------------------------------ param generation
// powers: out[i] = LO[i & 0xffff] * HI[i >> 16]
__global__ void k_powers(const fr_t *__restrict__ lo, const fr_t *__restrict__ hi, uint64_t n, fr_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = lo[i & 0xffff] * hi[i >> 16];
}
// h scalars in bit-reversed position order: hs[pos] = pw[bitrev(pos)] * coeff (canonical out)
__global__ void k_h_scalars(const fr_t *__restrict__ pw, unsigned L, uint64_t m, fr_t coeff, fr_t *__restrict__ hs) {
    uint64_t pos = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= m) return;
    uint64_t r = L ? (__builtin_bitreverse64(pos) >> (64 - L)) : 0;
    hs[pos] = from_mont(pw[r] * coeff);
}
__global__ void k_entry_rows(const uint64_t *__restrict__ rp, uint64_t n, uint32_t *__restrict__ rows) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    for (uint64_t e = rp[j]; e < rp[j + 1]; e++) rows[e] = (uint32_t)j;
}
__global__ void k_iota(uint32_t *__restrict__ x, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = (uint32_t)i;
}
__global__ void k_col_bounds(const uint32_t *__restrict__ cols, uint64_t nnz, uint32_t *__restrict__ start,
                             uint32_t *__restrict__ end) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nnz) return;
    uint32_t k = cols[i];
    if (i == 0 || cols[i - 1] != k) start[k] = (uint32_t)i;
    if (i == nnz - 1 || cols[i + 1] != k) end[k] = (uint32_t)i + 1;
}
// out[v] = sum over entries e of column v: coeff[e] * lag[row[e]]   (Montgomery)
__global__ void k_col_sums(const uint32_t *__restrict__ start, const uint32_t *__restrict__ end,
                           const uint32_t *__restrict__ perm, const uint32_t *__restrict__ rows,
                           const fr_t *__restrict__ coeff, const fr_t *__restrict__ lag, uint64_t nv,
                           fr_t *__restrict__ out) {
    uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nv) return;
    fr_t acc = fr_t::zero();
    for (uint32_t p = start[v]; p < end[v]; p++) {
        uint32_t e = perm[p];
        acc = acc + coeff[e] * lag[rows[e]];
    }
    out[v] = acc;
}
// prod[p] = coeff[perm[p]] * lag[rows[perm[p]]]   (entries in column-sorted order)
__global__ void k_entry_products(const uint32_t *__restrict__ perm, const uint32_t *__restrict__ rows,
                                 const uint32_t *__restrict__ cidx, const fr_t *__restrict__ ctab,
                                 const fr_t *__restrict__ lag, uint64_t nnz, fr_t *__restrict__ prod) {
    uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nnz) return;
    uint32_t e = perm[p];
    prod[p] = ctab[cidx[e]] * lag[rows[e]];
}
__global__ void k_scatter_runs(const uint32_t *__restrict__ keys, const fr_t *__restrict__ vals,
                               const uint32_t *__restrict__ nruns, fr_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < *nruns) out[keys[i]] = vals[i];
}
struct FrAdd {
    MI_HD fr_t operator()(const fr_t &a, const fr_t &b) const { return a + b; }
};
__global__ void k_add_input_rows(fr_t *__restrict__ at, const fr_t *__restrict__ lag, uint64_t n, uint64_t n_in) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_in) at[i] = at[i] + lag[n + i];
}
// ext[v] = (beta at + alpha bt + ct) * inv  -> canonical
__global__ void k_lc_scalars(const fr_t *__restrict__ at, const fr_t *__restrict__ bt, const fr_t *__restrict__ ct,
                             uint64_t off, uint64_t n, fr_t alpha, fr_t beta, fr_t inv, fr_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t v = off + i;
    out[i] = from_mont((beta * at[v] + alpha * bt[v] + ct[v]) * inv);
}
// Srs::a_aux: A point j (an aux variable's, j >= n_in: idx[j] - n_in) moves to its aux position; the rest stays the
// affine infinity (0, 0) of the zero-filled array
__global__ void k_gather_a_aux(const g1_affine_t *__restrict__ a, const uint32_t *__restrict__ idx, uint64_t m,
                               uint64_t n_in, uint64_t n_aux, g1_affine_t *__restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint64_t v = (uint64_t)idx[j] - n_in;
    if (v < n_aux) out[v] = a[j];
}

// Circuit::a_rank: a_rank[idx[r] - n_in] = r over the aux part of the A density (idx = idx_a + n_in, m entries)
__global__ void k_a_rank(const uint32_t *__restrict__ idx, uint64_t m, uint64_t n_in, uint64_t n_aux,
                         uint32_t *__restrict__ rank) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const uint64_t v = (uint64_t)idx[r] - n_in;
    if (v < n_aux) rank[v] = (uint32_t)r;
}

// Circuit::a_bits from a_rank: group g's density bits (word 2g) and their count (cnt[g], scanned into word 2g + 1)
__global__ void k_a_bits(const uint32_t *__restrict__ rank, uint64_t n_aux, uint64_t ng, uint32_t *__restrict__ bits,
                         uint32_t *__restrict__ cnt) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ng) return;
    uint32_t m = 0;
    for (unsigned k = 0; k < 32; k++) {
        const uint64_t v = 32 * g + k;
        if (v < n_aux && rank[v] != 0xffffffffu) m |= 1u << k;
    }
    bits[2 * g] = m;
    cnt[g] = __popc(m);
}
__global__ void k_a_bits_prefix(const uint32_t *__restrict__ pre, uint64_t ng, uint32_t *__restrict__ bits) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g < ng) bits[2 * g + 1] = pre[g];
}

__global__ void k_gather_canon(const fr_t *__restrict__ src, const uint32_t *__restrict__ idx, uint64_t n,
                               fr_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = from_mont(src[idx[i]]);
}

template <class F>
MI_HD uint32_t byte_of(const fr_t &s, unsigned j) {
    uint32_t w = 0;
    MI_UNROLL for (int q = 0; q < 8; q++) w = (j >> 2) == (unsigned)q ? s.v[q] : w;
    return (w >> (8 * (j & 3))) & 0xff;
}

// table[j*255 + m-1] = (m * 2^(8j)) * G, affine
template <class F>
__global__ void k_fb_table(Affine<F> G, Affine<F> *__restrict__ table) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 32 * 255) return;
    uint32_t j = t / 255, m = t % 255 + 1;
    uint32_t k[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned bit = 8 * j;
    k[bit / 32] |= m << (bit % 32);
    if (bit % 32 > 24 && bit / 32 + 1 < 9) k[bit / 32 + 1] |= m >> (32 - bit % 32);
    XYZZ<F> p = xyzz_mul_inl(xyzz_from_affine(G), k, 8);
    table[t] = xyzz_to_affine_inl(p);
}

template <class F>
__global__ void __launch_bounds__(256) k_fixed_base(const fr_t *__restrict__ k, uint64_t n,
                                                    const Affine<F> *__restrict__ table, XYZZ<F> *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fr_t s = k[i];
    XYZZ<F> acc = XYZZ<F>::inf();
#pragma unroll 1
    for (unsigned j = 0; j < 32; j++) {
        uint32_t m = byte_of<F>(s, j);
        if (m) acc = xyzz_add_affine_inl(acc, table[j * 255 + m - 1]);
    }
    out[i] = acc;
}

// batch XYZZ -> affine with Montgomery's trick over K consecutive points per thread
template <class F, int K>
__global__ void __launch_bounds__(256) k_batch_affine(const XYZZ<F> *__restrict__ in, uint64_t n,
                                                      F *__restrict__ pre, Affine<F> *__restrict__ out) {
    uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t beg = t * K;
    if (beg >= n) return;
    uint64_t end = beg + K < n ? beg + K : n;
    F prod = F::one();
    for (uint64_t i = beg; i < end; i++) {
        pre[i] = prod;
        XYZZ<F> p = in[i];
        if (!p.is_inf()) prod = prod * p.ZZZ;
    }
    F inv = inverse_inl(prod);
    for (uint64_t i = end; i-- > beg;) {
        XYZZ<F> p = in[i];
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

// 2^128 * P, XYZZ (128 doublings); batch-normalised by k_batch_affine
template <class F>
__global__ void __launch_bounds__(256) k_shift(const Affine<F> *__restrict__ in, uint64_t n, unsigned bits,
                                               XYZZ<F> *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    XYZZ<F> p = xyzz_from_affine(in[i]);
    for (unsigned k = 0; k < bits; k++) p = xyzz_dbl_inl(p);
    out[i] = p;
}

// block-level partial dot products sum z_i * e_i (z canonical -> montgomery on the fly)
__global__ void k_dot(const fr_t *__restrict__ z, const fr_t *__restrict__ e, uint64_t off, uint64_t n,
                      fr_t *__restrict__ partial) {
    __shared__ fr_t sh[256];
    fr_t acc = fr_t::zero();
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        acc = acc + to_mont(z[off + i]) * e[off + i];
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (unsigned h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) sh[threadIdx.x] = sh[threadIdx.x] + sh[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}

// ------------------------------------------------------------------------------ host helpers
void fq_to_be48(const fq_t &mont, uint8_t *out) {
    fq32_t raw = fq_to_raw(mont);
    for (int i = 0; i < 12; i++) {
        uint32_t w = raw.v[i];
        uint8_t *p = out + 4 * (11 - i);
        p[0] = (uint8_t)(w >> 24);
        p[1] = (uint8_t)(w >> 16);
        p[2] = (uint8_t)(w >> 8);
        p[3] = (uint8_t)w;
    }
}
bool fq_from_be48_host(const uint8_t *p, bool mask, fq_t &out) {
    fq32_t raw;
    for (int i = 0; i < 12; i++) {
        const uint8_t *q = p + 4 * (11 - i);
        uint32_t w = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
        if (i == 11 && mask) w &= 0x1fffffffu;
        raw.v[i] = w;
    }
    if (geq_raw(raw, fq32_t::modulus_raw())) return false;
    out = fq_from_raw(raw);
    return true;
}
bool fq_lex_largest(const fq_t &y) {
    fq32_t a = fq_to_raw(y), b = fq_to_raw(-y);
    for (int i = 11; i >= 0; i--)
        if (a.v[i] != b.v[i]) return a.v[i] > b.v[i];
    return false;
}

template <class T>
T *dalloc(uint64_t count) {
    T *p = nullptr;
    if (count) MI_HIP(hipMalloc(&p, sizeof(T) * count));
    return p;
}

template <class F>
Affine<F> host_mul_affine(const Affine<F> &p, const fr_t &k_raw) {
    return host::xyzz_to_affine(host::xyzz_mul(xyzz_from_affine(p), k_raw.v, 8));
}

}  // namespace

// ================================================================================ encodings
void g1_encode(const g1_affine_t &a, uint8_t out[96]) {
    if (a.is_inf()) {
        memset(out, 0, 96);
        out[0] = 0x40;
        return;
    }
    fq_to_be48(a.x, out);
    fq_to_be48(a.y, out + 48);
}
void g2_encode(const g2_affine_t &a, uint8_t out[192]) {
    if (a.is_inf()) {
        memset(out, 0, 192);
        out[0] = 0x40;
        return;
    }
    fq_to_be48(a.x.c1, out);
    fq_to_be48(a.x.c0, out + 48);
    fq_to_be48(a.y.c1, out + 96);
    fq_to_be48(a.y.c0, out + 144);
}
void g1_compress(const g1_affine_t &a, uint8_t out[48]) {
    if (a.is_inf()) {
        memset(out, 0, 48);
        out[0] = 0xc0;
        return;
    }
    fq_to_be48(a.x, out);
    out[0] |= 0x80;
    if (fq_lex_largest(a.y)) out[0] |= 0x20;
}
void g2_compress(const g2_affine_t &a, uint8_t out[96]) {
    if (a.is_inf()) {
        memset(out, 0, 96);
        out[0] = 0xc0;
        return;
    }
    fq_to_be48(a.x.c1, out);
    fq_to_be48(a.x.c0, out + 48);
    out[0] |= 0x80;
    bool largest = a.y.c1.is_zero() ? fq_lex_largest(a.y.c0) : fq_lex_largest(a.y.c1);
    if (largest) out[0] |= 0x20;
}
// zcash from_uncompressed flag rules (see k_g1_decode): 0x80 clear; infinity = 0x40 with every other
// bit zero; the sort bit 0x20 clear on finite points.  The curve equation is the caller's check.
static int uncompressed_flags_host(const uint8_t *p, int len) {
    const uint8_t f = p[0];
    if (f & 0x80) return -1;
    if (f & 0x40) {
        uint32_t any = f & 0x3f;
        for (int k = 1; k < len; k++) any |= p[k];
        return any ? -1 : 1;
    }
    return (f & 0x20) ? -1 : 0;
}
bool g1_decode_host(const uint8_t in[96], g1_affine_t &out) {
    const int f = uncompressed_flags_host(in, 96);
    if (f < 0) return false;
    if (f == 1) {
        out = g1_affine_t::inf();
        return true;
    }
    return fq_from_be48_host(in, true, out.x) && fq_from_be48_host(in + 48, false, out.y);
}
bool g2_decode_host(const uint8_t in[192], g2_affine_t &out) {
    const int f = uncompressed_flags_host(in, 192);
    if (f < 0) return false;
    if (f == 1) {
        out = g2_affine_t::inf();
        return true;
    }
    return fq_from_be48_host(in, true, out.x.c1) && fq_from_be48_host(in + 48, false, out.x.c0) &&
           fq_from_be48_host(in + 96, false, out.y.c1) && fq_from_be48_host(in + 144, false, out.y.c0);
}
fr_t fr_from_le(const uint8_t in[32]) {
    fr_t r;
    memcpy(r.v, in, 32);
    return r;
}
void fr_to_le(const fr_t &raw, uint8_t out[32]) { memcpy(out, raw.v, 32); }

// ================================================================================ objects
Circuit::~Circuit() {
    for (int m = 0; m < 3; m++) {
        if (row_ptr[m]) hipFree(row_ptr[m]);
        if (col[m]) hipFree(col[m]);
        if (cidx[m]) hipFree(cidx[m]);
        if (blk[m]) hipFree(blk[m]);
    }
    if (ctab) hipFree(ctab);
    if (idx_a) hipFree(idx_a);
    if (idx_b) hipFree(idx_b);
    if (a_rank) hipFree(a_rank);
    if (a_bits) hipFree(a_bits);
}
namespace {
std::mutex g_keys_mu;
std::vector<Srs *> g_keys;  // every live proving key (Srs::device says where it lives)
}  // namespace

Srs::Srs(int dev) : device(dev) {}

// A key joins the registry (and becomes visible to another context's out-of-memory release) only once it is
// complete: generation and stream loads build their queries and tables with no lock held, so a half-built key in
// the registry could have its tables freed under the kernels still filling them.
void srs_publish(Srs *S) {
    std::lock_guard<std::mutex> lk(g_keys_mu);
    g_keys.push_back(S);
}

Srs::~Srs() {
    {
        std::lock_guard<std::mutex> lk(g_keys_mu);
        for (size_t i = 0; i < g_keys.size(); i++)
            if (g_keys[i] == this) {
                g_keys.erase(g_keys.begin() + i);
                break;
            }
    }
    void *ps[] = {h_perm, l, a, b_g1, b_g2, at, bt, ct, h_hi, l_hi, a_hi, a_aux, wt[0], wt[1], wt[2], wt[3], wt[4]};
    for (void *p : ps)
        if (p) hipFree(p);
}

namespace {
// witness-map blocks of one matrix (k_eval_blocks): consecutive rows while the block holds at most
// EVAL_BLOCK entries and rows; a row with more entries stands alone
std::vector<uint32_t> eval_blocks(const uint64_t *rp, uint64_t n) {
    std::vector<uint32_t> b;
    uint64_t r = 0;
    while (r < n) {
        b.push_back((uint32_t)r);
        const uint64_t e0 = rp[r];
        uint64_t q = r + 1;
        if (rp[q] - e0 <= EVAL_BLOCK)
            while (q < n && q - r < EVAL_BLOCK && rp[q + 1] - e0 <= EVAL_BLOCK) q++;
        r = q;
    }
    b.push_back((uint32_t)n);
    return b;
}
}  // namespace

Circuit *circuit_load_compact(Ctx &c, const R1csCompact &cs) {
    if (cs.n_in < 1) throw std::invalid_argument("circuit must have at least the ONE input");
    uint64_t nv = cs.n_in + cs.n_aux;
    if (nv >= 0x80000000ull) throw std::invalid_argument("too many variables");
    if (cs.n >= 0xffffffffull) throw std::invalid_argument("too many constraints");
    if (!cs.n_ctab || !cs.ctab) throw std::invalid_argument("empty coefficient table");
    {
        fr_t one = fr_t::zero();
        one.v[0] = 1;
        if (memcmp(cs.ctab[0].v, one.v, 32) != 0) throw std::invalid_argument("coefficient table must start with 1");
    }
    Circuit *C = new Circuit();
    try {
        C->n = cs.n;
        C->n_in = cs.n_in;
        C->n_aux = cs.n_aux;
        uint64_t rows = cs.n + cs.n_in;
        C->log_d = 0;
        while ((1ull << C->log_d) < rows) C->log_d++;
        C->d = 1ull << C->log_d;
        if (C->log_d > 31) throw std::invalid_argument("domain too large");
        std::vector<uint8_t> a_den(cs.n_aux, 0), b_in(cs.n_in, 0), b_aux(cs.n_aux, 0);
        std::vector<uint32_t> blocks[3];
        std::string err[3];
        {  // validation, density and witness-map blocks: one host thread per matrix
            std::vector<std::thread> th;
            for (int m = 0; m < 3; m++)
                th.emplace_back([&, m] {
                    const uint64_t *rp = cs.row_ptr[m];
                    if (rp[0] != 0) {
                        err[m] = "row_ptr[0] must be 0";
                        return;
                    }
                    for (uint64_t j = 0; j < cs.n; j++)
                        if (rp[j + 1] < rp[j]) {
                            err[m] = "row_ptr not monotone";
                            return;
                        }
                    const uint64_t nnz = rp[cs.n];
                    for (uint64_t e = 0; e < nnz; e++) {
                        const uint32_t v = cs.col[m][e];
                        if (v >= nv) {
                            err[m] = "column index out of range";
                            return;
                        }
                        if (cs.cidx[m][e] >= cs.n_ctab) {
                            err[m] = "coefficient index out of range";
                            return;
                        }
                        if (m == 0 && v >= cs.n_in) a_den[v - cs.n_in] = 1;
                        if (m == 1) (v < cs.n_in ? b_in[v] : b_aux[v - cs.n_in]) = 1;
                    }
                    blocks[m] = eval_blocks(rp, cs.n);
                });
            for (auto &t : th) t.join();
            for (auto &e : err)
                if (!e.empty()) throw std::invalid_argument(e);
        }
        for (int m = 0; m < 3; m++) {
            const uint64_t nnz = cs.row_ptr[m][cs.n];
            C->nnz[m] = nnz;
            C->row_ptr[m] = dalloc<uint64_t>(cs.n + 1);
            MI_HIP(hipMemcpy(C->row_ptr[m], cs.row_ptr[m], 8 * (cs.n + 1), hipMemcpyHostToDevice));
            C->n_blk[m] = blocks[m].size() - 1;
            C->blk[m] = dalloc<uint32_t>(blocks[m].size());
            MI_HIP(hipMemcpy(C->blk[m], blocks[m].data(), 4 * blocks[m].size(), hipMemcpyHostToDevice));
            if (nnz) {
                C->col[m] = dalloc<uint32_t>(nnz);
                C->cidx[m] = dalloc<uint32_t>(nnz);
                MI_HIP(hipMemcpy(C->col[m], cs.col[m], 4 * nnz, hipMemcpyHostToDevice));
                MI_HIP(hipMemcpy(C->cidx[m], cs.cidx[m], 4 * nnz, hipMemcpyHostToDevice));
            }
        }
        C->n_ctab = cs.n_ctab;
        C->ctab = dalloc<fr_t>(cs.n_ctab);
        MI_HIP(hipMemcpy(C->ctab, cs.ctab, 32 * cs.n_ctab, hipMemcpyHostToDevice));
        fr_canonicalize(c, C->ctab, cs.n_ctab);
        fr_to_mont_inplace(c, C->ctab, cs.n_ctab);
        std::vector<uint32_t> ia, ib;
        for (uint64_t i = 0; i < cs.n_in; i++) ia.push_back((uint32_t)i);
        for (uint64_t i = 0; i < cs.n_aux; i++)
            if (a_den[i]) ia.push_back((uint32_t)(cs.n_in + i));
        for (uint64_t i = 0; i < cs.n_in; i++)
            if (b_in[i]) ib.push_back((uint32_t)i);
        C->n_b_in = ib.size();
        for (uint64_t i = 0; i < cs.n_aux; i++)
            if (b_aux[i]) ib.push_back((uint32_t)(cs.n_in + i));
        C->n_a = ia.size();
        C->n_b = ib.size();
        C->idx_a = dalloc<uint32_t>(ia.size());
        MI_HIP(hipMemcpy(C->idx_a, ia.data(), 4 * ia.size(), hipMemcpyHostToDevice));
        if (C->n_a > cs.n_in && cs.n_aux) {
            C->a_rank = dalloc<uint32_t>(cs.n_aux);
            MI_HIP(hipMemsetAsync(C->a_rank, 0xff, 4 * cs.n_aux, c.stream));
            const uint64_t m = C->n_a - cs.n_in;
            k_a_rank<<<grid1(m), 256, 0, c.stream>>>(C->idx_a + cs.n_in, m, cs.n_in, cs.n_aux, C->a_rank);
            MI_HIP(hipGetLastError());
            const uint64_t ng = (cs.n_aux + 31) / 32;
            C->a_bits = dalloc<uint32_t>(2 * ng);
            uint32_t *cnt = c.scratch[0].as<uint32_t>(2 * ng), *pre = cnt + ng;
            k_a_bits<<<grid1(ng), 256, 0, c.stream>>>(C->a_rank, cs.n_aux, ng, C->a_bits, cnt);
            MI_HIP(hipGetLastError());
            size_t tb = 0;
            MI_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, pre, ng, c.stream));
            void *tmp = c.scratch[4].get(tb);
            MI_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, pre, ng, c.stream));
            k_a_bits_prefix<<<grid1(ng), 256, 0, c.stream>>>(pre, ng, C->a_bits);
            MI_HIP(hipGetLastError());
        }
        if (!ib.empty()) {
            C->idx_b = dalloc<uint32_t>(ib.size());
            MI_HIP(hipMemcpy(C->idx_b, ib.data(), 4 * ib.size(), hipMemcpyHostToDevice));
        }
        MI_HIP(hipStreamSynchronize(c.stream));
    } catch (...) {
        delete C;
        throw;
    }
    return C;
}

// Full-coefficient R1CS (the C-ABI's mi_r1cs): the 32-byte coefficients interned into a table (1 first),
// chunk-parallel with a per-chunk table merged afterwards (circuits use few distinct coefficients, so the
// per-entry cost is one small hash lookup behind a last-value check)
Circuit *circuit_load(Ctx &c, const R1csHost &cs) {
    struct Key {
        uint64_t w[4];
        bool operator==(const Key &o) const { return !memcmp(w, o.w, 32); }
    };
    struct KH {
        size_t operator()(const Key &k) const {
            return (size_t)((k.w[0] ^ (k.w[1] * 0x9e3779b97f4a7c15ull) ^ (k.w[2] << 7) ^ (k.w[3] >> 3)) *
                            0xff51afd7ed558ccdull);
        }
    };
    auto key_at = [](const uint8_t *p) {
        Key k;
        memcpy(k.w, p, 32);
        return k;
    };
    std::vector<uint32_t> cidx[3];
    std::vector<Key> table;
    std::unordered_map<Key, uint32_t, KH> index;
    Key one{{1, 0, 0, 0}};
    table.push_back(one);
    index.emplace(one, 0);
    const unsigned nt = 16;
    for (int m = 0; m < 3; m++) {
        const uint64_t nnz = cs.n ? cs.row_ptr[m][cs.n] : 0;
        cidx[m].resize(nnz);
        if (!nnz) continue;
        const uint8_t *co = cs.coeff[m];
        std::vector<std::vector<Key>> local(nt);
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; t++)
            th.emplace_back([&, t] {  // local indices first
                std::unordered_map<Key, uint32_t, KH> li;
                const uint64_t lo = nnz * t / nt, hi = nnz * (t + 1) / nt;
                Key last{};
                uint32_t last_i = ~0u;
                for (uint64_t e = lo; e < hi; e++) {
                    const Key k = key_at(co + 32 * e);
                    if (last_i != ~0u && k == last) {
                        cidx[m][e] = last_i;
                        continue;
                    }
                    auto it = li.find(k);
                    uint32_t i;
                    if (it == li.end()) {
                        i = (uint32_t)local[t].size();
                        local[t].push_back(k);
                        li.emplace(k, i);
                    } else {
                        i = it->second;
                    }
                    cidx[m][e] = i;
                    last = k;
                    last_i = i;
                }
            });
        for (auto &t : th) t.join();
        th.clear();
        std::vector<std::vector<uint32_t>> remap(nt);
        for (unsigned t = 0; t < nt; t++)
            for (const Key &k : local[t]) {
                auto it = index.find(k);
                if (it == index.end()) {
                    if (table.size() >= 0xffffffffull) throw std::invalid_argument("too many distinct coefficients");
                    it = index.emplace(k, (uint32_t)table.size()).first;
                    table.push_back(k);
                }
                remap[t].push_back(it->second);
            }
        for (unsigned t = 0; t < nt; t++)
            th.emplace_back([&, t] {
                const uint64_t lo = nnz * t / nt, hi = nnz * (t + 1) / nt;
                for (uint64_t e = lo; e < hi; e++) cidx[m][e] = remap[t][cidx[m][e]];
            });
        for (auto &t : th) t.join();
    }
    std::vector<fr_t> ctab(table.size());
    for (size_t i = 0; i < table.size(); i++) memcpy(ctab[i].v, table[i].w, 32);
    R1csCompact cc{cs.n, cs.n_in, cs.n_aux, {}, {}, {}, ctab.data(), ctab.size()};
    for (int m = 0; m < 3; m++) {
        cc.row_ptr[m] = cs.row_ptr[m];
        cc.col[m] = cs.col[m];
        cc.cidx[m] = cidx[m].data();
    }
    return circuit_load_compact(c, cc);
}

// Proving-key upload as a stream of chunks (mi_srs_stream_*; srs_load is begin + whole queries + end).
// Each chunk is decoded on the device with bellman's Parameters::read rules: canonical coordinates, on
// the curve, the identity refused in every query ("point at infinity"), and with checked = true also
// r P = O (from_uncompressed vs _unchecked) once the query is complete.  Chunks come from host memory
// (staged through a bounded buffer) or from device memory (a received RCCL broadcast buffer: decoded in
// place, no host copy).  Per query the chunks must arrive in order.
namespace {
void build_hi_tables(Ctx &c, Srs &S, const uint32_t *a_idx = nullptr, uint64_t n_in = 0, uint64_t n_aux = 0);
const char *kQueryName[5] = {"h", "l", "a", "b_g1", "b_g2"};
}

SrsStream *srs_stream_begin(Ctx &c, const Circuit *circ, const SrsHost &h, bool checked) {
    SrsStream *st = new SrsStream();
    Srs *S = st->S = new Srs(c.device);
    try {
        st->checked = checked;
        if (h.n_h < 1) throw std::invalid_argument("empty h query");
        uint64_t d = h.n_h + 1;
        if (d & (d - 1)) throw std::invalid_argument("|h| + 1 must be a power of two");
        S->d = d;
        while ((1ull << S->log_d) < d) S->log_d++;
        if (circ) {
            if (circ->d != d) throw std::invalid_argument("SRS domain does not match the circuit");
            if (h.n_l != circ->n_aux) throw std::invalid_argument("|l| != number of aux variables");
            if (h.n_a != circ->n_a) throw std::invalid_argument("|a| != A-density of the circuit");
            if (h.n_b_g1 != circ->n_b || h.n_b_g2 != circ->n_b)
                throw std::invalid_argument("|b_g1| / |b_g2| != B-density of the circuit");
            if (h.n_ic != circ->n_in) throw std::invalid_argument("|ic| != number of inputs");
            if (circ->n_a > circ->n_in && circ->idx_a) {  // for Srs::a_aux at end (build_a_aux)
                st->a_idx = dalloc<uint32_t>(circ->n_a);
                MI_HIP(hipMemcpyAsync(st->a_idx, circ->idx_a, 4 * circ->n_a, hipMemcpyDeviceToDevice, c.stream));
                st->n_in = circ->n_in;
                st->n_aux = circ->n_aux;
            }
        }
        if (h.n_b_g1 != h.n_b_g2) throw std::invalid_argument("|b_g1| != |b_g2|");
        S->n_h = h.n_h;
        S->n_l = h.n_l;
        S->n_a = h.n_a;
        S->n_b = h.n_b_g1;
        // verifying key and ic on the host: curve equation always, subgroup when checked; ic points are
        // refused at infinity like the queries (bellman VerifyingKey::read)
        auto g1_ok = [&](const g1_affine_t &p) { return p.is_inf() || (g1_on_curve(p) && (!checked || in_prime_subgroup(p))); };
        auto g2_ok = [&](const g2_affine_t &p) { return p.is_inf() || (g2_on_curve(p) && (!checked || in_prime_subgroup(p))); };
        bool ok = g1_decode_host(h.vk, S->alpha_g1) && g1_decode_host(h.vk + 96, S->beta_g1) &&
                  g2_decode_host(h.vk + 192, S->beta_g2) && g2_decode_host(h.vk + 384, S->gamma_g2) &&
                  g1_decode_host(h.vk + 576, S->delta_g1) && g2_decode_host(h.vk + 672, S->delta_g2);
        if (!ok) throw std::invalid_argument("bad verifying key encoding");
        if (!g1_ok(S->alpha_g1) || !g1_ok(S->beta_g1) || !g1_ok(S->delta_g1) || !g2_ok(S->beta_g2) ||
            !g2_ok(S->gamma_g2) || !g2_ok(S->delta_g2))
            throw std::invalid_argument("verifying key point not on the curve / outside the subgroup");
        S->n_ic = h.n_ic;
        S->ic.resize(h.n_ic);
        for (uint64_t i = 0; i < h.n_ic; i++) {
            if (!g1_decode_host(h.ic + 96 * i, S->ic[i])) throw std::invalid_argument("bad ic encoding");
            if (S->ic[i].is_inf()) throw std::invalid_argument("ic point at infinity");
            if (!g1_ok(S->ic[i])) throw std::invalid_argument("ic point not on the curve / outside the subgroup");
        }
        st->n[0] = S->n_h;
        st->n[1] = S->n_l;
        st->n[2] = S->n_a;
        st->n[3] = S->n_b;
        st->n[4] = S->n_b;
        st->dst[0] = st->hnat = dalloc<g1_affine_t>(S->n_h);
        st->dst[1] = S->l = S->n_l ? dalloc<g1_affine_t>(S->n_l) : nullptr;
        st->dst[2] = S->a = S->n_a ? dalloc<g1_affine_t>(S->n_a) : nullptr;
        st->dst[3] = S->b_g1 = S->n_b ? dalloc<g1_affine_t>(S->n_b) : nullptr;
        st->dst[4] = S->b_g2 = S->n_b ? dalloc<g2_affine_t>(S->n_b) : nullptr;
        st->bad = dalloc<int>(15);
        MI_HIP(hipMemsetAsync(st->bad, 0, 15 * sizeof(int), c.stream));
    } catch (...) {
        srs_stream_abort(st);
        throw;
    }
    return st;
}

void srs_stream_part(Ctx &c, SrsStream &st, int which, uint64_t first, const uint8_t *bytes, uint64_t n,
                     bool on_device) {
    if (which < 0 || which > 4) throw std::invalid_argument("which must be 0..4");
    if (first != st.filled[which]) throw std::invalid_argument("SRS stream chunks must arrive in order per query");
    if (n > st.n[which] - first) throw std::invalid_argument("SRS stream chunk runs past the end of the query");
    if (!n) return;
    const bool g2 = which == 4;
    const size_t esz = g2 ? 192 : 96;
    int *bad = st.bad + 3 * which;
    const uint64_t chunk = 1ull << 22;
    uint8_t *stage = on_device ? nullptr : c.scratch[0].as<uint8_t>(esz * (n < chunk ? n : chunk));
    for (uint64_t o = 0; o < n; o += chunk) {
        uint64_t m = n - o < chunk ? n - o : chunk;
        const uint8_t *src = bytes + esz * o;
        if (!on_device) {
            MI_HIP(hipMemcpyAsync(stage, src, esz * m, hipMemcpyHostToDevice, c.stream));
            src = stage;
        }
        if (g2)
            g2_decode_uncompressed(c, src, (g2_affine_t *)st.dst[which] + first + o, m, bad, true);
        else
            g1_decode_uncompressed(c, src, (g1_affine_t *)st.dst[which] + first + o, m, bad, true);
    }
    // the staging buffer (and a caller's device chunk) may be reused as soon as this returns
    MI_HIP(hipStreamSynchronize(c.stream));
    st.filled[which] += n;
}

Srs *srs_stream_end(Ctx &c, SrsStream *st) {
    Srs *S = st->S;
    try {
        for (int q = 0; q < 5; q++)
            if (st->filled[q] != st->n[q])
                throw std::invalid_argument(std::string("SRS ") + kQueryName[q] + " query incomplete: " +
                                            std::to_string(st->filled[q]) + " of " + std::to_string(st->n[q]) +
                                            " points received");
        if (st->checked) {
            for (int q = 0; q < 4; q++) g1_subgroup_check(c, (const g1_affine_t *)st->dst[q], st->n[q], st->bad + 3 * q);
            g2_subgroup_check(c, (const g2_affine_t *)st->dst[4], st->n[4], st->bad + 12);
        }
        int nbad[15];
        MI_HIP(hipMemcpyAsync(nbad, st->bad, sizeof(nbad), hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipStreamSynchronize(c.stream));
        for (int q = 0; q < 5; q++) {
            const int *b = nbad + 3 * q;
            std::string m = std::string("SRS ") + kQueryName[q] + " query: ";
            if (b[0]) throw std::invalid_argument(m + std::to_string(b[0]) + " malformed or off-curve point(s)");
            if (b[1]) throw std::invalid_argument(m + std::to_string(b[1]) + " point(s) at infinity");
            if (b[2]) throw std::invalid_argument(m + std::to_string(b[2]) + " point(s) outside the prime-order subgroup");
        }
        S->h_perm = dalloc<g1_affine_t>(S->n_h);
        k_permute_h<<<grid1(S->n_h), 256, 0, c.stream>>>(st->hnat, S->h_perm, S->log_d, S->n_h);
        MI_HIP(hipStreamSynchronize(c.stream));
        hipFree(st->hnat);
        st->hnat = nullptr;
        S->in_subgroup = st->checked;
        build_hi_tables(c, *S, st->a_idx, st->n_in, st->n_aux);
    } catch (...) {
        srs_stream_abort(st);
        throw;
    }
    st->S = nullptr;
    srs_stream_abort(st);
    srs_publish(S);
    return S;
}

void srs_stream_abort(SrsStream *st) {
    if (!st) return;
    if (st->hnat) hipFree(st->hnat);
    if (st->bad) hipFree(st->bad);
    if (st->a_idx) hipFree(st->a_idx);
    delete st->S;  // ~Srs frees the queries allocated so far
    delete st;
}

namespace {
Srs *srs_load_once(Ctx &c, const Circuit *circ, const SrsHost &h, bool checked) {
    SrsStream *st = srs_stream_begin(c, circ, h, checked);
    const uint8_t *q[5] = {h.h, h.l, h.a, h.b_g1, h.b_g2};
    try {
        for (int k = 0; k < 5; k++) srs_stream_part(c, *st, k, 0, q[k], st->n[k], false);
    } catch (...) {
        (void)hipStreamSynchronize(c.stream);
        srs_stream_abort(st);
        throw;
    }
    return srs_stream_end(c, st);
}
}  // namespace

// a load out of memory releases the other keys' split tables and the idle scratch and loads once more
// (srs_generate's rule)
Srs *srs_load(Ctx &c, const Circuit *circ, const SrsHost &h, bool checked) {
    try {
        return srs_load_once(c, circ, h, checked);
    } catch (const hip_error &e) {
        if (e.code != hipErrorOutOfMemory) throw;
        c.stats.oom_retries += 1;
        c.stats.oom_freed_bytes += release_for_retry(c, nullptr, nullptr);
        return srs_load_once(c, circ, h, checked);
    }
}

uint64_t circuit_check(Ctx &c, const Circuit &C, const fr_t *z_dev, uint64_t *first_bad) {
    const uint64_t nv = C.n_in + C.n_aux;
    fr_t *zm = c.scratch[1].as<fr_t>(nv ? nv : 1);
    unsigned long long *out = c.scratch[9].as<unsigned long long>(2);
    const unsigned long long init[2] = {0ull, ~0ull};
    MI_HIP(hipMemcpyAsync(out, init, sizeof init, hipMemcpyHostToDevice, c.stream));
    k_copy_to_mont<<<grid1(nv), 256, 0, c.stream>>>(z_dev, zm, nv);
    if (C.n)
        k_check_rows<<<grid1(C.n), 256, 0, c.stream>>>(C.row_ptr[0], C.col[0], C.cidx[0], C.row_ptr[1], C.col[1],
                                                      C.cidx[1], C.row_ptr[2], C.col[2], C.cidx[2], C.ctab, zm, C.n,
                                                      out);
    MI_HIP(hipGetLastError());
    unsigned long long h[2];
    MI_HIP(hipMemcpyAsync(h, out, sizeof h, hipMemcpyDeviceToHost, c.stream));
    MI_HIP(hipStreamSynchronize(c.stream));
    if (first_bad) *first_bad = h[1];
    return h[0];
}

// ------------------------------------------------------------------------------ fixed-base helper
template <class F>
static void fixed_base_affine(Ctx &c, const Affine<F> *table, const fr_t *k_dev, uint64_t n, Affine<F> *out) {
    if (!n) return;
    const uint64_t chunk = 1ull << 24;
    XYZZ<F> *tmp = c.scratch[10].as<XYZZ<F>>(n < chunk ? n : chunk);
    F *pre = c.scratch[11].as<F>(n < chunk ? n : chunk);
    for (uint64_t o = 0; o < n; o += chunk) {
        uint64_t m = n - o < chunk ? n - o : chunk;
        k_fixed_base<F><<<grid1(m), 256, 0, c.stream>>>(k_dev + o, m, table, tmp);
        constexpr int K = 32;
        k_batch_affine<F, K><<<grid1((m + K - 1) / K), 256, 0, c.stream>>>(tmp, m, pre, out + o);
        MI_HIP(hipGetLastError());
    }
}

// out[i] = 2^bits in[i] (affine), queued on c's stream
template <class F>
static void shift_async(Ctx &c, const Affine<F> *in, uint64_t n, unsigned bits, Affine<F> *out) {
    const uint64_t chunk = 1ull << 24;
    XYZZ<F> *tmp = c.scratch[10].as<XYZZ<F>>(n < chunk ? (n ? n : 1) : chunk);
    F *pre = c.scratch[11].as<F>(n < chunk ? (n ? n : 1) : chunk);
    for (uint64_t o = 0; o < n; o += chunk) {
        uint64_t m = n - o < chunk ? n - o : chunk;
        k_shift<F><<<grid1(m), 256, 0, c.stream>>>(in + o, m, bits, tmp);
        constexpr int K = 32;
        k_batch_affine<F, K><<<grid1((m + K - 1) / K), 256, 0, c.stream>>>(tmp, m, pre, out + o);
        MI_HIP(hipGetLastError());
    }
}

void g1_shift128(Ctx &c, const g1_affine_t *in, uint64_t n, g1_affine_t *out) {
    shift_async<fq_t>(c, in, n, 128, out);
    MI_HIP(hipStreamSynchronize(c.stream));
}

template <class F>
static void window_table(Ctx &c, const Affine<F> *bases, uint64_t n, unsigned wbits, Affine<F> *dst) {
    const unsigned nwin = (256 + wbits - 1) / wbits;
    if (n) MI_HIP(hipMemcpyAsync(dst, bases, n * sizeof(Affine<F>), hipMemcpyDeviceToDevice, c.stream));
    for (unsigned w = 1; w < nwin; w++)
        shift_async<F>(c, dst + (uint64_t)(w - 1) * n, n, wbits, dst + (uint64_t)w * n);
    MI_HIP(hipStreamSynchronize(c.stream));
}
void g1_window_table(Ctx &c, const g1_affine_t *bases, uint64_t n, unsigned wbits, g1_affine_t *dst) {
    window_table<fq_t>(c, bases, n, wbits, dst);
}
void g2_window_table(Ctx &c, const g2_affine_t *bases, uint64_t n, unsigned wbits, g2_affine_t *dst) {
    window_table<fq2_t>(c, bases, n, wbits, dst);
}

namespace {
// Fixed-base window tables (WinTable) of the four G1 queries of a small key: domain <= 2^tune::MSM_WT_MAX_LOG (default
// 2^21; 0 turns them off), and only while they leave a proof its working set (the split tables' admission rule).
// A key's MSMs then run over one bucket set per query (msm_run_wt).  Read at each build (tests compare both).
void build_window_tables(Ctx &c, Srs &S) {
    const int64_t wt_max = tune::get(tune::MSM_WT_MAX_LOG, 21);
    const unsigned max_log = wt_max >= 0 && wt_max < 64 ? (unsigned)wt_max : 21u;
    if (max_log == 0 || S.log_d > max_log || S.has_tables()) return;
    const void *src[5] = {S.h_perm, S.l, S.a, S.b_g1, S.b_g2};
    uint64_t big = 0;
    for (int q = 0; q < 5; q++) big = S.wt_points(q) > big ? S.wt_points(q) : big;
    const unsigned wc = msm_wt_window_bits(big);
    const unsigned nwin = (256 + wc - 1) / wc;
    uint64_t need = 0;
    for (int q = 0; q < 5; q++)
        need += src[q] ? S.wt_points(q) * nwin * (q == 4 ? sizeof(g2_affine_t) : sizeof(g1_affine_t)) : 0;
    size_t free_b = 0, total_b = 0;
    MI_HIP(hipMemGetInfo(&free_b, &total_b));
    // a proof's scratch: the witness and QAP vectors, and per lane (four on small proofs) a plan of nwin entries per
    // point (keys / values sorted and unsorted, sort space: ~32 B an entry)
    const uint64_t work = 32 * (S.n_l + 3 * S.d) + 4ull * 32 * nwin * big;
    if (need + work + (8ull << 30) > free_b) return;
    S.wt_c = wc;
    try {
        for (int q = 0; q < 5; q++) {
            const uint64_t n = S.wt_points(q);
            if (!src[q] || !n) continue;
            if (q == 4) {
                g2_affine_t *t = dalloc<g2_affine_t>(n * nwin);
                S.wt[q] = t;
                g2_window_table(c, S.b_g2, n, wc, t);
            } else {
                g1_affine_t *t = dalloc<g1_affine_t>(n * nwin);
                S.wt[q] = t;
                g1_window_table(c, (const g1_affine_t *)src[q], n, wc, t);
            }
        }
    } catch (const hip_error &e) {
        if (e.code != hipErrorOutOfMemory) throw;
        (void)hipStreamSynchronize(c.stream);
        (void)hipGetLastError();
        srs_drop_split_tables(S);
    }
}

// split-mode tables of the three G1 queries whose MSMs run alone (B_G1 shares B_G2's plan, which has
// no table on the G2 side, so b_g1 gets none)
void build_split_tables(Ctx &c, Srs &S) {
    if (msm_glv_mode() == 1) return;  // GLV split mode needs no table (glv.h)
    struct Q {
        const g1_affine_t *src;
        uint64_t n;
        g1_affine_t **dst;
    } qs[] = {{S.h_perm, S.n_h, &S.h_hi},
              {S.a_aux ? nullptr : S.l, S.n_l, &S.l_hi},  // with a_aux, L and A run over one GLV plan: no table
              {S.a_aux ? nullptr : S.a, S.n_a, &S.a_hi}};
    if (msm_glv_mode() == 2) {  // auto: tables only while they leave the prover its working set
        uint64_t need = 0;
        for (auto &q : qs) need += q.src && msm_use_split(q.n) ? q.n * sizeof(g1_affine_t) : 0;
        size_t free_b = 0, total_b = 0;
        MI_HIP(hipMemGetInfo(&free_b, &total_b));
        // a proof's scratch: the Montgomery witness and the three QAP vectors (32 (m + 3 d) bytes), and per
        // lane one split-mode MSM plan (keys / values sorted and unsorted over ~6 windows of 2 n half-scalar
        // points, chunk partials and sort space) over the larger of h and l: measured 109 GB in all for a
        // 2^27-domain Window-PoSt partition (tools/post_mem.py), i.e. ~350 B per point and lane
        // Reserve that estimate + 10 % + 8 GB: the padded 128 / 256-byte records (curve.h) left the 32 GiB
        // Window-PoSt partition with tables 6 GB short of its working set (out of memory in the prove)
        // under the round-3 estimate + 1 GB, and earlier legs' buffers fragment what is free.
        const uint64_t big = S.d > S.n_l ? S.d : S.n_l;
        const uint64_t work = 32 * (S.n_l + 3 * S.d) + 2 * 360 * big;
        if (need + work + work / 10 + (8ull << 30) > free_b) return;  // the MSMs take the GLV split instead
    }
    // the tables are an optimisation: if one cannot be allocated (the free-memory estimate was wrong, or memory
    // is fragmented), the key keeps none and its MSMs take the GLV split
    try {
        for (auto &q : qs) {
            if (!q.src || !q.n || !msm_use_split(q.n)) continue;  // a query its MSM never splits needs no table
            *q.dst = dalloc<g1_affine_t>(q.n);
            g1_shift128(c, q.src, q.n, *q.dst);
        }
    } catch (const hip_error &e) {
        if (e.code != hipErrorOutOfMemory) throw;
        (void)hipStreamSynchronize(c.stream);
        (void)hipGetLastError();
        srs_drop_split_tables(S);
    }
}

// Srs::a_aux (the shared L/A plan): for subgroup keys whose L MSM takes the split path, while the gathered query
// leaves a proof its working set (the split tables' admission rule, counted before them).  a_idx = the circuit's A
// density (bellman a_aux_density: every input, then the aux variables with A entries, ascending).
void build_a_aux(Ctx &c, Srs &S, const uint32_t *a_idx, uint64_t n_in, uint64_t n_aux) {
    if (!a_idx || !S.a || !S.in_subgroup || msm_glv_mode() == 0 || n_aux != S.n_l || S.n_a <= n_in ||
        !msm_use_split(n_aux))
        return;
    // A's accumulation over the shared plan also adds the infinity points of the aux variables without A density
    // (a full mixed addition each: a wave's lanes run in lockstep), so the plan it saves must outweigh them: a plan
    // costs ~25 ps per entry against ~130 ps per mixed addition (profiles/r06_*), break-even near 84 % density.
    // The Window-PoSt partition's A covers 99.6 % of its aux variables; the synthetic config-3 circuit's 66 %
    // (measured there: 480 ms per proof shared, 461 ms with separate plans over the split tables).
    if ((S.n_a - n_in) * 10 < n_aux * 9) return;
    size_t free_b = 0, total_b = 0;
    MI_HIP(hipMemGetInfo(&free_b, &total_b));
    const uint64_t need = n_aux * sizeof(g1_affine_t);
    const uint64_t big = S.d > S.n_l ? S.d : S.n_l;
    const uint64_t work = 32 * (S.n_l + 3 * S.d) + 2 * 360 * big;
    if (need + work + work / 10 + (8ull << 30) > free_b) return;
    try {
        S.a_aux = dalloc<g1_affine_t>(n_aux);
        MI_HIP(hipMemsetAsync(S.a_aux, 0, need, c.stream));
        const uint64_t m = S.n_a - n_in;
        k_gather_a_aux<<<grid1(m), 256, 0, c.stream>>>(S.a + n_in, a_idx + n_in, m, n_in, n_aux, S.a_aux);
        MI_HIP(hipGetLastError());
    } catch (const hip_error &e) {
        if (e.code != hipErrorOutOfMemory) throw;
        (void)hipStreamSynchronize(c.stream);
        (void)hipGetLastError();
        if (S.a_aux) (void)hipFree(S.a_aux);
        S.a_aux = nullptr;
    }
}

// every MSM table of a key: the window tables of a small key, else the gathered A query (when the circuit's A density
// is given) and the split tables
void build_hi_tables(Ctx &c, Srs &S, const uint32_t *a_idx, uint64_t n_in, uint64_t n_aux) {
    build_window_tables(c, S);
    if (S.has_tables()) return;
    build_a_aux(c, S, a_idx, n_in, n_aux);
    build_split_tables(c, S);
}
}  // namespace

namespace {
// a device temporary freed on every path (keygen retries after an out-of-memory error must not leak)
struct DevTemp {
    void *p = nullptr;
    template <class T>
    T *alloc(uint64_t count) {
        p = dalloc<T>(count);
        return (T *)p;
    }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
    }
    ~DevTemp() { reset(); }
};

Srs *srs_generate_once(Ctx &c, const Circuit &circ, const fr_t toxic_canonical[5]) {
    Srs *S = new Srs(c.device);
    hipStream_t st = c.stream;
    DevTemp pw_t, ks_t, t1_t, t2_t;
    try {
        const uint64_t d = circ.d, n = circ.n, nv = circ.n_in + circ.n_aux;
        const unsigned L = circ.log_d;
        S->d = d;
        S->log_d = L;
        fr_t tau = to_mont(toxic_canonical[0]), alpha = to_mont(toxic_canonical[1]),
             beta = to_mont(toxic_canonical[2]), gamma = to_mont(toxic_canonical[3]),
             delta = to_mont(toxic_canonical[4]);
        for (int i = 0; i < 5; i++) S->toxic[i] = toxic_canonical[i];
        S->has_trapdoor = true;
        S->in_subgroup = true;  // k G for known k: every point is in the prime-order subgroup
        // powers of tau via two 65536-entry tables
        std::vector<fr_t> lo(65536), hi(65536);
        lo[0] = fr_t::one();
        for (int i = 1; i < 65536; i++) lo[i] = lo[i - 1] * tau;
        fr_t t16 = lo[65535] * tau;
        hi[0] = fr_t::one();
        for (int i = 1; i < 65536; i++) hi[i] = hi[i - 1] * t16;
        fr_t *dlo = c.scratch[12].as<fr_t>(65536 * 2), *dhi = dlo + 65536;
        MI_HIP(hipMemcpyAsync(dlo, lo.data(), 32 * 65536, hipMemcpyHostToDevice, st));
        MI_HIP(hipMemcpyAsync(dhi, hi.data(), 32 * 65536, hipMemcpyHostToDevice, st));
        fr_t *pw = pw_t.alloc<fr_t>(d);
        k_powers<<<grid1(d), 256, 0, st>>>(dlo, dhi, d, pw);
        fr_t tau_d = pow_u64(tau, d);
        fr_t t_tau = tau_d - fr_t::one();
        fr_t delta_inv = inverse(delta), gamma_inv = inverse(gamma);
        // h query scalars (bit-reversed order) -> points
        fr_t *ks = ks_t.alloc<fr_t>(nv > d ? nv : d);
        k_h_scalars<<<grid1(d - 1), 256, 0, st>>>(pw, L, d - 1, t_tau * delta_inv, ks);
        // Lagrange coefficients L_j(tau) = ifft(powers)
        ntt_dif(c, pw, L, true);
        bitrev_permute(c, pw, L);
        fr_t draw = fr_t::zero();
        draw.v[0] = (uint32_t)d;
        draw.v[1] = (uint32_t)(d >> 32);
        fr_t dinv = inverse(to_mont(draw));
        scale_all(c, pw, d, dinv);
        fr_t *lag = pw;
        // tables for fixed-base multiplication
        g1_affine_t g1;
        g2_affine_t g2;
        {
            static const uint8_t g1b[96] = {
                0x17, 0xf1, 0xd3, 0xa7, 0x31, 0x97, 0xd7, 0x94, 0x26, 0x95, 0x63, 0x8c, 0x4f, 0xa9, 0xac, 0x0f,
                0xc3, 0x68, 0x8c, 0x4f, 0x97, 0x74, 0xb9, 0x05, 0xa1, 0x4e, 0x3a, 0x3f, 0x17, 0x1b, 0xac, 0x58,
                0x6c, 0x55, 0xe8, 0x3f, 0xf9, 0x7a, 0x1a, 0xef, 0xfb, 0x3a, 0xf0, 0x0a, 0xdb, 0x22, 0xc6, 0xbb,
                0x08, 0xb3, 0xf4, 0x81, 0xe3, 0xaa, 0xa0, 0xf1, 0xa0, 0x9e, 0x30, 0xed, 0x74, 0x1d, 0x8a, 0xe4,
                0xfc, 0xf5, 0xe0, 0x95, 0xd5, 0xd0, 0x0a, 0xf6, 0x00, 0xdb, 0x18, 0xcb, 0x2c, 0x04, 0xb3, 0xed,
                0xd0, 0x3c, 0xc7, 0x44, 0xa2, 0x88, 0x8a, 0xe4, 0x0c, 0xaa, 0x23, 0x29, 0x46, 0xc5, 0xe7, 0xe1};
            static const uint8_t g2b[192] = {
                0x13, 0xe0, 0x2b, 0x60, 0x52, 0x71, 0x9f, 0x60, 0x7d, 0xac, 0xd3, 0xa0, 0x88, 0x27, 0x4f, 0x65,
                0x59, 0x6b, 0xd0, 0xd0, 0x99, 0x20, 0xb6, 0x1a, 0xb5, 0xda, 0x61, 0xbb, 0xdc, 0x7f, 0x50, 0x49,
                0x33, 0x4c, 0xf1, 0x12, 0x13, 0x94, 0x5d, 0x57, 0xe5, 0xac, 0x7d, 0x05, 0x5d, 0x04, 0x2b, 0x7e,
                0x02, 0x4a, 0xa2, 0xb2, 0xf0, 0x8f, 0x0a, 0x91, 0x26, 0x08, 0x05, 0x27, 0x2d, 0xc5, 0x10, 0x51,
                0xc6, 0xe4, 0x7a, 0xd4, 0xfa, 0x40, 0x3b, 0x02, 0xb4, 0x51, 0x0b, 0x64, 0x7a, 0xe3, 0xd1, 0x77,
                0x0b, 0xac, 0x03, 0x26, 0xa8, 0x05, 0xbb, 0xef, 0xd4, 0x80, 0x56, 0xc8, 0xc1, 0x21, 0xbd, 0xb8,
                0x06, 0x06, 0xc4, 0xa0, 0x2e, 0xa7, 0x34, 0xcc, 0x32, 0xac, 0xd2, 0xb0, 0x2b, 0xc2, 0x8b, 0x99,
                0xcb, 0x3e, 0x28, 0x7e, 0x85, 0xa7, 0x63, 0xaf, 0x26, 0x74, 0x92, 0xab, 0x57, 0x2e, 0x99, 0xab,
                0x3f, 0x37, 0x0d, 0x27, 0x5c, 0xec, 0x1d, 0xa1, 0xaa, 0xa9, 0x07, 0x5f, 0xf0, 0x5f, 0x79, 0xbe,
                0x0c, 0xe5, 0xd5, 0x27, 0x72, 0x7d, 0x6e, 0x11, 0x8c, 0xc9, 0xcd, 0xc6, 0xda, 0x2e, 0x35, 0x1a,
                0xad, 0xfd, 0x9b, 0xaa, 0x8c, 0xbd, 0xd3, 0xa7, 0x6d, 0x42, 0x9a, 0x69, 0x51, 0x60, 0xd1, 0x2c,
                0x92, 0x3a, 0xc9, 0xcc, 0x3b, 0xac, 0xa2, 0x89, 0xe1, 0x93, 0x54, 0x86, 0x08, 0xb8, 0x28, 0x01};
            g1_decode_host(g1b, g1);
            g2_decode_host(g2b, g2);
        }
        g1_affine_t *t1 = t1_t.alloc<g1_affine_t>(32 * 255);
        g2_affine_t *t2 = t2_t.alloc<g2_affine_t>(32 * 255);
        k_fb_table<fq_t><<<grid1(32 * 255), 256, 0, st>>>(g1, t1);
        k_fb_table<fq2_t><<<grid1(32 * 255), 256, 0, st>>>(g2, t2);
        MI_HIP(hipGetLastError());
        S->n_h = d - 1;
        S->h_perm = dalloc<g1_affine_t>(d - 1);
        fixed_base_affine<fq_t>(c, t1, ks, d - 1, S->h_perm);
        // QAP evaluations per variable: column sums of coeff * L_row(tau)
        S->n_vars = nv;
        S->at = dalloc<fr_t>(nv);
        S->bt = dalloc<fr_t>(nv);
        S->ct = dalloc<fr_t>(nv);
        fr_t *outs[3] = {S->at, S->bt, S->ct};
        for (int m = 0; m < 3; m++) {
            uint64_t nnz = circ.nnz[m];
            MI_HIP(hipMemsetAsync(outs[m], 0, 32 * nv, st));
            if (!nnz) continue;
            uint32_t *rows = c.scratch[0].as<uint32_t>(nnz);
            uint32_t *perm_in = c.scratch[1].as<uint32_t>(nnz);
            uint32_t *cols_s = c.scratch[2].as<uint32_t>(nnz);
            uint32_t *perm = c.scratch[3].as<uint32_t>(nnz);
            k_entry_rows<<<grid1(n), 256, 0, st>>>(circ.row_ptr[m], n, rows);
            k_iota<<<grid1(nnz), 256, 0, st>>>(perm_in, nnz);
            unsigned bits = 1;
            while ((1ull << bits) < nv) bits++;
            size_t tb = 0;
            MI_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, circ.col[m], cols_s, perm_in, perm, nnz, 0, bits,
                                                      st));
            void *tmp = c.scratch[4].get(tb);
            MI_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, circ.col[m], cols_s, perm_in, perm, nnz, 0, bits, st));
            // column sums by reduce-by-key over the column-sorted products: load-balanced whatever
            // the column lengths (ONE appears in ~half the rows of B)
            fr_t *prod = c.scratch[13].as<fr_t>(nnz);
            k_entry_products<<<grid1(nnz), 256, 0, st>>>(perm, rows, circ.cidx[m], circ.ctab, lag, nnz, prod);
            uint32_t *ukeys = c.scratch[5].as<uint32_t>(nnz);
            fr_t *uvals = c.scratch[14].as<fr_t>(nnz);
            uint32_t *nruns = c.scratch[6].as<uint32_t>(4);
            tb = 0;
            MI_HIP(hipcub::DeviceReduce::ReduceByKey(nullptr, tb, cols_s, ukeys, prod, uvals, nruns, FrAdd(), nnz, st));
            tmp = c.scratch[4].get(tb);
            MI_HIP(hipcub::DeviceReduce::ReduceByKey(tmp, tb, cols_s, ukeys, prod, uvals, nruns, FrAdd(), nnz, st));
            k_scatter_runs<<<grid1(nnz), 256, 0, st>>>(ukeys, uvals, nruns, outs[m]);
            MI_HIP(hipGetLastError());
        }
        k_add_input_rows<<<grid1(circ.n_in), 256, 0, st>>>(S->at, lag, n, circ.n_in);
        // l query: (beta at + alpha bt + ct) / delta over aux
        S->n_l = circ.n_aux;
        if (circ.n_aux) {
            k_lc_scalars<<<grid1(circ.n_aux), 256, 0, st>>>(S->at, S->bt, S->ct, circ.n_in, circ.n_aux, alpha, beta,
                                                            delta_inv, ks);
            S->l = dalloc<g1_affine_t>(circ.n_aux);
            fixed_base_affine<fq_t>(c, t1, ks, circ.n_aux, S->l);
        }
        // ic (host side, few points)
        {
            k_lc_scalars<<<grid1(circ.n_in), 256, 0, st>>>(S->at, S->bt, S->ct, 0, circ.n_in, alpha, beta, gamma_inv,
                                                           ks);
            std::vector<fr_t> ick(circ.n_in);
            MI_HIP(hipMemcpyAsync(ick.data(), ks, 32 * circ.n_in, hipMemcpyDeviceToHost, st));
            MI_HIP(hipStreamSynchronize(st));
            S->n_ic = circ.n_in;
            S->ic.resize(circ.n_in);
            for (uint64_t i = 0; i < circ.n_in; i++) S->ic[i] = host_mul_affine(g1, ick[i]);
        }
        // a, b queries
        S->n_a = circ.n_a;
        k_gather_canon<<<grid1(circ.n_a), 256, 0, st>>>(S->at, circ.idx_a, circ.n_a, ks);
        S->a = dalloc<g1_affine_t>(circ.n_a);
        fixed_base_affine<fq_t>(c, t1, ks, circ.n_a, S->a);
        S->n_b = circ.n_b;
        if (circ.n_b) {
            k_gather_canon<<<grid1(circ.n_b), 256, 0, st>>>(S->bt, circ.idx_b, circ.n_b, ks);
            S->b_g1 = dalloc<g1_affine_t>(circ.n_b);
            S->b_g2 = dalloc<g2_affine_t>(circ.n_b);
            fixed_base_affine<fq_t>(c, t1, ks, circ.n_b, S->b_g1);
            fixed_base_affine<fq2_t>(c, t2, ks, circ.n_b, S->b_g2);
        }
        MI_HIP(hipStreamSynchronize(st));
        ks_t.reset();
        pw_t.reset();
        t1_t.reset();
        t2_t.reset();
        // the column sums' sort and reduce-by-key buffers scale with the R1CS entries (tens of GB for a
        // 32 GiB partition): key generation is one-time, so give them back before the table decision and
        // the first proof
        for (auto &b : c.scratch) b.release();
        for (Ctx *x = c.aux; x; x = x->aux)  // and the auxiliary lanes' arenas (earlier proofs' B / L / A plans)
            for (auto &b : x->scratch) b.release();
        // verifying key
        S->alpha_g1 = host_mul_affine(g1, toxic_canonical[1]);
        S->beta_g1 = host_mul_affine(g1, toxic_canonical[2]);
        S->delta_g1 = host_mul_affine(g1, toxic_canonical[4]);
        S->beta_g2 = host_mul_affine(g2, toxic_canonical[2]);
        S->gamma_g2 = host_mul_affine(g2, toxic_canonical[3]);
        S->delta_g2 = host_mul_affine(g2, toxic_canonical[4]);
        build_hi_tables(c, *S, circ.idx_a, circ.n_in, circ.n_aux);
    } catch (...) {
        (void)hipStreamSynchronize(st);  // no kernel may still write the buffers freed below
        delete S;
        throw;
    }
    srs_publish(S);
    return S;
}
}  // namespace

// Key generation out of memory (several keys resident, earlier proofs' scratch): release the split tables of the
// keys on this device that no one is using and this context's idle scratch, and generate once more.
Srs *srs_generate(Ctx &c, const Circuit &circ, const fr_t toxic_canonical[5]) {
    try {
        return srs_generate_once(c, circ, toxic_canonical);
    } catch (const hip_error &e) {
        if (e.code != hipErrorOutOfMemory) throw;
        c.stats.oom_retries += 1;
        c.stats.oom_freed_bytes += release_for_retry(c, nullptr, nullptr);
        return srs_generate_once(c, circ, toxic_canonical);
    }
}

// ================================================================================ prove
namespace {
// One attempt at a proof's MSM sums.  inject_oom (tests, mi_ctx_inject_oom): after the NTT chain, while the
// auxiliary lane runs, the main lane asks a scratch buffer for more memory than the device has, so the attempt
// fails the way a short HBM makes it fail.
// The witness map and the QAP's NTT chain: A z, B z, C z, three coset round trips and (a b - c) / Z, then the
// inverse coset transform -> the d canonical H coefficients in bit-reversed order (the key's h_perm order),
// in the context's prover scratch (slot 20, after the Montgomery witness).
fr_t *compute_h(Ctx &c, const Circuit &circ, const fr_t *z_dev) {
    hipStream_t st = c.stream;
    const uint64_t d = circ.d, nv = circ.n_in + circ.n_aux;
    const unsigned L = circ.log_d;
    fr_t *zm = c.scratch[20].as<fr_t>(nv + 3 * d);
    fr_t *a = zm + nv, *b = a + d, *cc = b + d;
    k_copy_to_mont<<<grid1(nv), 256, 0, st>>>(z_dev, zm, nv);
    eval_witness_map(c, circ, zm, a, b, cc);
    fr_t dd = fr_t::zero();
    dd.v[0] = (uint32_t)d;
    dd.v[1] = (uint32_t)(d >> 32);
    fr_t dinv = inverse(to_mont(dd));
    fr_t g = fr_small_mont(7);
    fr_t zinv = inverse(pow_u64(g, d) - fr_t::one());
    // ifft, * g^i / d, fft on the coset (natural order) for a and b; c's last pass also forms
    // (a b - c) / Z and starts the inverse coset transform (ntt_coset_qap); tune::QAP_FUSED = 0 runs
    // the separate division pass (A/B)
    const bool qap_fused = tune::get(tune::QAP_FUSED, 1) != 0;
    ntt_coset_roundtrip(c, a, L, dinv);
    ntt_coset_roundtrip(c, b, L, dinv);
    if (!qap_fused || !ntt_coset_qap(c, a, b, cc, L, dinv, zinv)) {
        ntt_coset_roundtrip(c, cc, L, dinv);
        k_qap_divide<<<grid1(d), 256, 0, st>>>(a, b, cc, d, zinv);
        ntt_dif_coset_epilogue(c, a, L, true, true, dinv, true);  // icoset, canonical H (bit-reversed)
    }
    return a;
}

// h_in (optional): the H coefficients computed elsewhere (mi_groth16_h_coeffs_dev on a latency group's lead rank,
// broadcast to the group), so this share runs its H slice without the witness map and the NTT chain.
ProofSums groth16_sums_once(Ctx &c, const Srs &srs, const Circuit &circ, const fr_t *z_dev, const SumRanges &rg,
                            bool inject_oom, const fr_t *h_in) {
    std::shared_lock<std::shared_mutex> in_use(srs.use_mu);
    if (srs.d != circ.d || srs.n_l != circ.n_aux || srs.n_a != circ.n_a || srs.n_b != circ.n_b)
        throw std::invalid_argument("SRS does not match circuit");
    const uint64_t totals[4] = {circ.d - 1, circ.n_aux, circ.n_a, circ.n_b};
    for (int q = 0; q < 4; q++)
        if (rg.lo[q] > totals[q] || rg.cnt[q] > totals[q] - rg.lo[q])
            throw std::invalid_argument("MSM range past the end of its query");
    hipStream_t st = c.stream;
    const uint64_t d = circ.d, nv = circ.n_in + circ.n_aux;
    const unsigned L = circ.log_d;
    // the witness map and the NTT chain run only when this share holds part of the H MSM
    const bool need_h = rg.cnt[0] > 0;
    ProofSums out;
    g1_xyzz_t &H = out.H, &Lq = out.L, &As = out.A, &B1 = out.B1;
    g2_xyzz_t &B2 = out.B2;
    out.premul = rg.premul_r && rg.premul_s;
    auto premul_b1 = [&] {
        if (out.premul) out.rB1 = host::xyzz_mul(B1, rg.premul_r->v, 8);
    };
    {
    ScopedTimer whole(c, &c.stats.prove, circ.n);
    {
        // L, B_G1 and B_G2 do not depend on the QAP: they run on the auxiliary lane (second stream,
        // second host thread) while this stream runs the witness map, the NTT chain, H and A.
        // tune::PROVE_LANES = 1 runs the auxiliary work after the main lane on the same stream (measurement
        // only: every phase's device time without the other lane's kernels beside it; bench.py's one-lane proof)
        const bool one_lane = tune::get(tune::PROVE_LANES, 2) == 1;
        // Small proofs (domain <= 2^tune::PROVE_WIDE_LOG, default 2^21: Winning PoSt, 2^19) are latency-bound: their
        // MSMs' bucket reductions, sorts and host round trips leave most CUs idle, so B_G2, L and A + B_G1 each get
        // a lane of their own (three auxiliary streams and host threads beside the main lane's witness map, NTT
        // chain and H).  Large proofs keep two lanes: their accumulation fills the chip and every lane holds a scratch
        // arena sized to its MSMs.  Tests compare the two layouts.
        const int64_t wl = tune::get(tune::PROVE_WIDE_LOG, 21);
        const unsigned wide_log = wl >= 0 && wl < 64 ? (unsigned)wl : 21u;
        const bool wide = !one_lane && L <= wide_log;
        const unsigned nlanes = wide ? 3 : 1;
        Ctx *lane_ctx[3] = {one_lane ? &c : &ctx_aux(c), nullptr, nullptr};
        for (unsigned k = 1; k < nlanes; k++) lane_ctx[k] = &ctx_aux(*lane_ctx[k - 1]);
        hipEvent_t ready = c.timer.get(), done[3] = {nullptr, nullptr, nullptr};
        MI_HIP(hipEventRecord(ready, st));  // z_dev and everything queued before this prove
        for (unsigned k = 0; k < nlanes; k++) {
            done[k] = lane_ctx[k]->timer.get();
            MI_HIP(hipStreamWaitEvent(lane_ctx[k]->stream, ready, 0));
        }
        std::exception_ptr err[3];
        // B_G1 and B_G2 share the scalars (z over the B-density): sort them once on large proofs.  Small proofs run
        // B_G1 after A on A's lane (tune::PROVE_B1_LANE: 2 default, 1 after L, 0 with B_G2), which sorts the scalars
        // again for itself (no plan is shared between lanes: the G2 second level reuses its plan's scratch).
        // Same box, Winning PoSt: 23.1 ms with B_G1 beside B_G2, 20.5 ms after A.
        const int64_t b1t = tune::get(tune::PROVE_B1_LANE, 2);
        const unsigned b1_lane = wide ? (b1t < 0 || b1t > 2 ? 2u : (unsigned)b1t) : 0u;  // every value names a lane that computes B_G1
        auto run_b = [&](Ctx &x) {
            const uint64_t lo = rg.lo[3], cnt = rg.cnt[3];
            WinTable wt2 = srs.wt_of(4);
            wt2.sparse = true;  // witness scalars
            if (b1_lane != 0 && wt2.p) {  // B_G1 runs on another lane: B_G2 over its window table
                msm_g2(x, srs.b_g2 + lo, z_dev, circ.idx_b + lo, cnt, &B2, &wt2, lo);
                return;
            }
            MsmPlan pb;
            msm_prepare(x, z_dev, circ.idx_b + lo, cnt, pb);
            if (b1_lane == 0) {
                msm_g1_planned(x, pb, srs.b_g1 + lo, &B1);
                premul_b1();
            }
            msm_g2_planned(x, pb, srs.b_g2 + lo, &B2);
        };
        auto run_b1 = [&](Ctx &x) {
            const uint64_t lo = rg.lo[3], cnt = rg.cnt[3];
            WinTable wt = srs.wt_of(3);
            wt.sparse = true;  // witness scalars
            msm_g1(x, srs.b_g1 + lo, z_dev, circ.idx_b + lo, cnt, &B1, nullptr, srs.in_subgroup, &wt, lo);
            premul_b1();
        };
        auto run_l = [&](Ctx &x) {
            const uint64_t l_lo = rg.lo[1], l_cnt = rg.cnt[1];
            WinTable wt = srs.wt_of(1);
            wt.sparse = true;  // witness scalars
            msm_g1(x, srs.l + l_lo, z_dev + circ.n_in + l_lo, nullptr, l_cnt, &Lq, srs.l_hi ? srs.l_hi + l_lo : nullptr,
                   srs.in_subgroup, &wt, l_lo);
        };
        auto run_a = [&](Ctx &x) {
            const uint64_t a_lo = rg.lo[2], a_cnt = rg.cnt[2];
            WinTable wt = srs.wt_of(2);
            wt.sparse = true;  // witness scalars
            msm_g1(x, srs.a + a_lo, z_dev, circ.idx_a + a_lo, a_cnt, &As, srs.a_hi ? srs.a_hi + a_lo : nullptr,
                   srs.in_subgroup, &wt, a_lo);
            if (out.premul) out.sA = host::xyzz_mul(As, rg.premul_s->v, 8);
        };
        // Shared L/A plan (Srs::a_aux, VERDICT r5 #1b).  L sums z_aux over l and A's aux part sums the same z_aux over
        // a_aux (A's points in the aux index space, infinity where a variable has no A density), so ONE plan (digits,
        // sort, bucket bounds, chunking: a GLV plan for these subgroup keys) serves both, and the input part of A,
        // a[0, n_in) with z[0, n_in), is a small MSM of its own.  The auxiliary lane builds the plan after B and runs
        // L's accumulation over it; the main lane runs A's accumulation over the same plan after H (a host handoff
        // of the plan's counts plus a device event): one plan fewer per proof, the lanes' work as before.
        const bool shared_la = !wide && srs.a_aux && rg.lo[1] == 0 && rg.cnt[1] == circ.n_aux && rg.lo[2] == 0 &&
                               rg.cnt[2] == circ.n_a && circ.n_a > circ.n_in && msm_glv_mode() != 0;
        // A plan derived from L's (msm_derive_plan): keys below the shared plan's density rule (the synthetic config-3
        // circuit: A covers 66 % of the aux variables) keep A's own query, but A's digits are L's digits of the
        // variables with A density, already sorted into L's buckets.  The lane that runs L builds L's plan with those
        // entries marked (Circuit::a_rank), derives A's plan from it by filtering (no digit pass, no sort) into plan
        // slots of its own, hands it to the main lane and accumulates L; A's accumulation runs after H over A's points
        // and tables.  Both plans need the same split: the 2^128 tables of l and a, or GLV for both.
        const int glv_mode = msm_glv_mode();
        auto glv_for = [&](const g1_affine_t *hi) { return glv_mode == 1 || (glv_mode == 2 && !hi && srs.in_subgroup); };
        const bool la_glv = glv_for(srs.l_hi);
        const bool derive_a = !wide && !shared_la && circ.a_rank && circ.a_bits && tune::get(tune::A_FROM_L, 1) != 0 &&
                              rg.lo[1] == 0 && rg.cnt[1] == circ.n_aux && rg.lo[2] == 0 && rg.cnt[2] == circ.n_a &&
                              circ.n_a > circ.n_in && msm_use_split(circ.n_aux) && !srs.wt[1] && !srs.wt[2] &&
                              la_glv == glv_for(srs.a_hi) && (la_glv || (srs.l_hi && srs.a_hi)) &&
                              2 * (circ.n_aux + circ.n_a) < (1ull << 30);
        const bool hand_a = shared_la || derive_a;  // A's plan comes from the auxiliary lane
        std::promise<MsmPlan> la_plan;
        std::future<MsmPlan> la_plan_f = la_plan.get_future();
        std::atomic<bool> la_handed{false};
        hipEvent_t la_ready = hand_a ? c.timer.get() : nullptr;
        g1_xyzz_t A_aux = g1_xyzz_t::inf();
        auto run_la_plan = [&](Ctx &x) {  // the shared plan, on the lane that runs L; handed to A's lane
            MsmPlan pl;
            msm_prepare_g1_shared(x, z_dev + circ.n_in, circ.n_aux, pl);  // pl.total == 0: every scalar zero
            MI_HIP(hipEventRecord(la_ready, x.stream));
            la_handed = true;
            la_plan.set_value(pl);
            return pl;
        };
        auto run_l_shared = [&](Ctx &x) {
            const MsmPlan pl = run_la_plan(x);
            msm_g1_planned(x, pl, srs.l, &Lq);
            return pl;
        };
        auto finish_a = [&](Ctx &x) {  // A = A_aux + the inputs' part (idx_a starts with every input)
            g1_xyzz_t A_in = g1_xyzz_t::inf();
            msm_g1(x, srs.a, z_dev, nullptr, circ.n_in, &A_in, nullptr, srs.in_subgroup, nullptr, 0);
            As = host::xyzz_add(A_aux, A_in);
            if (out.premul) out.sA = host::xyzz_mul(As, rg.premul_s->v, 8);
        };
        auto run_a_shared = [&](Ctx &x) {  // A's lane: wait for the plan, accumulate A_aux over it
            const MsmPlan pl = la_plan_f.get();
            MI_HIP(hipStreamWaitEvent(x.stream, la_ready, 0));
            msm_g1_planned(x, pl, srs.a_aux, &A_aux);
            finish_a(x);
        };
        // derived: L's marked plan, A's plan from it (handed over), L's accumulation; returns A's plan
        auto run_l_derive = [&](Ctx &x) {
            MsmPlan pl, pa;
            const bool any = msm_prepare_marked(x, z_dev + circ.n_in, circ.n_aux, pl, la_glv, circ.a_rank);
            if (any) msm_derive_plan(x, pl, circ.a_bits, circ.n_a, (uint32_t)circ.n_in, pa);
            MI_HIP(hipEventRecord(la_ready, x.stream));
            la_handed = true;
            la_plan.set_value(pa);
            if (any) msm_g1_planned(x, pl, srs.l, &Lq, la_glv ? nullptr : srs.l_hi);
            return pa;
        };
        auto run_a_derived = [&](Ctx &x, const MsmPlan &pa) {  // A_aux over A's own points, then the inputs' part
            msm_g1_planned(x, pa, srs.a, &A_aux, la_glv ? nullptr : srs.a_hi);
            finish_a(x);
        };
        if (shared_la) c.stats.shared_la += 1;
        if (derive_a) c.stats.derived_a += 1;
        // aux-lane order: B before L (same-box A/B at 2^26: -2 ms per proof; tune::AUX_ORDER = 1
        // restores L first)
        const bool b_first = tune::get(tune::AUX_ORDER, 0) != 1;
        auto lane_work = [&](unsigned k) {
            try {
                Ctx &x = *lane_ctx[k];
                MI_HIP(hipSetDevice(c.device));
                if (!wide && shared_la) {
                    run_b(x);
                    const MsmPlan pl = run_l_shared(x);
                    if (one_lane) {  // the main lane is done: A over the same plan here, after L
                        msm_g1_planned(x, pl, srs.a_aux, &A_aux);
                        finish_a(x);
                    }
                } else if (!wide && derive_a) {
                    if (b_first) run_b(x);
                    const MsmPlan pa = run_l_derive(x);
                    if (!b_first) run_b(x);
                    if (one_lane) run_a_derived(x, pa);  // the main lane is done: A here, after L
                } else if (!wide) {
                    if (b_first) run_b(x);
                    run_l(x);
                    if (!b_first) run_b(x);
                } else if (k == 0) {
                    run_b(x);
                } else if (k == 1) {
                    run_l(x);
                    if (b1_lane == 1) run_b1(x);
                } else {
                    run_a(x);
                    if (b1_lane == 2) run_b1(x);
                }
                MI_HIP(hipEventRecord(done[k], x.stream));
            } catch (...) {
                err[k] = std::current_exception();
                // a lane that fails before handing over the shared plan must not leave A's lane waiting for it
                if (hand_a && k == 0 && !la_handed.exchange(true)) la_plan.set_exception(err[k]);
            }
        };
        std::thread lanes[3];
        if (!one_lane)
            for (unsigned k = 0; k < nlanes; k++) lanes[k] = std::thread(lane_work, k);
        std::exception_ptr err_main;
        try {
            const fr_t *a = h_in;
            if (need_h && !a) a = compute_h(c, circ, z_dev);
            if (inject_oom) (void)c.scratch[19].get(1ull << 50);  // a real failed growth (1 PiB), as a scratch
                                                                    // buffer's hipMalloc fails when HBM is short
            const uint64_t h_lo = rg.lo[0], h_cnt = rg.cnt[0];
            const WinTable wt_h = srs.wt_of(0);
            if (need_h)
                msm_g1(c, srs.h_perm + h_lo, a + h_lo, nullptr, h_cnt, &H, srs.h_hi ? srs.h_hi + h_lo : nullptr,
                       srs.in_subgroup, &wt_h, h_lo);
            else
                H = g1_xyzz_t::inf();
            if (!wide && !hand_a) run_a(c);
            if (shared_la && !one_lane) run_a_shared(c);
            if (derive_a && !one_lane) {
                const MsmPlan pa = la_plan_f.get();
                MI_HIP(hipStreamWaitEvent(c.stream, la_ready, 0));
                run_a_derived(c, pa);
            }
        } catch (...) {
            err_main = std::current_exception();
        }
        if (one_lane) {
            if (!err_main) lane_work(0);
        } else {
            for (unsigned k = 0; k < nlanes; k++) lanes[k].join();
        }
        if (err_main) std::rethrow_exception(err_main);
        for (unsigned k = 0; k < nlanes; k++)
            if (err[k]) std::rethrow_exception(err[k]);
        for (unsigned k = 0; k < nlanes; k++) {
            MI_HIP(hipStreamWaitEvent(st, done[k], 0));  // the prove timer ends after every lane
            lane_ctx[k]->timer.pool.push_back(done[k]);
        }
        c.timer.pool.push_back(ready);
        if (la_ready) c.timer.pool.push_back(la_ready);
        if (!one_lane) {
            for (unsigned k = 0; k < nlanes; k++) {
                Ctx &x = *lane_ctx[k];
                x.timer.resolve();
                c.stats.merge(x.stats);
                x.stats = Stats();
            }
        }
    }
    }
    MI_HIP(hipStreamSynchronize(st));
    c.timer.resolve();
    return out;
}

}  // namespace

uint64_t srs_drop_split_tables(Srs &S) {
    uint64_t freed = 0;
    const struct {
        g1_affine_t **p;
        uint64_t n;
    } ts[] = {{&S.h_hi, S.n_h}, {&S.l_hi, S.n_l}, {&S.a_hi, S.n_a}};
    for (auto &t : ts)
        if (*t.p) {
            (void)hipFree(*t.p);
            *t.p = nullptr;
            freed += t.n * sizeof(g1_affine_t);
        }
    if (S.a_aux) {  // derived like the tables; an out-of-memory retry runs L and A over plans of their own
        (void)hipFree(S.a_aux);
        S.a_aux = nullptr;
        freed += S.n_l * sizeof(g1_affine_t);
    }
    for (int q = 0; q < 5; q++)
        if (S.wt[q]) {
            freed += S.wt_bytes(q);
            (void)hipFree(S.wt[q]);
            S.wt[q] = nullptr;
        }
    return freed;
}

namespace {
// the split tables (and trapdoor evaluations) of every key on `device` that no one is using right now, the
// proving key first
uint64_t release_device_tables(int device, const Srs *first) {
    std::lock_guard<std::mutex> lk(g_keys_mu);
    std::vector<Srs *> order;
    for (Srs *k : g_keys)
        if (k == first) order.insert(order.begin(), k);
        else if (k->device == device) order.push_back(k);
    uint64_t freed = 0;
    for (Srs *k : order) {
        if (!k->has_tables() && !k->at) continue;
        std::unique_lock<std::shared_mutex> ex(k->use_mu, std::try_to_lock);
        if (!ex.owns_lock()) continue;
        const uint64_t t = srs_drop_split_tables(*k);
        if (t) k->tables_dropped += 1;  // mi_srs_readmit rebuilds them once memory allows
        freed += t;
        // a generated key's per-variable trapdoor evaluations (3 x 32 B per variable: 12.5 GB at 2^27) serve
        // only mi_groth16_trapdoor_dlogs, a test aid; they go too, and that call then reports them missing
        const struct {
            fr_t **p;
        } tv[] = {{&k->at}, {&k->bt}, {&k->ct}};
        for (auto &t : tv)
            if (*t.p) {
                (void)hipFree(*t.p);
                *t.p = nullptr;
                freed += 32 * k->n_vars;
            }
        k->has_trapdoor = false;
    }
    return freed;
}

// releases a context's grow-only scratch (every lane), except the witness slots of the batch uploader (21, 22:
// the next partition may be uploading into the other one) and any buffer holding `keep` (the proof's witness)
uint64_t release_prover_scratch(Ctx &c, const void *keep) {
    uint64_t freed = 0;
    auto rel = [&](Ctx &x, int upto) {
        for (int i = 0; i < upto; i++) {
            DevBuf &b = x.scratch[i];
            const char *lo = (const char *)b.p;
            if (b.p && (const char *)keep >= lo && (const char *)keep < lo + b.cap) continue;
            freed += b.p ? b.cap : 0;
            b.release();
        }
    };
    rel(c, 21);
    for (Ctx *x = c.aux; x; x = x->aux) rel(*x, 26);
    return freed;
}
}  // namespace

// Rebuilds the split tables an out-of-memory release took from a key, under the key-load admission rule
// (build_hi_tables: only while they leave a proof its working set).  Returns the bytes of tables rebuilt.
uint64_t srs_readmit(Ctx &c, Srs &S) {
    std::unique_lock<std::shared_mutex> ex(S.use_mu);  // no proof or MSM over the key while its tables change
    if (!S.tables_dropped || S.has_tables()) return 0;
    release_prover_scratch(c, nullptr);  // this context's idle arenas would count against the admission
    build_hi_tables(c, S);
    MI_HIP(hipStreamSynchronize(c.stream));
    uint64_t got = 0;
    if (S.h_hi) got += S.n_h * sizeof(g1_affine_t);
    if (S.l_hi) got += S.n_l * sizeof(g1_affine_t);
    if (S.a_hi) got += S.n_a * sizeof(g1_affine_t);
    for (int q = 0; q < 5; q++) got += S.wt_bytes(q);
    if (got) S.tables_dropped = 0;
    return got;
}

uint64_t release_for_retry(Ctx &c, const Srs *first, const void *keep) {
    (void)hipStreamSynchronize(c.stream);
    for (Ctx *x = c.aux; x; x = x->aux) (void)hipStreamSynchronize(x->stream);
    (void)hipGetLastError();  // the failed allocation's error, so the retry's launch checks start clean
    return release_device_tables(c.device, first) + release_prover_scratch(c, keep);
}

// A proof whose working set does not fit next to the resident keys degrades instead of failing: on an
// out-of-memory error the attempt is drained, the 2^128 split tables of the keys on this device (the proving
// key's first, then every other key no one is using: several keys stay resident side by side, as the
// reference's GROTH_PARAM_MEMORY_CACHE keeps them, caches.hpp:48-116) and this context's idle scratch are
// released, and the proof runs again; its G1 MSMs take the GLV split, which needs no table (glv.h).  The MSM
// sums are unique group elements, so the retried proof is byte-identical.  A second out-of-memory error
// propagates.
ProofSums groth16_sums_ranges(Ctx &c, const Srs &srs, const Circuit &circ, const fr_t *z_dev, const SumRanges &rg,
                               const fr_t *h_in) {
    // test hook (mi_ctx_inject_oom): a counter on the context, not an environment lookup in the production path
    bool inject = false;
    if (c.inject_oom != 0) {
        inject = true;
        if (c.inject_oom > 0) c.inject_oom -= 1;
    }
    try {
        return groth16_sums_once(c, srs, circ, z_dev, rg, inject, h_in);
    } catch (const hip_error &e) {
        if (e.code != hipErrorOutOfMemory) throw;
        c.stats.oom_retries += 1;
        c.stats.oom_freed_bytes += release_for_retry(c, &srs, h_in ? (const void *)h_in : (const void *)z_dev);
        return groth16_sums_once(c, srs, circ, z_dev, rg, false, h_in);
    }
}

void groth16_h_coeffs(Ctx &c, const Circuit &circ, const fr_t *z_dev, fr_t *out) {
    const fr_t *a = compute_h(c, circ, z_dev);
    MI_HIP(hipMemcpyAsync(out, a, 32 * circ.d, hipMemcpyDeviceToDevice, c.stream));
    MI_HIP(hipStreamSynchronize(c.stream));
}

SumRanges share_ranges(const Circuit &circ, unsigned rank, unsigned world) {
    if (world == 0 || rank >= world) throw std::invalid_argument("share rank out of range");
    const uint64_t totals[4] = {circ.d - 1, circ.n_aux, circ.n_a, circ.n_b};
    SumRanges r;
    for (int q = 0; q < 4; q++) {  // rank's contiguous slice [n k / W, n (k + 1) / W) of every query
        r.lo[q] = totals[q] * rank / world;
        r.cnt[q] = totals[q] * (rank + 1) / world - r.lo[q];
    }
    return r;
}

ProofSums groth16_sums(Ctx &c, const Srs &srs, const Circuit &circ, const fr_t *z_dev, unsigned rank,
                       unsigned world) {
    return groth16_sums_ranges(c, srs, circ, z_dev, share_ranges(circ, rank, world));
}

AssemblyKey assembly_key(const Srs &srs) {
    return AssemblyKey{srs.alpha_g1, srs.beta_g1, srs.delta_g1, srs.beta_g2, srs.delta_g2};
}

// libsnark r1cs_gg_ppzksnark_prover / bellman create_proof: the blinded proof from the five MSM sums
//   A = alpha + sum z_i A_i + r delta;  B = beta + sum z_i B_i + s delta (G2), B1 likewise in G1
//   C = H + L + s A + r B1 - r s delta, expanded so that A and B1 enter without their blinding:
//   s (alpha + A_sum + r delta) + r (beta + B1_sum + s delta) - r s delta = s alpha + r beta + s A_sum + r B1_sum + r s delta
BlindTerms groth16_blind_terms(const AssemblyKey &k, const fr_t &r, const fr_t &s) {
    const fr_t rs = from_mont(to_mont(r) * to_mont(s));
    BlindTerms t;
    t.A0 = host::xyzz_add_affine(host::xyzz_mul(xyzz_from_affine(k.delta_g1), r.v, 8), k.alpha_g1);
    t.B0 = host::xyzz_add_affine(host::xyzz_mul(xyzz_from_affine(k.delta_g2), s.v, 8), k.beta_g2);
    g1_xyzz_t C = host::xyzz_mul(xyzz_from_affine(k.delta_g1), rs.v, 8);
    C = host::xyzz_add(C, host::xyzz_mul(xyzz_from_affine(k.alpha_g1), s.v, 8));
    t.C0 = host::xyzz_add(C, host::xyzz_mul(xyzz_from_affine(k.beta_g1), r.v, 8));
    return t;
}

ProofPoints groth16_finish(const BlindTerms &t, const ProofSums &m, const fr_t &r, const fr_t &s) {
    // s A and r B1: from the lanes (premul), else side by side here (one on a helper thread)
    g1_xyzz_t sAv = m.sA, rB1 = m.rB1;
    if (!m.premul) {
        auto sA = std::async(std::launch::async, [&] { return host::xyzz_mul(m.A, s.v, 8); });
        rB1 = host::xyzz_mul(m.B1, r.v, 8);
        sAv = sA.get();
    }
    g1_xyzz_t C = host::xyzz_add(t.C0, sAv);
    C = host::xyzz_add(C, rB1);
    C = host::xyzz_add(C, m.H);
    C = host::xyzz_add(C, m.L);
    ProofPoints out;
    out.A = host::xyzz_to_affine(host::xyzz_add(m.A, t.A0));
    out.B = host::xyzz_to_affine(host::xyzz_add(m.B2, t.B0));
    out.C = host::xyzz_to_affine(C);
    return out;
}

ProofPoints groth16_assemble(const AssemblyKey &k, const ProofSums &m, const fr_t &r, const fr_t &s) {
    return groth16_finish(groth16_blind_terms(k, r, s), m, r, s);
}

ProofPoints groth16_prove(Ctx &c, const Srs &srs, const Circuit &circ, const fr_t *z_dev, const fr_t &r,
                          const fr_t &s) {
    // the blinding-only terms on a host thread while the device works (Winning PoSt: ~4 ms of host scalar
    // multiplications off a ~25 ms proof)
    const AssemblyKey key = assembly_key(srs);
    auto terms = std::async(std::launch::async, [&] { return groth16_blind_terms(key, r, s); });
    SumRanges rg = share_ranges(circ, 0, 1);
    rg.premul_r = &r;
    rg.premul_s = &s;
    const ProofSums m = groth16_sums_ranges(c, srs, circ, z_dev, rg);
    return groth16_finish(terms.get(), m, r, s);
}

void sums_encode(const ProofSums &m, uint8_t out[576]) {
    g1_encode(host::xyzz_to_affine(m.H), out);
    g1_encode(host::xyzz_to_affine(m.L), out + 96);
    g1_encode(host::xyzz_to_affine(m.A), out + 192);
    g1_encode(host::xyzz_to_affine(m.B1), out + 288);
    g2_encode(host::xyzz_to_affine(m.B2), out + 384);
}

Ctx &ctx_aux(Ctx &c) {
    if (!c.aux) {
        Ctx *x = new Ctx();
        x->device = c.device;
        c.aux = x;
    }
    int prio = 0, lo = 0, hi = 0;
    MI_HIP(hipStreamGetPriority(c.stream, &prio));
    MI_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // the auxiliary lane follows the caller's priority; tune::LANE_PRIO = 1 puts it above a normal main lane,
    // 2 keeps it normal under a high-priority main lane (lane-contention A/B)
    const int64_t lane_prio = tune::get(tune::LANE_PRIO, 0);
    const bool aux_hi = lane_prio == 1 ? true : lane_prio == 2 ? false : (prio == hi && hi != lo);
    // each lane's stream of the needed priority is created at its first use: every stream takes a hardware queue
    // (GPU_MAX_HW_QUEUES) or shares one, and two streams on one queue run in order (a lane behind another's
    // accumulation)
    hipStream_t &s = c.aux->aux_streams[aux_hi ? 1 : 0];
    if (!s) {
        if (aux_hi)
            MI_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
        else
            MI_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    c.aux->stream = s;
    return *c.aux;
}

void ctx_aux_free(Ctx &c) {
    if (!c.aux) return;
    ctx_aux_free(*c.aux);  // the lanes after it (small proofs use a chain of three)
    for (auto &b : c.aux->scratch) b.release();
    for (auto s : c.aux->aux_streams)
        if (s) hipStreamDestroy(s);
    if (c.aux->plan_stream) hipStreamDestroy(c.aux->plan_stream);
    for (auto e : c.aux->plan_ev)
        if (e) hipEventDestroy(e);
    delete c.aux;
    c.aux = nullptr;
}

static fr_t device_dot(Ctx &c, const fr_t *z, const fr_t *e, uint64_t off, uint64_t n) {
    if (!n) return fr_t::zero();
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (blocks > 1024) blocks = 1024;
    fr_t *part = c.scratch[14].as<fr_t>(blocks);
    k_dot<<<blocks, 256, 0, c.stream>>>(z, e, off, n, part);
    std::vector<fr_t> h(blocks);
    MI_HIP(hipMemcpyAsync(h.data(), part, 32 * blocks, hipMemcpyDeviceToHost, c.stream));
    MI_HIP(hipStreamSynchronize(c.stream));
    fr_t acc = fr_t::zero();
    for (auto &x : h) acc = acc + x;
    return acc;
}

void groth16_trapdoor_dlogs(Ctx &c, const Srs &srs, const Circuit &circ, const fr_t *z_dev, const fr_t &r,
                            const fr_t &s, fr_t out[3]) {
    // another context's out-of-memory release may free at / bt / ct and clear has_trapdoor: hold the key
    std::shared_lock<std::shared_mutex> in_use(srs.use_mu);
    if (!srs.has_trapdoor)
        throw std::invalid_argument("SRS was not generated from known toxic waste (or its trapdoor evaluations were "
                                    "released to make room for a proof)");
    uint64_t nv = circ.n_in + circ.n_aux;
    fr_t alpha = to_mont(srs.toxic[1]), beta = to_mont(srs.toxic[2]), delta = to_mont(srs.toxic[4]);
    fr_t u = device_dot(c, z_dev, srs.at, 0, nv);
    fr_t v = device_dot(c, z_dev, srs.bt, 0, nv);
    fr_t w = device_dot(c, z_dev, srs.ct, 0, nv);
    fr_t ua = device_dot(c, z_dev, srs.at, circ.n_in, circ.n_aux);
    fr_t va = device_dot(c, z_dev, srs.bt, circ.n_in, circ.n_aux);
    fr_t wa = device_dot(c, z_dev, srs.ct, circ.n_in, circ.n_aux);
    fr_t rm = to_mont(r), sm = to_mont(s);
    fr_t Ad = alpha + u + rm * delta;
    fr_t Bd = beta + v + sm * delta;
    fr_t lsum = beta * ua + alpha * va + wa;
    fr_t ht = u * v - w;
    fr_t Cd = (lsum + ht) * inverse(delta) + sm * Ad + rm * Bd - rm * sm * delta;
    out[0] = from_mont(Ad);
    out[1] = from_mont(Bd);
    out[2] = from_mont(Cd);
}

}  // namespace mi
