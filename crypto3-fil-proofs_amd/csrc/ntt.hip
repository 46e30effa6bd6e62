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
#include "ctx.h"

namespace mi {

namespace {

constexpr unsigned TILE_LOG = 10;  // 1024 elements = 32 KiB of LDS per workgroup
constexpr unsigned TILE = 1u << TILE_LOG;
constexpr unsigned NTT_THREADS = 256;

__device__ __forceinline__ fr_t tw_full(const fr_t *__restrict__ lo, const fr_t *__restrict__ hi, uint32_t e) {
    uint32_t l = e & 0xffffu, h = e >> 16;
    if (l == 0) return hi[h];
    if (h == 0) return lo[l];
    return lo[l] * hi[h];
}

__device__ __forceinline__ uint32_t brev(uint32_t x, unsigned bits) {
    return bits ? (__builtin_bitreverse32(x) >> (32 - bits)) : 0;
}

// One pass.  DIF: load -> b DIF stages -> optional inter-pass twiddle -> [epilogue] -> store.
//            DIT: load -> optional inter-pass twiddle -> b DIT stages (reverse) -> store.
// In-tile twiddles omega_{2^b}^j come from the 512-entry omega_1024 table (16 KiB, L1-resident), so
// the tile is the only LDS use (32 KiB: 5 workgroups per CU).
// Epilogue (last DIF pass only): epi = 1 multiplies the element at global position pos by
// G^bitrev_L(pos) * scale (coset shift of the bit-reversed coefficients, fused 1/d); epi = 2 also
// converts to canonical form (icoset: H for the MSM).
template <bool DIF>
__global__ void __launch_bounds__(NTT_THREADS) k_ntt_pass(fr_t *__restrict__ d, unsigned L, unsigned M, unsigned b,
                                                          unsigned Tlog, unsigned Glog, int twiddle,
                                                          const fr_t *__restrict__ lo,
                                                          const fr_t *__restrict__ hi,
                                                          const fr_t *__restrict__ tw10, int epi,
                                                          const fr_t *__restrict__ glo,
                                                          const fr_t *__restrict__ ghi, fr_t scale) {
    __shared__ fr_t sh[TILE];
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
        fr_t x = d[gi];
        if (!DIF && twiddle) {
            uint32_t k1 = brev(i1, b);
            uint32_t ex = (uint32_t)(((uint64_t)(i20 + t) * k1) << (32 - M));
            if (ex) x = x * tw_full(lo, hi, ex);
        }
        sh[e] = x;
    }
    __syncthreads();
    const unsigned nbf = tile >> 1;
    for (unsigned st = 0; st < b; st++) {
        unsigned s = DIF ? st : (b - 1 - st);  // DIF stage index
        unsigned hlog = b - 1 - s;
        unsigned h = 1u << hlog;
        for (unsigned q = threadIdx.x; q < nbf; q += NTT_THREADS) {
            unsigned t = q & (T - 1);
            unsigned r = q >> Tlog;
            unsigned g = r >> (b - 1);
            unsigned k = r & ((1u << (b - 1)) - 1);
            unsigned i1 = ((k >> hlog) << (hlog + 1)) | (k & (h - 1));
            unsigned j = (k & (h - 1)) << s;  // exponent of omega_{2^b}
            unsigned base = (g << b);
            unsigned e0 = ((base + i1) << Tlog) + t;
            unsigned e1 = e0 + (h << Tlog);
            fr_t u = sh[e0], v = sh[e1];
            if (DIF) {
                fr_t dd = u - v;
                sh[e0] = u + v;
                sh[e1] = j ? dd * tw10[j << (TILE_LOG - b)] : dd;
            } else {
                fr_t w = j ? v * tw10[j << (TILE_LOG - b)] : v;
                sh[e0] = u + w;
                sh[e1] = u - w;
            }
        }
        __syncthreads();
    }
    // store
    for (unsigned e = threadIdx.x; e < tile; e += NTT_THREADS) {
        unsigned t = e & (T - 1), i1 = (e >> Tlog) & bmask, g = e >> (Tlog + b);
        uint64_t gi = ((sub0 + g) << M) + ((uint64_t)i1 << Slog) + i20 + t;
        fr_t x = sh[e];
        if (DIF && twiddle) {
            uint32_t k1 = brev(i1, b);
            uint32_t ex = (uint32_t)(((uint64_t)(i20 + t) * k1) << (32 - M));
            if (ex) x = x * tw_full(lo, hi, ex);
        }
        if (DIF && epi) {
            uint32_t ex = brev((uint32_t)gi, L);
            if (ex) x = x * tw_full(glo, ghi, ex);
            x = x * scale;
            if (epi == 2) x = from_mont(x);
        }
        d[gi] = x;
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
        if (k < 2) {  // omega_1024^j = HI[j * 64] (HI[h] = omega_{2^16}^h), j < 512
            std::vector<fr_t> t10(TILE / 2);
            for (unsigned j = 0; j < TILE / 2; j++) t10[j] = hi[j << (16 - TILE_LOG)];
            fr_t **p10 = k == 0 ? &c.tw.fw_1024 : &c.tw.iv_1024;
            MI_HIP(hipMalloc(p10, sizeof(fr_t) * (TILE / 2)));
            MI_HIP(hipMemcpy(*p10, t10.data(), sizeof(fr_t) * (TILE / 2), hipMemcpyHostToDevice));
        }
    }
}

void ntt_free_tables(Ctx &c) {
    fr_t *ps[10] = {c.tw.fw_lo, c.tw.fw_hi, c.tw.iv_lo, c.tw.iv_hi, c.tw.g_lo,   c.tw.g_hi,
                    c.tw.gi_lo, c.tw.gi_hi, c.tw.fw_1024, c.tw.iv_1024};
    for (auto p : ps)
        if (p) hipFree(p);
    c.tw = NttTables();
}

static void ntt_run(Ctx &c, fr_t *d, unsigned L, bool inverse, bool dif, int epi = 0, bool inv_gen = false,
                    const fr_t &scale = fr_t::one()) {
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
    const fr_t *lo = inverse ? c.tw.iv_lo : c.tw.fw_lo;
    const fr_t *hi = inverse ? c.tw.iv_hi : c.tw.fw_hi;
    const fr_t *glo = inv_gen ? c.tw.gi_lo : c.tw.g_lo;
    const fr_t *ghi = inv_gen ? c.tw.gi_hi : c.tw.g_hi;
    const fr_t *tw10 = inverse ? c.tw.iv_1024 : c.tw.fw_1024;
    auto plan = plan_passes(L);
    if (dif) {
        for (size_t i = 0; i < plan.size(); i++) {
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
