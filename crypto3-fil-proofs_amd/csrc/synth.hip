// synth.hip -- deterministic synthetic R1CS + satisfying witness (host code, multithreaded).
//
// Workload generator for BASELINE configs 3/4 ("synthetic 2^26-constraint R1CS"): circuit
// synthesis is outside the prover boundary in the reference (StackedCircuit::synthesize,
// porep/stacked/circuit/proof.hpp:98-165), so this only has to produce a circuit with the
// statistics that matter to the prover -- rows of <= 3 terms, boolean-heavy witness, A/B
// densities well below 1 -- and a witness that satisfies it (so every proof verifies).
//
// n = 2^log_rows - n_in rows, so d = 2^log_rows exactly.  Variables: inputs (ONE, then n_in - 1
// random publics), then one aux variable v_j per row j.  Row kinds by j mod 4:
//   0 BOOL : v_j in {0,1}          v_j * (ONE - v_j) = 0
//   1 PACK : v_j random            v_j * ONE = v_j
//   2 MUL  : v_j = (v_a + k v_b) v_c     a, b, c BOOL/PACK rows, k small
//   3 MUL2 : v_j = v_a (v_b + x_i)       a a MUL row, b a BOOL/PACK row, x_i a public input
#include <string.h>

#include <thread>
#include <vector>

#include "ctx.h"

namespace mi {

namespace {

inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline uint64_t h3(uint64_t seed, uint64_t j, uint64_t k) { return mix64(mix64(seed ^ mix64(j)) + k); }

fr_t fr_rand(uint64_t seed, uint64_t j) {
    fr_t r;
    for (int w = 0; w < 4; w++) {
        uint64_t x = h3(seed, j, 16 + w);
        r.v[2 * w] = (uint32_t)x;
        r.v[2 * w + 1] = (uint32_t)(x >> 32);
    }
    r.v[7] &= 0x3fffffffu;  // < 2^254 < r
    return r;
}
fr_t fr_u32(uint32_t v) {
    fr_t r = fr_t::zero();
    r.v[0] = v;
    return r;
}

template <class Fn>
void parallel_for(uint64_t n, Fn fn) {
    unsigned T = std::thread::hardware_concurrency();
    if (T > 16) T = 16;
    if (T < 1) T = 1;
    if (n < 4096) T = 1;
    std::vector<std::thread> th;
    uint64_t chunk = (n + T - 1) / T;
    for (unsigned t = 0; t < T; t++) {
        uint64_t lo = t * chunk, hi = lo + chunk < n ? lo + chunk : n;
        if (lo >= hi) break;
        th.emplace_back([=] { fn(lo, hi); });
    }
    for (auto &x : th) x.join();
}

}  // namespace

struct Synth {
    uint64_t n, n_in, n_aux;
    std::vector<uint64_t> rp[3];
    std::vector<uint32_t> col[3];
    std::vector<fr_t> coeff[3];  // canonical
    std::vector<fr_t> z;         // canonical
};

Synth *synth_generate(unsigned log_rows, uint64_t n_in, uint64_t seed, unsigned flags) {
    // MI_SYNTH_UNIFORM_WITNESS: every BOOL row becomes a PACK row (v random, v * ONE = v), so each aux variable is
    // a uniform field element or a product of such -- the MSM scalars of a witness without small values
    const bool uniform = (flags & 1u) != 0;
    if (n_in < 1 || log_rows < 3 || log_rows > 31) throw std::invalid_argument("bad synthetic circuit shape");
    uint64_t d = 1ull << log_rows;
    if (n_in + 8 > d) throw std::invalid_argument("too many inputs for the domain");
    Synth *S = new Synth();
    const uint64_t n = d - n_in;
    S->n = n;
    S->n_in = n_in;
    S->n_aux = n;
    const uint64_t nv = n_in + n;
    S->z.resize(nv);
    const uint64_t nbase = (n + 3) / 4;  // number of 4-row groups
    auto base_row = [&](uint64_t j, uint64_t k) -> uint64_t {  // a BOOL/PACK row (index < n)
        uint64_t h = h3(seed, j, k);
        uint64_t g = (h >> 1) % nbase;
        uint64_t r = 4 * g + (h & 1);
        return r < n ? r : 0;
    };
    auto mul_row = [&](uint64_t j, uint64_t k) -> uint64_t {
        uint64_t h = h3(seed, j, k);
        uint64_t r = 4 * (h % nbase) + 2;
        return r < n ? r : 2;
    };
    auto var = [&](uint64_t row) { return (uint32_t)(n_in + row); };
    std::vector<fr_t> &z = S->z;
    // inputs
    z[0] = fr_u32(1);
    for (uint64_t i = 1; i < n_in; i++) z[i] = fr_rand(seed ^ 0x1234, i);
    // pass 1: BOOL / PACK values
    parallel_for(n, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t j = lo; j < hi; j++) {
            if (j % 4 == 0) z[n_in + j] = uniform ? fr_rand(seed ^ 0x5a5a, j) : fr_u32((uint32_t)(h3(seed, j, 1) & 1));
            if (j % 4 == 1) z[n_in + j] = fr_rand(seed, j);
        }
    });
    // pass 2: MUL
    parallel_for(n, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t j = lo; j < hi; j++) {
            if (j % 4 != 2) continue;
            uint64_t a = base_row(j, 2), b = base_row(j, 3), c = base_row(j, 4);
            uint32_t k = (uint32_t)(h3(seed, j, 5) % 7) + 1;
            fr_t A = to_mont(z[n_in + a]) + to_mont(fr_u32(k)) * to_mont(z[n_in + b]);
            z[n_in + j] = from_mont(A * to_mont(z[n_in + c]));
        }
    });
    // pass 3: MUL2
    parallel_for(n, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t j = lo; j < hi; j++) {
            if (j % 4 != 3) continue;
            uint64_t a = mul_row(j, 2), b = base_row(j, 3);
            uint64_t xi = n_in > 1 ? 1 + h3(seed, j, 6) % (n_in - 1) : 0;
            fr_t B = to_mont(z[n_in + b]);
            if (xi) B = B + to_mont(z[xi]);
            z[n_in + j] = from_mont(to_mont(z[n_in + a]) * B);
        }
    });
    // CSR: per-row term counts are a function of j mod 4 (A, B, C)
    const int cntA[4] = {1, 1, 2, 1}, cntC[4] = {uniform ? 1 : 0, 1, 1, 1};
    auto cntB = [&](uint64_t j) -> int {
        return j % 4 == 0 ? (uniform ? 1 : 2) : (j % 4 == 3 ? (n_in > 1 ? 2 : 1) : 1);
    };
    for (int m = 0; m < 3; m++) S->rp[m].resize(n + 1);
    S->rp[0][0] = S->rp[1][0] = S->rp[2][0] = 0;
    for (uint64_t j = 0; j < n; j++) {
        S->rp[0][j + 1] = S->rp[0][j] + cntA[j % 4];
        S->rp[1][j + 1] = S->rp[1][j] + cntB(j);
        S->rp[2][j + 1] = S->rp[2][j] + cntC[j % 4];
    }
    for (int m = 0; m < 3; m++) {
        S->col[m].resize(S->rp[m][n]);
        S->coeff[m].resize(S->rp[m][n]);
    }
    fr_t one = fr_u32(1);
    fr_t minus_one = from_mont(-fr_t::one());
    parallel_for(n, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t j = lo; j < hi; j++) {
            uint64_t ea = S->rp[0][j], eb = S->rp[1][j], ec = S->rp[2][j];
            uint32_t vj = var(j);
            switch (uniform && j % 4 == 0 ? 1 : j % 4) {
                case 0:  // BOOL: v * (1 - v) = 0
                    S->col[0][ea] = vj;
                    S->coeff[0][ea] = one;
                    S->col[1][eb] = 0;
                    S->coeff[1][eb] = one;
                    S->col[1][eb + 1] = vj;
                    S->coeff[1][eb + 1] = minus_one;
                    break;
                case 1:  // PACK: v * 1 = v
                    S->col[0][ea] = vj;
                    S->coeff[0][ea] = one;
                    S->col[1][eb] = 0;
                    S->coeff[1][eb] = one;
                    S->col[2][ec] = vj;
                    S->coeff[2][ec] = one;
                    break;
                case 2: {  // MUL
                    uint64_t a = base_row(j, 2), b = base_row(j, 3), c = base_row(j, 4);
                    uint32_t k = (uint32_t)(h3(seed, j, 5) % 7) + 1;
                    S->col[0][ea] = var(a);
                    S->coeff[0][ea] = one;
                    S->col[0][ea + 1] = var(b);
                    S->coeff[0][ea + 1] = fr_u32(k);
                    S->col[1][eb] = var(c);
                    S->coeff[1][eb] = one;
                    S->col[2][ec] = vj;
                    S->coeff[2][ec] = one;
                    break;
                }
                default: {  // MUL2
                    uint64_t a = mul_row(j, 2), b = base_row(j, 3);
                    S->col[0][ea] = var(a);
                    S->coeff[0][ea] = one;
                    S->col[1][eb] = var(b);
                    S->coeff[1][eb] = one;
                    if (n_in > 1) {
                        uint64_t xi = 1 + h3(seed, j, 6) % (n_in - 1);
                        S->col[1][eb + 1] = (uint32_t)xi;
                        S->coeff[1][eb + 1] = one;
                    }
                    S->col[2][ec] = vj;
                    S->coeff[2][ec] = one;
                }
            }
        }
    });
    return S;
}

void synth_free(Synth *s) { delete s; }

}  // namespace mi

// ---- C ABI (declared in include/mi355x_groth16.h) ----
#include "../../include/mi355x_groth16.h"

struct mi_synth {
    mi::Synth *p;
};

extern "C" {

int mi_synth_generate(unsigned log_rows, uint64_t num_inputs, uint64_t seed, mi_synth **out) {
    return mi_synth_generate_ex(log_rows, num_inputs, seed, 0, out);
}

int mi_synth_generate_ex(unsigned log_rows, uint64_t num_inputs, uint64_t seed, unsigned flags, mi_synth **out) {
    if (!out) return MI_ERR_ARG;
    try {
        *out = new mi_synth{mi::synth_generate(log_rows, num_inputs, seed, flags)};
        return MI_OK;
    } catch (const std::invalid_argument &) {
        return MI_ERR_ARG;
    } catch (...) {
        return MI_ERR_INTERNAL;
    }
}

int mi_synth_r1cs(const mi_synth *s, mi_r1cs *out) {
    if (!s || !out) return MI_ERR_ARG;
    out->num_constraints = s->p->n;
    out->num_inputs = s->p->n_in;
    out->num_aux = s->p->n_aux;
    for (int m = 0; m < 3; m++) {
        out->row_ptr[m] = s->p->rp[m].data();
        out->col[m] = s->p->col[m].data();
        out->coeff[m] = (const uint8_t *)s->p->coeff[m].data();
    }
    return MI_OK;
}

int mi_synth_witness(const mi_synth *s, const uint8_t **z, uint64_t *num_vars) {
    if (!s || !z || !num_vars) return MI_ERR_ARG;
    *z = (const uint8_t *)s->p->z.data();
    *num_vars = s->p->z.size();
    return MI_OK;
}

void mi_synth_free(mi_synth *s) {
    if (!s) return;
    mi::synth_free(s->p);
    delete s;
}

}  // extern "C"
