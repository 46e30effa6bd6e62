// Host builder of the stacked-PoRep circuit (stacked.h): synthesises the R1CS shape of one partition exactly
// as the reference's gadgets allocate and constrain (bellman boolean / uint32 / multieq / sha256 / num /
// multipack, rust-fil-proofs insertion / por / create_label / encode, neptune's Poseidon circuit; layout
// restated in oracle/stacked_circuit.py, counts pinned by the reference tests), and records the witness
// program the GPU runs.  No witness values are computed here: the shape depends only on which bits are
// constant, as for bellman's blank circuit.
#include <algorithm>
#include <array>
#include <map>
#include <stdexcept>
#include <string>
#include <cstring>
#include <mutex>
#include <thread>
#include <unordered_map>

#include "poseidon_math.h"
#include "stacked.h"

namespace mi {
namespace stacked {

uint64_t poseidon_constraints(unsigned arity) {
    int rf = 0, rp = 0;
    if (!pos_detail::round_numbers(arity, rf, rp)) throw std::invalid_argument("poseidon: arity must be 2, 4, 8 or 11");
    const uint64_t t = arity + 1;
    return 3 * (t - 1) + 4 * ((uint64_t)(rf - 1) * t + rp) + 1;
}

static std::vector<unsigned> tree_arities(uint64_t nodes, unsigned base, unsigned sub, unsigned top) {
    const uint64_t nb = (uint64_t)(sub ? sub : 1) * (top ? top : 1);
    if (nodes % nb) throw std::invalid_argument("stacked: nodes not divisible by the sub/top tree count");
    uint64_t per = nodes / nb;
    std::vector<unsigned> a;
    while (per > 1) {
        if (per % base) throw std::invalid_argument("stacked: base tree size is not a power of the base arity");
        a.push_back(base);
        per /= base;
    }
    if (sub) a.push_back(sub);
    if (top) a.push_back(top);
    return a;
}

Layout layout_for(const Shape &s) {
    Layout L;
    if (!s.nodes || (s.nodes & (s.nodes - 1))) throw std::invalid_argument("stacked: nodes must be a power of two");
    while ((1ull << L.depth_d) < s.nodes) L.depth_d++;
    for (unsigned a : {s.base, s.sub, s.top})
        if (a && a != 2 && a != 4 && a != 8) throw std::invalid_argument("stacked: tree arities must be 2, 4 or 8");
    if (!s.base) throw std::invalid_argument("stacked: base arity required");
    if (s.top && !s.sub) throw std::invalid_argument("stacked: a top tree needs a sub tree");
    L.c_arities = tree_arities(s.nodes, s.base, s.sub, s.top);
    for (unsigned a : L.c_arities) L.path_c += a - 1;
    if (s.sectors) {  // Fallback PoSt: sectors x (comm_r, comm_c, comm_r_last, challenges x (index, leaf, path))
        L.stride = 3 + (uint64_t)s.challenges * (2 + L.path_c);
        L.slots = (uint64_t)s.sectors * L.stride;
        L.unit0 = 0;
        return L;
    }
    L.stride = 2 + L.depth_d + 2 * L.path_c + 14ull * (1 + s.layers + L.path_c);
    L.slots = 5 + (uint64_t)s.challenges * L.stride;
    return L;
}

namespace {

// ------------------------------------------------------------------------------------------ constraint system
struct Term {
    uint64_t z;  // z index (ONE = 0, inputs, then aux), or a symbolic id in a template
    fr_t k;      // Montgomery
};
using LC = std::vector<Term>;
struct Row {
    LC a, b, c;
};

// symbolic ids of a template: ONE = 0, external operand j = EXT + j, internal allocation k = INT + k
constexpr uint64_t EXT = 1ull << 62, INT = 1ull << 61;

fr_t g_pow2[320];  // 2^i, Montgomery
fr_t g_one_m, g_neg1_m;
void init_consts() {
    static bool done = false;
    if (done) return;
    g_one_m = fr_t::one();
    g_neg1_m = -g_one_m;
    g_pow2[0] = g_one_m;
    for (int i = 1; i < 320; i++) g_pow2[i] = g_pow2[i - 1] + g_pow2[i - 1];
    done = true;
}

struct Poseidon {
    unsigned t = 0;
    int rf = 0, rp = 0;
    std::vector<fr_t> rc;   // Montgomery, (rf + rp) x t, unfolded (the literal permutation)
    std::vector<fr_t> mds;  // Montgomery, t x t
    fr_t tag;               // Montgomery, 2^arity - 1
};
const Poseidon &poseidon_consts(unsigned arity) {
    static std::map<unsigned, Poseidon> cache;
    auto it = cache.find(arity);
    if (it != cache.end()) return it->second;
    PoseidonHost h = poseidon_derive(arity, poseidon_sbox_field());
    Poseidon p;
    p.t = h.t;
    p.rf = h.rf;
    p.rp = h.rp;
    for (auto &x : h.plain_rc) p.rc.push_back(to_mont(x));
    for (auto &x : h.plain_mds) p.mds.push_back(to_mont(x));
    p.tag = pos_detail::fr_small((1ull << arity) - 1);  // already Montgomery
    return cache.emplace(arity, std::move(p)).first->second;
}

// Process-wide coefficient pool (canonical values -> dense indices, 0 = one): templates are cached across
// builds with their coefficients already interned, and each Built takes a snapshot of the pool.
struct CoefPool {
    struct H {
        size_t operator()(const fr_t &x) const {
            uint64_t h = 0x9e3779b97f4a7c15ull;
            for (int i = 0; i < 8; i++) h = (h ^ x.v[i]) * 0x100000001b3ull;
            return (size_t)h;
        }
    };
    struct E {
        bool operator()(const fr_t &a, const fr_t &b) const { return memcmp(a.v, b.v, 32) == 0; }
    };
    std::mutex mu;
    std::vector<fr_t> tab;
    std::unordered_map<fr_t, uint32_t, H, E> idx;
    CoefPool() {
        fr_t one = fr_t::zero();
        one.v[0] = 1;
        intern(one);
    }
    uint32_t intern(const fr_t &canonical) {
        std::lock_guard<std::mutex> g(mu);
        auto it = idx.find(canonical);
        if (it != idx.end()) return it->second;
        if (tab.size() >= 0xffffffffull) throw std::runtime_error("stacked: coefficient pool full");
        const uint32_t i = (uint32_t)tab.size();
        tab.push_back(canonical);
        idx.emplace(canonical, i);
        return i;
    }
    fr_t at(uint32_t i) {
        std::lock_guard<std::mutex> g(mu);
        return tab[i];
    }
    std::vector<fr_t> snapshot() {
        std::lock_guard<std::mutex> g(mu);
        return tab;
    }
};
CoefPool &pool() {
    static CoefPool p;
    return p;
}

void canon(LC &lc) {
    std::sort(lc.begin(), lc.end(), [](const Term &x, const Term &y) { return x.z < y.z; });
    size_t o = 0;
    for (size_t i = 0; i < lc.size();) {
        const uint64_t z = lc[i].z;
        fr_t k = lc[i].k;
        size_t j = i + 1;
        for (; j < lc.size() && lc[j].z == z; j++) k = k + lc[j].k;
        if (!k.is_zero()) lc[o++] = Term{z, k};
        i = j;
    }
    lc.resize(o);
}

void lc_add(LC &dst, const LC &src, const fr_t &scale) {
    for (auto &t : src) dst.push_back(Term{t.z, t.k * scale});
}

// Real mode: rows canonicalised and appended to the CSR of `out`.  Template mode (out == nullptr): rows
// kept raw with symbolic ids in `tpl`.
struct CS {
    Built *out = nullptr;
    bool keep = true;
    std::vector<Row> *tpl = nullptr;
    uint64_t n_in_total = 0, next_input = 1, next_aux = 0;

    uint64_t alloc() { return out ? n_in_total + next_aux++ : INT + next_aux++; }
    uint64_t alloc_input() {
        if (!out) throw std::logic_error("stacked: inputs inside a template");
        if (next_input >= n_in_total) throw std::logic_error("stacked: more inputs than the shape predicts");
        return next_input++;
    }
    void enforce(LC a, LC b, LC c) {
        if (!out) {
            tpl->push_back(Row{std::move(a), std::move(b), std::move(c)});
            return;
        }
        out->n_constraints++;
        if (!keep) return;
        LC *m[3] = {&a, &b, &c};
        for (int q = 0; q < 3; q++) {
            canon(*m[q]);
            for (auto &t : *m[q]) {
                out->col[q].push_back((uint32_t)t.z);
                out->cidx[q].push_back(pool().intern(from_mont(t.k)));
            }
            out->rp[q].push_back(out->col[q].size());
        }
    }
};

// ------------------------------------------------------------------------------------------ Boolean (bellman)
struct Bit {
    uint8_t kind;  // 0 constant, 1 Is, 2 Not
    uint8_t val;   // constant value
    uint64_t z;
};
inline Bit bconst(int v) { return Bit{0, (uint8_t)(v & 1), 0}; }
inline Bit bis(uint64_t z) { return Bit{1, 0, z}; }
inline bool is_false(const Bit &b) { return b.kind == 0 && b.val == 0; }
inline bool is_true(const Bit &b) { return b.kind == 0 && b.val == 1; }
inline Bit bnot(const Bit &b) { return b.kind == 0 ? bconst(1 - b.val) : Bit{(uint8_t)(3 - b.kind), 0, b.z}; }
LC blc(const Bit &b, const fr_t &coeff) {
    if (b.kind == 0) return b.val ? LC{Term{0, coeff}} : LC{};
    if (b.kind == 1) return LC{Term{b.z, coeff}};
    return LC{Term{0, coeff}, Term{b.z, -coeff}};
}
using U32 = std::array<Bit, 32>;  // bits[0] = least significant (bellman UInt32)

struct Gadgets {
    CS &cs;
    explicit Gadgets(CS &c) : cs(c) {}

    Bit alloc_bit() {  // AllocatedBit::alloc: (1 - a) * a = 0
        uint64_t v = cs.alloc();
        cs.enforce(LC{Term{0, g_one_m}, Term{v, g_neg1_m}}, LC{Term{v, g_one_m}}, LC{});
        return bis(v);
    }
    uint64_t xor_vars(uint64_t a, uint64_t b) {  // AllocatedBit::xor: (a + a) * b = a + b - c
        uint64_t c = cs.alloc();
        cs.enforce(LC{Term{a, g_pow2[1]}}, LC{Term{b, g_one_m}},
                   LC{Term{a, g_one_m}, Term{b, g_one_m}, Term{c, g_neg1_m}});
        return c;
    }
    Bit and_vars(uint64_t a, uint64_t b) {  // a * b = c
        uint64_t c = cs.alloc();
        cs.enforce(LC{Term{a, g_one_m}}, LC{Term{b, g_one_m}}, LC{Term{c, g_one_m}});
        return bis(c);
    }
    Bit and_not_vars(uint64_t a, uint64_t b) {  // a * (1 - b) = c
        uint64_t c = cs.alloc();
        cs.enforce(LC{Term{a, g_one_m}}, LC{Term{0, g_one_m}, Term{b, g_neg1_m}}, LC{Term{c, g_one_m}});
        return bis(c);
    }
    Bit nor_vars(uint64_t a, uint64_t b) {  // (1 - a) * (1 - b) = c
        uint64_t c = cs.alloc();
        cs.enforce(LC{Term{0, g_one_m}, Term{a, g_neg1_m}}, LC{Term{0, g_one_m}, Term{b, g_neg1_m}},
                   LC{Term{c, g_one_m}});
        return bis(c);
    }
    Bit bxor(const Bit &a, const Bit &b) {  // Boolean::xor
        if (is_false(a)) return b;
        if (is_false(b)) return a;
        if (is_true(a)) return bnot(b);
        if (is_true(b)) return bnot(a);
        if (a.kind != b.kind) {  // Is with Not: NOT(is XOR not's variable), the Is operand first
            uint64_t c = a.kind == 1 ? xor_vars(a.z, b.z) : xor_vars(b.z, a.z);
            return Bit{2, 0, c};
        }
        return bis(xor_vars(a.z, b.z));
    }
    Bit band(const Bit &a, const Bit &b) {  // Boolean::and
        if (is_false(a) || is_false(b)) return bconst(0);
        if (is_true(a)) return b;
        if (is_true(b)) return a;
        if (a.kind == 1 && b.kind == 2) return and_not_vars(a.z, b.z);
        if (a.kind == 2 && b.kind == 1) return and_not_vars(b.z, a.z);
        if (a.kind == 2 && b.kind == 2) return nor_vars(a.z, b.z);
        return and_vars(a.z, b.z);
    }
    Bit ch(const Bit &a, const Bit &b, const Bit &c) {  // Boolean::sha256_ch
        if (a.kind == 0 && b.kind == 0 && c.kind == 0) return bconst((a.val & b.val) ^ ((1 - a.val) & c.val));
        if (is_false(a)) return c;
        if (is_false(b)) return band(bnot(a), c);
        if (is_false(c)) return band(a, b);
        if (is_true(c)) return bnot(band(a, bnot(b)));
        if (is_true(b)) return bnot(band(bnot(a), bnot(c)));
        uint64_t v = cs.alloc();
        LC l1 = blc(b, g_one_m);
        lc_add(l1, blc(c, g_one_m), g_neg1_m);
        LC l3{Term{v, g_one_m}};
        lc_add(l3, blc(c, g_one_m), g_neg1_m);
        cs.enforce(l1, blc(a, g_one_m), l3);  // a (b - c) = ch - c
        return bis(v);
    }
    Bit maj(const Bit &a, const Bit &b, const Bit &c) {  // Boolean::sha256_maj
        if (a.kind == 0 && b.kind == 0 && c.kind == 0)
            return bconst((a.val & b.val) ^ (a.val & c.val) ^ (b.val & c.val));
        if (is_false(a)) return band(b, c);
        if (is_false(b)) return band(a, c);
        if (is_false(c)) return band(a, b);
        if (is_true(c)) return bnot(band(bnot(a), bnot(b)));
        if (is_true(b)) return bnot(band(bnot(a), bnot(c)));
        if (is_true(a)) return bnot(band(bnot(b), bnot(c)));
        uint64_t v = cs.alloc();
        Bit bc = band(b, c);
        LC l1 = blc(bc, g_pow2[1]);
        lc_add(l1, blc(b, g_one_m), g_neg1_m);
        lc_add(l1, blc(c, g_one_m), g_neg1_m);
        LC l3 = blc(bc, g_one_m);
        l3.push_back(Term{v, g_neg1_m});
        cs.enforce(l1, blc(a, g_one_m), l3);  // (2bc - b - c) a = bc - maj
        return bis(v);
    }

    static U32 u32c(uint32_t x) {
        U32 u;
        for (int i = 0; i < 32; i++) u[i] = bconst((x >> i) & 1);
        return u;
    }
    static U32 rotr(const U32 &u, int k) {
        U32 o;
        for (int i = 0; i < 32; i++) o[i] = u[(i + k) % 32];
        return o;
    }
    static U32 shr(const U32 &u, int k) {
        U32 o;
        for (int i = 0; i < 32; i++) o[i] = i + k < 32 ? u[i + k] : bconst(0);
        return o;
    }
    U32 x32(const U32 &a, const U32 &b) {
        U32 o;
        for (int i = 0; i < 32; i++) o[i] = bxor(a[i], b[i]);
        return o;
    }
    struct MultiEq {  // bellman MultiEq: equalities packed while they fit under CAPACITY (254) bits
        CS &cs;
        unsigned bits = 0;
        LC lhs, rhs;
        explicit MultiEq(CS &c) : cs(c) {}
        void accumulate() {
            cs.enforce(lhs, LC{Term{0, g_one_m}}, rhs);
            lhs.clear();
            rhs.clear();
            bits = 0;
        }
        void enforce_equal(unsigned nb, const LC &l, const LC &r) {
            if (254 <= bits + nb) accumulate();
            lc_add(lhs, l, g_pow2[bits]);
            lc_add(rhs, r, g_pow2[bits]);
            bits += nb;
        }
        void close() {
            if (bits > 0) accumulate();
        }
    };
    U32 addmany(MultiEq &me, const std::vector<const U32 *> &ops) {  // UInt32::addmany
        bool all_const = true;
        uint64_t cval = 0;
        for (auto *o : ops)
            for (int i = 0; i < 32; i++) {
                if ((*o)[i].kind != 0)
                    all_const = false;
                else
                    cval += (uint64_t)(*o)[i].val << i;
            }
        if (all_const) return u32c((uint32_t)cval);
        LC lc;
        for (auto *o : ops)
            for (int i = 0; i < 32; i++) {
                const Bit &b = (*o)[i];
                if (b.kind == 0) {
                    if (b.val) lc.push_back(Term{0, g_pow2[i]});
                } else if (b.kind == 1) {
                    lc.push_back(Term{b.z, g_pow2[i]});
                } else {
                    lc.push_back(Term{0, g_pow2[i]});
                    lc.push_back(Term{b.z, -g_pow2[i]});
                }
            }
        unsigned nb = 0;
        for (uint64_t mx = (uint64_t)ops.size() * 0xFFFFFFFFull; mx; mx >>= 1) nb++;
        U32 res;
        LC rlc;
        for (unsigned i = 0; i < nb; i++) {
            Bit b = alloc_bit();
            if (i < 32) res[i] = b;
            rlc.push_back(Term{b.z, g_pow2[i]});
        }
        me.enforce_equal(nb, lc, rlc);
        return res;
    }

    // bellman sha256_compression_function
    std::array<U32, 8> compress(const std::array<U32, 16> &msg, const std::array<U32, 8> &H) {
        static const uint32_t K[64] = {
            0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
            0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
            0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
            0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
            0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
            0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
            0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
            0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
        std::vector<U32> w(msg.begin(), msg.end());
        w.reserve(64);
        MultiEq me(cs);
        for (int i = 16; i < 64; i++) {
            U32 s0 = x32(rotr(w[i - 15], 7), rotr(w[i - 15], 18));
            s0 = x32(s0, shr(w[i - 15], 3));
            U32 s1 = x32(rotr(w[i - 2], 17), rotr(w[i - 2], 19));
            s1 = x32(s1, shr(w[i - 2], 10));
            U32 nw = addmany(me, {&w[i - 16], &s0, &w[i - 7], &s1});
            w.push_back(nw);
        }
        struct Maybe {  // a / e: a concrete word or a deferred operand list
            bool concrete;
            U32 v;
            std::vector<U32> ops;
        };
        auto compute = [&](const Maybe &m, std::vector<const U32 *> others) -> U32 {
            if (m.concrete) return m.v;
            std::vector<const U32 *> ops;
            for (auto &o : m.ops) ops.push_back(&o);
            for (auto *o : others) ops.push_back(o);
            return addmany(me, ops);
        };
        Maybe a{true, H[0], {}}, e{true, H[4], {}};
        U32 b = H[1], c = H[2], d = H[3], f = H[5], g = H[6], h = H[7];
        for (int i = 0; i < 64; i++) {
            U32 ne = compute(e, {});
            U32 s1 = x32(rotr(ne, 6), rotr(ne, 11));
            s1 = x32(s1, rotr(ne, 25));
            U32 chv;
            for (int q = 0; q < 32; q++) chv[q] = ch(ne[q], f[q], g[q]);
            const U32 kk = u32c(K[i]);
            U32 na = compute(a, {});
            U32 s0 = x32(rotr(na, 2), rotr(na, 13));
            s0 = x32(s0, rotr(na, 22));
            U32 mj;
            for (int q = 0; q < 32; q++) mj[q] = maj(na[q], b[q], c[q]);
            // temp1 = h + S1 + ch + k + w (this round's h); e = d + temp1; a = temp1 + S0 + maj
            Maybe ne_e{false, {}, {h, s1, chv, kk, w[i], d}};
            Maybe ne_a{false, {}, {h, s1, chv, kk, w[i], s0, mj}};
            h = g;
            g = f;
            f = ne;
            e = std::move(ne_e);
            d = c;
            c = b;
            b = na;
            a = std::move(ne_a);
        }
        std::array<U32, 8> out;
        out[0] = compute(a, {&H[0]});
        out[1] = addmany(me, {&H[1], &b});
        out[2] = addmany(me, {&H[2], &c});
        out[3] = addmany(me, {&H[3], &d});
        out[4] = compute(e, {&H[4]});
        out[5] = addmany(me, {&H[5], &f});
        out[6] = addmany(me, {&H[6], &g});
        out[7] = addmany(me, {&H[7], &h});
        me.close();
        return out;
    }

    // neptune poseidon_hash circuit in the layout oracle/stacked_circuit.py states: literal rounds (ARK,
    // S-box, state' = state * M), linear-combination state; 3 constraints per first-round S-box of an input
    // (the domain tag's is constant), 4 per later S-box (input LC allocated first), 1 for the digest.
    uint64_t poseidon(const std::vector<uint64_t> &inputs, unsigned arity) {
        const Poseidon &P = poseidon_consts(arity);
        const unsigned t = P.t;
        std::vector<LC> st(t);
        st[0] = LC{Term{0, P.tag}};
        for (unsigned i = 1; i < t; i++) st[i] = LC{Term{inputs[i - 1], g_one_m}};
        const int half = P.rf / 2;
        size_t k = 0;
        for (int rnd = 0; rnd < P.rf + P.rp; rnd++) {
            for (unsigned i = 0; i < t; i++) {
                st[i].push_back(Term{0, P.rc[k + i]});
                canon(st[i]);
            }
            k += t;
            const bool full = rnd < half || rnd >= half + P.rp;
            for (unsigned i = 0; i < (full ? t : 1u); i++) {
                LC &x = st[i];
                bool constant = true;
                for (auto &tm : x)
                    if (tm.z != 0) constant = false;
                if (constant) {
                    fr_t c = x.empty() ? fr_t::zero() : x[0].k;
                    fr_t c2 = c * c;
                    x = LC{Term{0, c2 * c2 * c}};
                    canon(x);
                    continue;
                }
                LC v_lc;
                if (rnd == 0) {
                    v_lc = x;
                } else {
                    uint64_t v = cs.alloc();
                    cs.enforce(x, LC{Term{0, g_one_m}}, LC{Term{v, g_one_m}});
                    v_lc = LC{Term{v, g_one_m}};
                }
                uint64_t l2 = cs.alloc();
                cs.enforce(v_lc, v_lc, LC{Term{l2, g_one_m}});
                uint64_t l4 = cs.alloc();
                cs.enforce(LC{Term{l2, g_one_m}}, LC{Term{l2, g_one_m}}, LC{Term{l4, g_one_m}});
                uint64_t l5 = cs.alloc();
                cs.enforce(LC{Term{l4, g_one_m}}, v_lc, LC{Term{l5, g_one_m}});
                x = LC{Term{l5, g_one_m}};
            }
            std::vector<LC> nst(t);
            for (unsigned j = 0; j < t; j++) {
                for (unsigned i = 0; i < t; i++) lc_add(nst[j], st[i], P.mds[i * t + j]);
                canon(nst[j]);
            }
            st.swap(nst);
        }
        uint64_t out = cs.alloc();
        cs.enforce(st[1], LC{Term{0, g_one_m}}, LC{Term{out, g_one_m}});
        return out;
    }
};

// ------------------------------------------------------------------------------------------ templates
struct Template {
    std::vector<Row> rows;  // as recorded (symbolic ids, Montgomery); released by flatten()
    uint64_t n_int = 0;
    std::vector<uint64_t> outs;  // symbolic ids of the outputs (SHA: 256 state bits as Is; Poseidon: digest)
    // flat form: per row and matrix the end offset of its terms; ids and pooled coefficient indices
    std::vector<uint32_t> ends;  // 3 per row
    std::vector<uint64_t> ids;
    std::vector<uint32_t> ks;
    void flatten() {
        for (const Row &r : rows)
            for (const LC *lc : {&r.a, &r.b, &r.c}) {
                LC x = *lc;
                canon(x);  // symbolic ids are distinct per operand; instantiate merges repeated operands
                for (auto &t : x) {
                    ids.push_back(t.z);
                    ks.push_back(pool().intern(from_mont(t.k)));
                }
                ends.push_back((uint32_t)ids.size());
            }
        rows.clear();
        rows.shrink_to_fit();
    }
};

// SHA-256 compression template over a constant pattern: message bit j (big-endian order) variable -> EXT + j,
// state bit (word w, bit i) variable -> EXT + 512 + 32 w + i (iv = 0), else the IV constants
const Template &sha_template(const std::string &pattern, bool iv) {
    static std::map<std::string, Template> cache;
    const std::string key = pattern + (iv ? "I" : "S");
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    static const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    Template T;
    CS cs;
    cs.tpl = &T.rows;
    Gadgets g(cs);
    std::array<U32, 16> msg;
    for (int wd = 0; wd < 16; wd++)
        for (int t = 0; t < 32; t++) {
            const int j = 32 * wd + t;
            const char p = pattern[j];
            msg[wd][31 - t] = p == 'v' ? bis(EXT + j) : bconst(p == '1');  // from_bits_be
        }
    std::array<U32, 8> H;
    for (int wd = 0; wd < 8; wd++)
        H[wd] = iv ? Gadgets::u32c(IV[wd]) : [&] {
            U32 u;
            for (int i = 0; i < 32; i++) u[i] = bis(EXT + 512 + 32 * wd + i);
            return u;
        }();
    auto out = g.compress(msg, H);
    for (int wd = 0; wd < 8; wd++)
        for (int i = 0; i < 32; i++) {
            if (out[wd][i].kind != 1) throw std::logic_error("stacked: SHA-256 compression output not allocated");
            T.outs.push_back(out[wd][i].z);
        }
    T.n_int = cs.next_aux;
    T.flatten();
    return cache.emplace(key, std::move(T)).first->second;
}

const Template &poseidon_template(unsigned arity) {
    static std::map<unsigned, Template> cache;
    auto it = cache.find(arity);
    if (it != cache.end()) return it->second;
    Template T;
    CS cs;
    cs.tpl = &T.rows;
    Gadgets g(cs);
    std::vector<uint64_t> in;
    for (unsigned j = 0; j < arity; j++) in.push_back(EXT + j);
    T.outs.push_back(g.poseidon(in, arity));
    T.n_int = cs.next_aux;
    T.flatten();
    return cache.emplace(arity, std::move(T)).first->second;
}

// instantiate: externals ext[j], internals base + k; rows remapped, canonicalised, appended
uint64_t instantiate(CS &cs, const Template &T, const std::vector<uint64_t> &ext) {
    const uint64_t base = cs.n_in_total + cs.next_aux;
    cs.next_aux += T.n_int;
    const size_t nrows = T.ends.size() / 3;
    cs.out->n_constraints += nrows;
    if (!cs.keep) return base;
    Built &b = *cs.out;
    struct ZK {
        uint64_t z;
        uint32_t k;  // pooled coefficient index
    };
    static thread_local std::vector<ZK> buf;
    uint32_t beg = 0;
    for (size_t r = 0; r < nrows; r++)
        for (int q = 0; q < 3; q++) {
            const uint32_t end = T.ends[3 * r + q];
            buf.clear();
            bool sorted = true;
            for (uint32_t e = beg; e < end; e++) {
                const uint64_t id = T.ids[e];
                const uint64_t z = id >= EXT ? ext[id - EXT] : id >= INT ? base + (id - INT) : id;
                if (!buf.empty() && z <= buf.back().z) sorted = false;
                buf.push_back(ZK{z, T.ks[e]});
            }
            beg = end;
            if (!sorted) {  // repeated operands (parents repeated in a message) or a remapped order
                std::sort(buf.begin(), buf.end(), [](const ZK &x, const ZK &y) { return x.z < y.z; });
                size_t o = 0;
                for (size_t i = 0; i < buf.size();) {
                    ZK t = buf[i];
                    size_t j = i + 1;
                    if (j < buf.size() && buf[j].z == t.z) {  // repeated operand: the summed coefficient (mod r)
                        fr_t k = pool().at(t.k);
                        for (; j < buf.size() && buf[j].z == t.z; j++) k = k + pool().at(buf[j].k);
                        if (k.is_zero()) {
                            i = j;
                            continue;
                        }
                        t.k = pool().intern(k);
                    }
                    buf[o++] = t;
                    i = j;
                }
                buf.resize(o);
            }
            for (auto &t : buf) {
                b.col[q].push_back((uint32_t)t.z);
                b.cidx[q].push_back(t.k);
            }
            b.rp[q].push_back(b.col[q].size());
        }
    return base;
}

// ------------------------------------------------------------------------------------------ the synthesis
struct Word {  // one SHA-256 message word: its descriptor and its bits in message (big-endian) order
    uint64_t desc;
    std::array<Bit, 32> be;
};

struct Synth {
    Built &b;
    CS cs;
    Gadgets g;
    std::vector<uint32_t> lvl;  // phase-A level of the op producing each aux variable
    explicit Synth(Built &bb, bool keep) : b(bb), g(cs) {
        cs.out = &bb;
        cs.keep = keep;
        cs.n_in_total = bb.shape.sectors ? 1 + (uint64_t)bb.shape.sectors * (1 + bb.shape.challenges)
                                         : 4 + 18ull * bb.shape.challenges;
        for (int m = 0; m < 3; m++) b.rp[m].assign(1, 0);
    }
    uint32_t level_of(uint64_t z) const {
        if (z < cs.n_in_total) return 0;
        const uint64_t a = z - cs.n_in_total;
        return a < lvl.size() ? lvl[a] : 0;
    }
    // an op at 1 + the deepest producer among deps; its output variables [out0, out0 + nout) get its level
    void emit(WOp op, std::initializer_list<uint64_t> deps, uint64_t out0, uint64_t nout) {
        std::vector<uint64_t> d(deps);
        emit_v(op, d, out0, nout);
    }
    void emit_v(WOp op, const std::vector<uint64_t> &deps, uint64_t out0, uint64_t nout) {
        uint32_t L = 0;
        for (uint64_t z : deps) L = std::max(L, level_of(z) + 1);
        op.level = L;
        b.ops.push_back(op);
        if (out0 >= cs.n_in_total) {
            const uint64_t a = out0 - cs.n_in_total;
            if (lvl.size() < a + nout) lvl.resize(a + nout, 0);
            for (uint64_t i = 0; i < nout; i++) lvl[a + i] = L;
        }
    }
    WOp mk(uint32_t type, uint64_t dst, uint64_t a = 0, uint64_t bb = 0, uint64_t c = 0, uint32_t n = 0) {
        WOp o{};
        o.type = type;
        o.n = n;
        o.dst = dst;
        o.a = a;
        o.b = bb;
        o.c = c;
        return o;
    }

    // ---- num / multipack
    uint64_t alloc_data(uint64_t slot) {
        uint64_t v = cs.alloc();
        emit(mk(W_DATA, v, slot), {}, v, 1);
        return v;
    }
    uint64_t inputize(uint64_t var) {  // input * 1 = var
        uint64_t in = cs.alloc_input();
        cs.enforce(LC{Term{in, g_one_m}}, LC{Term{0, g_one_m}}, LC{Term{var, g_one_m}});
        emit(mk(W_COPY, in, var), {var}, in, 1);
        return in;
    }
    uint64_t to_bits_le(uint64_t var) {  // 255 AllocatedBits, then 0 * 0 = sum 2^i b_i - x
        const uint64_t b0 = cs.n_in_total + cs.next_aux;
        LC lc;
        for (int i = 0; i < 255; i++) {
            Bit bt = g.alloc_bit();
            lc.push_back(Term{bt.z, g_pow2[i]});
        }
        lc.push_back(Term{var, g_neg1_m});
        cs.enforce(LC{}, LC{}, lc);
        emit(mk(W_BITS, b0, var, 0, 0, 255), {var}, b0, 255);
        return b0;
    }
    // pack_into_inputs of bits whose value is the low `nbits` bits of a data slot's u64 (path index bits,
    // the challenge UInt64)
    uint64_t pack_input_bits(const std::vector<Bit> &bits, uint64_t slot) {
        if (bits.size() > 253) throw std::logic_error("stacked: path longer than one packed input");
        LC lc;
        for (size_t i = 0; i < bits.size(); i++) {
            LC t = blc(bits[i], g_pow2[i]);
            lc.insert(lc.end(), t.begin(), t.end());
        }
        uint64_t in = cs.alloc_input();
        cs.enforce(lc, LC{Term{0, g_one_m}}, LC{Term{in, g_one_m}});
        emit(mk(W_DPACK, in, slot, 0, 0, (uint32_t)bits.size()), {}, in, 1);
        return in;
    }
    std::vector<Bit> data_bits(uint64_t slot, unsigned n, unsigned shift) {  // AllocatedBit::alloc x n
        const uint64_t b0 = cs.n_in_total + cs.next_aux;
        std::vector<Bit> out;
        for (unsigned i = 0; i < n; i++) out.push_back(g.alloc_bit());
        emit(mk(W_DBITS, b0, slot, shift, 0, n), {}, b0, n);
        return out;
    }
    void equal(uint64_t a, uint64_t bb) { cs.enforce(LC{Term{a, g_one_m}}, LC{Term{0, g_one_m}}, LC{Term{bb, g_one_m}}); }
    uint64_t add(uint64_t a, uint64_t bb) {  // constraint::add: (a + b) * 1 = sum
        uint64_t s = cs.alloc();
        cs.enforce(LC{Term{a, g_one_m}, Term{bb, g_one_m}}, LC{Term{0, g_one_m}}, LC{Term{s, g_one_m}});
        emit(mk(W_ADD, s, a, bb), {a, bb}, s, 1);
        return s;
    }
    uint64_t pick(const Bit &cond, uint64_t a, uint64_t bb) {  // (b - a) * cond = b - c
        uint64_t c = cs.alloc();
        cs.enforce(LC{Term{bb, g_one_m}, Term{a, g_neg1_m}}, blc(cond, g_one_m), LC{Term{bb, g_one_m}, Term{c, g_neg1_m}});
        emit(mk(W_PICK, c, a, bb, cond.z), {a, bb, cond.z}, c, 1);
        return c;
    }
    std::vector<uint64_t> insert(uint64_t el, const std::vector<Bit> &bits, const std::vector<uint64_t> &els) {
        const size_t size = els.size() + 1;
        if (size == 2) return {pick(bits[0], els[0], el), pick(bits[0], el, els[0])};
        if (size == 4) {
            const Bit &b0 = bits[0], &b1 = bits[1];
            uint64_t a = el, bb = els[0], c = els[1], d = els[2];
            uint64_t p0_x0 = pick(b0, bb, a), p0 = pick(b1, bb, p0_x0);
            uint64_t p1_x0 = pick(b0, a, bb), p1 = pick(b1, c, p1_x0);
            uint64_t p2_x1 = pick(b0, d, a), p2 = pick(b1, p2_x1, c);
            uint64_t p3_x1 = pick(b0, a, d), p3 = pick(b1, p3_x1, d);
            return {p0, p1, p2, p3};
        }
        if (size == 8) {
            const Bit &b0 = bits[0], &b1 = bits[1], &b2 = bits[2];
            uint64_t a = el, bb = els[0], c = els[1], d = els[2], e = els[3], f = els[4], gg = els[5], h = els[6];
            Bit nor01 = g.nor_vars(b0.z, b1.z);
            emit(mk(W_NOR, nor01.z, b0.z, b1.z), {b0.z, b1.z}, nor01.z, 1);
            Bit and01 = g.and_vars(b0.z, b1.z);
            emit(mk(W_AND, and01.z, b0.z, b1.z), {b0.z, b1.z}, and01.z, 1);
            uint64_t p0_xx0 = pick(nor01, a, bb), p0 = pick(b2, bb, p0_xx0);
            uint64_t p1_x00 = pick(b0, a, bb), p1_xx0 = pick(b1, c, p1_x00), p1 = pick(b2, c, p1_xx0);
            uint64_t p2_x10 = pick(b0, d, a), p2_xx0 = pick(b1, p2_x10, c), p2 = pick(b2, d, p2_xx0);
            uint64_t p3_xx0 = pick(and01, a, d), p3 = pick(b2, e, p3_xx0);
            uint64_t p4_xx1 = pick(nor01, a, f), p4 = pick(b2, p4_xx1, e);
            uint64_t p5_x01 = pick(b0, a, f), p5_xx1 = pick(b1, gg, p5_x01), p5 = pick(b2, p5_xx1, f);
            uint64_t p6_x11 = pick(b0, h, a), p6_xx1 = pick(b1, p6_x11, gg), p6 = pick(b2, p6_xx1, gg);
            uint64_t p7_xx1 = pick(and01, a, h), p7 = pick(b2, p7_xx1, h);
            return {p0, p1, p2, p3, p4, p5, p6, p7};
        }
        throw std::logic_error("stacked: insert arity");
    }

    // ---- hashes
    uint64_t poseidon(const std::vector<uint64_t> &in) {
        const unsigned arity = (unsigned)in.size();
        const Template &T = poseidon_template(arity);
        const uint64_t base = instantiate(cs, T, in);
        const uint64_t out = base + (T.outs[0] - INT);
        WOp op = mk(W_POSEIDON, base, b.pin.size(), out, 0, arity);
        b.pin.insert(b.pin.end(), in.begin(), in.end());
        emit_v(op, in, base, T.n_int);
        b.poseidon_ops.push_back(b.ops.size() - 1);
        return out;
    }
    // bellman sha256 over whole words (padding appended here), then pack_bits of the first 254 digest bits
    // in little-endian bit order per byte; one W_SHA op with its blocks
    uint64_t sha256_pack(std::vector<Word> words) {
        const uint64_t nbits = 32ull * words.size();
        auto cw = [&](uint32_t x) {
            Word w;
            w.desc = WD_CONST | x;
            for (int t = 0; t < 32; t++) w.be[t] = bconst((x >> (31 - t)) & 1);
            return w;
        };
        words.push_back(cw(0x80000000u));
        while ((words.size() * 32 + 64) % 512) words.push_back(cw(0));
        words.push_back(cw((uint32_t)(nbits >> 32)));
        words.push_back(cw((uint32_t)nbits));
        const size_t nblocks = words.size() / 16;
        std::vector<uint64_t> deps;
        for (auto &w : words)
            if ((w.desc >> 62) == 1) deps.push_back((w.desc & ((1ull << 62) - 1)) >> 3);
        const uint64_t op_index = b.ops.size();
        const uint64_t first_block = b.blocks.size();
        std::array<U32, 8> H;
        uint64_t base0 = 0;
        for (size_t k = 0; k < nblocks; k++) {
            std::string pat(512, '0');
            std::vector<uint64_t> ext(512 + 256, 0);
            ShaBlock blk{};
            for (int wd = 0; wd < 16; wd++) {
                const Word &w = words[16 * k + wd];
                blk.desc[wd] = w.desc;
                for (int t = 0; t < 32; t++) {
                    const Bit &bt = w.be[t];
                    const int j = 32 * wd + t;
                    if (bt.kind == 0) {
                        pat[j] = bt.val ? '1' : '0';
                    } else {
                        if (bt.kind != 1) throw std::logic_error("stacked: negated message bit");
                        pat[j] = 'v';
                        ext[j] = bt.z;
                    }
                }
            }
            if (k > 0)
                for (int wd = 0; wd < 8; wd++)
                    for (int i = 0; i < 32; i++) ext[512 + 32 * wd + i] = H[wd][i].z;
            const Template &T = sha_template(pat, k == 0);
            const uint64_t base = instantiate(cs, T, ext);
            if (k == 0) base0 = base;
            for (int wd = 0; wd < 8; wd++)
                for (int i = 0; i < 32; i++) H[wd][i] = bis(base + (T.outs[32 * wd + i] - INT));
            blk.base = base;
            blk.iv = k == 0;
            blk.op = (uint32_t)op_index;
            b.blocks.push_back(blk);
        }
        // output bits in big-endian order, then per byte reversed -> LE bits; first 254 packed
        std::vector<Bit> be;
        for (int wd = 0; wd < 8; wd++)
            for (int t = 0; t < 32; t++) be.push_back(H[wd][31 - t]);
        LC lc;
        int i = 0;
        for (int byte = 0; byte < 32 && i < 254; byte++)
            for (int q = 7; q >= 0 && i < 254; q--, i++) lc.push_back(Term{be[8 * byte + q].z, g_pow2[i]});
        const uint64_t pack = cs.alloc();
        cs.enforce(lc, LC{Term{0, g_one_m}}, LC{Term{pack, g_one_m}});
        WOp op = mk(W_SHA, base0, first_block, pack, 0, (uint32_t)nblocks);
        emit_v(op, deps, pack, 1);
        b.sha_ops.push_back(b.ops.size() - 1);
        return pack;
    }
    // the 8 words of reverse_bit_numbering(to_bits_le(var)) (bits at b0 .. b0 + 254, bit 255 constant 0)
    void fr_words(uint64_t var, uint64_t b0, std::vector<Word> &out) {
        std::array<Bit, 256> le;
        for (int i = 0; i < 255; i++) le[i] = bis(b0 + i);
        le[255] = bconst(0);
        for (int k = 0; k < 8; k++) {
            Word w;
            w.desc = WD_FR | (var << 3) | (uint64_t)k;
            for (int t = 0; t < 32; t++) {
                const int m = 32 * k + t;  // message bit: byte m / 8, reversed within the byte
                w.be[t] = le[8 * (m / 8) + 7 - (m % 8)];
            }
            out.push_back(w);
        }
    }
    uint64_t sha_hash2(uint64_t a, uint64_t bb) {  // Sha256Function::hash2_circuit
        const uint64_t ab = to_bits_le(a);
        const uint64_t bbits = to_bits_le(bb);
        std::vector<Word> m;
        fr_words(a, ab, m);
        fr_words(bb, bbits, m);
        return sha256_pack(std::move(m));
    }

    // ---- PoR (private): per level index bits, siblings, insert, hash; path packed into one input; root check
    void por(uint64_t leaf, uint64_t index_slot, uint64_t sib_slot, const std::vector<unsigned> &arities,
             bool sha, uint64_t root) {
        uint64_t cur = leaf;
        std::vector<Bit> path;
        unsigned shift = 0;
        for (unsigned a : arities) {
            const unsigned nb = a == 2 ? 1 : a == 4 ? 2 : 3;
            std::vector<Bit> bits = data_bits(index_slot, nb, shift);
            path.insert(path.end(), bits.begin(), bits.end());
            std::vector<uint64_t> sibs;
            for (unsigned j = 0; j + 1 < a; j++) sibs.push_back(alloc_data(sib_slot++));
            std::vector<uint64_t> ins = insert(cur, bits, sibs);
            cur = sha ? sha_hash2(ins[0], ins[1]) : poseidon(ins);
            shift += nb;
        }
        pack_input_bits(path, index_slot);
        equal(cur, root);
    }

    // ---- create_label (stacked/circuit/create_label.rs)
    uint64_t create_label(uint64_t rid, uint64_t rid_bits, const std::vector<std::pair<uint64_t, uint64_t>> &parents,
                          unsigned layer, uint64_t chal_slot, uint64_t chal_bits) {
        std::vector<Word> m;
        fr_words(rid, rid_bits, m);
        Word lw;
        lw.desc = WD_CONST | layer;
        for (int t = 0; t < 32; t++) lw.be[t] = bconst((layer >> (31 - t)) & 1);
        m.push_back(lw);
        for (int k = 0; k < 2; k++) {  // UInt64::to_bits_be
            Word w;
            w.desc = WD_U64 | (chal_slot << 1) | (uint64_t)k;
            for (int t = 0; t < 32; t++) w.be[t] = bis(chal_bits + 63 - (32 * k + t));
            m.push_back(w);
        }
        while (m.size() < 16) {
            Word w;
            w.desc = WD_CONST;
            for (int t = 0; t < 32; t++) w.be[t] = bconst(0);
            m.push_back(w);
        }
        for (auto &p : parents) fr_words(p.first, p.second, m);
        return sha256_pack(std::move(m));
    }

    struct Mark {
        uint64_t aux0 = 0, in0 = 0, row0[3] = {0, 0, 0}, ops0 = 0, blocks0 = 0, pin0 = 0, pos0 = 0, sha0 = 0, ncons0 = 0;
    } mark;

    // copies of unit 0 (a challenge; PoSt: a sector) for units 1 .. C - 1: unit-local aux variables shift by
    // c x (aux per unit), local inputs by c x (inputs per unit), unit slots by c x stride; rows keep their
    // canonical order (the shift is monotone and leaves global variables below local ones)
    void replicate(unsigned C, uint64_t inputs_per_unit) {
        const uint64_t nin = cs.n_in_total;
        const uint64_t A = cs.next_aux - mark.aux0, I = cs.next_input - mark.in0;
        const uint64_t zl = nin + mark.aux0;  // first unit-local aux z
        const uint64_t S = b.lay.stride, U0 = b.lay.unit0;
        if (I != inputs_per_unit) throw std::logic_error("stacked: unexpected input count per replicated unit");
        if (C == 1) return;
        auto zmap = [&](uint64_t z, uint64_t c) -> uint64_t {
            if (z >= zl) return z + c * A;
            if (z >= mark.in0 && z < mark.in0 + I) return z + c * I;
            return z;
        };
        auto smap = [&](uint64_t slot, uint64_t c) -> uint64_t { return slot >= U0 ? slot + c * S : slot; };
        // R1CS
        if (cs.keep) {
            std::vector<std::thread> th;
            for (int m = 0; m < 3; m++) {
                auto &rp = b.rp[m];
                auto &col = b.col[m];
                auto &co = b.cidx[m];
                const uint64_t r0 = mark.row0[m], r1 = rp.size() - 1, nr = r1 - r0;
                const uint64_t e0 = rp[r0], e1 = rp[r1], ne = e1 - e0;
                rp.resize(rp.size() + (C - 1) * nr);
                col.resize(col.size() + (C - 1) * ne);
                co.resize(co.size() + (C - 1) * ne);
                const unsigned nt = std::max(1u, std::min(C - 1, 5u));  // 3 matrices x 5 threads: within a 16-CPU share
                for (unsigned t = 0; t < nt; t++)
                    th.emplace_back([&, m, r0, nr, e0, ne, t, nt] {
                        for (uint64_t c = 1 + t; c < C; c += nt) {
                            const uint64_t ro = r0 + c * nr, eo = e0 + c * ne;
                            for (uint64_t r = 1; r <= nr; r++) b.rp[m][ro + r] = b.rp[m][r0 + r] + c * ne;
                            for (uint64_t e = 0; e < ne; e++) {
                                b.col[m][eo + e] = (uint32_t)zmap(b.col[m][e0 + e], c);
                                b.cidx[m][eo + e] = b.cidx[m][e0 + e];
                            }
                        }
                    });
            }
            for (auto &t : th) t.join();
        }
        b.n_constraints += (C - 1) * (b.n_constraints - mark.ncons0);
        // witness program
        const uint64_t o0 = mark.ops0, o1 = b.ops.size(), k0 = mark.blocks0, k1 = b.blocks.size();
        const uint64_t p0 = mark.pin0, p1 = b.pin.size();
        const uint64_t q0 = mark.pos0, q1 = b.poseidon_ops.size(), h0 = mark.sha0, h1 = b.sha_ops.size();
        for (uint64_t c = 1; c < C; c++) {
            const uint64_t dop = b.ops.size() - o0, dblk = b.blocks.size() - k0, dpin = b.pin.size() - p0;
            for (uint64_t i = o0; i < o1; i++) {
                WOp op = b.ops[i];
                op.dst = zmap(op.dst, c);
                switch (op.type) {
                    case W_DATA: case W_DBITS: case W_DPACK: op.a = smap(op.a, c); break;
                    case W_COPY: case W_BITS: op.a = zmap(op.a, c); break;
                    case W_PICK: op.a = zmap(op.a, c); op.b = zmap(op.b, c); op.c = zmap(op.c, c); break;
                    case W_AND: case W_NOR: case W_ADD: op.a = zmap(op.a, c); op.b = zmap(op.b, c); break;
                    case W_POSEIDON: op.a += dpin; op.b = zmap(op.b, c); break;
                    case W_SHA: op.a += dblk; op.b = zmap(op.b, c); break;
                    default: throw std::logic_error("stacked: unknown op");
                }
                b.ops.push_back(op);
            }
            for (uint64_t k = k0; k < k1; k++) {
                ShaBlock blk = b.blocks[k];
                blk.base = zmap(blk.base, c);
                blk.op = (uint32_t)(blk.op + dop);
                for (auto &d : blk.desc) {
                    const uint64_t kind = d >> 62, pay = d & ((1ull << 62) - 1);
                    if (kind == 1) d = WD_FR | (zmap(pay >> 3, c) << 3) | (pay & 7);
                    else if (kind == 2) d = WD_U64 | (smap(pay >> 1, c) << 1) | (pay & 1);
                }
                b.blocks.push_back(blk);
            }
            for (uint64_t i = p0; i < p1; i++) b.pin.push_back(zmap(b.pin[i], c));
            for (uint64_t i = q0; i < q1; i++) b.poseidon_ops.push_back(b.poseidon_ops[i] + dop);
            for (uint64_t i = h0; i < h1; i++) b.sha_ops.push_back(b.sha_ops[i] + dop);
        }
        cs.next_aux += (C - 1) * A;
        cs.next_input += (C - 1) * I;
    }

    void set_mark() {
        mark.aux0 = cs.next_aux;
        mark.in0 = cs.next_input;
        for (int m = 0; m < 3; m++) mark.row0[m] = b.rp[m].size() - 1;
        mark.ops0 = b.ops.size();
        mark.blocks0 = b.blocks.size();
        mark.pin0 = b.pin.size();
        mark.pos0 = b.poseidon_ops.size();
        mark.sha0 = b.sha_ops.size();
        mark.ncons0 = b.n_constraints;
    }

    // FallbackPoStCircuit::synthesize: sector 0 is synthesised, sectors 1.. are its shifted copies
    void run_post() {
        const Shape &s = b.shape;
        const Layout &L = b.lay;
        set_mark();
        const uint64_t sb = L.post_sector(0);
        const uint64_t comm_c = alloc_data(sb + 1);
        const uint64_t comm_r_last = alloc_data(sb + 2);
        const uint64_t comm_r = alloc_data(sb + 0);
        inputize(comm_r);
        const uint64_t h = poseidon({comm_c, comm_r_last});  // hash2_circuit
        equal(comm_r, h);
        for (unsigned n = 0; n < s.challenges; n++) {  // PoRCircuit (private): leaf, path, root = comm_r_last
            const uint64_t cb = L.post_challenge(0, n);
            const uint64_t leaf = alloc_data(cb + 1);
            por(leaf, cb, cb + 2, L.c_arities, false, comm_r_last);
        }
        replicate(s.sectors, 1 + s.challenges);
        if (cs.next_input != cs.n_in_total) throw std::logic_error("post: input count differs from the shape");
    }

    void run() {
        const Shape &s = b.shape;
        const Layout &L = b.lay;
        const uint64_t rid = alloc_data(0);
        inputize(rid);
        const uint64_t rid_bits = to_bits_le(rid);
        const uint64_t comm_d = alloc_data(1);
        inputize(comm_d);
        const uint64_t comm_r = alloc_data(2);
        inputize(comm_r);
        const uint64_t comm_r_last = alloc_data(3);
        const uint64_t comm_c = alloc_data(4);
        const uint64_t h = poseidon({comm_c, comm_r_last});
        equal(comm_r, h);
        std::vector<unsigned> d_ar(L.depth_d, 2);
        // challenge 0 is synthesised; challenges 1.. have the identical shape and are copies of it with the
        // challenge-local variables, inputs and instance slots shifted (replicate())
        set_mark();
        for (unsigned c = 0; c < 1; c++) {
            const uint64_t cb = L.ch_base(c);
            const uint64_t data_leaf = alloc_data(cb + 1);
            por(data_leaf, cb, cb + L.off_d(), d_ar, true, comm_d);
            std::vector<std::vector<uint64_t>> cols;  // 6 DRG then 8 expander parents
            for (unsigned p = 0; p < 14; p++) {
                const uint64_t pb = cb + L.off_parent(p, s.layers);
                std::vector<uint64_t> col;
                for (unsigned l = 0; l < s.layers; l++) col.push_back(alloc_data(pb + 1 + l));
                const uint64_t ch = poseidon(col);
                por(ch, pb, pb + 1 + s.layers, L.c_arities, false, comm_c);
                cols.push_back(col);
            }
            std::vector<Bit> chal = data_bits(cb, 64, 0);
            pack_input_bits(chal, cb);
            const uint64_t chal_bits = chal[0].z;
            std::vector<uint64_t> labels;
            for (unsigned layer = 1; layer <= s.layers; layer++) {
                std::vector<std::pair<uint64_t, uint64_t>> ps;
                for (unsigned p = 0; p < 6; p++) {
                    uint64_t v = cols[p][layer - 1];
                    ps.push_back({v, to_bits_le(v)});
                }
                if (layer > 1)
                    for (unsigned p = 6; p < 14; p++) {
                        uint64_t v = cols[p][layer - 2];
                        ps.push_back({v, to_bits_le(v)});
                    }
                std::vector<std::pair<uint64_t, uint64_t>> ex;  // params.hpp:199-212
                if (layer > 1) {
                    ex = ps;
                    ex.insert(ex.end(), ps.begin(), ps.end());
                    ex.insert(ex.end(), ps.begin(), ps.begin() + 9);
                } else {
                    for (int r = 0; r < 6; r++) ex.insert(ex.end(), ps.begin(), ps.end());
                    ex.push_back(ps[0]);
                }
                labels.push_back(create_label(rid, rid_bits, ex, layer, cb, chal_bits));
            }
            const uint64_t enc = add(labels.back(), data_leaf);
            por(enc, cb, cb + L.off_r(), L.c_arities, false, comm_r_last);
            const uint64_t colh = poseidon(labels);
            por(colh, cb, cb + L.off_cx(), L.c_arities, false, comm_c);
        }
        replicate(s.challenges, 18);
        if (cs.next_input != cs.n_in_total) throw std::logic_error("stacked: input count differs from the shape");
    }
};

}  // namespace

Built *build(const Shape &s, bool want_r1cs) {
    init_consts();
    if (!s.sectors && s.layers != 2 && s.layers != 11)
        throw std::invalid_argument("stacked: layers must be 2 or 11 (column hash arity)");
    if (!s.challenges) throw std::invalid_argument("stacked: at least one challenge");
    if (s.sectors && (uint64_t)s.sectors * (1 + s.challenges) >= (1ull << 31))
        throw std::invalid_argument("post: too many sectors x challenges");
    Built *b = new Built();
    try {
        b->shape = s;
        b->lay = layout_for(s);
        Synth sy(*b, want_r1cs);
        if (s.sectors)
            sy.run_post();
        else
            sy.run();
        b->n_in = sy.cs.n_in_total;
        b->n_aux = sy.cs.next_aux;
        b->ctab = pool().snapshot();
        // order the program by level (stable), remapping the op references of blocks and the phase-B lists
        const size_t n = b->ops.size();
        std::vector<uint64_t> perm(n), where(n);
        for (size_t i = 0; i < n; i++) perm[i] = i;
        auto kind = [](const WOp &o) -> uint32_t {
            if (o.type != W_POSEIDON) return 0;
            return o.n == 2 ? 1 : o.n == 4 ? 2 : o.n == 8 ? 3 : 4;
        };
        std::stable_sort(perm.begin(), perm.end(), [&](uint64_t x, uint64_t y) {
            const WOp &a = b->ops[x], &c = b->ops[y];
            return a.level != c.level ? a.level < c.level : kind(a) < kind(c);
        });
        std::vector<WOp> sorted(n);
        for (size_t i = 0; i < n; i++) {
            sorted[i] = b->ops[perm[i]];
            where[perm[i]] = i;
        }
        b->ops.swap(sorted);
        for (auto &blk : b->blocks) blk.op = (uint32_t)where[blk.op];
        for (auto &o : b->poseidon_ops) o = where[o];
        for (auto &o : b->sha_ops) o = where[o];
        uint32_t maxl = n ? b->ops.back().level : 0;
        b->level_off.assign(maxl + 2, 0);
        for (auto &op : b->ops) b->level_off[op.level + 1]++;
        for (uint32_t l = 0; l <= maxl; l++) b->level_off[l + 1] += b->level_off[l];
        b->seg_off.assign(5 * (maxl + 1) + 1, 0);
        for (auto &op : b->ops) b->seg_off[5 * op.level + kind(op) + 1]++;
        for (size_t q = 0; q + 1 < b->seg_off.size(); q++) b->seg_off[q + 1] += b->seg_off[q];
        for (uint32_t l = 0; l <= maxl; l++)  // every (level, kind) segment holds exactly its ops
            for (uint32_t k = 0; k < 5; k++)
                for (uint64_t i = b->seg_off[5 * l + k]; i < b->seg_off[5 * l + k + 1]; i++)
                    if (b->ops[i].level != l || kind(b->ops[i]) != k) throw std::logic_error("stacked: op segment");
        if (b->seg_off.back() != n) throw std::logic_error("stacked: op segments do not cover the program");
        for (uint64_t o : b->poseidon_ops)
            if (o >= n || b->ops[o].type != W_POSEIDON) throw std::logic_error("stacked: Poseidon op list");
        for (const ShaBlock &blk : b->blocks)
            if (blk.op >= n || b->ops[blk.op].type != W_SHA) throw std::logic_error("stacked: SHA block owner");
        // every variable is written by exactly one op (the witness program covers z)
        {
            std::vector<uint8_t> hit(b->n_in + b->n_aux, 0);
            hit[0] = 1;
            auto mark = [&](uint64_t z0, uint64_t cnt) {
                if (z0 + cnt > hit.size()) throw std::logic_error("stacked: op writes past z");
                for (uint64_t q = 0; q < cnt; q++) {
                    if (hit[z0 + q]) throw std::logic_error("stacked: variable written twice");
                    hit[z0 + q] = 1;
                }
            };
            std::vector<uint64_t> pos_vars(12, 0);
            for (unsigned a : {2u, 4u, 8u, 11u}) pos_vars[a] = poseidon_constraints(a);
            for (const WOp &op : b->ops) switch (op.type) {
                    case W_BITS: case W_DBITS: mark(op.dst, op.n); break;
                    case W_POSEIDON: mark(op.dst, pos_vars[op.n]); break;
                    case W_SHA: mark(op.b, 1); break;
                    default: mark(op.dst, 1); break;
                }
            for (size_t k = 0; k < b->blocks.size(); k++) {
                const uint64_t end = k + 1 < b->blocks.size() && b->blocks[k + 1].op == b->blocks[k].op
                                         ? b->blocks[k + 1].base
                                         : b->ops[b->blocks[k].op].b;  // the block's variables run to the next block or the pack
                mark(b->blocks[k].base, end - b->blocks[k].base);
            }
            for (size_t q = 0; q < hit.size(); q++)
                if (!hit[q]) throw std::logic_error("stacked: variable " + std::to_string(q) + " has no producer");
        }
    } catch (...) {
        delete b;
        throw;
    }
    return b;
}

void public_inputs(const Built &b, const uint8_t *slots, std::vector<fr_t> &out) {
    auto fr_at = [&](uint64_t slot) {
        fr_t x;
        memcpy(x.v, slots + 32 * slot, 32);
        return x;
    };
    auto u64_at = [&](uint64_t slot) {
        uint64_t v;
        memcpy(&v, slots + 32 * slot, 8);
        fr_t x = fr_t::zero();
        x.v[0] = (uint32_t)v;
        x.v[1] = (uint32_t)(v >> 32);
        return x;
    };
    out.clear();
    const Layout &L = b.lay;
    if (b.shape.sectors) {
        for (uint64_t s = 0; s < b.shape.sectors; s++) {
            out.push_back(fr_at(L.post_sector(s)));  // comm_r
            for (unsigned n = 0; n < b.shape.challenges; n++) out.push_back(u64_at(L.post_challenge(s, n)));
        }
        return;
    }
    out.push_back(fr_at(0));
    out.push_back(fr_at(1));
    out.push_back(fr_at(2));
    for (unsigned c = 0; c < b.shape.challenges; c++) {
        const uint64_t cb = L.ch_base(c);
        out.push_back(u64_at(cb));  // tree D path (packed index bits)
        for (unsigned p = 0; p < 14; p++) out.push_back(u64_at(cb + L.off_parent(p, b.shape.layers)));
        out.push_back(u64_at(cb));  // the challenge (UInt64)
        out.push_back(u64_at(cb));  // tree R-last path
        out.push_back(u64_at(cb));  // tree C path
    }
}

}  // namespace stacked
}  // namespace mi
