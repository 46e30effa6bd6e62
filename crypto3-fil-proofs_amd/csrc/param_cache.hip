// param_cache.hip -- the parameter-cache layer around the params loader (host code only): cache identifiers,
// file names under FIL_PROOFS_PARAMETER_CACHE and get_groth_params' read-or-generate policy.
//
// Restates libs/storage/include/nil/filecoin/storage/proofs/core/parameter_cache.hpp:
//   VERSION 28, PARAMETER_CACHE_ENV_VAR "FIL_PROOFS_PARAMETER_CACHE", PARAMETER_CACHE_DIR
//   "/var/tmp/filecoin-proof-parameters/", extensions params / meta / vk                          (:50-56)
//   parameter_cache_{params,metadata,verifying_key}_path: <dir>/v28-<id>.<ext>                      (:78-94)
//   ensure_ancestor_dirs_exist: the parent directory must exist, else invalid_argument             (:96-103)
//   cacheable_parameters::cache_identifier: <cache_prefix>-<hex sha256(pub_params.identifier())>  (:166-171)
//   get_param_metadata: read <id>.meta, else write {"sector_size": n}                               (:173-183)
//   get_groth_params: read_cached_params(<id>.params), else generate and write_cached_params       (:185-200)
//   get_verifying_key: read <id>.vk, else the generated key's vk, written                         (:202-219)
// The reference reads the environment variable with no fallback (:64-66, undefined when unset); here an unset
// variable means the reference's PARAMETER_CACHE_DIR constant, as rust-fil-proofs does.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sys/file.h>
#include <sys/random.h>
#include <sys/stat.h>
#include <unistd.h>

#include <stdexcept>
#include <string>

#include "../../include/mi355x_groth16.h"

namespace mi {
void set_last_error(const std::string &msg);  // capi.hip
}

namespace {

// FIPS 180-4 SHA-256 (host; the identifier strings are short)
struct Sha256 {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
    void block(const uint8_t *p) {
        static const uint32_t K[64] = {
            0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
            0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
            0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
            0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
            0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
            0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
            0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
            0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
        uint32_t w[64];
        for (int i = 0; i < 16; i++)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; i++) {
            const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
        for (int i = 0; i < 64; i++) {
            const uint32_t t1 = k + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            k = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
        }
        h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e, h[5] += f, h[6] += g, h[7] += k;
    }
    std::string hex_digest(const std::string &msg) {
        std::string m = msg;
        const uint64_t bits = 8ull * msg.size();
        m.push_back((char)0x80);
        while (m.size() % 64 != 56) m.push_back(0);
        for (int i = 7; i >= 0; i--) m.push_back((char)(bits >> (8 * i)));
        for (size_t o = 0; o < m.size(); o += 64) block((const uint8_t *)m.data() + o);
        static const char *hx = "0123456789abcdef";
        std::string out;
        for (uint32_t x : h)
            for (int i = 7; i >= 0; i--) out.push_back(hx[(x >> (4 * i)) & 15]);
        return out;
    }
};

int fail(int code, const std::string &msg) {
    mi::set_last_error(msg);  // the text mi_last_error() returns, like every other entry
    return code;
}

int put(const std::string &s, char *out, size_t cap) {
    if (!out || cap < s.size() + 1) return fail(MI_ERR_SIZE, "output buffer too small (need " + std::to_string(s.size() + 1) + ")");
    memcpy(out, s.c_str(), s.size() + 1);
    return MI_OK;
}

std::string cache_dir() {
    const char *e = getenv("FIL_PROOFS_PARAMETER_CACHE");
    return e && *e ? std::string(e) : std::string("/var/tmp/filecoin-proof-parameters/");
}

const char *ext_of(int kind) { return kind == 0 ? "params" : kind == 1 ? "meta" : kind == 2 ? "vk" : nullptr; }

std::string path_of(const std::string &id, int kind) {
    return cache_dir() + "/v" + std::to_string(MI_PARAMS_VERSION) + "-" + id + "." + ext_of(kind);
}

bool parent_exists(const std::string &p) {
    const size_t k = p.find_last_of('/');
    const std::string dir = k == std::string::npos ? "." : (k == 0 ? "/" : p.substr(0, k));
    struct stat st;
    return stat(dir.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

bool file_exists(const std::string &p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

// {"sector_size":N} (serde_json of cache_entry_metadata); returns false when the file is missing or malformed
bool read_meta(const std::string &p, uint64_t *sector_size) {
    FILE *f = fopen(p.c_str(), "rb");
    if (!f) return false;
    char buf[256] = {0};
    const size_t n = fread(buf, 1, sizeof buf - 1, f);
    fclose(f);
    buf[n] = 0;
    const char *k = strstr(buf, "\"sector_size\"");
    if (!k) return false;
    k = strchr(k, ':');
    if (!k) return false;
    char *end = nullptr;
    errno = 0;
    const unsigned long long v = strtoull(k + 1, &end, 10);
    if (errno || end == k + 1) return false;
    if (sector_size) *sector_size = v;
    return true;
}

bool write_meta(const std::string &p, uint64_t sector_size) {
    FILE *f = fopen(p.c_str(), "wb");
    if (!f) return false;
    const int ok = fprintf(f, "{\"sector_size\":%llu}", (unsigned long long)sector_size) > 0;
    return fclose(f) == 0 && ok;
}

// bellman generate_random_parameters draws tau, alpha, beta, gamma, delta from an OS RNG: 255-bit candidates
// below r (rejection), none zero
void random_toxic(uint8_t out[160]) {
    static const uint8_t R_BE[32] = {0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8,
                                     0x08, 0x09, 0xa1, 0xd8, 0x05, 0x53, 0xbd, 0xa4, 0x02, 0xff, 0xfe,
                                     0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01};
    for (int k = 0; k < 5; k++) {
        uint8_t *d = out + 32 * k;
        for (;;) {
            for (size_t o = 0; o < 32;) {
                const ssize_t got = getrandom(d + o, 32 - o, 0);
                if (got < 0) {
                    if (errno == EINTR) continue;
                    throw std::runtime_error("getrandom failed");
                }
                o += (size_t)got;
            }
            d[31] &= 0x7f;
            int cmp = 0;  // compare the little-endian candidate with r (big-endian constant)
            for (int i = 0; i < 32 && !cmp; i++) cmp = (d[31 - i] > R_BE[i]) - (d[31 - i] < R_BE[i]);
            bool zero = true;
            for (int i = 0; i < 32; i++) zero &= d[i] == 0;
            if (cmp < 0 && !zero) break;
        }
    }
}

}  // namespace

extern "C" {

int mi_param_cache_id(const char *cache_prefix, const char *identifier, char *out, size_t cap) {
    if (!cache_prefix || !identifier) return fail(MI_ERR_ARG, "null argument");
    return put(std::string(cache_prefix) + "-" + Sha256().hex_digest(identifier), out, cap);
}

int mi_param_cache_path(const char *id, int kind, char *out, size_t cap) {
    if (!id) return fail(MI_ERR_ARG, "null id");
    if (!ext_of(kind)) return fail(MI_ERR_ARG, "kind must be 0 (params), 1 (meta) or 2 (vk)");
    return put(path_of(id, kind), out, cap);
}

int mi_param_cache_metadata(const char *id, uint64_t sector_size, uint64_t *sector_size_out) {
    if (!id) return fail(MI_ERR_ARG, "null id");
    const std::string p = path_of(id, 1);
    if (!parent_exists(p)) return fail(MI_ERR_ARG, p + " has no parent directory");
    uint64_t got = 0;
    if (!read_meta(p, &got)) {
        if (!write_meta(p, sector_size)) return fail(MI_ERR_INTERNAL, "cannot write " + p);
        got = sector_size;
    }
    if (sector_size_out) *sector_size_out = got;
    return MI_OK;
}

int mi_get_groth_params(mi_ctx *ctx, const mi_circuit *circuit, const char *id, const uint8_t *toxic_or_null,
                        int checked, mi_srs **out, int *generated) {
    if (!ctx || !circuit || !id || !out) return fail(MI_ERR_ARG, "null argument");
    *out = nullptr;
    if (generated) *generated = 0;
    const std::string pp = path_of(id, 0), vp = path_of(id, 2);
    if (!parent_exists(pp)) return fail(MI_ERR_ARG, pp + " has no parent directory");
    // one reader-or-generator per file at a time: an exclusive lock on <params>.lock, so two processes that both
    // find the file missing (or malformed) do not pair one's .params with the other's .vk
    const std::string lp = pp + ".lock";
    const int lfd = open(lp.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
    if (lfd < 0) return fail(MI_ERR_INTERNAL, "cannot open " + lp);
    struct Unlock {
        int fd;
        ~Unlock() {
            flock(fd, LOCK_UN);
            close(fd);
        }
    } unlock{lfd};
    while (flock(lfd, LOCK_EX) != 0)
        if (errno != EINTR) return fail(MI_ERR_INTERNAL, "cannot lock " + lp);
    if (file_exists(pp)) {
        const int rc = mi_params_load(ctx, circuit, pp.c_str(), checked, out);
        if (rc == MI_OK) return MI_OK;
        if (rc != MI_ERR_ARG) return fail(rc, std::string("reading ") + pp + ": " + mi_last_error());
        // (MI_ERR_ARG: truncated, trailing bytes or an invalid point)
        // a malformed cache file is regenerated, as the reference's catch-all does (parameter_cache.hpp:195-199)
    }
    uint8_t tox[160];
    try {
        if (toxic_or_null) memcpy(tox, toxic_or_null, 160);
        else random_toxic(tox);
    } catch (const std::exception &e) {
        return fail(MI_ERR_INTERNAL, e.what());
    }
    mi_srs *srs = nullptr;
    int rc = mi_srs_generate(ctx, circuit, tox, &srs);
    memset(tox, 0, sizeof tox);
    if (rc != MI_OK) return fail(rc, std::string("generating parameters: ") + mi_last_error());
    // both files written under temporary names and renamed, so a reader never maps a half-written file; the vk is
    // rewritten whenever the params are (a .vk left by earlier parameters would no longer verify their proofs)
    const std::string tag = ".tmp" + std::to_string((unsigned long long)getpid());
    const std::string tmp = pp + tag, vtmp = vp + tag;
    rc = mi_params_write(ctx, srs, tmp.c_str());
    if (rc == MI_OK) rc = mi_vk_write(srs, vtmp.c_str());
    if (rc == MI_OK && rename(tmp.c_str(), pp.c_str()) != 0) rc = MI_ERR_INTERNAL;
    if (rc == MI_OK && rename(vtmp.c_str(), vp.c_str()) != 0) rc = MI_ERR_INTERNAL;
    if (rc != MI_OK) {
        remove(tmp.c_str());
        remove(vtmp.c_str());
        mi_srs_free(srs);
        return fail(rc, "cannot write " + pp + " / " + vp);
    }
    *out = srs;
    if (generated) *generated = 1;
    return MI_OK;
}

}  // extern "C"
