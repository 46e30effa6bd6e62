// capi.hip -- extern "C" boundary (include/mi355x_groth16.h).  Host code only: translates the
// wire formats, owns object lifetimes, serialises each context and turns C++ exceptions into
// status codes + mi_last_error().  No CPU fallback exists: every compute entry point runs the
// HIP kernels of this library or fails.
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/random.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <thread>

#include "../../include/mi355x_groth16.h"

#include <vector>
#ifdef MI_FQ_CHECK
namespace mi {
// the Fq invariant counters of every translation unit (field.h FqCheckRegistrar; a function-local list, so the
// registrations of other units' static initialisers never run before it exists)
struct FqCheckUnit {
    const void *symbol;
    const char *unit;
};
static std::vector<FqCheckUnit> &fq_check_syms() {
    static std::vector<FqCheckUnit> v;
    return v;
}
void fq_check_register(const void *symbol, const char *unit) { fq_check_syms().push_back({symbol, unit}); }
static const std::vector<FqCheckUnit> &fq_check_symbols() { return fq_check_syms(); }
}  // namespace mi
#endif
#include "poseidon_math.h"
#include "prover.h"
#include "sdr.h"
#include "stacked.h"

// Witness uploads (host z -> HBM) run on their own stream into one of two device slots, so the copy
// of partition k + 1 overlaps the proof of partition k (mi_groth16_prove_batch).  Pinned witnesses
// (mi_host_alloc, or memory the caller registered) go up in one DMA; pageable ones through two pinned
// staging buffers.  Each upload is followed on the same stream by the canonical-Fr check of its entries.
struct WitnessUploader {
    static constexpr uint64_t STAGE = 64ull << 20;
    hipStream_t copy = nullptr;
    int *flags_host = nullptr;  // pinned: [slot] = entries >= r
    int *flags_dev = nullptr;
    hipEvent_t done[2] = {nullptr, nullptr}, t0[2] = {nullptr, nullptr};
    uint8_t *stage[2] = {nullptr, nullptr};
    hipEvent_t stage_free[2] = {nullptr, nullptr};
    void release() {
        if (copy) hipStreamSynchronize(copy);
        for (int k = 0; k < 2; k++) {
            if (done[k]) hipEventDestroy(done[k]);
            if (t0[k]) hipEventDestroy(t0[k]);
            if (stage_free[k]) hipEventDestroy(stage_free[k]);
            if (stage[k]) hipHostFree(stage[k]);
            done[k] = t0[k] = stage_free[k] = nullptr;
            stage[k] = nullptr;
        }
        if (flags_host) hipHostFree(flags_host);
        if (flags_dev) hipFree(flags_dev);
        if (copy) hipStreamDestroy(copy);
        flags_host = nullptr;
        flags_dev = nullptr;
        copy = nullptr;
    }
};

struct mi_ctx {
    mi::Ctx c;
    hipStream_t normal = nullptr, high = nullptr;
    WitnessUploader up;
    // Stream-ordering contract of the entries that touch caller device memory (include/mi355x_groth16.h
    // "Device pointers"): their first device access waits, on the device, for everything queued on `caller`
    // before the call.  nullptr = the legacy default stream, which also waits for every blocking stream.
    hipStream_t caller = nullptr;
    hipEvent_t fence = nullptr;
};
struct mi_circuit {
    mi::Circuit *p;
    int device;
};
struct mi_srs {
    mi::Srs *p;
    int device;
};
struct mi_stacked {
    mi::stacked::Built *b;
    std::vector<mi::fr_t> full[3];  // 32-byte coefficients, materialised on the first mi_stacked_r1cs
};
struct mi_srs_stream {
    mi::SrsStream *p;
    mi_ctx *ctx;
};
struct mi_points {
    void *dev;
    uint64_t n;
    int is_g2;
    int owns;
    const void *hi = nullptr;  // 2^128 multiples (split-mode MSM table) of caller-uploaded points (none today)
    int subgroup = 0;          // every point known to be in the prime-order subgroup (GLV split allowed)
    // a proving-key query (mi_points_from_srs): its split table is looked up at use, since a proof that runs
    // out of memory may release the key's tables (prover.hip groth16_sums)
    const mi::Srs *srs = nullptr;
    int which = -1;
    // fixed-base window table (mi_points_precompute) of caller-owned points; a key query's is the key's (Srs::wt)
    void *wt_own = nullptr;
    mi::WinTable wt_user;
    // MSMs over these points hold it shared, mi_points_precompute exclusive while it swaps wt_own
    mutable std::shared_mutex wt_mu;
    mi::WinTable wtab() const {
        if (wt_own || !srs) return wt_user;  // a table built on this point set first
        return srs->wt_of(which);
    }
    const void *table() const {
        if (!srs) return hi;
        return which == 0 ? (const void *)srs->h_hi : which == 1 ? (const void *)srs->l_hi
                                                    : which == 2 ? (const void *)srs->a_hi : nullptr;
    }
};

namespace {

thread_local std::string g_err;

template <class Fn>
int guard(Fn &&f) {
    try {
        f();
        return MI_OK;
    } catch (const mi::hip_error &e) {
        g_err = e.what();
        return MI_ERR_HIP;
    } catch (const std::invalid_argument &e) {
        g_err = e.what();
        return MI_ERR_ARG;
    } catch (const std::domain_error &e) {
        g_err = e.what();
        return MI_ERR_INVALID_POINT;
    } catch (const std::length_error &e) {
        g_err = e.what();
        return MI_ERR_SIZE;
    } catch (const std::exception &e) {
        g_err = e.what();
        return MI_ERR_INTERNAL;
    } catch (...) {
        g_err = "unknown error";
        return MI_ERR_INTERNAL;
    }
}

void need(bool cond, const std::string &msg) {
    if (!cond) throw std::invalid_argument(msg);
}
void need(bool cond, const char *msg) {
    if (!cond) throw std::invalid_argument(msg);
}
void check_dev_canonical(mi::Ctx &c, const mi::fr_t *d, uint64_t n, const char *what);  // below

// ---- bellman / filecoin Groth16 parameter files (v28-*.params, *.vk) ----------------------
// Parameters::write: vk (MI_VK_BYTES) | u32 BE n_ic | ic (96 B each) | then for h, l, a, b_g1
// (96 B points) and b_g2 (192 B points): u32 BE count | points.  The reference mmaps the file and
// keeps offsets (core/crypto/mapped_scheme_params.hpp:43-84, read_cached_params at
// core/parameter_cache.hpp:125-129).
struct ParamsLayout {
    uint64_t n[6] = {0, 0, 0, 0, 0, 0};    // ic, h, l, a, b_g1, b_g2
    uint64_t off[6] = {0, 0, 0, 0, 0, 0};  // byte offset of the first point of each vector
};

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

ParamsLayout parse_params(const uint8_t *p, uint64_t len) {
    static const uint64_t esz[6] = {96, 96, 96, 96, 96, 192};
    static const char *names[6] = {"ic", "h", "l", "a", "b_g1", "b_g2"};
    ParamsLayout L;
    uint64_t o = MI_VK_BYTES;
    if (len < o) throw std::invalid_argument("params file truncated in the verifying key");
    for (int i = 0; i < 6; i++) {
        if (len - o < 4) throw std::invalid_argument(std::string("params file truncated before the ") + names[i] +
                                                     " length");
        L.n[i] = be32(p + o);
        o += 4;
        L.off[i] = o;
        if ((len - o) / esz[i] < L.n[i])
            throw std::invalid_argument(std::string("params file truncated in the ") + names[i] + " points");
        o += esz[i] * L.n[i];
    }
    if (o != len) throw std::invalid_argument("params file has trailing bytes after b_g2");
    return L;
}

struct MappedFile {
    int fd = -1;
    void *p = nullptr;
    uint64_t len = 0;
    explicit MappedFile(const char *path) {
        fd = open(path, O_RDONLY);
        if (fd < 0) throw std::invalid_argument(std::string("cannot open ") + path);
        struct stat st;
        if (fstat(fd, &st) != 0) throw std::runtime_error(std::string("cannot stat ") + path);
        len = (uint64_t)st.st_size;
        if (len) {
            p = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
            if (p == MAP_FAILED) {
                p = nullptr;
                throw std::runtime_error(std::string("cannot mmap ") + path);
            }
            madvise(p, len, MADV_SEQUENTIAL);
        }
    }
    ~MappedFile() {
        if (p) munmap(p, len);
        if (fd >= 0) close(fd);
    }
    const uint8_t *data() const { return (const uint8_t *)p; }
};

void write_all(FILE *f, const void *p, size_t n) {
    if (n && fwrite(p, 1, n, f) != n) throw std::runtime_error("short write");
}
void write_be32(FILE *f, uint64_t v) {
    if (v > 0xffffffffull) throw std::length_error("vector too long for a u32 length");
    uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    write_all(f, b, 4);
}

// Selects a context's device for the length of one C-ABI call and gives the calling thread its previous
// device back afterwards, so a call never moves the caller's (e.g. torch's) current device.
struct DeviceScope {
    int prev = -1;
    // strict: throw when the device cannot be selected (entries under guard); the free functions pass false
    explicit DeviceScope(int device, bool strict = true) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        hipError_t e = hipSetDevice(device);
        if (strict && e != hipSuccess) {
            if (prev >= 0) (void)hipSetDevice(prev);
            prev = -1;
            MI_HIP(e);
        }
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Orders the context's current stream after the caller's prior work (event recorded on the caller stream, waited
// for on the device: no host synchronisation).  The aux lanes and the copy stream fork from the context stream,
// so ordering it orders every library stream of the call.
void caller_fence(mi_ctx *ctx) {
    if (!ctx->fence) MI_HIP(hipEventCreateWithFlags(&ctx->fence, hipEventDisableTiming));
    MI_HIP(hipEventRecord(ctx->fence, ctx->caller));
    MI_HIP(hipStreamWaitEvent(ctx->c.stream, ctx->fence, 0));
}

enum { NO_FENCE = 0, FENCE = 1 };  // FENCE: the entry reads or writes caller device memory

struct CtxLock {
    mi_ctx *ctx;
    std::lock_guard<std::recursive_mutex> lk;
    DeviceScope dev;
    CtxLock(mi_ctx *c, int priority = 0, int fence = NO_FENCE) : ctx(c), lk(c->c.mu), dev(c->c.device) {
        if (priority && !c->high) {  // created at first use: every stream a process creates takes a hardware queue
            int lo = 0, hi = 0;     // (GPU_MAX_HW_QUEUES, 4 by default) or shares one with another stream
            MI_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
            MI_HIP(hipStreamCreateWithPriority(&c->high, hipStreamNonBlocking, hi));
        }
        c->c.stream = priority ? c->high : c->normal;
        if (fence == FENCE) caller_fence(c);
    }
};

void proof_bytes(const mi::ProofPoints &pp, uint8_t *proof, uint8_t *raw) {
    mi::g1_compress(pp.A, proof);
    mi::g2_compress(pp.B, proof + 48);
    mi::g1_compress(pp.C, proof + 144);
    if (raw) {
        mi::g1_encode(pp.A, raw);
        mi::g2_encode(pp.B, raw + 96);
        mi::g1_encode(pp.C, raw + 288);
    }
}

mi::fr_t fr_checked(const uint8_t *b) {
    mi::fr_t x = mi::fr_from_le(b);
    need(!mi::geq_raw(x, mi::fr_t::modulus_raw()), "scalar is not canonical (>= r)");
    return x;
}

// bellman create_random_proof draws r, s = E::Fr::random(&mut OsRng): uniform canonical Fr.  Here: 255-bit
// candidates from getrandom() with rejection (P(reject) = 1 - r / 2^255 ~ 0.09); out = count x (r | s).
void random_blinding(uint64_t count, uint8_t *out) {
    for (uint64_t k = 0; k < 2 * count; k++) {
        uint8_t *dst = out + 32 * k;
        for (;;) {
            for (size_t o = 0; o < 32;) {
                ssize_t got = getrandom(dst + o, 32 - o, 0);
                if (got < 0) {
                    if (errno == EINTR) continue;
                    throw std::runtime_error("getrandom failed");
                }
                o += (size_t)got;
            }
            dst[31] &= 0x7f;
            if (!mi::geq_raw(mi::fr_from_le(dst), mi::fr_t::modulus_raw())) break;
        }
    }
}

// upload z (host) to a device scratch buffer and reduce it mod r (building blocks: MSM scalars, NTT data)
mi::fr_t *upload_fr(mi::Ctx &c, int slot, const uint8_t *bytes, uint64_t n) {
    mi::fr_t *d = c.scratch[slot].as<mi::fr_t>(n ? n : 1);
    if (n) {
        MI_HIP(hipMemcpyAsync(d, bytes, 32 * n, hipMemcpyHostToDevice, c.stream));
        mi::fr_canonicalize(c, d, n);
    }
    return d;
}

WitnessUploader &uploader(mi_ctx *ctx) {
    WitnessUploader &u = ctx->up;
    if (!u.copy) {
        try {
            MI_HIP(hipStreamCreateWithFlags(&u.copy, hipStreamNonBlocking));
            MI_HIP(hipHostMalloc((void **)&u.flags_host, 2 * sizeof(int), hipHostMallocDefault));
            MI_HIP(hipMalloc((void **)&u.flags_dev, 2 * sizeof(int)));
            for (int k = 0; k < 2; k++) {
                MI_HIP(hipEventCreate(&u.done[k]));
                MI_HIP(hipEventCreate(&u.t0[k]));
                MI_HIP(hipEventCreateWithFlags(&u.stage_free[k], hipEventDisableTiming));
            }
        } catch (...) {
            u.release();
            throw;
        }
    }
    return u;
}

bool is_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: clear the error the query recorded
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Witness slot k (0 / 1) lives in ctx scratch 21 + k.  Queues the H2D copy of z and the canonical check
// on the copy stream and records done[k]; pageable inputs are staged by the calling thread.
mi::fr_t *witness_upload(mi_ctx *ctx, int k, const uint8_t *z, uint64_t n) {
    WitnessUploader &u = uploader(ctx);
    mi::Ctx &c = ctx->c;
    mi::fr_t *d = c.scratch[21 + k].as<mi::fr_t>(n ? n : 1);
    const uint64_t bytes = 32 * n;
    MI_HIP(hipEventRecord(u.t0[k], u.copy));
    MI_HIP(hipMemsetAsync(u.flags_dev + k, 0, sizeof(int), u.copy));
    if (bytes && is_pinned(z)) {
        MI_HIP(hipMemcpyAsync(d, z, bytes, hipMemcpyHostToDevice, u.copy));
    } else if (bytes) {
        for (int b = 0; b < 2; b++)
            if (!u.stage[b]) MI_HIP(hipHostMalloc((void **)&u.stage[b], WitnessUploader::STAGE, hipHostMallocDefault));
        uint64_t i = 0;
        for (uint64_t o = 0; o < bytes; o += WitnessUploader::STAGE, i++) {
            const uint64_t m = bytes - o < WitnessUploader::STAGE ? bytes - o : WitnessUploader::STAGE;
            const int b = (int)(i & 1);
            if (i >= 2) MI_HIP(hipEventSynchronize(u.stage_free[b]));  // its previous DMA has drained
            memcpy(u.stage[b], z + o, m);
            MI_HIP(hipMemcpyAsync((uint8_t *)d + o, u.stage[b], m, hipMemcpyHostToDevice, u.copy));
            MI_HIP(hipEventRecord(u.stage_free[b], u.copy));
        }
    }
    mi::fr_count_noncanonical(c, d, n, u.flags_dev + k, u.copy);
    MI_HIP(hipMemcpyAsync(u.flags_host + k, u.flags_dev + k, sizeof(int), hipMemcpyDeviceToHost, u.copy));
    MI_HIP(hipEventRecord(u.done[k], u.copy));
    return d;
}

// Waits for slot k's upload (the proof before it has normally hidden it), books its time, refuses a
// witness holding non-canonical entries (MI_ERR_ARG: an Fr32 "MUST represent a valid Fr",
// core/fr32.hpp:36-40) and orders the ctx stream after the copy.
void witness_ready(mi_ctx *ctx, int k, uint64_t n) {
    WitnessUploader &u = ctx->up;
    MI_HIP(hipEventSynchronize(u.done[k]));
    float ms = 0;
    if (hipEventElapsedTime(&ms, u.t0[k], u.done[k]) == hipSuccess) {
        ctx->c.stats.h2d.ms += ms;
        ctx->c.stats.h2d.launches += 1;
        ctx->c.stats.h2d.units += 32 * n;
    }
    if (u.flags_host[k])
        throw std::invalid_argument("witness entry is not a canonical Fr element (>= r): " +
                                    std::to_string(u.flags_host[k]) + " of " + std::to_string(n));
    MI_HIP(hipStreamWaitEvent(ctx->c.stream, u.done[k], 0));
}

// Device-resident witness: the same check on the ctx stream; read after the proof's final sync.
struct DevWitnessCheck {
    mi_ctx *ctx;
    DevWitnessCheck(mi_ctx *x, const mi::fr_t *z, uint64_t n) : ctx(x) {
        WitnessUploader &u = uploader(x);
        MI_HIP(hipMemsetAsync(u.flags_dev, 0, sizeof(int), x->c.stream));
        mi::fr_count_noncanonical(x->c, z, n, u.flags_dev, x->c.stream);
        MI_HIP(hipMemcpyAsync(u.flags_host, u.flags_dev, sizeof(int), hipMemcpyDeviceToHost, x->c.stream));
    }
    void verdict(uint64_t n) {
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
        if (ctx->up.flags_host[0])
            throw std::invalid_argument("witness entry is not a canonical Fr element (>= r): " +
                                        std::to_string(ctx->up.flags_host[0]) + " of " + std::to_string(n));
    }
};

}  // namespace

namespace mi {
void set_last_error(const std::string &msg) { g_err = msg; }
}  // namespace mi

extern "C" {

const char *mi_last_error(void) { return g_err.c_str(); }

int mi_device_count(int *out) {
    return guard([&] {
        need(out != nullptr, "null out");
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        *out = e == hipSuccess ? n : 0;
    });
}

int mi_ctx_create(int device, mi_ctx **out) {
    int rc = guard([&] {
        need(out != nullptr, "null out");
        *out = nullptr;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw std::runtime_error("no HIP device available");
        need(device >= 0 && device < n, "device index out of range");
        DeviceScope dev(device);
        mi_ctx *c = new mi_ctx();
        try {
            c->c.device = device;
            MI_HIP(hipStreamCreateWithFlags(&c->normal, hipStreamNonBlocking));
            c->c.stream = c->normal;  // the high-priority stream is created at its first use (CtxLock)
            mi::ntt_init_tables(c->c);
        } catch (...) {
            if (c->normal) hipStreamDestroy(c->normal);
            if (c->high) hipStreamDestroy(c->high);
            delete c;
            throw;
        }
        *out = c;
    });
    if (rc == MI_ERR_INTERNAL && g_err.find("no HIP device") != std::string::npos) return MI_ERR_NO_DEVICE;
    return rc;
}

void mi_ctx_destroy(mi_ctx *ctx) {
    if (!ctx) return;
    DeviceScope dev(ctx->c.device, false);
    hipDeviceSynchronize();
    ctx->up.release();
    for (mi::Ctx *x = &ctx->c; x; x = x->aux) mi::stacked::forget_ctx(x->uid);
    mi::ntt_free_tables(ctx->c);
    mi::ctx_aux_free(ctx->c);
    mi::poseidon_free(ctx->c);
    for (auto &b : ctx->c.scratch) b.release();
    if (ctx->normal) hipStreamDestroy(ctx->normal);
    if (ctx->high) hipStreamDestroy(ctx->high);
    if (ctx->c.plan_stream) hipStreamDestroy(ctx->c.plan_stream);
    for (auto e : ctx->c.plan_ev)
        if (e) hipEventDestroy(e);
    if (ctx->fence) hipEventDestroy(ctx->fence);
    delete ctx;
}

int mi_ctx_stream(mi_ctx *ctx, void **stream_out) {
    return guard([&] {
        need(ctx && stream_out, "null argument");
        *stream_out = (void *)ctx->normal;
    });
}

int mi_ctx_set_caller_stream(mi_ctx *ctx, void *stream) {
    return guard([&] {
        need(ctx != nullptr, "null ctx");
        CtxLock l(ctx);
        ctx->caller = (hipStream_t)stream;
    });
}

int mi_ctx_synchronize(mi_ctx *ctx) {
    return guard([&] {
        need(ctx != nullptr, "null ctx");
        CtxLock l(ctx);
        MI_HIP(hipStreamSynchronize(ctx->normal));
        if (ctx->high) MI_HIP(hipStreamSynchronize(ctx->high));
        ctx->c.timer.resolve();
    });
}

int mi_host_alloc(uint64_t bytes, void **out) {
    return guard([&] {
        need(out != nullptr, "null out");
        *out = nullptr;
        need(bytes > 0, "zero-byte host allocation");
        MI_HIP(hipHostMalloc(out, bytes, hipHostMallocDefault));
    });
}

void mi_host_free(void *p) {
    if (p) hipHostFree(p);
}

// ------------------------------------------------------------------------------------------
int mi_circuit_load(mi_ctx *ctx, const mi_r1cs *cs, mi_circuit **out) {
    return guard([&] {
        need(ctx && cs && out, "null argument");
        CtxLock l(ctx);
        mi::R1csHost h;
        h.n = cs->num_constraints;
        h.n_in = cs->num_inputs;
        h.n_aux = cs->num_aux;
        for (int m = 0; m < 3; m++) {
            need(cs->row_ptr[m] != nullptr, "null row_ptr");
            h.row_ptr[m] = cs->row_ptr[m];
            h.col[m] = cs->col[m];
            h.coeff[m] = cs->coeff[m];
            need(cs->row_ptr[m][cs->num_constraints] == 0 || (cs->col[m] && cs->coeff[m]), "null col/coeff");
        }
        mi::Circuit *p = mi::circuit_load(ctx->c, h);
        *out = new mi_circuit{p, ctx->c.device};
    });
}

int mi_circuit_info(const mi_circuit *c, uint64_t out[9]) {
    return guard([&] {
        need(c && out, "null argument");
        const mi::Circuit &p = *c->p;
        uint64_t v[9] = {p.n, p.n_in, p.n_aux, p.d, p.n_a, p.n_b, p.nnz[0], p.nnz[1], p.nnz[2]};
        memcpy(out, v, sizeof v);
    });
}

void mi_circuit_free(mi_circuit *c) {
    if (!c) return;
    DeviceScope dev(c->device, false);
    delete c->p;
    delete c;
}

int mi_srs_load(mi_ctx *ctx, const mi_circuit *circ, const mi_srs_host *h, int checked, mi_srs **out) {
    return guard([&] {
        need(ctx && h && out, "null argument");
        need(h->vk && (h->n_ic == 0 || h->ic) && h->h, "null query pointer");
        CtxLock l(ctx);
        mi::SrsHost sh;
        sh.vk = h->vk;
        sh.ic = h->ic;
        sh.n_ic = h->n_ic;
        sh.h = h->h;
        sh.n_h = h->n_h;
        sh.l = h->l;
        sh.n_l = h->n_l;
        sh.a = h->a;
        sh.n_a = h->n_a;
        sh.b_g1 = h->b_g1;
        sh.n_b_g1 = h->n_b_g1;
        sh.b_g2 = h->b_g2;
        sh.n_b_g2 = h->n_b_g2;
        mi::Srs *p = mi::srs_load(ctx->c, circ ? circ->p : nullptr, sh, checked != 0);
        *out = new mi_srs{p, ctx->c.device};
    });
}

int mi_srs_stream_begin(mi_ctx *ctx, const mi_circuit *circ, const uint8_t *vk, const uint8_t *ic, uint64_t n_ic,
                        const uint64_t counts[5], int checked, mi_srs_stream **out) {
    return guard([&] {
        need(ctx && vk && (n_ic == 0 || ic) && counts && out, "null argument");
        CtxLock l(ctx);
        mi::SrsHost sh{};
        sh.vk = vk;
        sh.ic = ic;
        sh.n_ic = n_ic;
        sh.n_h = counts[0];
        sh.n_l = counts[1];
        sh.n_a = counts[2];
        sh.n_b_g1 = counts[3];
        sh.n_b_g2 = counts[4];
        mi::SrsStream *st = mi::srs_stream_begin(ctx->c, circ ? circ->p : nullptr, sh, checked != 0);
        *out = new mi_srs_stream{st, ctx};
    });
}
int mi_srs_stream_part(mi_srs_stream *st, int which, uint64_t first, const void *bytes, uint64_t n_points,
                       int on_device) {
    return guard([&] {
        need(st && st->p && (bytes || !n_points), "null argument");
        CtxLock l(st->ctx, 0, on_device ? FENCE : NO_FENCE);
        mi::srs_stream_part(st->ctx->c, *st->p, which, first, (const uint8_t *)bytes, n_points, on_device != 0);
    });
}
int mi_srs_stream_end(mi_srs_stream *st, mi_srs **out) {
    if (!st) return guard([&] { need(false, "null argument"); });
    mi_ctx *ctx = st->ctx;
    mi::SrsStream *p = st->p;
    delete st;  // consumed whatever happens
    return guard([&] {
        need(out && p, "null argument");
        CtxLock l(ctx);
        mi::Srs *S = mi::srs_stream_end(ctx->c, p);
        *out = new mi_srs{S, ctx->c.device};
    });
}
void mi_srs_stream_abort(mi_srs_stream *st) {
    if (!st) return;
    try {
        CtxLock l(st->ctx);  // the context's device and lock, like every other stream entry
        mi::srs_stream_abort(st->p);
    } catch (...) {
    }
    delete st;
}

int mi_srs_generate(mi_ctx *ctx, const mi_circuit *circ, const uint8_t toxic[160], mi_srs **out) {
    return guard([&] {
        need(ctx && circ && toxic && out, "null argument");
        CtxLock l(ctx);
        mi::fr_t t[5];
        for (int i = 0; i < 5; i++) t[i] = fr_checked(toxic + 32 * i);
        need(!t[3].is_zero() && !t[4].is_zero(), "gamma and delta must be non-zero");
        mi::Srs *p = mi::srs_generate(ctx->c, *circ->p, t);
        *out = new mi_srs{p, ctx->c.device};
    });
}

int mi_srs_export_vk(const mi_srs *srs, uint8_t *vk, uint8_t *ic) {
    return guard([&] {
        need(srs != nullptr, "null srs");
        const mi::Srs &s = *srs->p;
        if (vk) {
            mi::g1_encode(s.alpha_g1, vk);
            mi::g1_encode(s.beta_g1, vk + 96);
            mi::g2_encode(s.beta_g2, vk + 192);
            mi::g2_encode(s.gamma_g2, vk + 384);
            mi::g1_encode(s.delta_g1, vk + 576);
            mi::g2_encode(s.delta_g2, vk + 672);
        }
        if (ic)
            for (size_t i = 0; i < s.ic.size(); i++) mi::g1_encode(s.ic[i], ic + 96 * i);
    });
}

int mi_srs_info(const mi_srs *srs, uint64_t out[6]) {
    return guard([&] {
        need(srs && out, "null argument");
        const mi::Srs &s = *srs->p;
        uint64_t v[6] = {s.d, s.n_h, s.n_l, s.n_a, s.n_b, s.n_ic};
        memcpy(out, v, sizeof v);
    });
}

int mi_srs_msm_info(const mi_srs *srs, uint64_t out[2]) {
    return guard([&] {
        need(srs && out, "null argument");
        const mi::Srs &s = *srs->p;
        out[0] = (s.h_hi || s.l_hi || s.a_hi) ? 1 : 0;
        out[1] = s.in_subgroup ? 1 : 0;
    });
}

int mi_srs_table_state(const mi_srs *srs, uint64_t out[3]) {
    return guard([&] {
        need(srs && out, "null argument");
        const mi::Srs &s = *srs->p;
        std::shared_lock<std::shared_mutex> in_use(s.use_mu);
        out[0] = (s.h_hi || s.l_hi || s.a_hi) ? 1 : 0;
        out[1] = s.tables_dropped;
        out[2] = s.in_subgroup ? 1 : 0;
    });
}

int mi_srs_shared_la(const mi_srs *srs, int *present) {
    return guard([&] {
        need(srs && present, "null argument");
        const mi::Srs &s = *srs->p;
        std::shared_lock<std::shared_mutex> in_use(s.use_mu);
        *present = s.a_aux ? 1 : 0;
    });
}

int mi_srs_window_tables(const mi_srs *srs, uint64_t out[3]) {
    return guard([&] {
        need(srs && out, "null argument");
        const mi::Srs &s = *srs->p;
        std::shared_lock<std::shared_mutex> in_use(s.use_mu);
        uint64_t q = 0;
        for (int i = 0; i < 5; i++) q += s.wt[i] ? 1 : 0;
        out[0] = q ? s.wt_c : 0;
        out[1] = q ? (256 + s.wt_c - 1) / s.wt_c : 0;
        out[2] = q;
    });
}

int mi_srs_readmit(mi_ctx *ctx, mi_srs *srs, uint64_t *rebuilt_bytes) {
    return guard([&] {
        need(ctx && srs, "null argument");
        need(srs->device == ctx->c.device, "key and context on different devices");
        CtxLock l(ctx);
        const uint64_t got = mi::srs_readmit(ctx->c, *srs->p);
        if (rebuilt_bytes) *rebuilt_bytes = got;
    });
}

int mi_ctx_inject_oom(mi_ctx *ctx, int64_t count) {
    return guard([&] {
        need(ctx != nullptr, "null ctx");
        CtxLock l(ctx);
        ctx->c.inject_oom = count;
    });
}

int mi_fq_check_read(uint64_t out[2], int reset) {
    return guard([&] {
        need(out != nullptr, "null argument");
        out[0] = out[1] = 0;
#ifdef MI_FQ_CHECK
        for (const auto &u : mi::fq_check_symbols()) {
            unsigned int h[4] = {0, 0, 0, 0};
            MI_HIP(hipMemcpyFromSymbol(h, u.symbol, sizeof h, 0, hipMemcpyDeviceToHost));
            out[0] += h[0];
            out[1] += h[1];
            // debug build: where the counts come from (per translation unit), the largest |k| of a zero test and the
            // largest |top limb| / 2^20 of a normalised value
            fprintf(stderr, "[fq-check] %s: top-limb %u, zero-test |k| > 3 %u, max |k| %u, max |top| %u x 2^20\n",
                    u.unit, h[0], h[1], h[2], h[3]);
            if (reset) {
                const unsigned int z[4] = {0, 0, 0, 0};
                MI_HIP(hipMemcpyToSymbol(u.symbol, z, sizeof z, 0, hipMemcpyHostToDevice));
            }
        }
#else
        (void)reset;
        throw std::invalid_argument("library built without MI_FQ_CHECK (make fqcheck)");
#endif
    });
}

int mi_tune_set(const char *name, int64_t value) {
    return guard([&] {
        const int k = mi::tune::find(name);
        need(k >= 0, std::string("unknown tuning switch: ") + (name ? name : "(null)"));
        need(value != mi::tune::UNSET, "value reserved for 'unset'");
        mi::tune::set((mi::tune::Knob)k, value);
    });
}

int mi_tune_clear(const char *name) {
    return guard([&] {
        if (!name) {
            mi::tune::reset();
            return;
        }
        const int k = mi::tune::find(name);
        need(k >= 0, std::string("unknown tuning switch: ") + name);
        mi::tune::set((mi::tune::Knob)k, mi::tune::UNSET);
    });
}

int mi_tune_get(const char *name, int64_t *value, int *is_set) {
    return guard([&] {
        const int k = mi::tune::find(name);
        need(k >= 0 && value && is_set, "unknown tuning switch or null argument");
        const int64_t v = mi::tune::get((mi::tune::Knob)k, mi::tune::UNSET);
        *is_set = v != mi::tune::UNSET;
        *value = *is_set ? v : 0;
    });
}

int mi_srs_export_query_dev(mi_ctx *ctx, const mi_srs *srs, int which, uint64_t first, uint64_t n, void *dev_out) {
    return guard([&] {
        need(ctx && srs && (dev_out || !n), "null argument");
        CtxLock l(ctx, 0, FENCE);
        const mi::Srs &s = *srs->p;
        uint64_t total = 0;
        switch (which) {
            case 0: total = s.n_h; break;
            case 1: total = s.n_l; break;
            case 2: total = s.n_a; break;
            case 3: case 4: total = s.n_b; break;
            default: throw std::invalid_argument("which must be 0..4");
        }
        need(first <= total && n <= total - first, "range past the end of the query");
        if (!n) return;
        uint8_t *o = (uint8_t *)dev_out;
        switch (which) {
            case 0: mi::g1_encode_uncompressed(ctx->c, s.h_perm, o, n, s.log_d, first); break;
            case 1: mi::g1_encode_uncompressed(ctx->c, s.l, o, n, 0, first); break;
            case 2: mi::g1_encode_uncompressed(ctx->c, s.a, o, n, 0, first); break;
            case 3: mi::g1_encode_uncompressed(ctx->c, s.b_g1, o, n, 0, first); break;
            case 4: mi::g2_encode_uncompressed(ctx->c, s.b_g2 + first, o, n); break;
        }
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}

int mi_srs_export_query(mi_ctx *ctx, const mi_srs *srs, int which, uint8_t *out, uint64_t cap) {
    return guard([&] {
        need(ctx && srs && out, "null argument");
        CtxLock l(ctx);
        const mi::Srs &s = *srs->p;
        const void *src = nullptr;
        uint64_t n = 0;
        bool g2 = false;
        switch (which) {
            case 0: src = s.h_perm; n = s.n_h; break;
            case 1: src = s.l; n = s.n_l; break;
            case 2: src = s.a; n = s.n_a; break;
            case 3: src = s.b_g1; n = s.n_b; break;
            case 4: src = s.b_g2; n = s.n_b; g2 = true; break;
            default: throw std::invalid_argument("which must be 0..4");
        }
        need(cap >= n, "output buffer too small");
        if (!n) return;
        const uint64_t chunk = 1ull << 22;
        const size_t esz = g2 ? 192 : 96;
        uint8_t *stage = ctx->c.scratch[0].as<uint8_t>(esz * (n < chunk ? n : chunk));
        if (which == 0 && s.log_d) {
            // h is stored bit-reversed: encode the whole query in one pass (source index un-permuted)
            uint8_t *all = ctx->c.scratch[1].as<uint8_t>(esz * n);
            mi::g1_encode_uncompressed(ctx->c, (const mi::g1_affine_t *)src, all, n, s.log_d);
            MI_HIP(hipMemcpyAsync(out, all, esz * n, hipMemcpyDeviceToHost, ctx->c.stream));
        } else {
            for (uint64_t o = 0; o < n; o += chunk) {
                uint64_t m = n - o < chunk ? n - o : chunk;
                if (g2)
                    mi::g2_encode_uncompressed(ctx->c, (const mi::g2_affine_t *)src + o, stage, m);
                else
                    mi::g1_encode_uncompressed(ctx->c, (const mi::g1_affine_t *)src + o, stage, m, 0);
                MI_HIP(hipMemcpyAsync(out + esz * o, stage, esz * m, hipMemcpyDeviceToHost, ctx->c.stream));
                MI_HIP(hipStreamSynchronize(ctx->c.stream));
            }
        }
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}

void mi_srs_free(mi_srs *s) {
    if (!s) return;
    DeviceScope dev(s->device, false);
    delete s->p;
    delete s;
}

// ------------------------------------------------------------------------------------------
static void prove_impl(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const mi::fr_t *z_dev,
                       const uint8_t r[32], const uint8_t s[32], uint8_t *proof, uint8_t *raw) {
    mi::fr_t rr = fr_checked(r), ss = fr_checked(s);
    mi::ProofPoints pp = mi::groth16_prove(ctx->c, *srs->p, *circ->p, z_dev, rr, ss);
    proof_bytes(pp, proof, raw);
}

int mi_groth16_prove(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const uint8_t *z, const uint8_t r[32],
                     const uint8_t s[32], int priority, uint8_t *proof, uint8_t *raw) {
    return guard([&] {
        need(ctx && srs && circ && z && r && s && proof, "null argument");
        CtxLock l(ctx, priority);
        uint64_t nv = circ->p->n_in + circ->p->n_aux;
        mi::fr_t *zd = witness_upload(ctx, 0, z, nv);
        witness_ready(ctx, 0, nv);
        prove_impl(ctx, srs, circ, zd, r, s, proof, raw);
    });
}

int mi_groth16_prove_dev(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const void *z_dev,
                         const uint8_t r[32], const uint8_t s[32], int priority, uint8_t *proof, uint8_t *raw) {
    return guard([&] {
        need(ctx && srs && circ && z_dev && r && s && proof, "null argument");
        CtxLock l(ctx, priority, FENCE);
        uint64_t nv = circ->p->n_in + circ->p->n_aux;
        DevWitnessCheck chk(ctx, (const mi::fr_t *)z_dev, nv);
        uint8_t p[MI_PROOF_BYTES], w[384];
        prove_impl(ctx, srs, circ, (const mi::fr_t *)z_dev, r, s, p, raw ? w : nullptr);
        chk.verdict(nv);
        memcpy(proof, p, MI_PROOF_BYTES);
        if (raw) memcpy(raw, w, 384);
    });
}

int mi_groth16_prove_batch(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, uint64_t count,
                           const uint8_t *const *z, const uint8_t *rs, int priority, uint8_t *proofs_out) {
    return guard([&] {
        need(ctx && srs && circ && z && rs && proofs_out, "null argument");
        for (uint64_t k = 0; k < count; k++) need(z[k] != nullptr, "null witness");
        CtxLock l(ctx, priority);
        uint64_t nv = circ->p->n_in + circ->p->n_aux;
        // partition k + 1's upload (and, for pageable witnesses, its host staging on a helper thread)
        // runs while partition k is proven; witness_ready(k) then finds it finished
        // the blinding scalars are checked before any GPU work
        std::vector<mi::fr_t> rr(count), ss(count);
        for (uint64_t k = 0; k < count; k++) {
            rr[k] = fr_checked(rs + 64 * k);
            ss[k] = fr_checked(rs + 64 * k + 32);
        }
        const mi::AssemblyKey key = mi::assembly_key(*srs->p);
        // proof k's host assembly (blinding scalar multiplications, affine conversion, compression: ~10 ms
        // of CPU) runs on a helper thread while proof k + 1's MSMs run on the GPU
        std::thread assembler;
        std::exception_ptr asm_err;
        auto join_assembler = [&] {
            if (assembler.joinable()) assembler.join();
            if (asm_err) std::rethrow_exception(asm_err);
        };
        mi::fr_t *zd[2] = {witness_upload(ctx, 0, z[0], nv), nullptr};
        try {
            for (uint64_t k = 0; k < count; k++) {
                const int slot = (int)(k & 1);
                witness_ready(ctx, slot, nv);
                std::thread next;
                std::exception_ptr up_err;
                if (k + 1 < count) {
                    const int ns = slot ^ 1;
                    const uint8_t *zn = z[k + 1];
                    next = std::thread([&, ns, zn] {
                        try {
                            MI_HIP(hipSetDevice(ctx->c.device));
                            zd[ns] = witness_upload(ctx, ns, zn, nv);
                        } catch (...) {
                            up_err = std::current_exception();
                        }
                    });
                }
                mi::ProofSums sums;
                try {
                    sums = mi::groth16_sums(ctx->c, *srs->p, *circ->p, zd[slot]);
                } catch (...) {
                    if (next.joinable()) next.join();
                    throw;
                }
                if (next.joinable()) next.join();
                if (up_err) std::rethrow_exception(up_err);
                join_assembler();
                assembler = std::thread([&, sums, k] {
                    try {
                        proof_bytes(mi::groth16_assemble(key, sums, rr[k], ss[k]), proofs_out + 192 * k, nullptr);
                    } catch (...) {
                        asm_err = std::current_exception();
                    }
                });
            }
        } catch (...) {
            if (assembler.joinable()) assembler.join();
            throw;
        }
        join_assembler();
    });
}

int mi_groth16_prove_random(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const uint8_t *z, int priority,
                            uint8_t *proof) {
    uint8_t rs[64];
    int rc = guard([&] { random_blinding(1, rs); });
    if (rc != MI_OK) return rc;
    rc = mi_groth16_prove(ctx, srs, circ, z, rs, rs + 32, priority, proof, nullptr);
    memset(rs, 0, sizeof rs);
    return rc;
}
int mi_groth16_prove_dev_random(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const void *z_dev,
                                int priority, uint8_t *proof) {
    uint8_t rs[64];
    int rc = guard([&] { random_blinding(1, rs); });
    if (rc != MI_OK) return rc;
    rc = mi_groth16_prove_dev(ctx, srs, circ, z_dev, rs, rs + 32, priority, proof, nullptr);
    memset(rs, 0, sizeof rs);
    return rc;
}
int mi_groth16_prove_batch_random(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, uint64_t count,
                                  const uint8_t *const *z, int priority, uint8_t *proofs_out) {
    std::vector<uint8_t> rs(64 * (count ? count : 1));
    int rc = guard([&] { random_blinding(count, rs.data()); });
    if (rc != MI_OK) return rc;
    rc = mi_groth16_prove_batch(ctx, srs, circ, count, z, rs.data(), priority, proofs_out);
    memset(rs.data(), 0, rs.size());
    return rc;
}

static void share_impl(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const mi::fr_t *z_dev, uint32_t rank,
                       uint32_t world, uint8_t *share) {
    need(world > 0 && rank < world, "share rank out of range (rank < world)");
    mi::sums_encode(mi::groth16_sums(ctx->c, *srs->p, *circ->p, z_dev, rank, world), share);
}

int mi_groth16_prove_share(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const uint8_t *z, uint32_t rank,
                           uint32_t world, int priority, uint8_t *share) {
    return guard([&] {
        need(ctx && srs && circ && z && share, "null argument");
        CtxLock l(ctx, priority);
        uint64_t nv = circ->p->n_in + circ->p->n_aux;
        mi::fr_t *zd = witness_upload(ctx, 0, z, nv);
        witness_ready(ctx, 0, nv);
        share_impl(ctx, srs, circ, zd, rank, world, share);
    });
}

int mi_groth16_prove_share_dev(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const void *z_dev,
                               uint32_t rank, uint32_t world, int priority, uint8_t *share) {
    return guard([&] {
        need(ctx && srs && circ && z_dev && share, "null argument");
        CtxLock l(ctx, priority, FENCE);
        uint64_t nv = circ->p->n_in + circ->p->n_aux;
        DevWitnessCheck chk(ctx, (const mi::fr_t *)z_dev, nv);
        uint8_t sh[MI_SHARE_BYTES];
        share_impl(ctx, srs, circ, (const mi::fr_t *)z_dev, rank, world, sh);
        chk.verdict(nv);
        memcpy(share, sh, MI_SHARE_BYTES);
    });
}

static mi::SumRanges ranges_of(const uint64_t r[8]) {
    mi::SumRanges g;
    for (int q = 0; q < 4; q++) {
        g.lo[q] = r[2 * q];
        g.cnt[q] = r[2 * q + 1];
    }
    return g;
}

int mi_groth16_prove_share_ranges(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const uint8_t *z,
                                  const uint64_t ranges[8], int priority, uint8_t *share) {
    return guard([&] {
        need(ctx && srs && circ && z && ranges && share, "null argument");
        CtxLock l(ctx, priority);
        uint64_t nv = circ->p->n_in + circ->p->n_aux;
        mi::fr_t *zd = witness_upload(ctx, 0, z, nv);
        witness_ready(ctx, 0, nv);
        mi::sums_encode(mi::groth16_sums_ranges(ctx->c, *srs->p, *circ->p, zd, ranges_of(ranges)), share);
    });
}

int mi_groth16_prove_share_ranges_dev(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const void *z_dev,
                                      const uint64_t ranges[8], int priority, uint8_t *share) {
    return guard([&] {
        need(ctx && srs && circ && z_dev && ranges && share, "null argument");
        CtxLock l(ctx, priority, FENCE);
        uint64_t nv = circ->p->n_in + circ->p->n_aux;
        DevWitnessCheck chk(ctx, (const mi::fr_t *)z_dev, nv);
        uint8_t sh[MI_SHARE_BYTES];
        mi::sums_encode(mi::groth16_sums_ranges(ctx->c, *srs->p, *circ->p, (const mi::fr_t *)z_dev, ranges_of(ranges)),
                        sh);
        chk.verdict(nv);
        memcpy(share, sh, MI_SHARE_BYTES);
    });
}

int mi_groth16_h_coeffs_dev(mi_ctx *ctx, const mi_circuit *circ, const void *z_dev, void *h_out_dev) {
    return guard([&] {
        need(ctx && circ && z_dev && h_out_dev, "null argument");
        CtxLock l(ctx, 0, FENCE);
        uint64_t nv = circ->p->n_in + circ->p->n_aux;
        DevWitnessCheck chk(ctx, (const mi::fr_t *)z_dev, nv);
        mi::groth16_h_coeffs(ctx->c, *circ->p, (const mi::fr_t *)z_dev, (mi::fr_t *)h_out_dev);
        chk.verdict(nv);
    });
}

int mi_groth16_prove_share_ranges_h_dev(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const void *z_dev,
                                        const void *h_dev, const uint64_t ranges[8], int priority, uint8_t *share) {
    return guard([&] {
        need(ctx && srs && circ && z_dev && ranges && share, "null argument");
        CtxLock l(ctx, priority, FENCE);
        uint64_t nv = circ->p->n_in + circ->p->n_aux;
        // received H coefficients are scalars like the witness: canonical Fr or refused
        if (h_dev) check_dev_canonical(ctx->c, (const mi::fr_t *)h_dev, circ->p->d, "H coefficient");
        DevWitnessCheck chk(ctx, (const mi::fr_t *)z_dev, nv);
        uint8_t sh[MI_SHARE_BYTES];
        mi::sums_encode(mi::groth16_sums_ranges(ctx->c, *srs->p, *circ->p, (const mi::fr_t *)z_dev, ranges_of(ranges),
                                                (const mi::fr_t *)h_dev),
                        sh);
        chk.verdict(nv);
        memcpy(share, sh, MI_SHARE_BYTES);
    });
}

int mi_groth16_assemble(const uint8_t *vk, const uint8_t *shares, uint64_t count, const uint8_t r[32],
                        const uint8_t s[32], uint8_t *proof, uint8_t *raw) {
    return guard([&] {
        need(vk && shares && r && s && proof, "null argument");
        need(count > 0, "no proof shares");
        proof_bytes(mi::groth16_assemble_shares(vk, shares, count, fr_checked(r), fr_checked(s)), proof, raw);
    });
}

int mi_groth16_trapdoor_dlogs(mi_ctx *ctx, const mi_srs *srs, const mi_circuit *circ, const void *z_dev,
                              const uint8_t r[32], const uint8_t s[32], uint8_t out[96]) {
    return guard([&] {
        need(ctx && srs && circ && z_dev && r && s && out, "null argument");
        CtxLock l(ctx, 0, FENCE);
        mi::fr_t d[3];
        mi::groth16_trapdoor_dlogs(ctx->c, *srs->p, *circ->p, (const mi::fr_t *)z_dev, fr_checked(r), fr_checked(s),
                                   d);
        for (int i = 0; i < 3; i++) mi::fr_to_le(d[i], out + 32 * i);
    });
}

// ------------------------------------------------------------------------------------------
static mi_points *points_upload(mi_ctx *ctx, const uint8_t *bytes, uint64_t n, bool g2) {
    mi::Ctx &c = ctx->c;
    const size_t esz = g2 ? 192 : 96, dsz = g2 ? sizeof(mi::g2_affine_t) : sizeof(mi::g1_affine_t);
    void *dev = nullptr;
    MI_HIP(hipMalloc(&dev, dsz * (n ? n : 1)));
    int *bad = c.scratch[9].as<int>(4);
    MI_HIP(hipMemsetAsync(bad, 0, 3 * sizeof(int), c.stream));
    const uint64_t chunk = 1ull << 22;
    uint8_t *stage = c.scratch[0].as<uint8_t>(esz * (n < chunk ? (n ? n : 1) : chunk));
    for (uint64_t o = 0; o < n; o += chunk) {
        uint64_t m = n - o < chunk ? n - o : chunk;
        MI_HIP(hipMemcpyAsync(stage, bytes + esz * o, esz * m, hipMemcpyHostToDevice, c.stream));
        if (g2)
            mi::g2_decode_uncompressed(c, stage, (mi::g2_affine_t *)dev + o, m, bad);
        else
            mi::g1_decode_uncompressed(c, stage, (mi::g1_affine_t *)dev + o, m, bad);
    }
    int nbad = 0;
    MI_HIP(hipMemcpyAsync(&nbad, bad, sizeof(int), hipMemcpyDeviceToHost, c.stream));
    MI_HIP(hipStreamSynchronize(c.stream));
    if (nbad) {
        hipFree(dev);
        throw std::invalid_argument("point encoding invalid (flags, non-canonical or not on curve)");
    }
    return new mi_points{dev, n, g2 ? 1 : 0, 1};
}

int mi_points_upload_g1(mi_ctx *ctx, const uint8_t *b, uint64_t n, mi_points **out) {
    return guard([&] {
        need(ctx && (b || !n) && out, "null argument");
        CtxLock l(ctx);
        *out = points_upload(ctx, b, n, false);
    });
}
int mi_points_upload_g2(mi_ctx *ctx, const uint8_t *b, uint64_t n, mi_points **out) {
    return guard([&] {
        need(ctx && (b || !n) && out, "null argument");
        CtxLock l(ctx);
        *out = points_upload(ctx, b, n, true);
    });
}
int mi_points_from_srs(mi_ctx *ctx, const mi_srs *srs, int which, mi_points **out) {
    return guard([&] {
        need(ctx && srs && out, "null argument");
        const mi::Srs &s = *srs->p;
        switch (which) {
            case 0: *out = new mi_points{s.h_perm, s.n_h, 0, 0, nullptr, s.in_subgroup}; break;
            case 1: *out = new mi_points{s.l, s.n_l, 0, 0, nullptr, s.in_subgroup}; break;
            case 2: *out = new mi_points{s.a, s.n_a, 0, 0, nullptr, s.in_subgroup}; break;
            case 3: *out = new mi_points{s.b_g1, s.n_b, 0, 0, nullptr, s.in_subgroup}; break;
            case 4: *out = new mi_points{s.b_g2, s.n_b, 1, 0, nullptr, s.in_subgroup}; break;
            default: throw std::invalid_argument("which must be 0..4");
        }
        (*out)->srs = &s;
        (*out)->which = which;
    });
}
int mi_points_check_subgroup(mi_ctx *ctx, mi_points *p) {
    return guard([&] {
        need(ctx && p, "null argument");
        CtxLock l(ctx);
        mi::Ctx &c = ctx->c;
        int *bad = c.scratch[9].as<int>(4);
        MI_HIP(hipMemsetAsync(bad, 0, 3 * sizeof(int), c.stream));
        if (p->is_g2)
            mi::g2_subgroup_check(c, (const mi::g2_affine_t *)p->dev, p->n, bad);
        else
            mi::g1_subgroup_check(c, (const mi::g1_affine_t *)p->dev, p->n, bad);
        int nbad[3] = {0, 0, 0};
        MI_HIP(hipMemcpyAsync(nbad, bad, sizeof(nbad), hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipStreamSynchronize(c.stream));
        if (nbad[2]) {
            p->subgroup = 0;
            throw std::invalid_argument(std::to_string(nbad[2]) + " point(s) outside the prime-order subgroup");
        }
        p->subgroup = 1;
    });
}
int mi_points_info(const mi_points *p, uint64_t out[3]) {
    return guard([&] {
        need(p && out, "null argument");
        out[0] = p->n;
        out[1] = p->table() ? 1 : 0;
        out[2] = p->subgroup ? 1 : 0;
    });
}
void mi_points_free(mi_points *p) {
    if (!p) return;
    if (p->owns && p->dev) hipFree(p->dev);
    if (p->wt_own) hipFree(p->wt_own);
    delete p;
}
int mi_points_precompute(mi_ctx *ctx, mi_points *p, unsigned window_bits, uint64_t n_points) {
    return guard([&] {
        need(ctx && p, "null argument");
        need(n_points >= 1 && n_points <= p->n, "n_points must be in [1, number of bases]");
        need(window_bits == 0 || (window_bits >= 8 && window_bits <= 22), "window_bits must be 0 or 8..22");
        CtxLock l(ctx);
        const unsigned wc = window_bits ? window_bits : mi::msm_wt_window_bits(n_points);
        const unsigned nwin = (256 + wc - 1) / wc;
        need(n_points * nwin < 0x80000000ull, "table too large for 31-bit point indices");
        void *t = nullptr;
        MI_HIP(hipMalloc(&t, (p->is_g2 ? sizeof(mi::g2_affine_t) : sizeof(mi::g1_affine_t)) * n_points * nwin));
        try {
            if (p->is_g2)
                mi::g2_window_table(ctx->c, (const mi::g2_affine_t *)p->dev, n_points, wc, (mi::g2_affine_t *)t);
            else
                mi::g1_window_table(ctx->c, (const mi::g1_affine_t *)p->dev, n_points, wc, (mi::g1_affine_t *)t);
        } catch (...) {
            (void)hipFree(t);
            throw;
        }
        std::unique_lock<std::shared_mutex> swap(p->wt_mu);  // no MSM over these points reads the old table now
        if (p->wt_own) (void)hipFree(p->wt_own);
        p->wt_own = t;
        p->wt_user.p = t;
        p->wt_user.stride = n_points;
        p->wt_user.c = wc;
        p->wt_user.nwin = nwin;
    });
}
int mi_points_table_info(const mi_points *p, uint64_t out[3]) {
    return guard([&] {
        need(p && out, "null argument");
        std::shared_lock<std::shared_mutex> own(p->wt_mu);
        std::shared_lock<std::shared_mutex> key;  // a key's tables may be released by another context's OOM retry
        if (p->srs) key = std::shared_lock<std::shared_mutex>(p->srs->use_mu);
        const mi::WinTable t = p->wtab();
        out[0] = t.p ? t.c : 0;
        out[1] = t.p ? t.nwin : 0;
        out[2] = t.p ? t.stride : 0;
    });
}
uint64_t mi_points_count(const mi_points *p) { return p ? p->n : 0; }

int mi_msm_g1_dev(mi_ctx *ctx, const mi_points *bases, const void *scalars_dev, uint64_t n, uint8_t out96[96]) {
    return guard([&] {
        need(ctx && bases && scalars_dev && out96, "null argument");
        need(!bases->is_g2, "G2 bases passed to mi_msm_g1_dev");
        need(n <= bases->n, "n exceeds the number of bases");
        CtxLock l(ctx, 0, FENCE);
        std::shared_lock<std::shared_mutex> own(bases->wt_mu);  // a precompute on these points waits for this MSM
        std::shared_lock<std::shared_mutex> in_use;  // a key's query: its split table stays while this MSM runs
        if (bases->srs) in_use = std::shared_lock<std::shared_mutex>(bases->srs->use_mu);
        mi::g1_xyzz_t r;
        const mi::WinTable wt = bases->wtab();  // used when it covers the n points
        mi::msm_g1(ctx->c, (const mi::g1_affine_t *)bases->dev, (const mi::fr_t *)scalars_dev, nullptr, n, &r,
                   (const mi::g1_affine_t *)bases->table(), bases->subgroup != 0, n <= wt.stride ? &wt : nullptr);
        mi::g1_encode(mi::xyzz_to_affine(r), out96);
    });
}
int mi_msm_g2_dev(mi_ctx *ctx, const mi_points *bases, const void *scalars_dev, uint64_t n, uint8_t out192[192]) {
    return guard([&] {
        need(ctx && bases && scalars_dev && out192, "null argument");
        need(bases->is_g2, "G1 bases passed to mi_msm_g2_dev");
        need(n <= bases->n, "n exceeds the number of bases");
        CtxLock l(ctx, 0, FENCE);
        std::shared_lock<std::shared_mutex> own(bases->wt_mu);  // a precompute on these points waits for this MSM
        std::shared_lock<std::shared_mutex> in_use;  // a key's query: its window table stays while this MSM runs
        if (bases->srs) in_use = std::shared_lock<std::shared_mutex>(bases->srs->use_mu);
        mi::g2_xyzz_t r;
        const mi::WinTable wt = bases->wtab();
        mi::msm_g2(ctx->c, (const mi::g2_affine_t *)bases->dev, (const mi::fr_t *)scalars_dev, nullptr, n, &r,
                   n <= wt.stride ? &wt : nullptr);
        mi::g2_encode(mi::xyzz_to_affine(r), out192);
    });
}

int mi_msm_g1(mi_ctx *ctx, const uint8_t *bases96, const uint8_t *scalars32, uint64_t n, uint8_t out96[96]) {
    return guard([&] {
        need(ctx && (n == 0 || (bases96 && scalars32)) && out96, "null argument");
        CtxLock l(ctx);
        mi_points *p = points_upload(ctx, bases96, n, false);
        try {
            mi::fr_t *sd = upload_fr(ctx->c, 21, scalars32, n);
            mi::g1_xyzz_t r;
            mi::msm_g1(ctx->c, (const mi::g1_affine_t *)p->dev, sd, nullptr, n, &r);
            mi::g1_encode(mi::xyzz_to_affine(r), out96);
        } catch (...) {
            mi_points_free(p);
            throw;
        }
        mi_points_free(p);
    });
}
int mi_msm_g2(mi_ctx *ctx, const uint8_t *bases192, const uint8_t *scalars32, uint64_t n, uint8_t out192[192]) {
    return guard([&] {
        need(ctx && (n == 0 || (bases192 && scalars32)) && out192, "null argument");
        CtxLock l(ctx);
        mi_points *p = points_upload(ctx, bases192, n, true);
        try {
            mi::fr_t *sd = upload_fr(ctx->c, 21, scalars32, n);
            mi::g2_xyzz_t r;
            mi::msm_g2(ctx->c, (const mi::g2_affine_t *)p->dev, sd, nullptr, n, &r);
            mi::g2_encode(mi::xyzz_to_affine(r), out192);
        } catch (...) {
            mi_points_free(p);
            throw;
        }
        mi_points_free(p);
    });
}

static void ntt_impl(mi::Ctx &c, mi::fr_t *d, unsigned log_n, int inverse, int coset) {
    uint64_t n = 1ull << log_n;
    mi::fr_to_mont_inplace(c, d, n);
    if (coset && !inverse) mi::coset_scale_natural(c, d, log_n, false, nullptr);
    mi::ntt_dif(c, d, log_n, inverse != 0);
    mi::bitrev_permute(c, d, log_n);
    if (inverse) {
        mi::fr_t dd = mi::fr_t::zero();
        dd.v[0] = (uint32_t)n;
        dd.v[1] = (uint32_t)(n >> 32);
        mi::fr_t ninv = mi::inverse(mi::to_mont(dd));
        if (coset)
            mi::coset_scale_natural(c, d, log_n, true, &ninv);
        else
            mi::scale_all(c, d, n, ninv);
    }
    mi::fr_from_mont_inplace(c, d, n);
}

int mi_ntt_fr_dev(mi_ctx *ctx, void *data_dev, unsigned log_n, int inverse, int coset) {
    return guard([&] {
        need(ctx && data_dev, "null argument");
        need(log_n <= 32, "log_n > 32 (Fr 2-adicity)");
        CtxLock l(ctx, 0, FENCE);
        mi::fr_canonicalize(ctx->c, (mi::fr_t *)data_dev, 1ull << log_n);
        ntt_impl(ctx->c, (mi::fr_t *)data_dev, log_n, inverse, coset);
        MI_HIP(hipStreamSynchronize(ctx->c.stream));  // data_dev complete on return (the _dev contract)
    });
}

int mi_ntt_fr(mi_ctx *ctx, uint8_t *data32, unsigned log_n, int inverse, int coset) {
    return guard([&] {
        need(ctx && data32, "null argument");
        need(log_n <= 32, "log_n > 32 (Fr 2-adicity)");
        CtxLock l(ctx);
        uint64_t n = 1ull << log_n;
        mi::fr_t *d = upload_fr(ctx->c, 21, data32, n);
        ntt_impl(ctx->c, d, log_n, inverse, coset);
        MI_HIP(hipMemcpyAsync(data32, d, 32 * n, hipMemcpyDeviceToHost, ctx->c.stream));
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}

// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------ stacked circuit
int mi_stacked_build(const mi_stacked_shape *sh, int with_r1cs, mi_stacked **out) {
    return guard([&] {
        need(sh && out, "null argument");
        mi::stacked::Shape s;
        s.layers = sh->layers;
        s.challenges = sh->challenges;
        s.nodes = sh->nodes;
        s.base = sh->base_arity;
        s.sub = sh->sub_arity;
        s.top = sh->top_arity;
        *out = new mi_stacked{mi::stacked::build(s, with_r1cs != 0)};
    });
}
int mi_post_build(const mi_post_shape *sh, int with_r1cs, mi_stacked **out) {
    return guard([&] {
        need(sh && out, "null argument");
        need(sh->sectors > 0, "at least one sector");
        mi::stacked::Shape s;
        s.sectors = sh->sectors;
        s.layers = 0;
        s.challenges = sh->challenges;
        s.nodes = sh->nodes;
        s.base = sh->base_arity;
        s.sub = sh->sub_arity;
        s.top = sh->top_arity;
        *out = new mi_stacked{mi::stacked::build(s, with_r1cs != 0)};
    });
}
int mi_stacked_info(const mi_stacked *s, uint64_t out[12]) {
    return guard([&] {
        need(s && out, "null argument");
        const mi::stacked::Built &b = *s->b;
        uint64_t v[12] = {b.n_constraints, b.n_in, b.n_aux, b.lay.slots, b.lay.stride, b.lay.depth_d, b.lay.path_c,
                          b.ops.size(), b.level_off.empty() ? 0 : b.level_off.size() - 1, b.blocks.size(),
                          b.poseidon_ops.size(), b.col[0].size() + b.col[1].size() + b.col[2].size()};
        memcpy(out, v, sizeof v);
    });
}
int mi_stacked_r1cs(const mi_stacked *s, mi_r1cs *out) {
    return guard([&] {
        need(s && out, "null argument");
        const mi::stacked::Built &b = *s->b;
        need(b.rp[0].size() == b.n_constraints + 1, "circuit was built without its R1CS (with_r1cs = 0)");
        mi_stacked *w = const_cast<mi_stacked *>(s);
        for (int m = 0; m < 3; m++)
            if (w->full[m].size() != b.cidx[m].size()) {
                w->full[m].resize(b.cidx[m].size());
                for (size_t e = 0; e < b.cidx[m].size(); e++) w->full[m][e] = b.ctab[b.cidx[m][e]];
            }
        out->num_constraints = b.n_constraints;
        out->num_inputs = b.n_in;
        out->num_aux = b.n_aux;
        for (int m = 0; m < 3; m++) {
            out->row_ptr[m] = b.rp[m].data();
            out->col[m] = b.col[m].data();
            out->coeff[m] = (const uint8_t *)w->full[m].data();
        }
    });
}
int mi_stacked_load(mi_ctx *ctx, const mi_stacked *s, mi_circuit **out) {
    return guard([&] {
        need(ctx && s && out, "null argument");
        const mi::stacked::Built &b = *s->b;
        need(b.rp[0].size() == b.n_constraints + 1, "circuit was built without its R1CS (with_r1cs = 0)");
        CtxLock l(ctx);
        mi::R1csCompact cc{b.n_constraints, b.n_in, b.n_aux, {}, {}, {}, b.ctab.data(), b.ctab.size()};
        for (int m = 0; m < 3; m++) {
            cc.row_ptr[m] = b.rp[m].data();
            cc.col[m] = b.col[m].data();
            cc.cidx[m] = b.cidx[m].data();
        }
        *out = new mi_circuit{mi::circuit_load_compact(ctx->c, cc), ctx->c.device};
    });
}
static void stacked_check_slots(const mi::stacked::Built &b, const uint8_t *slots) {
    const mi::stacked::Layout &L = b.lay;
    for (uint64_t q = 0; q < L.slots; q++)
        need(!mi::geq_raw(mi::fr_from_le(slots + 32 * q), mi::fr_t::modulus_raw()),
             "instance slot " + std::to_string(q) + " is not a canonical Fr element");
    std::vector<uint64_t> idx;  // slots holding node indices
    if (b.shape.sectors) {
        for (uint64_t s = 0; s < b.shape.sectors; s++)
            for (unsigned n = 0; n < b.shape.challenges; n++) idx.push_back(L.post_challenge(s, n));
    } else {
        for (unsigned c = 0; c < b.shape.challenges; c++) {
            idx.push_back(L.ch_base(c));
            for (unsigned p = 0; p < 14; p++) idx.push_back(L.ch_base(c) + L.off_parent(p, b.shape.layers));
        }
    }
    {
        for (uint64_t q : idx) {
            uint64_t v;
            memcpy(&v, slots + 32 * q, 8);
            bool high = false;
            for (int k = 8; k < 32; k++) high |= slots[32 * q + k] != 0;
            need(!high && v < b.shape.nodes, "challenge / parent index in slot " + std::to_string(q) +
                                                 " is not a node index (< nodes)");
        }
    }
}
int mi_stacked_public_inputs(const mi_stacked *s, const uint8_t *slots, uint8_t *out) {
    return guard([&] {
        need(s && slots && out, "null argument");
        stacked_check_slots(*s->b, slots);
        std::vector<mi::fr_t> in;
        mi::stacked::public_inputs(*s->b, slots, in);
        for (size_t i = 0; i < in.size(); i++) memcpy(out + 32 * i, in[i].v, 32);
    });
}
int mi_stacked_witness_dev(mi_ctx *ctx, mi_stacked *s, const void *slots_dev, void *z_dev) {
    return guard([&] {
        need(ctx && s && slots_dev && z_dev, "null argument");
        CtxLock l(ctx, 0, FENCE);
        std::vector<uint8_t> host(32 * s->b->lay.slots);
        MI_HIP(hipMemcpyAsync(host.data(), slots_dev, host.size(), hipMemcpyDeviceToHost, ctx->c.stream));
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
        stacked_check_slots(*s->b, host.data());
        mi::stacked::witness_dev(ctx->c, *s->b, (const uint8_t *)slots_dev, (mi::fr_t *)z_dev);
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}
int mi_stacked_witness(mi_ctx *ctx, mi_stacked *s, const uint8_t *slots, uint8_t *z_out) {
    return guard([&] {
        need(ctx && s && slots && z_out, "null argument");
        CtxLock l(ctx);
        const mi::stacked::Built &b = *s->b;
        stacked_check_slots(b, slots);
        const uint64_t nv = b.n_in + b.n_aux;
        mi::fr_t *z = ctx->c.scratch[2].as<mi::fr_t>(nv);
        uint8_t *sd = ctx->c.scratch[3].as<uint8_t>(32 * b.lay.slots);
        MI_HIP(hipMemcpyAsync(sd, slots, 32 * b.lay.slots, hipMemcpyHostToDevice, ctx->c.stream));
        mi::stacked::witness_dev(ctx->c, *s->b, sd, z);
        MI_HIP(hipMemcpyAsync(z_out, z, 32 * nv, hipMemcpyDeviceToHost, ctx->c.stream));
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}
void mi_stacked_free(mi_stacked *s) {
    if (!s) return;
    delete s->b;
    delete s;
}
int mi_circuit_check_dev(mi_ctx *ctx, const mi_circuit *circ, const void *z_dev, uint64_t out[2]) {
    return guard([&] {
        need(ctx && circ && z_dev && out, "null argument");
        CtxLock l(ctx, 0, FENCE);
        uint64_t first = ~0ull;
        out[0] = mi::circuit_check(ctx->c, *circ->p, (const mi::fr_t *)z_dev, &first);
        out[1] = first;
    });
}

int mi_ctx_get_stats(mi_ctx *ctx, double out[39]) {
    return guard([&] {
        need(ctx && out, "null argument");
        CtxLock l(ctx);
        MI_HIP(hipStreamSynchronize(ctx->normal));
        if (ctx->high) MI_HIP(hipStreamSynchronize(ctx->high));
        ctx->c.timer.resolve();
        const mi::Stats &s = ctx->c.stats;
        const mi::KStat *ks[mi::Stats::NK] = {&s.accum_g1, &s.accum_g2, &s.msm_g1, &s.msm_g2, &s.sort,
                                              &s.ntt,      &s.prove,    &s.h2d,    &s.poseidon, &s.tree_h2d,
                                              &s.wit_a,    &s.wit_sha,  &s.wit_pos};
        for (int i = 0; i < mi::Stats::NK; i++) {
            out[3 * i] = ks[i]->ms;
            out[3 * i + 1] = (double)ks[i]->launches;
            out[3 * i + 2] = (double)ks[i]->units;
        }
    });
}
int mi_ctx_reset_stats(mi_ctx *ctx) {
    return guard([&] {
        need(ctx != nullptr, "null ctx");
        CtxLock l(ctx);
        MI_HIP(hipStreamSynchronize(ctx->normal));
        if (ctx->high) MI_HIP(hipStreamSynchronize(ctx->high));
        if (ctx->up.copy) MI_HIP(hipStreamSynchronize(ctx->up.copy));
        ctx->c.timer.resolve();
        ctx->c.stats = mi::Stats();
    });
}
int mi_ctx_get_work(mi_ctx *ctx, uint64_t out[2]) {
    return guard([&] {
        need(ctx && out, "null argument");
        CtxLock l(ctx);
        out[0] = ctx->c.stats.madds_g1;
        out[1] = ctx->c.stats.madds_g2;
    });
}
int mi_ctx_get_shared_plans(mi_ctx *ctx, uint64_t *out) {
    return guard([&] {
        need(ctx && out, "null argument");
        CtxLock l(ctx);
        *out = ctx->c.stats.shared_la;
    });
}
int mi_ctx_get_derived_plans(mi_ctx *ctx, uint64_t *out) {
    return guard([&] {
        need(ctx && out, "null argument");
        CtxLock l(ctx);
        *out = ctx->c.stats.derived_a;
    });
}
int mi_ctx_get_table_msms(mi_ctx *ctx, uint64_t out[2]) {
    return guard([&] {
        need(ctx && out, "null argument");
        CtxLock l(ctx);
        out[0] = ctx->c.stats.wt_msms;
        out[1] = ctx->c.stats.wt_msms_g2;
    });
}
int mi_ctx_get_fallbacks(mi_ctx *ctx, uint64_t out[2]) {
    return guard([&] {
        need(ctx && out, "null argument");
        CtxLock l(ctx);
        out[0] = ctx->c.stats.oom_retries;
        out[1] = ctx->c.stats.oom_freed_bytes;
    });
}
unsigned mi_msm_window_bits(uint64_t n) { return mi::msm_window_bits(n); }

// ---- verification (host) ---------------------------------------------------------------------
int mi_groth16_verify(const uint8_t *vk, const uint8_t *ic, uint64_t n_ic, const uint8_t *inputs,
                      const uint8_t proof[MI_PROOF_BYTES], int *valid) {
    return guard([&] {
        need(vk && ic && proof && valid && (n_ic <= 1 || inputs), "null argument");
        *valid = 0;
        *valid = mi::groth16_verify(vk, ic, n_ic, inputs, proof) ? 1 : 0;
    });
}

int mi_groth16_verify_batch(const uint8_t *vk, const uint8_t *ic, uint64_t n_ic, uint64_t count,
                            const uint8_t *inputs, const uint8_t *proofs, int *valid) {
    return guard([&] {
        need(vk && ic && valid && (count == 0 || proofs) && (count == 0 || n_ic <= 1 || inputs), "null argument");
        *valid = 0;
        *valid = mi::groth16_verify_batch(vk, ic, n_ic, count, inputs, proofs, nullptr) ? 1 : 0;
    });
}

int mi_groth16_verify_batch_seeded(const uint8_t *vk, const uint8_t *ic, uint64_t n_ic, uint64_t count,
                                   const uint8_t *inputs, const uint8_t *proofs, const uint8_t seed32[32],
                                   int *valid) {
    return guard([&] {
        need(vk && ic && valid && seed32 && (count == 0 || proofs) && (count == 0 || n_ic <= 1 || inputs),
             "null argument");
        *valid = 0;
        *valid = mi::groth16_verify_batch(vk, ic, n_ic, count, inputs, proofs, seed32) ? 1 : 0;
    });
}

int mi_pairing(const uint8_t g1_96[96], const uint8_t g2_192[192], uint8_t out[576]) {
    return guard([&] {
        need(g1_96 && g2_192 && out, "null argument");
        mi::g1_affine_t p;
        mi::g2_affine_t q;
        if (!mi::g1_decode_host(g1_96, p) || !mi::g2_decode_host(g2_192, q))
            throw std::domain_error("invalid point encoding");
        mi::fq_t f[12];
        mi::pairing_host(p, q, f);
        for (int i = 0; i < 12; i++) {
            mi::fq32_t raw = mi::fq_to_raw(f[i]);
            for (int w = 0; w < 12; w++)
                for (int b = 0; b < 4; b++) out[48 * i + 4 * (11 - w) + b] = (uint8_t)(raw.v[w] >> (24 - 8 * b));
        }
    });
}

// ---- parameter files -------------------------------------------------------------------------
int mi_params_inspect(const char *path, uint64_t out[6]) {
    return guard([&] {
        need(path && out, "null argument");
        MappedFile f(path);
        ParamsLayout L = parse_params(f.data(), f.len);
        for (int i = 0; i < 6; i++) out[i] = L.n[i];
    });
}

int mi_params_load(mi_ctx *ctx, const mi_circuit *circ, const char *path, int checked, mi_srs **out) {
    int rc = MI_OK;
    int prc = guard([&] {
        need(ctx && path && out, "null argument");
        *out = nullptr;
        MappedFile f(path);
        ParamsLayout L = parse_params(f.data(), f.len);
        const uint8_t *b = f.data();
        mi_srs_host h{};
        h.vk = b;
        h.ic = b + L.off[0];
        h.n_ic = L.n[0];
        h.h = b + L.off[1];
        h.n_h = L.n[1];
        h.l = b + L.off[2];
        h.n_l = L.n[2];
        h.a = b + L.off[3];
        h.n_a = L.n[3];
        h.b_g1 = b + L.off[4];
        h.n_b_g1 = L.n[4];
        h.b_g2 = b + L.off[5];
        h.n_b_g2 = L.n[5];
        rc = mi_srs_load(ctx, circ, &h, checked, out);  // sets the error text itself on failure
    });
    return prc != MI_OK ? prc : rc;
}

int mi_params_write(mi_ctx *ctx, const mi_srs *srs, const char *path) {
    return guard([&] {
        need(ctx && srs && path, "null argument");
        uint64_t info[6];
        if (mi_srs_info(srs, info) != MI_OK) throw std::runtime_error(g_err);
        // info: d, |h|, |l|, |a|, |b|, |ic|
        std::vector<uint8_t> vk(MI_VK_BYTES), ic(96 * info[5]);
        if (mi_srs_export_vk(srs, vk.data(), ic.data()) != MI_OK) throw std::runtime_error(g_err);
        FILE *f = fopen(path, "wb");
        if (!f) throw std::invalid_argument(std::string("cannot create ") + path);
        try {
            write_all(f, vk.data(), vk.size());
            write_be32(f, info[5]);
            write_all(f, ic.data(), ic.size());
            const uint64_t counts[5] = {info[1], info[2], info[3], info[4], info[4]};
            for (int which = 0; which < 5; which++) {
                std::vector<uint8_t> buf((which == 4 ? 192 : 96) * counts[which]);
                if (mi_srs_export_query(ctx, srs, which, buf.data(), counts[which]) != MI_OK)
                    throw std::runtime_error(g_err);
                write_be32(f, counts[which]);
                write_all(f, buf.data(), buf.size());
            }
        } catch (...) {
            fclose(f);
            throw;
        }
        if (fclose(f) != 0) throw std::runtime_error("close failed");
    });
}

int mi_vk_write(const mi_srs *srs, const char *path) {
    return guard([&] {
        need(srs && path, "null argument");
        uint64_t info[6];
        if (mi_srs_info(srs, info) != MI_OK) throw std::runtime_error(g_err);
        std::vector<uint8_t> vk(MI_VK_BYTES), ic(96 * info[5]);
        if (mi_srs_export_vk(srs, vk.data(), ic.data()) != MI_OK) throw std::runtime_error(g_err);
        FILE *f = fopen(path, "wb");
        if (!f) throw std::invalid_argument(std::string("cannot create ") + path);
        try {
            write_all(f, vk.data(), vk.size());
            write_be32(f, info[5]);
            write_all(f, ic.data(), ic.size());
        } catch (...) {
            fclose(f);
            throw;
        }
        if (fclose(f) != 0) throw std::runtime_error("close failed");
    });
}

}  // extern "C"

// ---- Poseidon and the stacked-PoRep Merkle trees -------------------------
namespace {

// Input uploads of the tree builders: columns / leaves go up in batches on a copy stream into two
// device staging slots (scratch 21, 22), so batch k + 1's copy overlaps batch k's hashing.  Every
// uploaded entry is checked canonical (< r) on the device (an Fr32 must represent a valid Fr,
// core/fr32.hpp:36-40); the count is read once at the end.
struct TreeUploads {
    mi::Ctx &c;
    hipStream_t cp = nullptr;
    hipEvent_t ready[2] = {nullptr, nullptr}, freed[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    int *bad = nullptr;
    explicit TreeUploads(mi::Ctx &ctx) : c(ctx) {
        MI_HIP(hipStreamCreateWithFlags(&cp, hipStreamNonBlocking));
        for (int k = 0; k < 2; k++) {
            MI_HIP(hipEventCreateWithFlags(&ready[k], hipEventDisableTiming));
            MI_HIP(hipEventCreateWithFlags(&freed[k], hipEventDisableTiming));
        }
        bad = c.scratch[23].as<int>(1);
        MI_HIP(hipMemsetAsync(bad, 0, sizeof(int), c.stream));
    }
    ~TreeUploads() {
        if (cp) hipStreamSynchronize(cp);
        for (int k = 0; k < 2; k++) {
            if (ready[k]) hipEventDestroy(ready[k]);
            if (freed[k]) hipEventDestroy(freed[k]);
        }
        if (cp) hipStreamDestroy(cp);
    }
    // copy the n entries of each source (host) into slot k at [j * stride], then make the compute
    // stream wait for them and check them
    void put(int k, const uint8_t *const *src, unsigned nsrc, uint64_t first, uint64_t n, mi::fr_t *dst,
             uint64_t stride) {
        if (used[k]) MI_HIP(hipStreamWaitEvent(cp, freed[k], 0));
        {
            hipStream_t keep = c.stream;
            c.stream = cp;
            mi::ScopedTimer t(c, &c.stats.tree_h2d, 32ull * n * nsrc);
            for (unsigned j = 0; j < nsrc; j++)
                MI_HIP(hipMemcpyAsync(dst + j * stride, src[j] + 32 * first, 32 * n, hipMemcpyHostToDevice, cp));
            c.stream = keep;
        }
        MI_HIP(hipEventRecord(ready[k], cp));
        MI_HIP(hipStreamWaitEvent(c.stream, ready[k], 0));
        for (unsigned j = 0; j < nsrc; j++) mi::fr_count_noncanonical(c, dst + j * stride, n, bad, c.stream);
    }
    void release(int k) {  // slot k may be overwritten once the compute stream is past this point
        MI_HIP(hipEventRecord(freed[k], c.stream));
        used[k] = true;
    }
    void check(const char *what) {
        int h = 0;
        MI_HIP(hipMemcpyAsync(&h, bad, sizeof(int), hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipStreamSynchronize(c.stream));
        if (h) throw std::invalid_argument(std::string(what) + ": entry is not a canonical Fr (>= r)");
    }
};

uint64_t tree_batch() {  // columns / leaves per upload batch (tune::TREE_BATCH overrides, for tests)
    const int64_t v = mi::tune::get(mi::tune::TREE_BATCH, 0);
    return v > 0 ? (uint64_t)v : (1ull << 21);
}

void check_dev_canonical(mi::Ctx &c, const mi::fr_t *d, uint64_t n, const char *what) {
    int *bad = c.scratch[23].as<int>(1);
    MI_HIP(hipMemsetAsync(bad, 0, sizeof(int), c.stream));
    mi::fr_count_noncanonical(c, d, n, bad, c.stream);
    int h = 0;
    MI_HIP(hipMemcpyAsync(&h, bad, sizeof(int), hipMemcpyDeviceToHost, c.stream));
    MI_HIP(hipStreamSynchronize(c.stream));
    if (h) throw std::invalid_argument(std::string(what) + ": entry is not a canonical Fr (>= r)");
}

void need_tree_arity(unsigned a) { need(a == 2 || a == 4 || a == 8 || a == 11, "arity must be 2, 4, 8 or 11"); }

}  // namespace

extern "C" {

int mi_poseidon_constants(unsigned arity, uint8_t *round_constants, uint8_t *mds, uint32_t shape[3]) {
    return guard([&] {
        need(shape != nullptr, "null shape");
        need_tree_arity(arity);
        const mi::PoseidonHost h = mi::poseidon_derive(arity, mi::poseidon_sbox_field());
        shape[0] = h.t;
        shape[1] = (uint32_t)h.rf;
        shape[2] = (uint32_t)h.rp;
        if (round_constants)
            for (size_t i = 0; i < h.plain_rc.size(); i++) mi::fr_to_le(h.plain_rc[i], round_constants + 32 * i);
        if (mds)
            for (size_t i = 0; i < h.plain_mds.size(); i++) mi::fr_to_le(h.plain_mds[i], mds + 32 * i);
    });
}

int mi_poseidon_hash_dev(mi_ctx *ctx, unsigned arity, const void *preimages_dev, uint64_t count, void *digests_dev) {
    return guard([&] {
        need(ctx && (count == 0 || (preimages_dev && digests_dev)), "null argument");
        need_tree_arity(arity);
        CtxLock l(ctx, 0, FENCE);
        check_dev_canonical(ctx->c, (const mi::fr_t *)preimages_dev, count * arity, "poseidon preimage");
        mi::poseidon_hash_dev(ctx->c, arity, (const mi::fr_t *)preimages_dev, count, arity, 1,
                              (mi::fr_t *)digests_dev);
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}

int mi_poseidon_hash(mi_ctx *ctx, unsigned arity, const uint8_t *preimages, uint64_t count, uint8_t *digests) {
    return guard([&] {
        need(ctx && (count == 0 || (preimages && digests)), "null argument");
        need_tree_arity(arity);
        CtxLock l(ctx);
        if (!count) return;
        mi::fr_t *in = ctx->c.scratch[21].as<mi::fr_t>(count * arity);
        mi::fr_t *out = ctx->c.scratch[22].as<mi::fr_t>(count);
        MI_HIP(hipMemcpyAsync(in, preimages, 32 * count * arity, hipMemcpyHostToDevice, ctx->c.stream));
        check_dev_canonical(ctx->c, in, count * arity, "poseidon preimage");
        mi::poseidon_hash_dev(ctx->c, arity, in, count, arity, 1, out);
        MI_HIP(hipMemcpyAsync(digests, out, 32 * count, hipMemcpyDeviceToHost, ctx->c.stream));
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}

int mi_tree_cache_size(uint64_t leaves, unsigned arity, unsigned rows_to_discard, uint64_t *out) {
    return guard([&] {
        need(out != nullptr, "null out");
        *out = mi::tree_rows_size(leaves, arity, rows_to_discard);
    });
}

int mi_tree_build_dev(mi_ctx *ctx, unsigned arity, const void *leaves_dev, uint64_t leaves, unsigned rows_to_discard,
                      void *tree_dev) {
    return guard([&] {
        need(ctx && leaves_dev && tree_dev, "null argument");
        need_tree_arity(arity);
        CtxLock l(ctx, 0, FENCE);
        mi::tree_rows_size(leaves, arity, rows_to_discard);
        check_dev_canonical(ctx->c, (const mi::fr_t *)leaves_dev, leaves, "tree leaf");
        mi::fr_t *tmp = ctx->c.scratch[22].as<mi::fr_t>(2 * (leaves / arity) + 1);
        mi::tree_build_dev(ctx->c, arity, (const mi::fr_t *)leaves_dev, leaves, rows_to_discard,
                           (mi::fr_t *)tree_dev, tmp);
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}

int mi_tree_build(mi_ctx *ctx, unsigned arity, const uint8_t *leaves, uint64_t n, unsigned rows_to_discard,
                  uint8_t *tree_out) {
    return guard([&] {
        need(ctx && leaves && tree_out, "null argument");
        need_tree_arity(arity);
        CtxLock l(ctx);
        mi::Ctx &c = ctx->c;
        const uint64_t tsz = mi::tree_rows_size(n, arity, rows_to_discard);
        mi::fr_t *leaf_dev = c.scratch[20].as<mi::fr_t>(n + tsz);
        mi::fr_t *rows = leaf_dev + n;
        {
            TreeUploads up(c);
            const uint64_t B = tree_batch();
            int k = 0;
            for (uint64_t b = 0; b < n; b += B, k ^= 1) {
                const uint64_t nb = std::min(B, n - b);
                const uint8_t *src[1] = {leaves};
                up.put(k, src, 1, b, nb, leaf_dev + b, 0);
                up.release(k);
            }
            up.check("tree leaf");
        }
        mi::fr_t *tmp = c.scratch[22].as<mi::fr_t>(2 * (n / arity) + 1);
        mi::tree_build_dev(c, arity, leaf_dev, n, rows_to_discard, rows, tmp);
        MI_HIP(hipMemcpyAsync(tree_out, rows, 32 * tsz, hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipStreamSynchronize(c.stream));
    });
}

// ColumnTreeBuilder::add_final_columns: base = column hashes (nodes), tree = every row above the base
int mi_tree_c_build_dev(mi_ctx *ctx, unsigned layers, uint64_t nodes, const void *labels_dev, unsigned tree_arity,
                        void *base_dev, void *tree_dev) {
    return guard([&] {
        need(ctx && labels_dev && base_dev && tree_dev, "null argument");
        need_tree_arity(layers);
        need_tree_arity(tree_arity);
        CtxLock l(ctx, 0, FENCE);
        mi::Ctx &c = ctx->c;
        mi::tree_rows_size(nodes, tree_arity, 0);
        check_dev_canonical(c, (const mi::fr_t *)labels_dev, nodes * layers, "layer label");
        mi::poseidon_hash_dev(c, layers, (const mi::fr_t *)labels_dev, nodes, 1, nodes, (mi::fr_t *)base_dev);
        mi::tree_build_dev(c, tree_arity, (const mi::fr_t *)base_dev, nodes, 0, (mi::fr_t *)tree_dev, nullptr);
        MI_HIP(hipStreamSynchronize(c.stream));
    });
}

int mi_tree_c_build(mi_ctx *ctx, unsigned layers, uint64_t nodes, const uint8_t *const *layer_labels,
                    unsigned tree_arity, uint8_t *base_out, uint8_t *tree_out) {
    return guard([&] {
        need(ctx && layer_labels && base_out && tree_out, "null argument");
        need_tree_arity(layers);
        need_tree_arity(tree_arity);
        for (unsigned j = 0; j < layers; j++) need(layer_labels[j] != nullptr, "null layer");
        CtxLock l(ctx);
        mi::Ctx &c = ctx->c;
        const uint64_t tsz = mi::tree_rows_size(nodes, tree_arity, 0);
        mi::fr_t *base = c.scratch[20].as<mi::fr_t>(nodes + tsz);
        mi::fr_t *rows = base + nodes;
        const uint64_t B = std::min<uint64_t>(tree_batch(), nodes);
        mi::fr_t *stage[2] = {c.scratch[21].as<mi::fr_t>(B * layers), c.scratch[22].as<mi::fr_t>(B * layers)};
        {
            TreeUploads up(c);
            int k = 0;
            for (uint64_t b = 0; b < nodes; b += B, k ^= 1) {
                const uint64_t nb = std::min(B, nodes - b);
                up.put(k, layer_labels, layers, b, nb, stage[k], B);
                mi::poseidon_hash_dev(c, layers, stage[k], nb, 1, B, base + b);
                up.release(k);
            }
            up.check("layer label");
        }
        mi::tree_build_dev(c, tree_arity, base, nodes, 0, rows, nullptr);
        MI_HIP(hipMemcpyAsync(base_out, base, 32 * nodes, hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipMemcpyAsync(tree_out, rows, 32 * tsz, hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipStreamSynchronize(c.stream));
    });
}

// generate_tree_r_last: replica = label + data (written back over data), then TreeBuilder over it
int mi_tree_r_last_build_dev(mi_ctx *ctx, uint64_t nodes, const void *labels_dev, void *data_dev, unsigned tree_arity,
                             unsigned rows_to_discard, void *tree_dev) {
    return guard([&] {
        need(ctx && labels_dev && data_dev && tree_dev, "null argument");
        need_tree_arity(tree_arity);
        CtxLock l(ctx, 0, FENCE);
        mi::Ctx &c = ctx->c;
        mi::tree_rows_size(nodes, tree_arity, rows_to_discard);
        check_dev_canonical(c, (const mi::fr_t *)labels_dev, nodes, "last-layer label");
        check_dev_canonical(c, (const mi::fr_t *)data_dev, nodes, "sector data node");
        mi::encode_dev(c, (const mi::fr_t *)labels_dev, (mi::fr_t *)data_dev, nodes);
        mi::fr_t *tmp = c.scratch[22].as<mi::fr_t>(2 * (nodes / tree_arity) + 1);
        mi::tree_build_dev(c, tree_arity, (const mi::fr_t *)data_dev, nodes, rows_to_discard, (mi::fr_t *)tree_dev, tmp);
        MI_HIP(hipStreamSynchronize(c.stream));
    });
}

int mi_tree_r_last_build(mi_ctx *ctx, uint64_t nodes, const uint8_t *last_layer_labels, uint8_t *data,
                         unsigned tree_arity, unsigned rows_to_discard, uint8_t *tree_out) {
    return guard([&] {
        need(ctx && last_layer_labels && data && tree_out, "null argument");
        need_tree_arity(tree_arity);
        CtxLock l(ctx);
        mi::Ctx &c = ctx->c;
        const uint64_t tsz = mi::tree_rows_size(nodes, tree_arity, rows_to_discard);
        mi::fr_t *leaves = c.scratch[20].as<mi::fr_t>(nodes + tsz);
        mi::fr_t *rows = leaves + nodes;
        const uint64_t B = std::min<uint64_t>(tree_batch(), nodes);
        mi::fr_t *stage[2] = {c.scratch[21].as<mi::fr_t>(B), c.scratch[22].as<mi::fr_t>(B)};
        {
            TreeUploads up(c);
            int k = 0;
            for (uint64_t b = 0; b < nodes; b += B, k ^= 1) {
                const uint64_t nb = std::min(B, nodes - b);
                const uint8_t *lab[1] = {last_layer_labels}, *dat[1] = {data};
                up.put(k, lab, 1, b, nb, stage[k], 0);
                up.put(k, dat, 1, b, nb, leaves + b, 0);
                mi::encode_dev(c, stage[k], leaves + b, nb);
                up.release(k);
            }
            up.check("last-layer label / sector data node");
        }
        // the replica goes back to the caller (the reference overwrites the data buffer in place)
        MI_HIP(hipMemcpyAsync(data, leaves, 32 * nodes, hipMemcpyDeviceToHost, c.stream));
        mi::fr_t *tmp = c.scratch[22].as<mi::fr_t>(2 * (nodes / tree_arity) + 1);
        mi::tree_build_dev(c, tree_arity, leaves, nodes, rows_to_discard, rows, tmp);
        MI_HIP(hipMemcpyAsync(tree_out, rows, 32 * tsz, hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipStreamSynchronize(c.stream));
    });
}

}  // extern "C"

// ---- SDR labelling witness (sdr.hip) -------------------------------------------------
namespace {
__global__ void k_sdr_check(const uint32_t *layers, const uint32_t *parent_idx, uint64_t n, uint32_t per,
                            uint32_t n_layers, uint64_t nodes_per_layer, int *bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bool ok = layers[i] >= 1 && layers[i] <= n_layers;
    for (uint32_t k = 0; k < per; k++) ok &= parent_idx[i * per + k] < nodes_per_layer;
    if (!ok) atomicOr(bad, 1);
}
}  // namespace

int mi_sdr_labels_dev(mi_ctx *ctx, const uint8_t replica_id[32], uint64_t count, const void *layers_dev,
                      const void *nodes_dev, const void *parents_dev, unsigned n_parents, void *labels_dev) {
    return guard([&] {
        need(ctx && replica_id && (count == 0 || (layers_dev && nodes_dev && labels_dev)), "null argument");
        need(n_parents <= 37, "n_parents must be <= 37");
        need(count == 0 || n_parents == 0 || parents_dev, "null parents");
        CtxLock l(ctx, 0, FENCE);
        mi::sdr_labels_dev(ctx->c, mi::sdr_replica(replica_id), (const uint32_t *)layers_dev,
                           (const uint64_t *)nodes_dev, parents_dev, n_parents, count, labels_dev);
        MI_HIP(hipStreamSynchronize(ctx->c.stream));  // labels_dev complete on return, like the other _dev calls
    });
}

int mi_sdr_labels(mi_ctx *ctx, const uint8_t replica_id[32], uint64_t count, const uint32_t *layers,
                  const uint64_t *nodes, const uint8_t *parents, unsigned n_parents, uint8_t *labels) {
    return guard([&] {
        need(ctx && replica_id && (count == 0 || (layers && nodes && labels)), "null argument");
        need(n_parents <= 37, "n_parents must be <= 37");
        need(count == 0 || n_parents == 0 || parents, "null parents");
        CtxLock l(ctx);
        if (!count) return;
        mi::Ctx &c = ctx->c;
        uint8_t *idx = c.scratch[21].as<uint8_t>(count * 12);  // nodes (u64) then layers (u32)
        uint8_t *par = n_parents ? c.scratch[20].as<uint8_t>(count * n_parents * 32) : nullptr;
        uint8_t *out = c.scratch[22].as<uint8_t>(count * 32);
        MI_HIP(hipMemcpyAsync(idx, nodes, 8 * count, hipMemcpyHostToDevice, c.stream));
        MI_HIP(hipMemcpyAsync(idx + 8 * count, layers, 4 * count, hipMemcpyHostToDevice, c.stream));
        if (par) MI_HIP(hipMemcpyAsync(par, parents, 32ull * n_parents * count, hipMemcpyHostToDevice, c.stream));
        mi::sdr_labels_dev(c, mi::sdr_replica(replica_id), (const uint32_t *)(idx + 8 * count),
                           (const uint64_t *)idx, par, n_parents, count, out);
        MI_HIP(hipMemcpyAsync(labels, out, 32 * count, hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipStreamSynchronize(c.stream));
    });
}

int mi_sdr_labeling_proofs_dev(mi_ctx *ctx, const uint8_t replica_id[32], unsigned n_layers,
                               uint64_t nodes_per_layer, const void *layer_labels_dev, uint64_t count,
                               const void *layers_dev, const void *challenges_dev, const void *parent_idx_dev,
                               unsigned n_base, unsigned n_exp, void *labels_dev, void *parents_out_dev) {
    return guard([&] {
        need(ctx && replica_id && (count == 0 || (layer_labels_dev && layers_dev && challenges_dev &&
                                                  parent_idx_dev && labels_dev)),
             "null argument");
        need(n_base >= 1 && n_base + n_exp <= 37, "need 1 <= n_base and n_base + n_exp <= 37");
        need(n_layers >= 1 && nodes_per_layer >= 1, "need at least one layer and one node");
        need(nodes_per_layer <= (1ull << 32), "nodes_per_layer must fit the u32 parent indices");
        CtxLock l(ctx, 0, FENCE);
        if (!count) return;
        mi::Ctx &c = ctx->c;
        // every layer and parent index is checked on the device before the gather reads through them
        int *bad = c.scratch[23].as<int>(1);
        MI_HIP(hipMemsetAsync(bad, 0, sizeof(int), c.stream));
        k_sdr_check<<<(unsigned)((count + 255) / 256), 256, 0, c.stream>>>(
            (const uint32_t *)layers_dev, (const uint32_t *)parent_idx_dev, count, n_base + n_exp, n_layers,
            nodes_per_layer, bad);
        MI_LAUNCHED(c, "k_sdr_check");
        int h = 0;
        MI_HIP(hipMemcpyAsync(&h, bad, sizeof(int), hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipStreamSynchronize(c.stream));
        need(h == 0, "sdr: a layer is outside [1, n_layers] or a parent index is >= nodes_per_layer");
        mi::sdr_labels_gather_dev(c, mi::sdr_replica(replica_id), layer_labels_dev, nodes_per_layer,
                                  (const uint32_t *)layers_dev, (const uint64_t *)challenges_dev,
                                  (const uint32_t *)parent_idx_dev, n_base, n_exp, count, labels_dev,
                                  parents_out_dev);
        MI_HIP(hipStreamSynchronize(c.stream));
    });
}

// ---- Merkle inclusion paths over device-resident Poseidon trees (poseidon.hip) --------------------------
namespace {
__global__ void k_chal_check(const uint64_t *chal, uint64_t count, uint64_t n, int *bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count && chal[i] >= n) atomicOr(bad, 1);
}
}  // namespace

int mi_tree_inclusion_paths_dev(mi_ctx *ctx, unsigned arity, const void *leaves_dev, uint64_t leaf_count,
                                unsigned rows_to_discard, const void *tree_dev, uint64_t count,
                                const void *challenges_dev, void *leaf_out_dev, void *siblings_out_dev) {
    return guard([&] {
        need(ctx && leaves_dev && tree_dev && (count == 0 || (challenges_dev && leaf_out_dev && siblings_out_dev)),
             "null argument");
        need_tree_arity(arity);
        CtxLock l(ctx, 0, FENCE);
        mi::tree_rows_size(leaf_count, arity, rows_to_discard);
        if (!count) return;
        mi::Ctx &c = ctx->c;
        int *bad = c.scratch[23].as<int>(1);
        MI_HIP(hipMemsetAsync(bad, 0, sizeof(int), c.stream));
        k_chal_check<<<(unsigned)((count + 255) / 256), 256, 0, c.stream>>>((const uint64_t *)challenges_dev, count,
                                                                            leaf_count, bad);
        MI_LAUNCHED(c, "k_chal_check");
        int h = 0;
        MI_HIP(hipMemcpyAsync(&h, bad, sizeof(int), hipMemcpyDeviceToHost, c.stream));
        MI_HIP(hipStreamSynchronize(c.stream));
        need(h == 0, "tree: a challenge is >= the leaf count");
        uint64_t B = 1;
        for (unsigned r = 0; r <= rows_to_discard; r++) B *= arity;
        mi::fr_t *rec = rows_to_discard ? c.scratch[22].as<mi::fr_t>(2 * count * B) : nullptr;
        mi::tree_paths_dev(c, arity, (const mi::fr_t *)leaves_dev, leaf_count, rows_to_discard,
                           (const mi::fr_t *)tree_dev, (const uint64_t *)challenges_dev, count, rec,
                           (mi::fr_t *)leaf_out_dev, (mi::fr_t *)siblings_out_dev);
        MI_HIP(hipStreamSynchronize(c.stream));
    });
}
int mi_tree_d_inclusion_paths_dev(mi_ctx *ctx, const void *leaves_dev, uint64_t leaf_count, const void *tree_dev,
                                  uint64_t count, const void *challenges_dev, void *leaf_out_dev,
                                  void *siblings_out_dev) {
    // tree D keeps every row (binary SHA-256; rebuilding discarded rows would need the SHA-256 hasher), so its
    // openings are pure reads of the cached rows: arity 2, rows_to_discard 0, nothing recomputed
    return mi_tree_inclusion_paths_dev(ctx, 2, leaves_dev, leaf_count, 0, tree_dev, count, challenges_dev,
                                       leaf_out_dev, siblings_out_dev);
}

int mi_tree_d_build_dev(mi_ctx *ctx, const void *leaves_dev, uint64_t leaf_count, void *tree_dev) {
    return guard([&] {
        need(ctx && leaves_dev && tree_dev, "null argument");
        need(leaf_count >= 2 && (leaf_count & (leaf_count - 1)) == 0, "tree D: leaf count must be a power of two >= 2");
        CtxLock l(ctx, 0, FENCE);
        mi::tree_d_build_dev(ctx->c, leaves_dev, leaf_count, tree_dev);
        MI_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}
