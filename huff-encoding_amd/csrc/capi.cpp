// capi.cpp — the extern "C" boundary (include/huffgpu.h).
//
// Each entry point converts huff::Status into an int code plus the
// thread-local last-error message; nothing throws across the ABI.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <exception>
#include <new>
#include <string>
#include <vector>

#include "runtime/runtime.hpp"

#include "capi_util.hpp"

namespace huff::capi {

namespace {
thread_local std::string t_last_error;
thread_local uint8_t t_missing = 0;
}  // namespace

int report(const huff::Status& s) {
    if (s.code != HUFF_OK) {
        t_last_error = s.msg;
        if (s.code == HUFF_E_MISSING_LETTER) t_missing = s.missing_letter;
    }
    return s.code;
}

int fail(int code, const char* msg) {
    t_last_error = msg;
    return code;
}

const char* last_error() { return t_last_error.c_str(); }
uint8_t last_missing() { return t_missing; }

}  // namespace huff::capi

using huff::capi::fail;
using huff::capi::guarded;
using huff::capi::report;

extern "C" {

const char* huff_last_error(void) { return huff::capi::last_error(); }
uint8_t huff_last_missing_letter(void) { return huff::capi::last_missing(); }
const char* huff_version(void) { return "huffgpu 0.1 (gfx950)"; }

// --------------------------------------------------------------------------
int huff_ctx_create(int device, huff_ctx** out) {
    if (!out) return fail(HUFF_E_INVALID_ARG, "null output");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return fail(HUFF_E_NO_DEVICE, "no HIP device available (the GPU codec has no CPU fallback)");
    if (device < 0 || device >= count) return fail(HUFF_E_INVALID_ARG, "device index out of range");
    return guarded([&]() -> huff::Status {
        auto* c = new huff_ctx();
        c->device = device;
        huff::Status st = c->activate();
        // a blocking stream: ordered after work on the legacy default stream
        // (where PyTorch allocates and fills tensors unless told otherwise)
        if (!st && hipStreamCreateWithFlags(&c->own, hipStreamDefault) != hipSuccess)
            st = huff::Status::err(HUFF_E_HIP, "hipStreamCreate failed");
        if (!st && hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess)
            st = huff::Status::err(HUFF_E_HIP, "hipStreamCreate failed");
        if (!st && hipEventCreateWithFlags(&c->lut_free, hipEventDisableTiming) != hipSuccess)
            st = huff::Status::err(HUFF_E_HIP, "hipEventCreate failed");
        if (st) {
            delete c;
            return st;
        }
        c->stream = c->own;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            c->cu_count = cus;
        *out = c;
        return huff::Status::ok();
    });
}

int huff_ctx_destroy(huff_ctx* ctx) {
    if (!ctx) return HUFF_OK;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    ctx->file_ws.reset();
    for (auto& p : ctx->pending) {
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    for (auto e : ctx->free_events) hipEventDestroy(e);
    if (ctx->copy_stream) {
        hipStreamSynchronize(ctx->copy_stream);
        hipStreamDestroy(ctx->copy_stream);
    }
    if (ctx->lut_free) hipEventDestroy(ctx->lut_free);
    if (ctx->own) hipStreamDestroy(ctx->own);
    delete ctx;
    return HUFF_OK;
}

int huff_ctx_set_stream(huff_ctx* ctx, void* hip_stream) {
    if (!ctx) return fail(HUFF_E_INVALID_ARG, "null context");
    ctx->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->own;
    return HUFF_OK;
}

int huff_ctx_synchronize(huff_ctx* ctx) {
    if (!ctx) return fail(HUFF_E_INVALID_ARG, "null context");
    return guarded([&] {
        HUFF_TRY(ctx->activate());
        return ctx->sync();
    });
}

int huff_ctx_device(const huff_ctx* ctx) { return ctx ? ctx->device : -1; }

int huff_ctx_set_timing(huff_ctx* ctx, int on) {
    if (!ctx) return fail(HUFF_E_INVALID_ARG, "null context");
    ctx->timing = on != 0;
    return HUFF_OK;
}

int huff_ctx_kernel_time(huff_ctx* ctx, const char* name, double* total_ms, uint64_t* launches) {
    if (!ctx || !name || !total_ms || !launches) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        HUFF_TRY(ctx->activate());
        HUFF_TRY(ctx->collect_timing());
        auto it = ctx->kstats.find(name);
        *total_ms = it == ctx->kstats.end() ? 0.0 : it->second.first;
        *launches = it == ctx->kstats.end() ? 0 : it->second.second;
        return huff::Status::ok();
    });
}

int huff_ctx_reset_timing(huff_ctx* ctx) {
    if (!ctx) return fail(HUFF_E_INVALID_ARG, "null context");
    return guarded([&] {
        HUFF_TRY(ctx->activate());
        HUFF_TRY(ctx->collect_timing());
        ctx->kstats.clear();
        return huff::Status::ok();
    });
}

// --------------------------------------------------------------------------
void huff_weights_new(huff_byte_weights* out) {
    if (out) std::memset(out, 0, sizeof(*out));
}

static void to_c(const huff::ByteWeights& w, huff_byte_weights* out) {
    for (int b = 0; b < 256; ++b) out->weights[b] = w.weights[b];
    out->len = w.len;
}

static huff::ByteWeights from_c(const huff_byte_weights* in) {
    huff::ByteWeights w;
    for (int b = 0; b < 256; ++b) w.weights[b] = in->weights[b];
    w.len = in->len;
    return w;
}

int huff_weights_from_bytes(huff_ctx* ctx, const uint8_t* bytes, size_t n, huff_byte_weights* out) {
    if (!ctx || !out || (!bytes && n)) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        huff::ByteWeights w;
        HUFF_TRY(huff::weights_from_host(ctx, bytes, n, w));
        to_c(w, out);
        return huff::Status::ok();
    });
}

int huff_weights_threaded_from_bytes(huff_ctx* ctx, const uint8_t* bytes, size_t n, size_t thread_num,
                                     huff_byte_weights* out) {
    if (!ctx || !out || (!bytes && n)) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        huff::ByteWeights w;
        HUFF_TRY(huff::weights_threaded_from_host(ctx, bytes, n, thread_num, w));
        to_c(w, out);
        return huff::Status::ok();
    });
}

void huff_weights_add(huff_byte_weights* self, const huff_byte_weights* other) {
    if (!self || !other) return;
    huff::ByteWeights a = from_c(self);
    a.add(from_c(other));
    to_c(a, self);
}

size_t huff_weights_iter(const huff_byte_weights* w, uint8_t letters[257], uint64_t weights[257]) {
    if (!w || !letters || !weights) return 0;
    return from_c(w).iter(letters, weights);
}

// --------------------------------------------------------------------------
int huff_tree_from_weights(const huff_byte_weights* w, huff_tree** out) {
    if (!w || !out) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    return guarded([&] {
        auto t = std::make_unique<huff_tree>();
        HUFF_TRY(huff::HuffTree::from_weights(from_c(w), t->t));
        *out = t.release();
        return huff::Status::ok();
    });
}

int huff_tree_clone(const huff_tree* t, huff_tree** out) {
    if (!t || !out) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        auto c = std::make_unique<huff_tree>();
        c->t = t->t;
        *out = c.release();
        return huff::Status::ok();
    });
}

void huff_tree_free(huff_tree* t) { delete t; }

size_t huff_tree_num_leaves(const huff_tree* t) { return t ? t->t.num_leaves() : 0; }
uint64_t huff_tree_root_weight(const huff_tree* t) { return t ? t->t.root_weight() : 0; }

int huff_tree_read_codes(const huff_tree* t, uint64_t code[256], uint8_t len[256]) {
    if (!t || !code || !len) return fail(HUFF_E_INVALID_ARG, "null argument");
    const huff::EncTables& e = t->enc_tables();
    std::memcpy(code, e.code, sizeof(e.code));
    std::memcpy(len, e.len, sizeof(e.len));
    if (!e.fits64) return fail(HUFF_E_CODE_TOO_LONG, "a code is longer than 64 bits; use huff_tree_code_bits");
    return HUFF_OK;
}

int huff_tree_code_bits(const huff_tree* t, uint8_t letter, uint8_t* bits, size_t cap, size_t* nbits) {
    if (!t || !nbits) return fail(HUFF_E_INVALID_ARG, "null argument");
    std::array<std::vector<uint8_t>, 256> codes;
    t->t.read_codes(codes);
    const auto& c = codes[letter];
    *nbits = c.size();
    if (cap < c.size()) return fail(HUFF_E_BUFFER_TOO_SMALL, "bit buffer too small");
    if (bits && !c.empty()) std::memcpy(bits, c.data(), c.size());
    return HUFF_OK;
}

int huff_tree_as_bin(const huff_tree* t, uint8_t* out, size_t cap, size_t* nbits) {
    if (!t || !nbits) return fail(HUFF_E_INVALID_ARG, "null argument");
    std::vector<uint8_t> bits = t->t.as_bin();
    *nbits = bits.size();
    std::vector<uint8_t> packed = huff::pack_msb0(bits);
    if (cap < packed.size()) return fail(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
    if (out) std::memcpy(out, packed.data(), packed.size());
    return HUFF_OK;
}

int huff_tree_try_from_bin(const uint8_t* bits, size_t nbits, huff_tree** out) {
    if ((!bits && nbits) || !out) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    return guarded([&] {
        auto t = std::make_unique<huff_tree>();
        HUFF_TRY(huff::HuffTree::try_from_bin(huff::unpack_msb0(bits, nbits), t->t));
        *out = t.release();
        return huff::Status::ok();
    });
}

// tree navigation (tree_inner.rs:322-325, branch.rs:207-279, leaf.rs:61-73)
static bool valid_branch(const huff_tree* t, int32_t b) {
    return t && b >= 0 && static_cast<size_t>(b) < t->t.nodes().size();
}

int huff_tree_root(const huff_tree* t, int32_t* branch) {
    if (!t || !branch) return fail(HUFF_E_INVALID_ARG, "null argument");
    *branch = t->t.root();
    return HUFF_OK;
}

int huff_branch_children(const huff_tree* t, int32_t branch, int32_t* left, int32_t* right) {
    if (!valid_branch(t, branch)) return fail(HUFF_E_INVALID_ARG, "no such branch in the tree");
    const huff::HuffNode& n = t->t.nodes()[branch];
    if (left) *left = n.is_leaf ? -1 : n.left;
    if (right) *right = n.is_leaf ? -1 : n.right;
    return HUFF_OK;
}

int huff_branch_leaf(const huff_tree* t, int32_t branch, int* has_letter, uint8_t* letter, uint64_t* weight) {
    if (!valid_branch(t, branch)) return fail(HUFF_E_INVALID_ARG, "no such branch in the tree");
    const huff::HuffNode& n = t->t.nodes()[branch];
    if (has_letter) *has_letter = n.is_leaf ? 1 : 0;
    if (letter) *letter = n.is_leaf ? n.letter : 0;
    if (weight) *weight = n.weight;
    return HUFF_OK;
}

int huff_branch_code(const huff_tree* t, int32_t branch, uint8_t* bits, size_t cap, size_t* nbits, int* has_code) {
    if (!valid_branch(t, branch) || !nbits) return fail(HUFF_E_INVALID_ARG, "null argument or no such branch");
    std::vector<uint8_t> path;
    bool has = false;
    bool below;
    {
        std::lock_guard<std::mutex> g(t->m);
        if (t->up.empty()) t->up = huff::capi::parent_links(t->t.nodes(), t->t.root());
        below = huff::capi::branch_path(t->t.nodes(), t->up, t->t.root(), branch, path, has);
    }
    if (!below)
        return fail(HUFF_E_INVALID_ARG, "the branch is not below the root");
    if (has_code) *has_code = has ? 1 : 0;
    *nbits = path.size();
    if (cap < path.size()) return fail(HUFF_E_BUFFER_TOO_SMALL, "bit buffer too small");
    if (bits && !path.empty()) std::memcpy(bits, path.data(), path.size());
    return HUFF_OK;
}

// --------------------------------------------------------------------------
int huff_cd_new(const uint8_t* comp, size_t len, uint8_t padding, const huff_tree* t, huff_compress_data** out) {
    if (!t || !out || (!comp && len)) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    if (len == 0) return fail(HUFF_E_EMPTY_COMP, "provided comp_bytes are empty");       // comp.rs:56-58
    if (padding > 7) return fail(HUFF_E_PADDING, "padding bits cannot be larger than 7");  // comp.rs:59-61
    return guarded([&] {
        auto cd = std::make_unique<huff_compress_data>();
        cd->comp.assign(comp, comp + len);
        cd->padding = padding;
        cd->tree = new huff_tree();
        cd->tree->t = t->t;
        *out = cd.release();
        return huff::Status::ok();
    });
}

void huff_cd_free(huff_compress_data* cd) { delete cd; }

int huff_cd_comp_bytes(const huff_compress_data* cd, const uint8_t** ptr, size_t* len) {
    if (!cd || !ptr || !len) return fail(HUFF_E_INVALID_ARG, "null argument");
    *ptr = cd->comp.data();
    *len = cd->comp.size();
    return HUFF_OK;
}

uint8_t huff_cd_padding(const huff_compress_data* cd) { return cd ? cd->padding : 0; }
const huff_tree* huff_cd_tree(const huff_compress_data* cd) { return cd ? cd->tree : nullptr; }
int huff_cd_has_index(const huff_compress_data* cd) { return cd && cd->index ? 1 : 0; }

int huff_cd_to_bytes(const huff_compress_data* cd, uint8_t* out, size_t cap, size_t* out_len) {
    if (!cd || !out_len) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        std::vector<uint8_t> v;
        HUFF_TRY(huff::container_to_bytes(cd->tree->t, cd->comp.data(), cd->comp.size(), cd->padding, v));
        *out_len = v.size();
        if (cap < v.size()) return huff::Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
        if (out) std::memcpy(out, v.data(), v.size());
        return huff::Status::ok();
    });
}

int huff_cd_try_from_bytes(const uint8_t* bytes, size_t n, huff_compress_data** out) {
    if ((!bytes && n) || !out) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    return guarded([&] {
        auto cd = std::make_unique<huff_compress_data>();
        cd->tree = new huff_tree();
        size_t off = 0, len = 0;
        HUFF_TRY(huff::container_from_bytes(bytes, n, cd->tree->t, cd->padding, off, len));
        cd->comp.assign(bytes + off, bytes + off + len);
        *out = cd.release();
        return huff::Status::ok();
    });
}

int huff_compress_with_tree(huff_ctx* ctx, const uint8_t* bytes, size_t n, const huff_tree* t,
                            huff_compress_data** out) {
    if (!ctx || !t || !out || (!bytes && n)) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] { return huff::compress_host(ctx, bytes, n, t, out); });
}

int huff_compress_bytes(huff_ctx* ctx, const uint8_t* bytes, size_t n, huff_compress_data** out) {
    if (!ctx || !out || (!bytes && n)) return fail(HUFF_E_INVALID_ARG, "null argument");
    if (n == 0) return fail(HUFF_E_EMPTY_WEIGHTS, "provided empty weights");  // from_weights panics first
    return guarded([&] { return huff::compress_host(ctx, bytes, n, nullptr, out); });
}

int huff_decompress(huff_ctx* ctx, const huff_compress_data* cd, uint8_t* out, size_t cap, size_t* out_len) {
    if (!ctx || !cd || !out_len || (!out && cap)) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] { return huff::decompress_host(ctx, cd, out, cap, out_len); });
}

// --------------------------------------------------------------------------
int huff_enc_create(huff_ctx* ctx, const uint8_t* d_in, size_t n, huff_enc** out) {
    if (!ctx || !out || (!d_in && n)) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    return guarded([&] {
        HUFF_TRY(ctx->activate());
        auto e = std::make_unique<huff_enc>();
        HUFF_TRY(e->init(ctx, d_in, n));
        *out = e.release();
        return huff::Status::ok();
    });
}

void huff_enc_free(huff_enc* e) {
    if (!e) return;
    if (e->ctx) {
        hipSetDevice(e->ctx->device);
        if (e->ctx->hist_pending == e) e->ctx->hist_pending = nullptr;
    }
    delete e;
}

int huff_enc_hist(huff_enc* e, uint64_t weights[256]) {
    if (!e) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        HUFF_TRY(e->hist());
        if (weights) std::memcpy(weights, e->w, sizeof(e->w));
        return huff::Status::ok();
    });
}

int huff_enc_hist_launch(huff_enc* e) {
    if (!e) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] { return e->hist_launch(); });
}

int huff_enc_hist_row(huff_enc* e, int64_t* d_row) {
    if (!e || !d_row) return fail(HUFF_E_INVALID_ARG, "null argument");
    if (reinterpret_cast<uintptr_t>(d_row) & 7) return fail(HUFF_E_INVALID_ARG, "d_row must be 8-byte aligned");
    return guarded([&] { return e->hist_row(reinterpret_cast<long long*>(d_row)); });
}

int huff_enc_bits(huff_enc* e, const huff_tree* t, uint64_t* total_bits) {
    if (!e || !t || !total_bits) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] { return e->bits(t, total_bits); });
}

int huff_enc_pack(huff_enc* e, const huff_tree* t, uint64_t bit_base, const uint8_t* prev_tail, size_t prev_tail_len,
                  uint8_t* d_out, size_t out_cap, uint64_t* total_bits) {
    if (!e || !t || !d_out || (!prev_tail && prev_tail_len)) return fail(HUFF_E_INVALID_ARG, "null argument");
    if (reinterpret_cast<uintptr_t>(d_out) & 15) return fail(HUFF_E_INVALID_ARG, "d_out must be 16-byte aligned");
    return guarded([&] { return e->pack(t, bit_base, prev_tail, prev_tail_len, d_out, out_cap, total_bits); });
}

int huff_enc_pack_shards(huff_enc* e, const uint64_t* hists, uint32_t world, uint32_t rank, const uint8_t* tails,
                         const uint8_t* tail_lens, uint8_t* d_out, size_t out_cap, huff_tree** tree_out,
                         uint64_t* bit_base_out, uint64_t* bits_out) {
    if (!e || !hists || !world || rank >= world || !d_out || !tree_out || (rank && (!tails || !tail_lens)))
        return fail(HUFF_E_INVALID_ARG, "null or out-of-range argument");
    if (reinterpret_cast<uintptr_t>(d_out) & 15) return fail(HUFF_E_INVALID_ARG, "d_out must be 16-byte aligned");
    *tree_out = nullptr;
    return guarded([&]() -> huff::Status {
        if (!e->have_hist) {  // pass 1 ran as huff_enc_hist_row: this shard's row is hists[rank]
            std::memcpy(e->w, hists + static_cast<size_t>(rank) * 256, sizeof(e->w));
            e->have_hist = true;
        }
        auto t = std::make_unique<huff_tree>();
        HUFF_TRY(huff::HuffTree::from_weights(huff::shard_weights(hists, world), t->t));
        const huff::EncTables& et = t->enc_tables();
        const uint64_t base = huff::shard_bit_base(hists, rank, et.len);
        uint8_t prev[8];
        size_t np = 0;
        if (rank) huff::shard_prev_tail(tails, tail_lens, rank, prev, &np);
        if (bit_base_out) *bit_base_out = base;
        uint64_t bits = 0;
        huff::Status st = e->pack(t.get(), base, prev + 8 - np, np, d_out, out_cap, &bits);
        if (bits_out) *bits_out = bits;
        HUFF_TRY(st);
        const huff::DecTables* dt = nullptr;  // ready for the decode that follows (huff_enc_compress)
        HUFF_TRY(e->ctx->upload_dec_tables(t.get(), &dt, true));
        *tree_out = t.release();
        return huff::Status::ok();
    });
}

int huff_enc_compress(huff_enc* e, uint8_t* d_out, size_t out_cap, huff_tree** tree_out, uint64_t* bits_out) {
    if (!e || !d_out || !tree_out) return fail(HUFF_E_INVALID_ARG, "null argument");
    if (reinterpret_cast<uintptr_t>(d_out) & 15) return fail(HUFF_E_INVALID_ARG, "d_out must be 16-byte aligned");
    *tree_out = nullptr;
    return guarded([&]() -> huff::Status {
        // HUFF_HOST_TRACE=1: host time of each phase (pass 1 + weights read-back,
        // tree, pass 2 with its tables and launch), one stderr line per call
        static const bool trace = std::getenv("HUFF_HOST_TRACE") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        HUFF_TRY(e->hist());
        const auto t1 = std::chrono::steady_clock::now();
        auto t = std::make_unique<huff_tree>();
        HUFF_TRY(huff::HuffTree::from_weights(huff::ByteWeights::from_counts(e->w), t->t));
        const auto t2 = std::chrono::steady_clock::now();
        uint64_t bits = 0;
        huff::Status st = e->pack(t.get(), 0, nullptr, 0, d_out, out_cap, &bits);
        const auto tl = std::chrono::steady_clock::now();  // pass 2 launched
        // the decode tables of the new tree, built and queued for upload
        // while pass 2 runs: a decode that follows finds them ready (built
        // there, they held its launch back ~20-35 us past the pack at 128 MiB)
        if (st.code == HUFF_OK) {
            const huff::DecTables* dt = nullptr;
            HUFF_TRY(e->ctx->upload_dec_tables(t.get(), &dt, true));
        }
        if (trace) {
            const auto t3 = std::chrono::steady_clock::now();
            auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
            auto ns = [](auto a) {
                return static_cast<long long>(
                    std::chrono::duration_cast<std::chrono::nanoseconds>(a.time_since_epoch()).count());
            };
            const auto& ps = huff::pack_stamps();  // inside pass 2's call: bit count, launch start, launch end
            std::fprintf(stderr,
                         "huff_enc_compress host us: hist %.1f tree %.1f pack %.1f (bits %.1f args %.1f launch %.1f) "
                         "at %lld %lld %lld %lld %lld\n",
                         us(t0, t1), us(t1, t2), us(t2, t3), us(t2, ps.bits), us(ps.bits, ps.launch),
                         us(ps.launch, ps.launched), ns(t0), ns(t1), ns(t2), ns(tl), ns(t3));
        }
        if (bits_out) *bits_out = bits;
        HUFF_TRY(st);
        *tree_out = t.release();
        return huff::Status::ok();
    });
}

int huff_enc_decode(huff_enc* e, const huff_tree* t, const uint8_t* d_comp, uint8_t* d_out) {
    if (!e || !t || !d_comp || (!d_out && e->n)) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        const uint64_t bytes = ((e->bit_base & 7) + e->total_bits + 7) / 8;
        return e->decode(t, d_comp, bytes, d_out);
    });
}

int huff_dev_decompress(huff_ctx* ctx, const huff_tree* t, const uint8_t* d_comp, size_t comp_bytes,
                        uint8_t padding, uint8_t* d_out, size_t out_cap, size_t* n_out) {
    if (!ctx || !t || !n_out || (!d_comp && comp_bytes)) return fail(HUFF_E_INVALID_ARG, "null argument");
    if (padding > 7) return fail(HUFF_E_PADDING, "padding bits > 7");
    *n_out = 0;
    return guarded([&]() -> huff::Status {
        const uint64_t valid = comp_bytes ? comp_bytes * 8 - padding : 0;
        DevBuf unused;
        uint64_t n = 0;
        huff::Status st = huff::decode_indexless_dev(ctx, d_comp, comp_bytes, valid, t, unused, &n,
                                                     d_out ? d_out : reinterpret_cast<uint8_t*>(1), d_out ? out_cap : 0);
        *n_out = n;
        return st;
    });
}

int huff_batch_hist(huff_ctx* ctx, const uint8_t* d_in, const uint64_t* d_offsets, uint32_t nstreams,
                    uint64_t* d_hist) {
    if (!ctx || (nstreams && (!d_offsets || !d_hist))) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&]() -> huff::Status {
        HUFF_TRY(ctx->activate());
        HUFF_TRY(ctx->timed("hist_batch",
                            [&] { return huff::dev::launch_hist_batch(d_in, d_offsets, nstreams, d_hist, ctx->stream); }));
        return ctx->sync();
    });
}

int huff_batch_trees(huff_ctx* ctx, const uint64_t* d_hist, uint32_t nstreams, uint8_t* d_tree_bits,
                     size_t tree_stride, uint32_t* d_tree_nbits, uint64_t* d_codes, uint32_t* d_max_len,
                     uint32_t* d_status) {
    if (!ctx || (nstreams && (!d_hist || !d_tree_bits || !d_tree_nbits || !d_codes || !d_max_len || !d_status)))
        return fail(HUFF_E_INVALID_ARG, "null argument");
    if (tree_stride < HUFF_TREE_BITS_MAX_BYTES || tree_stride > 0xFFFFFFFFu)
        return fail(HUFF_E_INVALID_ARG, "tree_stride < HUFF_TREE_BITS_MAX_BYTES");
    static_assert(HUFF_TREE_BITS_MAX_BYTES == huff::dev::kTreeBitsMaxBytes, "as_bin of 257 leaves");
    static_assert(static_cast<int>(huff::dev::kTreeEmpty) == static_cast<int>(HUFF_E_EMPTY_WEIGHTS) &&
                      static_cast<int>(huff::dev::kTreeDeep) == static_cast<int>(HUFF_E_CODE_TOO_LONG),
                  "the kernel writes the C ABI's status codes");
    return guarded([&]() -> huff::Status {
        HUFF_TRY(ctx->activate());
        huff::dev::TreeBatchArgs a{};
        a.hist = d_hist;
        a.nstreams = nstreams;
        a.tree_bits = d_tree_bits;
        a.tree_stride = static_cast<uint32_t>(tree_stride);
        a.tree_nbits = d_tree_nbits;
        a.codes = d_codes;
        a.max_len = d_max_len;
        a.status = d_status;
        HUFF_TRY(ctx->timed("tree_batch", [&] { return huff::dev::launch_tree_batch(a, ctx->stream); }));
        return ctx->sync();
    });
}

int huff_dev_generate(huff_ctx* ctx, int kind, uint64_t seed, uint64_t offset, const uint64_t* cdf, uint8_t* d_out,
                      size_t n) {
    if (!ctx || (!d_out && n) || (kind == 1 && !cdf)) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&]() -> huff::Status {
        HUFF_TRY(ctx->activate());
        void* d_cdf = nullptr;
        if (kind == 1) {
            if (hipMalloc(&d_cdf, 2048) != hipSuccess) return huff::Status::err(HUFF_E_HIP, "hipMalloc failed");
            hipMemcpy(d_cdf, cdf, 2048, hipMemcpyHostToDevice);
        }
        hipError_t er = huff::dev::launch_generate(kind, seed, offset, static_cast<const uint64_t*>(d_cdf), d_out, n,
                                                   ctx->stream);
        hipStreamSynchronize(ctx->stream);
        if (d_cdf) hipFree(d_cdf);
        if (er != hipSuccess) return huff::Status::err(HUFF_E_HIP, hipGetErrorString(er));
        return huff::Status::ok();
    });
}

int huff_dev_calibrate(huff_ctx* ctx, const uint8_t* d_src, uint8_t* d_dst, size_t n, int iters,
                       double* read_gbps, double* copy_gbps) {
    if (!ctx || !d_src || !d_dst || !read_gbps || !copy_gbps || iters < 1 || n < 16 ||
        (reinterpret_cast<uintptr_t>(d_src) & 15) || (reinterpret_cast<uintptr_t>(d_dst) & 15))
        return fail(HUFF_E_INVALID_ARG, "calibrate: null, misaligned or too small");
    return guarded([&]() -> huff::Status {
        HUFF_TRY(ctx->activate());
        const uint64_t m = n & ~uint64_t(15);
        // events and the sink released on every path (RAII)
        struct Res {
            hipEvent_t a = nullptr, b = nullptr;
            unsigned* sink = nullptr;
            ~Res() {
                if (sink) hipFree(sink);
                if (a) hipEventDestroy(a);
                if (b) hipEventDestroy(b);
            }
        } r;
        HIP_TRY_RT(hipEventCreate(&r.a));
        HIP_TRY_RT(hipEventCreate(&r.b));
        HIP_TRY_RT(hipMalloc(&r.sink, 16));
        hipEvent_t a = r.a, b = r.b;
        unsigned* sink = r.sink;
        float best[2] = {1e30f, 1e30f};  // [read, copy] over the two shapes of each
        hipError_t er = hipSuccess;
        for (int mode = 0; mode < 4 && er == hipSuccess; ++mode)
            for (int it = 0; it < iters + 1 && er == hipSuccess; ++it) {  // + 1 warm-up launch
                hipEventRecord(a, ctx->stream);
                er = huff::dev::launch_calib(mode, d_src, d_dst, m, sink, static_cast<uint32_t>(ctx->cu_count), ctx->stream);
                hipEventRecord(b, ctx->stream);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (it) best[mode / 2] = std::min(best[mode / 2], ms);
            }
        if (er != hipSuccess) return huff::Status::err(HUFF_E_HIP, hipGetErrorString(er));
        *read_gbps = static_cast<double>(m) / (best[0] * 1e-3) / 1e9;
        *copy_gbps = 2.0 * static_cast<double>(m) / (best[1] * 1e-3) / 1e9;
        return huff::Status::ok();
    });
}

int huff_dev_alloc(huff_ctx* ctx, size_t bytes, void** d_ptr) {
    if (!ctx || !d_ptr) return fail(HUFF_E_INVALID_ARG, "null argument");
    hipSetDevice(ctx->device);
    hipError_t e = hipMalloc(d_ptr, bytes ? bytes : 1);
    return e == hipSuccess ? HUFF_OK : fail(HUFF_E_HIP, hipGetErrorString(e));
}

int huff_dev_free(huff_ctx* ctx, void* d_ptr) {
    if (!ctx) return fail(HUFF_E_INVALID_ARG, "null argument");
    hipSetDevice(ctx->device);
    hipError_t e = hipFree(d_ptr);
    return e == hipSuccess ? HUFF_OK : fail(HUFF_E_HIP, hipGetErrorString(e));
}

int huff_memcpy_htod(huff_ctx* ctx, void* d_dst, const void* src, size_t bytes) {
    if (!ctx) return fail(HUFF_E_INVALID_ARG, "null argument");
    hipSetDevice(ctx->device);
    hipError_t e = hipMemcpy(d_dst, src, bytes, hipMemcpyHostToDevice);
    return e == hipSuccess ? HUFF_OK : fail(HUFF_E_HIP, hipGetErrorString(e));
}

int huff_memcpy_dtoh(huff_ctx* ctx, void* dst, const void* d_src, size_t bytes) {
    if (!ctx) return fail(HUFF_E_INVALID_ARG, "null argument");
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    hipError_t e = hipMemcpy(dst, d_src, bytes, hipMemcpyDeviceToHost);
    return e == hipSuccess ? HUFF_OK : fail(HUFF_E_HIP, hipGetErrorString(e));
}

// --------------------------------------------------------------------------
int huff_file_compress(huff_ctx* ctx, const char* src_path, const char* dst_path, size_t block_size) {
    if (!ctx || !src_path || !dst_path) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] { return huff::file_compress(ctx, src_path, dst_path, block_size); });
}

int huff_file_decompress(huff_ctx* ctx, const char* src_path, const char* dst_path, size_t block_size) {
    if (!ctx || !src_path || !dst_path) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] { return huff::file_decompress(ctx, src_path, dst_path, block_size); });
}

int huff_parse_block_size(const char* s, size_t* out) {
    if (!out) return fail(HUFF_E_INVALID_ARG, "null argument");
    return report(huff::parse_block_size(s, out));
}

}  // extern "C"
