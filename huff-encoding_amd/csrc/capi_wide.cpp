// capi_wide.cpp — extern "C" boundary of the wider-letter path
// (include/huffgpu_wide.h).
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "capi_util.hpp"
#include "huffgpu_wide.h"
#include "runtime/wide_rt.hpp"

using huff::capi::fail;
using huff::capi::guarded;

namespace {
thread_local uint8_t t_missing_w[16] = {};
thread_local uint32_t t_missing_width = 0;

int report_missing(int rc, uint32_t width, huff::u128 v) {
    if (rc == HUFF_E_MISSING_LETTER) {
        huff::store_letter(t_missing_w, 16, 0);
        huff::store_letter(t_missing_w, width, v);
        t_missing_width = width;
    }
    return rc;
}
}  // namespace

extern "C" {

int huff_wtree_from_weights(uint32_t width, const void* letters, const uint64_t* weights, size_t n,
                            huff_wtree** out) {
    if (!out || (n && (!letters || !weights))) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    return guarded([&] {
        auto t = std::make_unique<huff_wtree>();
        HUFF_TRY(huff::WideTree::from_weights(width, static_cast<const uint8_t*>(letters), weights, n, t->t));
        *out = t.release();
        return huff::Status::ok();
    });
}

int huff_wtree_clone(const huff_wtree* t, huff_wtree** out) {
    if (!t || !out) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        auto c = std::make_unique<huff_wtree>();
        c->t = t->t;
        *out = c.release();
        return huff::Status::ok();
    });
}

void huff_wtree_free(huff_wtree* t) { delete t; }
uint32_t huff_wtree_width(const huff_wtree* t) { return t ? t->t.width() : 0; }
size_t huff_wtree_num_leaves(const huff_wtree* t) { return t ? t->t.num_leaves() : 0; }

int huff_wtree_read_codes(const huff_wtree* t, void* letters, uint64_t* code, uint8_t* len, size_t cap,
                          size_t* count) {
    if (!t || !count) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        std::vector<huff::WideLeaf> c;
        if (!t->t.read_codes(c)) return huff::Status::err(HUFF_E_CODE_TOO_LONG, "code longer than 64 bits");
        *count = c.size();
        if (cap < c.size()) return huff::Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
        const uint32_t W = t->t.width();
        for (size_t i = 0; i < c.size(); ++i) {
            if (letters) huff::store_letter(static_cast<uint8_t*>(letters) + i * W, W, c[i].letter);
            if (code) code[i] = c[i].code;
            if (len) len[i] = static_cast<uint8_t>(c[i].len);
        }
        return huff::Status::ok();
    });
}

int huff_wtree_as_bin(const huff_wtree* t, uint8_t* out, size_t cap, size_t* nbits) {
    if (!t || !nbits) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        const std::vector<uint8_t> bits = t->t.as_bin();
        *nbits = bits.size();
        const std::vector<uint8_t> packed = huff::pack_msb0(bits);
        if (!out) return huff::Status::ok();
        if (cap < packed.size()) return huff::Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
        std::memcpy(out, packed.data(), packed.size());
        return huff::Status::ok();
    });
}

int huff_wtree_try_from_bin(uint32_t width, const uint8_t* bits, size_t nbits, huff_wtree** out) {
    if (!out || (!bits && nbits)) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    return guarded([&] {
        auto t = std::make_unique<huff_wtree>();
        HUFF_TRY(huff::WideTree::try_from_bin(width, huff::unpack_msb0(bits, nbits), t->t));
        *out = t.release();
        return huff::Status::ok();
    });
}

// tree navigation (tree_inner.rs:322-325, branch.rs:207-279, leaf.rs:61-73)
static bool valid_wbranch(const huff_wtree* t, int32_t b) {
    return t && b >= 0 && static_cast<size_t>(b) < t->t.nodes().size();
}

int huff_wtree_root(const huff_wtree* t, int32_t* branch) {
    if (!t || !branch) return fail(HUFF_E_INVALID_ARG, "null argument");
    *branch = t->t.root();
    return HUFF_OK;
}

int huff_wbranch_children(const huff_wtree* t, int32_t branch, int32_t* left, int32_t* right) {
    if (!valid_wbranch(t, branch)) return fail(HUFF_E_INVALID_ARG, "no such branch in the tree");
    const huff::WideNode& n = t->t.nodes()[branch];
    if (left) *left = n.is_leaf ? -1 : n.left;
    if (right) *right = n.is_leaf ? -1 : n.right;
    return HUFF_OK;
}

int huff_wbranch_leaf(const huff_wtree* t, int32_t branch, int* has_letter, void* letter, uint64_t* weight) {
    if (!valid_wbranch(t, branch)) return fail(HUFF_E_INVALID_ARG, "no such branch in the tree");
    const huff::WideNode& n = t->t.nodes()[branch];
    if (has_letter) *has_letter = n.is_leaf ? 1 : 0;
    if (letter) huff::store_letter(static_cast<uint8_t*>(letter), t->t.width(), n.is_leaf ? n.letter : 0);
    if (weight) *weight = n.weight;
    return HUFF_OK;
}

int huff_wbranch_code(const huff_wtree* t, int32_t branch, uint8_t* bits, size_t cap, size_t* nbits,
                      int* has_code) {
    if (!valid_wbranch(t, branch) || !nbits) return fail(HUFF_E_INVALID_ARG, "null argument or no such branch");
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

int huff_wweights_map(huff_ctx* ctx, uint32_t width, const void* letters, size_t n, void* letters_out,
                      uint64_t* weights_out, size_t cap, size_t* count) {
    if (!ctx || !count || (n && !letters)) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        std::vector<uint8_t> u;
        std::vector<uint64_t> c;
        HUFF_TRY(huff::wweights_map_host(ctx, width, static_cast<const uint8_t*>(letters), n, u, c));
        *count = c.size();
        if (cap < c.size()) return huff::Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
        if (letters_out && !u.empty()) std::memcpy(letters_out, u.data(), u.size());
        if (weights_out && !c.empty()) std::memcpy(weights_out, c.data(), c.size() * 8);
        return huff::Status::ok();
    });
}

int huff_wcd_new(const uint8_t* comp, size_t len, uint8_t padding, const huff_wtree* t, huff_wcompress_data** out) {
    if (!t || !out || (!comp && len)) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    // CompressData::new (comp.rs:55-68)
    if (len == 0) return fail(HUFF_E_EMPTY_COMP, "provided comp_bytes are empty");
    if (padding > 7) return fail(HUFF_E_PADDING, "padding bits cannot be larger than 7");
    return guarded([&] {
        auto cd = std::make_unique<huff_wcompress_data>();
        cd->comp.assign(comp, comp + len);
        cd->padding = padding;
        cd->tree = new huff_wtree();
        cd->tree->t = t->t;
        *out = cd.release();
        return huff::Status::ok();
    });
}

void huff_wcd_free(huff_wcompress_data* cd) { delete cd; }

int huff_wcd_comp_bytes(const huff_wcompress_data* cd, const uint8_t** ptr, size_t* len) {
    if (!cd || !ptr || !len) return fail(HUFF_E_INVALID_ARG, "null argument");
    *ptr = cd->comp.data();
    *len = cd->comp.size();
    return HUFF_OK;
}

uint8_t huff_wcd_padding(const huff_wcompress_data* cd) { return cd ? cd->padding : 0; }
const huff_wtree* huff_wcd_tree(const huff_wcompress_data* cd) { return cd ? cd->tree : nullptr; }
int huff_wcd_has_index(const huff_wcompress_data* cd) { return cd && cd->index ? 1 : 0; }

int huff_wcd_to_bytes(const huff_wcompress_data* cd, uint8_t* out, size_t cap, size_t* out_len) {
    if (!cd || !out_len) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        std::vector<uint8_t> v;
        HUFF_TRY(huff::container_bits_to_bytes(cd->tree->t.as_bin(), cd->comp.data(), cd->comp.size(), cd->padding,
                                               v));
        *out_len = v.size();
        if (cap < v.size()) return huff::Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
        if (out) std::memcpy(out, v.data(), v.size());
        return huff::Status::ok();
    });
}

int huff_wcd_try_from_bytes(uint32_t width, const uint8_t* bytes, size_t n, huff_wcompress_data** out) {
    if ((!bytes && n) || !out) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    if (!huff::valid_width(width)) return fail(HUFF_E_INVALID_ARG, "letter width must be 1, 2, 4, 8 or 16 bytes");
    return guarded([&] {
        auto cd = std::make_unique<huff_wcompress_data>();
        cd->tree = new huff_wtree();
        size_t off = 0, len = 0;
        HUFF_TRY(huff::container_parse(
            bytes, n,
            [&](const std::vector<uint8_t>& bits) { return huff::WideTree::try_from_bin(width, bits, cd->tree->t); },
            cd->padding, off, len));
        cd->comp.assign(bytes + off, bytes + off + len);
        *out = cd.release();
        return huff::Status::ok();
    });
}

int huff_wcompress_with_tree(huff_ctx* ctx, const void* letters, size_t n, const huff_wtree* t,
                             huff_wcompress_data** out) {
    if (!ctx || !t || !out || (!letters && n)) return fail(HUFF_E_INVALID_ARG, "null argument");
    huff::u128 miss = 0;
    const uint32_t W = t->t.width();
    const int rc = guarded([&] {
        return huff::wcompress_host(ctx, W, static_cast<const uint8_t*>(letters), n, t, out, &miss);
    });
    return report_missing(rc, W, miss);
}

int huff_wcompress(huff_ctx* ctx, uint32_t width, const void* letters, size_t n, huff_wcompress_data** out) {
    if (!ctx || !out || (!letters && n)) return fail(HUFF_E_INVALID_ARG, "null argument");
    if (n == 0) return fail(HUFF_E_EMPTY_WEIGHTS, "provided empty weights");  // from_weights panics first
    huff::u128 miss = 0;
    const int rc = guarded([&] {
        return huff::wcompress_host(ctx, width, static_cast<const uint8_t*>(letters), n, nullptr, out, &miss);
    });
    return report_missing(rc, width, miss);
}

int huff_wdecompress(huff_ctx* ctx, const huff_wcompress_data* cd, void* out, size_t cap, size_t* n_out) {
    if (!ctx || !cd || !n_out || (!out && cap)) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] { return huff::wdecompress_host(ctx, cd, static_cast<uint8_t*>(out), cap, n_out); });
}

int huff_last_missing_wletter(void* out16, uint32_t* width) {
    if (out16) std::memcpy(out16, t_missing_w, 16);
    if (width) *width = t_missing_width;
    return HUFF_OK;
}

int huff_wenc_create(huff_ctx* ctx, uint32_t width, const void* d_in, size_t n, huff_wenc** out) {
    if (!ctx || !out || (!d_in && n)) return fail(HUFF_E_INVALID_ARG, "null argument");
    *out = nullptr;
    return guarded([&] {
        HUFF_TRY(ctx->activate());
        auto e = std::make_unique<huff_wenc>();
        HUFF_TRY(e->init(ctx, width, static_cast<const uint8_t*>(d_in), n));
        *out = e.release();
        return huff::Status::ok();
    });
}

void huff_wenc_free(huff_wenc* e) {
    if (!e) return;
    if (e->ctx) hipSetDevice(e->ctx->device);
    delete e;
}

int huff_wenc_bits(huff_wenc* e, const huff_wtree* t, uint64_t* total_bits) {
    if (!e || !t) return fail(HUFF_E_INVALID_ARG, "null argument");
    huff::u128 miss = 0;
    const int rc = guarded([&] { return e->bits(t, total_bits, &miss); });
    return report_missing(rc, e->width, miss);
}

int huff_wenc_pack(huff_wenc* e, const huff_wtree* t, uint8_t* d_out, size_t out_cap, uint64_t* total_bits) {
    if (!e || !t || !d_out) return fail(HUFF_E_INVALID_ARG, "null argument");
    huff::u128 miss = 0;
    const int rc = guarded([&] {
        if (e->bits_tree != t->id) HUFF_TRY(e->bits(t, nullptr, &miss));
        return e->pack(t, d_out, out_cap, total_bits);
    });
    return report_missing(rc, e->width, miss);
}

int huff_wenc_decode(huff_wenc* e, const huff_wtree* t, const uint8_t* d_comp, uint8_t* d_out) {
    if (!e || !t || !d_comp || !d_out) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&] {
        if (e->bits_tree == 0) return huff::Status::err(HUFF_E_STATE, "decode needs the job's restart index (pack first)");
        return e->decode(t, d_comp, (e->total_bits + 7) / 8, d_out);
    });
}

int huff_dev_wdecompress(huff_ctx* ctx, const huff_wtree* t, const uint8_t* d_comp, size_t comp_bytes,
                         uint8_t padding, void* d_out, size_t out_cap_letters, size_t* n_out) {
    if (!ctx || !t || !n_out || (!d_comp && comp_bytes)) return fail(HUFF_E_INVALID_ARG, "null argument");
    if (padding > 7) return fail(HUFF_E_PADDING, "padding bits cannot be larger than 7");
    return guarded([&] {
        const uint64_t valid = comp_bytes ? comp_bytes * 8 - padding : 0;
        uint64_t cnt = 0;
        huff::Status s = huff::wdecode_indexless_dev(ctx, t, d_comp, comp_bytes, valid, static_cast<uint8_t*>(d_out),
                                                     out_cap_letters, &cnt);
        *n_out = cnt;
        return s;
    });
}

}  // extern "C"
