// wide_rt.hpp — runtime objects of the wider-letter path (include/huffgpu_wide.h).
//
// huff_wtree: a HuffTree<L> (host/wide.hpp) with its device tables built once
// (hash table for encode, lookup table + leaf letters for decode, and the
// shape as a u8 tree for the self-synchronising decoder).
// huff_wenc: one job over n letters already in HBM: bits (pass A, restart
// index) -> pack (pass B) -> decode, as huff_enc is for bytes.
#pragma once

#include <memory>
#include <mutex>

#include "../host/wide.hpp"
#include "runtime.hpp"

struct huff_wtree {
    huff::WideTree t;
    uint64_t id;
    mutable std::mutex m;
    mutable std::unique_ptr<huff::WideEncTables> enc;
    mutable std::unique_ptr<huff::WideDecTables> dec;
    mutable std::unique_ptr<huff_tree> shape;
    mutable std::vector<int32_t> up;  // parent links for branch codes (capi_util.hpp parent_links), built once

    huff_wtree();
    huff::Status enc_tables(const huff::WideEncTables** out) const;
    huff::Status dec_tables(const huff::WideDecTables** out) const;
    const huff_tree* shape_tree() const;
};

struct huff_wcompress_data {
    std::vector<uint8_t> comp;
    uint8_t padding = 0;
    huff_wtree* tree = nullptr;  // owned clone
    std::unique_ptr<huff_index_host> index;
    ~huff_wcompress_data() { delete tree; }
};

struct huff_wenc {
    huff_ctx* ctx = nullptr;
    const uint8_t* d_in = nullptr;
    uint64_t n = 0;
    uint32_t width = 1;
    uint32_t nchunks = 0;
    DevBuf chunk_bits, chunk_start, tsum, sub_bit, missing;
    DevBuf table, lut, letters, stab;  // device tables of the last trees used
    uint64_t enc_tree = 0, dec_tree = 0;
    const huff::WideEncTables* et = nullptr;
    const huff::WideDecTables* dt = nullptr;
    uint64_t bits_tree = 0;  // tree of the last pass A (0: none)
    uint64_t total_bits = 0;

    huff::Status init(huff_ctx* c, uint32_t w, const uint8_t* d, uint64_t nletters);
    huff::dev::WideArgs enc_args(bool pack_pass) const;  // the table and job fields of a pass
    // pass A; a letter without a code -> HUFF_E_MISSING_LETTER, its value in *missing
    huff::Status bits(const huff_wtree* t, uint64_t* total, huff::u128* missing);
    huff::Status pack(const huff_wtree* t, uint8_t* d_out, size_t out_cap, uint64_t* total);
    huff::Status decode(const huff_wtree* t, const uint8_t* d_comp, uint64_t comp_bytes, uint8_t* d_out,
                        const uint64_t* sub_abs = nullptr, bool skip_packed = false);
    huff::Status upload_dec(const huff_wtree* t);
    huff::Status download_index(huff_index_host& idx);
    huff::Status upload_index(const huff_index_host& idx);
};

namespace huff {
Status wweights_map_host(huff_ctx* ctx, uint32_t width, const uint8_t* letters, size_t n,
                         std::vector<uint8_t>& uniq, std::vector<uint64_t>& counts);
Status wcompress_host(huff_ctx* ctx, uint32_t width, const uint8_t* letters, size_t n, const huff_wtree* t,
                      huff_wcompress_data** out, u128* missing);
Status wdecompress_host(huff_ctx* ctx, const huff_wcompress_data* cd, uint8_t* out, size_t cap_letters,
                        size_t* n_out);
// index-free decode of a device stream; d_out == nullptr: count only
Status wdecode_indexless_dev(huff_ctx* ctx, const huff_wtree* t, const uint8_t* d_comp, uint64_t comp_bytes,
                             uint64_t valid_bits, uint8_t* d_out, size_t cap_letters, uint64_t* n_out);
}  // namespace huff
