// wide.hpp — HuffTree<L> for the reference's other integer letter types
// (SURVEY.md §8f-3): L in {u8, u16, u32, u64, u128} and their signed twins
// (letter.rs:41-60 integer_letter_impl), i.e. letters of W = 1, 2, 4, 8 or 16
// bytes handled as their W-byte bit patterns (two's complement for the
// signed types: Rust's to_be_bytes / from_be_bytes are bit copies).
//
// What differs from the u8 path (huff_coding.hpp):
//  - weights are any `Weights<L>` in the caller's iteration order
//    (weights.rs:27-32; a HashMap<L, usize> from build_weights_map,
//    weights.rs:97-130): the tree is a function of that order, exactly as in
//    tree_inner.rs:281-320, so the boundary takes (letters[], weights[]) in it;
//  - as_bin / try_from_bin write and read W*8 letter bits (tree_inner.rs:
//    557-576, 657-661);
//  - the number of leaves is unbounded (a leaf per distinct letter).
#pragma once

#include <cstdint>
#include <vector>

#include "huff_coding.hpp"

namespace huff {

using u128 = unsigned __int128;

inline bool valid_width(uint32_t w) { return w == 1 || w == 2 || w == 4 || w == 8 || w == 16; }

// W little-endian bytes (native integer layout) <-> value
inline u128 load_letter(const uint8_t* p, uint32_t w) {
    u128 v = 0;
    for (uint32_t i = w; i-- > 0;) v = (v << 8) | p[i];
    return v;
}
inline void store_letter(uint8_t* p, uint32_t w, u128 v) {
    for (uint32_t i = 0; i < w; ++i) p[i] = static_cast<uint8_t>(v >> (8 * i));
}

struct WideNode {
    int32_t left = -1, right = -1;
    uint64_t weight = 0;
    u128 letter = 0;
    bool is_leaf = false;
};

struct WideLeaf {
    u128 letter;
    uint64_t code;  // right-aligned path bits (valid when len <= 64)
    uint32_t len;
};

class WideTree {
public:
    // tree_inner.rs:281-320 over `n` (letter, weight) pairs in iteration order
    static Status from_weights(uint32_t width, const uint8_t* letters, const uint64_t* weights, size_t n,
                               WideTree& out);
    // tree_inner.rs:522-604 with W*8 letter bits (bits one per element)
    static Status try_from_bin(uint32_t width, const std::vector<uint8_t>& bits, WideTree& out);
    // tree_inner.rs:632-668 (one bit per element)
    std::vector<uint8_t> as_bin() const;

    // every leaf in preorder (left first) with its path; a root leaf has the
    // code "0" (tree_inner.rs:313-315). false if some path exceeds 64 bits.
    bool leaves(std::vector<WideLeaf>& out) const;
    // read_codes (tree_inner.rs:356-419): one code per distinct letter, the
    // later leaf in preorder winning; sorted by letter value.
    bool read_codes(std::vector<WideLeaf>& out) const;
    // the same tree with every letter replaced by 0: the u8 tree the
    // self-synchronising decode kernels take (they only use code lengths)
    HuffTree shape() const;

    uint32_t width() const { return width_; }
    size_t num_leaves() const;
    uint32_t max_depth() const;
    bool root_is_leaf() const { return nodes_[root_].is_leaf; }
    const std::vector<WideNode>& nodes() const { return nodes_; }
    int32_t root() const { return root_; }

private:
    uint32_t width_ = 1;
    std::vector<WideNode> nodes_;
    int32_t root_ = -1;
};

// Device tables of a wide tree.
//  encode: two-choice cuckoo table (wide_buckets) of 2^k >= 2 * distinct
//          slots, keys of wide_key_bytes (native layout), value
//          (code << 8) | len (len 0 = empty); codes must fit 56 bits.
//  decode: primary table of 2^bits entries then 8-bit secondaries; leaf =
//          (len << 24) | leaf index, pointer = kLutPtr | secondary offset;
//          letters[leaf index] (W bytes each) in `letters`.
constexpr uint32_t kWideLutPtr = 0x80000000u;  // = dev::kLutPtr
constexpr uint32_t kWideLutMaxBits = 12;        // = dev::kLutMaxBits
constexpr uint32_t kWideMaxDecodeLen = 57;      // = dev::kLongMaxLen
constexpr uint32_t kWideMaxEncodeLen = 56;      // (code << 8) | len in a u64
constexpr uint64_t kWideFold0 = 0xC2B2AE3D27D4EB4Full;

struct WideEncTables {
    uint32_t width = 1;
    uint32_t log2_slots = 0;     // slots = 2 * buckets
    // 16-byte keys fold to lo ^ hi * fold before hashing; distinct keys that
    // fold alike under one multiplier separate under another (re-seeded)
    uint64_t fold = kWideFold0;
    std::vector<uint8_t> keys;   // slots * wide_key_bytes(width)
    std::vector<uint64_t> vals;  // slots
    std::vector<uint32_t> vals32;  // the same when every code has <= 24 bits (else empty)
    uint32_t maxlen = 0;
    size_t distinct = 0;
};
struct WideDecTables {
    std::vector<uint32_t> lut;
    uint32_t bits = 0, maxdepth = 0;
    std::vector<uint8_t> letters;  // leaves * W
};

// Two-choice cuckoo table for encode: buckets of 2 slots (slot = 2 b + j);
// a key lives in one of the slots of bucket b1 or b2, so a lookup is four
// fixed loads and no loop. Keys of <= 4 bytes are stored as u32. Same hashes
// on host and device (device/wide.hip buckets_of).
inline uint32_t wide_key_bytes(uint32_t width) { return width < 4 ? 4 : width; }
inline void wide_buckets(uint64_t lo, uint64_t hi, uint32_t lgb, uint32_t width, uint64_t fold, uint32_t* b1,
                         uint32_t* b2) {
    if (width <= 4) {
        const uint32_t x = static_cast<uint32_t>(lo);
        *b1 = static_cast<uint32_t>((static_cast<uint64_t>(x * 0x9E3779B1u)) >> (32 - lgb));
        *b2 = static_cast<uint32_t>((static_cast<uint64_t>(x * 0x85EBCA77u + 0x165667B1u)) >> (32 - lgb));
        return;
    }
    const uint64_t k = lo ^ (hi * fold);
    *b1 = static_cast<uint32_t>((k * 0x9E3779B97F4A7C15ull) >> (64 - lgb));
    *b2 = static_cast<uint32_t>((k * 0xD6E8FEB86659FD93ull + 0x165667B19E3779F9ull) >> (64 - lgb));
}

Status build_wide_enc_tables(const WideTree& t, WideEncTables& out);
Status build_wide_dec_tables(const WideTree& t, WideDecTables& out);

}  // namespace huff
