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
//  encode: a two-choice cuckoo table of single-slot buckets (wide_slots):
//          `slots` slots of slot_bytes, each {key, value} (wide_slot_layout),
//          value 0 = empty. Short codes (<= kWideShortMax bits): value u32
//          code << (32 - len) | len; long codes (<= 56 bits): u64
//          code << 6 | len (the byte path's CodeTable entries, kernels.hpp).
//          Letters are inserted shortest code first, so the frequent ones
//          sit in their first slot and a lookup rarely needs the second.
//  decode: primary table of 2^bits entries then 8-bit secondaries; leaf =
//          (len << 24) | leaf index, pointer = kLutPtr | secondary offset;
//          letters[leaf index] (W bytes each) in `letters`.
constexpr uint32_t kWideLutPtr = 0x80000000u;  // = dev::kLutPtr
constexpr uint32_t kWideLutMaxBits = 12;        // = dev::kLutMaxBits
constexpr uint32_t kWideMaxDecodeLen = 57;      // = dev::kLongMaxLen
constexpr uint32_t kWideMaxEncodeLen = 56;      // code << 6 | len in a u64 (= dev::kLongMaxLen - 1)
constexpr uint32_t kWideShortMax = 27;          // = dev::kShortMaxLen
constexpr uint64_t kWideFold0 = 0xC2B2AE3D27D4EB4Full;

struct WideEncTables {
    uint32_t width = 1;
    uint32_t slots = 0;
    uint32_t slot_bytes = 8;
    uint32_t val_off = 4;
    uint32_t mul1 = 0;            // odd hash multiplier (wide_slots)
    uint32_t hash_mode = 0;       // WideHash
    uint64_t fold = kWideFold0;   // 8- and 16-byte keys: 64-bit fold multiplier (wide_hkey)
    bool long_codes = false;
    std::vector<uint8_t> table;   // slots * slot_bytes
    uint32_t maxlen = 0;
    size_t distinct = 0;
};
struct WideDecTables {
    std::vector<uint32_t> lut;
    uint32_t bits = 0, maxdepth = 0;
    std::vector<uint8_t> letters;  // leaves * W
    // the task decoder's two-level table (device/wdecode.hip): level 1 of
    // 2^sbits entries, the first code of each window: its length in bits
    // [0, 6) and, in bits 8..31, the letter (W <= 2, and W = 4 when every
    // letter is below 2^24) or the leaf index (W >= 8, and W = 4 otherwise:
    // w4_leaf); or 0x80 | s with the offset of a level-2 table of 2^s entries
    // (indexed by the next s bits, lengths counted from the window start) in
    // bits 8..31. u32 entries, padded to 16 B.
    std::vector<uint8_t> stab;
    uint32_t sbits = 0;
    bool w4_leaf = false;
};

// Slot layout: the key at offset 0 (keys of <= 4 bytes as u32, native
// little-endian), the value at val_off, slots of 8 bytes ({u32 key, u32
// value}) or multiples of 16. Same layout as device/wide.hip Slot<>. An
// empty slot holds value 0 and a key that is no letter of the table, so a
// key match alone finds a letter.
inline uint32_t wide_key_bytes(uint32_t width) { return width < 4 ? 4 : width; }
inline void wide_slot_layout(uint32_t width, bool long_codes, uint32_t* val_off, uint32_t* slot_bytes) {
    const uint32_t kb = wide_key_bytes(width), vb = long_codes ? 8 : 4;
    *val_off = (kb + vb - 1) / vb * vb;
    *slot_bytes = kb + vb <= 8 ? 8 : (*val_off + vb + 15) / 16 * 16;
}
// The 32-bit hash key of a letter: the letter itself for <= 4 bytes, else
// the high half of a 64-bit multiply (16-byte letters fold lo ^ hi * fold
// first). Letters with equal hash keys share both slots, so at most two of
// them fit: the builder re-seeds `fold` when that fails.
inline uint32_t wide_hkey(uint64_t lo, uint64_t hi, uint32_t width, uint64_t fold) {
    if (width <= 4) return static_cast<uint32_t>(lo);
    const uint64_t k = width == 16 ? lo ^ (hi * fold) : lo;
    return static_cast<uint32_t>((k * fold) >> 32);
}
// The two slots of a hash key (= device/wide.hip wslots). Generic: h = x *
// mul, s1 = the high half of h * slots. Narrow (keys of <= 2 bytes, slots <
// 65536): h = (x * mul) on 24 bits, s1 = ((h >> 8) * (slots << 8)) >> 32 (the
// GPU's full-rate 24-bit multiplies). s2 = s1 ^ bits 8..15 of h (slots a
// multiple of 256; s2 = s1 leaves the key one slot). Direct (keys of <= 2
// bytes, slots = 65536): s1 = s2 = x.
enum WideHash : uint32_t { kWideHashGeneric = 0, kWideHashNarrow = 1, kWideHashDirect = 2 };
inline void wide_slots(uint32_t x, uint32_t mul, uint32_t slots, uint32_t mode, uint32_t* s1, uint32_t* s2) {
    uint32_t h;
    if (mode == kWideHashNarrow) {
        h = static_cast<uint32_t>(static_cast<uint64_t>(x & 0xFFFFFFu) * (mul & 0xFFFFFFu));
        *s1 = static_cast<uint32_t>((static_cast<uint64_t>(h >> 8) * ((slots << 8) & 0xFFFFFFu)) >> 32);
    } else if (mode == kWideHashDirect) {
        *s1 = *s2 = x;
        return;
    } else {
        h = x * mul;
        *s1 = static_cast<uint32_t>((static_cast<uint64_t>(h) * slots) >> 32);
    }
    *s2 = *s1 ^ ((h >> 8) & 255u);
}

Status build_wide_enc_tables(const WideTree& t, WideEncTables& out);
Status build_wide_dec_tables(const WideTree& t, WideDecTables& out);

}  // namespace huff
