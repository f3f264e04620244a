// huff_coding.hpp — C++ host mirror of the reference's `huff_coding::prelude`
// (huff_coding/src/prelude.rs:1-23) for the u8 alphabet: ByteWeights,
// HuffTree, CompressData. These run on the host by design: they touch <= 256
// letters. The per-byte work (histogram, encode, decode) is on
// the GPU (device/*.hip) and is reached through ctx.hpp.
#pragma once

#include <array>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "../common.hpp"

namespace huff {

// ---------------------------------------------------------------------------
// ByteWeights — huff_coding/src/weights.rs:174-443
// ---------------------------------------------------------------------------
struct ByteWeights {
    std::array<uint64_t, 256> weights{};  // weights.rs:176
    uint64_t len = 0;                     // weights.rs:177

    // weights.rs:265-279 semantics given a finished 256-bin count (the
    // counting itself is the hist256 kernel): len = number of non-zero bins.
    static ByteWeights from_counts(const uint64_t counts[256]);

    // weights.rs:423-441: ascending non-zero bins plus the wrap duplicate of
    // byte 0 when byte 0 is present and byte 255 absent.
    size_t iter(uint8_t letters[257], uint64_t w[257]) const;

    // weights.rs:374-387 add_byte_weights (iterates `other` with iter(), so
    // the duplicate of byte 0 is added twice).
    void add(const ByteWeights& other);

    bool is_empty() const { return len == 0; }
};

// utils.rs:6-28 ration_vec boundaries: [begin, end) of each ration.
std::vector<std::pair<size_t, size_t>> ration_bounds(size_t n, size_t ration_count);

// ---------------------------------------------------------------------------
// HuffTree — huff_coding/src/tree/tree_inner.rs
// ---------------------------------------------------------------------------
struct HuffNode {
    int32_t left = -1, right = -1;  // children (joint branch) or -1 (letter branch)
    uint64_t weight = 0;            // leaf.rs:27
    uint8_t letter = 0;             // leaf.rs:26 (Some(letter) iff is_leaf)
    bool is_leaf = false;
};

// A leaf as the decoder sees it: every leaf of the tree (duplicates included).
struct LeafCode {
    uint8_t letter;
    uint32_t len;                   // depth in bits (root-leaf tree: 1)
    std::vector<uint8_t> bits;      // path, one bit per element
};

class HuffTree {
public:
    // tree_inner.rs:281-320 from_weights; HUFF_E_EMPTY_WEIGHTS for empty.
    static Status from_weights(const ByteWeights& w, HuffTree& out);
    // Generic leaf list in push order (used for the tree_init known answer).
    static Status from_leaves(const uint8_t* letters, const uint64_t* weights, size_t n, HuffTree& out);
    // A tree of the given nodes (the generic-letter tree's shape, wide.hpp).
    static HuffTree from_nodes(std::vector<HuffNode> nodes, int32_t root) {
        HuffTree t;
        t.nodes_ = std::move(nodes);
        t.root_ = root;
        return t;
    }
    // tree_inner.rs:522-604 try_from_bin (bits one per element).
    static Status try_from_bin(const std::vector<uint8_t>& bits, HuffTree& out);

    // tree_inner.rs:632-668 as_bin (one bit per element).
    std::vector<uint8_t> as_bin() const;

    // tree_inner.rs:356-419 read_codes: per letter the code bits (overwrite
    // semantics: a later leaf in left-to-right order wins). len 0 = absent.
    void read_codes(std::array<std::vector<uint8_t>, 256>& codes) const;
    // Right-aligned u64 codes; false if any code is longer than 64 bits.
    bool read_codes_u64(uint64_t code[256], uint8_t len[256], uint32_t* maxlen) const;
    // Every leaf with its path (decode tables are built from these).
    std::vector<LeafCode> leaves() const;

    size_t num_leaves() const;
    uint32_t max_depth() const;
    // over the leaves (a root leaf counts 1), and the gcd of their depths
    void depth_range(uint32_t* min_depth, uint32_t* max_depth, uint32_t* gcd = nullptr) const;
    uint64_t root_weight() const { return nodes_[root_].weight; }
    bool root_is_leaf() const { return nodes_[root_].is_leaf; }
    const std::vector<HuffNode>& nodes() const { return nodes_; }
    int32_t root() const { return root_; }

private:
    std::vector<HuffNode> nodes_;
    int32_t root_ = -1;
};

// ---------------------------------------------------------------------------
// Sharded encode: shard `rank` of `world` contiguous shards.
// hists = world x 256 per-shard weights; tails[q*8 ..] holds shard q's last
// tail_lens[q] (<= 8) bytes. Fills the summed weights (ByteWeights::from_bytes
// of the whole stream: plain sums), and after the tree is known, the shard's
// first global bit (sum of the earlier shards' bits) and the <= 8 input bytes
// right before it (right-aligned in prev[8], count in *np).
// ---------------------------------------------------------------------------
ByteWeights shard_weights(const uint64_t* hists, uint32_t world);
uint64_t shard_bit_base(const uint64_t* hists, uint32_t rank, const uint8_t len[256]);
void shard_prev_tail(const uint8_t* tails, const uint8_t* tail_lens, uint32_t rank, uint8_t prev[8], size_t* np);

// ---------------------------------------------------------------------------
// CompressData container — huff_coding/src/comp.rs:40-184, 279-300
// ---------------------------------------------------------------------------
// Byte layout of to_bytes (comp.rs:279-300, huff/README.md):
//   [ (tree_pad << 4) + data_pad ][ u32 BE tree_len ][ tree (Msb0) ][ data ]
std::vector<uint8_t> pack_msb0(const std::vector<uint8_t>& bits);
std::vector<uint8_t> unpack_msb0(const uint8_t* bytes, size_t nbits);

Status container_to_bytes(const HuffTree& t, const uint8_t* comp, size_t len, uint8_t padding,
                          std::vector<uint8_t>& out);
Status container_bits_to_bytes(const std::vector<uint8_t>& tree_bits, const uint8_t* comp, size_t len,
                               uint8_t padding, std::vector<uint8_t>& out);
// comp.rs:128-184 with the tree parsed by `tree` (try_from_bin of the bits)
Status container_parse(const uint8_t* bytes, size_t n, const std::function<Status(const std::vector<uint8_t>&)>& tree,
                       uint8_t& padding, size_t& comp_off, size_t& comp_len);
// On success comp_off/comp_len locate the data inside `bytes`.
Status container_from_bytes(const uint8_t* bytes, size_t n, HuffTree& tree, uint8_t& padding,
                            size_t& comp_off, size_t& comp_len);

}  // namespace huff
