// container.cpp — CompressData byte container (huff_coding/src/comp.rs).
#include <cstring>
#include <functional>

#include "huff_coding.hpp"

namespace huff {

std::vector<uint8_t> pack_msb0(const std::vector<uint8_t>& bits) {
    // bitvec::BitVec<Msb0,u8>::into_vec: bit i -> byte i/8, mask 0x80>>(i%8),
    // unused tail bits zero.
    std::vector<uint8_t> out((bits.size() + 7) / 8, 0);
    for (size_t i = 0; i < bits.size(); ++i)
        if (bits[i]) out[i >> 3] |= static_cast<uint8_t>(0x80u >> (i & 7));
    return out;
}

std::vector<uint8_t> unpack_msb0(const uint8_t* bytes, size_t nbits) {
    std::vector<uint8_t> bits(nbits);
    for (size_t i = 0; i < nbits; ++i) bits[i] = (bytes[i >> 3] >> (7 - (i & 7))) & 1;
    return bits;
}

Status container_bits_to_bytes(const std::vector<uint8_t>& tree_bits, const uint8_t* comp, size_t len,
                               uint8_t padding, std::vector<uint8_t>& out) {
    // comp.rs:279-300
    uint8_t tree_pad = calc_padding_bits(tree_bits.size());
    uint32_t tree_len = static_cast<uint32_t>((tree_bits.size() + tree_pad) / 8);
    std::vector<uint8_t> tree_bytes = pack_msb0(tree_bits);
    out.clear();
    out.reserve(5 + tree_len + len);
    out.push_back(static_cast<uint8_t>((tree_pad << 4) + padding));
    out.push_back(static_cast<uint8_t>(tree_len >> 24));
    out.push_back(static_cast<uint8_t>(tree_len >> 16));
    out.push_back(static_cast<uint8_t>(tree_len >> 8));
    out.push_back(static_cast<uint8_t>(tree_len));
    out.insert(out.end(), tree_bytes.begin(), tree_bytes.end());
    out.insert(out.end(), comp, comp + len);
    return Status::ok();
}

Status container_to_bytes(const HuffTree& t, const uint8_t* comp, size_t len, uint8_t padding,
                          std::vector<uint8_t>& out) {
    return container_bits_to_bytes(t.as_bin(), comp, len, padding, out);
}

Status container_parse(const uint8_t* bytes, size_t n, const std::function<Status(const std::vector<uint8_t>&)>& tree,
                       uint8_t& padding, size_t& comp_off, size_t& comp_len) {
    // comp.rs:128-184, errors in the reference's order; its panics are
    // returned as their own status codes.
    if (n < 1) return Status::err(HUFF_E_FROM_BYTES, "slice is empty");
    const uint8_t tree_pad = bytes[0] >> 4;
    const uint8_t data_pad = bytes[0] & 0x0F;
    if (n < 5) return Status::err(HUFF_E_FROM_BYTES, "slice too short to read tree length");
    const size_t tree_len = (static_cast<size_t>(bytes[1]) << 24) | (static_cast<size_t>(bytes[2]) << 16) |
                            (static_cast<size_t>(bytes[3]) << 8) | bytes[4];
    if (tree_len < 2) return Status::err(HUFF_E_TREE_LEN, "stored tree length must be at least 2");
    if (n - 5 < tree_len) return Status::err(HUFF_E_FROM_BYTES, "slice too short to read tree");
    size_t nbits = tree_len * 8;
    nbits = tree_pad > nbits ? 0 : nbits - tree_pad;  // `for _ in 0..tree_padding_bits { b.pop(); }`
    std::vector<uint8_t> bits = unpack_msb0(bytes + 5, nbits);
    if (tree(bits)) return Status::err(HUFF_E_FROM_BYTES, "invalid tree in slice");
    comp_off = 5 + tree_len;
    comp_len = n - comp_off;
    // CompressData::new (comp.rs:55-68)
    if (comp_len == 0) return Status::err(HUFF_E_EMPTY_COMP, "provided comp_bytes are empty");
    if (data_pad > 7) return Status::err(HUFF_E_PADDING, "padding bits cannot be larger than 7");
    padding = data_pad;
    return Status::ok();
}

Status container_from_bytes(const uint8_t* bytes, size_t n, HuffTree& tree, uint8_t& padding,
                            size_t& comp_off, size_t& comp_len) {
    return container_parse(
        bytes, n, [&](const std::vector<uint8_t>& bits) { return HuffTree::try_from_bin(bits, tree); }, padding,
        comp_off, comp_len);
}

}  // namespace huff
