// filepath.cpp — the `huff` binary's file path (huff/src/comp.rs:32-280) with
// the per-byte work on the GPU.
//
// compress: pass 1 = per block, ByteWeights::threaded_from_bytes(block, 12)
// merged into the running weights (huff/src/comp.rs:161-172); host tree;
// header [0][u32 BE tree len][tree]; pass 2 = per block compress_with_tree,
// stitched onto the previous block exactly as the reference does
// (huff/src/comp.rs:196-201 + huff/src/utils.rs:2-25: when the previous block
// left padding q != 0, the block's bytes are shifted so its first bit lands at
// bit q of the previous last byte, that byte is OR-ed in and the writer steps
// back one byte — bug-compatible); the pad byte is patched last.
// decompress: header checks with the reference's ErrorKinds, then one stream
// decode of the payload (the reference carries its walk state across blocks);
// the last byte's padding is honoured unless the payload is an exact multiple
// of the block size (huff/src/comp.rs:262-278).
#include <cstdio>
#include <memory>
#include <string>
#include <sys/stat.h>

#include "runtime.hpp"

namespace huff {

namespace {

struct File {
    FILE* f = nullptr;
    ~File() {
        if (f) fclose(f);
    }
};

Status io_err(const std::string& what, const char* path) {
    return Status::err(HUFF_E_IO, what + " " + path);
}

Status read_exact(FILE* f, uint8_t* dst, size_t n, const char* path) {
    size_t got = n ? fread(dst, 1, n, f) : 0;
    if (got != n) return io_err("failed to read", path);
    return Status::ok();
}

// compress one block already in host memory: GPU hist + pack at bit offset q
Status compress_block(huff_ctx* ctx, const uint8_t* data, size_t n, const huff_tree* t, uint8_t q,
                      std::vector<uint8_t>& out, uint8_t* padding) {
    HUFF_TRY(ctx->activate());
    HUFF_TRY(ctx->d_in.ensure(n + 16));
    HIP_TRY_RT(hipMemcpyAsync(ctx->d_in.p, data, n, hipMemcpyHostToDevice, ctx->stream));
    huff_enc e;
    HUFF_TRY(e.init(ctx, static_cast<const uint8_t*>(ctx->d_in.p), n));
    HUFF_TRY(e.hist());
    uint64_t bits = 0;
    HUFF_TRY(e.bits(t, &bits));
    const uint64_t L = (bits + 7) / 8;
    const uint64_t packed_bytes = (q + bits + 7) / 8;
    HUFF_TRY(ctx->d_out.ensure(packed_bytes + 16));
    HUFF_TRY(e.pack(t, q, nullptr, 0, static_cast<uint8_t*>(ctx->d_out.p), packed_bytes, &bits));
    // offset_bytes re-emits all 8L bits of the block (its zero padding too)
    out.assign(q ? L + 1 : L, 0);
    HIP_TRY_RT(hipMemcpyAsync(out.data(), ctx->d_out.p, packed_bytes, hipMemcpyDeviceToHost, ctx->stream));
    HUFF_TRY(ctx->sync());
    *padding = calc_padding_bits(bits);
    return Status::ok();
}

}  // namespace

Status file_compress(huff_ctx* ctx, const char* src, const char* dst, size_t block_size) {
    if (block_size == 0) return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
    File in;
    in.f = fopen(src, "rb");
    if (!in.f) return io_err("cannot open", src);
    struct stat stt;
    if (fstat(fileno(in.f), &stt) != 0) return io_err("cannot stat", src);
    if (S_ISDIR(stt.st_mode)) return Status::err(HUFF_E_IO, std::string(src) + " is a directory");
    const size_t total = static_cast<size_t>(stt.st_size);
    File out;
    out.f = fopen(dst, "wb+");
    if (!out.f) return io_err("cannot create", dst);
    std::vector<uint8_t> buf(std::min(block_size, std::max<size_t>(total, 1)));

    // pass 1 (huff_tree_from_reader)
    ByteWeights bw;
    size_t left = total;
    while (left > 0) {
        const size_t n = left >= block_size ? block_size : left;
        HUFF_TRY(read_exact(in.f, buf.data(), n, src));
        ByteWeights part;
        HUFF_TRY(weights_threaded_from_host(ctx, buf.data(), n, 12, part));
        bw.add(part);
        left -= n;
    }
    auto tree = std::make_unique<huff_tree>();
    HUFF_TRY(HuffTree::from_weights(bw, tree->t));

    // header
    std::vector<uint8_t> tbits = tree->t.as_bin();
    const uint8_t tree_pad = calc_padding_bits(tbits.size());
    std::vector<uint8_t> tbytes = pack_msb0(tbits);
    const uint32_t tl = static_cast<uint32_t>(tbytes.size());
    const uint8_t hdr[5] = {0, static_cast<uint8_t>(tl >> 24), static_cast<uint8_t>(tl >> 16),
                            static_cast<uint8_t>(tl >> 8), static_cast<uint8_t>(tl)};
    if (fwrite(hdr, 1, 5, out.f) != 5 || fwrite(tbytes.data(), 1, tbytes.size(), out.f) != tbytes.size())
        return io_err("failed to write", dst);

    // pass 2 (compress_to_writer)
    if (fseek(in.f, 0, SEEK_SET) != 0) return io_err("cannot seek", src);
    uint8_t prev_padding = 0, prev_byte = 0;
    left = total;
    std::vector<uint8_t> comp;
    while (left > 0) {
        const size_t n = left >= block_size ? block_size : left;
        HUFF_TRY(read_exact(in.f, buf.data(), n, src));
        uint8_t pad = 0;
        HUFF_TRY(compress_block(ctx, buf.data(), n, tree.get(), prev_padding, comp, &pad));
        if (prev_padding != 0) {
            if (fseek(out.f, -1, SEEK_CUR) != 0) return io_err("cannot seek", dst);
            comp[0] |= prev_byte;
        }
        if (fwrite(comp.data(), 1, comp.size(), out.f) != comp.size()) return io_err("failed to write", dst);
        prev_padding = pad;
        prev_byte = comp.back();
        left -= n;
    }
    if (fseek(out.f, 0, SEEK_SET) != 0) return io_err("cannot seek", dst);
    const uint8_t pb = static_cast<uint8_t>((tree_pad << 4) + prev_padding);
    if (fwrite(&pb, 1, 1, out.f) != 1) return io_err("failed to write", dst);
    return Status::ok();
}

Status file_decompress(huff_ctx* ctx, const char* src, const char* dst, size_t block_size) {
    if (block_size == 0) return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
    File in;
    in.f = fopen(src, "rb");
    if (!in.f) return io_err("cannot open", src);
    struct stat stt;
    if (fstat(fileno(in.f), &stt) != 0) return io_err("cannot stat", src);
    const size_t total = static_cast<size_t>(stt.st_size);
    std::vector<uint8_t> data(total);
    HUFF_TRY(read_exact(in.f, data.data(), total, src));
    const std::string q = std::string("\"") + src + "\"";
    // take(5).read(buf): at most min(5, block_size) bytes (huff/src/comp.rs:93-100)
    if (std::min<size_t>(std::min<size_t>(total, 5), block_size) < 5)
        return Status::err(HUFF_E_MISSING_HEADER, q + " too short to decompress, missing header information");
    const uint8_t tree_pad = data[0] >> 4, data_pad = data[0] & 0x0F;
    if (tree_pad > 7 || data_pad > 7)
        return Status::err(HUFF_E_INVALID_HEADER, q + " stores invalid header information");
    const size_t tree_len = (static_cast<size_t>(data[1]) << 24) | (static_cast<size_t>(data[2]) << 16) |
                            (static_cast<size_t>(data[3]) << 8) | data[4];
    if (std::min<size_t>(std::min(tree_len, total - 5), block_size) < tree_len)
        return Status::err(HUFF_E_MISSING_HEADER, q + " too short to decompress, missing header information");
    size_t nbits = tree_len * 8;
    nbits = tree_pad > nbits ? 0 : nbits - tree_pad;
    auto tree = std::make_unique<huff_tree>();
    if (HuffTree::try_from_bin(unpack_msb0(data.data() + 5, nbits), tree->t))
        return Status::err(HUFF_E_INVALID_HEADER, q + " stores invalid header information");
    const uint8_t* payload = data.data() + 5 + tree_len;
    const size_t plen = total - 5 - tree_len;
    File out;
    out.f = fopen(dst, "wb");
    if (!out.f) return io_err("cannot create", dst);
    if (plen == 0) return Status::ok();
    const bool honour_pad = (plen % block_size) != 0;
    const uint64_t valid_bits = static_cast<uint64_t>(plen) * 8 - (honour_pad ? data_pad : 0);
    std::vector<uint8_t> sym;
    HUFF_TRY(decode_indexless_host(ctx, payload, plen, valid_bits, tree.get(), sym));
    if (!sym.empty() && fwrite(sym.data(), 1, sym.size(), out.f) != sym.size()) return io_err("failed to write", dst);
    return Status::ok();
}

}  // namespace huff
