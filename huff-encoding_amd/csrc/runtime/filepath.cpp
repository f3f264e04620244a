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
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

// One block's buffers: pinned host bytes (the fread target and H2D source),
// the block on the device, results on the device and back in pinned memory.
// Two slots alternate, so the host reads block k+1 (and writes block k-1)
// while the GPU works on block k; uploads and downloads run on streams of
// their own beside the compute stream.
struct Stream {
    hipStream_t s = nullptr;
    ~Stream() {
        if (s) hipStreamDestroy(s);
    }
};

struct Slot {
    PinnedBuf in, res;
    DevBuf din, dres;
    hipEvent_t h2d = nullptr, kern = nullptr, done = nullptr;  // input copied; kernels done; results back
    huff_enc job;
    ~Slot() {
        if (h2d) hipEventDestroy(h2d);
        if (kern) hipEventDestroy(kern);
        if (done) hipEventDestroy(done);
    }
    Status init() {
        if (!h2d) HIP_TRY_RT(hipEventCreateWithFlags(&h2d, hipEventDisableTiming));
        if (!kern) HIP_TRY_RT(hipEventCreateWithFlags(&kern, hipEventDisableTiming));
        if (!done) HIP_TRY_RT(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        return Status::ok();
    }
};

Status sync_event(hipEvent_t e) {
    HIP_TRY_RT(hipEventSynchronize(e));
    return Status::ok();
}

// fread block bytes into the slot (once its previous upload has left it),
// then upload them on the upload stream; the compute stream waits for them
Status load_block(huff_ctx* ctx, hipStream_t up, Slot& sl, FILE* f, size_t n, const char* path) {
    HUFF_TRY(sync_event(sl.h2d));
    HUFF_TRY(sl.in.ensure(n + 16));
    HUFF_TRY(read_exact(f, static_cast<uint8_t*>(sl.in.p), n, path));
    HUFF_TRY(sl.din.ensure(n + 16));
    if (n) HIP_TRY_RT(hipMemcpyAsync(sl.din.p, sl.in.p, n, hipMemcpyHostToDevice, up));
    HIP_TRY_RT(hipEventRecord(sl.h2d, up));
    HIP_TRY_RT(hipStreamWaitEvent(ctx->stream, sl.h2d, 0));
    return Status::ok();
}

// the block's results, once its kernels are done, back to pinned memory on
// the copy stream
Status fetch_results(huff_ctx* ctx, Slot& sl, size_t bytes) {
    HUFF_TRY(sl.res.ensure(bytes + 16));
    HIP_TRY_RT(hipEventRecord(sl.kern, ctx->stream));
    HIP_TRY_RT(hipStreamWaitEvent(ctx->copy_stream, sl.kern, 0));
    if (bytes) HIP_TRY_RT(hipMemcpyAsync(sl.res.p, sl.dres.p, bytes, hipMemcpyDeviceToHost, ctx->copy_stream));
    HIP_TRY_RT(hipEventRecord(sl.done, ctx->copy_stream));
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
    HUFF_TRY(ctx->activate());
    const size_t nblocks = (total + block_size - 1) / block_size;
    auto block_len = [&](size_t k) { return std::min(block_size, total - k * block_size); };
    Slot slots[2];
    for (Slot& sl : slots) HUFF_TRY(sl.init());
    Stream up;
    HIP_TRY_RT(hipStreamCreateWithFlags(&up.s, hipStreamNonBlocking));

    // pass 1 (huff_tree_from_reader, huff/src/comp.rs:161-172): per block
    // ByteWeights::threaded_from_bytes(block, 12) (one GPU histogram per
    // ration), merged into the running weights in block order; each block's
    // plain counts are kept for pass 2's sizes
    constexpr size_t kRations = 12;
    const size_t rows_bytes = kRations * dev::kHistCopies * 256 * 8;
    ByteWeights bw;
    std::vector<std::array<uint64_t, 256>> block_counts(nblocks);
    auto merge = [&](size_t k) -> Status {  // block k's rations, once copied back
        Slot& sl = slots[k % 2];
        HUFF_TRY(sync_event(sl.done));
        const uint64_t* h = static_cast<const uint64_t*>(sl.res.p);
        const auto rations = ration_bounds(block_len(k), kRations);
        std::vector<ByteWeights> parts(rations.size());
        auto& bc = block_counts[k];
        bc.fill(0);
        for (size_t r = 0; r < rations.size(); ++r) {
            uint64_t c[256];
            for (int b = 0; b < 256; ++b) {
                uint64_t v = 0;
                for (uint32_t q = 0; q < dev::kHistCopies; ++q) v += h[(r * dev::kHistCopies + q) * 256 + b];
                c[b] = v;
                bc[b] += v;
            }
            parts[r] = ByteWeights::from_counts(c);
        }
        if (!parts.empty()) {
            ByteWeights part = parts.back();  // weights.rs:293-319: w = W_last; w += W_0 .. W_{T-2}
            for (size_t r = 0; r + 1 < parts.size(); ++r) part.add(parts[r]);
            bw.add(part);
        }
        return Status::ok();
    };
    for (size_t k = 0; k < nblocks; ++k) {
        Slot& sl = slots[k % 2];
        if (k >= 2) HUFF_TRY(merge(k - 2));  // frees the slot's results
        const size_t n = block_len(k);
        HUFF_TRY(load_block(ctx, up.s, sl, in.f, n, src));
        HUFF_TRY(sl.dres.ensure(rows_bytes));
        HIP_TRY_RT(hipMemsetAsync(sl.dres.p, 0, rows_bytes, ctx->stream));
        const auto rations = ration_bounds(n, kRations);
        const uint8_t* d = static_cast<const uint8_t*>(sl.din.p);
        for (size_t r = 0; r < rations.size(); ++r) {
            const size_t lo = rations[r].first, hi = rations[r].second;
            if (hi == lo) continue;
            const size_t abase = lo & ~size_t(15);
            const uint32_t nch = static_cast<uint32_t>((hi - abase + dev::kChunk - 1) / dev::kChunk);
            HIP_TRY_RT(dev::launch_hist(d + abase, lo - abase, hi - abase, nch, nullptr,
                                        static_cast<unsigned long long*>(sl.dres.p) + r * dev::kHistCopies * 256,
                                        ctx->stream));
        }
        HUFF_TRY(fetch_results(ctx, sl, rows_bytes));
    }
    for (size_t k = nblocks >= 2 ? nblocks - 2 : 0; k < nblocks; ++k) HUFF_TRY(merge(k));
    auto tree = std::make_unique<huff_tree>();
    HUFF_TRY(HuffTree::from_weights(bw, tree->t));
    const EncTables& et = tree->enc_tables();

    // header
    std::vector<uint8_t> tbits = tree->t.as_bin();
    const uint8_t tree_pad = calc_padding_bits(tbits.size());
    std::vector<uint8_t> tbytes = pack_msb0(tbits);
    const uint32_t tl = static_cast<uint32_t>(tbytes.size());
    const uint8_t hdr[5] = {0, static_cast<uint8_t>(tl >> 24), static_cast<uint8_t>(tl >> 16),
                            static_cast<uint8_t>(tl >> 8), static_cast<uint8_t>(tl)};
    if (fwrite(hdr, 1, 5, out.f) != 5 || fwrite(tbytes.data(), 1, tbytes.size(), out.f) != tbytes.size())
        return io_err("failed to write", dst);

    // pass 2 (compress_to_writer): every block's size and padding follow from
    // its pass-1 counts, so the blocks pack back to back without a host wait;
    // block k is stitched onto block k-1 exactly as the reference does
    // (huff/src/comp.rs:196-201, utils.rs:2-25: when the previous block left
    // padding q != 0 its bytes are shifted to start at bit q of the previous
    // last byte, that byte is OR-ed in and the writer steps back one byte)
    if (fseek(in.f, 0, SEEK_SET) != 0) return io_err("cannot seek", src);
    std::vector<uint8_t> qs(nblocks), pads(nblocks);
    std::vector<uint64_t> nbits(nblocks);
    uint8_t prev_padding = 0, prev_byte = 0;
    for (size_t k = 0; k < nblocks; ++k) {
        uint64_t b = 0;
        for (int i = 0; i < 256; ++i) b += block_counts[k][i] * et.len[i];
        nbits[k] = b;
        qs[k] = prev_padding;
        pads[k] = calc_padding_bits(b);
        prev_padding = pads[k];
    }
    auto emit = [&](size_t k) -> Status {  // block k's bytes, once copied back
        Slot& sl = slots[k % 2];
        HUFF_TRY(sync_event(sl.done));
        const uint64_t L = (nbits[k] + 7) / 8;
        const uint64_t packed_bytes = (qs[k] + nbits[k] + 7) / 8;
        // offset_bytes re-emits all 8L bits of the block (its zero padding too)
        std::vector<uint8_t> comp(qs[k] ? L + 1 : L, 0);
        if (packed_bytes) std::memcpy(comp.data(), sl.res.p, packed_bytes);
        if (qs[k] != 0) {
            if (fseek(out.f, -1, SEEK_CUR) != 0) return io_err("cannot seek", dst);
            comp[0] |= prev_byte;
        }
        if (!comp.empty() && fwrite(comp.data(), 1, comp.size(), out.f) != comp.size())
            return io_err("failed to write", dst);
        if (!comp.empty()) prev_byte = comp.back();
        return Status::ok();
    };
    for (size_t k = 0; k < nblocks; ++k) {
        Slot& sl = slots[k % 2];
        if (k >= 2) HUFF_TRY(emit(k - 2));
        const size_t n = block_len(k);
        HUFF_TRY(load_block(ctx, up.s, sl, in.f, n, src));
        const uint64_t packed_bytes = (qs[k] + nbits[k] + 7) / 8;
        HUFF_TRY(sl.dres.ensure(packed_bytes + 16));
        HUFF_TRY(sl.job.init(ctx, static_cast<const uint8_t*>(sl.din.p), n));
        HUFF_TRY(sl.job.hist_known(block_counts[k].data()));
        uint64_t bits = 0;
        HUFF_TRY(sl.job.pack(tree.get(), qs[k], nullptr, 0, static_cast<uint8_t*>(sl.dres.p), packed_bytes, &bits));
        HUFF_TRY(fetch_results(ctx, sl, packed_bytes));
    }
    for (size_t k = nblocks >= 2 ? nblocks - 2 : 0; k < nblocks; ++k) HUFF_TRY(emit(k));
    if (fseek(out.f, 0, SEEK_SET) != 0) return io_err("cannot seek", dst);
    const uint8_t pb = static_cast<uint8_t>((tree_pad << 4) + prev_padding);
    if (fwrite(&pb, 1, 1, out.f) != 1) return io_err("failed to write", dst);
    return Status::ok();
}

// decompress in windows of the payload (at most kWindow compressed bytes on
// the host and the device at a time): window k decodes every complete code of
// its bits; the next window starts at the first bit after its last complete
// code (realigned on the GPU when that bit is inside a byte), so the walk
// state carries across windows as the reference carries it across its blocks
// (huff/src/comp.rs:232-280). The next window's bytes are read while the GPU
// decodes this one; the symbols are written as each window finishes.
Status file_decompress(huff_ctx* ctx, const char* src, const char* dst, size_t block_size) {
    if (block_size == 0) return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
    File in;
    in.f = fopen(src, "rb");
    if (!in.f) return io_err("cannot open", src);
    struct stat stt;
    if (fstat(fileno(in.f), &stt) != 0) return io_err("cannot stat", src);
    const size_t total = static_cast<size_t>(stt.st_size);
    const std::string q = std::string("\"") + src + "\"";
    // take(5).read(buf): at most min(5, block_size) bytes (huff/src/comp.rs:93-100)
    if (std::min<size_t>(std::min<size_t>(total, 5), block_size) < 5)
        return Status::err(HUFF_E_MISSING_HEADER, q + " too short to decompress, missing header information");
    uint8_t hdr[5];
    HUFF_TRY(read_exact(in.f, hdr, 5, src));
    const uint8_t tree_pad = hdr[0] >> 4, data_pad = hdr[0] & 0x0F;
    if (tree_pad > 7 || data_pad > 7) return Status::err(HUFF_E_INVALID_HEADER, q + " stores invalid header information");
    const size_t tree_len = (static_cast<size_t>(hdr[1]) << 24) | (static_cast<size_t>(hdr[2]) << 16) |
                            (static_cast<size_t>(hdr[3]) << 8) | hdr[4];
    if (std::min<size_t>(std::min(tree_len, total - 5), block_size) < tree_len)
        return Status::err(HUFF_E_MISSING_HEADER, q + " too short to decompress, missing header information");
    std::vector<uint8_t> tb(tree_len);
    HUFF_TRY(read_exact(in.f, tb.data(), tree_len, src));
    size_t nbits = tree_len * 8;
    nbits = tree_pad > nbits ? 0 : nbits - tree_pad;
    auto tree = std::make_unique<huff_tree>();
    if (HuffTree::try_from_bin(unpack_msb0(tb.data(), nbits), tree->t))
        return Status::err(HUFF_E_INVALID_HEADER, q + " stores invalid header information");
    const size_t plen = total - 5 - tree_len;
    File out;
    out.f = fopen(dst, "wb");
    if (!out.f) return io_err("cannot create", dst);
    if (plen == 0) return Status::ok();
    const bool honour_pad = (plen % block_size) != 0;
    const uint64_t valid_bits = static_cast<uint64_t>(plen) * 8 - (honour_pad ? data_pad : 0);
    HUFF_TRY(ctx->activate());

    // a window holds at most kWindow bytes; the next one starts at most
    // kCarry bytes before its predecessor's end (a code is <= 255 bits), so
    // the bytes [end - kCarry, end) are kept and the rest is read ahead
    // (HUFF_FILE_WINDOW=<bytes> shrinks the window, for tests of the carry)
    size_t kWindow = size_t(256) << 20;
    if (const char* e = getenv("HUFF_FILE_WINDOW")) {
        const unsigned long long v = strtoull(e, nullptr, 10);
        if (v >= 256) kWindow = static_cast<size_t>(v);
    }
    constexpr size_t kCarry = 64;
    const size_t W = std::min(plen, kWindow);
    PinnedBuf buf[2];  // payload bytes [base_i, base_i + len_i)
    size_t base[2] = {0, 0}, len[2] = {0, 0};
    DevBuf d_win, d_shift, d_sym, d_endv;
    HUFF_TRY(d_win.ensure(W + kCarry + 16));
    HUFF_TRY(d_shift.ensure(W + kCarry + 16));
    HUFF_TRY(d_endv.ensure(8));
    auto read_at = [&](int i, size_t off) -> Status {  // payload bytes [off, off + W) into buf[i]
        HUFF_TRY(buf[i].ensure(W + kCarry + 16));
        base[i] = off;
        len[i] = std::min(W, plen - off);
        if (fseek(in.f, static_cast<long>(5 + tree_len + off), SEEK_SET) != 0) return io_err("cannot seek", src);
        return read_exact(in.f, static_cast<uint8_t*>(buf[i].p), len[i], src);
    };
    HUFF_TRY(read_at(0, 0));
    uint64_t pos = 0;  // payload bit of the next code
    int cur = 0;
    std::vector<uint8_t> sym;
    while (pos < valid_bits) {
        const size_t b0 = static_cast<size_t>(pos / 8);
        const uint32_t r = static_cast<uint32_t>(pos % 8);
        if (b0 < base[cur] || b0 >= base[cur] + len[cur]) HUFF_TRY(read_at(cur, b0));
        const size_t nb = base[cur] + len[cur] - b0;  // window bytes from b0
        const bool last = base[cur] + len[cur] == plen;
        HIP_TRY_RT(hipMemcpyAsync(d_win.p, static_cast<uint8_t*>(buf[cur].p) + (b0 - base[cur]), nb,
                                  hipMemcpyHostToDevice, ctx->stream));
        const uint8_t* dwin = static_cast<const uint8_t*>(d_win.p);
        if (r) {  // the window's first code starts inside its first byte
            HIP_TRY_RT(dev::launch_shift_bits(dwin, static_cast<uint8_t*>(d_shift.p), nb, r, ctx->stream));
            dwin = static_cast<const uint8_t*>(d_shift.p);
        }
        const uint64_t wbits = last ? valid_bits - pos : static_cast<uint64_t>(nb) * 8 - r;
        // read the next window's bytes ahead (from kCarry before this one's end)
        // while the GPU decodes: the host buffer being read is the other one
        const int nxt = cur ^ 1;
        uint64_t n = 0;
        HUFF_TRY(decode_indexless_dev(ctx, dwin, nb, wbits, tree.get(), d_sym, &n, nullptr, 0,
                                      static_cast<unsigned long long*>(d_endv.p)));
        if (!last) {
            const size_t ahead = base[cur] + len[cur] - kCarry;
            if (base[nxt] != ahead || len[nxt] == 0) HUFF_TRY(read_at(nxt, ahead));
        }
        uint64_t wend = 0;
        HIP_TRY_RT(hipMemcpyAsync(&wend, d_endv.p, 8, hipMemcpyDeviceToHost, ctx->stream));
        sym.resize(n);
        if (n) HIP_TRY_RT(hipMemcpyAsync(sym.data(), d_sym.p, n, hipMemcpyDeviceToHost, ctx->stream));
        HUFF_TRY(ctx->sync());
        if (n && fwrite(sym.data(), 1, n, out.f) != n) return io_err("failed to write", dst);
        if (last) break;
        if (wend == 0) return Status::err(HUFF_E_CORRUPT, "no complete code in a window of the stream");
        pos += wend;
        cur = nxt;
    }
    return Status::ok();
}

}  // namespace huff
