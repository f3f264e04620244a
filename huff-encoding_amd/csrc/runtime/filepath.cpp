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
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <array>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>

#include "runtime.hpp"

namespace huff {

namespace {

// a descriptor with its own offset. Reads of 16 MiB and more are split over
// up to kIoThreads threads (pread at disjoint offsets): one thread moves a few
// GB/s from the page cache, well below what the GPU and PCIe sustain
struct File {
    int fd = -1;
    uint64_t pos = 0;
    ~File() {
        if (fd >= 0) close(fd);
    }
};

// HUFF_FILE_TRACE=1: seconds in reads, writes and GPU waits per call, on stderr
struct IoClock {
    double read = 0, write = 0, wait = 0, open = 0;
    bool on = false;
};
thread_local IoClock io_clock;

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Tick {
    double& acc;
    double t0 = now_s();
    explicit Tick(double& a) : acc(a) {}
    ~Tick() { acc += now_s() - t0; }
};

void trace_begin() {
    io_clock = IoClock{};
    const char* e = getenv("HUFF_FILE_TRACE");
    io_clock.on = e && *e == '1';
}

void trace_end(const char* what, double t0) {
    if (io_clock.on)
        fprintf(stderr, "[huff file] %s: %.1f ms (open %.1f, read %.1f, write %.1f, gpu wait %.1f)\n", what,
                (now_s() - t0) * 1e3, io_clock.open * 1e3, io_clock.read * 1e3, io_clock.write * 1e3,
                io_clock.wait * 1e3);
}

constexpr size_t kIoThreads = 8;
constexpr size_t kIoPart = size_t(8) << 20;

bool pio_one(bool wr, int fd, uint8_t* buf, size_t n, uint64_t off) {
    for (size_t lo = 0; lo < n;) {
        const ssize_t r = wr ? pwrite(fd, buf + lo, n - lo, static_cast<off_t>(off + lo))
                             : pread(fd, buf + lo, n - lo, static_cast<off_t>(off + lo));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        lo += static_cast<size_t>(r);
    }
    return true;
}

bool pio(bool wr, int fd, uint8_t* buf, size_t n, uint64_t off) {
    auto range = [=](size_t lo, size_t hi) { return pio_one(wr, fd, buf + lo, hi - lo, off + lo); };
    const size_t T = std::min(kIoThreads, n / kIoPart);
    if (T <= 1) return range(0, n);
    std::atomic<bool> ok{true};
    std::vector<std::thread> th;
    const size_t step = (n / T + 4095) & ~size_t(4095);
    for (size_t t = 1; t < T; ++t) {
        const size_t lo = std::min(n, t * step), hi = std::min(n, (t + 1) * step);
        th.emplace_back([&, lo, hi] {
            if (!range(lo, hi)) ok = false;
        });
    }
    if (!range(0, std::min(n, step))) ok = false;
    for (auto& x : th) x.join();
    return ok;
}

Status io_err(const std::string& what, const char* path) {
    return Status::err(HUFF_E_IO, what + " " + path);
}

Status read_exact(File& f, uint8_t* dst, size_t n, const char* path) {
    Tick t(io_clock.read);
    if (n && !pio(false, f.fd, dst, n, f.pos)) return io_err("failed to read", path);
    f.pos += n;
    return Status::ok();
}

// (writes stay on one thread: writers of one file serialise on its inode)
Status write_all(File& f, const void* src, size_t n, const char* path) {
    Tick t(io_clock.write);
    if (n && !pio_one(true, f.fd, static_cast<uint8_t*>(const_cast<void*>(src)), n, f.pos))
        return io_err("failed to write", path);
    f.pos += n;
    return Status::ok();
}

// One writer thread per call: writes run in submission order (a block's
// first byte may overwrite the previous block's last one) while the calling
// thread reads, uploads and waits on the GPU — on this path the page-cache
// writes are the largest host cost. Large writes point at pinned buffers the
// caller keeps until their ticket completes; small ones are copied.
class AsyncWriter {
public:
    AsyncWriter(int fd, const char* path) : fd_(fd), path_(path), th_([this] { run(); }) {}
    ~AsyncWriter() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    // a ticket: wait(ticket) returns once this write is on the file
    uint64_t submit(const void* p, size_t n, uint64_t off) {
        Job j{static_cast<const uint8_t*>(p), n, off, {}};
        if (n <= 4096) {  // small: copied (headers, pad bytes)
            j.copy.assign(j.p, j.p + n);
            j.p = j.copy.data();
        }
        std::lock_guard<std::mutex> g(m_);
        q_.push_back(std::move(j));
        ++submitted_;
        cv_.notify_all();
        return submitted_;
    }
    Status wait(uint64_t ticket) {
        Tick t(io_clock.write);
        std::unique_lock<std::mutex> g(m_);
        done_cv_.wait(g, [&] { return completed_ >= ticket || failed_; });
        if (failed_) return io_err("failed to write", path_);
        return Status::ok();
    }
    Status drain() { return wait(submitted_snapshot()); }

private:
    struct Job {
        const uint8_t* p;
        size_t n;
        uint64_t off;
        std::vector<uint8_t> copy;
    };
    uint64_t submitted_snapshot() {
        std::lock_guard<std::mutex> g(m_);
        return submitted_;
    }
    void run() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;  // stop requested and nothing left
                j = std::move(q_.front());
                q_.pop_front();
            }
            const bool ok = failed_ || !j.n || pio_one(true, fd_, const_cast<uint8_t*>(j.p), j.n, j.off);
            {
                std::lock_guard<std::mutex> g(m_);
                if (!ok) failed_ = true;
                ++completed_;
            }
            done_cv_.notify_all();
        }
    }
    int fd_;
    const char* path_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::deque<Job> q_;
    uint64_t submitted_ = 0, completed_ = 0;
    bool stop_ = false, failed_ = false;
    std::thread th_;  // last: started once the members above exist
};

// The file moves through pieces of at most kPiece bytes (a block longer than
// that is split; a piece never spans two blocks). One piece's buffers: pinned
// host bytes (the fread target and H2D source), the piece on the device,
// results on the device and back in pinned memory. Two slots alternate, so
// the host reads piece i+1 and writes piece i-1 while the GPU works on piece
// i; uploads run on a stream of their own, downloads on the copy stream.
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
    Tick t(io_clock.wait);
    HIP_TRY_RT(hipEventSynchronize(e));
    return Status::ok();
}

// HUFF_FILE_PIECE / HUFF_FILE_WINDOW=<bytes> shrink the pieces / windows (tests
// of the piece and window seams)
size_t env_size(const char* name, size_t dflt, size_t lo) {
    if (const char* e = getenv(name)) {
        const unsigned long long v = strtoull(e, nullptr, 10);
        if (v >= lo) return static_cast<size_t>(v);
    }
    return dflt;
}

}  // namespace

struct FileWs {
    Slot slots[2];
    hipStream_t up = nullptr;  // uploads
    // decompress: payload windows (pinned), the window on the device (and
    // realigned), the symbols on the device and in pinned memory
    PinnedBuf win[2], sym[3];
    PinnedBuf rres[3];  // compress pass 2: piece results, written out asynchronously
    DevBuf d_win, d_shift, d_sym, d_end;
    PinnedBuf end;
    ~FileWs() {
        if (up) {
            hipStreamSynchronize(up);
            hipStreamDestroy(up);
        }
    }
};

namespace {

Status file_ws(huff_ctx* ctx, FileWs** out) {
    if (!ctx->file_ws) {
        auto ws = std::make_shared<FileWs>();
        for (Slot& sl : ws->slots) HUFF_TRY(sl.init());
        HIP_TRY_RT(hipStreamCreateWithFlags(&ws->up, hipStreamNonBlocking));
        ctx->file_ws = ws;
    }
    *out = ctx->file_ws.get();
    return Status::ok();
}

// fread piece bytes into the slot (once its previous upload has left it),
// then upload them on the upload stream; the compute stream waits for them
Status load_piece(huff_ctx* ctx, hipStream_t up, Slot& sl, File& f, size_t n, const char* path) {
    HUFF_TRY(sync_event(sl.h2d));
    HUFF_TRY(sl.in.ensure(n + 16));
    HUFF_TRY(read_exact(f, static_cast<uint8_t*>(sl.in.p), n, path));
    HUFF_TRY(sl.din.ensure(n + 16));
    if (n) HIP_TRY_RT(hipMemcpyAsync(sl.din.p, sl.in.p, n, hipMemcpyHostToDevice, up));
    HIP_TRY_RT(hipEventRecord(sl.h2d, up));
    HIP_TRY_RT(hipStreamWaitEvent(ctx->stream, sl.h2d, 0));
    return Status::ok();
}

// the piece's results, once its kernels are done, back to pinned memory on
// the copy stream
Status fetch_results(huff_ctx* ctx, Slot& sl, size_t bytes, PinnedBuf* to = nullptr) {
    PinnedBuf& res = to ? *to : sl.res;
    HUFF_TRY(res.ensure(bytes + 16));
    HIP_TRY_RT(hipEventRecord(sl.kern, ctx->stream));
    HIP_TRY_RT(hipStreamWaitEvent(ctx->copy_stream, sl.kern, 0));
    if (bytes) HIP_TRY_RT(hipMemcpyAsync(res.p, sl.dres.p, bytes, hipMemcpyDeviceToHost, ctx->copy_stream));
    HIP_TRY_RT(hipEventRecord(sl.done, ctx->copy_stream));
    return Status::ok();
}

struct Piece {
    size_t block, lo, len;  // bytes [lo, lo + len) of block `block`
    bool first, last;       // first / last piece of its block
    std::vector<uint32_t> rations;  // pass 1: rations met, one histogram row each
    std::array<uint64_t, 256> counts{};
    uint8_t tail[8] = {};  // the piece's last bytes (pass 2's prev_tail for the next piece)
    uint32_t tail_len = 0;
    uint64_t off = 0, bits = 0;  // pass 2: first bit within the block's output, code bits
};

}  // namespace

static Status file_compress_impl(huff_ctx* ctx, const char* src, const char* dst, size_t block_size) {
    if (block_size == 0) return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
    File in;
    in.fd = open(src, O_RDONLY);
    if (in.fd < 0) return io_err("cannot open", src);
    struct stat stt;
    if (fstat(in.fd, &stt) != 0) return io_err("cannot stat", src);
    if (S_ISDIR(stt.st_mode)) return Status::err(HUFF_E_IO, std::string(src) + " is a directory");
    const size_t total = static_cast<size_t>(stt.st_size);
    File out;
    {
        Tick t(io_clock.open);
        out.fd = open(dst, O_RDWR | O_CREAT | O_TRUNC, 0666);
    }
    if (out.fd < 0) return io_err("cannot create", dst);
    HUFF_TRY(ctx->activate());
    FileWs* ws = nullptr;
    HUFF_TRY(file_ws(ctx, &ws));
    Slot* slots = ws->slots;
    const size_t nblocks = (total + block_size - 1) / block_size;
    auto block_len = [&](size_t k) { return std::min(block_size, total - k * block_size); };
    const size_t kPiece = env_size("HUFF_FILE_PIECE", size_t(64) << 20, 4096);
    std::vector<Piece> pieces;
    for (size_t k = 0; k < nblocks; ++k) {
        const size_t n = block_len(k);
        for (size_t lo = 0; lo < n; lo += kPiece) {
            Piece p;
            p.block = k;
            p.lo = lo;
            p.len = std::min(kPiece, n - lo);
            p.first = lo == 0;
            p.last = lo + p.len == n;
            pieces.push_back(std::move(p));
        }
    }
    const size_t np = pieces.size();

    // pass 1 (huff_tree_from_reader, huff/src/comp.rs:161-172): per block
    // ByteWeights::threaded_from_bytes(block, 12), merged into the running
    // weights in block order. Each piece histograms its share of every ration
    // it meets (one GPU row each); the rows add up to the rations' counts and
    // to the piece's own counts, which size pass 2's pieces
    constexpr size_t kRations = 12;
    const size_t row_bytes = dev::kHistCopies * 256 * 8;
    ByteWeights bw;
    std::vector<std::array<uint64_t, 256>> block_counts(nblocks);
    std::array<std::array<uint64_t, 256>, kRations> racc{};
    auto merge = [&](size_t i) -> Status {  // piece i's rows, once copied back
        Slot& sl = slots[i % 2];
        Piece& p = pieces[i];
        HUFF_TRY(sync_event(sl.done));
        const uint64_t* h = static_cast<const uint64_t*>(sl.res.p);
        for (size_t j = 0; j < p.rations.size(); ++j) {
            auto& acc = racc[p.rations[j]];
            for (int b = 0; b < 256; ++b) {
                uint64_t v = 0;
                for (uint32_t q = 0; q < dev::kHistCopies; ++q) v += h[(j * dev::kHistCopies + q) * 256 + b];
                acc[b] += v;
                p.counts[b] += v;
            }
        }
        if (p.last) {  // the block's rations are complete
            const auto rations = ration_bounds(block_len(p.block), kRations);
            auto& bc = block_counts[p.block];
            bc.fill(0);
            std::vector<ByteWeights> parts(rations.size());
            for (size_t r = 0; r < rations.size(); ++r) {
                for (int b = 0; b < 256; ++b) bc[b] += racc[r][b];
                parts[r] = ByteWeights::from_counts(racc[r].data());
                racc[r].fill(0);
            }
            if (!parts.empty()) {
                ByteWeights part = parts.back();  // weights.rs:293-319: w = W_last; w += W_0 .. W_{T-2}
                for (size_t r = 0; r + 1 < parts.size(); ++r) part.add(parts[r]);
                bw.add(part);
            }
        }
        return Status::ok();
    };
    for (size_t i = 0; i < np; ++i) {
        Slot& sl = slots[i % 2];
        Piece& p = pieces[i];
        if (i >= 2) HUFF_TRY(merge(i - 2));  // frees the slot's results
        HUFF_TRY(load_piece(ctx, ws->up, sl, in, p.len, src));
        p.tail_len = static_cast<uint32_t>(std::min<size_t>(8, p.len));
        std::memcpy(p.tail, static_cast<const uint8_t*>(sl.in.p) + p.len - p.tail_len, p.tail_len);
        const auto rations = ration_bounds(block_len(p.block), kRations);
        for (size_t r = 0; r < rations.size(); ++r) {
            const size_t lo = std::max(rations[r].first, p.lo), hi = std::min(rations[r].second, p.lo + p.len);
            if (hi > lo) p.rations.push_back(static_cast<uint32_t>(r));
        }
        const size_t used = p.rations.size() * row_bytes;
        HUFF_TRY(sl.dres.ensure(used + 16));
        if (used) HIP_TRY_RT(hipMemsetAsync(sl.dres.p, 0, used, ctx->stream));
        const uint8_t* d = static_cast<const uint8_t*>(sl.din.p);
        for (size_t j = 0; j < p.rations.size(); ++j) {
            const size_t lo = std::max(rations[p.rations[j]].first, p.lo) - p.lo;
            const size_t hi = std::min(rations[p.rations[j]].second, p.lo + p.len) - p.lo;
            const size_t abase = lo & ~size_t(15);
            const uint32_t nch = static_cast<uint32_t>((hi - abase + dev::kChunk - 1) / dev::kChunk);
            HIP_TRY_RT(dev::launch_hist(d + abase, lo - abase, hi - abase, nch, nullptr,
                                        static_cast<unsigned long long*>(sl.dres.p) + j * dev::kHistCopies * 256,
                                        ctx->stream));
        }
        HUFF_TRY(fetch_results(ctx, sl, used));
    }
    for (size_t i = np >= 2 ? np - 2 : 0; i < np; ++i) HUFF_TRY(merge(i));
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
    HUFF_TRY(write_all(out, hdr, 5, dst));
    HUFF_TRY(write_all(out, tbytes.data(), tbytes.size(), dst));

    // pass 2 (compress_to_writer): every block's size and padding, and every
    // piece's first bit, follow from pass 1's counts, so the pieces pack back
    // to back without a host wait. Block k is stitched onto block k-1 exactly
    // as the reference does (huff/src/comp.rs:196-201, utils.rs:2-25: when the
    // previous block left padding q != 0 its bytes are shifted to start at bit
    // q of the previous last byte, that byte is OR-ed in and the writer steps
    // back one byte). Within a block, piece i+1 packs from bit off_i + bits_i
    // with piece i's last letters as prev_tail, so its first byte is whole and
    // piece i writes only its whole bytes
    in.pos = 0;
    std::vector<uint8_t> qs(nblocks);
    std::vector<uint64_t> nbits(nblocks);
    uint8_t prev_padding = 0, prev_byte = 0;
    for (size_t k = 0; k < nblocks; ++k) {
        uint64_t b = 0;
        for (int i = 0; i < 256; ++i) b += block_counts[k][i] * et.len[i];
        nbits[k] = b;
        qs[k] = prev_padding;
        prev_padding = calc_padding_bits(b);
    }
    for (size_t i = 0; i < np; ++i) {
        Piece& p = pieces[i];
        p.off = p.first ? qs[p.block] : pieces[i - 1].off + pieces[i - 1].bits;
        for (int b = 0; b < 256; ++b) p.bits += p.counts[b] * et.len[b];
    }
    AsyncWriter writer(out.fd, dst);
    uint64_t ticket[3] = {0, 0, 0};  // the write of the piece whose results sit in rres[i % 3]
    auto emit = [&](size_t i) -> Status {  // piece i's bytes, once copied back
        Slot& sl = slots[i % 2];
        const Piece& p = pieces[i];
        HUFF_TRY(sync_event(sl.done));
        uint8_t* r = static_cast<uint8_t*>(ws->rres[i % 3].p);
        const uint64_t packed = ((p.off & 7) + p.bits + 7) / 8;
        const uint64_t q = qs[p.block];
        if (p.first && q != 0) {
            --out.pos;  // the header precedes every block
            r[0] |= prev_byte;
        }
        const uint64_t whole = p.last ? packed : ((p.off & 7) + p.bits) / 8;
        if (p.last) {  // read before the buffer is handed to the writer
            const uint64_t L = (nbits[p.block] + 7) / 8;
            const uint64_t size = q ? L + 1 : L, written = (q + nbits[p.block] + 7) / 8;
            if (size) prev_byte = size > written ? 0 : r[packed - 1];
        }
        ticket[i % 3] = writer.submit(r, whole, out.pos);
        out.pos += whole;
        if (p.last) {
            // offset_bytes re-emits all 8L bits of the block (its zero
            // padding too): the block is L bytes, L + 1 when q != 0
            const uint64_t L = (nbits[p.block] + 7) / 8;
            const uint64_t size = q ? L + 1 : L, written = (q + nbits[p.block] + 7) / 8;
            static const uint8_t zeros[2] = {};  // size - written <= 1
            if (size > written) writer.submit(zeros, size - written, out.pos);
            out.pos += size - written;
        }
        return Status::ok();
    };
    for (size_t i = 0; i < np; ++i) {
        Slot& sl = slots[i % 2];
        const Piece& p = pieces[i];
        if (i >= 2) HUFF_TRY(emit(i - 2));
        HUFF_TRY(load_piece(ctx, ws->up, sl, in, p.len, src));
        const uint64_t packed = ((p.off & 7) + p.bits + 7) / 8;
        HUFF_TRY(sl.dres.ensure(packed + 16));
        HUFF_TRY(sl.job.init(ctx, static_cast<const uint8_t*>(sl.din.p), p.len));
        HUFF_TRY(sl.job.hist_known(p.counts.data()));
        const Piece* prev = p.first ? nullptr : &pieces[i - 1];
        uint64_t bits = 0;
        HUFF_TRY(sl.job.pack(tree.get(), p.off, prev ? prev->tail : nullptr, prev ? prev->tail_len : 0,
                             static_cast<uint8_t*>(sl.dres.p), packed, &bits));
        if (ticket[i % 3]) HUFF_TRY(writer.wait(ticket[i % 3]));  // piece i - 3's bytes are out
        HUFF_TRY(fetch_results(ctx, sl, packed, &ws->rres[i % 3]));
    }
    for (size_t i = np >= 2 ? np - 2 : 0; i < np; ++i) HUFF_TRY(emit(i));
    const uint8_t pb = static_cast<uint8_t>((tree_pad << 4) + prev_padding);
    writer.submit(&pb, 1, 0);
    return writer.drain();
}

// decompress in windows of the payload (at most kWindow compressed bytes at a
// time): window k decodes every complete code of its bits; the next window
// starts at the first bit after its last complete code (realigned on the GPU
// when that bit is inside a byte), so the walk state carries across windows
// as the reference carries it across its blocks (huff/src/comp.rs:232-280).
// While the GPU decodes window k the host writes window k-1's symbols and
// reads window k+1's bytes.
static Status file_decompress_impl(huff_ctx* ctx, const char* src, const char* dst, size_t block_size) {
    if (block_size == 0) return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
    File in;
    in.fd = open(src, O_RDONLY);
    if (in.fd < 0) return io_err("cannot open", src);
    struct stat stt;
    if (fstat(in.fd, &stt) != 0) return io_err("cannot stat", src);
    const size_t total = static_cast<size_t>(stt.st_size);
    const std::string q = std::string("\"") + src + "\"";
    // take(5).read(buf): at most min(5, block_size) bytes (huff/src/comp.rs:93-100)
    if (std::min<size_t>(std::min<size_t>(total, 5), block_size) < 5)
        return Status::err(HUFF_E_MISSING_HEADER, q + " too short to decompress, missing header information");
    uint8_t hdr[5];
    HUFF_TRY(read_exact(in, hdr, 5, src));
    const uint8_t tree_pad = hdr[0] >> 4, data_pad = hdr[0] & 0x0F;
    if (tree_pad > 7 || data_pad > 7) return Status::err(HUFF_E_INVALID_HEADER, q + " stores invalid header information");
    const size_t tree_len = (static_cast<size_t>(hdr[1]) << 24) | (static_cast<size_t>(hdr[2]) << 16) |
                            (static_cast<size_t>(hdr[3]) << 8) | hdr[4];
    if (std::min<size_t>(std::min(tree_len, total - 5), block_size) < tree_len)
        return Status::err(HUFF_E_MISSING_HEADER, q + " too short to decompress, missing header information");
    std::vector<uint8_t> tb(tree_len);
    HUFF_TRY(read_exact(in, tb.data(), tree_len, src));
    size_t nbits = tree_len * 8;
    nbits = tree_pad > nbits ? 0 : nbits - tree_pad;
    auto tree = std::make_unique<huff_tree>();
    if (HuffTree::try_from_bin(unpack_msb0(tb.data(), nbits), tree->t))
        return Status::err(HUFF_E_INVALID_HEADER, q + " stores invalid header information");
    const size_t plen = total - 5 - tree_len;
    File out;
    {
        Tick t(io_clock.open);
        out.fd = open(dst, O_WRONLY | O_CREAT | O_TRUNC, 0666);
    }
    if (out.fd < 0) return io_err("cannot create", dst);
    if (plen == 0) return Status::ok();
    const bool honour_pad = (plen % block_size) != 0;
    const uint64_t valid_bits = static_cast<uint64_t>(plen) * 8 - (honour_pad ? data_pad : 0);
    HUFF_TRY(ctx->activate());
    FileWs* ws = nullptr;
    HUFF_TRY(file_ws(ctx, &ws));

    // a window holds at most kWindow bytes; the next one starts at most
    // kCarry bytes before its predecessor's end (a code is <= 255 bits), so
    // it is read ahead from there
    const size_t kWindow = env_size("HUFF_FILE_WINDOW", size_t(64) << 20, 256);
    constexpr size_t kCarry = 64;
    const size_t W = std::min(plen, kWindow);
    size_t base[2] = {0, 0}, len[2] = {0, 0};  // payload bytes [base_i, base_i + len_i) in win[i]
    HUFF_TRY(ws->d_win.ensure(W + kCarry + 16));
    HUFF_TRY(ws->d_shift.ensure(W + kCarry + 16));
    HUFF_TRY(ws->d_end.ensure(8));
    HUFF_TRY(ws->end.ensure(8));
    auto read_at = [&](int i, size_t off) -> Status {  // payload bytes [off, off + W) into win[i]
        HUFF_TRY(ws->win[i].ensure(W + kCarry + 16));
        base[i] = off;
        len[i] = std::min(W, plen - off);
        in.pos = 5 + tree_len + off;
        return read_exact(in, static_cast<uint8_t*>(ws->win[i].p), len[i], src);
    };
    AsyncWriter writer(out.fd, dst);
    uint64_t ticket[3] = {0, 0, 0};  // the write of the window whose letters sit in sym[k % 3]
    HUFF_TRY(read_at(0, 0));
    uint64_t pos = 0;  // payload bit of the next code
    int cur = 0, k = 0;
    while (pos < valid_bits) {
        const size_t b0 = static_cast<size_t>(pos / 8);
        const uint32_t r = static_cast<uint32_t>(pos % 8);
        if (b0 < base[cur] || b0 >= base[cur] + len[cur]) HUFF_TRY(read_at(cur, b0));
        const size_t nb = base[cur] + len[cur] - b0;  // window bytes from b0
        const bool last = base[cur] + len[cur] == plen;
        HIP_TRY_RT(hipMemcpyAsync(ws->d_win.p, static_cast<uint8_t*>(ws->win[cur].p) + (b0 - base[cur]), nb,
                                  hipMemcpyHostToDevice, ctx->stream));
        const uint8_t* dwin = static_cast<const uint8_t*>(ws->d_win.p);
        if (r) {  // the window's first code starts inside its first byte
            HIP_TRY_RT(dev::launch_shift_bits(dwin, static_cast<uint8_t*>(ws->d_shift.p), nb, r, ctx->stream));
            dwin = static_cast<const uint8_t*>(ws->d_shift.p);
        }
        const uint64_t wbits = last ? valid_bits - pos : static_cast<uint64_t>(nb) * 8 - r;
        uint64_t n = 0;
        HUFF_TRY(decode_indexless_dev(ctx, dwin, nb, wbits, tree.get(), ws->d_sym, &n, nullptr, 0,
                                      static_cast<unsigned long long*>(ws->d_end.p)));
        const int so = k % 3;
        if (ticket[so]) HUFF_TRY(writer.wait(ticket[so]));  // window k - 3's letters are out
        HUFF_TRY(ws->sym[so].ensure(n + 16));
        if (n) HIP_TRY_RT(hipMemcpyAsync(ws->sym[so].p, ws->d_sym.p, n, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY_RT(hipMemcpyAsync(ws->end.p, ws->d_end.p, 8, hipMemcpyDeviceToHost, ctx->stream));
        // beside the GPU (and the writer): the next window's bytes in
        const int nxt = cur ^ 1;
        if (!last) {
            const size_t ahead = base[cur] + len[cur] - kCarry;
            if (base[nxt] != ahead || len[nxt] == 0) HUFF_TRY(read_at(nxt, ahead));
        }
        {
            Tick t(io_clock.wait);
            HUFF_TRY(ctx->sync());
        }
        ticket[so] = writer.submit(ws->sym[so].p, n, out.pos);
        out.pos += n;
        ++k;
        if (last) break;
        const uint64_t wend = *static_cast<const uint64_t*>(ws->end.p);
        if (wend == 0) return Status::err(HUFF_E_CORRUPT, "no complete code in a window of the stream");
        pos += wend;
        cur = nxt;
    }
    return writer.drain();
}

Status file_compress(huff_ctx* ctx, const char* src, const char* dst, size_t block_size) {
    trace_begin();
    const double t0 = now_s();
    Status st = file_compress_impl(ctx, src, dst, block_size);
    trace_end("compress", t0);
    return st;
}

Status file_decompress(huff_ctx* ctx, const char* src, const char* dst, size_t block_size) {
    trace_begin();
    const double t0 = now_s();
    Status st = file_decompress_impl(ctx, src, dst, block_size);
    trace_end("decompress", t0);
    return st;
}

}  // namespace huff
