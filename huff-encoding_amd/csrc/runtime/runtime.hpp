// runtime.hpp — context, device workspace and the encode/decode pipeline.
//
// huff_ctx owns a HIP stream (or adopts the caller's), pinned staging for the
// tiny host<->device hops of the pipeline (weights down, code tables up) and
// the device staging buffers of the host-pointer API. huff_enc is one encode
// job over bytes already in HBM: hist -> (host) tree -> bits/scan -> pack ->
// decode, exactly the hot path of SURVEY.md §3.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../device/kernels.hpp"
#include "../host/huff_coding.hpp"

namespace huff {

inline Status hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return Status::ok();
    return Status::err(HUFF_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY_RT(expr) HUFF_TRY(::huff::hip_status((expr), #expr))

// Encode/decode tables derived from a tree (built once per tree, cached).
struct EncTables {
    uint64_t code[256];           // codes <= 64 bits (right-aligned); 0 for longer ones
    uint8_t len[256];             // every code's length (0: letter absent)
    uint32_t maxlen = 0;
    bool fits64 = true;
    // maxlen > dev::kLongMaxLen: every code left-aligned in dev::kDeepWords
    // words per letter (deep.hip)
    std::vector<uint32_t> deep;
};

struct DecTables {
    std::vector<uint32_t> lut;  // primary [1 << bits] then 8-bit secondaries
    uint32_t bits = 0;
    uint32_t maxdepth = 0;
    bool all8 = false;          // every leaf at depth 8: decode is a byte map
    // single-symbol u16 table (decode_wave.hip k_decode_fixed), packed two
    // entries per word at word `soff`: [1 << sbits] entries, used | letter << 8,
    // kSsSlow for windows whose first code is longer than sbits
    uint32_t sbits = 0, soff = 0;
    // multi-code walk table (indexless.hip's speculative pass): [1 << sbits]
    // u16 entries at word `woff`: first length | kSsSlow | used << 8 | count << 12
    uint32_t woff = 0;
    // level-2 length table for the sync kernels (codes longer than sbits,
    // <= 32 bits): `l2words` words at word `l2off` = nd u32 descriptors
    // (byte offset of the prefix's entries in this block << 5 | its index
    // bits E) then u8 code lengths; the slow entries of stab and the walk
    // table carry their descriptor index in bits [0, 7) and [8, 16). 0: none
    // l2E > 0: the uniform form instead, no descriptors: every slow window s
    // has 2^l2E lengths at byte s << l2E (l2E = the deepest leaf below any
    // slow window), indexed by the l2E bits after the first sbits; the slow
    // entries carry s the same way
    uint32_t l2off = 0, l2words = 0, l2E = 0;
    // mean code length weighted 2^-len (the Kraft mean: the mean of the
    // single-symbol table's lengths), the one-pass index-free decoder's guess
    // of bits per letter when it sizes its segments (syncdec.hip)
    double kraft_bits = 8.0;
    // the uniform form, and more than 1/64 of the windows slow (a 64-lane
    // step then nearly always has a slow lane)
    bool l2dense = false;
};


// HUFF_DISABLE_FIXED8=1 forces the general kernels even for all-8-bit codes
bool fixed8_disabled();
// HUFF_HOST_TRACE: when huff_enc::pack finished its bit count, started and
// returned from the byte-map launch (this thread's last pack)
struct PackStamps {
    std::chrono::steady_clock::time_point bits, launch, launched;
};
PackStamps& pack_stamps();
// HUFF_SMALL_STAGE=0 keeps the decoders' 4.5 KiB stage for every stream
bool small_stage_enabled();
uint32_t dma_decode_enabled();
// HUFF_DEC_VARIANT=11 -> k_decode_fixed's self-checking build (mode 1; else 0)
uint32_t decode_check_mode();

Status build_dec_tables(const HuffTree& t, DecTables& out);

}  // namespace huff

struct huff_tree {
    huff::HuffTree t;
    uint64_t id;
    mutable std::mutex m;
    mutable std::unique_ptr<huff::EncTables> enc;
    mutable std::unique_ptr<huff::DecTables> dec;
    mutable std::vector<int32_t> up;  // parent links for branch codes (capi_util.hpp parent_links), built once

    huff_tree();
    const huff::EncTables& enc_tables() const;
    huff::Status dec_tables(const huff::DecTables** out) const;
};

// Host-side copy of the encoder's restart index (travels with CompressData).
struct huff_index_host {
    uint64_t n = 0;
    std::vector<uint64_t> chunk_start;  // nchunks + 1
    std::vector<uint32_t> sub_bit;      // ceil(n / kIdx) (byte path), ceil(n / kSub) (wide path)
};

struct huff_compress_data {
    std::vector<uint8_t> comp;
    uint8_t padding = 0;
    huff_tree* tree = nullptr;  // owned clone
    std::unique_ptr<huff_index_host> index;
    ~huff_compress_data();
};

struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;  // last async copy out of/into p
    huff::Status ensure(size_t bytes);
    huff::Status wait();
    ~PinnedBuf();
};

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    huff::Status ensure(size_t bytes);
    void release();
    ~DevBuf() { release(); }
};

namespace huff {
struct IndexlessSync;
struct FileWs;
}

struct huff_wenc;

struct huff_ctx {
    int device = 0;
    int cu_count = 256;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t copy_stream = nullptr;  // table uploads beside the kernels
    hipEvent_t lut_free = nullptr;      // after the last kernel that read d_lut
    PinnedBuf pin_w;     // weights readback: 256 tagged totals written by pass 1
    void* pin_w_dev = nullptr;
    uint64_t hist_seq = 0;
    // a pass 1 queued ahead by huff_enc_hist_launch, not yet waited for: its
    // job and tag (one at a time, as pin_w is the context's)
    const huff_enc* hist_pending = nullptr;
    uint64_t hist_pending_tag = 0;
    PinnedBuf pin_total;  // the index-free decode's symbol count, tagged, written by its scan
    void* pin_total_dev = nullptr;
    uint64_t total_seq = 0;
    PinnedBuf pin_lut;   // decode table upload
    DevBuf d_in, d_out;  // staging of the host-pointer API
    DevBuf d_lut;
    DevBuf d_align;      // aligned decode target for a misaligned output pointer
    DevBuf d_comp_align; // aligned copy of a misaligned index-free input stream
    DevBuf d_err;        // k_decode_fixed self-check record (check builds)
    // index-free decode workspace, kept across calls (per-call allocations
    // of its ~100 MB per GiB of stream cost more than the kernels)
    std::shared_ptr<huff::IndexlessSync> idx_ws;
    DevBuf idx_sub_abs;
    DevBuf idx_mark32, idx_task_seg;  // the index-free decode's compact marks (k_mark_lite)
    DevBuf sd_ws, sd_jobs;            // the one-pass index-free decoder's tile words / control, its tail jobs
    huff::IndexlessSync& indexless_ws();
    // the .hff file path's pinned pieces and device buffers (filepath.cpp),
    // kept across calls: pinning ~0.5 GB per call costs more than the copies
    std::shared_ptr<huff::FileWs> file_ws;
    // the task decoder of index-free wide-letter decodes (wide_rt.cpp), kept
    // so repeated decodes reuse its buffers and uploaded tables
    std::shared_ptr<huff_wenc> wdec_ws;
    uint64_t lut_tree_id = 0;

    // kernel timing
    struct Timed {
        std::string name;
        hipEvent_t a, b;
    };
    bool timing = false;
    std::vector<Timed> pending;
    std::vector<hipEvent_t> free_events;
    std::map<std::string, std::pair<double, uint64_t>> kstats;
    huff::Status timed(const char* name, const std::function<hipError_t()>& launch);
    huff::Status collect_timing();

    huff::Status activate() const;
    // the tree's decode tables, built on the host and queued for upload;
    // for_decode: the upload is skipped when decode() will take the byte-map
    // path, which carries its map in the kernel arguments
    huff::Status upload_dec_tables(const huff_tree* t, const huff::DecTables** dt, bool for_decode = false);
    huff::Status sync();
};

struct huff_enc {
    huff_ctx* ctx = nullptr;
    const uint8_t* d_in = nullptr;
    uint64_t n = 0;
    uint32_t nchunks = 0;
    DevBuf chunk_hist, gw, chunk_bits, chunk_start, tsum, sub_bit, mask, pos;
    DevBuf deep_words;  // codes longer than 57 bits (deep.hip)
    // compact restart index (codes <= 16 bits, pack.hip): u64 per 4,096
    // symbols + u16 per 64, half the bytes of chunk_start + sub_bit;
    // expanded into sub_bit for the consumers that read that
    DevBuf task_base, sub16;
    bool compact_index = false;
    // decode check build (HUFF_DEC_VARIANT=11): the input's letter checksums
    // per decode task, recorded by pack (checksum.hip)
    DevBuf task_sums;
    bool sums_valid = false;
    huff::Status check_sums(const uint8_t* d_out);
    huff::Status expand_index();
    uint64_t w[256] = {};
    bool have_hist = false;
    // state of the last pack (for decode)
    bool packed = false;
    uint64_t packed_tree_id = 0;
    // code lengths and codes of the tree the stream was packed with (or whose
    // index was uploaded): decode refuses a tree with other codes
    uint8_t packed_len[256] = {};
    uint64_t packed_code[256] = {};
    std::vector<uint32_t> packed_deep;  // deep codes' words (EncTables::deep)
    bool packed_any_tree = false;  // an index uploaded without a tree
    void remember_tree(const huff_tree* t);
    bool codes_match(const huff_tree* t) const;
    uint64_t bit_base = 0, total_bits = 0;
    // the byte-map pack leaves the (arithmetic) restart index unwritten
    // until a consumer needs it: decode through a bit decoder, or download
    bool index_pending = false;
    huff::Status ensure_index();

    huff::Status init(huff_ctx* c, const uint8_t* d, uint64_t nbytes);
    huff::Status hist();
    // pass 1 queued on the stream, its weights waited for by the next hist()
    // (huff_enc_hist_launch)
    huff::Status hist_launch();
    huff::Status launch_publish(uint64_t* tag);
    huff::Status wait_weights(uint64_t tag);
    // pass 1 when the counts are already known (the file path's second pass):
    // the per-chunk rows only, no host wait
    huff::Status hist_known(const uint64_t counts[256]);
    // pass 1 without a host wait: weights + tail bytes as a device row (see
    // huff_enc_hist_row); the weights reach the host with the exchanged rows
    huff::Status hist_row(long long* d_row);
    huff::Status bits(const huff_tree* t, uint64_t* total);
    huff::Status pack(const huff_tree* t, uint64_t bit_base, const uint8_t* prev_tail, size_t prev_tail_len,
                      uint8_t* d_out, size_t out_cap, uint64_t* total);
    huff::Status decode(const huff_tree* t, const uint8_t* d_comp, uint64_t comp_bytes, uint8_t* d_out);
    huff::Status download_index(huff_index_host& idx);
    huff::Status upload_index(const huff_index_host& idx);
};

namespace huff {
// host-pointer pipelines used by the C ABI
Status weights_from_host(huff_ctx* ctx, const uint8_t* bytes, size_t n, ByteWeights& out);
Status weights_threaded_from_host(huff_ctx* ctx, const uint8_t* bytes, size_t n, size_t thread_num,
                                  ByteWeights& out);
Status compress_host(huff_ctx* ctx, const uint8_t* bytes, size_t n, const huff_tree* t, huff_compress_data** out);
Status decompress_host(huff_ctx* ctx, const huff_compress_data* cd, uint8_t* out, size_t cap, size_t* out_len);
Status file_compress(huff_ctx* ctx, const char* src, const char* dst, size_t block_size);
Status file_decompress(huff_ctx* ctx, const char* src, const char* dst, size_t block_size);
Status parse_block_size(const char* s, size_t* out);
Status run_checked_decode(huff_ctx* ctx, dev::DecodeArgs& a, const std::function<hipError_t()>& launch);
// decode without a restart index: valid_bits of the stream at d_comp; the
// symbols land in `out` (grown as needed), their count in *nsym
Status decode_indexless_dev(huff_ctx* ctx, const uint8_t* d_comp, uint64_t comp_bytes, uint64_t valid_bits,
                            const huff_tree* t, DevBuf& out, uint64_t* nsym, uint8_t* d_user = nullptr,
                            size_t user_cap = 0, unsigned long long* d_end = nullptr);
// (d_end, device: the bit after the last complete code, for a window of a
// longer stream)
// the self-synchronising part of the index-free decode (spec, fix, scan):
// symbol offsets per segment in `off`, the symbol count in `total`
struct IndexlessSync {
    const DecTables* dt = nullptr;  // tables of the tree, uploaded to ctx->d_lut
    DevBuf s, x0, c, off, flag, tsum, samp, tm, dl, fixlist, chain, rec;
    DevBuf wtot, woff;  // per-workgroup code counts of the staged pass and their exclusive scan
    dev::IndexlessArgs a{};
    uint64_t total = 0;
    bool block_off = false;  // offsets per workgroup (woff) only; off[] not written
};
// need_off: every segment's offset in `off` (else, on the staged path, only
// the per-workgroup offsets in `woff`: k_mark_lite's form)
// before_wait: launched after the scan, before the host waits for the
// total (work that does not need the count: k_mark_lite, so the host's wait
// overlaps it instead of stalling the stream)
Status indexless_sync(huff_ctx* ctx, const uint8_t* d_comp, uint64_t comp_bytes, uint64_t valid_bits,
                      const huff_tree* t, IndexlessSync& st, bool need_off = true,
                      const std::function<Status()>& before_wait = nullptr);
// sub_abs[g] = first bit of symbol g << shift (needs dev::indexless_staged(st.a))
Status indexless_mark(huff_ctx* ctx, IndexlessSync& st, DevBuf& sub_abs, uint32_t shift = 8);
Status decode_indexless_host(huff_ctx* ctx, const uint8_t* comp, size_t len, uint64_t valid_bits,
                             const huff_tree* t, std::vector<uint8_t>& out);
}  // namespace huff
