// kernels.hpp — launch interface of the gfx950 kernels.
//
// Data layout in HBM for one encode job of n input bytes:
//   in            u8[n]                 16-B aligned, read twice (hist, pack)
//   chunk_hist    u32[nchunks][256]     per 64 KiB chunk, written by hist
//   gw            u64[8][256]           global weights, one copy per XCD group
//   chunk_bits    u64[nchunks]          bits per chunk (after the tree is known)
//   chunk_start   u64[nchunks + 1]      exclusive scan of chunk_bits (+ bit base)
//   sub_bit       u32[ceil(n/64)]       restart index: bit offset of every
//                                       64th symbol (kIdx), relative to its chunk
//   out           u8[ceil(bits/8)]      the compress_with_tree byte stream
#pragma once

#include <hip/hip_runtime.h>
#ifdef __HIPCC__
#include <hip/hip_ext.h>
#endif

#include <cstdint>

namespace huff::dev {

// Kernel timing without marker packets. huff_ctx::timed() parks its event
// pair here; every launch inside the timed region carries the events on its
// own dispatch packet (hipExtLaunchKernelGGL) instead of two hipEventRecord
// markers around it: the first launch takes the start event, each launch
// re-records the stop event, so the pair spans the region's kernels. Outside
// a timed region launch_k is a plain launch.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents& launch_events();  // this thread's pair (runtime.cpp)
#ifdef __HIPCC__
template <typename F, typename... Args>
inline void launch_k(F kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t s, Args... args) {
    LaunchEvents& e = launch_events();
    if (e.stop) {
        hipExtLaunchKernelGGL(kernel, grid, block, lds, s, e.start, e.stop, 0, args...);
        e.start = nullptr;
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
    }
}
#endif

constexpr uint32_t kChunk = 65536;      // input bytes (= symbols) per chunk / workgroup
constexpr uint32_t kRound = 4096;       // bytes per workgroup round (256 lanes x 16 B)
constexpr uint32_t kSub = 256;          // symbols per lane of the long-code chunk decoder (decode.hip)
constexpr uint32_t kIdx = 64;           // restart index stride of the byte path (sub_bit): symbols
constexpr uint32_t kShortMaxLen = 27;   // u32 table entries: code << (32 - len) | len
constexpr uint32_t kLongMaxLen = 57;    // u64 table entries: code << 6 | len
constexpr uint32_t kHistCopies = 8;     // XCD-group copies of the global weights
constexpr uint32_t kLutMaxBits = 12;    // primary decode table index bits
constexpr uint32_t kLutPtr = 0x80000000u;
#ifndef HUFF_PACK_WAVES
#define HUFF_PACK_WAVES 8
#endif
constexpr uint32_t kPackWaves = HUFF_PACK_WAVES;  // waves per pack workgroup (short codes; long codes: 4)
// single-symbol u16 decode entry (k_decode_fixed): code length in bits
// [0, 6), letter in [8, 16); kSsSlow: the first code is longer than the
// table's index bits (<= kSsMaxBits)
constexpr uint32_t kSsMaxBits = 12;
constexpr uint32_t kSsSlow = 0x80u;


// The code table travels in the kernel arguments (no upload copy on the
// critical path between pass 1 and pass 2): u32 code << (32 - len) | len
// (left-aligned) for codes <= 27 bits, u64 code << 6 | len up to 57 bits.
union alignas(8) CodeTable {
    uint32_t s[256];
    uint64_t l[256];
};

struct PackArgs {
    CodeTable table;
    uint8_t prev_tail[8];         // right-aligned (prev_tail[7] precedes in[0])
    const uint8_t* in;
    uint64_t n;
    const uint64_t* chunk_start;  // [nchunks + 1], bits relative to out bit 0
    uint32_t nchunks;
    uint8_t* out;
    uint32_t* sub_bit;            // may be null
    // compact restart index (codes <= 16 bits; instead of sub_bit): the first
    // bit of every kTaskSym-symbol task (u64) and every 64th symbol's offset
    // from its task's first bit (u16: 4,096 codes of <= 16 bits fit)
    uint16_t* sub16;
    uint64_t* task_base;
    uint32_t prev_tail_len;
    uint32_t stage_words;         // per wave
    uint32_t grid;                // persistent workgroups (4 waves each)
    uint32_t max_len;             // longest code (groups codes for the OR emit)
};

struct DecodeArgs {
    const uint8_t* comp;          // stream, 4-B aligned; bit 0 = MSB of comp[0]
    uint64_t comp_bytes;          // readable bytes of comp
    const uint32_t* lut;          // primary [1 << K] then secondary tables
    uint32_t lut_bits;            // K
    uint32_t lut_words;           // total words (primary + secondary)
    const uint64_t* chunk_start;  // [nchunks + 1]
    const uint32_t* sub_bit;      // [ceil(n / kIdx)]
    uint32_t nchunks;
    uint32_t max_len;             // longest code (> 32: window slow path)
    const uint64_t* sub_abs;      // non-null: absolute start bit of every 256-symbol run
                                  // (index-free decode), instead of chunk_start + sub_bit
    const uint16_t* stab;         // single-symbol table [1 << stab_bits] (k_decode_fixed)
    uint32_t stab_bits;
    uint32_t cu_count;            // persistent grid of the checked k_decode_fixed
    uint64_t n;
    uint8_t* out;
    // k_decode_fixed on an index-free stream: absolute start bit of every
    // kIdx-th symbol (instead of chunk_start + sub_bit) and the stream's end
    const uint64_t* sub_abs64;
    uint64_t end_bit;
    // the compact restart index (PackArgs::sub16 / task_base), instead of
    // chunk_start + sub_bit (k_decode_fixed)
    const uint16_t* sub16;
    const uint64_t* task_base;
    // sub_abs64 entries as k_mark_lite writes them: a boundary at or before
    // the symbol in bits [0, 48) and the codes to skip from it in [48, 64)
    uint32_t skip_packed;
    // (skip_packed) k_mark_lite's compact marks instead of sub_abs64: a u32
    // per kIdx-th symbol (mark32_* below) and the segment index of every
    // task's first mark; seg_bits = the segments' S
    const uint32_t* mark32;
    const uint32_t* task_seg;
    uint32_t seg_bits;
    // k_decode_fixed: swizzle the input stage (16-B pieces XOR-permuted per
    // 128-B block, decode_wave.hip PaddedLdsWords): for mean code lengths
    // where the lanes' streams start ~32 m / k dwords apart every refill
    // would hit the same few LDS banks
    uint32_t pad_stage;
    // k_decode_fixed: the 3 KiB per-wave stage (8 workgroups per CU instead of
    // 6) for streams of at most kSmallStageBits bits per symbol (fixed_decode_small)
    uint32_t small_stage;
    // k_decode_fixed: 1 = the persistent LDS-DMA build (decode_wave.hip
    // k_decode_dma: the next task's input in flight while a task decodes)
    uint32_t dma_stage;
    // k_decode_fixed self-check build (0: production kernel; 1: checked).
    // err: u32[8] mismatch count + first (task, lane, want, got)
    uint32_t check_mode;
    uint32_t* err;
    uint64_t* stamps;             // timing builds (-DHUFF_STAMPS) only: per-wave phase stamps
};
// whether k_decode_fixed should swizzle its stage for this mean code
// length: the stride bands where a bank model of the 32-lane refill reads
// (lane starts jittered 0.6 dwords per 64 symbols; tools/stage_banks.py)
// gives the swizzled stage >= 1 LDS cycle fewer per read than the plain one
// A 4,096-symbol task in the 3 KiB stage: its bits plus the 32-B lookahead
// (and, index-free, the skip codes) within 3,072 B: 5.9 bits per symbol at
// most; a mean of up to 5.6 leaves ~20 standard deviations of a task's sum on
// the workloads measured (tasks that do not fit decode from global memory)
constexpr double kSmallStageBits = 5.6;
inline bool fixed_decode_small(uint64_t bits, uint64_t nsym) {
    return nsym && static_cast<double>(bits) <= kSmallStageBits * static_cast<double>(nsym);
}
inline bool fixed_decode_pad(uint64_t bits, uint64_t nsym) {
    if (nsym == 0) return false;
    const double s = 2.0 * static_cast<double>(bits) / static_cast<double>(nsym);  // dwords per 64 symbols
    static const double band[][2] = {{6.35, 6.45}, {7.75, 8.25}, {10.45, 10.95}, {15.55, 16.45}, {21.05, 21.65}, {23.85, 24.15}};
    for (const auto& b : band)
        if (s >= b[0] && s <= b[1]) return true;
    return false;
}

struct IndexlessArgs {
    const uint8_t* comp;
    uint64_t comp_bytes;
    uint64_t valid_bits;          // B
    uint64_t seg_bits;            // S (multiple of the gcd of code lengths)
    uint32_t lead_bits;           // the staged pass's lead-in (<= kLeadBitsLong, a multiple of the gcd; 0: none)
    uint64_t nseg;
    const uint32_t* lut;
    uint32_t lut_bits;
    uint64_t* s;                  // [nseg] settled segment starts
    uint64_t* x;                  // [nseg] exits
    uint64_t* c;                  // [nseg] symbol counts
    uint32_t max_len;
    // spec samples (LDS-staged path): segment i's slots at samp + stride i,
    // slot k the first chunk end of its speculative path at or after
    // i*S + kSampBits (k + 1) (indexless.hip: u16 offset past that / codes
    // since the previous slot; 0xFFFF none)
    uint16_t* samp;
    uint32_t nsamp;
    // how the settled path relates to the speculative one: past true-local
    // symbol tm[i] they coincide, true-local = spec-local + dl[i]
    // (tm = kNoMerge: never within the segment)
    uint32_t* tm;
    int32_t* dl;
    // (LDS-staged path) s, c, tm and dl of segment i packed in rec[i]
    // (indexless.hip rec_pack: count, tm, dl, start - i*S; 16 bits each); the
    // arrays above are then unused, but c for launch_indexless_counts
    uint64_t* rec;
    // [0, kFixRounds): round r found a changed exit; [kFixRounds]: fixlist
    // count; [kFixRounds + 1, +2]: the counts of the chain's two lists;
    // [kFixRounds + 3]: the chain's fixes in all
    unsigned int* flags;
    // (LDS-staged path) segments whose start may not be their predecessor's
    // exit after the speculative pass, besides every workgroup's first one:
    // the successors of segments the in-workgroup fix-up gave a new exit
    uint32_t* fixlist;
    // (LDS-staged path) 2 x nseg: the fix-up chain's lists (k_fix_chain)
    uint32_t* chain;
    const uint16_t* stab;         // single-symbol table (k_decode_fixed's): the LDS-staged kernels
    uint32_t stab_bits;
    // walk table over the same stab_bits-bit windows, for the speculative
    // pass (which needs lengths, not letters; it replaces stab there): bits
    // [0, 6) = the first code's length and kSsSlow as in stab, [8, 12) = the
    // bits of all the window's complete codes, [12, 16) = their count
    // (null: single steps from stab only)
    const uint16_t* wtab;
    // level-2 length table (DecTables::l2off: descriptors, then u8 lengths),
    // staged in LDS after the single-symbol table; null: the slow steps read
    // the global multi-level table `lut`
    const uint32_t* l2;
    uint32_t l2_words;
    // > 0: l2 is the uniform form, 2^l2_e u8 lengths per slow window, no
    // descriptors (DecTables::l2E)
    uint32_t l2_e;
    // uniform form with slow windows common (DecTables::l2dense): the walks
    // read a length at every step instead of branching (segwalk.hpp)
    uint32_t l2_dense;
    // (LDS-staged path) the code count of each workgroup's 256 segments,
    // written by the speculative pass and kept by the fix-up kernels (atomic
    // deltas): the scan runs over workgroups, k_mark_lite scans inside one
    unsigned long long* wtot;
    uint64_t* stamps;             // timing builds (-DHUFF_STAMPS) only: per-wave phase stamps
};
// the staged speculative pass starts each lane up to kLeadBits before its
// segment (indexless.hip k_spec_lds)
#ifndef HUFF_LEAD_BITS
#define HUFF_LEAD_BITS 128
#endif
constexpr uint32_t kLeadBits = HUFF_LEAD_BITS;
// trees with codes longer than the walk table's index take longer to fall
// onto the true path: twice the lead-in (wide letters, Zipf over 4,096:
// W = 4 index-free 1.35 -> 1.27 ms, W = 2 2.01 -> 1.98; byte streams whose
// codes all fit the table keep 128: 256 measured 1 % slower on text)
constexpr uint32_t kLeadBitsLong = 2 * kLeadBits;
// the speculative pass's sample spacing (indexless.hip); segments < 1024 bits
#ifndef HUFF_SAMP_BITS
#define HUFF_SAMP_BITS 96
#endif
constexpr uint32_t kSampBits = HUFF_SAMP_BITS;
constexpr uint32_t kSampMax = 1023 / kSampBits;  // samples kept per segment (nsamp <= kSampMax)
constexpr uint32_t kNoMerge = 0xFFFFFFFFu;
constexpr int kFixRounds = 4;     // device-side fix-up rounds before the sequential fallback

// dst[i] = map[src[i]] (+ arithmetic restart index)
struct BytemapArgs {
    uint8_t map[256];
    const uint8_t* src;
    uint8_t* dst;
    uint64_t n;
    uint64_t* chunk_start;        // may be null
    uint32_t nchunks;
    uint64_t base_bits;
    uint32_t* sub_bit;            // may be null
};
// the arithmetic restart index of an all-8-bit stream (what k_bytemap writes
// when asked), as its own launch: chunk_start[c] = base_bits + 8 c kChunk,
// sub_bit[g] = 8 (g kIdx mod kChunk)
hipError_t launch_arith_index(uint64_t n, uint32_t nchunks, uint64_t base_bits, uint64_t* chunk_start,
                              uint32_t* sub_bit, hipStream_t s);
constexpr uint32_t kTaskSym = 4096;  // symbols per decode task (k_decode_fixed) = per compact index base
// sub_bit[g] from the compact index (for the decoders that read sub_bit)
hipError_t launch_index_expand(uint64_t n, const uint64_t* task_base, const uint16_t* sub16,
                               const uint64_t* chunk_start, uint32_t* sub_bit, hipStream_t s);

// wider letters (wide.hip): W-byte keys, hash-table code lookup. The
// encoder's chunk is kWideChunk letters (one wave), its restart index
// chunk_start per chunk + u32 sub_bit per run of kWideRun letters (relative
// to the chunk start; sub_abs entries of index-free streams likewise per run).
constexpr uint32_t kWideRun = 64;
constexpr uint32_t kWideChunk = 256 * kWideRun;
struct WideArgs {
    const uint8_t* in;            // n letters of `width` bytes, native layout, 16-B aligned
    uint64_t n;
    uint32_t width;               // 1, 2, 4, 8, 16
    // code table (host/wide.hpp WideEncTables): `slots` slots of slot_bytes,
    // {key, value}; a letter's slots are wide_slots(wide_hkey(letter))
    const void* table;
    uint32_t slots, slot_bytes, mul1;
    uint32_t hash_mode;           // host/wide.hpp WideHash (0 generic, 1 narrow, 2 direct)
    uint64_t fold;
    uint32_t long_codes;          // values u64 code << 6 | len, else u32 code << (32 - len) | len
    uint32_t max_len;
    uint32_t table_in_lds;        // stage the table in LDS (wide_lds_bytes <= kWideLdsMax)
    uint32_t nchunks;             // ceil(n / kWideChunk)
    uint32_t cu_count;            // persistent grid size
    uint32_t stage_words;         // pack: LDS staging words per wave (wide_stage_words)
    uint64_t* chunk_bits;         // [nchunks]            (bits pass)
    const uint64_t* chunk_start;  // [nchunks + 1]        (pack pass)
    uint32_t* sub_bit;            // [ceil(n / kWideRun)] run start - chunk start
    unsigned long long* first_missing;  // min index of a letter without a code
    uint8_t* out;                 // any alignment: ceil(bits / 8) bytes
};
// LDS of a pass's workgroup (the table when in_lds, pack's staging images);
// the table is staged when a workgroup's total fits kWideLdsMax
constexpr size_t kWideLdsMax = 160 * 1024;
uint32_t wide_stage_words(uint32_t width, uint32_t max_len);
size_t wide_lds_bytes(const WideArgs& a, bool pack_pass, bool in_lds);
struct WideDecArgs {
    const uint8_t* comp;          // 4-B aligned
    uint64_t comp_bytes;
    const uint32_t* lut;          // leaf = (len << 24) | leaf, ptr = kLutPtr | offset
    uint32_t lut_bits;
    const void* stab;             // wdecode.hip: the two-level table (host/wide.hpp WideDecTables::stab)
    uint32_t stab_bits;           // its level-1 index bits
    uint32_t stab_bytes;
    const uint8_t* letters;       // [leaves * width]
    uint32_t nleaves;
    uint32_t width;
    uint32_t w4_leaf;             // W = 4: the table names leaves (letters >= 2^24), else letters
    const uint64_t* chunk_start;  // per wide chunk
    const uint32_t* sub_bit;      // per run of kWideRun letters
    const uint64_t* sub_abs;      // non-null: index-free restart points, per run of kWideRun letters
    uint32_t skip_packed;         // wdecode.hip: sub_abs entries as k_mark_lite writes them (a boundary at
                                  // or before the run in bits [0, 48), the codes to skip from it above)
    uint64_t end_bit;             // the stream's last bit + 1 (wdecode.hip: the last task's end)
    uint32_t nchunks;
    uint32_t cu_count;
    uint32_t max_len;             // longest code (<= 32: wdecode.hip)
    uint32_t stage_bytes;         // wdecode.hip: LDS stage per wave (a multiple of 16)
    uint64_t n;
    uint8_t* out;                 // n * width bytes
};
hipError_t launch_wide_bits(const WideArgs& a, hipStream_t s);
hipError_t launch_wide_pack(const WideArgs& a, hipStream_t s);
hipError_t launch_wide_decode(const WideDecArgs& a, hipStream_t s);       // codes > 32 bits (wide.hip)
hipError_t launch_wide_decode_task(const WideDecArgs& a, hipStream_t s);  // codes <= 32 bits (wdecode.hip)
// build_weights_map on the device (wweights.hip). width <= 2: counts = the
// 2^(8 width) bins (zeroed). width >= 4: an HBM table of `slots`
// (wcount_slots of a guess of the distinct letters) keys_lo (all ones),
// counts (zero), width 16 also keys_hi and state (zero); *used counts the
// claimed slots and *overflow (zeroed) is set when the table is too full (the
// host grows it and counts again; `unbounded`: the last size, no limits). Then
// wextract_launch appends the used slots to out_lo / out_hi / out_c
// (capacity *used), their number to *nout (zero); the all-ones u64 letter's
// count goes to *sent (zero; width 8).
struct WCountArgs {
    const uint8_t* in;  // n letters, 4-B aligned (width >= 4: width-aligned)
    uint64_t n;
    uint32_t width;
    uint64_t slots;
    unsigned long long *keys_lo, *keys_hi, *counts, *sent;
    unsigned int* state;
    unsigned long long *out_lo, *out_hi, *out_c, *nout;
    uint64_t out_cap;             // k_wextract stores only indices < out_cap (it counts them all in *nout)
    unsigned long long* used;
    unsigned int* overflow;
    uint32_t unbounded;
};
uint64_t wcount_slots(uint32_t width, uint64_t distinct);
hipError_t wcount_launch(const WCountArgs& a, hipStream_t s);
hipError_t wextract_launch(const WCountArgs& a, hipStream_t s);

// HuffTree of many small byte streams in one launch (tree_batch.hip)
constexpr uint32_t kTreeBitsMaxBytes = (2 * 257 - 1 + 8 * 257 + 7) / 8;  // as_bin of 257 leaves
constexpr uint32_t kTreeCodeMax = 56;  // codes[] holds code << 8 | len
enum : uint32_t { kTreeOk = 0, kTreeHeavy = 1, kTreeEmpty = 2, kTreeDeep = 7 };  // = HUFF_OK, HUFF_E_INVALID_ARG (weights sum >= 2^54), HUFF_E_EMPTY_WEIGHTS, HUFF_E_CODE_TOO_LONG
struct TreeBatchArgs {
    const uint64_t* hist;   // [nstreams][256] byte weights
    uint32_t nstreams;
    uint8_t* tree_bits;     // [nstreams][tree_stride]: as_bin (tree_inner.rs:632-663), MSB first
    uint32_t tree_stride;   // >= kTreeBitsMaxBytes
    uint32_t* tree_nbits;   // [nstreams]
    uint64_t* codes;        // [nstreams][256]: code << 8 | len; 0 = no code (or longer than kTreeCodeMax)
    uint32_t* max_len;      // [nstreams]
    uint32_t* status;       // [nstreams]: kTreeOk, kTreeEmpty (no weights), kTreeDeep (a code > kTreeCodeMax)
};
// hist[s] = the byte weights of in[off[s], off[s + 1])
hipError_t launch_hist_batch(const uint8_t* in, const uint64_t* off, uint32_t nstreams, uint64_t* hist,
                             hipStream_t s);
hipError_t launch_tree_batch(const TreeBatchArgs& a, hipStream_t s);

// codes longer than kLongMaxLen (deep.hip): up to 255 bits, kDeepWords
// left-aligned words per letter
constexpr uint32_t kDeepWords = 8;
struct DeepPackArgs;
struct DeepSerialArgs {
    const uint8_t* comp;
    uint64_t comp_bytes;
    uint64_t valid_bits;
    const uint32_t* lut;          // multi-level table (primary lut_bits, 8-bit secondaries)
    uint32_t lut_bits;
    uint8_t* out;
    uint64_t cap;
    unsigned long long* count;
    unsigned long long* end;      // may be null: the bit after the last complete code
};
struct WalkEndArgs {
    const uint8_t* comp;
    uint64_t comp_bytes;
    const uint32_t* lut;
    uint32_t lut_bits;
    const uint64_t* start;        // device value, or start_v when null
    uint64_t start_v;
    uint32_t start_packed;        // *start is a k_mark_lite entry (position | skip << 48)
    const uint64_t* count;        // device value, or count_v when null
    uint64_t count_v;
    unsigned long long* end;
};
hipError_t launch_walk_end(const WalkEndArgs& a, hipStream_t s);
hipError_t launch_shift_bits(const uint8_t* src, uint8_t* dst, uint64_t n, uint32_t r, hipStream_t s);
hipError_t launch_pack_deep(const DeepPackArgs& a, hipStream_t s);
hipError_t launch_decode_deep(const DecodeArgs& a, hipStream_t s);  // lut, lut_bits, restart index, n, out
hipError_t launch_decode_deep_serial(const DeepSerialArgs& a, hipStream_t s);

size_t pack_lds_bytes(bool long_codes, uint32_t max_len, uint32_t stage_words);
uint32_t pack_round_bytes();  // input bytes per wave round of k_pack (its LDS stage holds one round's bits)
uint32_t pack_waves_per_group(bool long_codes);
// resident k_pack workgroups per CU for this launch (its registers and LDS
// both limit; the persistent grid is this many per CU)
uint32_t pack_groups_per_cu(bool long_codes, uint32_t max_len, size_t lds);
size_t decode_lds_bytes(uint32_t lut_bits);
// HUFF_DEC_VARIANT: 10 = k_decode_fixed (the default for codes <= 32 bits),
// 11 = its self-checking build
constexpr uint32_t kDecodeFixed = 10;
constexpr uint32_t kDecodeFixedCheck = 11;

// Pass 1's totals straight to pinned host memory (device-visible pointer):
// host[b] = (tag << 48) | total_b. host == nullptr: the totals stay in gw.
// a result published straight to pinned host memory: (tag << 48) | value
// in one 8-byte store (pass 1's weights, a scan's grand total)
// Index-free decode in one pass (syncdec.hip): tiles of 256 segments, a lane
// per segment decoding its letters into registers, an in-tile fix-up, a
// decoupled look-back over the tiles for the output offsets, letters out
// through LDS windows; k_sync_tail then decodes the letters the lanes could
// not hold and publishes the count. Byte letters, max_len <= stab_bits <= 12.
constexpr uint32_t kSyncCap = 128;         // letters per lane in registers
constexpr uint32_t kSyncWin = 4096;        // output window per wave (bytes)
constexpr uint32_t kSyncLook = 256;        // staged bytes past a tile's last segment end
constexpr uint32_t kSyncTicket = 0, kSyncJobs = 1, kSyncErr = 2, kSyncMis = 3;  // ctrl words
constexpr uint64_t kSyncBad = (1ull << 48) - 1;  // published instead of the count: take the pipeline
struct SyncDecArgs {
    const uint8_t* comp;
    uint64_t comp_bytes;
    uint64_t valid_bits;
    uint64_t seg_bits;            // S: a multiple of the code lengths' gcd, lead_bits <= S
    uint64_t nseg;
    uint32_t lead_bits;           // a multiple of the gcd
    uint32_t lead0_bits;          // a tile's first lane's (its entry is the tile's), >= lead_bits
    const uint16_t* stab;         // single-symbol table (DecTables::soff), 2^stab_bits entries
    uint32_t stab_bits;
    uint8_t* out;                 // any alignment; nothing at or past out_cap is written
    uint64_t out_cap;
    unsigned long long* tile;     // [ceil(nseg / 256)] tile words, zeroed before the launch
    unsigned int* ctrl;           // [4] ticket, job count, error, look-back waits; zeroed before the launch
    unsigned long long* total;    // [1] the letter count (the last tile)
    uint64_t* jobs;               // [3 * job_cap]: start bit, first letter, letters
    uint64_t job_cap;
    unsigned long long* host_total;  // pinned: (tag << 48) | count (kSyncBad: failed), by k_sync_tail
    uint64_t tag;
    uint64_t* stamps;             // timing builds (HUFF_STAMPS): 10 words per wave (bitreader.hpp WaveStamps)
};
size_t sync_decode_lds_bytes(const SyncDecArgs& a);
hipError_t launch_sync_decode(const SyncDecArgs& a, hipStream_t s);

struct HistDone {
    unsigned long long* host = nullptr;
    uint64_t tag = 0;  // 16 bits
};
hipError_t launch_hist(const uint8_t* base, uint64_t lo, uint64_t hi, uint32_t nchunks, uint32_t* chunk_hist,
                       unsigned long long* gw, hipStream_t s, HistDone done = HistDone{});
// row[0..256) = gw summed over its copies, row[256] = in's last min(8, n)
// bytes (little-endian), row[257] = their count
hipError_t launch_hist_row(const unsigned long long* gw, const uint8_t* in, uint64_t n, long long* row,
                           hipStream_t s);
struct alignas(8) CodeLens {
    uint8_t len[256];
};
struct DeepPackArgs {
    CodeLens len;
    const uint32_t* words;        // [256][kDeepWords] left-aligned codes
    const uint8_t* in;
    uint64_t n;
    const uint64_t* chunk_start;  // [nchunks + 1], bits relative to out bit 0
    uint32_t nchunks;
    uint8_t* out;                 // zeroed beforehand (codes are ORed in)
    uint32_t* sub_bit;            // may be null
};
hipError_t launch_chunk_bits(const uint32_t* chunk_hist, uint32_t nchunks, const CodeLens& len, uint64_t* bits,
                             hipStream_t s);
// tsum: scratch of ceil(nchunks / 1024) (>= 1) u64
hipError_t launch_scan(const uint64_t* bits, uint32_t nchunks, uint64_t base, uint64_t* start, uint64_t* tsum,
                       hipStream_t s, HistDone done = HistDone{});
hipError_t launch_pack(bool long_codes, const PackArgs& a, hipStream_t s);
hipError_t launch_decode(const DecodeArgs& a, hipStream_t s);
hipError_t launch_decode_fixed(const DecodeArgs& a, hipStream_t s);
hipError_t launch_indexless_spec(const IndexlessArgs& a, hipStream_t s);
// LDS-staged path: k_fix_list (round 0 over the segments that can differ)
// then k_fix_chain (one workgroup following the changed exits, a no-op when
// round 0 changed none). Else kFixRounds fix-up rounds (each a no-op once the
// previous one changed nothing), then the sequential sweep only if the last
// round still changed an exit. No host round trip either way.
hipError_t launch_indexless_settle_all(const IndexlessArgs& a, hipStream_t s);
hipError_t launch_indexless_emit(const IndexlessArgs& a, const uint64_t* off, uint8_t* out, hipStream_t s);
// (LDS-staged path) c[i] = the packed records' counts, for a scan over every segment
hipError_t launch_indexless_counts(const IndexlessArgs& a, hipStream_t s);
// restart index for the ring decoder: sub_abs[g] = start bit of symbol 256 g
// sub_abs[g] = start bit of symbol g << shift (shift 8: the ring/wide
// decoders' 256-symbol runs; 6: k_decode_fixed's kIdx = 64)
// sub_abs[g] = (a boundary at or before symbol 64 g) | (codes from it to the
// symbol) << 48, without walking: the decoder skips the codes (k_mark_lite)
// off: per-segment offsets, or null and woff: per-workgroup offsets (the
// scan of IndexlessArgs::wtot; k_mark_lite scans inside each workgroup)
// sub_cap: entries of sub_abs that may be written (the marks past it are not;
// the caller sized sub_abs before the symbol count was known).
// mark32 / task_seg non-null: the compact form instead of sub_abs (4 B per
// mark + 4 B per task of kTaskSym symbols, half the u64 marks' traffic):
// mark = skip | offset from its segment's nominal start << 10 | the
// segment's index mod 2048 << 21; task_seg[t] = the segment index of task t's
// first mark, from which a decoder recovers the others (a task spans far
// fewer than 2048 segments).
constexpr uint32_t mark32_skip(uint32_t m) { return m & 0x3FFu; }
constexpr uint32_t mark32_rel(uint32_t m) { return (m >> 10) & 0x7FFu; }
constexpr uint32_t mark32_seg(uint32_t m, uint32_t base_seg) { return base_seg + (((m >> 21) - base_seg) & 0x7FFu); }
hipError_t launch_indexless_mark_lite(const IndexlessArgs& a, const uint64_t* off, const unsigned long long* woff,
                                      uint64_t* sub_abs, uint64_t sub_cap, hipStream_t st,
                                      uint32_t* mark32 = nullptr, uint32_t* task_seg = nullptr);
constexpr uint64_t kSkipPosMask = (1ull << 48) - 1;
hipError_t launch_indexless_mark(const IndexlessArgs& a, const uint64_t* off, uint64_t* sub_abs, uint32_t shift,
                                 hipStream_t s);
bool indexless_staged(const IndexlessArgs& a);  // k_spec/k_mark LDS variants apply
hipError_t launch_bytemap(const BytemapArgs& a, hipStream_t s);
// letter checksums of the decode check build (checksum.hip): per task of
// kTaskSym letters, sum and position-weighted sum (u64 = s2 << 32 | s1);
// the check counts differing tasks in err[0], the first one in err[1] (set
// err[1] to ~0u before)
hipError_t launch_task_sums(const uint8_t* x, uint64_t n, uint64_t* sums, hipStream_t s);
hipError_t launch_task_sums_check(const uint8_t* x, uint64_t n, const uint64_t* sums, unsigned int* err,
                                  hipStream_t s);
hipError_t launch_find_first(const uint8_t* in, uint64_t n, const uint8_t* missing_mask, unsigned long long* pos,
                             hipStream_t s);
hipError_t launch_generate(int kind, uint64_t seed, uint64_t offset, const uint64_t* cdf, uint8_t* out, uint64_t n,
                           hipStream_t s);
// HBM calibration (synth.hip, measurement only): modes 0/1 = streaming read
// of src (grid-stride / one-shot), 2/3 = streaming copy src -> dst (grid-
// stride / one-shot); n a multiple of 16, pointers 16-B aligned
hipError_t launch_calib(int mode, const uint8_t* src, uint8_t* dst, uint64_t n, unsigned* sink, uint32_t cu_count,
                        hipStream_t s);

}  // namespace huff::dev
