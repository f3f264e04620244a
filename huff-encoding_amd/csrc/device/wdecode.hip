// wdecode.hip — restart-index decode of the wider letters for codes <= 32
// bits (comp.rs:487-519 semantics), on k_decode_fixed's plan (decode_wave.hip):
//
// Work unit: a TASK of 4,096 consecutive letters per wave, lane l decoding
// letters [64 l, 64 l + 64) from the restart entry of its run (kWideRun = 64
// letters: the encoder's sub_bit, or sub_abs of an index-free stream). The
// task's compressed bits are one contiguous range: the wave stages it in LDS
// with coalesced 16-B loads (a range longer than the stage decodes from
// global memory instead), then every lane makes exactly 64 lookups in a
// two-level table (LDS when it fits): level 1 by the first K1 <= 11 bits,
// level 2 by exactly the bits the deepest code below needs (host/wtree.cpp
// build_wide_stab), two reads per letter for every lane, no divergence. An
// entry carries the code length and the letter itself for letters of <= 4
// bytes (u32 entries for <= 2-byte letters, u64 for 4-byte ones), the leaf
// index for wider ones (their letters in LDS).
// A lane's letters are joined in registers, 64 bytes at a time, and leave
// through the wave's LDS transpose buffer: every store instruction writes 16
// lanes' 64-byte parts whole.
//
// Roofline: HBM-bound in principle; ceil(bits/8) read + n W written + the
// restart index (4 B per 64 letters).
#include <type_traits>

#include "bitreader.hpp"

namespace huff::dev {

namespace {

// waves per workgroup: as many as the LDS holds beside one table copy, at
// most 16 (the 2-byte body fits the 128 registers of a 16-wave workgroup
// since its output stores take 32-bit buffer offsets; round 4 capped it at
// 12). HUFF_W2_WAVES: the cap for <= 2-byte letters (A/B builds).
#ifndef HUFF_W2_WAVES
#define HUFF_W2_WAVES 16
#endif
template <uint32_t W>
constexpr int max_waves() { return W <= 2 ? HUFF_W2_WAVES : 16; }
constexpr uint32_t kTaskLetters = 64 * kWideRun;  // 4,096
constexpr uint32_t kSlowFlag = 0x80;              // entry: the first code is longer than K
// a wave's transpose buffer: for <= 4-byte letters 32 rows of 64 B, the 64
// lanes' parts in two halves, stored through 32-bit buffer offsets (a 4 KiB
// buffer for all 64 rows at once held the 2-byte decoder to 13 waves per CU
// beside its table and stages: W = 2 0.628 -> 0.602 ms, W = 4 0.484 ->
// 0.474); wider letters (8 parts per lane and more) keep all 64 rows at once
// and plain stores: the halves' extra wave syncs cost the 8-byte decoder 11 %
// (0.366 -> 0.405 ms), the buffer stores 2 %
template <uint32_t W>
constexpr uint32_t row_halves() { return W <= 4 ? 2u : 1u; }
template <uint32_t W>
constexpr uint32_t row_bytes() { return 64 * 64 / row_halves<W>(); }

struct U128 {
    uint64_t lo, hi;
};

// u32 entries: the letter (<= 2 bytes; 4 bytes below 2^24) or the leaf
// (wider, and 4-byte alphabets with larger letters: WideDecArgs::w4_leaf)
template <uint32_t W>
using EntryT = uint32_t;
template <uint32_t W>
__device__ __forceinline__ uint32_t payload(EntryT<W> e) { return e >> 8; }
// letters in LDS beside the table: wide letters, and 4-byte leaves
template <uint32_t W>
__host__ __device__ __forceinline__ bool leaf_letters(const WideDecArgs& a) { return W >= 8 || (W == 4 && a.w4_leaf); }

// dword sources (stream order, most significant byte first)
struct StageWords {
    const uint32_t* w;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return w[i]; }
};
struct GlobalWords {
    const uint8_t* comp;
    uint64_t nbytes;
    uint64_t dw0;  // absolute dword index of word 0
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const {
        const uint64_t b = (dw0 + i) * 4;
        if (b + 4 <= nbytes) return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(comp + b));
        uint32_t v = 0;
        for (uint32_t k = 0; k < 4 && b + k < nbytes; ++k) v |= static_cast<uint32_t>(comp[b + k]) << (24 - 8 * k);
        return v;
    }
};

// letter `leaf` of the tree's leaf table, as dwords
template <uint32_t W>
__device__ __forceinline__ void leaf_letter(const uint8_t* letters, uint32_t leaf, uint32_t (&d)[W >= 4 ? W / 4 : 1]) {
    if constexpr (W == 1) d[0] = letters[leaf];
    else if constexpr (W == 2) d[0] = reinterpret_cast<const uint16_t*>(letters)[leaf];
    else {
#pragma unroll
        for (uint32_t k = 0; k < W / 4; ++k) d[k] = reinterpret_cast<const uint32_t*>(letters)[leaf * (W / 4) + k];
    }
}

// the window shifted left by len (1..32 bits, the entries' code lengths) as
// two 32-bit halves: no 64-bit shift by a VGPR amount, which the gfx950 shift
// hazard makes depend on the register allocation
__device__ __forceinline__ uint64_t shl_window(uint64_t buf, uint32_t len) {
    const uint32_t hi = static_cast<uint32_t>(buf >> 32), lo = static_cast<uint32_t>(buf);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32u - len);
    const uint32_t nlo = len >= 32 ? 0u : lo << len;
    return (static_cast<uint64_t>(nhi) << 32) | nlo;
}

// One lane's letters [from, from + PL) of its 64, decoded into o (PL * W
// bytes, PL * W / 4 dwords), window state carried between parts. Window:
// 64-bit buf, valid-bit count in the low 6 bits of X (the rest don't-care),
// refilled unconditionally (decode_wave.hip FX_REFILL): every two codes when
// codes have <= 16 bits, before every code otherwise (R1).
template <uint32_t W>
struct Lane {
    uint64_t buf;
    uint32_t X, rp, nextw;
};

// Lookup: level 1 by the window's first K1 bits; TWO: a pointer entry (0x80
// | s, offset in bits 8..31) continues at level 2 with the next s bits. Both
// reads are made by every lane (a lane with a level-1 leaf re-reads entry 0:
// one broadcast address), so lanes never diverge.
template <uint32_t W, uint32_t PL, bool TWO, bool R1, class Words>
__device__ __forceinline__ void decode_part(Lane<W>& s, const Words& src, uint32_t (&o)[PL * W / 4 > 0 ? PL * W / 4 : 1],
                                            const EntryT<W>* __restrict__ tab, uint32_t K1,
                                            const uint8_t* __restrict__ letters, bool leaf4) {
    auto refill = [&]() {
        s.buf |= (static_cast<uint64_t>(s.nextw) << 32) >> (s.X & 63);
        s.rp += (s.X & 32) ? 0u : 1u;
        s.X |= 32;
        s.nextw = src(s.rp);
    };
#pragma unroll
    for (uint32_t i = 0; i < PL; ++i) {
        if (R1 || (i & 1) == 0) refill();
        const uint32_t top = static_cast<uint32_t>(s.buf >> 32);
        EntryT<W> e = tab[top >> (32 - K1)];
        if constexpr (TWO) {
            const uint32_t lo = static_cast<uint32_t>(e);
            const bool ptr = (lo & kSlowFlag) != 0;
            const uint32_t sw = lo & 63u;
            const uint32_t i2 = ptr ? (lo >> 8) + ((top << K1) >> (32 - sw)) : 0u;
            const EntryT<W> e2 = tab[i2];
            e = ptr ? e2 : e;
        }
        const uint32_t len = static_cast<uint32_t>(e) & 63u;
        // (8- and 16-byte letters: the split shift keeps the build clear of
        // the shift hazard since the skip loop was added; others unchanged)
        if constexpr (W >= 8) s.buf = shl_window(s.buf, len);
        else s.buf <<= len;
        s.X -= len;
        const uint32_t v = payload<W>(e);
        if constexpr (W == 1) {
            if ((i & 3) == 0) o[i >> 2] = v;
            else o[i >> 2] |= v << (8 * (i & 3));
        } else if constexpr (W == 2) {
            if ((i & 1) == 0) o[i >> 1] = v;
            else o[i >> 1] |= v << 16;
        } else if constexpr (W == 4) {
            o[i] = leaf4 ? reinterpret_cast<const uint32_t*>(letters)[v] : v;
        } else {
            uint32_t d[W / 4];
            leaf_letter<W>(letters, v, d);
#pragma unroll
            for (uint32_t k = 0; k < W / 4; ++k) o[i * (W / 4) + k] = d[k];
        }
    }
}

template <uint32_t W, class Words>
__device__ __forceinline__ void lane_init(Lane<W>& s, const Words& src, uint32_t rel) {
    s.rp = rel >> 5;
    const uint32_t sh = rel & 31;
    s.buf = static_cast<uint64_t>(src(s.rp) << sh) << 32;
    s.X = 32 - sh;
    s.rp += 1;
    s.nextw = src(s.rp);
}

// n codes consumed without their letters (index-free marks: the codes between
// the boundary k_mark_lite names and the run's first letter); a refill before
// every code, so any length <= 32 fits
template <uint32_t W, bool TWO, class Words>
__device__ __forceinline__ void lane_skip(Lane<W>& s, const Words& src, const EntryT<W>* __restrict__ tab, uint32_t K1,
                                          uint32_t n) {
    for (uint32_t j = 0; j < n; ++j) {
        s.buf |= (static_cast<uint64_t>(s.nextw) << 32) >> (s.X & 63);
        s.rp += (s.X & 32) ? 0u : 1u;
        s.X |= 32;
        s.nextw = src(s.rp);
        const uint32_t top = static_cast<uint32_t>(s.buf >> 32);
        EntryT<W> e = tab[top >> (32 - K1)];
        if constexpr (TWO) {
            const uint32_t lo = static_cast<uint32_t>(e);
            if (lo & kSlowFlag) e = tab[(lo >> 8) + ((top << K1) >> (32 - (lo & 63u)))];
        }
        const uint32_t len = static_cast<uint32_t>(e) & 63u;
        s.buf = shl_window(s.buf, len);
        s.X -= len;
    }
}

// letters per part: 64 bytes of output (16 registers; 128-byte parts held
// 135 registers for 2-byte letters)
template <uint32_t W>
constexpr uint32_t part_letters() { return 64u / W; }

// 16-B piece q of row r of a wave's transpose buffer (64 rows of 64 B, the
// pieces XOR-swizzled by row: conflict-free ds_write_b128, as decode_wave.hip)
__device__ __forceinline__ uint32_t row_piece(uint32_t r, uint32_t q) { return r * 64 + 16 * (q ^ ((r >> 1) & 3)); }

// a full lane: 64 letters in parts of 64 B. ROWS (every lane of the wave
// full, 16-B aligned output): each part goes through the wave's transpose
// buffer, so a store instruction writes 16 lanes' parts as whole 64-B
// segments (4 lanes each) — lane-strided 16-B stores wrote 2.6x the output
// bytes to HBM and kept the TA busy (PMC). Else 16-B stores per lane, or
// bytes when unaligned.
template <uint32_t W, bool TWO, bool R1, class Words>
__device__ __forceinline__ void lane_full(const Words& src, uint32_t rel, uint8_t* dst, const EntryT<W>* tab,
                                          uint32_t K1, const uint8_t* letters, bool aligned, uint8_t* rows,
                                          uint8_t* task_out, uint32_t lane, uint32_t skip, bool leaf4) {
    constexpr uint32_t PL = part_letters<W>();
    constexpr uint32_t ND = PL * W / 4;
    static_assert(ND == 16, "64-B parts");
    Lane<W> s;
    lane_init<W>(s, src, rel);
    lane_skip<W, TWO>(s, src, tab, K1, skip);
    for (uint32_t p = 0; p < kWideRun / PL; ++p) {
        uint32_t o[ND];
        decode_part<W, PL, TWO, R1>(s, src, o, tab, K1, letters, leaf4);
        if (rows) {
            if constexpr (W >= 8) {
                wave_order();  // the previous part's row reads were issued first
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q)
                    *reinterpret_cast<uint4*>(rows + row_piece(lane, q)) =
                        make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
                wave_order();
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t r = 16 * j + (lane >> 2), q = lane & 3;
                    const uint4 v = *reinterpret_cast<const uint4*>(rows + row_piece(r, q));
                    *reinterpret_cast<uint4*>(task_out + r * (kWideRun * W) + p * 64 + 16 * q) = v;
                }
                continue;
            }
            // through a buffer resource over the task's output: 32-bit
            // offsets (64-bit addresses per store held ~8 more registers)
            const auto ro = buf_rsrc(task_out, kTaskLetters * W);
            constexpr uint32_t H = row_halves<W>(), RH = 64 / H;  // halves, rows per half
#pragma unroll
            for (uint32_t h = 0; h < H; ++h) {  // lanes [RH h, RH h + RH)
                wave_order();  // the previous rows were read first
                if (H == 1 || lane / RH == h) {
#pragma unroll
                    for (uint32_t q = 0; q < 4; ++q)
                        *reinterpret_cast<uint4*>(rows + row_piece(lane % RH, q)) =
                            make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
                }
                wave_order();
#pragma unroll
                for (uint32_t j = 0; j < RH / 16; ++j) {
                    const uint32_t r = 16 * j + (lane >> 2), q = lane & 3;
                    const uint4 v = *reinterpret_cast<const uint4*>(rows + row_piece(r, q));
                    u32x4_t w = {v.x, v.y, v.z, v.w};
                    __builtin_amdgcn_raw_buffer_store_b128(
                        w, ro, static_cast<int>((RH * h + r) * (kWideRun * W) + p * 64 + 16 * q), 0, 0);
                }
            }
            continue;
        }
        uint8_t* d = dst + p * PL * W;
        if (aligned) {
            uint4* d4 = reinterpret_cast<uint4*>(d);
#pragma unroll
            for (uint32_t q = 0; q < ND / 4; ++q) d4[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        } else {
#pragma unroll
            for (uint32_t q = 0; q < ND; ++q)
#pragma unroll
                for (uint32_t b = 0; b < 4; ++b) d[4 * q + b] = static_cast<uint8_t>(o[q] >> (8 * b));
        }
    }
}

// the stream's last lane (fewer than 64 letters): one letter at a time
template <uint32_t W, bool TWO, bool R1, class Words>
__device__ __forceinline__ void lane_tail(const Words& src, uint32_t rel, uint32_t cnt, uint8_t* dst,
                                          const EntryT<W>* tab, uint32_t K1, const uint8_t* letters, uint32_t skip,
                                          bool leaf4) {
    Lane<W> s;
    lane_init<W>(s, src, rel);
    lane_skip<W, TWO>(s, src, tab, K1, skip);
    for (uint32_t j = 0; j < cnt; j += 2) {
        uint32_t o[2 * W / 4 > 0 ? 2 * W / 4 : 1];
        decode_part<W, 2, TWO, R1>(s, src, o, tab, K1, letters, leaf4);
        // bytes [0, 2 W) of o: the pair's letters (the second one past cnt is dropped)
#pragma unroll
        for (uint32_t b = 0; b < 2 * W; ++b)
            if (b < W || j + 1 < cnt) dst[j * W + b] = static_cast<uint8_t>(o[b / 4] >> (8 * (b % 4)));
    }
}

template <uint32_t W, bool TWO, bool R1, bool LDS>
__global__ __launch_bounds__((LDS ? max_waves<W>() : 4) * 64) void k_wdec_task(WideDecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t K1 = a.stab_bits;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = wave_index();
    // LDS: [the table][leaf letters (W >= 8, 4-byte leaves)] when LDS, then the waves' stages
    const uint32_t tab_bytes = LDS ? a.stab_bytes : 0u;
    const uint32_t let_bytes = LDS && leaf_letters<W>(a) ? (a.nleaves * W + 15) & ~15u : 0u;
    if constexpr (LDS) {
        for (uint32_t i = t; i < tab_bytes / 16; i += blockDim.x)
            reinterpret_cast<uint4*>(lds)[i] = reinterpret_cast<const uint4*>(a.stab)[i];
        for (uint32_t i = t; i < let_bytes / 16; i += blockDim.x)
            reinterpret_cast<uint4*>(lds + tab_bytes)[i] = reinterpret_cast<const uint4*>(a.letters)[i];
    }
    __syncthreads();
    // one pointer origin per instantiation (ds_read or global_load, never flat)
    const EntryT<W>* tab = LDS ? reinterpret_cast<const EntryT<W>*>(lds) : static_cast<const EntryT<W>*>(a.stab);
    const uint8_t* letters = LDS && leaf_letters<W>(a) ? lds + tab_bytes : a.letters;
    const bool leaf4 = W == 4 && a.w4_leaf;
    uint8_t* wave_lds = lds + tab_bytes + let_bytes + wave * (a.stage_bytes + row_bytes<W>());
    uint32_t* stage = reinterpret_cast<uint32_t*>(wave_lds);
    uint8_t* rows = wave_lds + a.stage_bytes;
    const bool aligned = (reinterpret_cast<uintptr_t>(a.out) & 15) == 0;
    const uint64_t nruns = (a.n + kWideRun - 1) / kWideRun;
    const uint64_t ntasks = (a.n + kTaskLetters - 1) / kTaskLetters;
    const uint32_t np_max = a.stage_bytes / 16;
    const uint32_t waves = blockDim.x / 64;
    for (uint64_t task = static_cast<uint64_t>(blockIdx.x) * waves + wave; task < ntasks;
         task += static_cast<uint64_t>(gridDim.x) * waves) {
        const uint64_t run = task * 64 + lane;
        const uint64_t l0 = run * kWideRun;
        const uint32_t cnt = l0 >= a.n ? 0u : static_cast<uint32_t>(a.n - l0 < kWideRun ? a.n - l0 : kWideRun);
        uint64_t lane_bit = !cnt ? 0 : (a.sub_abs ? a.sub_abs[run] : a.chunk_start[run >> 8] + a.sub_bit[run]);
        uint32_t skip = 0;
        if (a.skip_packed) {
            skip = static_cast<uint32_t>(lane_bit >> 48);
            lane_bit &= kSkipPosMask;
        }
        // the task's range: lane 0's start to the next task's start
        const uint32_t f_lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(lane_bit)));
        const uint32_t f_hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(lane_bit >> 32)));
        const uint64_t first = (static_cast<uint64_t>(f_hi) << 32) | f_lo;
        const uint64_t nrun = (task + 1) * 64;
        uint64_t end = nrun < nruns ? (a.sub_abs ? a.sub_abs[nrun] : a.chunk_start[nrun >> 8] + a.sub_bit[nrun])
                                    : a.end_bit;
        if (a.skip_packed && nrun < nruns)  // the next task's first letter lies within its skipped codes
            end = (end & kSkipPosMask) + (end >> 48) * a.max_len;
        const uint64_t b0 = (first >> 3) & ~15ull;
        const uint64_t b1 = ((((end + 7) >> 3) + 32) + 15) & ~15ull;  // + the window's lookahead
        const uint32_t np = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
            static_cast<int>(b1 - b0 <= 16ull * np_max ? (b1 - b0) / 16 : 0)));
        uint8_t* dst = a.out + l0 * W;
        // the transpose needs every lane of the task (wave-uniform)
        const bool whole = (task + 1) * kTaskLetters <= a.n && aligned;
        uint8_t* trows = whole ? rows : nullptr;
        uint8_t* task_out = a.out + task * kTaskLetters * W;
        if (np) {
            // stage: coalesced 16-B pieces through a buffer resource clamped to
            // the stream's last dword (pieces past it read zero)
            const uint64_t end4 = (a.comp_bytes + 3) & ~3ull;
            const uint64_t avail = end4 > b0 ? end4 - b0 : 0;
            const uint32_t nb = static_cast<uint32_t>(avail < 16ull * np ? avail : 16ull * np);
            const auto rs = buf_rsrc(nb ? a.comp + b0 : a.comp, nb);
            for (uint32_t p = lane; p < np; p += 64) {
                const uint4 v = buf_ld16(rs, p * 16);
                reinterpret_cast<uint4*>(stage)[p] = make_uint4(__builtin_bswap32(v.x), __builtin_bswap32(v.y),
                                                                __builtin_bswap32(v.z), __builtin_bswap32(v.w));
            }
            wave_sync();
            const StageWords src{stage};
            const uint32_t rel = static_cast<uint32_t>(lane_bit - b0 * 8);
            if (cnt == kWideRun)
                lane_full<W, TWO, R1>(src, rel, dst, tab, K1, letters, aligned, trows, task_out, lane, skip, leaf4);
            else if (cnt)
                lane_tail<W, TWO, R1>(src, rel, cnt, dst, tab, K1, letters, skip, leaf4);
            wave_sync();  // the stage is reused by the next task
        } else {  // longer than the stage: straight from global memory
            const GlobalWords src{a.comp, a.comp_bytes, (lane_bit >> 5)};
            const uint32_t grel = static_cast<uint32_t>(lane_bit & 31);
            if (cnt == kWideRun)
                lane_full<W, TWO, R1>(src, grel, dst, tab, K1, letters, aligned, trows, task_out, lane, skip, leaf4);
            else if (cnt)
                lane_tail<W, TWO, R1>(src, grel, cnt, dst, tab, K1, letters, skip, leaf4);
        }
    }
}

template <uint32_t W, bool LDS>
hipError_t launch_as(const WideDecArgs& a, size_t shared, uint32_t waves, hipStream_t s) {
    using Kern = void (*)(WideDecArgs);
    const bool two = a.max_len > a.stab_bits;
    const bool r1 = a.max_len > 16;
    const Kern k = !two ? k_wdec_task<W, false, false, LDS>
                        : (r1 ? k_wdec_task<W, true, true, LDS> : k_wdec_task<W, true, false, LDS>);
    const size_t lds = shared + size_t(waves) * (a.stage_bytes + row_bytes<W>());
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, waves * 64, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const uint64_t ntasks = (a.n + kTaskLetters - 1) / kTaskLetters;
    const uint64_t want = (ntasks + waves - 1) / waves;
    const uint64_t cap = uint64_t(a.cu_count ? a.cu_count : 256) * per_cu;
    const uint32_t grid = static_cast<uint32_t>(want < cap ? want : cap);
    launch_k(k, dim3(grid), dim3(waves * 64), lds, s, a);
    return hipGetLastError();
}

// the table (and wide letters) in LDS when they fit: one copy per workgroup,
// with as many waves beside it as the LDS holds (4..16)
template <uint32_t W>
hipError_t by_place(const WideDecArgs& a, hipStream_t s) {
    constexpr size_t kLds = 160 * 1024;
    const size_t tab = a.stab_bytes;
    const size_t let = leaf_letters<W>(a) ? (static_cast<size_t>(a.nleaves) * W + 15) & ~size_t(15) : 0;
    const size_t per_wave = a.stage_bytes + row_bytes<W>();
    if (tab + let <= 96 * 1024 && tab + let + 4 * per_wave <= kLds) {
        size_t waves = (kLds - tab - let) / per_wave;
        waves = waves > size_t(max_waves<W>()) ? size_t(max_waves<W>()) : waves;
        return launch_as<W, true>(a, tab + let, static_cast<uint32_t>(waves), s);
    }
    return launch_as<W, false>(a, 0, 4, s);
}

}  // namespace

hipError_t launch_wide_decode_task(const WideDecArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    if (a.max_len > 32 || a.stab_bits > 16 || a.stab_bytes % 16 || a.stage_bytes % 16 || a.stage_bytes < 1024)
        return hipErrorInvalidValue;
    switch (a.width) {
        case 1: return by_place<1>(a, s);
        case 2: return by_place<2>(a, s);
        case 4: return by_place<4>(a, s);
        case 8: return by_place<8>(a, s);
        case 16: return by_place<16>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace huff::dev
