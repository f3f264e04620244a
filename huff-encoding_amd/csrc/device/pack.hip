// pack.hip — the encode loop of compress_with_tree on the GPU
// (huff_coding/src/comp.rs:419-451: per letter, look the code up and append
// its bits MSB-first to the output bytes).
//
// Work unit: one 64 KiB chunk per WAVE, whose first output bit is known
// (chunk_start = exclusive scan of per-chunk bit counts). Workgroups are
// persistent (8 waves sharing one code table in LDS, grid sized to
// residency: 3 workgroups = 6 waves per SIMD); each wave walks its chunks in
// rounds of 1 KiB (64 lanes x 16 consecutive bytes) with no workgroup
// barrier:
//   1. 16 lookups per lane in the LDS code table, replicated 32x as
//      [letter][copy] (lane l reads copy l % 32: bank-conflict-free on any
//      data), summing the lane's bit count;
//   2. a wave-wide exclusive scan of the lanes' bit counts (DPP row shifts
//      and row broadcasts: no LDS round trips);
//   3. codes <= 27 bits: groups of G codes (G * max_len <= 32) are joined in
//      a register and ORed (ds_or) into the two 32-bit words of the wave's
//      LDS staging image they can touch, each group at its own bit offset
//      (no per-code branch, no serial dependence between groups). Codes
//      > 27 bits: a 64-bit accumulator emitting whole words;
//   4. complete 16-byte segments leave as one dwordx4 store per lane
//      (byte-swapped: the stream is MSB-first); the partial last segment is
//      carried to the next round.
// Loads run 2 rounds ahead of the encoder through a buffer resource clamped
// to the chunk (unconditional: out-of-range loads read zero), ~80 VGPRs.
// A chunk's first output byte is shared with the previous chunk: the wave
// recomputes the previous chunk's last <= 7 bits from the input bytes before
// it (from prev_tail for the first chunk of a shard), so every output byte is
// written by exactly one wave: no fix-up pass and no global atomics. Chunk c
// owns bytes [cs/8, ce/8) (the last chunk through ceil(ce/8), zero-padded as
// comp.rs:446-447 pads).
//
// Roofline: HBM-bound; algorithmic traffic n (read) + ceil(bits/8) (write).
#include "pack_emit.hpp"

namespace huff::dev {

namespace {

// waves per workgroup: 8 for short codes (one 32 KiB table shared by 8
// waves: 2 workgroups = 4 waves per SIMD fit the LDS), 4 for long codes (a
// 64 KiB table)
template <bool LONG>
constexpr int pack_waves() { return LONG ? 4 : static_cast<int>(kPackWaves); }
// consecutive input bytes per lane per round (HUFF_PACK_BPL) and rounds of
// loads in flight ahead of the encoder (HUFF_PACK_AHEAD)
#ifndef HUFF_PACK_BPL
#define HUFF_PACK_BPL 16
#endif
#ifndef HUFF_PACK_AHEAD
#define HUFF_PACK_AHEAD 2
#endif
constexpr uint32_t kBPL = HUFF_PACK_BPL;
constexpr uint32_t kRoundB = 64 * kBPL;  // bytes per wave round
constexpr int kAhead = HUFF_PACK_AHEAD;
static_assert(kBPL % 16 == 0, "lanes load whole 16-byte pieces");
static_assert(kBPL <= kIdx && kTaskSym % kRoundB == 0, "an index entry starts a lane; a task is whole rounds");
constexpr int kPieces = kBPL / 16;

struct LaneIn {
    uint4 v[kPieces];
};

// 32 lane copies of each letter's entry ([letter][copy], lane l reads copy
// l % 32: conflict-free on any data).
// (64 copies, so that letter b's address is one v_perm ((b << 8) | 4 lane)
// instead of bfe + lshl_or, measured slower: the 64 KiB table leaves 4 waves
// per SIMD instead of 6 — Zipf 0.481 vs 0.446 ms, text 0.440 vs 0.417)
#ifndef HUFF_PACK_COPIES
#define HUFF_PACK_COPIES 32
#endif
constexpr int kCopies = HUFF_PACK_COPIES;
template <bool LONG>
constexpr uint32_t table_words() { return 256u * kCopies * (LONG ? 2u : 1u); }

template <bool LONG, int G = 1>
__global__ __launch_bounds__(pack_waves<LONG>() * 64) void k_pack(PackArgs a) {
    constexpr int kWaves = pack_waves<LONG>();
    constexpr int kThreads = kWaves * 64;
    constexpr int C = kCopies;
    constexpr int LOGC = C == 32 ? 5 : C == 16 ? 4 : C == 8 ? 3 : -1;
    static_assert(LOGC > 0, "8, 16 or 32 table copies");
    using E = Entry<LONG>;
    using T = typename E::T;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    T* tab = reinterpret_cast<T*>(lds);
    // wave_index(): the chunk, its buffer resource and the round bounds are scalar
    const uint32_t t = threadIdx.x, lane = t & 63, copy = t & (C - 1), wave = wave_index();
    uint32_t* stage = lds + table_words<LONG>() + wave * a.stage_words;

    // replicate the table: thread t writes copy t % C of letters t / C + (kThreads / C) i
    const T* tg = reinterpret_cast<const T*>(LONG ? static_cast<const void*>(a.table.l) : static_cast<const void*>(a.table.s));
#pragma unroll 4
    for (int i = 0; i < 256 / (kThreads / C); ++i) {
        const uint32_t e = (t >> LOGC) + (kThreads / C) * i;
        tab[(e << LOGC) | copy] = tg[e];
    }
    for (uint32_t i = lane; i < a.stage_words; i += 64) stage[i] = 0;
    __syncthreads();

    for (uint32_t c = blockIdx.x * kWaves + wave; c < a.nchunks; c += a.grid * kWaves) {
        const uint64_t sym0 = static_cast<uint64_t>(c) * kChunk;
        const uint64_t nsym = (a.n - sym0 < kChunk) ? a.n - sym0 : kChunk;
        // the 8 input bytes before the chunk (chunks start 64 KiB apart: an
        // aligned load), read with the chunk's first loads for the shared
        // first byte below (byte-by-byte reads there waited out a memory
        // latency per byte)
        const uint64_t prev8 = (lane == 0 && sym0 >= 8) ? *reinterpret_cast<const uint64_t*>(a.in + sym0 - 8) : 0;
        const uint64_t cs = a.chunk_start[c];
        const uint64_t ce = a.chunk_start[c + 1];
        uint64_t stage_bit0 = (cs >> 7) << 7;  // global bit of stage word 0's MSB (16-B aligned)
        const uint64_t own_lo = cs >> 3;
        const uint64_t own_hi = (c + 1 == a.nchunks) ? (ce + 7) >> 3 : ce >> 3;
        const uint32_t nrounds = static_cast<uint32_t>((nsym + kRoundB - 1) / kRoundB);
        // the chunk's bytes through a buffer resource (rounded up to the 16-B
        // granule of its end: bytes past n are masked by nvalid): loads past
        // it, and whole rounds past the chunk, read zeros, so the loads run
        // 2 rounds ahead unconditionally and stay in flight
        const auto rin = buf_rsrc(a.in + sym0, static_cast<uint32_t>((nsym + 15) & ~15ull));

        auto load_round = [&](uint32_t r) {
            LaneIn x;
#pragma unroll
            for (int q = 0; q < kPieces; ++q) x.v[q] = buf_ld16(rin, r * kRoundB + lane * kBPL + 16 * q);
            return x;
        };
        LaneIn vq[kAhead];
#pragma unroll
        for (int i = 0; i < kAhead; ++i) vq[i] = load_round(i);

        // bits of the shared first byte that belong to the symbols before this chunk
        if (lane == 0 && (cs & 7)) {
            const int64_t floor8 = static_cast<int64_t>(cs & ~7ull);
            int64_t pos = static_cast<int64_t>(cs);
            for (uint32_t k = 1; k <= 8 && pos > floor8; ++k) {
                uint8_t b;
                if (sym0 >= k) {  // sym0 is 0 or >= 64 KiB
                    b = static_cast<uint8_t>(prev8 >> (8 * (8 - k)));
                } else {
                    const uint32_t j = k - static_cast<uint32_t>(sym0);
                    if (j > a.prev_tail_len) break;
                    b = a.prev_tail[8 - j];
                }
                const T ent = tab[static_cast<uint32_t>(b) << LOGC];
                const int64_t len = static_cast<int64_t>(ent & E::kMask);
                const uint64_t code = E::code(ent);
                if (len == 0) break;
                const int64_t start = pos - len;  // may precede bit 0 of out (a shard's first byte)
                for (int64_t q = (start > floor8 ? start : floor8); q < pos; ++q) {
                    if ((code >> (pos - 1 - q)) & 1) {
                        const uint64_t sb = static_cast<uint64_t>(q) - stage_bit0;
                        stage[sb >> 5] |= 0x80000000u >> (sb & 31);
                    }
                }
                pos = start;
            }
        }
        wave_sync();

        uint64_t round_bit = cs, task_bit0 = cs;
        constexpr uint32_t kRoundsPerTask = kTaskSym / kRoundB;
        for (uint32_t r = 0; r < nrounds; ++r) {
            const LaneIn v = vq[0];
#pragma unroll
            for (int i = 0; i + 1 < kAhead; ++i) vq[i] = vq[i + 1];
            vq[kAhead - 1] = load_round(r + kAhead);
            // 32-bit: a chunk holds at most 65536 symbols
            const uint32_t s_in_chunk = r * kRoundB + lane * kBPL;
            const uint32_t nsym32 = static_cast<uint32_t>(nsym);
            const int nvalid = s_in_chunk >= nsym32 ? 0
                                                    : static_cast<int>(nsym32 - s_in_chunk < kBPL ? nsym32 - s_in_chunk : kBPL);

            uint32_t bits = 0;
            uint32_t wv[4 * kPieces];
#pragma unroll
            for (int q = 0; q < kPieces; ++q) {
                wv[4 * q] = v.v[q].x;
                wv[4 * q + 1] = v.v[q].y;
                wv[4 * q + 2] = v.v[q].z;
                wv[4 * q + 3] = v.v[q].w;
            }
            T ent[kBPL];
            auto lookup = [&](int k) -> T { return tab[(((wv[k >> 2] >> (8 * (k & 3))) & 0xFFu) << LOGC) | copy]; };
            if ((r + 1ull) * kRoundB <= nsym) {  // whole round (wave-uniform): no per-letter masks
#pragma unroll
                for (int k = 0; k < static_cast<int>(kBPL); ++k) ent[k] = lookup(k);
            } else {
#pragma unroll
                for (int k = 0; k < static_cast<int>(kBPL); ++k) ent[k] = (k < nvalid) ? lookup(k) : T(0);
            }
            uint32_t Lp[kBPL / 2];  // pair lengths (SDWA) for the grouped emit
            if constexpr (!LONG && G >= 2) {
#pragma unroll
                for (int k = 0; k < static_cast<int>(kBPL / 2); ++k) {
                    Lp[k] = len2(static_cast<uint32_t>(ent[2 * k]), static_cast<uint32_t>(ent[2 * k + 1]));
                    bits += Lp[k];
                }
            } else {
#pragma unroll
                for (int k = 0; k < static_cast<int>(kBPL); ++k) bits += static_cast<uint32_t>(ent[k] & E::kMask);
            }
            // wave exclusive scan of the bit counts
            const uint32_t incl = wave_scan_incl(bits);
            const uint32_t tot = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
            const uint32_t excl = incl - bits;

            if (a.sub16) {  // compact index: a u64 base per task of 4 rounds, u16 offsets
                if ((r % kRoundsPerTask) == 0) {
                    task_bit0 = round_bit;
                    if (lane == 0) a.task_base[(sym0 + r * kRoundB) / kTaskSym] = round_bit;
                }
                if (nvalid > 0 && (s_in_chunk & (kIdx - 1)) == 0)
                    a.sub16[(sym0 + s_in_chunk) / kIdx] = static_cast<uint16_t>(round_bit - task_bit0 + excl);
            } else if (a.sub_bit && nvalid > 0 && (s_in_chunk & (kIdx - 1)) == 0) {
                a.sub_bit[(sym0 + s_in_chunk) / kIdx] = static_cast<uint32_t>(round_bit - cs + excl);
            }

            if constexpr (LONG) {
                if (bits) emit_codes<LONG, static_cast<int>(kBPL)>(stage, round_bit - stage_bit0 + excl, ent);
            } else {
                emit_codes_or<G>(stage, static_cast<uint32_t>(round_bit - stage_bit0 + excl), ent, Lp);
            }
            wave_order();

            const uint64_t end_bit = round_bit + tot;
            const bool last = (r + 1 == nrounds);
            const uint32_t nseg_done = static_cast<uint32_t>((end_bit - stage_bit0) >> 7);
            const uint32_t nseg_store = last ? static_cast<uint32_t>((end_bit - stage_bit0 + 127) >> 7) : nseg_done;
            const uint64_t sb0 = stage_bit0 >> 3;  // global byte of stage segment 0
            const uint32_t full_lo = own_lo > sb0 ? static_cast<uint32_t>((own_lo - sb0 + 15) >> 4) : 0u;
            const uint64_t hi_rel = own_hi > sb0 ? (own_hi - sb0) >> 4 : 0;
            const uint32_t full_hi = static_cast<uint32_t>(hi_rel < 0x7FFFFFFFull ? hi_rel : 0x7FFFFFFFull);
            for (uint32_t s = lane; s < nseg_store; s += 64)
                store_segment(stage, s, sb0 + 16ull * s, full_lo, full_hi, own_lo, own_hi, a.out);
            const uint32_t used_words = static_cast<uint32_t>((end_bit - stage_bit0 + 31) >> 5);
            uint32_t keep = 0;
            if (!last && lane < 4) keep = stage[nseg_done * 4 + lane];
            wave_order();
            // clear what this round wrote (16-B stores); carry the partial segment to the front
            for (uint32_t i = lane; i < (used_words + 3) / 4; i += 64)
                reinterpret_cast<uint4*>(stage)[i] = make_uint4(0, 0, 0, 0);
            wave_order();
            if (!last) {
                if (lane < 4) stage[lane] = keep;
                stage_bit0 += static_cast<uint64_t>(nseg_done) << 7;
                wave_order();
            }
            round_bit = end_bit;
        }
    }
}

}  // namespace

size_t pack_lds_bytes(bool long_codes, uint32_t max_len, uint32_t stage_words) {
    (void)max_len;
    const uint32_t table = long_codes ? table_words<true>() : table_words<false>();
    const uint32_t waves = long_codes ? pack_waves<true>() : pack_waves<false>();
    return static_cast<size_t>(table + waves * stage_words) * 4;
}

uint32_t pack_round_bytes() { return kRoundB; }

uint32_t pack_waves_per_group(bool long_codes) { return long_codes ? pack_waves<true>() : pack_waves<false>(); }

namespace {
using PackKern = void (*)(PackArgs);
PackKern pack_kernel(bool long_codes, uint32_t max_len) {
    if (long_codes) return k_pack<true>;
    if (max_len <= 8) return k_pack<false, 4>;  // 4 codes per OR pair
    if (max_len <= 16) return k_pack<false, 2>;
    return k_pack<false, 1>;
}
}  // namespace

uint32_t pack_groups_per_cu(bool long_codes, uint32_t max_len, size_t lds) {
    int per = 0;
    const int threads = (long_codes ? pack_waves<true>() : pack_waves<false>()) * 64;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pack_kernel(long_codes, max_len), threads, lds) !=
            hipSuccess ||
        per < 1) {  // the LDS bound alone
        const size_t by_lds = lds ? (160 * 1024) / lds : 8;
        per = static_cast<int>(by_lds < 1 ? 1 : by_lds > 8 ? 8 : by_lds);
    }
    return static_cast<uint32_t>(per);
}

hipError_t launch_pack(bool long_codes, const PackArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    const size_t lds = pack_lds_bytes(long_codes, a.max_len, a.stage_words);
    launch_k(pack_kernel(long_codes, a.max_len), dim3(a.grid),
             dim3((long_codes ? pack_waves<true>() : pack_waves<false>()) * 64), lds, s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
