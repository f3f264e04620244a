// segwalk.hpp — lane walks over a workgroup's staged bit range, shared by the
// index-free decoders (indexless.hip; the round-4 isplit.hip is gone).
//
// A workgroup's 256 consecutive segments are one contiguous bit range: it is
// staged in LDS once with coalesced 16-B loads (plus lookahead for the code
// that crosses the last segment end), and each lane then reads its bits from
// LDS: a 64-bit window refilled 32 bits at a time, single-code steps from the
// u16 single-symbol table or multi-code steps from the walk table (all
// complete codes of a K-bit window). Codes longer than the table's index go
// through the level-2 length table in LDS, else the global multi-level table.
//
// The args type `A` of the templates needs the IndexlessArgs field names:
// comp, comp_bytes, valid_bits, seg_bits, nseg (staging) and stab, stab_bits,
// wtab, l2, l2_words (tables).
#pragma once

#include "bitreader.hpp"

namespace huff::dev {

struct Staged {
    const uint32_t* w;
    uint64_t base;       // bit position of w[0]'s most significant bit
    const uint32_t* l2;  // the level-2 length table in LDS (null: the global multi-level table)
    uint32_t l2e = 0;    // > 0: its uniform form (IndexlessArgs::l2_e), else descriptors
    bool nofill = false; // every code <= 16 bits: a slow step needs no refill of its own
    bool dense = false;  // nofill, and slow windows common enough that every step reads a length
};

// The block's range from its 16-B granule, 8 loads of 16 B per lane in
// flight per batch through a buffer resource over the range rounded up to
// its last 16-B granule (pieces past it, incl. the two zero words the lanes'
// lookahead may read, come back zero): the one-dword-at-a-time loop this
// replaces waited out a memory latency per dword. Words stay in stream byte
// order (the cursor swaps them).
// the loads' results materialised here (an empty asm using them), so none
// is sunk into a later conditional use
template <int N>
__device__ __forceinline__ void keep_loads(uint4 (&v)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) asm volatile("" : "+v"(v[k].x), "+v"(v[k].y), "+v"(v[k].z), "+v"(v[k].w));
}

// lead: bits staged before the block's first segment (its first lane's
// lead-in walk, indexless.hip k_spec_lds)
template <uint32_t NSEG = 256, class A>
__device__ __forceinline__ Staged stage_block(const A& a, uint32_t* w, uint32_t lead = 0) {
    constexpr uint32_t kT = 256;  // threads
    const uint64_t seg0 = static_cast<uint64_t>(blockIdx.x) * NSEG;
    const uint64_t bit_lo = seg0 * a.seg_bits - (seg0 * a.seg_bits < lead ? seg0 * a.seg_bits : lead);
    const uint64_t seg_end = seg0 + NSEG < a.nseg ? seg0 + NSEG : a.nseg;
    const uint64_t bit_hi = seg_end * a.seg_bits < a.valid_bits ? seg_end * a.seg_bits : a.valid_bits;
    const uint64_t byte_lo = (bit_lo >> 3) & ~15ull;
    uint64_t byte_hi = ((bit_hi + 7) >> 3) + 64;  // lookahead: a chunk's overshoot past the last end
    if (byte_hi > a.comp_bytes) byte_hi = a.comp_bytes;
    const uint32_t nbytes = static_cast<uint32_t>(byte_hi - byte_lo);
    const uint32_t np = (nbytes + 8 + 15) / 16;  // + the two zero words
    const auto rs = buf_rsrc(a.comp + byte_lo, (nbytes + 15) & ~15u);
    uint4* w4 = reinterpret_cast<uint4*>(w);
    for (uint32_t p0 = threadIdx.x; p0 < np; p0 += 8 * kT) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = buf_ld16(rs, (p0 + k * kT) * 16);
        // every load issued before the first store: without this the
        // compiler sank a load into its store's branch, issued it after the
        // wait for the others, and paid a second memory latency per stage
        keep_loads(v);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (p0 + k * kT < np) w4[p0 + k * kT] = v[k];
    }
    return Staged{w, byte_lo * 8, nullptr};
}

// The staged kernels walk the stream one code per lookup in unrolled chunks
// of 8 (u16 single-symbol table in LDS, as k_decode_fixed; no branch inside a
// chunk), then settle where the walk should have stopped from the chunk's 8
// code lengths kept in registers: a data-dependent loop per code (and a slow
// path per lookup) cost ~40 VALU and ~40 SALU per step in the multi-symbol
// form this replaces (PMC: 344 K VALU per SIMD per GiB).
constexpr int kChunkSteps = 8;
// refills every 3rd / 4th step for tables of <= 10 / <= 8 bits
// (HUFF_WALK_R=0: every 2nd, for the A/B build)
#ifndef HUFF_WALK_R
#define HUFF_WALK_R 1
#endif
constexpr bool kWalkR = HUFF_WALK_R != 0;

// lane cursor over the staged range: 64-bit window, valid bits in the low 6
// bits of X (X -= entry borrows only above them), refilled unconditionally
// every two codes (the next dword is read one refill ahead)
struct Cursor {
    const uint32_t* w;
    const uint32_t* l2;
    uint64_t buf;
    uint32_t X, rp, nextw;
    uint32_t l2e;
    bool nofill, dense;
    __device__ __forceinline__ void init(const Staged& st, uint64_t p) {
        w = st.w;
        l2 = st.l2;
        l2e = st.l2e;
        nofill = st.nofill;
        dense = st.dense;
        const uint64_t rel = p - st.base;
        rp = static_cast<uint32_t>(rel >> 5);
        const uint32_t sh = static_cast<uint32_t>(rel & 31);
        buf = static_cast<uint64_t>(__builtin_bswap32(w[rp]) << sh) << 32;
        X = 32 - sh;
        rp += 1;
        nextw = __builtin_bswap32(w[rp]);
    }
    __device__ __forceinline__ void refill() {
        buf |= (static_cast<uint64_t>(nextw) << 32) >> (X & 63);
        rp += (X & 32) ? 0u : 1u;
        X |= 32;
        nextw = __builtin_bswap32(w[rp]);
    }
    // the length of the next code, consumed; codes longer than the table's
    // index (kSsSlow) through the level-2 length table in LDS (the window's
    // index in the entry's bits [0, 7) and [8, 16)), else the global
    // multi-level table. Uniform form (l2e > 0): the window's 2^l2e lengths
    // at l2e * index, one read; with every code <= 16 bits the chunk's refill
    // every two codes covers it (>= 32 valid bits then), so no refills here.
    template <bool SLOW>
    __device__ __forceinline__ uint32_t step(const uint16_t* stab, uint32_t K, const uint32_t* glut, uint32_t Kg) {
        return step_entry<SLOW>(stab[static_cast<uint32_t>(buf >> 32) >> (32 - K)], K, glut, Kg);
    }
    // the same from the window's entry already read (a walk-table entry of a
    // slow window is the single-symbol table's: the multi-code walk does not
    // read it twice)
    // dense: the length of a slow window's code read by every lane (a
    // broadcast of byte 0 for the others), no divergent branch: when most
    // steps of a wave have a slow lane anyway (wide Zipf over 4,096 letters:
    // 16 % of the codes) the branch only added its exec-mask work
    __device__ __forceinline__ uint32_t dense_len(uint32_t e, uint32_t K) const {
        const uint32_t s = (e & 0x7Fu) | ((e >> 8) << 7);
        const uint32_t j = (static_cast<uint32_t>(buf >> 32) << K) >> (32 - l2e);
        return reinterpret_cast<const uint8_t*>(l2)[(e & kSsSlow) ? (s << l2e) + j : 0u];
    }
    template <bool SLOW>
    __device__ __forceinline__ uint32_t step_entry(uint32_t e, uint32_t K, const uint32_t* glut, uint32_t Kg) {
        if (SLOW && dense) {
            const uint32_t l1 = dense_len(e, K);
            const uint32_t len = (e & kSsSlow) ? l1 : (e & 63u);
            buf <<= len;
            X -= len;
            return len;
        }
        if (SLOW && (e & kSsSlow) && l2 && l2e) {
            if (!nofill) refill();  // >= 32 valid bits: the whole code (<= 32 bits)
            const uint32_t s = (e & 0x7Fu) | ((e >> 8) << 7);
            const uint32_t j = (static_cast<uint32_t>(buf >> 32) << K) >> (32 - l2e);
            const uint32_t l1 = reinterpret_cast<const uint8_t*>(l2)[(s << l2e) + j];
            buf <<= l1;
            X -= l1;
            if (!nofill) refill();
            return l1;
        }
        if (SLOW && (e & kSsSlow) && l2) {
            refill();  // >= 32 valid bits: the whole code (<= 32 bits)
            const uint32_t d = l2[(e & 0x7Fu) | ((e >> 8) << 7)];
            const uint32_t E = d & 31u;
            const uint32_t j = (static_cast<uint32_t>(buf >> 32) << K) >> (32 - E);
            const uint32_t l1 = reinterpret_cast<const uint8_t*>(l2)[(d >> 5) + j];
            buf <<= l1;
            X -= l1;
            refill();
            return l1;
        }
        if (SLOW && (e & kSsSlow)) {
            refill();
            uint32_t e1 = glut[static_cast<uint32_t>(buf >> (64 - Kg))];
            uint32_t d = Kg;
            while (e1 & kLutPtr) {
                const uint32_t idx = static_cast<uint32_t>((buf >> (56 - d)) & 0xFFu);
                e1 = glut[(e1 & ~kLutPtr) + idx];
                d += 8;
            }
            const uint32_t l1 = (e1 >> 8) & 0xFFu;
            buf <<= l1;
            X -= l1;
            refill();
            return l1;
        }
        buf <<= (e & 63u);
        X -= e;
        return e & 63u;
    }
    // the steps of a chunk that refill first: a refill leaves >= 32 valid
    // bits and a step consumes <= K bits when no code is longer than the
    // K-bit table (K = min(depth, 12)), so every 4th step for K <= 8, every
    // 3rd for K <= 10, else every 2nd (K is wave-uniform: a scalar branch)
    __device__ __forceinline__ static uint32_t refill_steps(uint32_t K) {
        return !kWalkR || K > 10 ? 0x55u : K > 8 ? 0x49u : 0x11u;
    }
    template <bool SLOW>
    __device__ __forceinline__ void chunk(uint32_t (&L)[kChunkSteps], const uint16_t* stab, uint32_t K,
                                          const uint32_t* glut, uint32_t Kg) {
        const uint32_t rs = SLOW ? 0x55u : refill_steps(K);
#pragma unroll
        for (int k = 0; k < kChunkSteps; ++k) {
            if ((rs >> k) & 1u) refill();
            L[k] = step<SLOW>(stab, K, glut, Kg);
        }
    }
    // kChunkSteps windows, each consuming ALL its complete codes (walk table:
    // bits used, count): U bits and N codes in total, ~2 codes per lookup on
    // Zipf bytes. A window whose first code is longer than K takes that code.
    template <bool SLOW>
    __device__ __forceinline__ void multi_chunk(uint32_t& U, uint32_t& N, const uint16_t* wtab, const uint16_t* stab,
                                                uint32_t K, const uint32_t* glut, uint32_t Kg) {
        U = 0;
        N = 0;
        const uint32_t rs = SLOW ? 0x55u : refill_steps(K);
#pragma unroll
        for (int k = 0; k < kChunkSteps; ++k) {
            if ((rs >> k) & 1u) refill();
            const uint32_t e = wtab[static_cast<uint32_t>(buf >> 32) >> (32 - K)];
            if (SLOW && dense) {
                const uint32_t l1 = dense_len(e, K);
                const bool slow = (e & kSsSlow) != 0;
                const uint32_t u = slow ? l1 : (e >> 8) & 15u;
                buf <<= u;
                X -= u;
                U += u;
                N += slow ? 1u : e >> 12;
            } else if (SLOW && (e & kSsSlow)) {
                U += step_entry<SLOW>(e, K, glut, Kg);
                N += 1;
            } else {
                const uint32_t u = (e >> 8) & 15u;
                buf <<= u;
                X -= u;
                U += u;
                N += e >> 12;
            }
        }
    }
    // as above, with the running totals after each window: q[k] = U | N << 16
    template <bool SLOW>
    __device__ __forceinline__ void multi_chunk(uint32_t& U, uint32_t& N, uint32_t (&q)[kChunkSteps],
                                                const uint16_t* wtab, const uint16_t* stab, uint32_t K,
                                                const uint32_t* glut, uint32_t Kg) {
        uint32_t Q = 0;
        const uint32_t rs = SLOW ? 0x55u : refill_steps(K);
#pragma unroll
        for (int k = 0; k < kChunkSteps; ++k) {
            if ((rs >> k) & 1u) refill();
            const uint32_t e = wtab[static_cast<uint32_t>(buf >> 32) >> (32 - K)];
            if (SLOW && (e & kSsSlow)) {
                Q += step_entry<SLOW>(e, K, glut, Kg) + (1u << 16);
            } else {
                const uint32_t u = (e >> 8) & 15u;
                buf <<= u;
                X -= u;
                Q += u + ((e >> 12) << 16);
            }
            q[k] = Q;
        }
        U = Q & 0xFFFFu;
        N = Q >> 16;
    }
};

// LDS: [single-symbol table][level-2 table][staged input ...]
template <class A>
__device__ __forceinline__ uint32_t stab_words(const A& a) {
    return ((((1u << a.stab_bits) + 1) / 2) + 3) & ~3u;
}
template <class A>
__device__ __forceinline__ uint32_t tables_words(const A& a) {
    return stab_words(a) + a.l2_words;
}
// The tables in LDS by 16-B buffer loads, all of a thread's issued at once
// (issue_tables) and stored after the block's stage loads have been issued
// too (store_tables), so the table and stage latencies overlap: the loop of
// 4-B loads and LDS stores this replaces waited out an L2 round trip per
// iteration, ~8 of them per workgroup before the first code was read.
// Tables: the walk table when there is one (its low bits are stab's lengths),
// else stab (<= 8 KiB: 2 pieces per thread), then the level-2 table
// (<= kL2MaxWords: 6 pieces per thread).
constexpr uint32_t kTabPieces = 2, kL2Pieces = 6;
constexpr uint32_t kL2MaxWords = 4 * 256 * kL2Pieces;
struct TabLoad {
    uint4 t[kTabPieces];
    uint4 l[kL2Pieces];
};
template <class A>
__device__ __forceinline__ void issue_tables(const A& a, TabLoad& tl) {
    const uint32_t words = ((1u << a.stab_bits) + 1) / 2;
    const auto r1 = buf_rsrc(a.wtab ? a.wtab : a.stab, words * 4);
#pragma unroll
    for (uint32_t k = 0; k < kTabPieces; ++k) tl.t[k] = buf_ld16(r1, (threadIdx.x + 256 * k) * 16);
    if (a.l2_words) {
        const auto r2 = buf_rsrc(a.l2, a.l2_words * 4);
#pragma unroll
        for (uint32_t k = 0; k < kL2Pieces; ++k) tl.l[k] = buf_ld16(r2, (threadIdx.x + 256 * k) * 16);
    }
}
template <class A>
__device__ __forceinline__ const uint16_t* store_tables(const A& a, const TabLoad& tl, uint32_t* lds) {
    const uint32_t sp = stab_words(a) / 4, lp = (a.l2_words + 3) / 4;
    uint4* l4 = reinterpret_cast<uint4*>(lds);
#pragma unroll
    for (uint32_t k = 0; k < kTabPieces; ++k)
        if (threadIdx.x + 256 * k < sp) l4[threadIdx.x + 256 * k] = tl.t[k];
    if (a.l2_words) {
#pragma unroll
        for (uint32_t k = 0; k < kL2Pieces; ++k)
            if (threadIdx.x + 256 * k < lp) l4[sp + threadIdx.x + 256 * k] = tl.l[k];
    }
    return reinterpret_cast<const uint16_t*>(lds);
}
template <class A>
__device__ __forceinline__ const uint16_t* load_stab(const A& a, uint32_t* lds) {
    TabLoad tl;
    issue_tables(a, tl);
    return store_tables(a, tl, lds);
}
template <class A>
__device__ __forceinline__ Staged with_l2(Staged st, const A& a, const uint32_t* lds) {
    st.l2 = a.l2_words ? lds + stab_words(a) : nullptr;
    st.l2e = a.l2_words ? a.l2_e : 0u;
    st.nofill = st.l2e && a.max_len <= 16;
    st.dense = st.nofill && a.l2_dense;
    return st;
}

}  // namespace huff::dev
