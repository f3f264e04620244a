// wide.hip — encode / decode of the wider integer letters (u16 ... u128 and
// their signed twins; SURVEY.md §8f-3, letter.rs:41-60) with
// compress_with_tree / decompress semantics (comp.rs:419-451, 487-519).
//
// Encode is the byte path's two passes (pass 1 + pack, pack.hip) with the
// code lookup in a cuckoo hash table instead of a 256-entry array. Work unit:
// one wide chunk of kWideChunk = 16,384 letters per WAVE; 16 waves per
// workgroup share the table in LDS (when it fits, else it is read from L2).
// Every round a wave reads 1 KiB (W = 1) or 2 KiB of letters, 16 or 32
// consecutive bytes per lane (coalesced dwordx4, two rounds in flight through
// a buffer resource clamped to the chunk: loads past it read zero).
//
//  lookup    a letter is in one of two slots (host/wide.hpp wide_slots: two
//            multiplicative hashes of its 32-bit hash key, reduced to the
//            table size by a high multiply). Slots are {key, value} in one
//            ds_read_b64 (keys of <= 4 bytes, short codes) or _b128. All the
//            lane's first slots are read; then the second slots of the
//            letters that missed, with every other lane reading slot 0 (one
//            broadcast address): the second read costs only the misses'
//            bank conflicts. The host inserts letters shortest code first,
//            so frequent letters sit in their first slot.
//  k_wbits   pass 1: per-lane code-length sums and a wave scan per round;
//            the first lane of every run of kWideRun = 64 letters stores the
//            run's start (sub_bit, relative to the chunk start), the round
//            total carries into the next; chunk_bits at the end. The first
//            letter with no code (input order) goes to first_missing
//            (CompressError, comp.rs:426-432).
//  k_wpack   pass 2 (pack.hip's scheme, pack_emit.hpp): a wave scan of the
//            round's lengths gives each lane its bit offset; the codes are
//            ORed into the wave's LDS staging image (short codes in groups of
//            G per OR pair), whole 16-byte segments leave as dwordx4 stores.
//            A chunk owns output bytes [cs / 8, ce / 8) (the last one through
//            ceil(ce / 8)); the bits of its first byte that belong to the
//            letters before it are recomputed from those letters, so no byte
//            is written twice and the output needs no zero fill. Any output
//            alignment: the image is aligned to the 16-byte granule below.
//  k_wdecode codes longer than 32 bits (or a task-decoder table over 4 Mi
//            entries): one lane per 256-letter run from the restart index (or
//            the index-free decoder's sub_abs), primary table in LDS,
//            secondary tables and the leaf letters in global memory. Codes of
//            <= 32 bits: the task decoder of wdecode.hip.
//
// Roofline: HBM-bound. Pass 1 reads n W bytes, pass 2 n W + writes C.
#include <type_traits>

#include "pack_emit.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;    // decoder workgroup
constexpr int kEncWaves = 16;    // encoder workgroup: waves sharing one LDS table
constexpr size_t kLetterLdsMax = 32 * 1024;  // stage the decoder's leaf letters in LDS up to this

struct U128 {
    uint64_t lo, hi;
};

// ---------------------------------------------------------------------------
// code table (host/wide.hpp wide_slot_layout)
template <uint32_t W>
using KeyT = std::conditional_t<(W <= 4), uint32_t, std::conditional_t<(W == 8), uint64_t, U128>>;

template <typename K, typename V>
struct Slot;
template <>
struct alignas(8) Slot<uint32_t, uint32_t> {
    uint32_t key, val;
};
template <>
struct alignas(16) Slot<uint32_t, uint64_t> {
    uint32_t key, pad;
    uint64_t val;
};
template <>
struct alignas(16) Slot<uint64_t, uint32_t> {
    uint64_t key;
    uint32_t val, pad;
};
template <>
struct alignas(16) Slot<uint64_t, uint64_t> {
    uint64_t key, val;
};
template <>
struct alignas(16) Slot<U128, uint32_t> {
    U128 key;
    uint32_t val, pad[3];
};
template <>
struct alignas(16) Slot<U128, uint64_t> {
    U128 key;
    uint64_t val, pad;
};
static_assert(sizeof(Slot<uint32_t, uint32_t>) == 8 && sizeof(Slot<uint32_t, uint64_t>) == 16 &&
                  sizeof(Slot<uint64_t, uint32_t>) == 16 && sizeof(Slot<U128, uint64_t>) == 32,
              "slots as host/wide.hpp wide_slot_layout");

__device__ __forceinline__ bool key_eq(uint32_t a, uint32_t b) { return a == b; }
__device__ __forceinline__ bool key_eq(uint64_t a, uint64_t b) { return a == b; }
__device__ __forceinline__ bool key_eq(U128 a, U128 b) { return a.lo == b.lo && a.hi == b.hi; }

// host/wide.hpp wide_hkey
template <uint32_t W>
__device__ __forceinline__ uint32_t hkey(KeyT<W> k, uint64_t fold) {
    if constexpr (W <= 4) {
        return k;
    } else if constexpr (W == 8) {
        return static_cast<uint32_t>((k * fold) >> 32);
    } else {
        const uint64_t x = k.lo ^ (k.hi * fold);
        return static_cast<uint32_t>((x * fold) >> 32);
    }
}

// host/wide.hpp wide_slots. Generic: h = x * mul, s1 = high half of h *
// slots (two quarter-rate multiplies). Narrow (keys < 2^16, slots < 65536):
// h = x * mul on 24 bits, s1 = ((h >> 8) * (slots << 8)) >> 32, both full-rate
// 24-bit multiplies. s2 = s1 ^ bits 8..15 of h (slots a multiple of 256).
// Direct (keys < 2^16, slots = 65536): s1 = s2 = x.
enum : uint32_t { kHashGeneric = 0, kHashNarrow = 1, kHashDirect = 2 };
__device__ __forceinline__ void wslots(uint32_t x, uint32_t mul, uint32_t slots, uint32_t mode, uint32_t& s1,
                                       uint32_t& s2) {
    uint32_t h;
    if (mode == kHashNarrow) {
        h = __umul24(x, mul);
        s1 = static_cast<uint32_t>((static_cast<uint64_t>(h >> 8) * ((slots << 8) & 0xFFFFFFu)) >> 32);
    } else if (mode == kHashDirect) {
        s1 = s2 = x;
        return;
    } else {
        h = x * mul;
        s1 = __umulhi(h, slots);
    }
    s2 = s1 ^ ((h >> 8) & 255u);
}

template <uint32_t W, typename V>
struct Tab {
    const Slot<KeyT<W>, V>* s;
    uint32_t slots, mul1, mode;
    uint64_t fold;
};

// the values of N letters (0 = no code), two reads per letter as above.
// Selects as masks: a select between two loaded values is otherwise turned
// into a load from a selected address (flat, through scratch).
template <typename V>
__device__ __forceinline__ V keep_if(bool c, V v) {
    return v & (V(0) - V(c));
}
template <uint32_t W, typename V, int B>
__device__ __forceinline__ void lookup_group(const Tab<W, V>& t, const KeyT<W>* key, V* val) {
    using S = Slot<KeyT<W>, V>;
    uint32_t s1[B], s2[B];
#pragma unroll
    for (int k = 0; k < B; ++k) wslots(hkey<W>(key[k], t.fold), t.mul1, t.slots, t.mode, s1[k], s2[k]);
    S e1[B];
#pragma unroll
    for (int k = 0; k < B; ++k) e1[k] = t.s[s1[k]];
    // an empty slot's key is no letter of the table (host/wide.hpp), so a
    // key match alone means the slot holds the letter
    bool m1[B];
    uint32_t a2[B];
#pragma unroll
    for (int k = 0; k < B; ++k) {
        m1[k] = key_eq(e1[k].key, key[k]);
        a2[k] = m1[k] ? 0u : s2[k];
    }
    S e2[B];
#pragma unroll
    for (int k = 0; k < B; ++k) e2[k] = t.s[a2[k]];
#pragma unroll
    for (int k = 0; k < B; ++k) val[k] = m1[k] ? e1[k].val : keep_if(key_eq(e2[k].key, key[k]), e2[k].val);
}
// in groups of <= 8 letters (4 with long values and small keys): the
// slots of a group are in flight together
template <uint32_t W, typename V, int N>
__device__ __forceinline__ void lookup_n(const Tab<W, V>& t, const KeyT<W> (&key)[N], V (&val)[N]) {
    constexpr int B0 = sizeof(V) == 8 && W <= 2 ? 4 : 8;
    constexpr int B = N < B0 ? N : B0;
#pragma unroll
    for (int g = 0; g < N; g += B) lookup_group<W, V, B>(t, key + g, val + g);
}

// bytes of letters per lane per round, and the round
// lane bytes per round (16 or 32) of pass 1 and pass 2 by letter width, and
// the rounds of loads in flight ahead of the encoder (tuning knobs)
#ifndef WIDE_LB_BITS2
#define WIDE_LB_BITS2 32
#endif
#ifndef WIDE_LB_BITS4
#define WIDE_LB_BITS4 32
#endif
#ifndef WIDE_LB_PACK2
#define WIDE_LB_PACK2 32
#endif
#ifndef WIDE_LB_PACK4
#define WIDE_LB_PACK4 32
#endif
#ifndef WIDE_BITS_AHEAD
#define WIDE_BITS_AHEAD 2
#endif
#ifndef WIDE_PACK_AHEAD
#define WIDE_PACK_AHEAD 2
#endif
#ifndef WIDE_BITS_WAVES
#define WIDE_BITS_WAVES 1
#endif
template <uint32_t W, bool PACK>
constexpr uint32_t lane_bytes() {
    if constexpr (W == 1) return 16u;
    if constexpr (W == 2) return PACK ? WIDE_LB_PACK2 : WIDE_LB_BITS2;
    if constexpr (W == 4) return PACK ? WIDE_LB_PACK4 : WIDE_LB_BITS4;
    return 32u;
}
template <uint32_t LB>
struct LaneIn {
    uint4 v[LB / 16];
};
template <uint32_t LB>
__device__ __forceinline__ LaneIn<LB> load_round(__amdgpu_buffer_rsrc_t r, uint32_t round, uint32_t lane) {
    LaneIn<LB> x;
#pragma unroll
    for (uint32_t q = 0; q < LB / 16; ++q) x.v[q] = buf_ld16(r, round * 64 * LB + lane * LB + 16 * q);
    return x;
}

// letter k of the lane's bytes
template <uint32_t W, int NW>
__device__ __forceinline__ KeyT<W> letter_of(const uint32_t (&w)[NW], int k) {
    if constexpr (W == 1) {
        return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
    } else if constexpr (W == 2) {
        return (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
    } else if constexpr (W == 4) {
        return w[k];
    } else if constexpr (W == 8) {
        return w[2 * k] | (static_cast<uint64_t>(w[2 * k + 1]) << 32);
    } else {
        return U128{w[4 * k] | (static_cast<uint64_t>(w[4 * k + 1]) << 32),
                    w[4 * k + 2] | (static_cast<uint64_t>(w[4 * k + 3]) << 32)};
    }
}

template <uint32_t W>
__device__ __forceinline__ KeyT<W> letter_at(const uint8_t* __restrict__ in, uint64_t i) {
    if constexpr (W == 1) return in[i];
    else if constexpr (W == 2) return reinterpret_cast<const uint16_t*>(in)[i];
    else if constexpr (W == 4) return reinterpret_cast<const uint32_t*>(in)[i];
    else if constexpr (W == 8) return reinterpret_cast<const uint64_t*>(in)[i];
    else return U128{reinterpret_cast<const uint64_t*>(in)[2 * i], reinterpret_cast<const uint64_t*>(in)[2 * i + 1]};
}

template <typename V>
__device__ __forceinline__ uint32_t len_of(V v) {
    return static_cast<uint32_t>(v) & (sizeof(V) == 8 ? 63u : 31u);
}

__host__ __device__ constexpr uint32_t table_lds_bytes(uint32_t slots, uint32_t slot_bytes) {
    return (slots * slot_bytes + 15u) & ~15u;
}

// the table: copied into LDS (the host pads it to 16 bytes), or read in place
template <uint32_t W, typename V, bool LDS>
__device__ __forceinline__ Tab<W, V> stage_table(const WideArgs& a, uint8_t* lds) {
    using S = Slot<KeyT<W>, V>;
    // the hash form: compile-time for wide keys and for tables in LDS (those
    // of 16-bit keys are always narrow), else the table's
    const uint32_t mode = W > 2 ? kHashGeneric : (LDS ? kHashNarrow : a.hash_mode);
    Tab<W, V> t{nullptr, a.slots, a.mul1, mode, a.fold};
    if constexpr (LDS) {
        const uint32_t q = table_lds_bytes(a.slots, a.slot_bytes) / 16;
        for (uint32_t i = threadIdx.x; i < q; i += blockDim.x)
            reinterpret_cast<uint4*>(lds)[i] = static_cast<const uint4*>(a.table)[i];
        t.s = reinterpret_cast<const S*>(lds);
    } else {
        t.s = static_cast<const S*>(a.table);
    }
    return t;
}

// ---------------------------------------------------------------------------
// pass 1
template <uint32_t W, typename V, bool LDS>
__global__ __launch_bounds__(kEncWaves * 64) __attribute__((amdgpu_waves_per_eu(WIDE_BITS_WAVES, 8))) void k_wbits(WideArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t wlds[];
    constexpr uint32_t LB = lane_bytes<W, false>(), RB = 64 * LB;
    constexpr int N = static_cast<int>(LB / W);
    const Tab<W, V> tab = stage_table<W, V, LDS>(a, wlds);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = wave_index();
    unsigned long long first_miss = ~0ull;
    for (uint32_t c = blockIdx.x * kEncWaves + wave; c < a.nchunks; c += gridDim.x * kEncWaves) {
        const uint64_t i0 = static_cast<uint64_t>(c) * kWideChunk;
        const uint32_t cnt = static_cast<uint32_t>(a.n - i0 < kWideChunk ? a.n - i0 : kWideChunk);
        const auto rin = buf_rsrc(a.in + i0 * W, (cnt * W + 15) & ~15u);
        const uint32_t nrounds = (cnt * W + RB - 1) / RB;
        LaneIn<LB> v0 = load_round<LB>(rin, 0, lane);
#if WIDE_BITS_AHEAD > 1
        LaneIn<LB> v1 = load_round<LB>(rin, 1, lane);
#endif
        uint32_t round_base = 0;  // code bits of the chunk before this round
        for (uint32_t r = 0; r < nrounds; ++r) {
            const LaneIn<LB> v = v0;
#if WIDE_BITS_AHEAD > 1
            v0 = v1;
            v1 = load_round<LB>(rin, r + 2, lane);
#else
            v0 = load_round<LB>(rin, r + 1, lane);
#endif
            uint32_t w[LB / 4];
#pragma unroll
            for (uint32_t q = 0; q < LB / 16; ++q) {
                w[4 * q] = v.v[q].x;
                w[4 * q + 1] = v.v[q].y;
                w[4 * q + 2] = v.v[q].z;
                w[4 * q + 3] = v.v[q].w;
            }
            KeyT<W> key[N];
#pragma unroll
            for (int k = 0; k < N; ++k) key[k] = letter_of<W>(w, k);
            V val[N];
            lookup_n<W, V, N>(tab, key, val);
            const uint32_t l0 = (r * RB + lane * LB) / W;  // the lane's first letter in the chunk
            if ((r + 1) * RB > cnt * W) {  // the chunk's last round (wave-uniform): letters past the end count nothing
#pragma unroll
                for (int k = 0; k < N; ++k) val[k] = l0 + k < cnt ? val[k] : V(1u << 31);  // length 0, not missing
            }
            // the code lengths (two per add3) and the smallest value: 0 = a
            // letter without a code (rare: then its index is looked for)
            uint32_t bits = 0;
            V lowest = val[0];
#pragma unroll
            for (int k = 0; k + 1 < N; k += 2) {
                bits += len_of(val[k]) + len_of(val[k + 1]);
                lowest = min(lowest, min(val[k], val[k + 1]));
            }
            if constexpr (N & 1) {
                bits += len_of(val[N - 1]);
                lowest = min(lowest, val[N - 1]);
            }
            if (lowest == 0) {
                uint32_t k = 0;
                while (val[k] != 0) ++k;
                const uint64_t i = i0 + l0 + k;
                first_miss = i < first_miss ? i : first_miss;
            }
            // the restart index: every run of kWideRun letters starts at a
            // lane (LPR lanes per run); the run's first lane stores its start
            const uint32_t incl = wave_scan_incl(bits);
            constexpr uint32_t LPR = kWideRun * W / LB;  // lanes per run
            static_assert(LPR >= 1 && 64 % LPR == 0, "whole runs per round");
            if (lane % LPR == 0 && l0 < cnt)
                a.sub_bit[static_cast<uint64_t>(c) * (kWideChunk / kWideRun) + l0 / kWideRun] = round_base + incl - bits;
            round_base += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
        }
        if (lane == 0) a.chunk_bits[c] = round_base;
    }
    if (first_miss != ~0ull) atomicMin(a.first_missing, first_miss);
}

// ---------------------------------------------------------------------------
// pass 2
template <uint32_t W, typename V, bool LDS, int G>
__global__ __launch_bounds__(kEncWaves * 64) void k_wpack(WideArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t wlds[];
    constexpr bool LONG = sizeof(V) == 8;
    constexpr uint32_t LB = lane_bytes<W, true>(), RB = 64 * LB;
    constexpr int N = static_cast<int>(LB / W);
    using E = Entry<LONG>;
    const Tab<W, V> tab = stage_table<W, V, LDS>(a, wlds);
    const uint32_t lane = threadIdx.x & 63, wave = wave_index();
    uint32_t* stage = reinterpret_cast<uint32_t*>(wlds + (LDS ? table_lds_bytes(a.slots, a.slot_bytes) : 0u)) +
                      wave * a.stage_words;
    for (uint32_t i = lane; i < a.stage_words; i += 64) stage[i] = 0;
    __syncthreads();
    // the output as 16-byte granules: bit b of the stream is bit b + 8 mis of base
    const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a.out) & 15);
    uint8_t* const base = a.out - mis;

    for (uint32_t c = blockIdx.x * kEncWaves + wave; c < a.nchunks; c += gridDim.x * kEncWaves) {
        const uint64_t i0 = static_cast<uint64_t>(c) * kWideChunk;
        const uint32_t cnt = static_cast<uint32_t>(a.n - i0 < kWideChunk ? a.n - i0 : kWideChunk);
        const auto rin = buf_rsrc(a.in + i0 * W, (cnt * W + 15) & ~15u);
        const uint32_t nrounds = (cnt * W + RB - 1) / RB;
        const uint64_t cs = a.chunk_start[c] + 8ull * mis;
        const uint64_t ce = a.chunk_start[c + 1] + 8ull * mis;
        uint64_t stage_bit0 = (cs >> 7) << 7;  // bit of base at stage word 0's MSB (16-B aligned)
        const uint64_t own_lo = cs >> 3;
        const uint64_t own_hi = (c + 1 == a.nchunks) ? (ce + 7) >> 3 : ce >> 3;
        LaneIn<LB> v0 = load_round<LB>(rin, 0, lane);
#if WIDE_PACK_AHEAD > 1
        LaneIn<LB> v1 = load_round<LB>(rin, 1, lane);
#endif

        // bits of the shared first byte that belong to the letters before the chunk
        if (lane == 0 && (cs & 7)) {
            const int64_t floor8 = static_cast<int64_t>(cs & ~7ull);
            int64_t pos = static_cast<int64_t>(cs);
            for (uint64_t k = 1; k <= 8 && k <= i0 && pos > floor8; ++k) {
                const KeyT<W> key[1] = {letter_at<W>(a.in, i0 - k)};
                V val[1];
                lookup_n<W, V, 1>(tab, key, val);
                const int64_t len = static_cast<int64_t>(len_of(val[0]));
                const uint64_t code = E::code(static_cast<typename E::T>(val[0]));
                if (len == 0) break;
                const int64_t start = pos - len;
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

        uint64_t round_bit = cs;
        for (uint32_t r = 0; r < nrounds; ++r) {
            const LaneIn<LB> v = v0;
#if WIDE_PACK_AHEAD > 1
            v0 = v1;
            v1 = load_round<LB>(rin, r + 2, lane);
#else
            v0 = load_round<LB>(rin, r + 1, lane);
#endif
            uint32_t w[LB / 4];
#pragma unroll
            for (uint32_t q = 0; q < LB / 16; ++q) {
                w[4 * q] = v.v[q].x;
                w[4 * q + 1] = v.v[q].y;
                w[4 * q + 2] = v.v[q].z;
                w[4 * q + 3] = v.v[q].w;
            }
            KeyT<W> key[N];
#pragma unroll
            for (int k = 0; k < N; ++k) key[k] = letter_of<W>(w, k);
            V ent[N];
            lookup_n<W, V, N>(tab, key, ent);
            const uint32_t l0 = (r * RB + lane * LB) / W;
            if ((r + 1) * RB > cnt * W) {  // the chunk's last round (wave-uniform): letters past the end emit nothing
#pragma unroll
                for (int k = 0; k < N; ++k) ent[k] = l0 + k < cnt ? ent[k] : V(0);
            }
            uint32_t bits = 0;
            uint32_t Lp[N / 2];  // pair lengths (SDWA) for the grouped emit
            if constexpr (!LONG && G >= 2) {
#pragma unroll
                for (int k = 0; k < N / 2; ++k) {
                    Lp[k] = len2(ent[2 * k], ent[2 * k + 1]);
                    bits += Lp[k];
                }
            } else {
#pragma unroll
                for (int k = 0; k < N; ++k) bits += len_of(ent[k]);
            }
            const uint32_t incl = wave_scan_incl(bits);
            const uint32_t tot = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
            const uint32_t excl = incl - bits;
            if constexpr (LONG) {
                if (bits) emit_codes<true, N>(stage, round_bit - stage_bit0 + excl, ent);
            } else {
                emit_codes_or<G, N>(stage, static_cast<uint32_t>(round_bit - stage_bit0 + excl), ent, Lp);
            }
            wave_order();

            const uint64_t end_bit = round_bit + tot;
            const bool last = (r + 1 == nrounds);
            const uint32_t nseg_done = static_cast<uint32_t>((end_bit - stage_bit0) >> 7);
            const uint32_t nseg_store = last ? static_cast<uint32_t>((end_bit - stage_bit0 + 127) >> 7) : nseg_done;
            const uint64_t sb0 = stage_bit0 >> 3;  // byte of base at stage segment 0
            const uint32_t full_lo = own_lo > sb0 ? static_cast<uint32_t>((own_lo - sb0 + 15) >> 4) : 0u;
            const uint64_t hi_rel = own_hi > sb0 ? (own_hi - sb0) >> 4 : 0;
            const uint32_t full_hi = static_cast<uint32_t>(hi_rel < 0x7FFFFFFFull ? hi_rel : 0x7FFFFFFFull);
            for (uint32_t s = lane; s < nseg_store; s += 64)
                store_segment(stage, s, sb0 + 16ull * s, full_lo, full_hi, own_lo, own_hi, base);
            const uint32_t used_words = static_cast<uint32_t>((end_bit - stage_bit0 + 31) >> 5);
            uint32_t keep = 0;
            if (!last && lane < 4) keep = stage[nseg_done * 4 + lane];
            wave_order();
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

// ---------------------------------------------------------------------------
// decode

// the last partial 16 bytes of a buffer (zero past the end); out of line:
// it runs once per stream end and would otherwise be inlined at every load
__device__ __attribute__((noinline)) uint4 load_tail(const uint8_t* __restrict__ p, uint64_t off, uint64_t nbytes) {
    uint32_t w[4] = {0, 0, 0, 0};
    for (int i = 0; i < 16; ++i)
        if (off + i < nbytes) w[i >> 2] |= static_cast<uint32_t>(p[off + i]) << (8 * (i & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// 16 bytes at byte offset off of a buffer of nbytes (zero past the end)
__device__ __forceinline__ uint4 load_vec(const uint8_t* __restrict__ p, uint64_t off, uint64_t nbytes) {
    if (off + 16 <= nbytes) return *reinterpret_cast<const uint4*>(p + off);
    return load_tail(p, off, nbytes);
}

// workgroups of 256 runs (4 wide chunks)
__device__ __forceinline__ uint32_t dec_groups(const WideDecArgs& a) {
    return static_cast<uint32_t>((a.n + uint64_t(kThreads) * kSub - 1) / (uint64_t(kThreads) * kSub));
}
inline uint32_t dec_groups_host(const WideDecArgs& a) {
    return static_cast<uint32_t>((a.n + uint64_t(kThreads) * kSub - 1) / (uint64_t(kThreads) * kSub));
}

// letter j of a 16-byte vector of letters
template <typename T>
__device__ __forceinline__ void put_letter(uint32_t (&w)[4], uint32_t j, T v) {
    if constexpr (sizeof(T) >= 4) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
        for (uint32_t k = 0; k < sizeof(T) / 4; ++k) w[j * (sizeof(T) / 4) + k] = p[k];
    } else {
        constexpr uint32_t per = 4 / sizeof(T);
        const uint32_t sh = 8 * sizeof(T) * (j % per);
        w[j / per] |= static_cast<uint32_t>(v) << sh;
    }
}

template <typename T>
__device__ __forceinline__ void wdecode_chunk(const WideDecArgs& a, const uint32_t* plut, const T* letters,
                                              uint32_t chunk) {
    const uint32_t K = a.lut_bits;
    const uint32_t t = threadIdx.x;
    const uint64_t run = static_cast<uint64_t>(chunk) * kThreads + t;
    const uint64_t i0 = run * kSub;
    if (i0 >= a.n) return;
    const uint32_t cnt = static_cast<uint32_t>(a.n - i0 < kSub ? a.n - i0 : kSub);
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    T* out = reinterpret_cast<T*>(a.out) + i0;
    uint64_t pos = a.sub_abs ? a.sub_abs[run * 4] : a.chunk_start[run >> 6] + a.sub_bit[run * 4];
    // the lane's stream through a 4 x 16-byte register ring (48 bytes in
    // flight ahead of the dword being consumed), as decode.hip k_decode
    uint4 cur, n1, n2, n3;
    uint64_t slot = 0;
    uint32_t k = 0;
    auto seek = [&](uint64_t p) {
        const uint64_t dw = p >> 5;
        slot = dw >> 2;
        k = static_cast<uint32_t>(dw & 3);
        cur = load_vec(a.comp, slot * 16, a.comp_bytes);
        n1 = load_vec(a.comp, slot * 16 + 16, a.comp_bytes);
        n2 = load_vec(a.comp, slot * 16 + 32, a.comp_bytes);
        n3 = load_vec(a.comp, slot * 16 + 48, a.comp_bytes);
    };
    auto dword = [&]() -> uint32_t {
        if (k == 4) {
            cur = n1;
            n1 = n2;
            n2 = n3;
            n3 = load_vec(a.comp, (slot + 4) * 16, a.comp_bytes);
            ++slot;
            k = 0;
        }
        const uint32_t d = k == 0 ? cur.x : (k == 1 ? cur.y : (k == 2 ? cur.z : cur.w));
        ++k;
        return __builtin_bswap32(d);
    };
    uint64_t buf = 0;
    uint32_t nb = 0;
    auto start_at = [&](uint64_t p) {
        seek(p);
        const uint32_t sh = static_cast<uint32_t>(p & 31);
        buf = (static_cast<uint64_t>(dword()) << 32) << sh;
        nb = 32 - sh;
        if (nb < 32) {
            buf |= static_cast<uint64_t>(dword()) << (32 - nb);
            nb += 32;
        }
    };
    start_at(pos);
    auto next = [&]() -> T {
        if (nb < 32) {
            buf |= static_cast<uint64_t>(dword()) << (32 - nb);
            nb += 32;
        }
        uint32_t e = plut[buf >> (64 - K)];
        uint32_t d = K;
        while (e & kLutPtr) {  // secondaries on the window: exact for codes <= nb bits
            e = a.lut[(e & ~kLutPtr) + static_cast<uint32_t>((buf >> (56 - d)) & 0xFFu)];
            d += 8;
        }
        uint32_t len = (e >> 24) & 0x7Fu;
        if (len > nb) {  // a code longer than the window: look it up afresh, re-seek
            const uint64_t win = src.window(pos);
            e = plut[win >> (64 - K)];
            d = K;
            while (e & kLutPtr) {
                e = a.lut[(e & ~kLutPtr) + static_cast<uint32_t>((win >> (56 - d)) & 0xFFu)];
                d += 8;
            }
            len = (e >> 24) & 0x7Fu;
            pos += len;
            start_at(pos);
        } else {
            buf <<= len;
            nb -= len;
            pos += len;
        }
        return letters[e & 0xFFFFFFu];
    };
    constexpr uint32_t L = 16 / sizeof(T);  // letters per 16-byte store
    uint32_t j = 0;
    if ((reinterpret_cast<uintptr_t>(out) & 15) == 0) {
        for (; j + L <= cnt; j += L) {
            uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
            for (uint32_t k = 0; k < L; ++k) put_letter<T>(w, k, next());
            *reinterpret_cast<uint4*>(out + j) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
    for (; j < cnt; ++j) out[j] = next();
}

template <typename T, bool LLDS>
__global__ __launch_bounds__(kThreads) void k_wdecode(WideDecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t plut[];
    const uint32_t nprim = 1u << a.lut_bits;
    for (uint32_t i = threadIdx.x; i < nprim; i += kThreads) plut[i] = a.lut[i];
    // one pointer origin per instantiation, so the loads compile to ds_read
    // (LDS) or global_load, never to flat loads
    if constexpr (LLDS) {  // the leaf letters too (a.nleaves * W <= kLetterLdsMax)
        uint32_t* ll = plut + nprim;
        const uint32_t words = (a.nleaves * static_cast<uint32_t>(sizeof(T)) + 3) / 4;
        for (uint32_t i = threadIdx.x; i < words; i += kThreads) ll[i] = reinterpret_cast<const uint32_t*>(a.letters)[i];
        __syncthreads();
        for (uint32_t c = blockIdx.x; c < dec_groups(a); c += gridDim.x)
            wdecode_chunk<T>(a, plut, reinterpret_cast<const T*>(ll), c);
    } else {
        __syncthreads();
        for (uint32_t c = blockIdx.x; c < dec_groups(a); c += gridDim.x)
            wdecode_chunk<T>(a, plut, reinterpret_cast<const T*>(a.letters), c);
    }
}

// persistent grid: as many 256-thread workgroups as fit on the chip at once
// (LDS and the 8-workgroup-per-CU wave limit), at most one per group
inline uint32_t grid_for(uint32_t ngroups, uint32_t cus, size_t lds) {
    uint32_t per_cu = 8;
    if (lds) {
        const uint32_t f = static_cast<uint32_t>((160 * 1024) / (lds + 64));
        per_cu = f < 1 ? 1 : (f < 8 ? f : 8);
    }
    const uint32_t g = (cus ? cus : 256) * per_cu;
    return ngroups < g ? ngroups : g;
}

// encoder grid: 1024-thread workgroups, at most 2 per CU (32 waves), fewer
// where the LDS table and stages do not fit twice
inline uint32_t enc_grid(const WideArgs& a, size_t lds) {
    const uint32_t per_cu = lds * 2 + 2048 <= 160 * 1024 ? 2u : 1u;
    const uint32_t g = (a.cu_count ? a.cu_count : 256) * per_cu;
    const uint32_t need = (a.nchunks + kEncWaves - 1) / kEncWaves;
    return need < g ? need : g;
}

template <typename K>
hipError_t allow_lds(K kernel, size_t lds) {
    if (lds <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024);
}

template <uint32_t W, typename V, bool LDS>
hipError_t bits_go(const WideArgs& a, hipStream_t s) {
    const size_t lds = wide_lds_bytes(a, false, LDS);
    static const hipError_t attr = allow_lds(k_wbits<W, V, LDS>, 128 * 1024);
    if (attr != hipSuccess) return attr;
    launch_k((k_wbits<W, V, LDS>), dim3(enc_grid(a, lds)), dim3(kEncWaves * 64), lds, s, a);
    return hipGetLastError();
}

template <uint32_t W, typename V, bool LDS, int G>
hipError_t pack_go(const WideArgs& a, hipStream_t s) {
    const size_t lds = wide_lds_bytes(a, true, LDS);
    static const hipError_t attr = allow_lds(k_wpack<W, V, LDS, G>, 128 * 1024);
    if (attr != hipSuccess) return attr;
    launch_k((k_wpack<W, V, LDS, G>), dim3(enc_grid(a, lds)), dim3(kEncWaves * 64), lds, s, a);
    return hipGetLastError();
}

template <uint32_t W, bool PACK>
hipError_t enc_as(const WideArgs& a, hipStream_t s) {
    if constexpr (!PACK) {
        if (a.long_codes) return a.table_in_lds ? bits_go<W, uint64_t, true>(a, s) : bits_go<W, uint64_t, false>(a, s);
        return a.table_in_lds ? bits_go<W, uint32_t, true>(a, s) : bits_go<W, uint32_t, false>(a, s);
    } else {
        if (a.long_codes)
            return a.table_in_lds ? pack_go<W, uint64_t, true, 1>(a, s) : pack_go<W, uint64_t, false, 1>(a, s);
        if constexpr (W <= 4) {  // groups of codes per OR pair, as pack.hip
            if (a.max_len <= 8)
                return a.table_in_lds ? pack_go<W, uint32_t, true, 4>(a, s) : pack_go<W, uint32_t, false, 4>(a, s);
            if (a.max_len <= 16)
                return a.table_in_lds ? pack_go<W, uint32_t, true, 2>(a, s) : pack_go<W, uint32_t, false, 2>(a, s);
        }
        return a.table_in_lds ? pack_go<W, uint32_t, true, 1>(a, s) : pack_go<W, uint32_t, false, 1>(a, s);
    }
}

template <bool PACK>
hipError_t by_width(const WideArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    if (a.table_in_lds && wide_lds_bytes(a, PACK, true) > kWideLdsMax) return hipErrorInvalidValue;
    switch (a.width) {
        case 1: return enc_as<1, PACK>(a, s);
        case 2: return enc_as<2, PACK>(a, s);
        case 4: return enc_as<4, PACK>(a, s);
        case 8: return enc_as<8, PACK>(a, s);
        case 16: return enc_as<16, PACK>(a, s);
        default: return hipErrorInvalidValue;
    }
}

template <typename T>
void decode_as(const WideDecArgs& a, hipStream_t s) {
    const size_t prim = (size_t(1) << a.lut_bits) * 4;
    const size_t lw = (static_cast<size_t>(a.nleaves) * sizeof(T) + 15) / 16 * 16;
    if (lw <= kLetterLdsMax)
        launch_k((k_wdecode<T, true>), dim3(grid_for(dec_groups_host(a), a.cu_count, prim + lw)), dim3(kThreads),
                           prim + lw, s, a);
    else
        launch_k((k_wdecode<T, false>), dim3(grid_for(dec_groups_host(a), a.cu_count, prim)), dim3(kThreads), prim,
                           s, a);
}

}  // namespace

size_t wide_lds_bytes(const WideArgs& a, bool pack_pass, bool in_lds) {
    return (in_lds ? table_lds_bytes(a.slots, a.slot_bytes) : 0) +
           (pack_pass ? size_t(kEncWaves) * a.stage_words * 4 : 0);
}

uint32_t wide_stage_words(uint32_t width, uint32_t max_len) {
    const uint32_t lb = width == 1 ? 16u : width == 2 ? WIDE_LB_PACK2 : width == 4 ? WIDE_LB_PACK4 : 32u;
    const uint32_t letters = 64u * lb / width;  // per round
    return (letters / 32 * (max_len ? max_len : 1) + 12 + 3) & ~3u;
}

hipError_t launch_wide_bits(const WideArgs& a, hipStream_t s) { return by_width<false>(a, s); }
hipError_t launch_wide_pack(const WideArgs& a, hipStream_t s) { return by_width<true>(a, s); }

hipError_t launch_wide_decode(const WideDecArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    switch (a.width) {
        case 1: decode_as<uint8_t>(a, s); break;
        case 2: decode_as<uint16_t>(a, s); break;
        case 4: decode_as<uint32_t>(a, s); break;
        case 8: decode_as<uint64_t>(a, s); break;
        case 16: decode_as<U128>(a, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace huff::dev
