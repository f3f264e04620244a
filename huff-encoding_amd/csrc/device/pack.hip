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
#include "bitreader.hpp"

namespace huff::dev {

namespace {

// waves per workgroup: 8 for short codes (one 32 KiB table shared by 8
// waves: 2 workgroups = 4 waves per SIMD fit the LDS), 4 for long codes (a
// 64 KiB table)
template <bool LONG>
constexpr int pack_waves() { return LONG ? 4 : static_cast<int>(kPackWaves); }
constexpr uint32_t kBPL = kPackWaveRound / 64;  // consecutive input bytes per lane per round
static_assert(kBPL % 16 == 0, "lanes load whole 16-byte pieces");
constexpr int kPieces = kBPL / 16;

struct LaneIn {
    uint4 v[kPieces];
};

template <bool LONG>
struct Entry;
template <>
struct Entry<false> {
    using T = uint32_t;
    static constexpr uint32_t kShift = 5;
    static constexpr uint32_t kMask = 31;
    static constexpr uint32_t kTableWords = 256 * 32;
};
template <>
struct Entry<true> {
    using T = uint64_t;
    static constexpr uint32_t kShift = 6;
    static constexpr uint32_t kMask = 63;
    static constexpr uint32_t kTableWords = 256 * 32 * 2;
};

template <bool LONG>
__device__ __forceinline__ void emit_codes(uint32_t* __restrict__ stage, uint64_t p,
                                           const typename Entry<LONG>::T (&ent)[kBPL]) {
    using E = Entry<LONG>;
    uint32_t w = static_cast<uint32_t>(p >> 5);
    uint32_t nacc = static_cast<uint32_t>(p & 31);
    bool shared_first = nacc != 0;
    uint64_t acc = 0;
    auto flush = [&]() {
        if (nacc >= 32) {
            const uint32_t word = static_cast<uint32_t>(acc >> (nacc - 32));
            if (shared_first) {
                __hip_atomic_fetch_or(&stage[w], word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                shared_first = false;
            } else {
                stage[w] = word;
            }
            ++w;
            nacc -= 32;
        }
    };
#pragma unroll
    for (int k = 0; k < static_cast<int>(kBPL); ++k) {
        const uint32_t len = static_cast<uint32_t>(ent[k] & E::kMask);
        const uint64_t code = static_cast<uint64_t>(ent[k] >> E::kShift);
        if (LONG && len > 32) {
            const uint32_t hl = len - 32;
            acc = (acc << hl) | (code >> 32);
            nacc += hl;
            flush();
            acc = (acc << 32) | (code & 0xFFFFFFFFull);
            nacc += 32;
            flush();
        } else {
            acc = (acc << len) | code;
            nacc += len;
            flush();
        }
    }
    if (nacc) {
        const uint32_t word = static_cast<uint32_t>(acc << (32 - nacc));
        __hip_atomic_fetch_or(&stage[w], word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// short codes: groups of G consecutive codes (G * max_len <= 32) are joined
// in a register and ORed into their (at most) two stage words at the group's
// bit offset: no serial 64-bit accumulator, no per-code branch. An empty
// entry past the chunk end has len 0 and code 0 and ORs zero. (Re-reading the
// entries from the table here instead of keeping them live measured 30 %
// slower.)
template <int G>
__device__ __forceinline__ void emit_codes_or(uint32_t* __restrict__ stage, uint32_t p, const uint32_t (&ent)[kBPL]) {
    uint32_t o = p;
#pragma unroll
    for (int k = 0; k < static_cast<int>(kBPL); k += G) {
        uint32_t code = 0, len = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t l = ent[k + g] & 31u;
            code = (code << l) | (ent[k + g] >> 5);
            len += l;
        }
        const uint32_t s = o & 31u;
        // the group left-aligned at bit s of a 64-bit window starting at word o/32
        const uint64_t v = static_cast<uint64_t>(code) << ((64u - s - len) & 63u);
        uint32_t* w = stage + (o >> 5);
        __hip_atomic_fetch_or(w, static_cast<uint32_t>(v >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_or(w + 1, static_cast<uint32_t>(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        o += len;
    }
}

__device__ __forceinline__ void store_segment(const uint32_t* __restrict__ stage, uint32_t s, uint64_t gbyte,
                                              uint64_t own_lo, uint64_t own_hi, uint8_t* __restrict__ out) {
    uint4 v = reinterpret_cast<const uint4*>(stage)[s];  // one ds_read_b128
    v.x = __builtin_bswap32(v.x);
    v.y = __builtin_bswap32(v.y);
    v.z = __builtin_bswap32(v.z);
    v.w = __builtin_bswap32(v.w);
    if (gbyte >= own_lo && gbyte + 16 <= own_hi) {
        *reinterpret_cast<uint4*>(out + gbyte) = v;
        return;
    }
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint64_t g = gbyte + i;
        if (g >= own_lo && g < own_hi) out[g] = static_cast<uint8_t>(wv[i >> 2] >> (8 * (i & 3)));
    }
}

template <bool LONG, int G = 1>
__global__ __launch_bounds__(pack_waves<LONG>() * 64) void k_pack(PackArgs a) {
    constexpr int kWaves = pack_waves<LONG>();
    constexpr int kThreads = kWaves * 64;
    using E = Entry<LONG>;
    using T = typename E::T;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    T* tab = reinterpret_cast<T*>(lds);
    // wave_index(): the chunk, its buffer resource and the round bounds are scalar
    const uint32_t t = threadIdx.x, lane = t & 63, copy = t & 31, wave = wave_index();
    uint32_t* stage = lds + E::kTableWords + wave * a.stage_words;

    // replicate the table: thread t writes copy t%32 of letters t/32 + 8i
    const T* tg = reinterpret_cast<const T*>(LONG ? static_cast<const void*>(a.table.l) : static_cast<const void*>(a.table.s));
#pragma unroll 4
    for (int i = 0; i < 256 / (kThreads / 32); ++i) {
        const uint32_t e = (t >> 5) + (kThreads / 32) * i;
        tab[(e << 5) | copy] = tg[e];
    }
    for (uint32_t i = lane; i < a.stage_words; i += 64) stage[i] = 0;
    __syncthreads();

    for (uint32_t c = blockIdx.x * kWaves + wave; c < a.nchunks; c += a.grid * kWaves) {
        const uint64_t sym0 = static_cast<uint64_t>(c) * kChunk;
        const uint64_t nsym = (a.n - sym0 < kChunk) ? a.n - sym0 : kChunk;
        const uint64_t cs = a.chunk_start[c];
        const uint64_t ce = a.chunk_start[c + 1];
        uint64_t stage_bit0 = (cs >> 7) << 7;  // global bit of stage word 0's MSB (16-B aligned)
        const uint64_t own_lo = cs >> 3;
        const uint64_t own_hi = (c + 1 == a.nchunks) ? (ce + 7) >> 3 : ce >> 3;
        const uint32_t nrounds = static_cast<uint32_t>((nsym + kPackWaveRound - 1) / kPackWaveRound);
        // the chunk's bytes through a buffer resource (rounded up to the 16-B
        // granule of its end: bytes past n are masked by nvalid): loads past
        // it, and whole rounds past the chunk, read zeros, so the loads run
        // 2 rounds ahead unconditionally and stay in flight
        const auto rin = buf_rsrc(a.in + sym0, static_cast<uint32_t>((nsym + 15) & ~15ull));

        auto load_round = [&](uint32_t r) {
            LaneIn x;
#pragma unroll
            for (int q = 0; q < kPieces; ++q) x.v[q] = buf_ld16(rin, r * kPackWaveRound + lane * kBPL + 16 * q);
            return x;
        };
        LaneIn v0 = load_round(0);
        LaneIn v1 = load_round(1);

        // bits of the shared first byte that belong to the symbols before this chunk
        if (lane == 0 && (cs & 7)) {
            const int64_t floor8 = static_cast<int64_t>(cs & ~7ull);
            int64_t pos = static_cast<int64_t>(cs);
            for (uint32_t k = 1; k <= 8 && pos > floor8; ++k) {
                uint8_t b;
                if (sym0 >= k) {
                    b = a.in[sym0 - k];
                } else {
                    const uint32_t j = k - static_cast<uint32_t>(sym0);
                    if (j > a.prev_tail_len) break;
                    b = a.prev_tail[8 - j];
                }
                const T ent = tab[static_cast<uint32_t>(b) << 5];
                const int64_t len = static_cast<int64_t>(ent & E::kMask);
                const uint64_t code = static_cast<uint64_t>(ent >> E::kShift);
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

        uint64_t round_bit = cs;
        for (uint32_t r = 0; r < nrounds; ++r) {
            const LaneIn v = v0;
            v0 = v1;
            v1 = load_round(r + 2);
            const uint64_t s_in_chunk = static_cast<uint64_t>(r) * kPackWaveRound + lane * kBPL;
            const int nvalid = s_in_chunk >= nsym ? 0 : (nsym - s_in_chunk >= kBPL ? static_cast<int>(kBPL)
                                                                                     : static_cast<int>(nsym - s_in_chunk));

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
            if ((r + 1ull) * kPackWaveRound <= nsym) {  // whole round (wave-uniform): no per-letter masks
#pragma unroll
                for (int k = 0; k < static_cast<int>(kBPL); ++k)
                    ent[k] = tab[(((wv[k >> 2] >> (8 * (k & 3))) & 0xFFu) << 5) | copy];
            } else {
#pragma unroll
                for (int k = 0; k < static_cast<int>(kBPL); ++k) {
                    const uint32_t b = (wv[k >> 2] >> (8 * (k & 3))) & 0xFFu;
                    ent[k] = (k < nvalid) ? tab[(b << 5) | copy] : T(0);
                }
            }
#pragma unroll
            for (int k = 0; k < static_cast<int>(kBPL); ++k) bits += static_cast<uint32_t>(ent[k] & E::kMask);
            // wave exclusive scan of the bit counts
            const uint32_t incl = wave_scan_incl(bits);
            const uint32_t tot = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
            const uint32_t excl = incl - bits;

            if (a.sub_bit && nvalid > 0 && (s_in_chunk & (kIdx - 1)) == 0)
                a.sub_bit[(sym0 + s_in_chunk) / kIdx] = static_cast<uint32_t>(round_bit - cs + excl);

            if constexpr (LONG) {
                if (bits) emit_codes<LONG>(stage, round_bit - stage_bit0 + excl, ent);
            } else {
                emit_codes_or<G>(stage, static_cast<uint32_t>(round_bit - stage_bit0 + excl), ent);
            }
            wave_sync();

            const uint64_t end_bit = round_bit + tot;
            const bool last = (r + 1 == nrounds);
            const uint32_t nseg_done = static_cast<uint32_t>((end_bit - stage_bit0) >> 7);
            const uint32_t nseg_store = last ? static_cast<uint32_t>((end_bit - stage_bit0 + 127) >> 7) : nseg_done;
            for (uint32_t s = lane; s < nseg_store; s += 64)
                store_segment(stage, s, (stage_bit0 >> 3) + 16ull * s, own_lo, own_hi, a.out);
            const uint32_t used_words = static_cast<uint32_t>((end_bit - stage_bit0 + 31) >> 5);
            uint32_t keep = 0;
            if (!last && lane < 4) keep = stage[nseg_done * 4 + lane];
            wave_sync();
            // clear what this round wrote (16-B stores); carry the partial segment to the front
            for (uint32_t i = lane; i < (used_words + 3) / 4; i += 64)
                reinterpret_cast<uint4*>(stage)[i] = make_uint4(0, 0, 0, 0);
            wave_sync();
            if (!last) {
                if (lane < 4) stage[lane] = keep;
                stage_bit0 += static_cast<uint64_t>(nseg_done) << 7;
                wave_sync();
            }
            round_bit = end_bit;
        }
    }
}

}  // namespace

size_t pack_lds_bytes(bool long_codes, uint32_t stage_words) {
    const uint32_t table = long_codes ? Entry<true>::kTableWords : Entry<false>::kTableWords;
    const uint32_t waves = long_codes ? pack_waves<true>() : pack_waves<false>();
    return static_cast<size_t>(table + waves * stage_words) * 4;
}

uint32_t pack_waves_per_group(bool long_codes) { return long_codes ? pack_waves<true>() : pack_waves<false>(); }

hipError_t launch_pack(bool long_codes, const PackArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    const size_t lds = pack_lds_bytes(long_codes, a.stage_words);
    if (long_codes) {
        hipLaunchKernelGGL(k_pack<true>, dim3(a.grid), dim3(pack_waves<true>() * 64), lds, s, a);
    } else if (a.max_len <= 8) {  // 4 codes per OR pair
        hipLaunchKernelGGL((k_pack<false, 4>), dim3(a.grid), dim3(pack_waves<false>() * 64), lds, s, a);
    } else if (a.max_len <= 16) {
        hipLaunchKernelGGL((k_pack<false, 2>), dim3(a.grid), dim3(pack_waves<false>() * 64), lds, s, a);
    } else {
        hipLaunchKernelGGL((k_pack<false, 1>), dim3(a.grid), dim3(pack_waves<false>() * 64), lds, s, a);
    }
    return hipGetLastError();
}

}  // namespace huff::dev
