// pack_emit.hpp — the code-emitting half of the encoders (pack.hip for byte
// letters, wide.hip for the wider ones): a wave's round of looked-up codes is
// appended MSB-first (comp.rs:424-444) into the wave's LDS staging image at
// the lane's bit offset, and complete 16-byte segments of the image leave as
// dwordx4 stores. N = codes per lane per round.
#pragma once

#include "bitreader.hpp"

namespace huff::dev {

// Table entries. Short codes (<= 27 bits): u32, the code LEFT-aligned (its
// first bit at bit 31) and the length in bits [0, 5): groups join with one
// shift and one and-or per code, and a group lands at bit s of its two stage
// words as (J >> s, alignbit(J, 0, s)) with no 64-bit shift. Long codes: u64
// code << 6 | len, right-aligned.
template <bool LONG>
struct Entry;
template <>
struct Entry<false> {
    using T = uint32_t;
    static constexpr uint32_t kMask = 31;
    __device__ static uint64_t code(T e) {
        const uint32_t len = e & 31u;
        return len ? e >> (32 - len) : 0u;
    }
};
template <>
struct Entry<true> {
    using T = uint64_t;
    static constexpr uint32_t kMask = 63;
    __device__ static uint64_t code(T e) { return e >> 6; }
};

// long codes: a 64-bit accumulator emitting whole words; the first word (it
// may hold bits of the previous lane) and the last partial word are ORed
template <bool LONG, int N>
__device__ __forceinline__ void emit_codes(uint32_t* __restrict__ stage, uint64_t p,
                                           const typename Entry<LONG>::T (&ent)[N]) {
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
    for (int k = 0; k < N; ++k) {
        const uint32_t len = static_cast<uint32_t>(ent[k] & E::kMask);
        const uint64_t code = E::code(ent[k]);
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
// left-aligned in a register (J = e0 & ~31 | (e1 & ~31) >> l0, the shift
// taking l0 from e0's low bits) and ORed into their (at most) two stage
// words at the group's bit offset s: J >> s and alignbit(J, 0, s) = the bits
// shifted past the first word (0 for s = 0). No 64-bit shift, no per-code
// branch; an empty entry past the end is 0 and ORs zero. (Re-reading the
// entries from the table here instead of keeping them live measured 30 %
// slower in pack.hip.)
__device__ __forceinline__ uint32_t join2(uint32_t e0, uint32_t e1) {
    // (e1 & ~31) >> (e0 & 31): v_lshrrev uses the low 5 bits of its shift
    return (e0 & ~31u) | ((e1 & ~31u) >> (e0 & 31u));
}

// the code lengths of two entries, summed by one SDWA add of their low bytes
// (codes of <= 24 bits leave bits 5-7 of an entry zero; G >= 2 means <= 16)
__device__ __forceinline__ uint32_t len2(uint32_t e0, uint32_t e1) {
    uint32_t r;
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0"
        : "=v"(r)
        : "v"(e0), "v"(e1));
    return r;
}

// Lp[i] = len2(ent[2i], ent[2i+1]) (G >= 2)
template <int G, int N>
__device__ __forceinline__ void emit_codes_or(uint32_t* __restrict__ stage, uint32_t p, const uint32_t (&ent)[N],
                                              const uint32_t (&Lp)[N / 2]) {
    const uint32_t stage_addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
        (__attribute__((address_space(3))) uint32_t*)(stage)));
    uint32_t o = p;
#pragma unroll
    for (int k = 0; k < N; k += G) {
        uint32_t J, len;
        if constexpr (G == 1) {
            J = ent[k] & ~31u;
            len = ent[k] & 31u;
        } else if constexpr (G == 2) {
            J = join2(ent[k], ent[k + 1]);
            len = Lp[k / 2];
        } else {
            static_assert(G == 4, "groups of 1, 2 or 4 codes");
            const uint32_t l01 = Lp[k / 2];
            const uint32_t J23 = join2(ent[k + 2], ent[k + 3]);
            J = join2(ent[k], ent[k + 1]) | (J23 >> l01);
            len = l01 + Lp[k / 2 + 1];
        }
        const uint32_t s = o & 31u;
        // the word's LDS address, lshr + lshl_add (opaque: the compiler's
        // canonical (o >> 3 & ~3) + base costs one more op per group)
        uint32_t wa;
        asm volatile("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(wa) : "v"(o >> 5), "v"(stage_addr));
        auto* w = (__attribute__((address_space(3))) uint32_t*)(static_cast<uintptr_t>(wa));
        __hip_atomic_fetch_or(w, J >> s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_or(w + 1, __builtin_amdgcn_alignbit(J, 0u, s), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WORKGROUP);
        o += len;
    }
}

// segment s of the stage (global bytes [gbyte, gbyte + 16)); segments
// [full_lo, full_hi) lie inside the wave's bytes [own_lo, own_hi) (wave-uniform
// 32-bit bounds), the others are stored byte by byte where owned
__device__ __forceinline__ void store_segment(const uint32_t* __restrict__ stage, uint32_t s, uint64_t gbyte,
                                              uint32_t full_lo, uint32_t full_hi, uint64_t own_lo, uint64_t own_hi,
                                              uint8_t* __restrict__ out) {
    uint4 v = reinterpret_cast<const uint4*>(stage)[s];  // one ds_read_b128
    v.x = __builtin_bswap32(v.x);
    v.y = __builtin_bswap32(v.y);
    v.z = __builtin_bswap32(v.z);
    v.w = __builtin_bswap32(v.w);
    if (s >= full_lo && s < full_hi) {
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

}  // namespace huff::dev
