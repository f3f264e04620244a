// bitreader.hpp — MSB-first bit reader + table lookup shared by the decoders.
//
// The stream is the reference's byte layout (bit i -> byte i/8, mask
// 0x80 >> (i%8)); it is read as big-endian 32-bit words into a 64-bit
// left-aligned window. A code is looked up with the top K bits in the
// primary table (LDS); longer codes follow 8-bit secondary tables in global
// memory on a freshly loaded window. Table entries: leaf = (len << 8) | letter,
// pointer = kLutPtr | index of the secondary table.
#pragma once

#include "kernels.hpp"

namespace huff::dev {

// wave-level LDS ordering: every lane's LDS ops issued before this point are
// visible to every lane of the wave after it (no workgroup barrier needed)
__device__ __forceinline__ void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// orders a wave's LDS accesses across lanes without waiting for them: the LDS
// executes one wave's DS instructions in issue order, so a later read sees an
// earlier write (or ds_or) of any lane; only the compiler must not move
// memory operations across (register results still get their own waits)
__device__ __forceinline__ void wave_order() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// 16-byte streaming load that does not pollute the caches
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Raw buffer resource over [p, p + bytes): loads at offsets past `bytes`
// return zero without touching memory (the range check is per dword), so a
// wave can issue loads for a partial or absent range unconditionally — a
// bounds-checked load (a branch with a byte-wise fallback) makes the
// compiler wait for every outstanding load right after it, which defeats
// any prefetch. Dword 3 = the gfx9 default format word.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, static_cast<int>(bytes), 0x00020000);
}
// the wave's index in its workgroup, in an SGPR: values derived from it (the
// wave's chunk or task, a buffer resource over its range) stay scalar; from a
// VGPR every buffer load over such a resource compiles to a waterfall loop
__device__ __forceinline__ uint32_t wave_index() {
    return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
}
// 16-byte buffer load; AUX 2 = nontemporal
template <int AUX = 0>
__device__ __forceinline__ uint4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(off), 0, AUX);
    return make_uint4(static_cast<uint32_t>(v[0]), static_cast<uint32_t>(v[1]), static_cast<uint32_t>(v[2]),
                      static_cast<uint32_t>(v[3]));
}

// inclusive prefix sum over the 64 lanes of a wave with DPP (no LDS round
// trips): row_shr 1/2/4/8 within each 16-lane row, then row_bcast 15 / 31
// carry the row totals upward. Lanes with no source read `old` = 0.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x111, 0xf, 0xf, false));
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x112, 0xf, 0xf, false));
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x114, 0xf, 0xf, false));
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x118, 0xf, 0xf, false));
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x142, 0xa, 0xf, false));
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x143, 0xc, 0xf, false));
    return x;
}

// 16-byte streaming store
__device__ __forceinline__ void st_nt(uint4* p, uint4 v) {
    u32x4_t w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(p));
}

// Phase stamps of a timing build (-DHUFF_STAMPS, tools/build_variant.sh; never
// in the product library): a wave keeps s_memtime at up to 8 phase
// boundaries in SGPRs and writes them, with its hardware id, to a buffer of
// its own (DecodeArgs/IndexlessArgs::stamps) by ONE vector store (lanes
// 0..9 each write one word at a lane-indexed address). Slot layout per
// wave: [0, 8) stamps, [8] HW_ID (CU / SIMD / wave slot), [9] XCC id.
#ifdef HUFF_STAMPS
struct WaveStamps {
    uint64_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void mark(int k) { t[k] = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void flush(uint64_t* buf, uint64_t wave_slot) const {
        if (!buf) return;
        const uint32_t lane = threadIdx.x & 63;
        uint64_t v = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) v = lane == static_cast<uint32_t>(k) ? t[k] : v;
        if (lane == 8) v = static_cast<uint64_t>(__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)));  // HW_ID
        if (lane == 9) v = static_cast<uint64_t>(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)));  // XCC_ID
        if (lane < 10) buf[wave_slot * 10 + lane] = v;
    }
};
#define HUFF_STAMP(ws, k) (ws).mark(k)
#else
struct WaveStamps {
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush(uint64_t*, uint64_t) const {}
};
#define HUFF_STAMP(ws, k) ((void)0)
#endif

struct BitSrc {
    const uint32_t* w;
    const uint8_t* b;
    uint64_t nbytes;

    __device__ __forceinline__ uint32_t word(uint64_t i) const {
        const uint64_t byte = i * 4;
        if (byte + 4 <= nbytes) return __builtin_bswap32(w[i]);
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
            v <<= 8;
            if (byte + k < nbytes) v |= b[byte + k];
        }
        return v;
    }
    // 64 bits starting at bit pos, left-aligned
    __device__ __forceinline__ uint64_t window(uint64_t pos) const {
        const uint64_t wi = pos >> 5;
        const uint32_t sh = static_cast<uint32_t>(pos & 31);
        const uint64_t hi = (static_cast<uint64_t>(word(wi)) << 32) | word(wi + 1);
        if (sh == 0) return hi;
        return (hi << sh) | (word(wi + 2) >> (32 - sh));
    }
};

struct Lut {
    const uint32_t* prim;  // LDS copy of the primary table
    const uint32_t* glob;  // full table in global memory (secondaries)
    uint32_t K;
};

// slow path: the code at an arbitrary bit position
__device__ __forceinline__ uint32_t lut_lookup_at(const BitSrc& src, const Lut& t, uint64_t pos) {
    const uint64_t win = src.window(pos);
    uint32_t e = t.prim[win >> (64 - t.K)];
    uint32_t d = t.K;
    while (e & kLutPtr) {
        const uint32_t idx = static_cast<uint32_t>((win >> (56 - d)) & 0xFFu);
        e = t.glob[(e & ~kLutPtr) + idx];
        d += 8;
    }
    return e;
}

struct BitReader {
    uint64_t pos, buf, wi;
    uint32_t nb;

    __device__ __forceinline__ void seek(const BitSrc& src, uint64_t p) {
        pos = p;
        wi = p >> 5;
        const uint32_t sh = static_cast<uint32_t>(p & 31);
        buf = ((static_cast<uint64_t>(src.word(wi)) << 32) | src.word(wi + 1)) << sh;
        nb = 64 - sh;
        wi += 2;
    }
    // entry of the code at pos (does not advance)
    __device__ __forceinline__ uint32_t peek(const BitSrc& src, const Lut& t) {
        if (nb < 32) {
            buf |= static_cast<uint64_t>(src.word(wi)) << (32 - nb);
            ++wi;
            nb += 32;
        }
        const uint32_t e = t.prim[buf >> (64 - t.K)];
        if ((e & kLutPtr) || ((e >> 8) & 0xFFu) > nb) return lut_lookup_at(src, t, pos);
        return e;
    }
    __device__ __forceinline__ void advance(const BitSrc& src, uint32_t len) {
        if (len <= nb) {
            buf <<= len;
            nb -= len;
            pos += len;
        } else {
            seek(src, pos + len);
        }
    }
};

}  // namespace huff::dev
