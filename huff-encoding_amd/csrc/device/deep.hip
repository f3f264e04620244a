// deep.hip — codes longer than 57 bits (up to 255: a 256-leaf tree's depth).
//
// The reference's codes are unbounded bit vectors (tree_inner.rs:422-440),
// so compress_with_tree (comp.rs:419-451) and decompress (comp.rs:487-519)
// accept any tree, including the Fibonacci-weighted ones whose depth exceeds
// the 57-bit table entries of pack.hip / decode*.hip. Such trees are rare
// (they need letters whose counts grow like Fibonacci numbers), so this path
// is correct first and simple:
//  k_pack_deep   : one wave per 64 KiB chunk, rounds of 64 lanes x 16 bytes
//                  as k_pack (lengths in LDS, DPP scan of the lanes' bit
//                  counts, the restart index every kIdx symbols), each code
//                  ORed into the zeroed output with 32-bit global atomics
//                  from its left-aligned words (LDS, 8 words per letter);
//  k_decode_deep : per lane kIdx symbols from the restart index, codes looked
//                  up in the multi-level table (primary K bits in LDS, 8-bit
//                  secondaries in global memory) on 64-bit windows re-read at
//                  every level, so any depth resolves;
//  k_decode_deep_serial : streams without an index (reference-written bytes,
//                  .hff files): one lane walks the whole stream.
// Two small helpers of the file path's windowed decode live here too, as they
// walk codes of any length: k_walk_end (the end of a window's last complete
// code) and k_shift_bits (realign a window that starts inside a byte).
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kDeepWaves = 4;
constexpr uint32_t kDeepBPL = 16;  // input bytes per lane per round

// the left-aligned 32 code bits at code offset o (may be negative) of letter
// b: words[b*8 + q] hold code bits [32q, 32q + 32), zero past the code
__device__ __forceinline__ uint32_t code_bits_at(const uint32_t* words, uint32_t b, int32_t o) {
    const int32_t q = o >> 5;  // floor
    const uint32_t r = static_cast<uint32_t>(o) & 31u;
    const uint32_t w0 = (q >= 0 && q < static_cast<int32_t>(kDeepWords)) ? words[b * kDeepWords + q] : 0u;
    const uint32_t w1 = (q + 1 >= 0 && q + 1 < static_cast<int32_t>(kDeepWords)) ? words[b * kDeepWords + q + 1] : 0u;
    return r ? (w0 << r) | (w1 >> (32 - r)) : w0;
}

__global__ __launch_bounds__(kDeepWaves * 64) void k_pack_deep(DeepPackArgs a) {
    __shared__ uint32_t len_s[256];
    __shared__ uint32_t words_s[256 * kDeepWords];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = wave_index();
    for (uint32_t i = t; i < 256; i += blockDim.x) len_s[i] = a.len.len[i];
    for (uint32_t i = t; i < 256 * kDeepWords; i += blockDim.x) words_s[i] = a.words[i];
    __syncthreads();
    // output words: bit g of the stream (relative to out) is bit g + off0 of
    // the 4-B aligned base
    const uintptr_t ob = reinterpret_cast<uintptr_t>(a.out);
    unsigned int* wbase = reinterpret_cast<unsigned int*>(ob & ~uintptr_t(3));
    const uint64_t off0 = 8 * (ob & 3);
    for (uint32_t c = blockIdx.x * kDeepWaves + wave; c < a.nchunks; c += gridDim.x * kDeepWaves) {
        const uint64_t sym0 = static_cast<uint64_t>(c) * kChunk;
        const uint64_t nsym = (a.n - sym0 < kChunk) ? a.n - sym0 : kChunk;
        const uint64_t cs = a.chunk_start[c];
        uint64_t round_bit = cs;
        const uint32_t rounds = static_cast<uint32_t>((nsym + 64 * kDeepBPL - 1) / (64 * kDeepBPL));
        for (uint32_t r = 0; r < rounds; ++r) {
            const uint64_t s_in = static_cast<uint64_t>(r) * 64 * kDeepBPL + lane * kDeepBPL;
            const uint32_t nv = s_in >= nsym ? 0u : static_cast<uint32_t>(nsym - s_in < kDeepBPL ? nsym - s_in : kDeepBPL);
            uint8_t b[kDeepBPL];
            uint32_t bits = 0;
#pragma unroll
            for (uint32_t k = 0; k < kDeepBPL; ++k) {
                b[k] = k < nv ? a.in[sym0 + s_in + k] : 0;
                bits += k < nv ? len_s[b[k]] : 0u;
            }
            const uint32_t incl = wave_scan_incl(bits);
            const uint32_t tot = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
            uint64_t p = round_bit + (incl - bits);
            if (a.sub_bit && nv > 0 && (s_in & (kIdx - 1)) == 0)
                a.sub_bit[(sym0 + s_in) / kIdx] = static_cast<uint32_t>(p - cs);
            for (uint32_t k = 0; k < nv; ++k) {
                const uint32_t L = len_s[b[k]];
                const uint64_t P = p + off0;  // code's first bit in the aligned word grid
                for (uint64_t d = P >> 5; d <= (P + L - 1) >> 5; ++d) {
                    const int32_t o = static_cast<int32_t>(static_cast<int64_t>(32 * d) - static_cast<int64_t>(P));
                    const uint32_t v = code_bits_at(words_s, b[k], o);
                    if (v) atomicOr(wbase + d, __builtin_bswap32(v));
                }
                p += L;
            }
            round_bit += tot;
        }
    }
}

// the table entry of the code at `pos`: primary K bits (LDS), then 8-bit
// secondaries, each level on a window re-read at its own offset
__device__ __forceinline__ uint32_t deep_lookup(const BitSrc& src, const uint32_t* prim, uint32_t K,
                                                const uint32_t* glut, uint64_t pos) {
    uint32_t e = prim[static_cast<uint32_t>(src.window(pos) >> (64 - K))];
    uint64_t d = K;
    while (e & kLutPtr) {
        const uint32_t idx = static_cast<uint32_t>(src.window(pos + d) >> 56);
        e = glut[(e & ~kLutPtr) + idx];
        d += 8;
    }
    return e;  // (total length << 8) | letter
}

__global__ __launch_bounds__(256) void k_decode_deep(DecodeArgs a) {
    extern __shared__ uint32_t prim[];
    for (uint32_t i = threadIdx.x; i < (1u << a.lut_bits); i += blockDim.x) prim[i] = a.lut[i];
    __syncthreads();
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    const uint64_t ngroups = (a.n + kIdx - 1) / kIdx;
    for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < ngroups;
         g += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        const uint64_t s0 = g * kIdx;
        const uint32_t cnt = static_cast<uint32_t>(a.n - s0 < kIdx ? a.n - s0 : kIdx);
        uint64_t pos = a.chunk_start[s0 / kChunk] + a.sub_bit[g];
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t e = deep_lookup(src, prim, a.lut_bits, a.lut, pos);
            a.out[s0 + j] = static_cast<uint8_t>(e);
            pos += (e >> 8) & 0xFFu;
        }
    }
}

// one lane: every code of [0, valid_bits), an incomplete final code dropped
// (comp.rs:493-516); *count = symbols, only the first `cap` are written
__global__ void k_decode_deep_serial(DeepSerialArgs a) {
    extern __shared__ uint32_t prim[];
    for (uint32_t i = threadIdx.x; i < (1u << a.lut_bits); i += blockDim.x) prim[i] = a.lut[i];
    __syncthreads();
    if (threadIdx.x != 0) return;
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    uint64_t pos = 0, n = 0;
    while (pos < a.valid_bits) {
        const uint32_t e = deep_lookup(src, prim, a.lut_bits, a.lut, pos);
        const uint32_t len = (e >> 8) & 0xFFu;
        if (pos + len > a.valid_bits) break;
        if (n < a.cap) a.out[n] = static_cast<uint8_t>(e);
        ++n;
        pos += len;
    }
    *a.count = n;
    if (a.end) *a.end = pos;
}

// the bit after `count` codes from the boundary *start (or start_v when
// start is null): the end of a window's last complete code, for the file
// path's windowed decode
__global__ void k_walk_end(WalkEndArgs a) {
    extern __shared__ uint32_t prim[];
    for (uint32_t i = threadIdx.x; i < (1u << a.lut_bits); i += blockDim.x) prim[i] = a.lut[i];
    __syncthreads();
    if (threadIdx.x != 0) return;
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    uint64_t pos = a.start ? *a.start : a.start_v;
    uint64_t cnt = a.count ? *a.count : a.count_v;
    if (a.start_packed) {  // a k_mark_lite entry: boundary | codes to skip << 48
        cnt += pos >> 48;
        pos &= kSkipPosMask;
    }
    for (uint64_t j = 0; j < cnt; ++j) pos += (deep_lookup(src, prim, a.lut_bits, a.lut, pos) >> 8) & 0xFFu;
    *a.end = pos;
}

// dst[i] = the 8 stream bits starting at bit r of src[i] (a window that
// starts inside a byte, realigned to bit 0)
__global__ void k_shift_bits(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t n, uint32_t r) {
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        const uint32_t hi = src[i], lo = i + 1 < n ? src[i + 1] : 0u;
        dst[i] = static_cast<uint8_t>((hi << r) | (lo >> (8 - r)));
    }
}

}  // namespace

hipError_t launch_walk_end(const WalkEndArgs& a, hipStream_t s) {
    launch_k(k_walk_end, dim3(1), dim3(64), (1u << a.lut_bits) * 4, s, a);
    return hipGetLastError();
}

hipError_t launch_shift_bits(const uint8_t* src, uint8_t* dst, uint64_t n, uint32_t r, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t want = (n + 255) / 256;
    launch_k(k_shift_bits, dim3(static_cast<uint32_t>(want < 8192 ? want : 8192)), dim3(256), 0, s, src,
                       dst, n, r);
    return hipGetLastError();
}

hipError_t launch_pack_deep(const DeepPackArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    const uint32_t grid = (a.nchunks + kDeepWaves - 1) / kDeepWaves;
    launch_k(k_pack_deep, dim3(grid < 4096 ? grid : 4096), dim3(kDeepWaves * 64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_decode_deep(const DecodeArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const uint64_t groups = (a.n + kIdx - 1) / kIdx;
    const uint64_t want = (groups + 255) / 256;
    launch_k(k_decode_deep, dim3(static_cast<uint32_t>(want < 4096 ? want : 4096)), dim3(256),
                       (1u << a.lut_bits) * 4, s, a);
    return hipGetLastError();
}

hipError_t launch_decode_deep_serial(const DeepSerialArgs& a, hipStream_t s) {
    launch_k(k_decode_deep_serial, dim3(1), dim3(64), (1u << a.lut_bits) * 4, s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
