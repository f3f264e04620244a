// wide.hip — encode / decode of the wider integer letters (u16 ... u128 and
// their signed twins; SURVEY.md §8f-3, letter.rs:41-60) with
// compress_with_tree / decompress semantics (comp.rs:419-451, 487-519).
//
// Layout is that of the byte path: a chunk of 65,536 letters per workgroup,
// one lane per 256-letter run, a restart index of u32 sub_bit per run and u64
// chunk_bits / chunk_start per chunk (kernels.hpp). What changes is the code
// lookup: letters are W-byte keys, so the tree's codes live in an
// open-addressing hash table (<= 50 % full, so a probe always ends), staged
// into LDS when it fits.
//
//  k_wbits   pass A: look up every letter, sum code lengths per run, scan the
//            256 runs of the chunk (-> sub_bit, chunk_bits); the first letter
//            with no code (input order) goes to first_missing (CompressError).
//  k_wpack   pass B: every lane re-emits its run's codes as 32-bit words. A
//            lane writes exactly the words whose first bit lies in its run
//            (no atomics, no zero fill): it drops the bits before its first
//            word boundary and completes its last word by looking ahead into
//            the following letters.
//  k_wdecode one lane per 256-letter run from the restart index (or from the
//            index-free decoder's sub_abs), primary table in LDS, secondary
//            tables and the leaf letters in global memory.
//
// Roofline: HBM-bound in principle (pass A reads n*W, pass B n*W + writes C);
// in practice latency-bound on the per-letter probe chain.
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;

struct U128 {
    uint64_t lo, hi;
};

template <typename T>
struct KeyOps {
    __device__ static uint64_t lo(T v) { return static_cast<uint64_t>(v); }
    __device__ static uint64_t hi(T) { return 0; }
    __device__ static bool eq(T a, T b) { return a == b; }
    // letter j of a 16-byte vector (little-endian)
    __device__ static T get(const uint4& v, uint32_t j) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        if (sizeof(T) == 8) return static_cast<T>(w[2 * j] | (static_cast<uint64_t>(w[2 * j + 1]) << 32));
        constexpr uint32_t per = 4 / (sizeof(T) < 4 ? sizeof(T) : 4);  // letters per dword
        const uint32_t word = w[j / per];
        return static_cast<T>(word >> (8 * sizeof(T) * (j % per)));
    }
};
template <>
struct KeyOps<U128> {
    __device__ static uint64_t lo(U128 v) { return v.lo; }
    __device__ static uint64_t hi(U128 v) { return v.hi; }
    __device__ static bool eq(U128 a, U128 b) { return a.lo == b.lo && a.hi == b.hi; }
    __device__ static U128 get(const uint4& v, uint32_t) {
        return {v.x | (static_cast<uint64_t>(v.y) << 32), v.z | (static_cast<uint64_t>(v.w) << 32)};
    }
};

// host/wide.hpp wide_slot
__device__ __forceinline__ uint32_t slot_of(uint64_t lo, uint64_t hi, uint32_t lg) {
    const uint64_t k = lo ^ (hi * 0xC2B2AE3D27D4EB4Full);
    return static_cast<uint32_t>((k * 0x9E3779B97F4A7C15ull) >> (64 - lg));
}

template <typename T>
__device__ __forceinline__ uint64_t probe(const T* keys, const uint64_t* vals, uint32_t lg, T key) {
    using K = KeyOps<T>;
    const uint32_t mask = (1u << lg) - 1;
    uint32_t h = slot_of(K::lo(key), K::hi(key), lg);
    for (;;) {  // the table is at most half full: an empty slot ends every probe
        const uint64_t v = vals[h];
        if (v == 0) return 0;
        if (K::eq(keys[h], key)) return v;
        h = (h + 1) & mask;
    }
}

// 16 bytes at byte offset off of a buffer of nbytes (zero past the end)
__device__ __forceinline__ uint4 load_vec(const uint8_t* __restrict__ p, uint64_t off, uint64_t nbytes) {
    if (off + 16 <= nbytes) return *reinterpret_cast<const uint4*>(p + off);
    uint32_t w[4] = {0, 0, 0, 0};
    for (int i = 0; i < 16; ++i)
        if (off + i < nbytes) w[i >> 2] |= static_cast<uint32_t>(p[off + i]) << (8 * (i & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// the table, from LDS (staged here) or global memory
template <typename T, bool LDS>
__device__ __forceinline__ void table(const WideArgs& a, uint64_t* lds, const T*& keys, const uint64_t*& vals) {
    if (!LDS) {
        keys = reinterpret_cast<const T*>(a.keys);
        vals = a.vals;
        return;
    }
    const uint32_t slots = 1u << a.log2_slots;
    uint64_t* lv = lds;
    uint8_t* lk = reinterpret_cast<uint8_t*>(lds + slots);
    for (uint32_t i = threadIdx.x; i < slots; i += kThreads) lv[i] = a.vals[i];
    const uint32_t kw = slots * sizeof(T) / 4;  // key bytes are a multiple of 4 (slots >= 64)
    for (uint32_t i = threadIdx.x; i < kw; i += kThreads)
        reinterpret_cast<uint32_t*>(lk)[i] = reinterpret_cast<const uint32_t*>(a.keys)[i];
    __syncthreads();
    keys = reinterpret_cast<const T*>(lk);
    vals = lv;
}

template <typename T, bool LDS>
__global__ __launch_bounds__(kThreads) void k_wbits(WideArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    __shared__ uint32_t wsum[kThreads / 64];
    const T* keys;
    const uint64_t* vals;
    table<T, LDS>(a, lds, keys, vals);
    constexpr uint32_t W = sizeof(T);
    constexpr uint32_t L = 16 / W;  // letters per 16-byte load
    const uint32_t t = threadIdx.x;
    const uint64_t run = static_cast<uint64_t>(blockIdx.x) * kThreads + t;
    const uint64_t i0 = run * kSub;
    const uint32_t cnt = i0 >= a.n ? 0u : static_cast<uint32_t>(a.n - i0 < kSub ? a.n - i0 : kSub);
    const uint64_t nbytes = a.n * W;
    uint32_t bits = 0;
    for (uint32_t g = 0; g < cnt; g += L) {
        const uint4 v = load_vec(a.in, (i0 + g) * W, nbytes);
#pragma unroll
        for (uint32_t j = 0; j < L; ++j) {
            if (g + j < cnt) {
                const uint64_t e = probe<T>(keys, vals, a.log2_slots, KeyOps<T>::get(v, j));
                if (e == 0) atomicMin(a.first_missing, static_cast<unsigned long long>(i0 + g + j));
                bits += static_cast<uint32_t>(e & 0xFF);
            }
        }
    }
    // exclusive scan of the 256 runs' bit counts
    const uint32_t lane = t & 63, wave = t >> 6;
    const uint32_t incl = wave_scan_incl(bits);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (uint32_t k = 0; k < kThreads / 64; ++k) {
        before += k < wave ? wsum[k] : 0u;
        total += wsum[k];
    }
    if (cnt) a.sub_bit[run] = before + incl - bits;
    if (t == 0) a.chunk_bits[blockIdx.x] = total;
}

template <typename T, bool LDS>
__global__ __launch_bounds__(kThreads) void k_wpack(WideArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const T* keys;
    const uint64_t* vals;
    table<T, LDS>(a, lds, keys, vals);
    constexpr uint32_t W = sizeof(T);
    constexpr uint32_t L = 16 / W;
    const uint32_t t = threadIdx.x;
    const uint64_t run = static_cast<uint64_t>(blockIdx.x) * kThreads + t;
    const uint64_t i0 = run * kSub;
    if (i0 >= a.n) return;
    const uint32_t cnt = static_cast<uint32_t>(a.n - i0 < kSub ? a.n - i0 : kSub);
    const uint64_t nbytes = a.n * W;
    const uint64_t start = a.chunk_start[blockIdx.x] + a.sub_bit[run];
    uint32_t skip = (32u - static_cast<uint32_t>(start & 31)) & 31u;  // bits of the word before ours
    uint64_t w = (start + 31) >> 5;                                    // first word we own
    uint64_t acc = 0;
    uint32_t nacc = 0;
    uint32_t* __restrict__ out = a.out;
    // append <= 32 bits; a completed word is stored; returns whether one was
    auto append = [&](uint64_t code, uint32_t len) -> bool {
        acc = (acc << len) | code;
        nacc += len;
        if (nacc < 32) return false;
        out[w++] = __builtin_bswap32(static_cast<uint32_t>(acc >> (nacc - 32)));
        nacc -= 32;
        return true;
    };
    // a code (<= 56 bits), minus the leading bits that belong to the word before ours
    auto put = [&](uint64_t e, bool stop_after_word) -> bool {
        uint32_t len = static_cast<uint32_t>(e & 0xFF);
        uint64_t code = e >> 8;
        if (skip) {
            if (len <= skip) {
                skip -= len;
                return false;
            }
            len -= skip;
            code &= (1ull << len) - 1;
            skip = 0;
        }
        if (len > 32) {
            if (append(code >> 32, len - 32) && stop_after_word) return true;
            return append(code & 0xFFFFFFFFull, 32);
        }
        return append(code, len);
    };
    for (uint32_t g = 0; g < cnt; g += L) {
        const uint4 v = load_vec(a.in, (i0 + g) * W, nbytes);
#pragma unroll
        for (uint32_t j = 0; j < L; ++j)
            if (g + j < cnt) put(probe<T>(keys, vals, a.log2_slots, KeyOps<T>::get(v, j)), false);
    }
    if (skip || nacc == 0) return;  // no word starts in our run, or the last one is complete
    // complete the last word from the letters after the run (the next lanes'
    // first bits), or pad it with zeros at the end of the stream
    const T* in = reinterpret_cast<const T*>(a.in);
    for (uint64_t i = i0 + cnt; i < a.n; ++i)
        if (put(probe<T>(keys, vals, a.log2_slots, in[i]), true)) return;
    out[w] = __builtin_bswap32(static_cast<uint32_t>(acc << (32 - nacc)));
}

template <typename T>
__global__ __launch_bounds__(kThreads) void k_wdecode(WideDecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t plut[];
    const uint32_t K = a.lut_bits;
    for (uint32_t i = threadIdx.x; i < (1u << K); i += kThreads) plut[i] = a.lut[i];
    __syncthreads();
    const uint32_t t = threadIdx.x;
    const uint64_t run = static_cast<uint64_t>(blockIdx.x) * kThreads + t;
    const uint64_t i0 = run * kSub;
    if (i0 >= a.n) return;
    const uint32_t cnt = static_cast<uint32_t>(a.n - i0 < kSub ? a.n - i0 : kSub);
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    const T* letters = reinterpret_cast<const T*>(a.letters);
    T* out = reinterpret_cast<T*>(a.out) + i0;
    uint64_t pos = a.sub_abs ? a.sub_abs[run] : a.chunk_start[blockIdx.x] + a.sub_bit[run];
    uint64_t wi = pos >> 5;
    uint64_t buf = ((static_cast<uint64_t>(src.word(wi)) << 32) | src.word(wi + 1)) << (pos & 31);
    uint32_t nb = 64 - static_cast<uint32_t>(pos & 31);
    wi += 2;
    for (uint32_t j = 0; j < cnt; ++j) {
        if (nb < 32) {
            buf |= static_cast<uint64_t>(src.word(wi)) << (32 - nb);
            ++wi;
            nb += 32;
        }
        uint32_t e = plut[buf >> (64 - K)];
        uint32_t len = (e >> 24) & 0x7Fu;
        if ((e & kLutPtr) || len > nb) {  // secondary tables on a fresh window
            const uint64_t win = src.window(pos);
            e = plut[win >> (64 - K)];
            uint32_t d = K;
            while (e & kLutPtr) {
                e = a.lut[(e & ~kLutPtr) + static_cast<uint32_t>((win >> (56 - d)) & 0xFFu)];
                d += 8;
            }
            len = (e >> 24) & 0x7Fu;
        }
        out[j] = letters[e & 0xFFFFFFu];
        pos += len;
        if (len <= nb) {
            buf <<= len;
            nb -= len;
        } else {  // re-seek
            wi = pos >> 5;
            buf = ((static_cast<uint64_t>(src.word(wi)) << 32) | src.word(wi + 1)) << (pos & 31);
            nb = 64 - static_cast<uint32_t>(pos & 31);
            wi += 2;
        }
    }
}

}  // namespace

size_t wide_table_lds_bytes(uint32_t width, uint32_t log2_slots) {
    return (size_t(1) << log2_slots) * (8 + width);
}

hipError_t launch_wide_bits(const WideArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    const size_t lds = a.table_in_lds ? wide_table_lds_bytes(a.width, a.log2_slots) : 0;
#define WB(T)                                                                       \
    do {                                                                            \
        if (a.table_in_lds)                                                         \
            hipLaunchKernelGGL((k_wbits<T, true>), dim3(a.nchunks), dim3(kThreads), lds, s, a); \
        else                                                                        \
            hipLaunchKernelGGL((k_wbits<T, false>), dim3(a.nchunks), dim3(kThreads), 0, s, a); \
    } while (0)
    switch (a.width) {
        case 1: WB(uint8_t); break;
        case 2: WB(uint16_t); break;
        case 4: WB(uint32_t); break;
        case 8: WB(uint64_t); break;
        case 16: WB(U128); break;
        default: return hipErrorInvalidValue;
    }
#undef WB
    return hipGetLastError();
}

hipError_t launch_wide_pack(const WideArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    const size_t lds = a.table_in_lds ? wide_table_lds_bytes(a.width, a.log2_slots) : 0;
#define WP(T)                                                                       \
    do {                                                                            \
        if (a.table_in_lds)                                                         \
            hipLaunchKernelGGL((k_wpack<T, true>), dim3(a.nchunks), dim3(kThreads), lds, s, a); \
        else                                                                        \
            hipLaunchKernelGGL((k_wpack<T, false>), dim3(a.nchunks), dim3(kThreads), 0, s, a); \
    } while (0)
    switch (a.width) {
        case 1: WP(uint8_t); break;
        case 2: WP(uint16_t); break;
        case 4: WP(uint32_t); break;
        case 8: WP(uint64_t); break;
        case 16: WP(U128); break;
        default: return hipErrorInvalidValue;
    }
#undef WP
    return hipGetLastError();
}

hipError_t launch_wide_decode(const WideDecArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    const size_t lds = (size_t(1) << a.lut_bits) * 4;
    switch (a.width) {
        case 1: hipLaunchKernelGGL(k_wdecode<uint8_t>, dim3(a.nchunks), dim3(kThreads), lds, s, a); break;
        case 2: hipLaunchKernelGGL(k_wdecode<uint16_t>, dim3(a.nchunks), dim3(kThreads), lds, s, a); break;
        case 4: hipLaunchKernelGGL(k_wdecode<uint32_t>, dim3(a.nchunks), dim3(kThreads), lds, s, a); break;
        case 8: hipLaunchKernelGGL(k_wdecode<uint64_t>, dim3(a.nchunks), dim3(kThreads), lds, s, a); break;
        case 16: hipLaunchKernelGGL(k_wdecode<U128>, dim3(a.nchunks), dim3(kThreads), lds, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace huff::dev
