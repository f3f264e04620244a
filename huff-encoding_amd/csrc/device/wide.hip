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
#include <type_traits>

#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;
constexpr size_t kLetterLdsMax = 32 * 1024;  // stage the decoder's leaf letters in LDS up to this

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

// stored key type: keys of <= 4 bytes are kept as u32 (host/wide.hpp wide_key_bytes)
template <typename T>
using KeyStore = std::conditional_t<(sizeof(T) < 4), uint32_t, T>;

template <typename T>
__device__ __forceinline__ KeyStore<T> to_store(T v) {
    if constexpr (sizeof(T) < 4) return static_cast<uint32_t>(v);
    else return v;
}

// host/wide.hpp wide_buckets
template <typename T>
__device__ __forceinline__ void buckets_of(T key, uint32_t lgb, uint64_t fold, uint32_t& b1, uint32_t& b2) {
    using K = KeyOps<T>;
    if constexpr (sizeof(T) <= 4) {
        const uint32_t x = static_cast<uint32_t>(K::lo(key));
        b1 = (x * 0x9E3779B1u) >> (32 - lgb);
        b2 = (x * 0x85EBCA77u + 0x165667B1u) >> (32 - lgb);
    } else {
        const uint64_t k = K::lo(key) ^ (K::hi(key) * fold);
        b1 = static_cast<uint32_t>((k * 0x9E3779B97F4A7C15ull) >> (64 - lgb));
        b2 = static_cast<uint32_t>((k * 0xD6E8FEB86659FD93ull + 0x165667B19E3779F9ull) >> (64 - lgb));
    }
}

// value of a key: the four slots of its two buckets, no loop, no branch (a
// key is stored once; empty slots hold value 0)
template <typename T, typename V>
__device__ __forceinline__ V lookup(const KeyStore<T>* keys, const V* vals, uint32_t lgs, uint64_t fold, T key) {
    using K = KeyOps<KeyStore<T>>;
    uint32_t b1, b2;
    buckets_of<T>(key, lgs - 1, fold, b1, b2);
    const KeyStore<T> k = to_store<T>(key);
    const uint32_t s1 = 2 * b1, s2 = 2 * b2;
    const KeyStore<T> k10 = keys[s1], k11 = keys[s1 + 1], k20 = keys[s2], k21 = keys[s2 + 1];
    const V v10 = vals[s1], v11 = vals[s1 + 1], v20 = vals[s2], v21 = vals[s2 + 1];
    return (K::eq(k10, k) ? v10 : V(0)) | (K::eq(k11, k) ? v11 : V(0)) | (K::eq(k20, k) ? v20 : V(0)) |
           (K::eq(k21, k) ? v21 : V(0));
}

// the values of the letters of a 16-byte vector (0 = no code)
template <typename T, typename V, uint32_t L>
__device__ __forceinline__ void probe_vec(const KeyStore<T>* keys, const V* vals, uint32_t lgs, uint64_t fold,
                                          const uint4& in, V (&e)[L]) {
#pragma unroll
    for (uint32_t j = 0; j < L; ++j) e[j] = lookup<T, V>(keys, vals, lgs, fold, KeyOps<T>::get(in, j));
}

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

// a lane's letters as 16-byte vectors, four in flight: vector q of group g
// is handed out by take(q, g) and replaced by the load of vector q of the
// next group (a run is 256 letters, so every group but the last is whole)
template <uint32_t W>
struct InRing {
    static constexpr uint32_t L = 16 / W;
    const uint8_t* p;
    uint64_t base;  // byte offset of the run
    uint32_t cnt;
    uint64_t nbytes;
    uint4 v[4];
    __device__ InRing(const uint8_t* p_, uint64_t i0, uint32_t cnt_, uint64_t nbytes_)
        : p(p_), base(i0 * W), cnt(cnt_), nbytes(nbytes_) {
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) v[q] = q * L < cnt ? load_vec(p, base + q * 16, nbytes) : make_uint4(0, 0, 0, 0);
    }
    __device__ __forceinline__ uint4 take(uint32_t q, uint32_t g) {
        const uint4 r = v[q];
        const uint32_t nx = g + 4 * L;
        if (nx < cnt) v[q] = load_vec(p, base + static_cast<uint64_t>(nx) * W, nbytes);
        return r;
    }
};

// the table, from LDS (staged here) or global memory
template <typename T, bool LDS, typename V>
__device__ __forceinline__ void table(const WideArgs& a, uint64_t* lds, const KeyStore<T>*& keys, const V*& vals) {
    if (!LDS) {
        keys = reinterpret_cast<const KeyStore<T>*>(a.keys);
        vals = static_cast<const V*>(a.vals);
        return;
    }
    const uint32_t slots = 1u << a.log2_slots;
    V* lv = reinterpret_cast<V*>(lds);
    KeyStore<T>* lk = reinterpret_cast<KeyStore<T>*>(lv + slots);
    const uint32_t vq = slots * sizeof(V) / 16, kq = slots * sizeof(KeyStore<T>) / 16;  // slots >= 64
    for (uint32_t i = threadIdx.x; i < vq; i += kThreads)
        reinterpret_cast<uint4*>(lv)[i] = static_cast<const uint4*>(a.vals)[i];
    for (uint32_t i = threadIdx.x; i < kq; i += kThreads)
        reinterpret_cast<uint4*>(lk)[i] = reinterpret_cast<const uint4*>(a.keys)[i];
    __syncthreads();
    keys = lk;
    vals = lv;
}

template <typename T, typename V>
__device__ __forceinline__ void wbits_chunk(const WideArgs& a, const KeyStore<T>* keys, const V* vals, uint32_t chunk,
                                            uint32_t* wsum) {
    constexpr uint32_t W = sizeof(T);
    constexpr uint32_t L = 16 / W;  // letters per 16-byte load
    const uint32_t t = threadIdx.x;
    const uint64_t run = static_cast<uint64_t>(chunk) * kThreads + t;
    const uint64_t i0 = run * kSub;
    const uint32_t cnt = i0 >= a.n ? 0u : static_cast<uint32_t>(a.n - i0 < kSub ? a.n - i0 : kSub);
    const uint64_t nbytes = a.n * W;
    uint32_t bits = 0;
    InRing<W> in(a.in, i0, cnt, nbytes);
    uint64_t miss = ~0ull;
    for (uint32_t g = 0; g < cnt; g += 4 * L) {
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t gg = g + q * L;
            const uint4 v = in.take(q, gg);
            V e[L];
            probe_vec<T, V, L>(keys, vals, a.log2_slots, a.fold, v, e);
#pragma unroll
            for (uint32_t j = 0; j < L; ++j) {
                const bool ok = gg + j < cnt;
                const uint64_t idx = i0 + gg + j;
                miss = (ok && e[j] == 0 && idx < miss) ? idx : miss;
                bits += ok ? static_cast<uint32_t>(e[j] & 0xFF) : 0u;
            }
        }
    }
    if (miss != ~0ull) atomicMin(a.first_missing, static_cast<unsigned long long>(miss));
    // exclusive scan of the 256 runs' bit counts
    const uint32_t lane = t & 63, wave = wave_index();
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
    if (t == 0) a.chunk_bits[chunk] = total;
}

// persistent: the table is staged once per workgroup, chunks taken in turn
template <typename T, bool LDS, typename V>
__global__ __launch_bounds__(kThreads) void k_wbits(WideArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    __shared__ uint32_t wsum[kThreads / 64];
    const KeyStore<T>* keys;
    const V* vals;
    table<T, LDS, V>(a, lds, keys, vals);
    for (uint32_t c = blockIdx.x; c < a.nchunks; c += gridDim.x) {
        wbits_chunk<T, V>(a, keys, vals, c, wsum);
        __syncthreads();  // wsum is reused
    }
}

template <typename T, typename V>
__device__ __forceinline__ void wpack_chunk(const WideArgs& a, const KeyStore<T>* keys, const V* vals, uint32_t chunk) {
    constexpr uint32_t W = sizeof(T);
    constexpr uint32_t L = 16 / W;
    const uint32_t t = threadIdx.x;
    const uint64_t run = static_cast<uint64_t>(chunk) * kThreads + t;
    const uint64_t i0 = run * kSub;
    if (i0 >= a.n) return;
    const uint32_t cnt = static_cast<uint32_t>(a.n - i0 < kSub ? a.n - i0 : kSub);
    const uint64_t nbytes = a.n * W;
    const uint64_t start = a.chunk_start[chunk] + a.sub_bit[run];
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
    InRing<W> in(a.in, i0, cnt, nbytes);
    for (uint32_t g = 0; g < cnt; g += 4 * L) {
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t gg = g + q * L;
            const uint4 v = in.take(q, gg);
            if (gg < cnt) {
                V e[L];
                probe_vec<T, V, L>(keys, vals, a.log2_slots, a.fold, v, e);
#pragma unroll
                for (uint32_t j = 0; j < L; ++j) put(gg + j < cnt ? static_cast<uint64_t>(e[j]) : 0ull, false);
            }
        }
    }
    if (skip || nacc == 0) return;  // no word starts in our run, or the last one is complete
    // complete the last word from the letters after the run (the next lanes'
    // first bits), or pad it with zeros at the end of the stream
    const T* letters = reinterpret_cast<const T*>(a.in);
    for (uint64_t i = i0 + cnt; i < a.n; ++i)
        if (put(lookup<T, V>(keys, vals, a.log2_slots, a.fold, letters[i]), true)) return;
    out[w] = __builtin_bswap32(static_cast<uint32_t>(acc << (32 - nacc)));
}

template <typename T, bool LDS, typename V>
__global__ __launch_bounds__(kThreads) void k_wpack(WideArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const KeyStore<T>* keys;
    const V* vals;
    table<T, LDS, V>(a, lds, keys, vals);
    for (uint32_t c = blockIdx.x; c < a.nchunks; c += gridDim.x) wpack_chunk<T, V>(a, keys, vals, c);
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
    uint64_t pos = a.sub_abs ? a.sub_abs[run] : a.chunk_start[chunk] + a.sub_bit[run];
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
        for (uint32_t c = blockIdx.x; c < a.nchunks; c += gridDim.x)
            wdecode_chunk<T>(a, plut, reinterpret_cast<const T*>(ll), c);
    } else {
        __syncthreads();
        for (uint32_t c = blockIdx.x; c < a.nchunks; c += gridDim.x)
            wdecode_chunk<T>(a, plut, reinterpret_cast<const T*>(a.letters), c);
    }
}

// Codes <= 32 bits (the usual case): the lane's stream in 64-byte units, the
// four 16-byte loads of the next unit issued before the current one is
// decoded and consumed at static register positions (as decode.hip
// k_decode_short), so no load result is waited for inside a branch. Letters
// of <= 4 bytes gather in a lane-private LDS row of 16 dwords and leave as one
// 64-byte piece; wider letters are stored one by one.
constexpr uint32_t kRowStride = 17;  // dwords per lane row (+1: bank spread)

template <typename T>
__device__ __forceinline__ void wdecode_short_chunk(const WideDecArgs& a, const uint32_t* plut, const T* letters,
                                                    uint32_t* rows, uint32_t chunk) {
    constexpr uint32_t W = sizeof(T);
    constexpr uint32_t per = W <= 4 ? 4 / W : 1;  // letters per dword (W <= 4)
    const uint32_t K = a.lut_bits;
    const uint32_t t = threadIdx.x;
    const uint64_t run = static_cast<uint64_t>(chunk) * kThreads + t;
    const uint64_t i0 = run * kSub;
    if (i0 >= a.n) return;
    const uint32_t cnt = static_cast<uint32_t>(a.n - i0 < kSub ? a.n - i0 : kSub);
    T* out = reinterpret_cast<T*>(a.out) + i0;
    uint32_t* row = rows + t * kRowStride;
    const uint64_t pos = a.sub_abs ? a.sub_abs[run] : a.chunk_start[chunk] + a.sub_bit[run];
    uint64_t unit = pos >> 9;
    uint32_t drop = static_cast<uint32_t>(pos & 511);
    uint4 A0 = load_vec(a.comp, unit * 64 + 0, a.comp_bytes);
    uint4 A1 = load_vec(a.comp, unit * 64 + 16, a.comp_bytes);
    uint4 A2 = load_vec(a.comp, unit * 64 + 32, a.comp_bytes);
    uint4 A3 = load_vec(a.comp, unit * 64 + 48, a.comp_bytes);
    uint64_t buf = 0;
    uint32_t nb = 0, j = 0, acc = 0;
    auto emit = [&](T v) {
        if constexpr (W <= 4) {
            acc |= static_cast<uint32_t>(v) << (8 * W * (j % per));
            if (j % per == per - 1) {
                row[(j / per) & 15] = acc;
                acc = 0;
                if ((j + 1) % (16 * per) == 0) {  // a whole row: letters [j + 1 - 16 per, j + 1)
                    uint4* d4 = reinterpret_cast<uint4*>(out + (j + 1 - 16 * per));
                    d4[0] = make_uint4(row[0], row[1], row[2], row[3]);
                    d4[1] = make_uint4(row[4], row[5], row[6], row[7]);
                    d4[2] = make_uint4(row[8], row[9], row[10], row[11]);
                    d4[3] = make_uint4(row[12], row[13], row[14], row[15]);
                }
            }
        } else {
            out[j] = v;
        }
    };
    auto dec_dword = [&](uint32_t dw) {
        if (nb < 32) {
            buf |= static_cast<uint64_t>(__builtin_bswap32(dw)) << (32 - nb);
            nb += 32;
        }
        if (drop) {
            const uint32_t k = drop < nb ? drop : nb;
            buf <<= k;
            nb -= k;
            drop -= k;
        }
        while (nb >= 32 && j < cnt) {
            uint32_t e = plut[buf >> (64 - K)];
            if (e & kLutPtr) {  // codes <= 32 bits: the window holds the whole code
                uint32_t d = K;
                do {
                    e = a.lut[(e & ~kLutPtr) + static_cast<uint32_t>((buf >> (56 - d)) & 0xFFu)];
                    d += 8;
                } while (e & kLutPtr);
            }
            const uint32_t len = (e >> 24) & 0x7Fu;
            buf <<= len;
            nb -= len;
            emit(letters[e & 0xFFFFFFu]);
            ++j;
        }
    };
    while (j < cnt) {
        ++unit;
        const uint4 B0 = load_vec(a.comp, unit * 64 + 0, a.comp_bytes);
        const uint4 B1 = load_vec(a.comp, unit * 64 + 16, a.comp_bytes);
        const uint4 B2 = load_vec(a.comp, unit * 64 + 32, a.comp_bytes);
        const uint4 B3 = load_vec(a.comp, unit * 64 + 48, a.comp_bytes);
        dec_dword(A0.x); dec_dword(A0.y); dec_dword(A0.z); dec_dword(A0.w);
        dec_dword(A1.x); dec_dword(A1.y); dec_dword(A1.z); dec_dword(A1.w);
        dec_dword(A2.x); dec_dword(A2.y); dec_dword(A2.z); dec_dword(A2.w);
        dec_dword(A3.x); dec_dword(A3.y); dec_dword(A3.z); dec_dword(A3.w);
        A0 = B0;
        A1 = B1;
        A2 = B2;
        A3 = B3;
    }
    if constexpr (W <= 4) {  // ragged end: letters [j rounded down to a row, j)
        const uint32_t rl = 16 * per;
        if (j % rl) {
            if (j % per) row[(j / per) & 15] = acc;
            for (uint32_t i = j - j % rl; i < j; ++i)
                out[i] = static_cast<T>(row[(i / per) & 15] >> (8 * W * (i % per)));
        }
    }
}

template <typename T, bool LLDS>
__global__ __launch_bounds__(kThreads) void k_wdecode_short(WideDecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t plut[];
    const uint32_t nprim = 1u << a.lut_bits;
    for (uint32_t i = threadIdx.x; i < nprim; i += kThreads) plut[i] = a.lut[i];
    const uint32_t lw = LLDS ? (a.nleaves * static_cast<uint32_t>(sizeof(T)) + 15) / 16 * 4 : 0;
    uint32_t* rows = plut + nprim + lw;
    if constexpr (LLDS) {
        uint32_t* ll = plut + nprim;
        for (uint32_t i = threadIdx.x; i < lw; i += kThreads) ll[i] = reinterpret_cast<const uint32_t*>(a.letters)[i];
        __syncthreads();
        for (uint32_t c = blockIdx.x; c < a.nchunks; c += gridDim.x)
            wdecode_short_chunk<T>(a, plut, reinterpret_cast<const T*>(ll), rows, c);
    } else {
        __syncthreads();
        for (uint32_t c = blockIdx.x; c < a.nchunks; c += gridDim.x)
            wdecode_short_chunk<T>(a, plut, reinterpret_cast<const T*>(a.letters), rows, c);
    }
}

// persistent grid: as many 256-thread workgroups as fit on the chip at once
// (LDS and the 8-workgroup-per-CU wave limit), at most one per chunk
inline uint32_t grid_for(uint32_t nchunks, uint32_t cus, size_t lds) {
    uint32_t per_cu = 8;
    if (lds) {
        const uint32_t f = static_cast<uint32_t>((160 * 1024) / (lds + 64));
        per_cu = f < 1 ? 1 : (f < 8 ? f : 8);
    }
    const uint32_t g = (cus ? cus : 256) * per_cu;
    return nchunks < g ? nchunks : g;
}

struct BitsL {
    template <typename T, bool LDS, typename V>
    static void go(const WideArgs& a, size_t lds, hipStream_t s) {
        hipLaunchKernelGGL((k_wbits<T, LDS, V>), dim3(grid_for(a.nchunks, a.cu_count, lds)), dim3(kThreads), lds, s, a);
    }
};
struct PackL {
    template <typename T, bool LDS, typename V>
    static void go(const WideArgs& a, size_t lds, hipStream_t s) {
        hipLaunchKernelGGL((k_wpack<T, LDS, V>), dim3(grid_for(a.nchunks, a.cu_count, lds)), dim3(kThreads), lds, s, a);
    }
};

template <class L, typename T>
void by_table(const WideArgs& a, hipStream_t s) {
    const size_t lds = a.table_in_lds ? wide_table_lds_bytes(a.width, a.log2_slots, a.val32) : 0;
    if (a.table_in_lds) {
        if (a.val32) L::template go<T, true, uint32_t>(a, lds, s);
        else L::template go<T, true, uint64_t>(a, lds, s);
    } else {
        if (a.val32) L::template go<T, false, uint32_t>(a, 0, s);
        else L::template go<T, false, uint64_t>(a, 0, s);
    }
}

template <class L>
hipError_t by_width(const WideArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    switch (a.width) {
        case 1: by_table<L, uint8_t>(a, s); break;
        case 2: by_table<L, uint16_t>(a, s); break;
        case 4: by_table<L, uint32_t>(a, s); break;
        case 8: by_table<L, uint64_t>(a, s); break;
        case 16: by_table<L, U128>(a, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
void decode_as(const WideDecArgs& a, hipStream_t s) {
    const size_t prim = (size_t(1) << a.lut_bits) * 4;
    const size_t lw = (static_cast<size_t>(a.nleaves) * sizeof(T) + 15) / 16 * 16;
    const bool llds = lw <= kLetterLdsMax;
    if (a.max_len <= 32) {
        const size_t rows = sizeof(T) <= 4 ? size_t(kThreads) * kRowStride * 4 : 0;
        const size_t lds = prim + (llds ? lw : 0) + rows;
        const uint32_t g = grid_for(a.nchunks, a.cu_count, lds);
        if (llds)
            hipLaunchKernelGGL((k_wdecode_short<T, true>), dim3(g), dim3(kThreads), lds, s, a);
        else
            hipLaunchKernelGGL((k_wdecode_short<T, false>), dim3(g), dim3(kThreads), lds, s, a);
        return;
    }
    if (llds)
        hipLaunchKernelGGL((k_wdecode<T, true>), dim3(grid_for(a.nchunks, a.cu_count, prim + lw)), dim3(kThreads),
                           prim + lw, s, a);
    else
        hipLaunchKernelGGL((k_wdecode<T, false>), dim3(grid_for(a.nchunks, a.cu_count, prim)), dim3(kThreads), prim,
                           s, a);
}

}  // namespace

hipError_t launch_wide_bits(const WideArgs& a, hipStream_t s) { return by_width<BitsL>(a, s); }
hipError_t launch_wide_pack(const WideArgs& a, hipStream_t s) { return by_width<PackL>(a, s); }

hipError_t launch_wide_decode(const WideDecArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
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
