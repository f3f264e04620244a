// decode_ring.hip — restart-index decode, multi-symbol, with batched ring
// maintenance (comp.rs:487-519 semantics; the restart index and the chunk
// layout are those of decode.hip).
//
// One workgroup per 65,536-symbol chunk, one lane per 256-symbol run, as in
// decode.hip. What differs is how a lane is fed and drained, arranged so that
// every lane executes the same instruction stream (the decode loop has no
// per-lane rare events, which on a 64-wide wave turn into a branch taken
// almost every iteration):
//  - the lane's compressed bits come from a 16-dword ring in LDS, read one
//    dword per 32 bits consumed (the read of the next dword is issued a refill
//    ahead); a 32-byte register buffer B holds the next half-ring, loaded
//    from HBM two halves ahead of use;
//  - one lookup of the top K (= 12) window bits in the multi-symbol table
//    (LDS) yields up to 3 letters and the bits they use; a code longer than
//    K bits (only when the tree has one: template SLOW) goes through the
//    single-symbol tables;
//  - letters gather in a 64-bit accumulator; every lookup writes its low
//    dword into a 16-dword output ring in LDS;
//  - every 8 lookups, a lane that has consumed a half of its input ring gets
//    B written into it (and reloads B), and a lane with a complete half of
//    output stores it as one 32-byte piece. Rates bound the work between two
//    such points (<= 96 bits in, <= 24 letters out), so one half per point
//    suffices.
// Lanes may decode past their 256 letters in their last round (reading the
// next lane's bits); nothing past a lane's count is ever stored.
//
// Roofline: HBM-bound in principle (ceil(bits/8) read + n written); in
// practice issue-bound: ~25-35 instructions per lookup.
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;
constexpr uint32_t kRing = 18;  // dwords per lane row (16 used; 8-B aligned, bank-spread)

// 32-byte half-unit h of the stream (dword-guarded at the end)
__device__ __forceinline__ void load_half(const uint8_t* __restrict__ comp, uint64_t nbytes, uint64_t h, uint4& p,
                                          uint4& q) {
    const uint64_t b = h * 32;
    if (b + 32 <= nbytes) {
        const uint4* s = reinterpret_cast<const uint4*>(comp + b);
        p = s[0];
        q = s[1];
    } else {
        const uint32_t* s = reinterpret_cast<const uint32_t*>(comp + b);
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = (b + 4 * i < nbytes) ? s[i] : 0u;
        p = make_uint4(w[0], w[1], w[2], w[3]);
        q = make_uint4(w[4], w[5], w[6], w[7]);
    }
}

__device__ __forceinline__ void put_half(uint32_t* row, uint32_t slot, const uint4& p, const uint4& q) {
    uint2* r = reinterpret_cast<uint2*>(row + slot);  // slot is 0 or 8: 8-B aligned
    r[0] = make_uint2(p.x, p.y);
    r[1] = make_uint2(p.z, p.w);
    r[2] = make_uint2(q.x, q.y);
    r[3] = make_uint2(q.z, q.w);
}

template <bool SLOW>
__global__ __launch_bounds__(kThreads) void k_decode_ring(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t K = a.mlut_bits;
    const uint32_t nent = 1u << K;
    uint32_t* mlut = lds;
    uint32_t* inr = lds + nent;
    uint32_t* outr = inr + kThreads * kRing;
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < nent; i += kThreads) mlut[i] = a.mlut[i];

    const uint32_t c = blockIdx.x;
    const uint64_t sym0 = static_cast<uint64_t>(c) * kChunk;
    const uint64_t nsym = (a.n - sym0 < kChunk) ? a.n - sym0 : kChunk;
    const uint64_t lsym0 = static_cast<uint64_t>(t) * kSub;
    const uint32_t cnt = lsym0 >= nsym ? 0u : static_cast<uint32_t>(nsym - lsym0 < kSub ? nsym - lsym0 : kSub);
    uint32_t* ir = inr + t * kRing;
    uint32_t* orw = outr + t * kRing;

    uint64_t pos = 0;
    uint64_t h0 = 0;
    uint4 Bp, Bq;
    if (cnt) {
        pos = a.sub_abs ? a.sub_abs[(sym0 + lsym0) / kSub] : a.chunk_start[c] + a.sub_bit[(sym0 + lsym0) / kIdx];
        h0 = pos >> 8;  // first 32-byte half
        uint4 p, q;
        load_half(a.comp, a.comp_bytes, h0, p, q);
        put_half(ir, 0, p, q);
        load_half(a.comp, a.comp_bytes, h0 + 1, p, q);
        put_half(ir, 8, p, q);
        load_half(a.comp, a.comp_bytes, h0 + 2, Bp, Bq);
    }
    __syncthreads();  // table staged (rings are lane-private)
    if (cnt == 0) return;

    const uint32_t Ks = a.lut_bits;
    const uint32_t* glut = a.lut;
    uint8_t* dst = a.out + sym0 + lsym0;
    uint32_t rp = static_cast<uint32_t>(pos & 255) >> 5;  // next ring dword (absolute, from half h0)
    uint32_t filled = 16;                                 // ring holds dwords [filled - 16, filled)
    uint32_t nextw = ir[rp & 15];
    uint64_t buf = 0;
    uint32_t nb = 0;

#define RING_REFILL()                                                                   \
    do {                                                                                \
        const bool need_ = nb < 32;                                                     \
        const uint64_t add_ = static_cast<uint64_t>(__builtin_bswap32(nextw)) << ((32 - nb) & 63); \
        buf |= need_ ? add_ : 0ull;                                                     \
        nb += need_ ? 32u : 0u;                                                         \
        rp += need_ ? 1u : 0u;                                                          \
        nextw = ir[rp & 15];                                                            \
    } while (0)

    RING_REFILL();
    {
        const uint32_t sh = static_cast<uint32_t>(pos & 31);
        buf <<= sh;
        nb -= sh;
    }
    uint64_t acc = 0;
    uint32_t fill8 = 0, wp = 0, flushed = 0, j = 0;
    const uint32_t flush_lim = cnt >> 2;  // complete output dwords of this lane

#define RING_LOOKUP()                                                                   \
    do {                                                                                \
        uint32_t e = mlut[static_cast<uint32_t>(buf >> (64 - K))];                      \
        if (SLOW && (e & kMsSlow)) {                                                    \
            RING_REFILL();                                                              \
            uint32_t e1 = glut[static_cast<uint32_t>(buf >> (64 - Ks))];                \
            uint32_t d = Ks;                                                            \
            while (e1 & kLutPtr) {                                                      \
                const uint32_t idx = static_cast<uint32_t>((buf >> (56 - d)) & 0xFFu);  \
                e1 = glut[(e1 & ~kLutPtr) + idx];                                       \
                d += 8;                                                                 \
            }                                                                           \
            e = (e1 & 0xFFu) | (((e1 >> 8) & 0xFFu) << 24) | (1u << 29);                \
        }                                                                               \
        const uint32_t used = (e >> 24) & 31u;                                          \
        const uint32_t cn = e >> 29;                                                    \
        buf <<= used;                                                                   \
        nb -= used;                                                                     \
        acc |= static_cast<uint64_t>(e & 0xFFFFFFu) << fill8;                           \
        fill8 += cn << 3;                                                               \
        j += cn;                                                                        \
        orw[wp & 15] = static_cast<uint32_t>(acc);                                      \
        const bool full_ = fill8 >= 32;                                                 \
        wp += full_ ? 1u : 0u;                                                          \
        acc = full_ ? (acc >> 32) : acc;                                                \
        fill8 -= full_ ? 32u : 0u;                                                      \
    } while (0)

    while (j < cnt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            RING_REFILL();
            RING_LOOKUP();
            RING_LOOKUP();
        }
        // ring maintenance: at most one half in, one half out
        if (rp + 8 >= filled) {  // the half [filled - 16, filled - 8) is consumed
            put_half(ir, filled & 15, Bp, Bq);
            filled += 8;
            load_half(a.comp, a.comp_bytes, h0 + (filled >> 3), Bp, Bq);
        }
        if (wp >= flushed + 8 && flushed + 8 <= flush_lim) {
            const uint2* r = reinterpret_cast<const uint2*>(orw + (flushed & 15));
            const uint2 x0 = r[0], x1 = r[1], x2 = r[2], x3 = r[3];
            uint4* d4 = reinterpret_cast<uint4*>(dst + flushed * 4);
            d4[0] = make_uint4(x0.x, x0.y, x1.x, x1.y);
            d4[1] = make_uint4(x2.x, x2.y, x3.x, x3.y);
            flushed += 8;
        }
    }
#undef RING_LOOKUP
#undef RING_REFILL
    // what is left: whole halves not yet stored, then the ragged end
    while (flushed + 8 <= flush_lim) {
        const uint2* r = reinterpret_cast<const uint2*>(orw + (flushed & 15));
        const uint2 x0 = r[0], x1 = r[1], x2 = r[2], x3 = r[3];
        uint4* d4 = reinterpret_cast<uint4*>(dst + flushed * 4);
        d4[0] = make_uint4(x0.x, x0.y, x1.x, x1.y);
        d4[1] = make_uint4(x2.x, x2.y, x3.x, x3.y);
        flushed += 8;
    }
    for (uint32_t i = flushed * 4; i < cnt; ++i) {
        const uint32_t v = i < 4 * wp ? orw[(i >> 2) & 15] >> (8 * (i & 3))
                                      : static_cast<uint32_t>(acc >> (8 * (i - 4 * wp)));
        dst[i] = static_cast<uint8_t>(v);
    }
}

}  // namespace

size_t decode_ring_lds_bytes(uint32_t mlut_bits) {
    return static_cast<size_t>((1u << mlut_bits) + 2 * kThreads * kRing) * 4;
}

hipError_t launch_decode_ring(const DecodeArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    const size_t lds = decode_ring_lds_bytes(a.mlut_bits);
    if (a.max_len > a.mlut_bits)
        hipLaunchKernelGGL(k_decode_ring<true>, dim3(a.nchunks), dim3(kThreads), lds, s, a);
    else
        hipLaunchKernelGGL(k_decode_ring<false>, dim3(a.nchunks), dim3(kThreads), lds, s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
