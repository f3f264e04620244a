// decode.hip — block-parallel decompress (huff_coding/src/comp.rs:487-519).
//
// The reference walks the tree bit by bit. Here every lane decodes a run of
// 256 consecutive symbols starting at a restart point the encoder recorded
// (sub_bit, relative to the chunk's first bit), so the 65,536 symbols of a
// chunk are decoded by the 256 lanes of one workgroup at once.
//
// Per lane: the compressed bits stream through a 4-slot register ring of
// 16-byte loads (64 bytes in flight ahead of the decoder, so HBM latency is
// paid once per ring, not once per refill), a 64-bit left-aligned window
// refilled 32 bits at a time, and one lookup of the top K bits in a primary
// table in LDS giving (letter, length). Codes longer than K bits continue in
// 8-bit secondary tables (global, L2-resident). The tables are built from
// every leaf of the tree (duplicated letters included, tree_inner.rs:281-320 +
// weights.rs:396-415), so they decode exactly what the reference's walk does.
// Symbols are staged in LDS, 64 per lane per phase, and leave as 16-B stores.
//
// Roofline: HBM-bound; algorithmic traffic ceil(bits/8) (read) + n (write).
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;
constexpr uint32_t kPhase = 64;                    // symbols per lane per phase
constexpr uint32_t kStageStride = kPhase / 4 + 1;  // words per lane row (+1: bank spread)

// one 16-byte slot of the stream (zero past the end, never read past it)
__device__ __forceinline__ uint4 load_slot(const uint8_t* __restrict__ comp, uint64_t nbytes, uint64_t s) {
    const uint64_t b = s * 16;
    if (b + 16 <= nbytes) return *reinterpret_cast<const uint4*>(comp + b);
    uint32_t x = 0, y = 0, z = 0, w = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t v = (b + i < nbytes) ? static_cast<uint32_t>(comp[b + i]) << (8 * (i & 3)) : 0u;
        if (i < 4) x |= v;
        else if (i < 8) y |= v;
        else if (i < 12) z |= v;
        else w |= v;
    }
    return make_uint4(x, y, z, w);
}

// Codes of 33-57 bits (a tree deeper than the fixed-count decoder's 32): per
// lane a 4 x 16-B register ring, global window slow path.
template <bool LONG>
__global__ __launch_bounds__(kThreads) void k_decode(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t K = a.lut_bits;
    const uint32_t nprim = 1u << K;
    uint32_t* plut = lds;
    uint32_t* stage = lds + ((nprim + 3) & ~3u);
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < nprim; i += kThreads) plut[i] = a.lut[i];

    const uint32_t c = blockIdx.x;
    const uint64_t sym0 = static_cast<uint64_t>(c) * kChunk;
    const uint64_t nsym = (a.n - sym0 < kChunk) ? a.n - sym0 : kChunk;
    const uint64_t lsym0 = static_cast<uint64_t>(t) * kSub;
    const uint32_t cnt = lsym0 >= nsym ? 0u : static_cast<uint32_t>(nsym - lsym0 < kSub ? nsym - lsym0 : kSub);

    // 4 x 16-byte register ring over the lane's part of the stream: cur is
    // being consumed (dword k next), n1..n3 are in flight
    uint4 cur = make_uint4(0, 0, 0, 0), n1 = cur, n2 = cur, n3 = cur;
    uint64_t slot = 0;
    uint32_t k = 0;
    uint64_t buf = 0, pos = 0;
    uint32_t nb = 0;
#define RING_SEEK(p_)                                                    \
    do {                                                                 \
        const uint64_t dw_ = (p_) >> 5;                                  \
        slot = dw_ >> 2;                                                 \
        k = static_cast<uint32_t>(dw_ & 3);                              \
        cur = load_slot(a.comp, a.comp_bytes, slot);                     \
        n1 = load_slot(a.comp, a.comp_bytes, slot + 1);                  \
        n2 = load_slot(a.comp, a.comp_bytes, slot + 2);                  \
        n3 = load_slot(a.comp, a.comp_bytes, slot + 3);                  \
    } while (0)
#define RING_NEXT(out_)                                                   \
    do {                                                                  \
        if (k == 4) {                                                     \
            cur = n1;                                                     \
            n1 = n2;                                                      \
            n2 = n3;                                                      \
            n3 = load_slot(a.comp, a.comp_bytes, slot + 4);               \
            ++slot;                                                       \
            k = 0;                                                        \
        }                                                                 \
        const uint32_t d_ = k == 0 ? cur.x : (k == 1 ? cur.y : (k == 2 ? cur.z : cur.w)); \
        ++k;                                                              \
        (out_) = __builtin_bswap32(d_);                                   \
    } while (0)
#define START_AT(p_)                                                      \
    do {                                                                  \
        RING_SEEK(p_);                                                    \
        uint32_t w0_;                                                     \
        RING_NEXT(w0_);                                                   \
        const uint32_t sh_ = static_cast<uint32_t>((p_) & 31);            \
        buf = (static_cast<uint64_t>(w0_) << 32) << sh_;                  \
        nb = 32 - sh_;                                                    \
        if (nb < 32) {                                                    \
            uint32_t w1_;                                                 \
            RING_NEXT(w1_);                                               \
            buf |= static_cast<uint64_t>(w1_) << (32 - nb);               \
            nb += 32;                                                     \
        }                                                                 \
    } while (0)
    if (cnt) {
        pos = a.chunk_start[c] + a.sub_bit[(sym0 + lsym0) / kIdx];
        START_AT(pos);
    }
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    __syncthreads();

    for (uint32_t ph = 0; ph < kSub / kPhase; ++ph) {
        const uint32_t j0 = ph * kPhase;
        const uint32_t j1 = cnt < j0 + kPhase ? cnt : j0 + kPhase;
        uint32_t acc = 0;
        uint32_t* row = stage + t * kStageStride;
        for (uint32_t j = j0; j < j1; ++j) {
            if (nb < 32) {
                uint32_t wn;
                RING_NEXT(wn);
                buf |= static_cast<uint64_t>(wn) << (32 - nb);
                nb += 32;
            }
            uint32_t e = plut[buf >> (64 - K)];
            uint32_t len;
            if (!LONG) {
                // codes <= 32 bits: the window holds the whole code (nb >= 32)
                if (e & kLutPtr) {
                    uint32_t d = K;
                    do {
                        const uint32_t idx = static_cast<uint32_t>((buf >> (56 - d)) & 0xFFu);
                        e = a.lut[(e & ~kLutPtr) + idx];
                        d += 8;
                    } while (e & kLutPtr);
                }
                len = (e >> 8) & 0xFFu;
                buf <<= len;
                nb -= len;
            } else {
                len = (e >> 8) & 0xFFu;
                if ((e & kLutPtr) || len > nb) {
                    const Lut lut{plut, a.lut, K};
                    e = lut_lookup_at(src, lut, pos);
                    len = (e >> 8) & 0xFFu;
                    pos += len;
                    START_AT(pos);
                } else {
                    buf <<= len;
                    nb -= len;
                    pos += len;
                }
            }
            acc |= (e & 0xFFu) << (8 * (j & 3));
            if ((j & 3) == 3) {
                row[(j - j0) >> 2] = acc;
                acc = 0;
            }
        }
        if (j1 > j0 && (j1 & 3)) row[(j1 - 1 - j0) >> 2] = acc;
        __syncthreads();
        // lane L's phase output = chunk bytes [L*256 + j0, +64): 4 pieces of 16 B
        for (uint32_t q = t; q < kThreads * 4; q += kThreads) {
            const uint32_t L = q >> 2, part = q & 3;
            const uint64_t off = static_cast<uint64_t>(L) * kSub + j0 + part * 16;
            if (off >= nsym) continue;
            const uint32_t* r = stage + L * kStageStride + part * 4;
            uint4 v = make_uint4(r[0], r[1], r[2], r[3]);
            if (off + 16 <= nsym) {
                *reinterpret_cast<uint4*>(a.out + sym0 + off) = v;
            } else {
                const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
                for (uint32_t i = 0; off + i < nsym; ++i)
                    a.out[sym0 + off + i] = static_cast<uint8_t>(wv[i >> 2] >> (8 * (i & 3)));
            }
        }
        __syncthreads();
    }
#undef START_AT
#undef RING_NEXT
#undef RING_SEEK
}

}  // namespace

size_t decode_lds_bytes(uint32_t lut_bits) {
    const uint32_t nprim = ((1u << lut_bits) + 3) & ~3u;
    return static_cast<size_t>(nprim + kThreads * kStageStride) * 4;
}

// codes of 33-57 bits here; every code <= 32 bits: the fixed-count task
// decoder (decode_wave.hip)
hipError_t launch_decode(const DecodeArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    if (a.max_len <= 32) return a.stab ? launch_decode_fixed(a, s) : hipErrorInvalidValue;
    launch_k(k_decode<true>, dim3(a.nchunks), dim3(kThreads), decode_lds_bytes(a.lut_bits), s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
