// decode.hip — block-parallel decompress (huff_coding/src/comp.rs:487-519).
//
// The reference walks the tree bit by bit. Here every lane decodes a run of
// 256 consecutive symbols starting at a restart point the encoder recorded
// (sub_bit, relative to the chunk's first bit), so the 65,536 symbols of a
// chunk are decoded by 256 lanes at once. Per symbol: a 64-bit left-aligned
// bit window (refilled 32 bits at a time from big-endian words), one lookup
// of the top K bits in a primary table in LDS giving (letter, length); codes
// longer than K bits follow 8-bit secondary tables from global memory. The
// table is built from every leaf of the tree (duplicated letters included,
// tree_inner.rs:281-320 + weights.rs:396-415), so it decodes exactly what the
// tree walk decodes. Output goes through LDS in 4 phases of 64 symbols per
// lane and leaves as 16-byte stores.
//
// Roofline: HBM-bound; algorithmic traffic ceil(bits/8) (read) + n (write).
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;
constexpr uint32_t kPhase = 64;              // symbols per lane per phase
constexpr uint32_t kStageStride = kPhase / 4 + 1;  // words per lane row (+1: bank spread)

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

    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    const Lut lut{plut, a.lut, K};
    BitReader rd{};
    __syncthreads();
    if (cnt) rd.seek(src, a.chunk_start[c] + a.sub_bit[(sym0 + lsym0) / kSub]);

    for (uint32_t ph = 0; ph < kSub / kPhase; ++ph) {
        const uint32_t j0 = ph * kPhase;
        const uint32_t j1 = cnt < j0 + kPhase ? cnt : j0 + kPhase;
        uint32_t acc = 0;
        uint32_t* row = stage + t * kStageStride;
        for (uint32_t j = j0; j < j1; ++j) {
            const uint32_t e = rd.peek(src, lut);
            rd.advance(src, (e >> 8) & 0xFFu);
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
}

}  // namespace

size_t decode_lds_bytes(uint32_t lut_bits) {
    const uint32_t nprim = ((1u << lut_bits) + 3) & ~3u;
    return static_cast<size_t>(nprim + kThreads * kStageStride) * 4;
}

hipError_t launch_decode(const DecodeArgs& a, hipStream_t s) {
    if (a.nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode, dim3(a.nchunks), dim3(kThreads), decode_lds_bytes(a.lut_bits), s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
