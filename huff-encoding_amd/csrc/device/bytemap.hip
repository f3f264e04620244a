// bytemap.hip — fixed-length fast path.
//
// When every code of the tree is exactly 8 bits (the reference's tree for
// near-uniform byte frequencies: 256 equal-ish weights always merge leaf
// pairs first, tree_inner.rs:289-303, giving a complete depth-8 tree), the
// byte-aligned stream of compress_with_tree (comp.rs:424-444) is a byte-for-
// byte substitution: out[i] = code[in[i]], and decode is the inverse map.
// One streaming kernel does both: 16-byte coalesced loads, a 256-entry LDS
// table replicated 32x ([byte][copy], lane l reads copy l % 32: no bank
// conflicts), 16-byte stores. It also writes the restart index, which for
// 8-bit codes is arithmetic (symbol s starts at bit 8 s).
//
// Roofline: HBM-bound, n bytes read + n bytes written.
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;
// 16-B pieces per lane: a workgroup maps kThreads * 16 * kPieces bytes and
// stages its 32 KiB table once for them. Same-box A/B, 1 GiB: alone
// (tools/kbench.py, pass 2 / decode ms) 2 pieces 0.533 / 0.536, 4 0.373-0.378
// / 0.381, 8 0.371-0.372 / 0.360, 16 0.395-0.403 / 0.394-0.399; but inside
// the bench's step (hist, pass 2, decode back to back) 4 pieces 0.351 /
// 0.350 against 8 pieces 0.380 / 0.367 (1150 vs 1093 GB/s, 3 runs each):
// 4 it is
#ifndef HUFF_BYTEMAP_PIECES
#define HUFF_BYTEMAP_PIECES 4
#endif
constexpr int kPieces = HUFF_BYTEMAP_PIECES;

__device__ __forceinline__ uint32_t map4(const uint32_t* tab, uint32_t w, uint32_t copy) {
    const uint32_t b0 = tab[((w & 0xFFu) << 5) | copy];
    const uint32_t b1 = tab[(((w >> 8) & 0xFFu) << 5) | copy];
    const uint32_t b2 = tab[(((w >> 16) & 0xFFu) << 5) | copy];
    const uint32_t b3 = tab[((w >> 24) << 5) | copy];
    return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
}


// One-shot grid: workgroup w maps the 16 KiB [w * 16 KiB, +16 KiB), lane t
// the kPieces (4) 16-B pieces t, t+256, t+512, t+768 of it (each a coalesced
// 4 KiB row per wave set). The data loads are issued before the table is staged in
// LDS, so the table setup hides under the HBM latency.
__global__ __launch_bounds__(kThreads) void k_bytemap(BytemapArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[256 * 32];
    const uint32_t t = threadIdx.x, copy = t & 31;
    const uint64_t nvec = a.n / 16;
    const uint64_t v0 = static_cast<uint64_t>(blockIdx.x) * (kThreads * kPieces) + t;
    const uint4* src = reinterpret_cast<const uint4*>(a.src);
    uint4* dst = reinterpret_cast<uint4*>(a.dst);
    uint4 x[kPieces];
#pragma unroll
    for (int k = 0; k < kPieces; ++k) {
        const uint64_t v = v0 + k * kThreads;
        x[k] = v < nvec ? ld_nt(src + v) : make_uint4(0, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    {  // store i of lane t fills the 16-B piece i * 256 + t (entry (i * 256 + t) / 8):
       // a wave's ds_write_b128 covers 1 KiB contiguous, so every 8-lane group
       // spans all 32 banks. (Lane t writing its own 128-B row put each group's
       // 8 lanes on the same 4 banks: 8-way conflicts, 117 M conflict cycles
       // per GiB, 70 % of the kernel's LDS cycles.)
        uint4* p = reinterpret_cast<uint4*>(tab);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t e = a.map[i * 32 + (t >> 3)];
            p[i * kThreads + t] = make_uint4(e, e, e, e);
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): table stores done; data loads stay in flight
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int k = 0; k < kPieces; ++k) {
        const uint64_t v = v0 + k * kThreads;
        if (v < nvec) {
            uint4 y;
            y.x = map4(tab, x[k].x, copy);
            y.y = map4(tab, x[k].y, copy);
            y.z = map4(tab, x[k].z, copy);
            y.w = map4(tab, x[k].w, copy);
            st_nt(dst + v, y);
        }
    }
    const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * kThreads + t;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    if (blockIdx.x == gridDim.x - 1)
        for (uint64_t i = nvec * 16 + t; i < a.n; i += kThreads) a.dst[i] = static_cast<uint8_t>(tab[(a.src[i] << 5) | copy]);
    // restart index of an 8-bit-per-symbol stream
    if (a.chunk_start)
        for (uint64_t c = gid; c <= a.nchunks; c += stride)
            a.chunk_start[c] = a.base_bits + (c * kChunk < a.n ? c * kChunk : a.n) * 8;
    if (a.sub_bit) {
        const uint64_t nsub = (a.n + kIdx - 1) / kIdx;
        for (uint64_t g = gid; g < nsub; g += stride) a.sub_bit[g] = static_cast<uint32_t>(((g * kIdx) % kChunk) * 8);
    }
}

__global__ __launch_bounds__(256) void k_arith_index(uint64_t n, uint32_t nchunks, uint64_t base_bits,
                                                     uint64_t* __restrict__ chunk_start, uint32_t* __restrict__ sub_bit) {
    const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
    // the last entry is the stream's end (n symbols), as the bit pack writes it
    for (uint64_t c = gid; c <= nchunks; c += stride)
        chunk_start[c] = base_bits + (c * kChunk < n ? c * kChunk : n) * 8;
    const uint64_t nsub = (n + kIdx - 1) / kIdx;
    for (uint64_t g = gid; g < nsub; g += stride) sub_bit[g] = static_cast<uint32_t>(((g * kIdx) % kChunk) * 8);
}

}  // namespace

// sub_bit[g] = task_base[g / 64] + sub16[g] - chunk_start[g / 1024]
__global__ __launch_bounds__(256) void k_index_expand(uint64_t nsub, const uint64_t* __restrict__ task_base,
                                                      const uint16_t* __restrict__ sub16,
                                                      const uint64_t* __restrict__ chunk_start,
                                                      uint32_t* __restrict__ sub_bit) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nsub; g += stride)
        sub_bit[g] = static_cast<uint32_t>(task_base[g * kIdx / kTaskSym] + sub16[g] - chunk_start[g * kIdx / kChunk]);
}

hipError_t launch_index_expand(uint64_t n, const uint64_t* task_base, const uint16_t* sub16,
                               const uint64_t* chunk_start, uint32_t* sub_bit, hipStream_t s) {
    const uint64_t nsub = (n + kIdx - 1) / kIdx;
    if (nsub == 0) return hipSuccess;
    const uint64_t want = (nsub + 255) / 256;
    launch_k(k_index_expand, dim3(static_cast<uint32_t>(want < 4096 ? want : 4096)), dim3(256), 0, s, nsub,
                       task_base, sub16, chunk_start, sub_bit);
    return hipGetLastError();
}

hipError_t launch_arith_index(uint64_t n, uint32_t nchunks, uint64_t base_bits, uint64_t* chunk_start,
                              uint32_t* sub_bit, hipStream_t s) {
    launch_k(k_arith_index, dim3(1024), dim3(256), 0, s, n, nchunks, base_bits, chunk_start, sub_bit);
    return hipGetLastError();
}

hipError_t launch_bytemap(const BytemapArgs& a, hipStream_t s) {
    if (a.n == 0 && !a.chunk_start) return hipSuccess;
    const uint64_t nvec = a.n / 16;
    uint64_t blocks = (nvec + kThreads * kPieces - 1) / (kThreads * kPieces);
    if (blocks < 1) blocks = 1;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    launch_k(k_bytemap, dim3(static_cast<uint32_t>(blocks)), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
