// indexless.hip — decompress without a restart index (streams written by the
// reference CPU path or read from `.hff` files carry none: comp.rs:279-300).
//
// Self-synchronising parallel decode. The valid bits [0, B) are cut into
// segments of S bits (S a multiple of g = gcd of all code lengths, so every
// segment start has the residue of a true codeword boundary).
//  k_spec : lane i decodes speculatively from bit i*S until the first codeword
//           boundary >= (i+1)*S: exit x[i] and symbol count c[i].
//  k_fix  : (repeated until stable) lane i restarts from its predecessor's
//           exit x[i-1] with a second cursor on its old path; the cursor that
//           is behind advances; when both sit on the same boundary the paths
//           have merged (exit unchanged, count corrected), otherwise the new
//           exit is published and the successor re-checks next round.
//           Huffman codes resynchronise within a few codewords in practice, so
//           one or two rounds settle; a bounded host loop falls back to a
//           sequential sweep (k_settle) for codes that never synchronise.
//  scan   : exclusive scan of c[] -> output offsets (k_scan, hist.hip).
//  k_emit : lane i decodes c[i] symbols from its settled start.
// A codeword that would cross B is dropped, as the reference's walk drops an
// incomplete final code (comp.rs:493-516).
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;

struct Seg {
    const uint8_t* comp;
    uint64_t comp_bytes;
    uint64_t B;        // valid bits
    uint64_t S;        // segment bits
    uint64_t nseg;
    const uint32_t* lut;
    uint32_t K;
};

__device__ __forceinline__ void load_prim(uint32_t* plut, const Seg& g) {
    for (uint32_t i = threadIdx.x; i < (1u << g.K); i += blockDim.x) plut[i] = g.lut[i];
    __syncthreads();
}

// one codeword step; false (and pos = B) when the code would cross B
__device__ __forceinline__ bool step(BitReader& rd, const BitSrc& src, const Lut& lut, uint64_t B) {
    const uint32_t e = rd.peek(src, lut);
    const uint32_t len = (e >> 8) & 0xFFu;
    if (rd.pos + len > B) {
        rd.pos = B;
        return false;
    }
    rd.advance(src, len);
    return true;
}

__global__ __launch_bounds__(kThreads) void k_spec(Seg g, uint64_t* __restrict__ s, uint64_t* __restrict__ x,
                                                   uint64_t* __restrict__ c) {
    extern __shared__ uint32_t plut[];
    load_prim(plut, g);
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= g.nseg) return;
    const BitSrc src{reinterpret_cast<const uint32_t*>(g.comp), g.comp, g.comp_bytes};
    const Lut lut{plut, g.lut, g.K};
    const uint64_t start = i * g.S;
    const uint64_t end = (i + 1 == g.nseg) ? g.B : (start + g.S < g.B ? start + g.S : g.B);
    BitReader rd;
    rd.seek(src, start);
    uint64_t cnt = 0;
    while (rd.pos < end) {
        if (!step(rd, src, lut, g.B)) break;
        ++cnt;
    }
    s[i] = start;
    x[i] = rd.pos;
    c[i] = cnt;
}

__global__ __launch_bounds__(kThreads) void k_fix(Seg g, uint64_t* __restrict__ s, const uint64_t* __restrict__ xin,
                                                  uint64_t* __restrict__ xout, uint64_t* __restrict__ c,
                                                  unsigned int* __restrict__ changed) {
    extern __shared__ uint32_t plut[];
    load_prim(plut, g);
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= g.nseg) return;
    if (i == 0) {
        xout[0] = xin[0];
        return;
    }
    const uint64_t ns = xin[i - 1];
    const uint64_t old_s = s[i];
    if (ns == old_s) {
        xout[i] = xin[i];
        return;
    }
    const BitSrc src{reinterpret_cast<const uint32_t*>(g.comp), g.comp, g.comp_bytes};
    const Lut lut{plut, g.lut, g.K};
    const uint64_t end = (i + 1 == g.nseg) ? g.B : ((i + 1) * g.S < g.B ? (i + 1) * g.S : g.B);
    BitReader a, b;
    a.seek(src, ns);
    b.seek(src, old_s);
    uint64_t ca = 0, cb = 0;
    bool a_alive = true, b_alive = true;
    for (;;) {
        if (a.pos == b.pos) {  // merged: same exit, count corrected
            s[i] = ns;
            c[i] = c[i] - cb + ca;
            xout[i] = xin[i];
            return;
        }
        if (a.pos >= end || !a_alive) {  // new exit
            s[i] = ns;
            c[i] = ca;
            xout[i] = a.pos;
            if (a.pos != xin[i]) atomicOr(changed, 1u);
            return;
        }
        if (a.pos < b.pos || !b_alive) {
            a_alive = step(a, src, lut, g.B);
            ca += a_alive ? 1 : 0;
        } else {
            b_alive = step(b, src, lut, g.B);
            cb += b_alive ? 1 : 0;
        }
    }
}

// sequential fallback: settle every segment in order (one lane)
__global__ void k_settle(Seg g, uint64_t* __restrict__ s, uint64_t* __restrict__ x, uint64_t* __restrict__ c) {
    extern __shared__ uint32_t plut[];
    load_prim(plut, g);
    if (threadIdx.x != 0) return;
    const BitSrc src{reinterpret_cast<const uint32_t*>(g.comp), g.comp, g.comp_bytes};
    const Lut lut{plut, g.lut, g.K};
    for (uint64_t i = 1; i < g.nseg; ++i) {
        const uint64_t ns = x[i - 1];
        if (ns == s[i]) continue;
        const uint64_t end = (i + 1 == g.nseg) ? g.B : ((i + 1) * g.S < g.B ? (i + 1) * g.S : g.B);
        BitReader rd;
        rd.seek(src, ns);
        uint64_t cnt = 0;
        while (rd.pos < end) {
            if (!step(rd, src, lut, g.B)) break;
            ++cnt;
        }
        s[i] = ns;
        x[i] = rd.pos;
        c[i] = cnt;
    }
}

__global__ __launch_bounds__(kThreads) void k_emit(Seg g, const uint64_t* __restrict__ s,
                                                   const uint64_t* __restrict__ c, const uint64_t* __restrict__ off,
                                                   uint8_t* __restrict__ out) {
    extern __shared__ uint32_t plut[];
    load_prim(plut, g);
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= g.nseg) return;
    const uint64_t cnt = c[i];
    if (cnt == 0) return;
    const BitSrc src{reinterpret_cast<const uint32_t*>(g.comp), g.comp, g.comp_bytes};
    const Lut lut{plut, g.lut, g.K};
    BitReader rd;
    rd.seek(src, s[i]);
    uint8_t* o = out + off[i];
    for (uint64_t j = 0; j < cnt; ++j) {
        const uint32_t e = rd.peek(src, lut);
        rd.advance(src, (e >> 8) & 0xFFu);
        o[j] = static_cast<uint8_t>(e);
    }
}

Seg make_seg(const IndexlessArgs& a) {
    return Seg{a.comp, a.comp_bytes, a.valid_bits, a.seg_bits, a.nseg, a.lut, a.lut_bits};
}

}  // namespace

hipError_t launch_indexless_spec(const IndexlessArgs& a, hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    const Seg g = make_seg(a);
    const size_t lds = (1u << a.lut_bits) * 4;
    hipLaunchKernelGGL(k_spec, dim3((a.nseg + kThreads - 1) / kThreads), dim3(kThreads), lds, st, g, a.s, a.x,
                       a.c);
    return hipGetLastError();
}

hipError_t launch_indexless_fix(const IndexlessArgs& a, const uint64_t* xin, uint64_t* xout, unsigned int* changed,
                                hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    const Seg g = make_seg(a);
    const size_t lds = (1u << a.lut_bits) * 4;
    hipLaunchKernelGGL(k_fix, dim3((a.nseg + kThreads - 1) / kThreads), dim3(kThreads), lds, st, g, a.s, xin, xout,
                       a.c, changed);
    return hipGetLastError();
}

hipError_t launch_indexless_settle(const IndexlessArgs& a, uint64_t* x, hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    const Seg g = make_seg(a);
    const size_t lds = (1u << a.lut_bits) * 4;
    hipLaunchKernelGGL(k_settle, dim3(1), dim3(64), lds, st, g, a.s, x, a.c);
    return hipGetLastError();
}

hipError_t launch_indexless_emit(const IndexlessArgs& a, const uint64_t* off, uint8_t* out, hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    const Seg g = make_seg(a);
    const size_t lds = (1u << a.lut_bits) * 4;
    hipLaunchKernelGGL(k_emit, dim3((a.nseg + kThreads - 1) / kThreads), dim3(kThreads), lds, st, g, a.s, a.c, off,
                       out);
    return hipGetLastError();
}

}  // namespace huff::dev
