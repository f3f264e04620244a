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
//  k_mark : (codes <= 32 bits) lane i walks its settled segment once more and
//           records the start bit of every symbol whose index is a multiple
//           of 256: the restart index the ring decoder (decode_ring.hip) then
//           decodes from, as it does for streams this encoder wrote.
//  k_emit : (longer codes) lane i decodes c[i] symbols from its settled start.
// k_spec and k_mark stage each workgroup's 256 segments in LDS (k_*_lds).
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

// ---- LDS-staged variants (every code <= 32 bits) ---------------------------
// A workgroup's 256 consecutive segments are one contiguous bit range: it is
// staged in LDS once with coalesced dword loads (plus 32 bytes of lookahead
// for the code that crosses the last segment end), and each lane then reads
// its bits from LDS: a 64-bit window refilled 32 bits at a time, multi-symbol
// lookups (top 12 bits -> up to 3 letters) while the whole entry stays inside
// the lane's range, single codes otherwise.

struct Staged {
    const uint32_t* w;
    uint64_t base;  // bit position of w[0]'s most significant bit
};

// The block's range from its 16-B granule, 8 loads of 16 B per lane in
// flight per batch through a buffer resource over the range rounded up to
// its last 16-B granule (pieces past it, incl. the two zero words the lanes'
// lookahead may read, come back zero): the one-dword-at-a-time loop this
// replaces waited out a memory latency per dword.
__device__ Staged stage_block(const IndexlessArgs& a, uint32_t* w) {
    const uint64_t seg0 = static_cast<uint64_t>(blockIdx.x) * kThreads;
    const uint64_t bit_lo = seg0 * a.seg_bits;
    const uint64_t seg_end = seg0 + kThreads < a.nseg ? seg0 + kThreads : a.nseg;
    const uint64_t bit_hi = seg_end * a.seg_bits < a.valid_bits ? seg_end * a.seg_bits : a.valid_bits;
    const uint64_t byte_lo = (bit_lo >> 3) & ~15ull;
    uint64_t byte_hi = ((bit_hi + 7) >> 3) + 32;
    if (byte_hi > a.comp_bytes) byte_hi = a.comp_bytes;
    const uint32_t nbytes = static_cast<uint32_t>(byte_hi - byte_lo);
    const uint32_t np = (nbytes + 8 + 15) / 16;  // + the two zero words
    const auto rs = buf_rsrc(a.comp + byte_lo, (nbytes + 15) & ~15u);
    uint4* w4 = reinterpret_cast<uint4*>(w);
    for (uint32_t p0 = threadIdx.x; p0 < np; p0 += 8 * kThreads) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = buf_ld16(rs, (p0 + k * kThreads) * 16);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (p0 + k * kThreads < np) w4[p0 + k * kThreads] = v[k];
    }
    return Staged{w, byte_lo * 8};
}

struct LaneBits {
    const uint32_t* w;
    uint64_t buf;
    uint32_t nb, rp;
    uint64_t pos;
    __device__ __forceinline__ void init(const Staged& st, uint64_t p) {
        w = st.w;
        pos = p;
        const uint64_t off = p - st.base;
        rp = static_cast<uint32_t>(off >> 5);
        const uint32_t sh = static_cast<uint32_t>(off & 31);
        buf = (static_cast<uint64_t>(__builtin_bswap32(w[rp])) << 32) | __builtin_bswap32(w[rp + 1]);
        buf <<= sh;
        nb = 64 - sh;
        rp += 2;
    }
    __device__ __forceinline__ void refill() {
        if (nb < 32) {
            buf |= static_cast<uint64_t>(__builtin_bswap32(w[rp++])) << (32 - nb);
            nb += 32;
        }
    }
    __device__ __forceinline__ void consume(uint32_t len) {
        buf <<= len;
        nb -= len;
        pos += len;
    }
};

// one code from the single-symbol tables (global, L2-resident: only segment
// ends and codes longer than the multi table's index take this path)
__device__ __forceinline__ uint32_t single_code(const LaneBits& r, const uint32_t* glut, uint32_t Ks) {
    uint32_t e = glut[static_cast<uint32_t>(r.buf >> (64 - Ks))];
    uint32_t d = Ks;
    while (e & kLutPtr) {
        const uint32_t idx = static_cast<uint32_t>((r.buf >> (56 - d)) & 0xFFu);
        e = glut[(e & ~kLutPtr) + idx];
        d += 8;
    }
    return e;  // (len << 8) | letter
}

// LDS: [multi table 1 << K][staged input]
__global__ __launch_bounds__(kThreads) void k_spec_lds(IndexlessArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t K = a.mlut_bits, Ks = a.lut_bits;
    uint32_t* mlut = lds;
    for (uint32_t i = threadIdx.x; i < (1u << K); i += blockDim.x) mlut[i] = a.mlut[i];
    const Staged st = stage_block(a, mlut + (((1u << K) + 3) & ~3u));
    __syncthreads();
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= a.nseg) return;
    const uint64_t B = a.valid_bits;
    const uint64_t start = i * a.seg_bits;
    const uint64_t end = (i + 1 == a.nseg) ? B : (start + a.seg_bits < B ? start + a.seg_bits : B);
    LaneBits r;
    r.init(st, start);
    uint64_t cnt = 0;
    while (r.pos < end) {
        r.refill();
        const uint32_t e = mlut[static_cast<uint32_t>(r.buf >> (64 - K))];
        const uint32_t used = (e >> 24) & 31u;
        if (!(e & kMsSlow) && r.pos + used < end) {  // every code of the entry ends before `end`
            r.consume(used);
            cnt += e >> 29;
            continue;
        }
        const uint32_t len = (single_code(r, a.lut, Ks) >> 8) & 0xFFu;
        if (r.pos + len > B) {  // an incomplete final code is dropped (comp.rs:493-516)
            r.pos = B;
            break;
        }
        r.consume(len);
        ++cnt;
    }
    a.s[i] = start;
    a.x[i] = r.pos;
    a.c[i] = cnt;
}

// sub_abs[g] = start bit of symbol g << shift, from the settled segments
__global__ __launch_bounds__(kThreads) void k_mark_lds(IndexlessArgs a, const uint64_t* __restrict__ off,
                                                       uint64_t* __restrict__ sub_abs, uint32_t shift) {
    const uint64_t mask = (1ull << shift) - 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t K = a.mlut_bits, Ks = a.lut_bits;
    uint32_t* mlut = lds;
    for (uint32_t i = threadIdx.x; i < (1u << K); i += blockDim.x) mlut[i] = a.mlut[i];
    const Staged st = stage_block(a, mlut + (((1u << K) + 3) & ~3u));
    __syncthreads();
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= a.nseg) return;
    uint64_t j = off[i];
    const uint64_t jend = j + a.c[i];
    if (j == jend) return;
    LaneBits r;
    r.init(st, a.s[i]);
    while (j < jend) {
        if ((j & mask) == 0) sub_abs[j >> shift] = r.pos;
        r.refill();
        const uint32_t e = mlut[static_cast<uint32_t>(r.buf >> (64 - K))];
        const uint32_t cn = e >> 29;
        if (!(e & kMsSlow) && (j & mask) + cn <= mask + 1 && j + cn <= jend) {  // no mark inside the entry
            r.consume((e >> 24) & 31u);
            j += cn;
            continue;
        }
        r.consume((single_code(r, a.lut, Ks) >> 8) & 0xFFu);
        ++j;
    }
}

}  // namespace

static size_t lds_staged_bytes(const IndexlessArgs& a) {
    return static_cast<size_t>(((1u << a.mlut_bits) + 3) & ~3u) * 4 + ((kThreads * a.seg_bits + 7) / 8 + 96 + 15) / 16 * 16;
}

static bool use_staged(const IndexlessArgs& a) { return a.mlut && a.max_len <= 32 && lds_staged_bytes(a) <= 160 * 1024; }

hipError_t launch_indexless_mark(const IndexlessArgs& a, const uint64_t* off, uint64_t* sub_abs, uint32_t shift,
                                 hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    if (!use_staged(a)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_mark_lds, dim3((a.nseg + kThreads - 1) / kThreads), dim3(kThreads), lds_staged_bytes(a), st,
                       a, off, sub_abs, shift);
    return hipGetLastError();
}

bool indexless_staged(const IndexlessArgs& a) { return use_staged(a); }

hipError_t launch_indexless_spec(const IndexlessArgs& a, hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    if (use_staged(a)) {
        hipLaunchKernelGGL(k_spec_lds, dim3((a.nseg + kThreads - 1) / kThreads), dim3(kThreads), lds_staged_bytes(a),
                           st, a);
        return hipGetLastError();
    }
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
