// indexless.hip — decompress without a restart index (streams written by the
// reference CPU path or read from `.hff` files carry none: comp.rs:279-300).
//
// Self-synchronising parallel decode. The valid bits [0, B) are cut into
// segments of S bits (S a multiple of g = gcd of all code lengths, so every
// segment start has the residue of a true codeword boundary).
//  k_spec : lane i decodes speculatively from its segment to the first
//           codeword boundary >= (i+1)*S: exit x[i] and symbol count c[i].
//           The staged form (k_spec_lds, codes <= 32 bits, the default) first
//           walks a lead-in (kLeadBits; kLeadBitsLong for codes past the
//           walk table) before its segment and starts
//           at the first boundary at or past i*S (nearly always the true
//           one), keeps a sample slot every kSampBits bits, fixes its
//           workgroup's segments in place and writes per-workgroup counts;
//           its segment records (start, count, merge point) are packed in one
//           u64 each (SegRec / rec_pack below).
//  fix-up : a segment whose start differs from its predecessor's exit is
//           walked again from that exit with a second cursor on its old path;
//           the cursor that is behind advances; when both sit on the same
//           boundary the paths have merged (exit unchanged, count corrected,
//           merge point and index shift against the speculative path
//           recorded), otherwise the new exit is published and the successor
//           looks again (staged path: lengths from the walk and level-2
//           tables in LDS). Staged path: k_fix_list (every workgroup's first
//           segment and the segments the speculative pass listed) then
//           k_fix_chain (one workgroup following the changed exits, a no-op
//           when there are none). Otherwise kFixRounds k_fix launches (each a
//           no-op once the previous round changed nothing) and k_settle (a
//           sequential sweep, only if the last round still changed an exit).
//           Decided on the device: the host does not wait between rounds.
//  scan   : exclusive scan of the counts (per workgroup on the staged path,
//           k_scan in hist.hip) -> output offsets, the total to the host.
//  k_mark_lite : (codes <= 32 bits) for every 64th symbol the nearest sample
//           slot at or before it and the codes to skip from there; the
//           fixed-count decoder's skip build decodes and drops those codes.
//           (k_mark_lds walks to the exact boundaries instead: the
//           self-checking build.)
//  k_emit : (longer codes) lane i decodes c[i] symbols from its settled start.
// The staged kernels read each workgroup's 256 segments from LDS (segwalk.hpp).
// A codeword that would cross B is dropped, as the reference's walk drops an
// incomplete final code (comp.rs:493-516).
#include <algorithm>

#include "segwalk.hpp"

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
    unsigned long long* wtot;  // per-workgroup code counts of the staged pass (256 segments each), or null
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

// how fix_one walks a code: the decoder's table (LDS primary, global
// secondaries), or — on the staged path, whose fix-up needs only lengths —
// the walk table and the level-2 length table, both in LDS (LenStep: a code
// past the 12-bit walk table was two global reads, a window re-read and a
// secondary table; wide Zipf over 4,096 letters has 16 % of them)
struct LutStep {
    Lut lut;
    __device__ __forceinline__ bool operator()(BitReader& rd, const BitSrc& src, uint64_t B) const {
        return step(rd, src, lut, B);
    }
};
struct LenStep {
    const uint16_t* wt;  // walk table: first code's length in bits [0, 6), kSsSlow
    const uint8_t* l2;   // level-2 lengths (uniform: l2e > 0; else descriptors first)
    uint32_t K, l2e;
    __device__ __forceinline__ bool operator()(BitReader& rd, const BitSrc& src, uint64_t B) const {
        if (rd.nb < 32) {  // >= 32 valid bits: any code (<= 32 bits)
            rd.buf |= static_cast<uint64_t>(src.word(rd.wi)) << (32 - rd.nb);
            ++rd.wi;
            rd.nb += 32;
        }
        const uint32_t top = static_cast<uint32_t>(rd.buf >> 32);
        const uint32_t e = wt[top >> (32 - K)];
        uint32_t len = e & 63u;
        if (e & kSsSlow) {
            const uint32_t s = (e & 0x7Fu) | ((e >> 8) << 7);
            if (l2e) {
                len = l2[(s << l2e) + ((top << K) >> (32 - l2e))];
            } else {
                const uint32_t d = reinterpret_cast<const uint32_t*>(l2)[s];
                len = l2[(d >> 5) + ((top << K) >> (32 - (d & 31u)))];
            }
        }
        if (rd.pos + len > B) {
            rd.pos = B;
            return false;
        }
        rd.advance(src, len);
        return true;
    }
};

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

// a segment's settled record: start, code count, and how its path relates to
// the speculative one (IndexlessArgs::tm/dl). The unstaged path keeps it in
// four arrays; the staged path packs it in one u64 (IndexlessArgs::rec): 8
// bytes written by k_spec_lds and read by k_mark_lite per segment, not 24.
struct SegRec {
    uint64_t s, c;
    uint32_t tm;
    int32_t dl;
};
struct ArrayRecs {
    uint64_t* s;
    uint64_t* c;
    uint32_t* tm;
    int32_t* dl;
    __device__ SegRec load(uint64_t i) const { return SegRec{s[i], c[i], tm[i], dl[i]}; }
    __device__ void store(uint64_t i, const SegRec& v) const {
        s[i] = v.s;
        c[i] = v.c;
        tm[i] = v.tm;
        dl[i] = v.dl;
    }
};
// bits [0, 16) count, [16, 32) tm (0xFFFF: kNoMerge), [32, 48) dl (int16),
// [48, 64) start - i*S (staged segments < 1024 bits, codes <= 32 bits: every
// field fits)
__device__ __forceinline__ SegRec rec_unpack(uint64_t r, uint64_t i, uint64_t S) {
    const uint32_t tm = static_cast<uint32_t>(r >> 16) & 0xFFFFu;
    return SegRec{i * S + (r >> 48), r & 0xFFFFu, tm == 0xFFFFu ? kNoMerge : tm,
                  static_cast<int32_t>(static_cast<int16_t>(static_cast<uint16_t>(r >> 32)))};
}
__device__ __forceinline__ uint64_t rec_pack(const SegRec& v, uint64_t i, uint64_t S) {
    return (v.c & 0xFFFFu) | (static_cast<uint64_t>(v.tm == kNoMerge ? 0xFFFFu : v.tm & 0xFFFFu) << 16) |
           (static_cast<uint64_t>(static_cast<uint16_t>(v.dl)) << 32) | ((v.s - i * S) << 48);
}
struct PackedRecs {
    uint64_t* rec;
    uint64_t S;
    __device__ SegRec load(uint64_t i) const { return rec_unpack(rec[i], i, S); }
    __device__ void store(uint64_t i, const SegRec& v) const { rec[i] = rec_pack(v, i, S); }
};

// round r of the fix-up, in place on x (a lane may read its predecessor's exit
// from this round or the last: either is a boundary of a valid path, and a
// changed exit sets flags[r], so the next round looks again)
// nl / ncnt: a list the successor of a changed exit is appended to (the chain)
template <class Recs, class Step>
__device__ __forceinline__ void fix_one(const Seg& g, const Recs& R, uint64_t* __restrict__ x,
                                        unsigned int* __restrict__ flags, int r, uint64_t i, const Step& step,
                                        uint32_t* nl = nullptr, unsigned int* ncnt = nullptr) {
    const uint64_t ns = x[i - 1];
    SegRec v = R.load(i);
    const uint64_t old_s = v.s;
    if (ns == old_s) return;
    const BitSrc src{reinterpret_cast<const uint32_t*>(g.comp), g.comp, g.comp_bytes};
    const uint64_t end = (i + 1 == g.nseg) ? g.B : ((i + 1) * g.S < g.B ? (i + 1) * g.S : g.B);
    BitReader a, b;
    a.seek(src, ns);
    b.seek(src, old_s);
    uint64_t ca = 0, cb = 0;
    bool a_alive = true, b_alive = true;
    for (;;) {
        if (a.pos == b.pos) {  // merged: same exit, count corrected
            v.s = ns;
            v.c = v.c - cb + ca;
            if (g.wtot && ca != cb) atomicAdd(g.wtot + i / kThreads, static_cast<unsigned long long>(ca - cb));
            // the old path met the speculative one at old-local tm1 with shift
            // dl1; the new path meets the old one at (ca, cb)
            if (v.tm != kNoMerge) {
                const int64_t sh = static_cast<int64_t>(ca) - static_cast<int64_t>(cb);
                const int64_t t2 = static_cast<int64_t>(v.tm) + sh;
                v.tm = static_cast<uint32_t>(t2 > static_cast<int64_t>(ca) ? t2 : static_cast<int64_t>(ca));
                v.dl += static_cast<int32_t>(sh);
            }
            R.store(i, v);
            return;
        }
        if (a.pos >= end || !a_alive) {  // new exit
            v.s = ns;
            if (g.wtot && ca != v.c) atomicAdd(g.wtot + i / kThreads, static_cast<unsigned long long>(ca - v.c));
            v.c = ca;
            v.tm = kNoMerge;
            R.store(i, v);
            x[i] = a.pos;
            // the successor looks again: a new exit is rare, and comparing
            // with the old one is not possible (the staged pass writes x only
            // where a fix-up reads it), nor with the successor's start (its
            // own fix may be rewriting it in this round). A successor whose
            // start already is this exit returns at once.
            atomicOr(flags + r, 1u);
            if (nl && i + 1 < g.nseg) nl[atomicAdd(ncnt, 1u)] = static_cast<uint32_t>(i + 1);
            return;
        }
        if (a.pos < b.pos || !b_alive) {
            a_alive = step(a, src, g.B);
            ca += a_alive ? 1 : 0;
        } else {
            b_alive = step(b, src, g.B);
            cb += b_alive ? 1 : 0;
        }
    }
}

// grid-stride: nearly every lane finds its start settled already (the staged
// speculative pass fixes the segments inside each workgroup)
__global__ __launch_bounds__(kThreads) void k_fix(Seg g, uint64_t* __restrict__ s, uint64_t* __restrict__ x,
                                                  uint64_t* __restrict__ c, uint32_t* __restrict__ tm,
                                                  int32_t* __restrict__ dl, unsigned int* __restrict__ flags, int r) {
    if (r > 0 && __builtin_nontemporal_load(flags + r - 1) == 0) return;  // converged: nothing to do
    extern __shared__ uint32_t plut[];
    load_prim(plut, g);
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < g.nseg;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
        if (i) fix_one(g, ArrayRecs{s, c, tm, dl}, x, flags, r, i, LutStep{Lut{plut, g.lut, g.K}});
}

// the staged path's length tables for the fix-up (LenStep), copied to LDS;
// wt null: the decoder's table (LutStep)
struct FixTabs {
    const uint16_t* wt;
    const uint32_t* l2;
    uint32_t K, l2_words, l2e;
};
// the stepper over the tables in LDS (`lds`: 2^K u16 then l2_words words)
__device__ __forceinline__ LenStep load_len_step(const FixTabs& f, uint32_t* lds) {
    const uint32_t tw = ((1u << f.K) + 1) / 2;
    const uint32_t* w32 = reinterpret_cast<const uint32_t*>(f.wt);
    for (uint32_t i = threadIdx.x; i < tw; i += blockDim.x) lds[i] = w32[i];
    for (uint32_t i = threadIdx.x; i < f.l2_words; i += blockDim.x) lds[tw + i] = f.l2[i];
    __syncthreads();
    return LenStep{reinterpret_cast<const uint16_t*>(lds), reinterpret_cast<const uint8_t*>(lds + tw), f.K, f.l2e};
}

// round 0 after the staged speculative pass: only the segments that can
// differ from their predecessor's exit — every workgroup's first segment and
// the listed successors of in-workgroup new exits (each index once, so no two
// lanes update one segment's merge record)
template <class Step>
__device__ __forceinline__ void fix_list_body(const Seg& g, const PackedRecs& R, uint64_t* __restrict__ x,
                                              unsigned int* __restrict__ flags, const uint32_t* __restrict__ list,
                                              uint32_t* __restrict__ chain, const Step& step) {
    const uint64_t firsts = (g.nseg - 1) / kThreads;  // segments 256, 512, ...
    const uint64_t n = firsts + __builtin_nontemporal_load(flags + kFixRounds);
    for (uint64_t j = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < n;
         j += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        const uint64_t i = j < firsts ? (j + 1) * kThreads : list[j - firsts];
        fix_one(g, R, x, flags, 0, i, step, chain, flags + kFixRounds + 1);
    }
}
__global__ __launch_bounds__(kThreads) void k_fix_list(Seg g, PackedRecs R, uint64_t* __restrict__ x,
                                                       unsigned int* __restrict__ flags,
                                                       const uint32_t* __restrict__ list, uint32_t* __restrict__ chain,
                                                       FixTabs f) {
    extern __shared__ uint32_t plut[];
    if (f.wt) {
        fix_list_body(g, R, x, flags, list, chain, load_len_step(f, plut));
    } else {
        load_prim(plut, g);
        fix_list_body(g, R, x, flags, list, chain, LutStep{Lut{plut, g.lut, g.K}});
    }
}

// The rest of the fix-up in one workgroup: round after round over only the
// successors of the exits the previous round changed (two lists in turn),
// until a round changes none. Segments resynchronise within a few codes, so
// after round 0 the list is nearly always empty and this is a no-op; the
// three no-op k_fix launches and the k_settle launch it replaced cost ~20 us.
// Each segment is listed at most once per round (only its predecessor's fix
// appends it); a lane reading an exit its predecessor changes in the same
// round gets the successor listed again for the next round.
constexpr int kChainThreads = 1024;
template <class Step>
__device__ __forceinline__ void fix_chain_body(const Seg& g, const PackedRecs& R, uint64_t* __restrict__ x,
                                               unsigned int* __restrict__ flags, uint32_t* __restrict__ chain,
                                               const Step& step);
__global__ __launch_bounds__(kChainThreads) void k_fix_chain(Seg g, PackedRecs R, uint64_t* __restrict__ x,
                                                             unsigned int* __restrict__ flags,
                                                             uint32_t* __restrict__ chain, FixTabs f) {
    if (__builtin_nontemporal_load(flags + kFixRounds + 1) == 0) return;  // round 0 changed no exit
    extern __shared__ uint32_t plut[];
    if (f.wt) {
        fix_chain_body(g, R, x, flags, chain, load_len_step(f, plut));
    } else {
        load_prim(plut, g);
        fix_chain_body(g, R, x, flags, chain, LutStep{Lut{plut, g.lut, g.K}});
    }
}
template <class Step>
__device__ __forceinline__ void fix_chain_body(const Seg& g, const PackedRecs& R, uint64_t* __restrict__ x,
                                               unsigned int* __restrict__ flags, uint32_t* __restrict__ chain,
                                               const Step& step) {
    __shared__ uint32_t n_sh;
    uint32_t cur = 0;
    for (;;) {
        unsigned int* cnt = flags + kFixRounds + 1 + cur;
        unsigned int* ncnt = flags + kFixRounds + 2 - cur;
        if (threadIdx.x == 0) n_sh = atomicAdd(cnt, 0u);
        __syncthreads();
        const uint32_t n = n_sh;
        if (n == 0) break;
        const uint32_t* list = chain + static_cast<uint64_t>(cur) * g.nseg;
        uint32_t* nl = chain + static_cast<uint64_t>(cur ^ 1u) * g.nseg;
        for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) fix_one(g, R, x, flags, 0, list[j], step, nl, ncnt);
        __syncthreads();  // every fix of the round done (and n_sh read by every lane)
        if (threadIdx.x == 0) {
            atomicExch(cnt, 0u);
            atomicAdd(flags + kFixRounds + 3, n);  // the chain's fixes in all (diagnostics: HUFF_FIX_STATS)
        }
        cur ^= 1u;
    }
}

// sequential fallback: settle every segment in order (one lane), only when
// the last fix-up round still changed an exit
__global__ void k_settle(Seg g, uint64_t* __restrict__ s, uint64_t* __restrict__ x, uint64_t* __restrict__ c,
                         uint32_t* __restrict__ tm, const unsigned int* __restrict__ flags) {
    if (__builtin_nontemporal_load(flags + kFixRounds - 1) == 0) return;
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
        if (g.wtot) g.wtot[i / kThreads] += cnt - c[i];  // one lane: no other writer
        c[i] = cnt;
        tm[i] = kNoMerge;
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
    return Seg{a.comp, a.comp_bytes, a.valid_bits, a.seg_bits, a.nseg, a.lut, a.lut_bits, a.wtot};
}

// ---- LDS-staged variants (every code <= 32 bits; segwalk.hpp) -------------

// Samples: slot k of a segment (k = 0 .. nsamp-1) is the first chunk end of
// the speculative path at or after start + kSampBits (k + 1), as a u16: bits
// [0, 8) = how far past that threshold it lies, [8, 16) = the codes since
// the previous recorded slot (or since the entry); 0xFFFF = none (not
// reached, or a field would overflow). A segment's slots take kSampStride
// u16 (whole dwords). Round 4's u32 slots every 128 bits (absolute offset and
// index, plus a "half" boundary between slots) took 28 B per segment.
constexpr uint32_t kSampStride = (kSampMax + 1) & ~1u;
constexpr uint32_t kSampNone = 0xFFFFu;
struct SampWords {
    uint32_t d[kSampStride / 2];
};
// 16-B loads at 4-B alignment (a segment's slots start at 20 i bytes): one
// dwordx4 and one dword per lane instead of five dword loads
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ SampWords samp_load(const uint16_t* samp, uint64_t i) {
    SampWords w;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(samp + i * kSampStride);
    constexpr uint32_t kD = kSampStride / 2;
    uint32_t k = 0;
#pragma unroll
    for (; k + 4 <= kD; k += 4) {
        const u32x4_a4 v = *reinterpret_cast<const u32x4_a4*>(p + k);
        w.d[k] = v.x;
        w.d[k + 1] = v.y;
        w.d[k + 2] = v.z;
        w.d[k + 3] = v.w;
    }
#pragma unroll
    for (; k < kD; ++k) w.d[k] = p[k];
    return w;
}
__device__ __forceinline__ void samp_store(uint16_t* samp, uint64_t i, const SampWords& w) {
    uint32_t* p = reinterpret_cast<uint32_t*>(samp + i * kSampStride);
    constexpr uint32_t kD = kSampStride / 2;
    uint32_t k = 0;
#pragma unroll
    for (; k + 4 <= kD; k += 4)
        *reinterpret_cast<u32x4_a4*>(p + k) = u32x4_a4{w.d[k], w.d[k + 1], w.d[k + 2], w.d[k + 3]};
#pragma unroll
    for (; k < kD; ++k) p[k] = w.d[k];
}
// slot k (a run-time index) by selects, so the words stay in registers
__device__ __forceinline__ uint32_t samp_get(const SampWords& w, uint32_t k) {
    uint32_t d = 0;
#pragma unroll
    for (uint32_t j = 0; j < kSampStride / 2; ++j) d |= w.d[j] & (j == (k >> 1) ? ~0u : 0u);
    return (d >> (16 * (k & 1))) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t samp_slot(const SampWords& w, uint32_t k) {
    return (w.d[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
}
// the nearest recorded slot at or before spec-local code u: (code index, bit
// offset from the segment start); (0, 0): none
__device__ __forceinline__ void samp_pick(const SampWords& w, uint32_t nsamp, uint32_t u, uint32_t& idx,
                                          uint32_t& rel) {
    idx = 0;
    rel = 0;
    uint32_t cum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSampMax; ++k) {
        const uint32_t v = samp_slot(w, k);
        const bool valid = k < nsamp && v != kSampNone;
        cum += valid ? v >> 8 : 0u;
        const bool ok = valid && cum <= u;
        idx = ok ? cum : idx;
        rel = ok ? kSampBits * (k + 1) + (v & 0xFFu) : rel;
    }
}

// Lead-in: a lane starts its walk kLeadBits before its segment and takes the
// first boundary at or after the segment start as its entry. Huffman codes
// resynchronise within a few codes (1 GiB Zipf: half of all walks from an
// arbitrary bit within 11 bits, 0.4 % beyond 96; tools/sync_stats.py), so the
// entry is nearly always the true boundary, the predecessor's exit: the
// in-workgroup fix-up below and k_fix_list's check of every workgroup's first
// segment then find nothing to walk. Without it every lane walked from its
// predecessor's exit to its first sample (>= 128 bits) and each wave waited
// for its slowest lane.
// The lead (IndexlessArgs::lead_bits; kLeadBitsLong when codes exceed the
// walk table's index) is kLeadBits rounded down to a multiple
// of the gcd of the code lengths, like the segment starts, so a lane never
// starts out of phase: with all codes 6 bits long a 128-bit lead-in walked a
// path that never met the true one and the fix-up chained through every
// segment.

template <bool SLOW>
__global__ __launch_bounds__(kThreads) void k_spec_lds(IndexlessArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    WaveStamps ws;  // timing builds: 0 entry, 1 staged, 2 multi-code walk, 3 exit walk, 4 fix-up start, 5 fix-up end
    HUFF_STAMP(ws, 0);
    TabLoad tl;
    issue_tables(a, tl);
    const Staged st = with_l2(stage_block(a, lds + tables_words(a), a.lead_bits), a, lds);
    const uint16_t* stab = store_tables(a, tl, lds);
    const uint16_t* wtab = a.wtab ? stab : nullptr;  // one table serves single and multi-code steps
    __syncthreads();
    HUFF_STAMP(ws, 1);
    const uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const bool live = i0 < a.nseg;  // no early return: the fix-up below has a barrier
    const uint64_t i = live ? i0 : a.nseg - 1;
    const uint32_t K = a.stab_bits, Kg = a.lut_bits;
    const uint64_t B = a.valid_bits;
    const uint64_t start = i * a.seg_bits;
    const uint64_t end = (i + 1 == a.nseg) ? B : (start + a.seg_bits < B ? start + a.seg_bits : B);
    Cursor c;
    uint64_t cur = start, cnt = 0;
    if (a.lead_bits && start) {  // the entry: the lead-in walk's first boundary >= start
        uint64_t p = start > a.lead_bits ? start - a.lead_bits : 0;
        c.init(st, p);
#ifndef HUFF_LEAD_MULTI
#define HUFF_LEAD_MULTI 1
#endif
#if HUFF_LEAD_MULTI
        // multi-code chunks up to the last window end below start (window ends
        // are boundaries), single codes from there: lead-in 4.0 K -> 2.3 K
        // cycles per wave, Zipf 1.114 -> 1.092 ms (same box)
        if (wtab) {
            for (;;) {
                uint32_t U, N, q[kChunkSteps];
                c.multi_chunk<SLOW>(U, N, q, wtab, stab, K, a.lut, Kg);
                if (p + U < start) {
                    p += U;
                    continue;
                }
                uint32_t back = 0;
#pragma unroll
                for (int k = 0; k < kChunkSteps; ++k) {
                    const uint32_t u = q[k] & 0xFFFFu;
                    back = p + u < start ? u : back;
                }
                p += back;
                c.init(st, p);
                break;
            }
        }
#endif
        for (;;) {
            uint32_t L[kChunkSteps];
            c.chunk<SLOW>(L, stab, K, a.lut, Kg);
            uint64_t ex = ~0ull;
#pragma unroll
            for (int k = 0; k < kChunkSteps; ++k) {
                p += L[k];
                ex = (ex == ~0ull && p >= start) ? p : ex;
            }
            if (ex != ~0ull) {
                cur = ex < B ? ex : B;  // a code crossing B: no code starts in the segment
                break;
            }
        }
    }
    c.init(st, cur);
    // samples: the first chunk end of this path at or after every kSampBits
    // bits past start (the slots above)
    // the slots in registers (all "none" until noted), stored at the end as
    // whole dwords: ten scattered 2-B stores per lane were the alternative
    SampWords sw;
#pragma unroll
    for (uint32_t j = 0; j < kSampStride / 2; ++j) sw.d[j] = 0xFFFFFFFFu;
    uint32_t next_k = 1;
    uint64_t next_bit = (a.nsamp && live) ? start + kSampBits : ~0ull;
    uint64_t last_idx = 0;  // the code index of the last recorded slot (the entry: 0)
    const uint64_t entry = cur;
    auto note_sample = [&]() {
        if (cur >= next_bit) {
            const uint64_t off = cur - next_bit, didx = cnt - last_idx;
            const bool ok = off < 256 && didx < 255;
            const uint32_t v16 = ok ? static_cast<uint32_t>(off | (didx << 8)) : kSampNone;
            const uint32_t k = next_k - 1, sh = 16 * (k & 1);
#pragma unroll
            for (uint32_t j = 0; j < kSampStride / 2; ++j) {  // every word written: no indexed access
                const uint32_t m = j == (k >> 1) ? 0xFFFFu << sh : 0u;
                sw.d[j] = (sw.d[j] & ~m) | ((v16 << sh) & m);
            }
            last_idx = ok ? cnt : last_idx;
            next_bit = ++next_k <= a.nsamp ? next_bit + kSampBits : ~0ull;
        }
    };
    if (wtab) {
        // multi-code chunks while the chunk's last boundary stays below `end`
        // (so no boundary inside it can be the exit); single codes after.
        // (Cutting the chunk that reaches `end` back to its window, so the
        // single codes walk one window instead of ~8 K bits: exit walk 3.8 K
        // -> 1.2 K cycles per wave, the multi-code walk 18.0 K -> 21.1 K for
        // the running totals it needs; phase stamps, DESIGN §11. Not kept.)
        const uint64_t span = static_cast<uint64_t>(kChunkSteps) * (a.max_len > K ? a.max_len : K);
        while (cur + span < end) {
            uint32_t U, N;
            c.multi_chunk<SLOW>(U, N, wtab, stab, K, a.lut, Kg);
            cur += U;
            cnt += N;
            note_sample();
        }
    }
    HUFF_STAMP(ws, 2);
    for (;;) {
        uint32_t L[kChunkSteps];
        c.chunk<SLOW>(L, stab, K, a.lut, Kg);
        // the first boundary at or past `end` inside this chunk?
        uint64_t p = cur, ex = ~0ull;
        uint32_t ec = 0;
#pragma unroll
        for (int k = 0; k < kChunkSteps; ++k) {
            p += L[k];
            const bool hit = ex == ~0ull && p >= end;
            ex = hit ? p : ex;
            ec = hit ? static_cast<uint32_t>(k + 1) : ec;
        }
        if (ex != ~0ull) {
            cnt += ec;
            if (ex > B) {  // an incomplete final code is dropped (comp.rs:493-516)
                ex = B;
                --cnt;
            }
            cur = ex;
            break;
        }
        cur = p;
        cnt += kChunkSteps;
        note_sample();
    }
    HUFF_STAMP(ws, 3);
    if (live)
        samp_store(a.samp, i, sw);

    // fix-up inside the workgroup, on the staged bits: lane i restarts from
    // lane i-1's exit (the first lane's predecessor is in another workgroup:
    // k_fix's rounds) and walks, in branch-free chunks, until it lands on one
    // of this lane's samples (a boundary of the speculative path: the paths
    // have merged there; exit unchanged, count and index shift corrected) or
    // passes the end (a new exit: the successor's check in k_fix catches it).
    // Walking both paths alternately, one code at a time, cost a third of the
    // speculative pass in divergent branches.
    // the predecessor's exit: from lane l - 1 of the wave (a lane shuffle of
    // the exit relative to the stage), across waves through 4 LDS words (a
    // 2 KiB exit array here kept the workgroup above 40 KiB: 3 per CU, not 4)
    __shared__ uint32_t ex_w[kThreads / 64];
    const uint32_t cur_rel = static_cast<uint32_t>(cur - st.base);
    const uint32_t prev_rel = static_cast<uint32_t>(__shfl_up(static_cast<int>(cur_rel), 1));
    if ((threadIdx.x & 63) == 63) ex_w[threadIdx.x >> 6] = cur_rel;
    __syncthreads();
    const uint64_t cur0 = cur;
    uint64_t s_out = entry;
    uint32_t tm_out = 0;
    int32_t dl_out = 0;
    HUFF_STAMP(ws, 4);
    const uint64_t ns = !threadIdx.x ? entry
                        : st.base + ((threadIdx.x & 63) ? prev_rel : ex_w[(threadIdx.x >> 6) - 1]);
    if (ns != entry) {
        Cursor ca_;
        ca_.init(st, ns);
        uint64_t pa = ns, na = 0;
        uint64_t pk = 0;  // current sample: position, spec-local index (read back from the slots)
        uint32_t ik = 0, cum = 0, k = 0;
        // passed the sample without landing on it: the next recorded one
        auto next_sample = [&]() {
            while (pa > pk) {
                const uint32_t v = k < a.nsamp ? samp_get(sw, k) : kSampNone;
                ++k;
                if (v != kSampNone) {
                    cum += v >> 8;
                    pk = start + kSampBits * k + (v & 0xFFu);
                    ik = cum;
                } else if (k >= a.nsamp) {
                    pk = ~0ull;
                }
            }
        };
        next_sample();
        for (;;) {
            uint32_t L[kChunkSteps];
            ca_.chunk<SLOW>(L, stab, K, a.lut, Kg);
            uint64_t p = pa;
            int hit = -1, ex = -1;
            uint64_t pex = 0;
#pragma unroll
            for (int j = 0; j < kChunkSteps; ++j) {
                p += L[j];
                hit = (hit < 0 && ex < 0 && p == pk) ? j : hit;
                const bool e = ex < 0 && hit < 0 && p >= end;
                ex = e ? j : ex;
                pex = e ? p : pex;
            }
            if (hit >= 0) {  // merged on the sample: true-local index na + hit + 1
                const uint64_t t = na + static_cast<uint64_t>(hit) + 1;
                tm_out = static_cast<uint32_t>(t);
                dl_out = static_cast<int32_t>(static_cast<int64_t>(t) - static_cast<int64_t>(ik));
                cnt = static_cast<uint64_t>(static_cast<int64_t>(cnt) + dl_out);
                break;
            }
            if (ex >= 0) {  // a new exit
                cnt = na + static_cast<uint64_t>(ex) + 1;
                if (pex > B) {  // an incomplete final code is dropped
                    pex = B;
                    --cnt;
                }
                cur = pex;
                tm_out = kNoMerge;
                break;
            }
            pa = p;
            na += kChunkSteps;
            next_sample();
        }
        s_out = ns;
        // a new exit: the successor started from the old one (a workgroup's
        // first segment is checked anyway)
        if (live && tm_out == kNoMerge && cur != cur0 && i + 1 < a.nseg &&
            ((i + 1) % kThreads) != 0 && a.fixlist)
            a.fixlist[atomicAdd(a.flags + kFixRounds, 1u)] = static_cast<uint32_t>(i + 1);
    }
    HUFF_STAMP(ws, 5);
    ws.flush(a.stamps, static_cast<uint64_t>(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6));
    if (a.wtot) {  // the workgroup's code count, for the scan over workgroups (k_mark_lite scans inside)
        __shared__ uint32_t wsum[kThreads / 64];
        const uint32_t incl = wave_scan_incl(live ? static_cast<uint32_t>(cnt) : 0u);
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t tot = 0;
#pragma unroll
            for (int w = 0; w < kThreads / 64; ++w) tot += wsum[w];
            a.wtot[blockIdx.x] = tot;
        }
    }
    if (!live) return;
    a.rec[i] = rec_pack(SegRec{s_out, cnt, tm_out, dl_out}, i, a.seg_bits);
    // the exit only where a fix-up reads it (fix_one reads its predecessor's):
    // the workgroup's last segment, and a new exit whose successor was listed
    if (threadIdx.x == kThreads - 1 || i + 1 == a.nseg || (tm_out == kNoMerge && cur != cur0)) a.x[i] = cur;
}

// the position `n` codes past the boundary `pos` of the staged range
template <bool SLOW>
__device__ __forceinline__ uint64_t walk(const Staged& st, uint64_t pos, uint32_t n, const uint16_t* stab, uint32_t K,
                                         const uint32_t* glut, uint32_t Kg) {
    Cursor c;
    c.init(st, pos);
    while (n) {
        uint32_t L[kChunkSteps];
        c.chunk<SLOW>(L, stab, K, glut, Kg);
#pragma unroll
        for (int k = 0; k < kChunkSteps; ++k) pos += static_cast<uint32_t>(k) < n ? L[k] : 0u;
        n = n > kChunkSteps ? n - kChunkSteps : 0u;
    }
    return pos;
}

// sub_abs[g] = start bit of symbol g << shift, from the settled segments:
// mark m of segment i (true-local index t) is reached by decoding forward from
// the true start when t precedes the merge with the speculative path (or the
// paths never merged), else from the last speculative sample at or before
// spec-local index t - dl[i]
template <bool SLOW>
__global__ __launch_bounds__(kThreads) void k_mark_lds(IndexlessArgs a, const uint64_t* __restrict__ off,
                                                       uint64_t* __restrict__ sub_abs, uint32_t shift) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    TabLoad tl;
    issue_tables(a, tl);
    const Staged st = with_l2(stage_block(a, lds + tables_words(a)), a, lds);
    const uint16_t* stab = store_tables(a, tl, lds);
    __syncthreads();
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= a.nseg) return;
    const uint32_t K = a.stab_bits, Kg = a.lut_bits;
    const uint64_t j0 = off[i];
    const SegRec v = rec_unpack(a.rec[i], i, a.seg_bits);
    const uint64_t cnt = v.c;
    const uint64_t step = 1ull << shift;
    uint64_t m = (j0 + step - 1) & ~(step - 1);
    if (m >= j0 + cnt) return;
    const uint64_t s_true = v.s;
    const uint64_t s_spec = i * a.seg_bits;
    const uint32_t tm = v.tm;
    const int64_t dl = v.dl;
    // the lane's samples, loaded at once (a dependent load per sample tried
    // cost a memory latency each)
    const SampWords sw = samp_load(a.samp, i);
    for (; m < j0 + cnt; m += step) {
        const uint64_t t = m - j0;
        uint64_t pos;
        if (tm == kNoMerge || t < tm) {
            pos = walk<SLOW>(st, s_true, static_cast<uint32_t>(t), stab, K, a.lut, Kg);
        } else {
            const uint32_t u = static_cast<uint32_t>(static_cast<int64_t>(t) - dl);
            uint32_t idx, rel;
            samp_pick(sw, a.nsamp, u, idx, rel);
            // no sample at or before u: the speculative path's origin is its
            // entry (lead-in), not recorded; the true path from its start is
            pos = rel ? walk<SLOW>(st, s_spec + rel, u - idx, stab, K, a.lut, Kg)
                      : walk<SLOW>(st, s_true, static_cast<uint32_t>(t), stab, K, a.lut, Kg);
        }
        sub_abs[m >> shift] = pos;
    }
}

// the same marks as k_mark_lds without walking: each is written as the
// boundary it would walk from and the number of codes to walk, and the
// fixed-count decoder (skip build) decodes those codes without storing them.
// No staging and no table: only the segment records and its samples.
// Segment offsets: off[i] (the scan over segments), or, with woff (the scan
// over the speculative pass's workgroups, 256 segments each), the
// workgroup's offset plus the exclusive scan of its segments' counts done
// here (DPP wave scans + 4 wave totals): the segment-wide scan kernels and
// the off[] round trip are not run.
__global__ __launch_bounds__(kThreads) void k_mark_lite(IndexlessArgs a, const uint64_t* __restrict__ off,
                                                        const unsigned long long* __restrict__ woff,
                                                        uint64_t* __restrict__ sub_abs, uint64_t sub_cap,
                                                        uint32_t* __restrict__ mark32,
                                                        uint32_t* __restrict__ task_seg) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const SegRec v = rec_unpack(i < a.nseg ? a.rec[i] : 0, i, a.seg_bits);
    uint64_t j0, cnt = i < a.nseg ? v.c : 0;
    if (woff) {
        __shared__ uint32_t wsum[kThreads / 64];
        const uint32_t incl = wave_scan_incl(static_cast<uint32_t>(cnt));  // a workgroup's counts sum < 2^32
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
        __syncthreads();
        uint32_t pre = 0;
#pragma unroll
        for (uint32_t w = 0; w < kThreads / 64; ++w) pre += w < (threadIdx.x >> 6) ? wsum[w] : 0u;
        j0 = woff[blockIdx.x] + pre + incl - static_cast<uint32_t>(cnt);
        if (i >= a.nseg) return;
    } else {
        if (i >= a.nseg) return;
        j0 = off[i];
    }
    uint64_t m = (j0 + kIdx - 1) & ~static_cast<uint64_t>(kIdx - 1);
    const uint64_t m_end = j0 + cnt < sub_cap * kIdx ? j0 + cnt : sub_cap * kIdx;
    if (m >= m_end) return;
    const uint64_t s_true = v.s;
    const uint64_t s_spec = i * a.seg_bits;
    const uint32_t tm = v.tm;
    const int64_t dl = v.dl;
    const SampWords sw = samp_load(a.samp, i);
    for (; m < m_end; m += kIdx) {
        const uint32_t t = static_cast<uint32_t>(m - j0);
        uint64_t pos;
        uint32_t skip;
        if (tm == kNoMerge || t < tm) {
            pos = s_true;
            skip = t;
        } else {
            const uint32_t u = static_cast<uint32_t>(static_cast<int64_t>(t) - dl);
            uint32_t idx, rel;
            samp_pick(sw, a.nsamp, u, idx, rel);
            // no sample at or before u: the speculative path's origin is its
            // entry (lead-in), not recorded; the true path from its start is
            pos = rel ? s_spec + rel : s_true;
            skip = rel ? u - idx : t;
        }
        if (mark32) {  // the compact form: offset from the segment's nominal start (< 2048), skip < 1024
            mark32[m / kIdx] = skip | (static_cast<uint32_t>(pos - s_spec) << 10) |
                               (static_cast<uint32_t>(i & 0x7FFu) << 21);
            if ((m % kTaskSym) == 0) task_seg[m / kTaskSym] = static_cast<uint32_t>(i);
        } else {
            sub_abs[m / kIdx] = pos | (static_cast<uint64_t>(skip) << 48);
        }
    }
}

// c[i] from the packed records, for a scan over every segment (need_off)
__global__ __launch_bounds__(kThreads) void k_rec_counts(const uint64_t* __restrict__ rec, uint64_t* __restrict__ c,
                                                         uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) c[i] = rec[i] & 0xFFFFu;
}

}  // namespace

hipError_t launch_indexless_mark_lite(const IndexlessArgs& a, const uint64_t* off, const unsigned long long* woff,
                                      uint64_t* sub_abs, uint64_t sub_cap, hipStream_t st, uint32_t* mark32,
                                      uint32_t* task_seg) {
    if (a.nseg == 0) return hipSuccess;
    if (!a.samp || !a.rec || (!off && !woff) || (!mark32 != !task_seg)) return hipErrorInvalidValue;
    launch_k(k_mark_lite, dim3((a.nseg + kThreads - 1) / kThreads), dim3(kThreads), 0, st, a, off, woff,
                       sub_abs, sub_cap < (~0ull / kIdx) ? sub_cap : (~0ull / kIdx), mark32, task_seg);
    return hipGetLastError();
}

static size_t lds_staged_bytes(const IndexlessArgs& a, uint32_t segs) {
    return static_cast<size_t>((((((1u << a.stab_bits) + 1) / 2) + 3) & ~3u) + a.l2_words) * 4 +
           ((segs * a.seg_bits + 7) / 8 + (a.lead_bits + 7) / 8 + 128 + 15) / 16 * 16;
}

static bool use_staged(const IndexlessArgs& a) {
    // (the sample words hold 10-bit offsets and counts: segments < 1024 bits)
    return a.stab && a.stab_bits && a.max_len <= 32 && a.seg_bits < 1024 &&
           lds_staged_bytes(a, kThreads) <= 160 * 1024;
}

hipError_t launch_indexless_mark(const IndexlessArgs& a, const uint64_t* off, uint64_t* sub_abs, uint32_t shift,
                                 hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    if (!use_staged(a) || !a.samp || !a.rec) return hipErrorInvalidValue;
    const bool slow = a.max_len > a.stab_bits;
    IndexlessArgs m = a;
    m.wtab = nullptr;  // single steps: the walks stop at exact counts
    launch_k(slow ? k_mark_lds<true> : k_mark_lds<false>, dim3((m.nseg + kThreads - 1) / kThreads),
                       dim3(kThreads), lds_staged_bytes(m, kThreads), st, m, off, sub_abs, shift);
    return hipGetLastError();
}

bool indexless_staged(const IndexlessArgs& a) { return use_staged(a); }

hipError_t launch_indexless_spec(const IndexlessArgs& a, hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    if (use_staged(a)) {
        if (!a.samp || !a.rec) return hipErrorInvalidValue;
        const bool slow = a.max_len > a.stab_bits;
        launch_k(slow ? k_spec_lds<true> : k_spec_lds<false>, dim3((a.nseg + kThreads - 1) / kThreads),
                           dim3(kThreads), lds_staged_bytes(a, kThreads), st, a);
        return hipGetLastError();
    }
    const Seg g = make_seg(a);
    const size_t lds = (1u << a.lut_bits) * 4;
    launch_k(k_spec, dim3((a.nseg + kThreads - 1) / kThreads), dim3(kThreads), lds, st, g, a.s, a.x,
                       a.c);
    return hipGetLastError();
}

hipError_t launch_indexless_settle_all(const IndexlessArgs& a, hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    const Seg g = make_seg(a);
    const size_t lds = (1u << a.lut_bits) * 4;
    // grid-stride rounds: a few resident workgroups per CU cover the segments
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((a.nseg + kThreads - 1) / kThreads, 2048));
    if (a.fixlist && a.chain && use_staged(a)) {  // the staged pass listed what round 0 must look at
        const uint32_t lgrid = static_cast<uint32_t>(std::min<uint64_t>(((a.nseg / kThreads) + kThreads) / kThreads, 256));
        const PackedRecs R{a.rec, a.seg_bits};
        // lengths only: the walk table and the level-2 lengths in LDS, when
        // every code past the table has its level-2 entry
        FixTabs f{};
        size_t flds = lds;
        if (a.stab && (a.max_len <= a.stab_bits || a.l2_words)) {
            f = FixTabs{a.wtab ? a.wtab : a.stab, a.l2, a.stab_bits, a.l2_words, a.l2_e};
            flds = std::max<size_t>(lds, (((1u << a.stab_bits) + 1) / 2 + a.l2_words) * 4);
        }
        launch_k(k_fix_list, dim3(std::max<uint32_t>(lgrid, 1)), dim3(kThreads), flds, st, g, R, a.x,
                           a.flags, a.fixlist, a.chain, f);
        launch_k(k_fix_chain, dim3(1), dim3(kChainThreads), flds, st, g, R, a.x, a.flags, a.chain, f);
        return hipGetLastError();
    }
    for (int r = 0; r < kFixRounds; ++r)
        launch_k(k_fix, dim3(grid), dim3(kThreads), lds, st, g, a.s, a.x, a.c, a.tm, a.dl, a.flags, r);
    launch_k(k_settle, dim3(1), dim3(64), lds, st, g, a.s, a.x, a.c, a.tm, a.flags);
    return hipGetLastError();
}

hipError_t launch_indexless_counts(const IndexlessArgs& a, hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    if (!a.rec || !a.c) return hipErrorInvalidValue;
    launch_k(k_rec_counts, dim3((a.nseg + kThreads - 1) / kThreads), dim3(kThreads), 0, st, a.rec, a.c,
                       a.nseg);
    return hipGetLastError();
}

hipError_t launch_indexless_emit(const IndexlessArgs& a, const uint64_t* off, uint8_t* out, hipStream_t st) {
    if (a.nseg == 0) return hipSuccess;
    const Seg g = make_seg(a);
    const size_t lds = (1u << a.lut_bits) * 4;
    launch_k(k_emit, dim3((a.nseg + kThreads - 1) / kThreads), dim3(kThreads), lds, st, g, a.s, a.c, off,
                       out);
    return hipGetLastError();
}

}  // namespace huff::dev
