// decode_wave.hip — restart-index decode with wave-contiguous memory traffic
// (comp.rs:487-519 semantics; restart index = chunk_start + sub_bit or the
// compact task_base + sub16 form, one entry per kIdx = 64 symbols, written by
// pack).
//
// Work unit: a TASK of 4,096 consecutive symbols per wave (lane l decodes
// symbols [64 l, 64 l + 64) of the task). A task's compressed bits are one
// contiguous range, and so is its output, so both move as whole lines: the
// wave stages its compressed range in LDS with coalesced 16-B loads, every
// lane decodes exactly 64 letters from the stage (k_decode_fixed below), and
// the wave's 4 KiB of letters leave through an LDS transpose as 1 KiB
// contiguous stores. A task whose range exceeds the stage (long local codes)
// decodes straight from global memory instead.
//
// Roofline: HBM-bound; algorithmic traffic ceil(bits/8) (read) + n (write)
// + the restart index (2 B per 64 symbols + 8 B per task in the compact form).
#include <algorithm>
#include <cstdlib>

#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kLaneSym = kIdx;              // symbols per lane per task
static_assert(kTaskSym == 64 * kLaneSym, "4,096 symbols per wave task");
// k_decode_fixed's per-wave stage: the task's input, then (after the decode)
// its 64 output rows of 64 B. Two sizes: 4,608 B (9 bits per symbol), or, for
// the index-free skip build of streams of <= 5.6 bits per symbol
// (fixed_decode_small), 3,072 B: 20 KiB per workgroup with the table, so 8
// workgroups share a CU instead of 5-6, the rows leaving in two halves. A
// task whose range exceeds its stage decodes from global memory.
constexpr uint32_t kInCap = 4608;
constexpr uint32_t kInCapSmall = 3072;
constexpr uint32_t kRowBytes = 64;  // 16-B pieces XOR-swizzled by (row >> 1) & 3: conflict-free ds_write_b128
template <bool SMALL>
constexpr uint32_t fx_stage_bytes() { return SMALL ? kInCapSmall : kInCap; }
static_assert(64 * kRowBytes <= kInCap && 32 * kRowBytes <= kInCapSmall, "the output rows (or half) fit the stage");
__device__ __forceinline__ uint32_t row_piece(uint32_t row, uint32_t q) { return row * kRowBytes + 16 * (q ^ ((row >> 1) & 3)); }
template <bool SMALL>
constexpr uint32_t load_rounds() { return (fx_stage_bytes<SMALL>() / 16 + 63) / 64; }  // 5 or 3
static_assert(kChunk % kTaskSym == 0, "a task never straddles a chunk");
// The first task's loads issued before the table copy (HUFF_DEC_EARLY_LOADS=0
// for the A/B build without), and the minimum waves per SIMD of the PAD
// bodies (their register floor)
#ifndef HUFF_DEC_EARLY_LOADS
#define HUFF_DEC_EARLY_LOADS 1
#endif
#ifndef HUFF_DEC_PAD_WAVES
#define HUFF_DEC_PAD_WAVES 5
#endif
constexpr bool kEarlyLoads = HUFF_DEC_EARLY_LOADS != 0;
// the index-free skip codes at 4 per refill too when the letters take 4
// (HUFF_SKIP_R=0: two, for the A/B build)
#ifndef HUFF_SKIP_R
#define HUFF_SKIP_R 1
#endif
constexpr bool kSkipR = HUFF_SKIP_R != 0;
constexpr int kPadWaves = HUFF_DEC_PAD_WAVES;

struct Task {
    uint64_t sym0;      // first symbol
    uint32_t nsym;      // symbols in the task (<= kTaskSym)
    uint64_t lane_bit;  // this lane's first bit (valid when cnt > 0)
    uint32_t cnt;       // this lane's symbols
    uint64_t b0;        // first staged byte (16-B aligned)
    uint32_t len;       // staged bytes
    uint64_t end;       // the task's end bit (= the next task's first bit; SKIP: a bound)
    uint32_t skip;      // SKIP: codes to decode and drop before this lane's letters
};

// A task's index entries in two steps: task_load issues the loads (nothing
// in it reads a loaded value, so the compiler places no wait there) and
// task_finish derives the task from them. k_decode_dma issues the loads of
// the task after next before it decodes and finishes them a task later, so
// their latency hides behind the decode and no wait drains its in-flight
// LDS-DMA early (a vmcnt wait covers every older VMEM operation).
// Every load is unconditional (indices clamped to the arrays) and lands in a
// field of its own width: a select or a widening copy of a loaded value is a
// use, and the compiler would wait for it right there.
struct TaskLoad {
    uint32_t m = 0, m1 = 0, s0 = 0, s1 = 0;  // u16/u32 entries (zero-extended by the load)
    uint64_t q = 0, q1 = 0, q2 = 0;          // u64 entries
};
// SKIP: the index-free path's k_mark_lite entries (boundary | skip << 48).
// MODE: which index the task reads, when known at compile time (k_decode_dma:
// the branches over the index forms made the compiler join their registers
// and wait for the loads at the join): kIdxAny (run time), kIdxMark32
// (compact marks), kIdxSub16 (the compact restart index)
constexpr int kIdxAny = 0, kIdxMark32 = 1, kIdxSub16 = 2;
template <bool SKIP = false, int MODE = kIdxAny>
__device__ __forceinline__ TaskLoad task_load(const DecodeArgs& a, uint64_t t, uint32_t lane) {
    TaskLoad r;
    // vz = 0 in every lane, but divergent to the compiler: the wave-uniform
    // entries then load into VGPRs and stay there until task_finish (as
    // uniform values they were moved to SGPRs by a readfirstlane right after
    // the load, i.e. waited for at once)
    const uint64_t vz = MODE == kIdxAny ? 0u : __builtin_amdgcn_mbcnt_lo(0u, 0u);
    const uint64_t ntasks = (a.n + kTaskSym - 1) / kTaskSym;
    const uint64_t last = (a.n - 1) / kIdx;  // the last mark / index entry
    const uint64_t sym0 = t * kTaskSym;
    const uint64_t next = sym0 + kTaskSym;
    const uint64_t li = sym0 / kIdx + lane < last ? sym0 / kIdx + lane : last;  // the lane's entry (clamped)
    const uint64_t ni = (next / kIdx < last ? next / kIdx : last) + vz;         // the next task's first
    const uint64_t t1 = (t + 1 < ntasks ? t + 1 : ntasks - 1) + vz;
    const uint64_t t0 = t + vz;
    // the task's end (the next task's first bit) beside the lane's entry: a
    // scalar load with no dependence on it, so both are in flight together
    if (MODE == kIdxMark32 || (MODE == kIdxAny && SKIP && a.mark32)) {  // compact marks (k_mark_lite)
        r.m1 = a.mark32[ni];
        r.s1 = a.task_seg[t1];  // the next task's first mark's own segment
        r.s0 = a.task_seg[t0];
        r.m = a.mark32[li];
    } else if (MODE == kIdxAny && a.sub_abs64) {  // index-free streams: absolute start bit of every 64th symbol
        r.q1 = a.sub_abs64[ni];
        r.q = a.sub_abs64[li];
    } else if (MODE == kIdxSub16 || (MODE == kIdxAny && a.sub16)) {  // compact index: task base + u16 offset
        r.q1 = a.task_base[t1];
        r.q2 = a.chunk_start[a.nchunks + vz];
        r.q = a.task_base[t0];
        r.m = a.sub16[li];
    } else {
        r.q1 = a.chunk_start[(next < a.n ? next : sym0) / kChunk];
        r.m1 = a.sub_bit[ni];
        r.q2 = a.chunk_start[a.nchunks];
        r.q = a.chunk_start[sym0 / kChunk];
        r.m = a.sub_bit[li];
    }
    return r;
}
template <bool SKIP = false, int MODE = kIdxAny>
__device__ __forceinline__ Task task_finish(const DecodeArgs& a, uint64_t t, uint32_t lane, const TaskLoad& r) {
    Task k;
    k.sym0 = t * kTaskSym;
    k.nsym = static_cast<uint32_t>(a.n - k.sym0 < kTaskSym ? a.n - k.sym0 : kTaskSym);
    const uint32_t ls = lane * kLaneSym;
    k.cnt = ls >= k.nsym ? 0u : (k.nsym - ls < kLaneSym ? k.nsym - ls : kLaneSym);
    k.skip = 0;
    const uint64_t next = k.sym0 + kTaskSym;
    const bool tail = next >= a.n;  // the stream's last task
    uint64_t end;
    if (MODE == kIdxMark32 || (MODE == kIdxAny && SKIP && a.mark32)) {
        end = !tail ? static_cast<uint64_t>(r.s1) * a.seg_bits + mark32_rel(r.m1) +
                          static_cast<uint64_t>(mark32_skip(r.m1)) * a.max_len
                    : a.end_bit;
        k.lane_bit = k.cnt ? static_cast<uint64_t>(mark32_seg(r.m, r.s0)) * a.seg_bits + mark32_rel(r.m) : 0;
        k.skip = k.cnt ? mark32_skip(r.m) : 0u;
    } else if (MODE == kIdxAny && a.sub_abs64) {
        end = !tail ? r.q1 : a.end_bit;
        k.lane_bit = k.cnt ? r.q : 0;
        if constexpr (SKIP) {
            k.skip = static_cast<uint32_t>(k.lane_bit >> 48);
            k.lane_bit &= kSkipPosMask;
        }
    } else if (MODE == kIdxSub16 || (MODE == kIdxAny && a.sub16)) {
        end = !tail ? r.q1 : r.q2;
        k.lane_bit = k.cnt ? r.q + r.m : 0;
    } else {
        end = !tail ? r.q1 + r.m1 : r.q2;
        k.lane_bit = k.cnt ? r.q + r.m : 0;
    }
    // readfirstlane returns int: widen through uint32_t (no sign extension)
    const uint32_t f_lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(k.lane_bit)));
    const uint32_t f_hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(k.lane_bit >> 32)));
    const uint64_t first = (static_cast<uint64_t>(f_hi) << 32) | f_lo;
    if constexpr (SKIP)  // the next task's first bit lies within its skipped codes (used only now)
        if (MODE == kIdxAny && !a.mark32 && a.sub_abs64 && !tail) end = (end & kSkipPosMask) + (end >> 48) * a.max_len;
    k.end = end;
    k.b0 = (first >> 3) & ~15ull;
    uint64_t b1 = ((end + 7) >> 3) + 32;  // lookahead: window + the dword read ahead
    b1 = (b1 + 15) & ~15ull;
    k.len = static_cast<uint32_t>(b1 - k.b0 < 0xFFFFFFFFull ? b1 - k.b0 : 0xFFFFFFFFull);
    k.len = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(k.len)));  // uniform (scalar)
    return k;
}
template <bool SKIP = false>
__device__ __forceinline__ Task task_info(const DecodeArgs& a, uint64_t t, uint32_t lane) {
    return task_finish<SKIP>(a, t, lane, task_load<SKIP>(a, t, lane));
}

// The task's staged pieces (np = len / 16 when the range fits the stage)
// through a buffer resource clamped to the stream's last dword:
// unconditional loads (pieces past the range read zero), so they stay in
// flight while the current task decodes — a bounds-checked load with a
// byte-wise fallback made the compiler wait for them right after issue.
template <uint32_t CAP, uint32_t R>
__device__ __forceinline__ void issue_task_loads(const DecodeArgs& a, const Task& k, uint32_t lane, uint4 (&pre)[R]) {
    const uint32_t np = k.len <= CAP ? k.len / 16 : 0u;
    // the stream is only 4-B aligned: the readable range ends at the dword
    // holding its last byte (the buffer range check is per dword, so a 16-B
    // piece straddling the end returns its readable dwords and zeros)
    const uint64_t end4 = (a.comp_bytes + 3) & ~3ull;
    const uint64_t avail = end4 > k.b0 ? end4 - k.b0 : 0;
    const uint32_t nb = static_cast<uint32_t>(avail < 16ull * np ? avail : 16ull * np);
    const auto rs = buf_rsrc(nb ? a.comp + k.b0 : a.comp, nb);
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) pre[r] = buf_ld16(rs, (lane + 64 * r) * 16);
}

// dword sources for the lane decoders (stream order: the first byte is the
// most significant): the LDS stage (byte-swapped when staged), or global memory
struct LdsWords {
    const uint32_t* w;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return w[i]; }
};
// PAD stages (DecodeArgs::pad_stage): dword i of the stream at i ^ (((i >> 5)
// & 7) << 2) — the 16-B pieces of every 128-B block XOR-permuted by the
// block index, so lanes whose starts are ~32 m / k dwords apart (mean code
// lengths near 3.2, 4, 5.33, 8, 10.67 or 12 bits) spread over the banks
// instead of queueing on a few; same size as the plain stage (the round-1
// layout padded one piece per 8: 1/8 more LDS, 5 waves per SIMD instead of
// 6). Zipf (10.6 dwords per lane) decode 0.505 -> 0.497 ms, same box.
struct PaddedLdsWords {
    const uint32_t* w;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return w[i ^ ((i >> 3) & 28u)]; }
};
__device__ __forceinline__ uint32_t padded_piece(uint32_t p) { return p ^ ((p >> 3) & 7u); }
struct GlobalWords {
    const uint8_t* comp;
    uint64_t nbytes;
    uint64_t dw0;  // absolute dword index of word 0
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const {
        const uint64_t b = (dw0 + i) * 4;
        if (b + 4 <= nbytes) return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(comp + b));
        uint32_t v = 0;
        for (uint32_t k = 0; k < 4 && b + k < nbytes; ++k) v |= static_cast<uint32_t>(comp[b + k]) << (24 - 8 * k);
        return v;
    }
};

// ---------------------------------------------------------------------------
// k_decode_fixed: the same tasks, one letter per lookup. Every lane makes
// exactly 64 lookups, so every letter has a static place: four letters are
// joined in a register (v_perm) and a lane's 64 letters (16 registers) leave
// as four 16-B stores that together cover whole lines. There is no output
// stage in LDS (6 workgroups per CU instead of 3) and no lane waits for
// another (the multi-symbol decoder's lanes need different lookup counts).
// Per lookup: index, u16 table read, 64-bit shift by the entry (its low 6 bits
// are the code length), one subtraction for the valid-bit count and one
// v_perm; per two lookups a refill that ORs the next dword in unconditionally
// (the bits it lands on are the same stream bits) and advances when fewer
// than 32 bits were valid.
// ---------------------------------------------------------------------------

// nb (valid window bits) lives in the low 6 bits of X; the bits above are
// don't-care (X -= entry borrows only from them)
// Invariant: the window's valid bits end at stream bit 32 rp, so the lane's
// position after its 64 letters is 32 rp - nb (*end_rel, for the self-check).
// R: lookups per refill. After a refill the window holds >= 32 valid bits,
// so R codes of <= 32 / R bits fit: 2 for codes of <= 16 bits, 3 for <= 10,
// 4 for <= 8 (fewer stage reads per letter for shallow trees)
template <bool SLOW, bool SKIP, int R = 2, class Words>
__device__ __forceinline__ void decode_fixed64(const Words& src, uint32_t rel, uint32_t (&o)[16],
                                               const uint16_t* __restrict__ stab, uint32_t K,
                                               const uint32_t* __restrict__ glut, uint32_t Ks, uint32_t* end_rel,
                                               uint32_t skip, WaveStamps* ws, uint32_t* rp_out = nullptr) {
    uint32_t rp = rel >> 5;
    const uint32_t sh = rel & 31;
    uint64_t buf = static_cast<uint64_t>(src(rp) << sh) << 32;
    uint32_t X = 32 - sh;
    rp += 1;
    uint32_t nextw = src(rp);

#define FX_REFILL()                                                              \
    do {                                                                         \
        buf |= (static_cast<uint64_t>(nextw) << 32) >> (X & 63);                 \
        rp += (X & 32) ? 0u : 1u;                                                \
        X |= 32;                                                                 \
        nextw = src(rp);                                                         \
    } while (0)

#define FX_LOOKUP(i)                                                                          \
    do {                                                                                      \
        uint32_t e = stab[static_cast<uint32_t>(buf >> 32) >> (32 - K)];                      \
        if (SLOW && (e & kSsSlow)) {                                                          \
            FX_REFILL();                                                                      \
            uint32_t e1 = glut[static_cast<uint32_t>(buf >> (64 - Ks))];                      \
            uint32_t d = Ks;                                                                  \
            while (e1 & kLutPtr) {                                                            \
                const uint32_t idx = static_cast<uint32_t>((buf >> (56 - d)) & 0xFFu);        \
                e1 = glut[(e1 & ~kLutPtr) + idx];                                             \
                d += 8;                                                                       \
            }                                                                                 \
            const uint32_t l1 = (e1 >> 8) & 0xFFu;                                            \
            buf <<= l1;                                                                       \
            X -= l1;                                                                          \
            FX_REFILL();                                                                      \
            e = (e1 & 0xFFu) << 8;                                                            \
        }                                                                                     \
        buf <<= (e & 63u);                                                                    \
        X -= e;                                                                               \
        if (((i) & 3) == 0) o[(i) >> 2] = e >> 8;                                             \
        else o[(i) >> 2] = __builtin_amdgcn_perm(e, o[(i) >> 2],                              \
                                                 ((i) & 3) == 1 ? 0x0C0C0500u                 \
                                                 : ((i) & 3) == 2 ? 0x0C050100u : 0x05020100u); \
    } while (0)
// one code consumed, its letter dropped (the SKIP build's leading codes)
#define FX_STEP()                                                                             \
    do {                                                                                      \
        uint32_t e = stab[static_cast<uint32_t>(buf >> 32) >> (32 - K)];                      \
        if (SLOW && (e & kSsSlow)) {                                                          \
            FX_REFILL();                                                                      \
            uint32_t e1 = glut[static_cast<uint32_t>(buf >> (64 - Ks))];                      \
            uint32_t d1 = Ks;                                                                 \
            while (e1 & kLutPtr) {                                                            \
                const uint32_t idx = static_cast<uint32_t>((buf >> (56 - d1)) & 0xFFu);       \
                e1 = glut[(e1 & ~kLutPtr) + idx];                                             \
                d1 += 8;                                                                      \
            }                                                                                 \
            const uint32_t l1 = (e1 >> 8) & 0xFFu;                                            \
            buf <<= l1;                                                                       \
            X -= l1;                                                                          \
            FX_REFILL();                                                                      \
            e = 0;                                                                            \
        }                                                                                     \
        buf <<= (e & 63u);                                                                    \
        X -= e;                                                                               \
    } while (0)

#ifdef HUFF_SKIP_EXPERIMENT  // timing only (wrong letters): 1 = no skip codes, 2 = the wave's max for all lanes
    if constexpr (SKIP) skip = HUFF_SKIP_EXPERIMENT == 1 ? 0u : __reduce_max_sync(~0ull, skip);
#endif
    if constexpr (SKIP && R == 4 && kSkipR) {  // the same at 4 codes per refill (codes of <= 8 bits)
        for (uint32_t j = skip; j >= 4; j -= 4) {
            FX_REFILL();
            FX_STEP();
            FX_STEP();
            FX_STEP();
            FX_STEP();
        }
        if (skip & 2u) {
            FX_REFILL();
            FX_STEP();
            FX_STEP();
        }
        if (skip & 1u) {
            FX_REFILL();
            FX_STEP();
        }
    } else if constexpr (SKIP) {  // codes before this lane's first letter: decoded, not kept
        for (uint32_t j = skip; j >= 2; j -= 2) {
            FX_REFILL();
            FX_STEP();
            FX_STEP();
        }
        if (skip & 1u) {
            FX_REFILL();
            FX_STEP();
        }
    }
    if (ws) HUFF_STAMP(*ws, 3);
    static_assert(R >= 2 && R <= 4 && (!SLOW || R == 2), "2-4 lookups per refill (slow codes: 2)");
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        if (i % R == 0) FX_REFILL();
        FX_LOOKUP(i);
    }
    *end_rel = 32 * rp - (X & 63u);
    if (rp_out) *rp_out = rp;  // dwords [0, rp) became valid bits; dword rp was read ahead
#undef FX_STEP
#undef FX_LOOKUP
#undef FX_REFILL
}

template <bool SLOW, bool PAD, bool SKIP = false, int R = 2>
__device__ __forceinline__ void decode_fixed64_stage(const uint32_t* stage, uint32_t rel, uint32_t (&o)[16],
                                                     const uint16_t* __restrict__ stab, uint32_t K,
                                                     const uint32_t* __restrict__ glut, uint32_t Ks,
                                                     uint32_t* end_rel, uint32_t skip = 0,
                                                     WaveStamps* ws = nullptr) {
    if constexpr (PAD)
        decode_fixed64<SLOW, SKIP, R>(PaddedLdsWords{stage}, rel, o, stab, K, glut, Ks, end_rel, skip, ws);
    else
        decode_fixed64<SLOW, SKIP, R>(LdsWords{stage}, rel, o, stab, K, glut, Ks, end_rel, skip, ws);
}

// fallback for a task whose compressed range exceeds the stage: a compact
// loop straight from global memory, one letter per lookup stored as a byte
template <class Words>
__device__ __forceinline__ uint32_t decode_fixed_global(const Words& src, uint32_t rel, uint32_t cnt, uint8_t* dst,
                                                     const uint32_t* __restrict__ glut, uint32_t Ks,
                                                     uint32_t skip = 0) {
    uint32_t rp = rel >> 5;
    const uint32_t sh = rel & 31;
    uint64_t buf = ((static_cast<uint64_t>(src(rp)) << 32) | src(rp + 1)) << sh;
    uint32_t nb = 64 - sh;
    rp += 2;
    for (uint32_t j = 0; j < skip + cnt; ++j) {  // the first `skip` letters are dropped
        if (nb < 32) {
            buf |= static_cast<uint64_t>(src(rp)) << (32 - nb);
            nb += 32;
            ++rp;
        }
        uint32_t e1 = glut[static_cast<uint32_t>(buf >> (64 - Ks))];
        uint32_t d = Ks;
        while (e1 & kLutPtr) {
            const uint32_t idx = static_cast<uint32_t>((buf >> (56 - d)) & 0xFFu);
            e1 = glut[(e1 & ~kLutPtr) + idx];
            d += 8;
        }
        const uint32_t l1 = (e1 >> 8) & 0xFFu;
        buf <<= l1;
        nb -= l1;
        if (j >= skip) dst[j - skip] = static_cast<uint8_t>(e1);
    }
    return 32 * rp - nb;  // end position (valid bits end at 32 rp)
}

// 16-B LDS stage accesses: one may_alias vector type for every 16-B write
// and read of the stage, which the lane decoders also read as dwords
typedef uint32_t u32x4_alias __attribute__((ext_vector_type(4), may_alias));
__device__ __forceinline__ void st_stage16(void* p, uint4 v) {
    *reinterpret_cast<u32x4_alias*>(p) = u32x4_alias{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ uint4 ld_stage16(const void* p) {
    const u32x4_alias v = *reinterpret_cast<const u32x4_alias*>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Self-check (the CHECK build, HUFF_DEC_VARIANT=11): every lane's letters
// must end exactly where the next lane's restart entry (or, for the task's
// last lane, the next task's first bit) begins. A mismatch is counted in
// err[0]; the first one records (task, lane, expected, got) in err[1..6]. No
// trap and no device printf (a call would change the body's register
// allocation): the kernel drains and the host reports HUFF_E_CORRUPT.
__device__ __forceinline__ void fx_report(uint32_t* err, uint64_t task, uint32_t lane, uint64_t want, uint64_t got) {
    if (atomicAdd(err, 1u) == 0) {
        err[1] = static_cast<uint32_t>(task);
        err[2] = lane;
        err[3] = static_cast<uint32_t>(want);
        err[4] = static_cast<uint32_t>(want >> 32);
        err[5] = static_cast<uint32_t>(got);
        err[6] = static_cast<uint32_t>(got >> 32);
    }
}
template <bool CHECK>
__device__ __forceinline__ void fx_check(const DecodeArgs& a, const Task& k, uint64_t task, uint32_t lane,
                                         uint64_t got_abs, bool active) {
    if constexpr (CHECK) {
        const uint32_t nlo = static_cast<uint32_t>(__shfl_down(static_cast<int>(k.lane_bit), 1));
        const uint32_t nhi = static_cast<uint32_t>(__shfl_down(static_cast<int>(k.lane_bit >> 32), 1));
        const uint32_t ncnt = static_cast<uint32_t>(__shfl_down(static_cast<int>(k.cnt), 1));
        const uint64_t want = (lane < 63 && ncnt) ? ((static_cast<uint64_t>(nhi) << 32) | nlo) : k.end;
        if (active && got_abs != want) fx_report(a.err, task, lane, want, got_abs);
    }
}

template <bool SLOW, bool PAD, bool CHECK, bool SKIP = false, bool SMALL = false, int R = 2>
__device__ __forceinline__ void decode_fixed_body(const DecodeArgs& a) {
    constexpr uint32_t CAP = fx_stage_bytes<SMALL>();
    constexpr uint32_t kLoadRounds = load_rounds<SMALL>();
    constexpr int NT = kThreads;
    static_assert(!(CHECK && SKIP), "the self-check needs exact lane starts");
    constexpr int NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t K = a.stab_bits;
    const uint32_t nent = 1u << K;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = wave_index();
    uint16_t* stab = reinterpret_cast<uint16_t*>(lds);
    const uint32_t tab_words = (nent + 1) / 2;
    const uint32_t tab_rw = (tab_words + 3) & ~3u;
    // the wave's stage: dword view for the lane decoders, byte view for the
    // 16-B pieces (all 16-B accesses through u32x4_alias)
    uint32_t* stage = lds + tab_rw + wave * (CAP / 4);
    uint8_t* sb = reinterpret_cast<uint8_t*>(stage);
    const uint64_t ntasks = (a.n + kTaskSym - 1) / kTaskSym;
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * NW;
    uint64_t task = static_cast<uint64_t>(blockIdx.x) * NW + wave;
    Task cur{};
    uint4 pre[kLoadRounds];
    // timing builds: 0 entry, 1 table staged, 2 input staged, 3 skips done,
    // 4 letters done, 5 transposed, 6 stores issued (one-shot grid: a task per wave)
    WaveStamps ws;
    HUFF_STAMP(ws, 0);
    if constexpr (kEarlyLoads) {
        // the first task's index and input loads go out before the table is
        // staged (they hide the table copy of the one-shot grid), joined by a
        // bare barrier: the loads stay in flight across it
        const bool have = task < ntasks;
        const uint32_t tab_pieces = (tab_words + 3) / 4;
        const auto rtab = buf_rsrc(a.stab, tab_words * 4);
        constexpr int TP = (512 + NT - 1) / NT;  // 16-B pieces per thread: a table is <= 8 KiB
        uint4 tp[TP];
#pragma unroll
        for (int i = 0; i < TP; ++i) tp[i] = buf_ld16(rtab, (t + NT * i) * 16);
        if (have) {
            cur = task_info<SKIP>(a, task, lane);
            issue_task_loads<CAP>(a, cur, lane, pre);
        }
#pragma unroll
        for (int i = 0; i < TP; ++i)
            if (t + NT * i < tab_pieces) st_stage16(lds + 4 * (t + NT * i), tp[i]);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): table stores done; the input loads stay in flight
        __builtin_amdgcn_s_barrier();
        HUFF_STAMP(ws, 1);
        if (!have) return;
    } else {
        for (uint32_t i = t; i < tab_words; i += NT) lds[i] = reinterpret_cast<const uint32_t*>(a.stab)[i];
        __syncthreads();
        if (task >= ntasks) return;
        cur = task_info<SKIP>(a, task, lane);
    }

    // no software prefetch of the next task: its 20 registers would cost a
    // wave per SIMD; the other resident waves hide the load latency instead.
    // Stage ordering within the wave (no workgroup barrier: a wave's LDS ops
    // execute in issue order, wave_sync() = lgkmcnt(0) + a compiler barrier):
    //   stage writes (input) -> sync -> lane reads -> sync -> row writes
    //   (output transpose) -> sync -> row reads -> sync -> next task's writes
    while (true) {
        if constexpr (!kEarlyLoads) issue_task_loads<CAP>(a, cur, lane, pre);
        const uint32_t np = cur.len <= CAP ? cur.len / 16 : 0u;
#pragma unroll
        for (uint32_t r = 0; r < kLoadRounds; ++r) {
            const uint32_t p = lane + 64 * r;
            if (p < np) {
                const uint4 v = pre[r];
                st_stage16(sb + 16 * (PAD ? padded_piece(p) : p),
                           make_uint4(__builtin_bswap32(v.x), __builtin_bswap32(v.y), __builtin_bswap32(v.z),
                                      __builtin_bswap32(v.w)));
            }
        }
        const uint64_t nxt_task = task + step;
        const bool more = nxt_task < ntasks;
        wave_sync();
        HUFF_STAMP(ws, 2);

        const uint32_t rel = static_cast<uint32_t>(cur.lane_bit - cur.b0 * 8);
        uint8_t* dst = a.out + cur.sym0 + lane * kLaneSym;
        if (cur.len > CAP) {
            uint32_t e = 0;
            if (cur.cnt) e = decode_fixed_global(GlobalWords{a.comp, a.comp_bytes, cur.b0 / 4}, rel, cur.cnt, dst,
                                                 a.lut, a.lut_bits, SKIP ? cur.skip : 0u);
            fx_check<CHECK>(a, cur, task, lane, cur.b0 * 8 + e, cur.cnt != 0);
        } else if (cur.nsym == kTaskSym) {  // wave-uniform: every lane has 64 letters
            uint32_t o[16];
            uint32_t e = 0;
            decode_fixed64_stage<SLOW, PAD, SKIP, R>(stage, rel, o, stab, K, a.lut, a.lut_bits, &e, cur.skip, &ws);
            fx_check<CHECK>(a, cur, task, lane, cur.b0 * 8 + e, true);
            HUFF_STAMP(ws, 4);
            // transpose through the stage so every store instruction writes
            // 1 KiB contiguous (16 B per lane): lane-strided 16-B pieces cost
            // 4x the L2 write requests and stalled the TA (PMC)
            wave_sync();  // the wave's stage reads are done
            // nontemporal stores: the letters are written once and not read
            // back here (-2 % decode time against default-policy stores, same box)
            uint4* d4 = reinterpret_cast<uint4*>(a.out + cur.sym0) + lane;
            if constexpr (!SMALL) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    st_stage16(sb + row_piece(lane, q), make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]));
                wave_sync();
                HUFF_STAMP(ws, 5);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    st_nt(d4 + 64 * q, ld_stage16(sb + row_piece(16 * q + (lane >> 2), lane & 3)));
            } else {  // rows 0-31, then rows 32-63, through the 2 KiB they need
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h) {
                    if ((lane >> 5) == h) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            st_stage16(sb + row_piece(lane & 31, q),
                                       make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]));
                    }
                    wave_sync();
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        st_nt(d4 + 64 * (2 * h + q), ld_stage16(sb + row_piece(16 * q + (lane >> 2), lane & 3)));
                    wave_sync();  // the half's rows are read before the next half overwrites them
                }
                HUFF_STAMP(ws, 5);
            }
            HUFF_STAMP(ws, 6);
        } else if (cur.cnt) {
            uint32_t o[16];
            uint32_t e = 0;
            decode_fixed64_stage<SLOW, PAD, SKIP, R>(stage, rel, o, stab, K, a.lut, a.lut_bits, &e, cur.skip);
            // a lane with fewer than 64 letters decodes past its end: only full lanes are checked
            fx_check<CHECK>(a, cur, task, lane, cur.b0 * 8 + e, cur.cnt == kLaneSym);
            if (cur.cnt == kLaneSym) {
                uint4* d4 = reinterpret_cast<uint4*>(dst);
#pragma unroll
                for (int q = 0; q < 4; ++q) d4[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
            } else {
#pragma unroll
                for (uint32_t i = 0; i < kLaneSym; ++i)
                    if (i < cur.cnt) dst[i] = static_cast<uint8_t>(o[i >> 2] >> (8 * (i & 3)));
            }
        } else {
            fx_check<CHECK>(a, cur, task, lane, 0, false);  // keeps the shuffles wave-uniform
        }
        ws.flush(a.stamps, task);
        if (!more) break;
        wave_sync();  // the input stage is reused by the next task
        task = nxt_task;
        cur = task_info<SKIP>(a, task, lane);
        if constexpr (kEarlyLoads) issue_task_loads<CAP>(a, cur, lane, pre);
    }
}

// ---------------------------------------------------------------------------
// k_decode_dma: the same tasks and lane decoder, PERSISTENT waves with the
// next task's input in flight while the current one decodes. Where the time
// goes in the one-shot decoder (round-5 stamps, 1 GiB Zipf): of a wave's
// 16.6 K-cycle life, ~6 K wait for its table copy and first loads (HBM
// latency), 1.8 K stage the input, 7.5 K decode the 64 letters per lane. A
// register prefetch of the next task cost a wave per SIMD and lost (round 5,
// decode_prefetch/); here the prefetch goes straight to LDS by LDS-DMA
// (buffer_load_dwordx4 ... lds: no VGPR destination, no staging stores) into
// the wave's second stage buffer, so the load latency hides behind the
// decode. The stage holds the raw stream bytes (words are byte-swapped as
// they are read); the swizzled (PAD) layout is made on the SOURCE side
// (slot p receives piece padded_piece(p), an involution: the register path's
// layout). Column-stage A/B of this round (each lane loading its own rows so
// that refill reads are conflict-free): LDS cycles -16 %, time +1..8 %.
// PMC (profiles/r06/lds/): the one-shot decoder's LDS array is 87 % busy,
// 62 % of it bank conflicts, yet cutting those cycles did not pay: the wave's
// serial latency (memory, then the lookup chain) bounds it.
// ---------------------------------------------------------------------------
struct LdsWordsBS {  // raw stream bytes in LDS: big-endian words
    const uint32_t* w;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return __builtin_bswap32(w[i]); }
};
struct PaddedLdsWordsBS {
    const uint32_t* w;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return __builtin_bswap32(w[i ^ ((i >> 3) & 28u)]); }
};

typedef __attribute__((address_space(3))) void* lds_void_p;

// the task's pieces into the stage at `buf` (16 B per lane per instruction,
// LDS address = buf + 16 lane + 1 KiB r); pieces past the task's range or the
// stream read zero (the buffer range check), and a task longer than the
// stage loads nothing (it decodes from global memory)
template <uint32_t CAPB, bool PAD>
__device__ __forceinline__ void issue_task_dma(const DecodeArgs& a, const Task& k, uint32_t lane, uint32_t* buf) {
    constexpr uint32_t NPC = CAPB / 16;
    constexpr uint32_t R = (NPC + 63) / 64;
    const uint32_t np = k.len <= CAPB ? k.len / 16 : 0u;
    const uint64_t end4 = (a.comp_bytes + 3) & ~3ull;
    const uint64_t avail = end4 > k.b0 ? end4 - k.b0 : 0;
    const uint32_t nb = static_cast<uint32_t>(avail < 16ull * np ? avail : 16ull * np);
    const auto rs = buf_rsrc(nb ? a.comp + k.b0 : a.comp, nb);
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t p = lane + 64 * r;
        const uint32_t src = PAD ? padded_piece(p) : p;
        if (NPC % 64 == 0 || r + 1 < R || p < NPC)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_p)(buf + 256 * r), 16, src * 16, 0, 0, 0);
    }
}

template <bool SKIP, bool PAD, uint32_t CAPB>
__device__ __forceinline__ void decode_dma_body(const DecodeArgs& a) {
    constexpr int MODE = SKIP ? kIdxMark32 : kIdxSub16;  // the index forms the launcher admits
    // allocation floor of 80 VGPRs (the LDS of the small stages holds 5 waves
    // per SIMD anyway): at the compiler's 72 the window shift took its
    // amount from v71, the last register of the allocation — the gfx950
    // 64-bit shift hazard (tools/check_shift64.py)
    asm volatile("" ::: "v79");
    constexpr int NT = kThreads;
    constexpr int NW = NT / 64;
    constexpr bool HALVES = CAPB < 64 * kRowBytes;  // the output rows leave in two halves
    static_assert(CAPB % 16 == 0 && 32 * kRowBytes <= CAPB, "the output rows (or half) fit the stage");
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t K = a.stab_bits;
    const uint32_t nent = 1u << K;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = wave_index();
    const uint16_t* stab = reinterpret_cast<const uint16_t*>(lds);
    const uint32_t tab_words = (nent + 1) / 2;
    const uint32_t tab_rw = (tab_words + 3) & ~3u;
    uint32_t* const st0 = lds + tab_rw + wave * (2 * CAPB / 4);
    uint32_t* const st1 = st0 + CAPB / 4;
    const uint64_t ntasks = (a.n + kTaskSym - 1) / kTaskSym;
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * NW;
    uint64_t task = static_cast<uint64_t>(blockIdx.x) * NW + wave;
    Task cur{};
    TaskLoad nxt_raw{};
    WaveStamps ws;
    HUFF_STAMP(ws, 0);
    {
        // the table copy overlaps the first task's DMA and the second task's entries
        const uint32_t tab_pieces = (tab_words + 3) / 4;
        const auto rtab = buf_rsrc(a.stab, tab_words * 4);
        constexpr int TP = (512 + NT - 1) / NT;
        uint4 tp[TP];
#pragma unroll
        for (int i = 0; i < TP; ++i) tp[i] = buf_ld16(rtab, (t + NT * i) * 16);
        if (task < ntasks) {
            cur = task_finish<SKIP, MODE>(a, task, lane, task_load<SKIP, MODE>(a, task, lane));
            issue_task_dma<CAPB, PAD>(a, cur, lane, st0);
            nxt_raw = task_load<SKIP, MODE>(a, task + step < ntasks ? task + step : ntasks - 1, lane);
        }
#pragma unroll
        for (int i = 0; i < TP; ++i)
            if (t + NT * i < tab_pieces) st_stage16(lds + 4 * (t + NT * i), tp[i]);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): table stores done; the DMA stays in flight
        __builtin_amdgcn_s_barrier();
        HUFF_STAMP(ws, 1);
        if (task >= ntasks) return;
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the first stage has landed
    }
    bool odd = false;
    while (true) {
        // invariant: cur's bytes are in this wave's `stage` (its DMA retired by
        // a vmcnt wait of this wave), nxt's entries are loaded
        uint32_t* const stage = odd ? st1 : st0;
        uint8_t* const sb = reinterpret_cast<uint8_t*>(stage);
        const uint64_t ntask = task + step;
        const bool more = ntask < ntasks;
        Task nxt{};
        if (more) {
            nxt = task_finish<SKIP, MODE>(a, ntask, lane, nxt_raw);
            issue_task_dma<CAPB, PAD>(a, nxt, lane, odd ? st0 : st1);
        }
        // (a clamped task index past the last: loaded, never finished)
        const TaskLoad nn_raw = task_load<SKIP, MODE>(a, ntask + step < ntasks ? ntask + step : ntasks - 1, lane);
        HUFF_STAMP(ws, 2);
        const uint32_t rel = static_cast<uint32_t>(cur.lane_bit - cur.b0 * 8);
        uint8_t* dst = a.out + cur.sym0 + lane * kLaneSym;
        bool plain = false;  // the last VMEM ops of the task are its 4 row stores
        if (cur.len > CAPB) {
            if (cur.cnt)
                decode_fixed_global(GlobalWords{a.comp, a.comp_bytes, cur.b0 / 4}, rel, cur.cnt, dst, a.lut,
                                    a.lut_bits, SKIP ? cur.skip : 0u);
        } else if (cur.nsym == kTaskSym) {
            uint32_t o[16];
            uint32_t e = 0;
            if constexpr (PAD)
                decode_fixed64<false, SKIP>(PaddedLdsWordsBS{stage}, rel, o, stab, K, a.lut, a.lut_bits, &e, cur.skip, &ws);
            else
                decode_fixed64<false, SKIP>(LdsWordsBS{stage}, rel, o, stab, K, a.lut, a.lut_bits, &e, cur.skip, &ws);
            HUFF_STAMP(ws, 4);
            wave_sync();  // the wave's stage reads are done
            uint4* d4 = reinterpret_cast<uint4*>(a.out + cur.sym0) + lane;
            if constexpr (!HALVES) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    st_stage16(sb + row_piece(lane, q), make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]));
                wave_sync();
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    st_nt(d4 + 64 * q, ld_stage16(sb + row_piece(16 * q + (lane >> 2), lane & 3)));
            } else {
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h) {
                    if ((lane >> 5) == h) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            st_stage16(sb + row_piece(lane & 31, q),
                                       make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]));
                    }
                    wave_sync();
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        st_nt(d4 + 64 * (2 * h + q), ld_stage16(sb + row_piece(16 * q + (lane >> 2), lane & 3)));
                    wave_sync();
                }
            }
            plain = true;
            HUFF_STAMP(ws, 5);
        } else if (cur.cnt) {
            uint32_t o[16];
            uint32_t e = 0;
            if constexpr (PAD)
                decode_fixed64<false, SKIP>(PaddedLdsWordsBS{stage}, rel, o, stab, K, a.lut, a.lut_bits, &e, cur.skip, nullptr);
            else
                decode_fixed64<false, SKIP>(LdsWordsBS{stage}, rel, o, stab, K, a.lut, a.lut_bits, &e, cur.skip, nullptr);
            if (cur.cnt == kLaneSym) {
                uint4* d4 = reinterpret_cast<uint4*>(dst);
#pragma unroll
                for (int q = 0; q < 4; ++q) d4[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
            } else {
#pragma unroll
                for (uint32_t i = 0; i < kLaneSym; ++i)
                    if (i < cur.cnt) dst[i] = static_cast<uint8_t>(o[i >> 2] >> (8 * (i & 3)));
            }
        }
        HUFF_STAMP(ws, 6);
        ws.flush(a.stamps, task);
        if (!more) break;
        // the next stage has landed (and nn's entries): all but the row stores
        if (plain) __builtin_amdgcn_s_waitcnt(0x0f74);  // vmcnt(4)
        else __builtin_amdgcn_s_waitcnt(0x0f70);
        wave_sync();  // this stage's reads are done before a DMA rewrites it
        task = ntask;
        cur = nxt;
        nxt_raw = nn_raw;
        odd = !odd;
    }
}

// the DMA build's stage per buffer: 3 KiB (two halves of output rows) for
// streams of <= kSmallStageBits bits per symbol, else 4.5 KiB
template <bool SKIP, bool PAD, uint32_t CAPB>
__global__ __launch_bounds__(kThreads) void k_decode_dma(DecodeArgs a) {
    decode_dma_body<SKIP, PAD, CAPB>(a);
}

// Production kernels. The register allocation is the compiler's, with one
// floor for every swizzled-stage (PAD) body, the plain and the index-free skip
// build alike (kPadWaves waves per SIMD); `make` rejects any build in which a
// 64-bit shift takes its amount from the last allocated VGPR
// (tools/check_shift64.py, DESIGN.md §3 "The 64-bit shift hazard"), the
// hardware hazard behind every wrong-letter build of rounds 1-2.
// (R > 2 bodies unfloored took 90-113 VGPRs, the scheduler hoisting the
// lookups that the refills no longer separate: floored at the R = 2 body's
// occupancy)
template <bool PAD, int R = 2>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(PAD ? kPadWaves : (R > 2 ? 6 : 1), 8))) void k_decode_fixed(DecodeArgs a) {
    decode_fixed_body<false, PAD, false, false, false, R>(a);
}
template <bool PAD>
__global__ __launch_bounds__(kThreads) void k_decode_fixed_slow(DecodeArgs a) { decode_fixed_body<true, PAD, false>(a); }

// Self-checking build of the same body (HUFF_DEC_VARIANT=11): every lane's
// end bit is compared with its successor's restart entry
// (tests/test_gpu_decode_check.py)
template <bool SLOW, bool PAD>
__global__ __launch_bounds__(kThreads) void k_decode_fixed_chk(DecodeArgs a) { decode_fixed_body<SLOW, PAD, true>(a); }
// index-free streams with k_mark_lite's entries: each lane first decodes and
// drops its skip codes
// (forcing 7 or 8 waves per SIMD on the small-stage body spills 20 bytes
// per lane: not built)
template <bool SLOW, bool PAD, bool SMALL, int R = 2>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(PAD && !SLOW ? kPadWaves : (R > 2 ? (SMALL ? 7 : 6) : 1), 8))) void k_decode_fixed_skip(DecodeArgs a) {
    decode_fixed_body<SLOW, PAD, false, true, SMALL, R>(a);
}

}  // namespace

}  // namespace huff::dev

namespace huff::dev {

size_t decode_fixed_lds_bytes(uint32_t stab_bits, bool small) {
    const size_t tab_words = ((1u << stab_bits) + 1) / 2;
    return ((tab_words + 3) & ~size_t(3)) * 4 +
           static_cast<size_t>(kWaves) * (small ? fx_stage_bytes<true>() : fx_stage_bytes<false>());
}

// lookups per refill for codes of at most max_len bits (decode_fixed64's R)
static int lookups_per_refill(uint32_t max_len) {
    const char* e = std::getenv("HUFF_DEC_REFILL");  // read per call: tests flip it
    const int cap = e && e[0] >= '2' && e[0] <= '4' ? e[0] - '0' : 4;
    const int r = max_len <= 8 ? 4 : max_len <= 10 ? 3 : 2;
    return r < cap ? r : cap;
}

hipError_t launch_decode_fixed(const DecodeArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    // the small stage: the skip build with every code in the table (same-box
    // A/B, 1 GiB: index-free Zipf 1.153 vs 1.183 ms, text 1.055 vs 1.067; the
    // indexed decoder lost with it: Zipf 0.498 vs 0.478, text 0.416 vs 0.408,
    // its swizzled 4.5 KiB stage at 6 waves per SIMD beats the unswizzled
    // 3 KiB one at 8; profiles/r05/decode_stage/)
    const bool small = a.small_stage && a.skip_packed && a.max_len <= a.stab_bits;
    const size_t lds = decode_fixed_lds_bytes(a.stab_bits, small);
    const uint64_t ntasks = (a.n + kTaskSym - 1) / kTaskSym;
    const bool slow = a.max_len > a.stab_bits;
    const bool pad = a.pad_stage != 0;
    using K = void (*)(DecodeArgs);
    // [check mode][slow][pad]
    static const K table[2][2][2] = {
        {{k_decode_fixed<false>, k_decode_fixed<true>},
         {k_decode_fixed_slow<false>, k_decode_fixed_slow<true>}},
        {{k_decode_fixed_chk<false, false>, k_decode_fixed_chk<false, true>},
         {k_decode_fixed_chk<true, false>, k_decode_fixed_chk<true, true>}},
    };
    static const K skip_table[2][2] = {{k_decode_fixed_skip<false, false, false>, k_decode_fixed_skip<false, true, false>},
                                       {k_decode_fixed_skip<true, false, false>, k_decode_fixed_skip<true, true, false>}};
    // the small stage unswizzled: 79 VGPRs keep 6 waves per SIMD (the
    // swizzled body needs 81: 5)
    const K small_kern = k_decode_fixed_skip<false, false, true>;
    if (a.check_mode > 1 || (a.check_mode && !a.err)) return hipErrorInvalidValue;
    if (a.skip_packed && (a.check_mode || (!a.sub_abs64 && !(a.mark32 && a.task_seg && a.seg_bits))))
        return hipErrorInvalidValue;
    K kern = small ? small_kern
                   : (a.skip_packed ? skip_table[slow][pad] : table[a.check_mode][slow][pad]);
    // shallow trees: 3 or 4 lookups per refill (the production builds;
    // HUFF_DEC_REFILL=2 keeps two, for A/B)
    const int r = lookups_per_refill(a.max_len);
    if (!slow && !a.check_mode && r > 2) {
        static const K fx_r[2][2] = {{k_decode_fixed<false, 3>, k_decode_fixed<true, 3>},
                                     {k_decode_fixed<false, 4>, k_decode_fixed<true, 4>}};
        static const K skip_r[2][2] = {{k_decode_fixed_skip<false, false, false, 3>, k_decode_fixed_skip<false, true, false, 3>},
                                       {k_decode_fixed_skip<false, false, false, 4>, k_decode_fixed_skip<false, true, false, 4>}};
        static const K small_r[2] = {k_decode_fixed_skip<false, false, true, 3>, k_decode_fixed_skip<false, false, true, 4>};
        kern = small ? small_r[r - 3] : (a.skip_packed ? skip_r[r - 3][pad] : fx_r[r - 3][pad]);
    }
    size_t lds_bytes = lds;
    // (the index forms it reads: compact marks / the compact restart index)
    const bool dma = a.dma_stage && !a.check_mode && !slow &&
                     (a.skip_packed ? a.mark32 != nullptr : (a.sub16 != nullptr && !a.sub_abs64));
    if (dma) {  // k_decode_dma: persistent waves, two stage buffers each
        static const K dma_table[2][2][2] = {
            {{k_decode_dma<false, false, kInCap>, k_decode_dma<false, false, kInCapSmall>},
             {k_decode_dma<false, true, kInCap>, k_decode_dma<false, true, kInCapSmall>}},
            {{k_decode_dma<true, false, kInCap>, k_decode_dma<true, false, kInCapSmall>},
             {k_decode_dma<true, true, kInCap>, k_decode_dma<true, true, kInCapSmall>}}};
        const bool sm = a.small_stage != 0;
        kern = dma_table[a.skip_packed ? 1 : 0][pad][sm];
        const size_t tab_words = ((size_t(1) << a.stab_bits) + 1) / 2;
        lds_bytes = ((tab_words + 3) & ~size_t(3)) * 4 + size_t(kWaves) * 2 * (sm ? kInCapSmall : kInCap);
    }
    const uint64_t want = (ntasks + kWaves - 1) / kWaves;
    // production: one task per wave (a one-shot grid, as the byte map's): the
    // dispatcher refills the CUs as waves finish — same-box A/B against the
    // resident persistent grid Zipf 0.506 -> 0.501 ms, text 0.433 -> 0.423,
    // index-free text 1.18 -> 1.14 ms. The check build keeps the persistent
    // grid (and so does a HUFF_DIAG build run with HUFF_DEC_ONESHOT=0).
#ifdef HUFF_DIAG
    const char* o = std::getenv("HUFF_DEC_ONESHOT");
    const bool oneshot = !(o && *o == '0');
#else
    constexpr bool oneshot = true;
#endif
    uint64_t cap = want;
    if (a.check_mode || !oneshot || dma) {  // persistent grid = resident workgroups (registers and LDS both limit)
        int per_cu = 0;
        const hipError_t err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kThreads, lds_bytes);
        if (err != hipSuccess || per_cu < 1) per_cu = 1;
        cap = uint64_t(a.cu_count ? a.cu_count : 256) * per_cu;
    }
    const uint32_t grid = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(want, cap)));
    launch_k(kern, dim3(grid), dim3(kThreads), lds_bytes, s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
