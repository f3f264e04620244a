// ifdec.hip — single-pass index-free decode (comp.rs:487-519 on a stream
// with no restart index: every reference-written CompressData and .hff file).
//
// One kernel reads the compressed bits once and writes the letters once.
// The valid bits [0, B) are cut into segments of S bits (S a multiple of the
// gcd of the code lengths, so a segment start has a codeword boundary's
// residue). A BLOCK is one 256-lane workgroup over 256 consecutive segments;
// blocks overlap by one segment (block b covers segments 255 b ... 255 b +
// 255), so lane 0 of block b > 0 re-decodes block b-1's last segment only to
// find its exit, the block's ANCHOR.
//
//  1. stage: the block's bits (+ lookahead) go to LDS with coalesced 16-B
//     loads; a dynamic ticket orders the blocks (the look-back below only
//     waits on blocks that hold earlier tickets, so it cannot deadlock).
//  2. speculative decode: every lane decodes 64 codes from its segment's
//     first bit, one single-symbol lookup per code (u16 table in LDS, as
//     k_decode_fixed), keeping the letters in 16 registers and the position
//     after every 4th code (16 u16 in 8 registers). The exit (first boundary
//     at or past the segment end) and the letter count follow from those
//     positions plus at most 4 single steps; a lane with more than 64 codes
//     counts the rest with single steps.
//  3. fix-up: lane k restarts from lane k-1's exit (a true boundary once
//     lane k-1's path is true) and walks, keeping the letters (<= 32, in LDS),
//     until it lands on one of its recorded positions: from there the
//     speculative letters are the true ones (Huffman codes resynchronise
//     within a few codes: p50 11 bits, p99 81 bits on Zipf(1.2),
//     tools/sync_stats.py). A lane that does not land within 32 letters is a
//     SLOW lane (re-decoded whole from its true start at write-out); a slow
//     lane whose exit differs from its speculative exit makes its successor
//     walk again (a loop that is almost never entered).
//  4. counts: block scan of the true letter counts; the block's count is
//     published and its output offset found by decoupled look-back over the
//     blocks' (status, value) words. Lane 255's final exit must equal its
//     speculative exit (= the next block's anchor), else the kernel raises the
//     fallback flag and the host reruns the stream through the multi-kernel
//     path (indexless.hip). With bit 0 a true boundary and every anchor
//     confirmed, induction makes every block's path the true one.
//  5. write-out: every lane places its letters (the walk's prefix from LDS,
//     the kept register letters, a tail) in the block's LDS output image at
//     its offset, aligned so the image's 16-B pieces are the output's; the
//     image leaves as coalesced 16-B stores (byte stores at the two shared
//     ends). A block whose letters exceed the image writes bytes to HBM.
//
// Traffic: ceil(B/8) read + n written + 8 B per block; nothing in between
// goes to HBM.
#include <algorithm>

#include "bitreader.hpp"

// Blocks are numbered by a dynamic ticket (one device-scope atomic per block),
// so a block only ever waits on blocks that started before it. IFD_TICKET=0
// numbers them by blockIdx instead (relies on in-order dispatch; a violation
// ends in the spin limit and the host's fallback, not a hang): measured the
// same on 1 GiB Zipf/text (3.31 vs 3.31 ms), so the ticket stays.
#ifndef IFD_TICKET
#define IFD_TICKET 1
#endif
// IFD_DBG builds (tools/build_variant.sh) write each block's phase timestamps
// (s_memrealtime, 100 MHz) to a.dbg[8 b ...]: entry, staged, decoded, fixed,
// aggregate published, offset known, written; [7] = CU id << 32 | slow lanes
#ifndef IFD_DBG
#define IFD_DBG 0
#endif
#if IFD_DBG
#define IFD_T(k) do { if (t == 0 && a.dbg) a.dbg[8ull * b + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define IFD_T(k) do { } while (0)
#endif

namespace huff::dev {

namespace {

constexpr uint32_t kT = 256;
constexpr uint32_t kBlockSegs = kT - 1;  // segments a block owns (lane 0 is the anchor lane)
constexpr uint32_t kQn = 16;             // positions kept: after codes 4, 8, ..., 64
constexpr uint32_t kQm = 8;              // of them in LDS for the fix-up walk (codes 4 ... 32)
constexpr uint32_t kPfCap = kIfdPrefixCap;
// look-back word: status in bits [62, 64) (1 aggregate, 2 inclusive prefix),
// kStBroken (this block's true exit is not the next block's anchor), value
constexpr uint64_t kStAgg = 1ull << 62, kStIncl = 2ull << 62, kStBroken = 1ull << 61, kStVal = (1ull << 61) - 1;
constexpr uint32_t kSpinLimit = 1u << 20;  // look-back polls (>= ~1 s) before the kernel gives up (flag 4: the host
                                           // reruns the stream through the multi-kernel path)

struct Lds {
    uint16_t* stab;
    const uint32_t* stage;
    uint32_t stage_last;  // last readable dword of the stage
    uint16_t* qm;         // [kQm / 2][kT] u16 pairs, column-major (lane t's dword at row*kT + t)
    uint8_t* pf;          // [kPfCap / 4][kT] dwords of 4 letters, column-major
    uint32_t* ex;         // [kT] exits (bits from the stage's first bit)
    uint32_t* cnt;        // [8] wave totals of the scan
    uint32_t* misc;       // [16]
    uint8_t* out;         // the block's output image
};

__device__ __forceinline__ Lds lds_layout(const IfdArgs& a, uint8_t* base) {
    Lds L;
    L.stab = reinterpret_cast<uint16_t*>(base);
    L.stage = reinterpret_cast<const uint32_t*>(base + a.stage_off);
    L.stage_last = a.stage_bytes / 4 - 1;
    L.qm = reinterpret_cast<uint16_t*>(base + a.qm_off);
    L.pf = base + a.pf_off;
    L.ex = reinterpret_cast<uint32_t*>(base + a.ex_off);
    L.cnt = reinterpret_cast<uint32_t*>(base + a.cnt_off);
    L.misc = reinterpret_cast<uint32_t*>(base + a.misc_off);
    L.out = base + a.out_off;
    return L;
}

// A lane cursor over the stage (the fixed decoder's window): 64-bit window,
// valid bits in the low 6 bits of X (X -= entry borrows only above them), the
// next dword read one refill ahead; stage reads clamped to the stage.
struct Cur {
    const uint32_t* w;
    uint32_t last;
    uint64_t buf;
    uint32_t X, rp, nextw;
    __device__ __forceinline__ uint32_t word(uint32_t i) const { return w[i < last ? i : last]; }
    __device__ __forceinline__ void init(const Lds& L, uint32_t rel) {
        w = L.stage;
        last = L.stage_last;
        rp = rel >> 5;
        const uint32_t sh = rel & 31;
        buf = static_cast<uint64_t>(word(rp) << sh) << 32;
        X = 32 - sh;
        rp += 1;
        nextw = word(rp);
    }
    __device__ __forceinline__ void refill() {
        buf |= (static_cast<uint64_t>(nextw) << 32) >> (X & 63);
        rp += (X & 32) ? 0u : 1u;
        X |= 32;
        nextw = word(rp);
    }
    __device__ __forceinline__ uint32_t pos() const { return 32 * rp - (X & 63); }
    // the next code's entry (length in bits [0, 6), letter in [8, 16)),
    // consumed; codes longer than K through the global multi-level table
    template <bool SLOW>
    __device__ __forceinline__ uint32_t step(const uint16_t* stab, uint32_t K, const uint32_t* glut, uint32_t Kg) {
        uint32_t e = stab[static_cast<uint32_t>(buf >> 32) >> (32 - K)];
        if (SLOW && (e & kSsSlow)) {
            refill();
            uint32_t e1 = glut[static_cast<uint32_t>(buf >> (64 - Kg))];
            uint32_t d = Kg;
            while (e1 & kLutPtr) {
                const uint32_t idx = static_cast<uint32_t>((buf >> (56 - d)) & 0xFFu);
                e1 = glut[(e1 & ~kLutPtr) + idx];
                d += 8;
            }
            const uint32_t l1 = (e1 >> 8) & 0xFFu;
            buf <<= l1;
            X -= l1;
            refill();
            return ((e1 & 0xFFu) << 8) | l1;
        }
        buf <<= (e & 63u);
        X -= e;
        return e;
    }
    // one code with a refill first (walks that stop anywhere)
    template <bool SLOW>
    __device__ __forceinline__ uint32_t step1(const uint16_t* stab, uint32_t K, const uint32_t* glut, uint32_t Kg) {
        refill();
        return step<SLOW>(stab, K, glut, Kg);
    }
};

// Walk single codes from boundary p (< end) to the first boundary at or past
// end: n codes, ending at the returned exit. last: the stream's final
// segment, whose final code is dropped when it crosses B (= end), as the
// reference's walk drops an incomplete code (comp.rs:493-516).
template <bool SLOW>
__device__ __forceinline__ uint32_t walk_count(const Lds& L, const IfdArgs& a, uint32_t p, uint32_t end, bool last,
                                               uint32_t& n) {
    Cur c;
    c.init(L, p);
    uint32_t prev = p;
    while (p < end) {
        const uint32_t e = c.step1<SLOW>(L.stab, a.stab_bits, a.lut, a.lut_bits);
        prev = p;
        p += e & 63u;
        ++n;
    }
    if (last && p > end) {
        --n;
        p = prev;
    }
    return p;
}

// `count` letters decoded from boundary p into dst[0, count) (LDS image or HBM)
template <bool SLOW, class Dst>
__device__ __forceinline__ void emit_run(const Lds& L, const IfdArgs& a, uint32_t p, uint32_t count, Dst dst) {
    Cur c;
    c.init(L, p);
    for (uint32_t j = 0; j < count; ++j) dst[j] = static_cast<uint8_t>(c.step1<SLOW>(L.stab, a.stab_bits, a.lut, a.lut_bits) >> 8);
}

__device__ __forceinline__ uint32_t qget(const uint32_t (&q)[kQn / 2], int c) { return (q[c >> 1] >> (16 * (c & 1))) & 0xFFFFu; }

template <bool SLOW>
__global__ __launch_bounds__(kT) void k_ifd(IfdArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const Lds L = lds_layout(a, smem);
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t K = a.stab_bits;
#if IFD_DBG
    const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
#endif

    // ---- 1. ticket, table, stage -------------------------------------------
#if IFD_TICKET
    if (t == 0) L.misc[0] = atomicAdd(a.ticket, 1u);
#endif
    {
        const uint32_t tab_words = ((1u << K) + 1) / 2;
        uint32_t* tw = reinterpret_cast<uint32_t*>(L.stab);
        for (uint32_t i = t; i < tab_words; i += kT) tw[i] = reinterpret_cast<const uint32_t*>(a.stab)[i];
    }
    __syncthreads();
#if IFD_TICKET
    const uint32_t b = __builtin_amdgcn_readfirstlane(L.misc[0]);
#else
    const uint32_t b = blockIdx.x;
#endif
    if (b >= a.nblocks) return;  // never: the grid is nblocks workgroups
#if IFD_DBG
    if (t == 0 && a.dbg) a.dbg[8ull * b] = t_entry;
#endif
    const uint64_t seg0 = static_cast<uint64_t>(b) * kBlockSegs;
    const uint64_t byte_lo = ((seg0 * a.seg_bits) >> 3) & ~15ull;
    const uint64_t bit_lo = byte_lo * 8;
    {
        const uint64_t avail = a.comp_bytes > byte_lo ? ((a.comp_bytes + 3) & ~3ull) - byte_lo : 0;
        const uint32_t nb = static_cast<uint32_t>(avail < a.stage_bytes ? avail : a.stage_bytes);
        const auto rs = buf_rsrc(nb ? a.comp + byte_lo : a.comp, nb);
        uint4* w4 = reinterpret_cast<uint4*>(const_cast<uint32_t*>(L.stage));
        const uint32_t np = a.stage_bytes / 16;
        for (uint32_t p0 = t; p0 < np; p0 += 8 * kT) {
            uint4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = buf_ld16(rs, (p0 + k * kT) * 16);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (p0 + k * kT < np)
                    w4[p0 + k * kT] = make_uint4(__builtin_bswap32(v[k].x), __builtin_bswap32(v[k].y),
                                                 __builtin_bswap32(v[k].z), __builtin_bswap32(v[k].w));
        }
    }
    __syncthreads();

    IFD_T(1);
    // ---- 2. speculative decode of 64 codes -----------------------------------
    const uint64_t k = seg0 + t;
    const bool live = k < a.nseg;
    const bool last_seg = k + 1 == a.nseg;
    const uint32_t rel0 = static_cast<uint32_t>(seg0 * a.seg_bits - bit_lo) + t * a.seg_bits;
    uint64_t end_abs = (k + 1) * a.seg_bits;
    if (end_abs > a.valid_bits) end_abs = a.valid_bits;
    const uint32_t relend = live ? static_cast<uint32_t>(end_abs - bit_lo) : rel0;
    const uint32_t Lk = relend - rel0;

    uint32_t o[16], q[kQn / 2];
    {
        Cur c;
        c.init(L, rel0);
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            if ((i & 1) == 0) c.refill();
            const uint32_t e = c.step<SLOW>(L.stab, K, a.lut, a.lut_bits);
            if ((i & 3) == 0) o[i >> 2] = e >> 8;
            else o[i >> 2] = __builtin_amdgcn_perm(e, o[i >> 2], (i & 3) == 1 ? 0x0C0C0500u : (i & 3) == 2 ? 0x0C050100u : 0x05020100u);
            if ((i & 3) == 3) {
                const uint32_t p = c.pos() - rel0;
                const int cq = i >> 2;
                q[cq >> 1] = (cq & 1) ? (q[cq >> 1] | (p << 16)) : p;
            }
        }
    }
    // the exit: after the last recorded position below the segment end, at
    // most 4 single steps (or, past 64 codes, as many as the lane has)
    uint32_t n_spec = 0, pstart = 0;
#pragma unroll
    for (int c = 0; c < static_cast<int>(kQn); ++c) {
        const uint32_t v = qget(q, c);
        const bool below = v < Lk;
        pstart = below ? v : pstart;
        n_spec = below ? static_cast<uint32_t>(4 * (c + 1)) : n_spec;
    }
    const bool ovf = n_spec == 64;  // all 64 codes start before the end: more may follow
    const uint32_t q15 = qget(q, 15);
    uint32_t x_spec = rel0;
    if (live && Lk) x_spec = walk_count<SLOW>(L, a, rel0 + pstart, relend, last_seg, n_spec);
    // the merge list (positions after codes 4 ... 32) for the fix-up walk
#pragma unroll
    for (int r = 0; r < static_cast<int>(kQm / 2); ++r) reinterpret_cast<uint32_t*>(L.qm)[r * kT + t] = q[r];
    L.ex[t] = x_spec;
    __syncthreads();
    IFD_T(2);

    // ---- 3. fix-up -----------------------------------------------------------
    const bool owned = live && (t > 0 || b == 0);
    uint32_t ns = rel0, tp = 0, qk = 0;
    bool slow = false;
    if (owned && t > 0) {
        ns = L.ex[t - 1];
        if (ns != rel0) {
            Cur w;
            w.init(L, ns);
            uint32_t pos = ns, c = 0;
            uint32_t qc = rel0 + L.qm[2 * t];
            bool merged = false;
            while (tp < kPfCap && pos < relend) {
                const uint32_t e = w.step1<SLOW>(L.stab, K, a.lut, a.lut_bits);
                L.pf[4 * ((tp >> 2) * kT + t) + (tp & 3)] = static_cast<uint8_t>(e >> 8);
                ++tp;
                pos += e & 63u;
                while (qc < pos && c + 1 < kQm) {
                    ++c;
                    qc = rel0 + L.qm[2 * ((c >> 1) * kT + t) + (c & 1)];
                }
                if (qc == pos && pos < relend) {
                    merged = true;
                    qk = 4 * (c + 1);
                    break;
                }
                if (qc < pos) break;  // past every recorded position
            }
            slow = !merged;
        }
    }
    uint32_t n_true = 0, x_true = x_spec;
    if (owned) {
        if (slow) x_true = walk_count<SLOW>(L, a, ns, relend, last_seg, n_true);
        else n_true = tp + n_spec - qk;
    }
    // a slow lane that left its segment elsewhere: the successor walks again
    // (rounds until nothing changes; each round is a full walk of the lanes
    // concerned, and almost never runs). Also run after an anchor repair
    // (lane 0's exit replaced by the previous block's true exit).
    auto settle = [&](uint32_t changed) {
        while (__syncthreads_or(changed)) {
            L.ex[t] = x_true;
            __syncthreads();
            changed = 0;
            if (owned && t > 0) {
                const uint32_t nn = L.ex[t - 1];
                if (nn != ns) {
                    ns = nn;
                    slow = true;
                    n_true = 0;
                    const uint32_t xn = walk_count<SLOW>(L, a, ns, relend, last_seg, n_true);
                    changed = xn != x_true;
                    x_true = xn;
                }
            }
        }
    };
    settle(owned && x_true != x_spec);
    IFD_T(3);
#if IFD_DBG
    {
        const int ns_slow = __syncthreads_count(slow);
        if (t == 0 && a.dbg) a.dbg[8ull * b + 7] = (static_cast<uint64_t>(__smid()) << 32) | static_cast<uint32_t>(ns_slow);
    }
#endif

    // ---- 4. counts, anchors, look-back ---------------------------------------
    // The block's count assumes its anchor (lane 0's speculative exit) is
    // true. Lane 255 checks the NEXT block's anchor: its true exit must equal
    // its speculative exit; if not, the block publishes its status with the
    // BROKEN bit and its true exit (ex_w), and the next block repairs itself
    // from that exit (settle above) before publishing its inclusive prefix;
    // a scanning block that meets a BROKEN record drops the next block's
    // aggregate and waits for its inclusive prefix instead.
    auto count = [&](uint32_t& off, uint32_t& total) {
        const uint32_t mine = owned ? n_true : 0u;
        const uint32_t inc = wave_scan_incl(mine);
        __syncthreads();  // L.cnt may still be read by a previous count
        if (lane == 63) L.cnt[wave] = inc;
        __syncthreads();
        uint32_t before = 0, cb = 0;
#pragma unroll
        for (uint32_t w = 0; w < kT / 64; ++w) {
            before += w < wave ? L.cnt[w] : 0u;
            cb += L.cnt[w];
        }
        off = before + inc - mine;
        total = cb;
    };
    uint32_t off_l = 0, cb = 0;
    count(off_l, cb);
    const bool has_next = b + 1 < a.nblocks;
    if (t == kT - 1) L.misc[4] = has_next && live && x_true != x_spec;
    __syncthreads();
    auto spin_load = [&](uint64_t v) -> uint64_t {  // thread 0: a status word once published
        for (uint32_t spins = 0;; ++spins) {
            const uint64_t s = __hip_atomic_load(a.status + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((s >> 62) != 0) return s;
            if (spins > kSpinLimit) {
                atomicOr(a.flags, 4u);  // a predecessor never published: report, do not hang
                return kStIncl;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    };
    // Look-back (wave 0, lane 0 publishes). The aggregate published first assumes this
    // block's anchor is true; a BROKEN bit on any record met on the way back
    // means some later block may be repairing itself, so the scan then waits
    // for the predecessor's inclusive record instead, whose BROKEN bit and
    // value are final (a record's BROKEN bit changes only in a block that
    // repairs, and only a BROKEN predecessor makes a block repair).
    if (wave == 0) {
        const uint64_t brk = L.misc[4] ? kStBroken : 0ull;
        uint64_t O = 0;
        uint32_t repair = 0;
        if (b > 0) {
            if (lane == 0)
                __hip_atomic_store(a.status + b, kStAgg | brk | cb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            IFD_T(4);
            // windows of 64 predecessors, nearest in lane 0: the window is
            // used once every word up to its nearest inclusive prefix (or all
            // 64 words) is published; the aggregates before that prefix, and
            // the prefix, are summed (words before block 0 read as prefix 0)
            bool seen = false;
            int64_t top = static_cast<int64_t>(b) - 1;
            for (uint32_t spins = 0;;) {
                const int64_t v = top - static_cast<int64_t>(lane);
                const uint64_t s = v >= 0 ? __hip_atomic_load(a.status + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                          : kStIncl;
                const uint64_t incl = __ballot((s >> 62) == 2);
                const uint64_t ready = __ballot((s >> 62) != 0);
                const uint32_t fi = incl ? static_cast<uint32_t>(__builtin_ctzll(incl)) : 64u;
                const uint64_t need = fi >= 63 ? ~0ull : ((2ull << fi) - 1);
                if ((ready & need) != need) {
                    if (++spins > kSpinLimit) {
                        if (lane == 0) atomicOr(a.flags, 4u);  // a predecessor never published: report, do not hang
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                const uint32_t av = lane < fi ? static_cast<uint32_t>(s & kStVal) : 0u;
                O += __builtin_amdgcn_readlane(static_cast<int>(wave_scan_incl(av)), 63) & 0xFFFFFFFFull;
                seen |= __ballot(lane <= fi && (s & kStBroken) != 0) != 0;
                if (fi < 64) {
                    const uint64_t iv = s & kStVal;
                    O += (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(iv >> 32), static_cast<int>(fi)))) << 32) |
                         static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(iv), static_cast<int>(fi)));
                    break;
                }
                top -= 64;
            }
            if (lane == 0 && seen) {
                uint64_t r = spin_load(b - 1);
                for (uint32_t spins = 0; (r >> 62) != 2; ++spins) {
                    if (spins > kSpinLimit) {
                        atomicOr(a.flags, 4u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    r = spin_load(b - 1);
                }
                O = r & kStVal;
                if (r & kStBroken) {  // this block's anchor is not a true boundary: its true exit
                    uint64_t entry = 0;
                    for (uint32_t spins = 0; spins <= kSpinLimit && !entry; ++spins)
                        entry = __hip_atomic_load(a.exits + b - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (!entry) atomicOr(a.flags, 4u);
                    repair = 1;
                    L.misc[5] = entry ? static_cast<uint32_t>(entry - 1 - bit_lo) : 0u;
                }
            }
        }
        if (lane == 0) {
            L.misc[1] = static_cast<uint32_t>(O);
            L.misc[2] = static_cast<uint32_t>(O >> 32);
            L.misc[6] = repair;
        }
    }
    __syncthreads();
    IFD_T(5);
    if (L.misc[6]) {  // repair: lane 0's exit is the previous block's true exit
        if (t == 0) x_true = L.misc[5];
        settle(t == 0);
        count(off_l, cb);
    }
    // the final exit for the next block (read only if this block's final
    // record is BROKEN), then the final record
    if (t == kT - 1) {
        L.misc[4] = has_next && live && x_true != x_spec;
        if (has_next) __hip_atomic_store(a.exits + b, bit_lo + x_true + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (t == 0) {
        const uint64_t O = (static_cast<uint64_t>(L.misc[2]) << 32) | L.misc[1];
        __hip_atomic_store(a.status + b, kStIncl | (L.misc[4] ? kStBroken : 0ull) | (O + cb), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        if (b + 1 == a.nblocks) *a.total = O + cb;
    }
    if (live && last_seg && a.end_bit) *a.end_bit = bit_lo + x_true;
    __syncthreads();
    const uint64_t O = (static_cast<uint64_t>(L.misc[2]) << 32) | L.misc[1];
    if (O + cb > a.out_cap) {  // the caller's buffer is too small: count only
        if (t == 0) atomicOr(a.flags, 2u);
        return;
    }

    // ---- 5. write-out ----------------------------------------------------------
    const uint32_t img0 = static_cast<uint32_t>(O & 15);
    const bool big = img0 + cb > a.out_img;
    if (big) {  // straight to HBM, a byte at a time (rare: letters beyond the image)
        if (owned) emit_run<SLOW>(L, a, ns, n_true, a.out + O + off_l);
        return;
    }
    const uint32_t D = img0 + off_l;  // the lane's first letter in the image
    if (owned) {
        if (slow) {
            emit_run<SLOW>(L, a, ns, n_true, L.out + D);
        } else {
            for (uint32_t j = 0; j < tp; ++j) L.out[D + j] = L.pf[4 * ((j >> 2) * kT + t) + (j & 3)];
            // register letters [qk, nk): letter j at image byte F + j
            const uint32_t nk = n_spec < 64 ? n_spec : 64u;
            const int32_t F = static_cast<int32_t>(D + tp) - static_cast<int32_t>(qk);
            const uint32_t r = static_cast<uint32_t>(F) & 3u;
            const int32_t m0 = F >> 2;  // floor
            uint32_t* img32 = reinterpret_cast<uint32_t*>(L.out);
            uint32_t vf = 0, vl = 0;
            const int32_t jf = static_cast<int32_t>(qk + r) >> 2, jl = static_cast<int32_t>(nk - 1 + r) >> 2;
#pragma unroll
            for (int i = 0; i <= 16; ++i) {
                const uint32_t hi = i < 16 ? o[i] : 0u, lo = i > 0 ? o[i - 1] : 0u;
                const uint32_t v = r ? __builtin_amdgcn_alignbyte(hi, lo, 4 - r) : hi;
                const int32_t j0 = 4 * i - static_cast<int32_t>(r);  // letter in the dword's byte 0
                if (nk > qk && j0 >= static_cast<int32_t>(qk) && j0 + 4 <= static_cast<int32_t>(nk)) img32[m0 + i] = v;
                vf = i == jf ? v : vf;
                vl = i == jl ? v : vl;
            }
            if (nk > qk) {
                // the partial dwords at both ends: byte stores of this lane's letters only
                for (int32_t s = 0; s < 4; ++s) {
                    const int32_t jA = 4 * jf - static_cast<int32_t>(r) + s;
                    if (jA >= static_cast<int32_t>(qk) && jA < static_cast<int32_t>(nk) &&
                        !(4 * jf - static_cast<int32_t>(r) >= static_cast<int32_t>(qk) && 4 * jf - static_cast<int32_t>(r) + 4 <= static_cast<int32_t>(nk)))
                        L.out[4 * (m0 + jf) + s] = static_cast<uint8_t>(vf >> (8 * s));
                    const int32_t jB = 4 * jl - static_cast<int32_t>(r) + s;
                    if (jl != jf && jB >= static_cast<int32_t>(qk) && jB < static_cast<int32_t>(nk) &&
                        !(4 * jl - static_cast<int32_t>(r) >= static_cast<int32_t>(qk) && 4 * jl - static_cast<int32_t>(r) + 4 <= static_cast<int32_t>(nk)))
                        L.out[4 * (m0 + jl) + s] = static_cast<uint8_t>(vl >> (8 * s));
                }
            }
            if (ovf && n_spec > 64) emit_run<SLOW>(L, a, rel0 + q15, n_spec - 64, L.out + D + tp + (64 - qk));
        }
    }
    __syncthreads();
    // the image to HBM: 16-B pieces, whole where the block owns all 16 bytes
    const uint64_t gbase = O - img0;
    const uint32_t end = img0 + cb;
    const uint32_t npieces = (end + 15) / 16;
    for (uint32_t p = t; p < npieces; p += kT) {
        const uint32_t lo = 16 * p;
        if (lo >= img0 && lo + 16 <= end) {
            st_nt(reinterpret_cast<uint4*>(a.out + gbase + lo), *reinterpret_cast<const uint4*>(L.out + lo));
        } else {
            for (uint32_t i = lo; i < lo + 16; ++i)
                if (i >= img0 && i < end) a.out[gbase + i] = L.out[i];
        }
    }
    IFD_T(6);
}

}  // namespace

size_t ifd_lds_bytes(const IfdArgs& a) { return a.out_off + a.out_img; }

IfdArgs ifd_layout(uint32_t stab_bits, uint32_t seg_bits, uint32_t max_len) {
    IfdArgs a{};
    auto up16 = [](uint32_t x) { return (x + 15u) & ~15u; };
    const uint32_t tab = up16(((1u << stab_bits) + 1) / 2 * 4);
    // the block's bits from its 16-B aligned first byte (< 128 bits before the
    // first segment), 256 segments, the last code's overrun and the refill's
    // read-ahead
    a.stage_bytes = up16((128 + kT * seg_bits + max_len + 96 + 7) / 8) + 16;
    a.stage_off = tab;
    a.qm_off = a.stage_off + a.stage_bytes;
    a.pf_off = a.qm_off + (kQm / 2) * kT * 4;
    a.ex_off = a.pf_off + (kPfCap / 4) * kT * 4;
    a.cnt_off = a.ex_off + kT * 4;
    a.misc_off = a.cnt_off + 64;
    a.out_off = a.misc_off + 64;
    a.out_img = up16(16 + kT * 64);
    return a;
}

uint32_t ifd_blocks(uint64_t nseg) { return nseg <= 1 ? 1u : static_cast<uint32_t>((nseg - 1 + kBlockSegs - 1) / kBlockSegs); }

hipError_t launch_ifd(const IfdArgs& a, hipStream_t s) {
    if (a.nseg == 0) return hipSuccess;
    const bool slow = a.max_len > a.stab_bits;
    hipLaunchKernelGGL(slow ? k_ifd<true> : k_ifd<false>, dim3(a.nblocks), dim3(kT), ifd_lds_bytes(a), s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
