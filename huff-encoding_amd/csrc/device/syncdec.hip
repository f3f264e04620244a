// syncdec.hip — index-free decode in ONE pass over the stream: every
// reference-written stream (CompressData::to_bytes containers, `.hff` files)
// carries no restart index (comp.rs:279-300), so decompress (comp.rs:487-519)
// must find the code boundaries itself.
//
// The pipeline of indexless.hip walks the stream twice: a speculative pass
// that only counts codes per segment, fix-up and scan kernels, marks, and a
// decoder that re-reads the stream and skips codes from the nearest sample.
// Here one kernel does it all, per TILE of 256 segments of S bits (one
// workgroup, a lane per segment):
//  1. stage the tile's bits in LDS (one read of the stream), walk a short
//     lead-in before each segment to its first code boundary (codes
//     resynchronise within ~11 bits at the median), and decode the segment's
//     letters straight into registers (kCap letters, static places: four per
//     VGPR), counting them, until the first boundary at or past the segment
//     end (the exit; a code that would cross the valid bits is dropped);
//  2. in-tile fix-up: a lane whose entry differs from its predecessor's exit
//     walks both paths until they meet (merged: a few true letters before the
//     merge point, the rest of its register letters shifted), or, rarely, is
//     re-counted from the true entry and its letters left to k_sync_tail;
//  3. decoupled look-back over the tiles (a dynamic ticket orders them): each
//     tile publishes its count, first entry and last exit in one 8-B word (A),
//     sums its predecessors' words back to one with an inclusive prefix (P),
//     checking that every tile on the way started at its predecessor's exit
//     (else it waits for its predecessor's P), then fixes its first lane if
//     its entry was wrong and publishes P;
//  4. output: each wave ORs its lanes' letters, realigned to their byte
//     offsets, into a zeroed LDS window (aliasing the now dead stage) and
//     stores it as 16-B pieces, contiguous per instruction.
// Letters a lane could not hold (more than kCap, or a lane re-counted from a
// new entry) become jobs for k_sync_tail, which decodes them serially from
// global memory after this kernel; it also publishes the letter count to the
// host. HBM traffic: the stream once, the letters once (plus ~8 B per tile).
//
// Applies to byte letters with every code in the single-symbol table
// (max_len <= stab_bits <= 12); other streams keep indexless.hip's pipeline.
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kCap = kSyncCap;       // letters per lane held in registers
constexpr uint32_t kRegs = kCap / 4;
constexpr uint32_t kBlocks = kCap / 8;    // decode steps in blocks of 8 (a refill every 2)
constexpr uint32_t kHead = 32;            // a merged lane's true letters before the merge point, at most
constexpr uint32_t kHeadRegs = kHead / 4;
constexpr uint32_t kWin = kSyncWin;       // output window per wave (bytes), aliasing the stage
constexpr uint32_t kSpinMax = 1u << 20;   // look-back polls before giving up (a hang guard, never expected)
constexpr uint32_t kMisMax = 64;          // look-backs that met a tile started off its predecessor's exit, at most

// tile word: [62, 64) state (1 = aggregate A, 2 = inclusive prefix P)
//   A: [0, 44) the tile's letter count, [44, 50) its first entry - tile start,
//      [50, 56) its last exit - tile end
//   P: [0, 50) inclusive prefix (letters of tiles 0..t), [50, 56) last exit - tile end
constexpr uint64_t kStA = 1ull << 62, kStP = 2ull << 62;
__device__ __forceinline__ uint64_t word_a(uint64_t agg, uint32_t e0, uint32_t xl) {
    return kStA | (static_cast<uint64_t>(xl) << 50) | (static_cast<uint64_t>(e0) << 44) | agg;
}
__device__ __forceinline__ uint64_t word_p(uint64_t incl, uint32_t xl) {
    return kStP | (static_cast<uint64_t>(xl) << 50) | incl;
}

// stage cursor (the words are byte-swapped when staged): 64-bit window, valid
// bits in the low 6 bits of X, refilled unconditionally every two codes (as
// decode_wave.hip's decode_fixed64); the window's valid bits end at 32 rp
struct Cur {
    uint64_t buf;
    uint32_t X, rp, nextw;
    __device__ __forceinline__ void init(const uint32_t* w, uint32_t p) {
        rp = p >> 5;
        const uint32_t sh = p & 31;
        buf = static_cast<uint64_t>(w[rp] << sh) << 32;
        X = 32 - sh;
        rp += 1;
        nextw = w[rp];
    }
    __device__ __forceinline__ void refill(const uint32_t* w) {
        buf |= (static_cast<uint64_t>(nextw) << 32) >> (X & 63);
        rp += (X & 32) ? 0u : 1u;
        X |= 32;
        nextw = w[rp];
    }
    __device__ __forceinline__ uint32_t pos() const { return 32 * rp - (X & 63); }
    __device__ __forceinline__ uint32_t step(const uint16_t* tab, uint32_t K) {
        const uint32_t e = tab[static_cast<uint32_t>(buf >> 32) >> (32 - K)];
        buf <<= (e & 63u);
        X -= e;
        return e;
    }
};

// the entry of the code at stage bit p (no cursor: the rare fix-up walks)
__device__ __forceinline__ uint32_t peek(const uint32_t* w, const uint16_t* tab, uint32_t K, uint32_t p) {
    const uint32_t i = p >> 5, sh = p & 31;
    const uint32_t top = sh ? (w[i] << sh) | (w[i + 1] >> (32 - sh)) : w[i];
    return tab[top >> (32 - K)];
}

// codes from stage bit p to the first boundary at or past `end`: count and
// exit; a code crossing the valid bits (vb) is dropped (comp.rs:493-516)
__device__ __forceinline__ void count_walk(const uint32_t* w, const uint16_t* tab, uint32_t K, uint32_t p,
                                           uint32_t end, uint32_t vb, uint32_t& cnt, uint32_t& ex) {
    uint32_t c = 0;
    while (p < end) {
        p += peek(w, tab, K, p) & 63u;
        ++c;
    }
    if (p > vb) {
        p = vb;
        --c;
    }
    cnt = c;
    ex = p;
}

// Writes bytes [lo, hi) of a lane's byte stream v (R registers,
// little-endian: byte j of the stream is byte j % 4 of v[j / 4]) to the
// window, the stream's byte 0 at window byte `rel` (may be negative or past
// the window: only the window's bytes are touched). Dwords wholly inside are
// plain stores; the two partial dwords at the ends (shared with the
// neighbouring lanes' letters) go byte by byte.
template <int R>
__device__ __forceinline__ void put_stream(uint8_t* win, const uint32_t (&v)[R], int32_t rel, int32_t lo, int32_t hi) {
    const int32_t b0 = rel + lo > 0 ? rel + lo : 0;
    const int32_t b1 = rel + hi < static_cast<int32_t>(kWin) ? rel + hi : static_cast<int32_t>(kWin);
    if (b0 >= b1) return;
    const int32_t s = rel & 3;
    const int32_t base = (rel >> 2) - (s == 0 ? 1 : 0);
    const uint32_t sh = static_cast<uint32_t>(4 - s) & 3u;
    uint32_t* w32 = reinterpret_cast<uint32_t*>(win);
#pragma unroll
    for (int k = 0; k <= R; ++k) {
        const int32_t d = base + k;
        const int32_t x0 = 4 * d, x1 = 4 * d + 4;  // the dword's window bytes
        if (x1 <= b0 || x0 >= b1) continue;
        const uint32_t hv = k < R ? v[k] : 0u, lv = k > 0 ? v[k - 1] : 0u;
        const uint32_t val = __builtin_amdgcn_alignbyte(hv, lv, sh);
        if (x0 >= b0 && x1 <= b1) {
            w32[d] = val;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (x0 + q >= b0 && x0 + q < b1) win[x0 + q] = static_cast<uint8_t>(val >> (8 * q));
        }
    }
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* red) {
    const uint32_t incl = wave_scan_incl(v);
    if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) t += red[k];
    __syncthreads();
    return t;
}

struct LaneFix {  // a lane's state against its (current) true entry
    uint32_t te;       // the entry it assumes (stage bit)
    uint32_t ca, cb;   // merged: true letters before the merge point, speculative ones skipped
    uint32_t head[kHeadRegs];  // the ca true letters (bytes)
    uint32_t cf, xf;   // final count and exit
    bool redo;         // letters from k_sync_tail (no merge, or a long way to it)
};

// the lane's state for entry te against its speculative path from es
__device__ __forceinline__ void fix_lane(LaneFix& f, const uint32_t* w, const uint16_t* tab, uint32_t K,
                                         uint32_t te, uint32_t es, uint32_t cs, uint32_t xs, uint32_t end,
                                         uint32_t vb) {
    f.te = te;
    f.ca = f.cb = 0;
#pragma unroll
    for (uint32_t k = 0; k < kHeadRegs; ++k) f.head[k] = 0;
    f.redo = false;
    f.cf = cs;
    f.xf = xs;
    if (te == es) return;
    uint32_t pa = te, pb = es, ca = 0, cb = 0;
    uint32_t h[kHeadRegs];
#pragma unroll
    for (uint32_t k = 0; k < kHeadRegs; ++k) h[k] = 0;
    bool merged = false;
    for (;;) {
        if (pa == pb) {
            merged = true;
            break;
        }
        if (pa >= end || pa > vb || pb > vb || ca > kHead || cb > kHead) break;
        if (pa < pb) {
            const uint32_t e = peek(w, tab, K, pa);
            if (ca < kHead) {  // (static register places: a select per word)
                const uint32_t b = ((e >> 8) & 0xFFu) << (8 * (ca & 3));
#pragma unroll
                for (uint32_t k = 0; k < kHeadRegs; ++k) h[k] |= (ca >> 2) == k ? b : 0u;
            }
            ++ca;
            pa += e & 63u;
        } else {
            pb += peek(w, tab, K, pb) & 63u;
            ++cb;
        }
    }
    if (merged && ca <= kHead && cb <= kHead && cb <= cs) {
        f.ca = ca;
        f.cb = cb;
#pragma unroll
        for (uint32_t k = 0; k < kHeadRegs; ++k) f.head[k] = h[k];
        f.cf = ca + cs - cb;
        return;
    }
    f.redo = true;
    count_walk(w, tab, K, te, end, vb, f.cf, f.xf);
}

__global__ __launch_bounds__(kThreads) void k_sync_decode(SyncDecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    __shared__ uint32_t ex_s[kThreads], red[kWaves], misc[8];
    __shared__ unsigned long long excl_s;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    // timing builds: 0 entry, 1 staged, 2 lead-in, 3 letters, 4 in-tile
    // fix-up, 5 look-back, 6 prefix, 7 letters out
    WaveStamps ws;
    HUFF_STAMP(ws, 0);
#ifdef HUFF_SD_NOTICKET  // timing experiment only: tiles in blockIdx order (no forward-progress guarantee)
    if (t == 0) misc[0] = blockIdx.x;
#else
    if (t == 0) misc[0] = atomicAdd(a.ctrl + kSyncTicket, 1u);
#endif
    // tables: the single-symbol u16 table first
    const uint32_t K = a.stab_bits;
    const uint32_t tab_words = ((1u << K) + 1) / 2;
    const uint32_t tab_rw = (tab_words + 3) & ~3u;
    {
        const auto rt = buf_rsrc(a.stab, tab_words * 4);
        uint4 tp[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) tp[i] = buf_ld16(rt, (t + kThreads * i) * 16);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            if (t + kThreads * i < tab_rw / 4) reinterpret_cast<uint4*>(lds)[t + kThreads * i] = tp[i];
    }
    __syncthreads();
    const uint64_t tile = misc[0];
    const uint16_t* tab = reinterpret_cast<const uint16_t*>(lds);
    uint32_t* w = lds + tab_rw;  // the stage, then (phase 4) the output windows
    const uint64_t S = a.seg_bits, B = a.valid_bits;
    const uint64_t seg0 = tile * kThreads;
    const uint64_t tile_bit = seg0 * S;
    const uint64_t tile_end = tile_bit + kThreads * S;  // nominal: exits are relative to it
    // stage [byte_lo, byte_hi): the lead-in before the first segment, the
    // lookahead past the last (the last code and lanes still stepping while
    // others finish read there)
    const uint64_t bit_lo = tile_bit - (tile_bit < a.lead0_bits ? tile_bit : a.lead0_bits);
    const uint64_t byte_lo = (bit_lo >> 3) & ~15ull;
    const uint64_t base = byte_lo * 8;
    {
        const uint64_t hi_bit = tile_end < B ? tile_end : B;
        uint64_t byte_hi = ((hi_bit + 7) >> 3) + kSyncLook;
        if (byte_hi > a.comp_bytes) byte_hi = a.comp_bytes;
        const uint32_t nbytes = static_cast<uint32_t>(byte_hi - byte_lo);
        const uint32_t np = (nbytes + 8 + 15) / 16;  // + the two zero words
        const auto rs = buf_rsrc(a.comp + byte_lo, (nbytes + 15) & ~15u);
        uint4* w4 = reinterpret_cast<uint4*>(w);
        for (uint32_t p0 = t; p0 < np; p0 += 8 * kThreads) {
            uint4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = buf_ld16(rs, (p0 + k * kThreads) * 16);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (p0 + k * kThreads < np)
                    w4[p0 + k * kThreads] = make_uint4(__builtin_bswap32(v[k].x), __builtin_bswap32(v[k].y),
                                                       __builtin_bswap32(v[k].z), __builtin_bswap32(v[k].w));
        }
    }
    __syncthreads();
    HUFF_STAMP(ws, 1);

    // ---- phase 1: lead-in, then the segment's letters into registers ------
    const uint64_t gi = seg0 + t;
    const bool have = gi < a.nseg;
    const uint32_t vb = static_cast<uint32_t>((B < tile_end + 4096 ? B : tile_end + 4096) - base);  // valid bits, stage-relative (clamped)
    const uint64_t s_abs = have ? gi * S : tile_bit;
    const uint32_t start = static_cast<uint32_t>(s_abs - base);
    const uint32_t end = have ? static_cast<uint32_t>((gi + 1 == a.nseg ? B : s_abs + S) - base) : start;
    Cur c;
    uint32_t es = start;
    if (have && s_abs) {
        // lane 0 walks a longer lead-in: its entry is the tile's, which the
        // successors' look-backs check against this tile's predecessor
        const uint32_t lw = t == 0 ? a.lead0_bits : a.lead_bits;
        const uint32_t lead = lw < s_abs ? lw : static_cast<uint32_t>(s_abs);
        uint32_t p = start - lead;
        c.init(w, p);
        for (;;) {
            uint32_t L[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if ((k & 1) == 0) c.refill(w);
                L[k] = c.step(tab, K) & 63u;
            }
            uint32_t ex = ~0u;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                p += L[k];
                ex = (ex == ~0u && p >= start) ? p : ex;
            }
            if (ex != ~0u) {
                es = ex < vb ? ex : vb;  // a code crossing the valid bits: none starts in the segment
                break;
            }
        }
    }
    HUFF_STAMP(ws, 2);
    uint32_t o[kRegs];
#pragma unroll
    for (uint32_t k = 0; k < kRegs; ++k) o[k] = 0;
    bool live = have && es < end && es < vb;
    uint32_t cs = 0, xs = es, pcap = 0;
    bool ov = false;
    uint32_t pos = es;
    c.init(w, es);
#pragma unroll
    for (uint32_t blk = 0; blk < kBlocks; ++blk) {
        if (__ballot(live) == 0) break;
        if (live) {
            uint32_t e[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                if ((k & 1) == 0) c.refill(w);
                e[k] = c.step(tab, K);
                const uint32_t r = 2 * blk + k / 4;
                if ((k & 3) == 0) o[r] = e[k] >> 8;
                else o[r] = __builtin_amdgcn_perm(e[k], o[r], (k & 3) == 1 ? 0x0C0C0500u
                                                               : (k & 3) == 2 ? 0x0C050100u : 0x05020100u);
            }
            const uint32_t pe = c.pos();
            if (pe >= end) {  // the exit lies in this block
                uint32_t q = pos, ex = 0;
                int h = -1;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    q += e[k] & 63u;
                    const bool f = h < 0 && q >= end;
                    h = f ? k : h;
                    ex = f ? q : ex;
                }
                uint32_t n = 8 * blk + static_cast<uint32_t>(h) + 1;
                if (ex > vb) {  // an incomplete final code is dropped
                    ex = vb;
                    --n;
                }
                cs = n;
                xs = ex;
                // the block's letters past the exit are not this lane's
                const uint32_t keep = n - 8 * blk;  // 0..8
                const uint64_t m = keep >= 8 ? ~0ull : ((1ull << (8 * keep)) - 1);
                o[2 * blk] &= static_cast<uint32_t>(m);
                o[2 * blk + 1] &= static_cast<uint32_t>(m >> 32);
                live = false;
            }
            pos = pe;
        }
    }
    if (live) {  // more than kCap letters: count on; the rest go to k_sync_tail
        ov = true;
        pcap = pos;
        uint32_t n;
        count_walk(w, tab, K, pos, end, vb, n, xs);
        cs = kCap + n;
    }
    if (!have) {
        cs = 0;
        xs = es;
    }
    HUFF_STAMP(ws, 3);

    // ---- phase 2: in-tile fix-up ----------------------------------------
    // te of lane i is lane i-1's exit; lane 0's comes from the look-back
    LaneFix f;
    f.te = es;
    f.ca = f.cb = 0;
#pragma unroll
    for (uint32_t k = 0; k < kHeadRegs; ++k) f.head[k] = 0;
    f.cf = cs;
    f.xf = xs;
    f.redo = false;
    ex_s[t] = xs;
    auto settle = [&](uint32_t te0) {
        for (;;) {
            __syncthreads();
            const uint32_t te = t ? ex_s[t - 1] : te0;
            bool changed = false;
            if (have && te != f.te) {
                fix_lane(f, w, tab, K, te, es, cs, xs, end, vb);
                if (f.xf != ex_s[t]) {
                    ex_s[t] = f.xf;
                    changed = true;
                }
            }
            if (!__syncthreads_or(changed)) break;
        }
    };
    settle(es);
    HUFF_STAMP(ws, 4);

    // ---- phase 3: decoupled look-back over the tiles (wave 0) ------------
    // lane l of wave 0 reads the word of tile t-1-64r-l (round r), so a round
    // costs one memory latency for 64 tiles; the predecessors' aggregates are
    // summed back to the nearest inclusive prefix, and every tile on the way
    // must have started at its predecessor's exit (the pairs of neighbouring
    // lanes), else the tile waits for its predecessor's prefix (and many
    // such waits abort the decode: the host then takes the pipeline)
    const uint32_t agg = block_sum(have ? f.cf : 0u, red);
#if defined(HUFF_SD_NOLOOK)  // timing experiment only (wrong output): no look-back wait
    if (t == 0) {
        __hip_atomic_store(a.tile + tile, word_p(tile * 20000ull, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        excl_s = tile * 20000ull;
        misc[1] = static_cast<uint32_t>(es + base - tile_bit);
    }
    if (false) {
#else
    if (wave == 0) {
#endif
        uint64_t excl = 0;
        uint32_t X = 0;  // the previous tile's last exit - this tile's start
        if (tile > 0) {
            if (lane == 0) {
                const uint32_t e0 = static_cast<uint32_t>(es + base - tile_bit);  // lane 0's entry - tile start
                const uint32_t xl = static_cast<uint32_t>(ex_s[kThreads - 1] + base - tile_end);
                __hip_atomic_store(a.tile + tile, word_a(agg, e0 & 63u, xl & 63u), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            auto poll = [&](uint64_t j, uint64_t need) {
                uint64_t v;
                for (uint32_t it = 0;; ++it) {
                    v = __hip_atomic_load(a.tile + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (v >= need) break;
                    // never expected: say so instead of hanging the GPU (one
                    // tile's timeout releases every other waiting tile)
                    if (it > kSpinMax ||
                        ((it & 255) == 255 &&
                         __hip_atomic_load(a.ctrl + kSyncErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                        atomicOr(a.ctrl + kSyncErr, 1u);
                        v = kStP;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                return v;
            };
            uint64_t acc = 0;
            uint32_t carry_e0 = 0;
            bool mism = false;
            for (uint32_t r = 0;; ++r) {
                const int64_t j = static_cast<int64_t>(tile) - 1 - 64 * static_cast<int64_t>(r) - lane;
                const uint64_t v = j >= 0 ? poll(static_cast<uint64_t>(j), kStA) : kStP;  // before tile 0: prefix 0
                const bool isP = v >= kStP;
                const uint32_t xr = static_cast<uint32_t>(v >> 50) & 63u, e0v = static_cast<uint32_t>(v >> 44) & 63u;
                if (r == 0) X = static_cast<uint32_t>(__shfl(static_cast<int>(xr), 0));
                uint32_t e0n = static_cast<uint32_t>(__shfl_up(static_cast<int>(e0v), 1));  // tile j+1's entry
                if (lane == 0) e0n = carry_e0;
                const bool mis = j >= 0 && (lane > 0 || r > 0) && xr != e0n;
                const uint64_t pm = __ballot(isP);
                const uint32_t fp = pm ? static_cast<uint32_t>(__builtin_ctzll(pm)) : 64u;
                const uint64_t rel = fp >= 63 ? ~0ull : ((2ull << fp) - 1);  // lanes up to the nearest prefix
                if (__ballot(mis) & rel) {
                    mism = true;
                    break;
                }
                const uint32_t sc = wave_scan_incl(isP ? 0u : static_cast<uint32_t>(v & ((1ull << 44) - 1)));
                if (fp < 64) {
                    const uint64_t ip = static_cast<uint64_t>(__shfl(static_cast<long long>(v & ((1ull << 50) - 1)),
                                                                     static_cast<int>(fp)));
                    const uint32_t before = fp ? static_cast<uint32_t>(__shfl(static_cast<int>(sc), static_cast<int>(fp) - 1)) : 0u;
                    acc += before + ip;
                    break;
                }
                acc += static_cast<uint32_t>(__shfl(static_cast<int>(sc), 63));
                carry_e0 = static_cast<uint32_t>(__shfl(static_cast<int>(e0v), 63));
            }
            excl = acc;
            if (mism) {  // a tile on the way started off its predecessor's exit: its own prefix, when final
                if (lane == 0 && atomicAdd(a.ctrl + kSyncMis, 1u) >= kMisMax) atomicOr(a.ctrl + kSyncErr, 1u);
                const uint64_t v = poll(tile - 1, kStP);
                excl = v & ((1ull << 50) - 1);
                X = static_cast<uint32_t>(v >> 50) & 63u;
            }
        }
        if (lane == 0) {
            excl_s = excl;
            misc[1] = X;
        }
    }
    __syncthreads();
    HUFF_STAMP(ws, 5);
    // lane 0 from the true entry (nearly always its own)
    settle(static_cast<uint32_t>(tile_bit + misc[1] - base));
    const uint32_t cf = have ? f.cf : 0u;
    const uint32_t pre = [&] {  // exclusive prefix of the final counts in the tile
        const uint32_t incl = wave_scan_incl(cf);
        if (lane == 63) red[wave] = incl;
        __syncthreads();
        uint32_t p = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) p += k < static_cast<int>(wave) ? red[k] : 0u;
        return p + incl - cf;
    }();
    const uint64_t excl = excl_s;
    HUFF_STAMP(ws, 6);
    if (t == kThreads - 1) {
        const uint64_t incl = excl + pre + cf;
        const uint32_t xl = static_cast<uint32_t>(f.xf + base - tile_end);
        __hip_atomic_store(a.tile + tile, word_p(incl, xl & 63u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (seg0 + kThreads >= a.nseg) a.total[0] = incl;  // the last tile: the letter count (k_sync_tail publishes it)
    }

    // ---- phase 4: letters out --------------------------------------------
    const uint64_t G = excl + pre;  // this lane's first letter
    if (have && cf) {
        if (f.redo) {
            const uint32_t j = atomicAdd(a.ctrl + kSyncJobs, 1u);
            if (j < a.job_cap) {
                a.jobs[3 * j] = base + f.te;
                a.jobs[3 * j + 1] = G;
                a.jobs[3 * j + 2] = cf;
            }
        } else if (ov) {  // the speculative letters past kCap
            const uint32_t j = atomicAdd(a.ctrl + kSyncJobs, 1u);
            if (j < a.job_cap) {
                a.jobs[3 * j] = base + pcap;
                a.jobs[3 * j + 1] = G + f.ca + (kCap - f.cb);
                a.jobs[3 * j + 2] = cs - kCap;
            }
        }
    }
    const bool regs = have && !f.redo && cs > f.cb;  // letters to write from the registers
    // the wave's span of letters, clipped to the caller's capacity
    const uint64_t cap = a.out_cap;
    const uint64_t lo_l = __shfl(static_cast<long long>(G), 0);
    const uint64_t hi_l = __shfl(static_cast<long long>(G + cf), 63);
    const uint64_t lo = lo_l < cap ? lo_l : cap, hi = hi_l < cap ? hi_l : cap;
    __syncthreads();  // every lane is done with the stage: it becomes the output windows
    if (lo >= hi) {
        HUFF_STAMP(ws, 7);
        ws.flush(a.stamps, tile * kWaves + wave);
        return;
    }
#ifdef HUFF_SD_NOOUT  // timing experiment only: no letters out
    if (lo < hi) return;
#endif
    uint32_t* win = w + wave * (kWin / 4);
    uint8_t* winb = reinterpret_cast<uint8_t*>(win);
    const uintptr_t o0 = reinterpret_cast<uintptr_t>(a.out);
    const uintptr_t A = (o0 + lo) & ~static_cast<uintptr_t>(15);
    const uint32_t rounds = static_cast<uint32_t>((o0 + hi - A + kWin - 1) / kWin);

    for (uint32_t r = 0; r < rounds; ++r) {
        const uintptr_t wa = A + static_cast<uintptr_t>(r) * kWin;

        // the letters [cb, min(cs, kCap)) from the registers after the ca true
        // letters of a merged lane (none for the others)
        if (regs)
            put_stream<kRegs>(winb, o, static_cast<int32_t>(static_cast<int64_t>(o0 + G + f.ca - f.cb - wa)),
                              static_cast<int32_t>(f.cb), static_cast<int32_t>(cs < kCap ? cs : kCap));
        if (regs && f.ca)
            put_stream<kHeadRegs>(winb, f.head, static_cast<int32_t>(static_cast<int64_t>(o0 + G - wa)), 0,
                                  static_cast<int32_t>(f.ca));
        wave_sync();
#pragma unroll
        for (uint32_t i = 0; i < kWin / 1024; ++i) {
            const uint32_t q = lane + 64 * i;
            const uintptr_t pa = wa + 16 * q;
            const uintptr_t b0 = pa > o0 + lo ? pa : o0 + lo, b1 = pa + 16 < o0 + hi ? pa + 16 : o0 + hi;
            if (b0 >= b1) continue;
            const uint4 v = reinterpret_cast<const uint4*>(win)[q];
            if (b0 == pa && b1 == pa + 16) {
                st_nt(reinterpret_cast<uint4*>(pa), v);
            } else {  // the span's first and last pieces (shared with the neighbouring waves)
                const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
                for (uintptr_t b = b0; b < b1; ++b)
                    *reinterpret_cast<uint8_t*>(b) = static_cast<uint8_t>(vv[(b - pa) >> 2] >> (8 * ((b - pa) & 3)));
            }
        }
        wave_sync();
    }
    HUFF_STAMP(ws, 7);
    ws.flush(a.stamps, tile * kWaves + wave);
}

// The letters k_sync_decode left (lanes re-counted from a new entry, letters
// past kCap): one job per lane, decoded serially from global memory with the
// single-symbol table; then the letter count to the host (tagged, as
// k_hist_publish) once every earlier kernel of the decode is done.
__global__ __launch_bounds__(256) void k_sync_tail(SyncDecArgs a) {
    const uint32_t nj = __hip_atomic_load(a.ctrl + kSyncJobs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t njobs = nj < a.job_cap ? nj : a.job_cap;
    const uint32_t K = a.stab_bits;
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    for (uint64_t j = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < njobs;
         j += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        uint64_t p = a.jobs[3 * j];
        const uint64_t off = a.jobs[3 * j + 1], n = a.jobs[3 * j + 2];
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t win = src.window(p);
            const uint32_t e = a.stab[static_cast<uint32_t>(win >> (64 - K))];
            if (off + i < a.out_cap) a.out[off + i] = static_cast<uint8_t>(e >> 8);
            p += e & 63u;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.host_total) {
        const uint32_t err = __hip_atomic_load(a.ctrl + kSyncErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t tot = err || nj > a.job_cap ? kSyncBad : a.total[0];
        __hip_atomic_store(a.host_total, (a.tag << 48) | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

size_t sync_decode_lds_bytes(const SyncDecArgs& a) {
    const size_t tab = (((((1u << a.stab_bits) + 1) / 2) + 3) & ~3u) * 4;
    const size_t stage = ((static_cast<size_t>(kThreads) * a.seg_bits + a.lead0_bits + 7) / 8 + kSyncLook + 64 + 15) / 16 * 16;
    return tab + (stage > kWaves * kWin ? stage : kWaves * kWin);
}

hipError_t launch_sync_decode(const SyncDecArgs& a, hipStream_t s) {
    if (a.nseg == 0) return hipSuccess;
    if (a.stab_bits == 0 || a.stab_bits > 12 || a.lead_bits > a.seg_bits || a.lead0_bits < a.lead_bits ||
        !a.ctrl || !a.tile || !a.total)
        return hipErrorInvalidValue;
    const uint64_t ntiles = (a.nseg + kThreads - 1) / kThreads;
    launch_k(k_sync_decode, dim3(static_cast<uint32_t>(ntiles)), dim3(kThreads), sync_decode_lds_bytes(a), s, a);
    launch_k(k_sync_tail, dim3(64), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
