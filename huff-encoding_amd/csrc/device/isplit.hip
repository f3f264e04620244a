// isplit.hip — index-free decode split at the scan (comp.rs:487-519 on a
// stream with no restart index: every CompressData the reference writes,
// comp.rs:279-300, and every .hff file, huff/src/comp.rs:232-280).
//
// The valid bits [0, B) are cut into SEGMENTS of S bits (S a multiple of the
// gcd g of the code lengths, so a segment start has a codeword boundary's
// residue) and every segment into R LANES: lane q of segment i owns the codes
// from the first boundary at or past theta(i, q) = i S + q S / R (for q > 0
// the first boundary the walk met there, see below) to the next lane's start.
//
//  A  k_split_sync: one workgroup over 256 segments staged in LDS (segwalk.hpp).
//     Each lane walks its segment speculatively from i S (multi-code steps
//     through the walk table), noting a merge sample every kSampBits bits and
//     a CHECKPOINT at the first step end at or past each theta(i, q): the
//     start of output lane q, with the letters before it. Then the in-group
//     fix-up: lane i restarts from lane i-1's exit and walks single codes
//     until it lands on one of its samples (the paths have merged; counts
//     shift by the index difference) or passes its end (a new exit: the
//     successor is listed for k_fix_rec). Checkpoints the fix-up walk passes
//     before the merge are replaced by boundaries of the true path. Output
//     per lane: rec = (start - theta) | letters << 10; per segment the exit
//     (xd = exit - end, < 32); per output block of 256 lanes its letters.
//     Nothing else: no samples, marks or 64-bit records leave the workgroup.
//  F  k_fix_rec: the segments whose start is not their predecessor's exit
//     (every workgroup's first one, the listed ones) walk the new and the old
//     path in step until they meet; records before the meeting point come
//     from the new path, the rest keep their positions with counts shifted.
//     Rounds until no exit changes (decided on the device), then a sweep.
//  scan of the block letters -> each block's first output letter.
//  B  k_split_emit: one workgroup over 256 lanes: their bits staged in LDS, every
//     lane decodes its letters from its settled start (u16 single-symbol
//     table, 64 letters per pass kept in registers by v_perm) into the
//     block's LDS image at its offset, and the image leaves as coalesced
//     16-B stores.
//
// Algorithmic traffic: ceil(B/8) twice (A and B) + n written; the records
// add 4 B per lane (~1/50 of the letters at R = 4, S = 992).
#include <algorithm>

#include "segwalk.hpp"

namespace huff::dev {

namespace {

constexpr uint32_t kT = 256;
constexpr uint32_t kRecD = 10;  // rec: start - theta in bits [0, 10), letters above

// the nominal start of lane q of segment i (clamped to the stream end)
__device__ __forceinline__ uint64_t theta(const SplitArgs& a, uint64_t i, uint32_t q) {
    const uint64_t t = i * a.seg_bits + ((static_cast<uint64_t>(q) * a.seg_bits) >> a.lg_r);
    return t < a.valid_bits ? t : a.valid_bits;
}

// register-array writes at a run-time index (unrolled selects: no scratch)
template <int N>
__device__ __forceinline__ void put_at(uint32_t (&v)[N], uint32_t k, uint32_t x) {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = static_cast<uint32_t>(q) == k ? x : v[q];
}
template <int N>
__device__ __forceinline__ uint32_t get_at(const uint32_t (&v)[N], uint32_t k) {
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < N; ++q) x = static_cast<uint32_t>(q) == k ? v[q] : x;
    return x;
}

// ---- A: speculative walk + in-workgroup fix-up -> lane records -------------

// The checkpoints at the first of a single-code chunk's boundaries po[0, kmax)
// (offsets from the segment start, c0 letters before the chunk) at or past
// each threshold theta(i, nq + 1), ...: exact lane starts, so the lanes'
// letter counts stay close to the host's sizing
__device__ __forceinline__ void mark_ck(uint32_t (&ck)[kSplitRmax - 1], uint32_t& nq, uint64_t& next_th,
                                        const SplitArgs& a, uint64_t i, uint64_t start,
                                        const uint32_t (&po)[kChunkSteps], uint32_t c0, uint32_t kmax) {
    const uint32_t R = 1u << a.lg_r;
    while (nq + 1 < R && kmax && next_th - start <= get_at(po, kmax - 1)) {
        const uint32_t th = static_cast<uint32_t>(next_th - start);
        uint32_t v = 0;
        bool f = false;
#pragma unroll
        for (uint32_t k = 0; k < kChunkSteps; ++k) {
            const bool h = !f && k < kmax && po[k] >= th;
            v = h ? po[k] | ((c0 + k + 1) << 16) : v;
            f = f || h;
        }
        put_at(ck, nq, v);
        ++nq;
        next_th = nq + 1 < R ? theta(a, i, nq + 1) : ~0ull;
    }
}

template <bool SLOW>
__global__ __launch_bounds__(kT) void k_split_sync(SplitArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    __shared__ uint64_t ex_l[kT];
    __shared__ uint32_t bt[kSplitRmax];
    const uint32_t t = threadIdx.x;
    TabLoad tl;
    issue_tables(a, tl);
    const uint32_t tw = (tables_words(a) + 3) & ~3u;
    const Staged st = with_l2(stage_block(a, lds + tw), a, lds);
    const uint16_t* stab = store_tables(a, tl, lds);
    const uint16_t* wtab = a.wtab ? stab : nullptr;  // one table serves single and multi-code steps
    if (t < kSplitRmax) bt[t] = 0;
    __syncthreads();
    const uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * kT + t;
    const bool live = i0 < a.nseg;  // no early return: the fix-up below has barriers
    const uint64_t i = live ? i0 : a.nseg - 1;
    const uint32_t K = a.stab_bits, Kg = a.lut_bits;
    const uint32_t R = 1u << a.lg_r;
    const uint64_t B = a.valid_bits;
    const uint64_t start = i * a.seg_bits;
    const uint64_t end = (i + 1 == a.nseg) ? B : (start + a.seg_bits < B ? start + a.seg_bits : B);
    Cursor c;
    c.init(st, start);
    uint64_t cur = start;
    uint32_t cnt = 0;
    // merge samples: the first step end at or past every kSampBits bits
    uint32_t next_k = 0;
    // the samples (offset from the segment start | spec index << 16; ~0:
    // none) stay in this lane's registers: only its own fix-up reads them
    uint32_t smp[kSampMax];
#pragma unroll
    for (uint32_t q = 0; q < kSampMax; ++q) smp[q] = ~0u;
    uint64_t next_bit = (a.nsamp && live) ? start + kSampBits : ~0ull;
    // checkpoints ck[q - 1] = lane q's start (offset from `start`) | letters before it << 16
    uint32_t ck[kSplitRmax - 1];
#pragma unroll
    for (uint32_t q = 0; q < kSplitRmax - 1; ++q) ck[q] = 0;
    uint32_t nq = 0;
    uint64_t next_th = R > 1 ? theta(a, i, 1) : ~0ull;
    auto note = [&]() {
        if (cur >= next_bit) {
            put_at(smp, next_k, static_cast<uint32_t>(cur - start) | (cnt << 16));
            next_bit = ++next_k < a.nsamp ? next_bit + kSampBits : ~0ull;
        }
    };
    // multi-code chunks while the chunk's last boundary stays below `end` (so
    // no boundary inside one is the exit), a checkpoint at the first window
    // end at or past each threshold (a lane starts within one window's codes
    // of its threshold); single codes to the exit
    if (wtab) {
        const uint64_t span = static_cast<uint64_t>(kChunkSteps) * (a.max_len > K ? a.max_len : K);
        while (cur + span < end) {
            uint32_t U, N, q[kChunkSteps];
            c.multi_chunk<SLOW>(U, N, q, wtab, stab, K, a.lut, Kg);
            while (next_th <= cur + U) {  // (no threshold left: ~0)
                const uint32_t th = static_cast<uint32_t>(next_th - cur);
                uint32_t v = 0;
                bool f = false;
#pragma unroll
                for (uint32_t k = 0; k < kChunkSteps; ++k) {
                    const bool h = !f && (q[k] & 0xFFFFu) >= th;
                    v = h ? q[k] : v;
                    f = f || h;
                }
                put_at(ck, nq, static_cast<uint32_t>(cur - start + (v & 0xFFFFu)) | ((cnt + (v >> 16)) << 16));
                ++nq;
                next_th = nq + 1 < R ? theta(a, i, nq + 1) : ~0ull;
            }
            cur += U;
            cnt += N;
            note();
        }
    }
    for (;;) {
        uint32_t L[kChunkSteps], po[kChunkSteps];
        c.chunk<SLOW>(L, stab, K, a.lut, Kg);
        // the first boundary at or past `end` inside this chunk?
        uint64_t p = cur, ex = ~0ull;
        uint32_t ec = 0;
#pragma unroll
        for (int k = 0; k < kChunkSteps; ++k) {
            p += L[k];
            po[k] = static_cast<uint32_t>(p - start);
            const bool hit = ex == ~0ull && p >= end;
            ex = hit ? p : ex;
            ec = hit ? static_cast<uint32_t>(k + 1) : ec;
        }
        if (ex != ~0ull) {
            mark_ck(ck, nq, next_th, a, i, start, po, cnt, ec - 1);  // thresholds past those boundaries start at the exit
            cnt += ec;
            if (ex > B) {  // an incomplete final code is dropped (comp.rs:493-516)
                ex = B;
                --cnt;
            }
            cur = ex;
            break;
        }
        mark_ck(ck, nq, next_th, a, i, start, po, cnt, kChunkSteps);
        cur = p;
        cnt += kChunkSteps;
        note();
    }
    for (; nq + 1 < R; ++nq) put_at(ck, nq, static_cast<uint32_t>(cur - start) | (cnt << 16));
    const uint32_t s0 = smp[0];  // the first sample

    // fix-up inside the workgroup (the first lane's predecessor is in another
    // workgroup: k_fix_rec)
    ex_l[t] = cur;
    __syncthreads();
    uint64_t s_out = start;
    bool new_exit = false;
    const uint64_t ns = t ? ex_l[t - 1] : start;
    if (ns != start) {
        Cursor w;
        w.init(st, ns);
        uint64_t pa = ns;
        uint32_t na = 0;
        uint64_t pk = s0 == ~0u ? ~0ull : start + (s0 & 0xFFFFu);  // current sample: position, spec index
        uint32_t ik = s0 >> 16, k = 1;
        uint32_t fq = 0;  // checkpoints re-recorded on the true path: ck[0, fq)
        uint64_t fth = R > 1 ? theta(a, i, 1) : ~0ull;
        for (;;) {
            uint32_t L[kChunkSteps], po[kChunkSteps];
            w.chunk<SLOW>(L, stab, K, a.lut, Kg);
            uint64_t p = pa, pex = 0;
            int hit = -1, ex = -1;
#pragma unroll
            for (int j = 0; j < kChunkSteps; ++j) {
                p += L[j];
                po[j] = static_cast<uint32_t>(p - start);
                hit = (hit < 0 && ex < 0 && p == pk) ? j : hit;
                const bool e = ex < 0 && hit < 0 && p >= end;
                ex = e ? j : ex;
                pex = e ? p : pex;
            }
            if (hit >= 0) {  // merged on the sample: true-local index tt
                const uint32_t tt = na + static_cast<uint32_t>(hit) + 1;
                const uint32_t dl = tt - ik;  // (mod 2^32) true-local = spec-local + dl past the merge
                // thresholds up to the merge point: on this chunk; later ones:
                // the speculative checkpoint (on the merged path)
                mark_ck(ck, fq, fth, a, i, start, po, na, static_cast<uint32_t>(hit) + 1);
                for (uint32_t q = fq; q + 1 < R; ++q) put_at(ck, q, get_at(ck, q) + (dl << 16));
                cnt += dl;
                break;
            }
            if (ex >= 0) {  // a new exit
                mark_ck(ck, fq, fth, a, i, start, po, na, static_cast<uint32_t>(ex));
                cnt = na + static_cast<uint32_t>(ex) + 1;
                if (pex > B) {  // an incomplete final code is dropped
                    pex = B;
                    --cnt;
                }
                cur = pex;
                new_exit = true;
                for (uint32_t q = fq; q + 1 < R; ++q) put_at(ck, q, static_cast<uint32_t>(cur - start) | (cnt << 16));
                break;
            }
            mark_ck(ck, fq, fth, a, i, start, po, na, kChunkSteps);
            pa = p;
            na += kChunkSteps;
            while (pa > pk) {  // passed the sample without landing on it: the next one
                const uint32_t sv = k < a.nsamp ? get_at(smp, k) : ~0u;
                ++k;
                pk = sv == ~0u ? ~0ull : start + (sv & 0xFFFFu);
                ik = sv >> 16;
            }
        }
        s_out = ns;
        // a new exit: the successor started from the old one (a workgroup's
        // first segment is checked anyway)
        if (live && new_exit && cur != ex_l[t] && i + 1 < a.nseg && ((i + 1) % kT) != 0 && a.fixlist)
            a.fixlist[atomicAdd(a.flags + kFixRounds, 1u)] = static_cast<uint32_t>(i + 1);
    }
    if (live) {
        atomicAdd(&bt[(t << a.lg_r) >> 8], cnt);
        uint32_t prev = 0;
        for (uint32_t q = 0; q < R; ++q) {
            const uint32_t cq = q ? get_at(ck, q - 1) : 0u;
            const uint64_t pos = q ? start + (cq & 0xFFFFu) : s_out;
            const uint32_t c1 = q + 1 < R ? get_at(ck, q) >> 16 : cnt;
            a.rec[(i << a.lg_r) + q] = static_cast<uint32_t>(pos - theta(a, i, q)) | ((c1 - prev) << kRecD);
            prev = c1;
        }
        a.xd[i] = static_cast<uint8_t>(cur - end);
    }
    __syncthreads();
    const uint64_t ob = static_cast<uint64_t>(blockIdx.x) * R + t;
    if (t < R && ob < split_blocks(a.nseg, a.lg_r)) a.btot[ob] = bt[t];
}

// ---- F: cross-workgroup fix-up of the records --------------------------------

__device__ __forceinline__ bool gstep(BitReader& rd, const BitSrc& src, const Lut& lut, uint64_t B) {
    const uint32_t e = rd.peek(src, lut);
    const uint32_t len = (e >> 8) & 0xFFu;
    if (rd.pos + len > B) {
        rd.pos = B;
        return false;
    }
    rd.advance(src, len);
    return true;
}

// Segment i against its predecessor's exit: nothing when it already starts
// there; else walk the new path (from the exit) and the old one (from the
// recorded start) in step until they meet or the new path leaves the segment.
// r >= 0: the round whose flag a changed exit sets.
__device__ void fix_rec_one(const SplitArgs& a, const BitSrc& src, const Lut& lut, uint64_t i, int r) {
    const uint32_t R = 1u << a.lg_r;
    const uint64_t B = a.valid_bits;
    const uint64_t start = i * a.seg_bits;
    const uint64_t ns = start + a.xd[i - 1];  // segment i-1 ends at `start`
    uint32_t rr[kSplitRmax];
#pragma unroll
    for (uint32_t q = 0; q < kSplitRmax; ++q) rr[q] = q < R ? a.rec[(i << a.lg_r) + q] : 0u;
    const uint64_t old_s = start + (rr[0] & ((1u << kRecD) - 1));
    if (ns == old_s) return;
    const uint64_t end = (i + 1 == a.nseg) ? B : (start + a.seg_bits < B ? start + a.seg_bits : B);
    const uint64_t old_x = end + a.xd[i];
    uint32_t old_total = 0;
#pragma unroll
    for (uint32_t q = 0; q < kSplitRmax; ++q) old_total += rr[q] >> kRecD;
    // new lane starts (offset from `start`) and letters before them, lanes 1..R-1
    uint32_t npos[kSplitRmax], ncum[kSplitRmax];
#pragma unroll
    for (uint32_t q = 0; q < kSplitRmax; ++q) npos[q] = ncum[q] = 0;
    BitReader na, nb;
    na.seek(src, ns);
    nb.seek(src, old_s);
    uint32_t ca = 0, cb = 0;
    bool a_alive = true, b_alive = true;
    uint32_t fq = 1;
    uint64_t fth = R > 1 ? theta(a, i, 1) : ~0ull;
    uint64_t nx;
    uint32_t total;
    for (;;) {
        if (na.pos == nb.pos) {  // merged: later lanes keep their starts, counts shift
            uint32_t cum = 0;
#pragma unroll
            for (uint32_t q = 0; q < kSplitRmax; ++q) {
                if (q >= fq && q < R) {
                    npos[q] = static_cast<uint32_t>(theta(a, i, q) + (rr[q] & ((1u << kRecD) - 1)) - start);
                    ncum[q] = cum - cb + ca;
                }
                cum += rr[q] >> kRecD;
            }
            total = old_total - cb + ca;
            nx = old_x;
            break;
        }
        if (na.pos >= end || !a_alive) {  // a new exit
#pragma unroll
            for (uint32_t q = 0; q < kSplitRmax; ++q)
                if (q >= fq && q < R) {
                    npos[q] = static_cast<uint32_t>(na.pos - start);
                    ncum[q] = ca;
                }
            total = ca;
            nx = na.pos;
            break;
        }
        if (na.pos < nb.pos || !b_alive) {
            a_alive = gstep(na, src, lut, B);
            ca += a_alive ? 1 : 0;
            while (fq < R && na.pos >= fth) {
                put_at(npos, fq, static_cast<uint32_t>(na.pos - start));
                put_at(ncum, fq, ca);
                ++fq;
                fth = fq < R ? theta(a, i, fq) : ~0ull;
            }
        } else {
            b_alive = gstep(nb, src, lut, B);
            cb += b_alive ? 1 : 0;
        }
    }
    npos[0] = static_cast<uint32_t>(ns - start);
    ncum[0] = 0;
#pragma unroll
    for (uint32_t q = 0; q < kSplitRmax; ++q) {
        if (q < R) {
            const uint32_t c1 = q + 1 < R ? ncum[q + 1 < kSplitRmax ? q + 1 : q] : total;
            a.rec[(i << a.lg_r) + q] =
                static_cast<uint32_t>(start + npos[q] - theta(a, i, q)) | ((c1 - ncum[q]) << kRecD);
        }
    }
    if (nx != old_x) {
        a.xd[i] = static_cast<uint8_t>(nx - end);
        if (r >= 0) atomicOr(a.flags + r, 1u);
    }
    if (total != old_total)
        atomicAdd(a.btot + ((i << a.lg_r) >> 8),
                  static_cast<unsigned long long>(static_cast<int64_t>(total) - static_cast<int64_t>(old_total)));
}

__device__ __forceinline__ void load_lut(uint32_t* plut, const SplitArgs& a) {
    for (uint32_t k = threadIdx.x; k < (1u << a.lut_bits); k += blockDim.x) plut[k] = a.lut[k];
    __syncthreads();
}

// round 0: every workgroup's first segment and the listed ones (each index once)
__global__ __launch_bounds__(kT) void k_fix_rec_list(SplitArgs a) {
    extern __shared__ uint32_t plut[];
    load_lut(plut, a);
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    const Lut lut{plut, a.lut, a.lut_bits};
    const uint64_t firsts = (a.nseg - 1) / kT;  // segments 256, 512, ...
    const uint64_t n = firsts + __builtin_nontemporal_load(a.flags + kFixRounds);
    for (uint64_t j = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < n;
         j += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        const uint64_t i = j < firsts ? (j + 1) * kT : a.fixlist[j - firsts];
        fix_rec_one(a, src, lut, i, 0);
    }
}

// round r >= 1 over every segment (a no-op once round r - 1 changed nothing)
__global__ __launch_bounds__(kT) void k_fix_rec(SplitArgs a, int r) {
    if (__builtin_nontemporal_load(a.flags + r - 1) == 0) return;
    extern __shared__ uint32_t plut[];
    load_lut(plut, a);
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    const Lut lut{plut, a.lut, a.lut_bits};
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.nseg;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
        if (i) fix_rec_one(a, src, lut, i, r);
}

// sequential sweep (one lane), only when the last round still changed an exit
__global__ void k_fix_rec_sweep(SplitArgs a) {
    if (__builtin_nontemporal_load(a.flags + kFixRounds - 1) == 0) return;
    extern __shared__ uint32_t plut[];
    load_lut(plut, a);
    if (threadIdx.x != 0) return;
    const BitSrc src{reinterpret_cast<const uint32_t*>(a.comp), a.comp, a.comp_bytes};
    const Lut lut{plut, a.lut, a.lut_bits};
    for (uint64_t i = 1; i < a.nseg; ++i) fix_rec_one(a, src, lut, i, -1);
}

// ---- B: every lane's letters from its settled start --------------------------

// a lane cursor over B's stage (words already in stream order): the fixed
// decoder's window, reads clamped to the stage
struct ECur {
    const uint32_t* w;
    uint32_t last;
    uint64_t buf;
    uint32_t X, rp, nextw;
    __device__ __forceinline__ uint32_t word(uint32_t i) const { return w[i < last ? i : last]; }
    __device__ __forceinline__ void init(const uint32_t* stage, uint32_t stage_last, uint32_t rel) {
        w = stage;
        last = stage_last;
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
};

// letters [0, m) of o (letter j in byte j & 3 of o[j >> 2]) at image bytes
// [F, F + m): whole dwords shifted into place by v_alignbyte, byte stores for
// the partial dwords at both ends (shared with the neighbouring runs)
__device__ __forceinline__ void put_run(uint8_t* img, uint32_t F, const uint32_t (&o)[16], uint32_t m) {
    const uint32_t r = F & 3u;
    const uint32_t m0 = F >> 2;
    const uint32_t il = (m - 1 + r) >> 2;  // the dword holding the last letter (m >= 1)
    uint32_t* img32 = reinterpret_cast<uint32_t*>(img);
    uint32_t vl = 0;
#pragma unroll
    for (int i = 0; i <= 16; ++i) {
        const uint32_t hi = i < 16 ? o[i] : 0u, lo = i > 0 ? o[i - 1] : 0u;
        const uint32_t v = r ? __builtin_amdgcn_alignbyte(hi, lo, 4 - r) : hi;
        const int32_t j0 = 4 * i - static_cast<int32_t>(r);  // the letter in the dword's byte 0
        if (j0 >= 0 && j0 + 4 <= static_cast<int32_t>(m)) img32[m0 + i] = v;
        vl = static_cast<uint32_t>(i) == il ? v : vl;
    }
    // the partial dwords at both ends, shared with the neighbouring runs: byte
    // stores of this run's letters only
    const uint32_t e = (m + r) & 3u;  // letters in the last dword when it is partial
    if (r) {  // the first dword: bytes r .. 3 (letters 0 .. 3 - r, those below m)
        const uint32_t v0 = o[0] << (8 * r);
        const uint32_t hi = il == 0 && e ? e : 4u;
        for (uint32_t s = r; s < hi; ++s) img[4 * m0 + s] = static_cast<uint8_t>(v0 >> (8 * s));
    }
    if (e && (il > 0 || !r))  // the last dword (when not also the first): bytes 0 .. e - 1
        for (uint32_t s = 0; s < e; ++s) img[4 * (m0 + il) + s] = static_cast<uint8_t>(vl >> (8 * s));
}

template <bool SLOW>
__global__ __launch_bounds__(kT) void k_split_emit(SplitArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint32_t wtot[kT / 64];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t K = a.stab_bits;
    const uint32_t tab_words = ((1u << K) + 1) / 2;
    const uint32_t tab_bytes = (tab_words * 4 + 15) & ~15u;
    uint16_t* stab = reinterpret_cast<uint16_t*>(smem);
    uint32_t* stage = reinterpret_cast<uint32_t*>(smem + tab_bytes);
    uint8_t* img = smem + tab_bytes;  // the output image lies over the stage (written after the decode)
    const uint64_t nl = a.nseg << a.lg_r;
    const uint64_t j = static_cast<uint64_t>(blockIdx.x) * kT + t;
    const bool live = j < nl;
    // every global read of the prologue goes out before the first wait: the
    // lane record, the block's output offset (and the total, for the end
    // bit), the table and the stage
    const uint32_t rec = live ? a.rec[j] : 0u;
    const uint64_t O = a.boff[blockIdx.x];
    const uint64_t total = a.end_bit ? a.boff[gridDim.x] : 0;
    const auto rt = buf_rsrc(a.stab, tab_words * 4);
    uint4 tv[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) tv[k] = buf_ld16(rt, (t + kT * k) * 16);
    // the block's bits from its first segment's 16-B granule
    const uint64_t byte_lo = (((static_cast<uint64_t>(blockIdx.x) * kT >> a.lg_r) * a.seg_bits) >> 3) & ~15ull;
    {
        const uint64_t avail = a.comp_bytes > byte_lo ? ((a.comp_bytes + 3) & ~3ull) - byte_lo : 0;
        const uint32_t nb = static_cast<uint32_t>(avail < a.stage_bytes ? avail : a.stage_bytes);
        const auto rs = buf_rsrc(nb ? a.comp + byte_lo : a.comp, nb);
        uint4* w4 = reinterpret_cast<uint4*>(stage);
        const uint32_t np = a.stage_bytes / 16;
        for (uint32_t p0 = t; p0 < np; p0 += 4 * kT) {
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = buf_ld16(rs, (p0 + k * kT) * 16);
            keep_loads(v);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (p0 + k * kT < np)
                    w4[p0 + k * kT] = make_uint4(__builtin_bswap32(v[k].x), __builtin_bswap32(v[k].y),
                                                 __builtin_bswap32(v[k].z), __builtin_bswap32(v[k].w));
        }
        uint4* s4 = reinterpret_cast<uint4*>(stab);  // the table (its loads went out first)
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (t + kT * k < tab_bytes / 16) s4[t + kT * k] = tv[k];
    }
    const uint32_t n = rec >> kRecD;
    const uint64_t start = live ? theta(a, j >> a.lg_r, static_cast<uint32_t>(j & ((1u << a.lg_r) - 1))) +
                                      (rec & ((1u << kRecD) - 1))
                                : 0;
    // the lanes' output offsets in the block
    const uint32_t inc = wave_scan_incl(n);
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    uint32_t before = 0, cb = 0;
#pragma unroll
    for (uint32_t w = 0; w < kT / 64; ++w) {
        before += w < wave ? wtot[w] : 0u;
        cb += wtot[w];
    }
    const uint32_t off_l = before + inc - n;
    // the lane with the stream's last code records the bit after it (the
    // file path's windows continue from there)
    const bool last_code = n && a.end_bit && O + off_l + n == total;
    const uint32_t img0 = static_cast<uint32_t>(O & 15);
    const uint32_t stage_last = a.stage_bytes / 4 - 1;
    const uint32_t rel = static_cast<uint32_t>(start - byte_lo * 8);
    // more letters than the image, or a lane with more than its registers
    // hold: straight to HBM, byte by byte (rare: the host sizes the lanes for
    // ~48 letters)
    if (img0 + cb > a.img_bytes || __syncthreads_or(n > 64)) {
        if (n) {
            ECur c;
            c.init(stage, stage_last, rel);
            uint8_t* dst = a.out + O + off_l;
            for (uint32_t k = 0; k < n; ++k) {
                c.refill();
                dst[k] = static_cast<uint8_t>(c.step<SLOW>(stab, K, a.lut, a.lut_bits) >> 8);
            }
            if (last_code) *a.end_bit = byte_lo * 8 + c.pos();
        }
        return;
    }
    // As k_decode_fixed: no per-lane predicate on the steps. Every lane makes
    // as many lookups as the wave's longest lane (a scalar bound, checked
    // every 4 letters); a shorter lane decodes on into its successor's bits
    // and drops those letters (the stage reads are clamped). The letters wait
    // in registers until every lane has read its bits, then go into the
    // image, which lies over the stage.
    uint32_t o0[16];
    {
        uint32_t wmax = n;
#pragma unroll
        for (int k = 1; k < 64; k <<= 1) {
            const uint32_t y = static_cast<uint32_t>(__shfl_xor(static_cast<int>(wmax), k));
            wmax = y > wmax ? y : wmax;
        }
        const uint32_t steps = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(wmax)));
        ECur c;
        c.init(stage, stage_last, rel);
#pragma unroll
        for (int s = 0; s < 64; ++s) {
            if ((s & 3) == 0 && static_cast<uint32_t>(s) >= steps) break;
            if ((s & 1) == 0) c.refill();
            const uint32_t e = c.step<SLOW>(stab, K, a.lut, a.lut_bits);
            if ((s & 3) == 0) o0[s >> 2] = e >> 8;
            else o0[s >> 2] = __builtin_amdgcn_perm(e, o0[s >> 2], (s & 3) == 1 ? 0x0C0C0500u : (s & 3) == 2 ? 0x0C050100u : 0x05020100u);
        }
    }
    if (last_code) {  // the bit after exactly n codes (one lane of the grid walks them again)
        ECur c;
        c.init(stage, stage_last, rel);
        for (uint32_t k = 0; k < n; ++k) {
            c.refill();
            c.step<SLOW>(stab, K, a.lut, a.lut_bits);
        }
        *a.end_bit = byte_lo * 8 + c.pos();
    }
    __syncthreads();  // every lane has read its bits: the image may overwrite the stage
    if (n) put_run(img, img0 + off_l, o0, n);
    __syncthreads();
    // the image to HBM: 16-B pieces, whole where the block owns all 16 bytes
    const uint64_t gbase = O - img0;
    const uint32_t endb = img0 + cb;
    const uint32_t npieces = (endb + 15) / 16;
    for (uint32_t p = t; p < npieces; p += kT) {
        const uint32_t lo = 16 * p;
        if (lo >= img0 && lo + 16 <= endb) {
            st_nt(reinterpret_cast<uint4*>(a.out + gbase + lo), *reinterpret_cast<const uint4*>(img + lo));
        } else {
            for (uint32_t x = lo; x < lo + 16; ++x)
                if (x >= img0 && x < endb) a.out[gbase + x] = img[x];
        }
    }
}

}  // namespace

size_t split_sync_lds_bytes(const SplitArgs& a) {
    const size_t tw = (((((1u << a.stab_bits) + 1) / 2 + 3) & ~3u) + a.l2_words + 3) & ~size_t(3);
    const size_t stage = ((kT * a.seg_bits + 7) / 8 + 128 + 15) / 16 * 16;
    return tw * 4 + stage;
}

size_t split_emit_lds_bytes(const SplitArgs& a) {
    const size_t tab = ((((1u << a.stab_bits) + 1) / 2) * 4 + 15) & ~size_t(15);
    return tab + std::max<size_t>(a.stage_bytes, a.img_bytes);
}

hipError_t launch_split_sync(const SplitArgs& a, hipStream_t s) {
    if (a.nseg == 0) return hipSuccess;
    if (a.max_len > 32 || a.seg_bits > 2048 || (1u << a.lg_r) > kSplitRmax || a.nsamp > kSampMax || !a.stab)
        return hipErrorInvalidValue;
    const bool slow = a.max_len > a.stab_bits;
    hipLaunchKernelGGL(slow ? k_split_sync<true> : k_split_sync<false>, dim3((a.nseg + kT - 1) / kT), dim3(kT),
                       split_sync_lds_bytes(a), s, a);
    return hipGetLastError();
}

hipError_t launch_split_fix(const SplitArgs& a, hipStream_t s) {
    if (a.nseg == 0) return hipSuccess;
    const size_t lds = (1u << a.lut_bits) * 4;
    const uint32_t lgrid = static_cast<uint32_t>(std::min<uint64_t>(((a.nseg / kT) + kT) / kT, 256));
    hipLaunchKernelGGL(k_fix_rec_list, dim3(std::max<uint32_t>(lgrid, 1)), dim3(kT), lds, s, a);
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((a.nseg + kT - 1) / kT, 2048));
    for (int r = 1; r < kFixRounds; ++r) hipLaunchKernelGGL(k_fix_rec, dim3(grid), dim3(kT), lds, s, a, r);
    hipLaunchKernelGGL(k_fix_rec_sweep, dim3(1), dim3(64), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_split_emit(const SplitArgs& a, hipStream_t s) {
    if (a.nseg == 0) return hipSuccess;
    if ((reinterpret_cast<uintptr_t>(a.out) & 15) || (a.stage_bytes & 15) || (a.img_bytes & 15) ||
        split_emit_lds_bytes(a) > 160 * 1024)
        return hipErrorInvalidValue;
    const bool slow = a.max_len > a.stab_bits;
    hipLaunchKernelGGL(slow ? k_split_emit<true> : k_split_emit<false>, dim3(split_blocks(a.nseg, a.lg_r)), dim3(kT),
                       split_emit_lds_bytes(a), s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
