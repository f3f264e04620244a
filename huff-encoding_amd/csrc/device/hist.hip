// hist.hip — hist256: ByteWeights::from_bytes on the GPU
// (huff_coding/src/weights.rs:265-279: one increment per byte).
//
// Roofline: HBM-bound, 1 byte read per input byte. Each workgroup owns whole
// 64 KiB chunks (grid-stride), reads them with 16-B coalesced loads and counts
// into an LDS histogram replicated 32x as [bin][copy]: lane l increments copy
// l % 32, so the ds_add_u32 address of every lane of a 32-lane LDS group sits
// in its own bank whatever the data (no bank conflicts on skewed inputs, the
// two 32-lane halves of a wave are serviced in separate LDS cycles). After a
// chunk the 32 copies are summed (rotated reads, conflict-free) into the
// per-chunk histogram row; the workgroup's totals go to one of 8 XCD-group
// copies of the global weights with one atomic per bin.
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kThreads = 256;
constexpr int kCopies = 32;
// log2 of the one-shot histogram's LDS copies (k_hist1): 32 copies (32 KiB,
// conflict-free on any data, 5 workgroups per CU) by default
#ifndef HUFF_HIST_LOGC
#define HUFF_HIST_LOGC 5
#endif


template <int LOGC = 5>
__device__ __forceinline__ void count_word(uint32_t* h, uint32_t w, uint32_t lane_c) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t b = (w >> (8 * k)) & 0xFFu;
        __hip_atomic_fetch_add(&h[(b << LOGC) | lane_c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

template <int LOGC = 5>
__device__ __forceinline__ void count_masked(uint32_t* h, uint4 v, uint64_t off, uint64_t lo, uint64_t hi,
                                             uint32_t lane_c) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        uint64_t g = off + k;
        if (g >= lo && g < hi) {
            uint32_t b = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
            __hip_atomic_fetch_add(&h[(b << LOGC) | lane_c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// bytes [lo, hi) of `base` (base 16-B aligned); chunk c = base bytes
// [c*kChunk, (c+1)*kChunk).
__global__ __launch_bounds__(kThreads) void k_hist(const uint8_t* __restrict__ base, uint64_t lo, uint64_t hi,
                                                   uint32_t nchunks, uint32_t* __restrict__ chunk_hist,
                                                   unsigned long long* __restrict__ gw) {
    __shared__ __attribute__((aligned(16))) uint32_t h[256 * kCopies];
    const uint32_t t = threadIdx.x;
    const uint32_t lane32 = t & 31;
    for (uint32_t i = t; i < 256 * kCopies; i += kThreads) h[i] = 0;
    uint64_t total = 0;
    __syncthreads();

    for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const uint64_t cbeg = static_cast<uint64_t>(c) * kChunk;
        const bool full = cbeg >= lo && cbeg + kChunk <= hi;
        if (full) {
            const uint4* p = reinterpret_cast<const uint4*>(base + cbeg) + t;
            // 16 rounds of 4 KiB; 4 loads in flight per lane
#pragma unroll 1
            for (int r = 0; r < 16; r += 4) {
                uint4 v0 = ld_nt(p + (r + 0) * kThreads);
                uint4 v1 = ld_nt(p + (r + 1) * kThreads);
                uint4 v2 = ld_nt(p + (r + 2) * kThreads);
                uint4 v3 = ld_nt(p + (r + 3) * kThreads);
                count_word(h, v0.x, lane32); count_word(h, v0.y, lane32);
                count_word(h, v0.z, lane32); count_word(h, v0.w, lane32);
                count_word(h, v1.x, lane32); count_word(h, v1.y, lane32);
                count_word(h, v1.z, lane32); count_word(h, v1.w, lane32);
                count_word(h, v2.x, lane32); count_word(h, v2.y, lane32);
                count_word(h, v2.z, lane32); count_word(h, v2.w, lane32);
                count_word(h, v3.x, lane32); count_word(h, v3.y, lane32);
                count_word(h, v3.z, lane32); count_word(h, v3.w, lane32);
            }
        } else {
            for (int r = 0; r < 16; ++r) {
                const uint64_t off = cbeg + static_cast<uint64_t>(r) * kRound + t * 16;
                if (off + 16 <= lo || off >= hi) continue;
                uint4 v;
                if (off + 16 <= hi) {
                    v = *reinterpret_cast<const uint4*>(base + off);
                } else {  // never read past hi
                    uint32_t w[4] = {0, 0, 0, 0};
                    for (int k = 0; off + k < hi; ++k) w[k >> 2] |= static_cast<uint32_t>(base[off + k]) << (8 * (k & 3));
                    v = make_uint4(w[0], w[1], w[2], w[3]);
                }
                count_masked(h, v, off, lo, hi, lane32);
            }
        }
        __syncthreads();
        // thread t owns bin t: sum its 32 copies (rotated: conflict-free) and clear
        uint32_t s = 0;
#pragma unroll 8
        for (int j = 0; j < kCopies; ++j) {
            uint32_t k = (j + t) & 31;
            s += h[(t << 5) | k];
            h[(t << 5) | k] = 0;
        }
        if (chunk_hist) chunk_hist[static_cast<uint64_t>(c) * 256 + t] = s;
        total += s;
        __syncthreads();
    }
    if (total) atomicAdd(&gw[(blockIdx.x % kHistCopies) * 256 + t], static_cast<unsigned long long>(total));
}

// One chunk per workgroup (one-shot grid: the streaming-read shape that
// measured fastest on this chip, tools/calib.hip): all 16 loads of a lane are
// issued before the first count, the chunk's row is written, and the global
// weights are summed from the rows afterwards (k_rows_sum) instead of with
// per-workgroup atomics.
// HUFF_HIST_THREADS: the workgroup's threads (256: 16 loads of 16 B per
// lane; 512: 8 per lane with twice the waves sharing one LDS histogram)
#ifndef HUFF_HIST_THREADS
#define HUFF_HIST_THREADS 256
#endif
template <int LOGC, int T = HUFF_HIST_THREADS>
__global__ __launch_bounds__(T) void k_hist1(const uint8_t* __restrict__ base, uint64_t lo, uint64_t hi,
                                             uint32_t* __restrict__ chunk_hist,
                                             unsigned long long* __restrict__ gw) {
    constexpr uint32_t C = 1u << LOGC;  // LDS copies of the histogram
    constexpr int NL = kChunk / 16 / T;  // 16-B loads per lane
    if (blockIdx.x == 0)  // k_rows_sum / k_rows_publish (next on the stream) accumulate into gw
        for (uint32_t i = threadIdx.x; i < kHistCopies * 256 + 1; i += T) gw[i] = 0;
    __shared__ __attribute__((aligned(16))) uint32_t h[256 * C];
    const uint32_t t = threadIdx.x;
    const uint32_t lane_c = t & (C - 1);
    const uint32_t c = blockIdx.x;
    const uint64_t cbeg = static_cast<uint64_t>(c) * kChunk;
    const bool full = cbeg >= lo && cbeg + kChunk <= hi;
    uint4 v[NL];
    if (full) {
        const uint4* p = reinterpret_cast<const uint4*>(base + cbeg) + t;
#pragma unroll
        for (int r = 0; r < NL; ++r) v[r] = ld_nt(p + r * T);
    }
    __builtin_amdgcn_sched_barrier(0);  // loads first, no use of v[] hoisted above them
    uint4* h4 = reinterpret_cast<uint4*>(h);
#pragma unroll
    for (uint32_t i = 0; i < 256 * C / 4 / T; ++i) h4[t + i * T] = make_uint4(0, 0, 0, 0);
    // a bare barrier (no fence): the LDS zeroing is complete, the loads stay in flight
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0), vmcnt/expcnt untouched
    __builtin_amdgcn_s_barrier();
    if (full) {
#pragma unroll
        for (int r = 0; r < NL; ++r) {
            count_word<LOGC>(h, v[r].x, lane_c);
            count_word<LOGC>(h, v[r].y, lane_c);
            count_word<LOGC>(h, v[r].z, lane_c);
            count_word<LOGC>(h, v[r].w, lane_c);
        }
    } else {
        for (int r = 0; r < NL; ++r) {
            const uint64_t off = cbeg + static_cast<uint64_t>(r) * (16 * T) + t * 16;
            if (off + 16 <= lo || off >= hi) continue;
            uint4 x;
            if (off + 16 <= hi) {
                x = *reinterpret_cast<const uint4*>(base + off);
            } else {  // never read past hi
                uint32_t w[4] = {0, 0, 0, 0};
                for (int k = 0; off + k < hi; ++k) w[k >> 2] |= static_cast<uint32_t>(base[off + k]) << (8 * (k & 3));
                x = make_uint4(w[0], w[1], w[2], w[3]);
            }
            count_masked<LOGC>(h, x, off, lo, hi, lane_c);
        }
    }
    __syncthreads();
    if (t < 256) {
        uint32_t s = 0;
#pragma unroll 8
        for (uint32_t j = 0; j < C; ++j) s += h[(t << LOGC) | ((j + t) & (C - 1))];
        chunk_hist[static_cast<uint64_t>(c) * 256 + t] = s;
    }
}

// Two chunks per 512-thread workgroup sharing ONE 32-copy LDS image: the
// first chunk's threads add 1, the second's 1 << 16 (a copy counts at most
// 8 threads x 256 bytes = 2,048 of a chunk, so neither half overflows), the
// halves are split when the copies are summed. Twice the input in flight
// per byte of LDS (the one-shot grid was LDS-bound at 5 workgroups per CU,
// 320 KiB in flight against ~450 KiB for the calibration read): same-box
// pass 1 uniform 0.215 -> 0.210 ms, Zipf 0.198 -> 0.193 (profiles/r05/hist_x2/).
// The default; k_hist1 stays for HUFF_HIST_X2=0.
template <int LOGC>
__global__ __launch_bounds__(512) void k_hist1x2(const uint8_t* __restrict__ base, uint64_t lo, uint64_t hi,
                                                 uint32_t nchunks, uint32_t* __restrict__ chunk_hist,
                                                 unsigned long long* __restrict__ gw) {
    constexpr uint32_t C = 1u << LOGC;
    constexpr int T = 256;               // threads per chunk
    // the zeroing loop below clears 256 C / 4 words in strides of 2 T, and a
    // copy's 16-bit half counts up to kChunk / C bytes: both need C >= 8
    // (HUFF_HIST_LOGC is a build knob; smaller values would miscount silently)
    static_assert(LOGC >= 3 && LOGC <= 6, "k_hist1x2 needs 8..64 LDS copies (64 KiB of static LDS at most)");
    static_assert(kChunk / C < 65536, "a copy's 16-bit half counter must not overflow");
    constexpr int NL = kChunk / 16 / T;  // 16-B loads per lane
    if (blockIdx.x == 0)  // the weights and k_rows_publish's ticket (gw[kHistCopies * 256])
        for (uint32_t i = threadIdx.x; i < kHistCopies * 256 + 1; i += 2 * T) gw[i] = 0;
    __shared__ __attribute__((aligned(16))) uint32_t h[256 * C];
    const uint32_t t = threadIdx.x, tl = t & (T - 1), half = t / T;
    const uint32_t lane_c = t & (C - 1);
    const uint32_t inc = half ? 0x10000u : 1u;
    const uint32_t c = 2 * blockIdx.x + half;
    const uint64_t cbeg = static_cast<uint64_t>(c) * kChunk;
    const bool live = c < nchunks;
    const bool full = live && cbeg >= lo && cbeg + kChunk <= hi;
    uint4 v[NL];
    if (full) {
        const uint4* p = reinterpret_cast<const uint4*>(base + cbeg) + tl;
#pragma unroll
        for (int r = 0; r < NL; ++r) v[r] = ld_nt(p + r * T);
    }
    __builtin_amdgcn_sched_barrier(0);
    uint4* h4 = reinterpret_cast<uint4*>(h);
#pragma unroll
    for (uint32_t i = 0; i < 256 * C / 4 / (2 * T); ++i) h4[t + i * 2 * T] = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
    auto add = [&](uint32_t w) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __hip_atomic_fetch_add(&h[(((w >> (8 * k)) & 0xFFu) << LOGC) | lane_c], inc, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    if (full) {
#pragma unroll
        for (int r = 0; r < NL; ++r) {
            add(v[r].x);
            add(v[r].y);
            add(v[r].z);
            add(v[r].w);
        }
    } else if (live) {
        for (int r = 0; r < NL; ++r) {
            const uint64_t off = cbeg + static_cast<uint64_t>(r) * (16 * T) + tl * 16;
            if (off + 16 <= lo || off >= hi) continue;
            for (int k = 0; k < 16; ++k)
                if (off + k >= lo && off + k < hi)
                    __hip_atomic_fetch_add(&h[(static_cast<uint32_t>(base[off + k]) << LOGC) | lane_c], inc,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    if (t < 256) {
        uint32_t s0 = 0, s1 = 0;
#pragma unroll 8
        for (uint32_t j = 0; j < C; ++j) {
            const uint32_t x = h[(t << LOGC) | ((j + t) & (C - 1))];
            s0 += x & 0xFFFFu;
            s1 += x >> 16;
        }
        chunk_hist[static_cast<uint64_t>(2 * blockIdx.x) * 256 + t] = s0;
        if (2 * blockIdx.x + 1 < nchunks) chunk_hist[static_cast<uint64_t>(2 * blockIdx.x + 1) * 256 + t] = s1;
    }
}

// gw[copy][b] += sum over a stripe of chunks of chunk_hist[c][b]
__global__ __launch_bounds__(256) void k_rows_sum(const uint32_t* __restrict__ chunk_hist, uint32_t nchunks,
                                                  unsigned long long* __restrict__ gw) {
    const uint32_t t = threadIdx.x;
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    uint32_t c = blockIdx.x;
    const uint32_t g = gridDim.x;
    for (; c + 3 * g < nchunks; c += 4 * g) {
        s0 += chunk_hist[static_cast<uint64_t>(c) * 256 + t];
        s1 += chunk_hist[static_cast<uint64_t>(c + g) * 256 + t];
        s2 += chunk_hist[static_cast<uint64_t>(c + 2 * g) * 256 + t];
        s3 += chunk_hist[static_cast<uint64_t>(c + 3 * g) * 256 + t];
    }
    for (; c < nchunks; c += g) s0 += chunk_hist[static_cast<uint64_t>(c) * 256 + t];
    const uint64_t s = s0 + s1 + s2 + s3;
    if (s) atomicAdd(&gw[(blockIdx.x % kHistCopies) * 256 + t], static_cast<unsigned long long>(s));
}

// k_rows_sum and k_hist_publish in one launch (pass 1 with a host reader):
// 16 waves per workgroup, a wave per chunk row at a time (16 B per lane,
// bins 4l..4l+3) with four rows in flight, the waves summed in LDS and added
// into gw's XCD copy, then the last workgroup to take a ticket
// (gw[kHistCopies * 256], zeroed by pass 1's first workgroup) publishes the
// totals as k_hist_publish does. Few workgroups (<= 128): each pays one
// agent-scope release (an L2 write-back) before its ticket, and a 1,024-group
// version spent 26 us there (profiles/r06/pipeline).
#ifndef HUFF_ROWS_PUBLISH
#define HUFF_ROWS_PUBLISH 1
#endif
#ifndef HUFF_RP_GROUPS
#define HUFF_RP_GROUPS 128
#endif
constexpr uint32_t kRpWaves = 16;
__global__ __launch_bounds__(kRpWaves * 64) void k_rows_publish(const uint32_t* __restrict__ chunk_hist,
                                                                uint32_t nchunks, unsigned long long* gw,
                                                                unsigned long long* host, uint64_t tag) {
    __shared__ uint64_t part[kRpWaves][256];
    __shared__ uint32_t last;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t stride = gridDim.x * kRpWaves;
    const uint4* rows = reinterpret_cast<const uint4*>(chunk_hist) + lane;  // 64 uint4 per row
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    uint32_t c = blockIdx.x * kRpWaves + wave;
    for (; c + 3 * stride < nchunks; c += 4 * stride) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = rows[static_cast<uint64_t>(c + k * stride) * 64];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            a0 += v[k].x;
            a1 += v[k].y;
            a2 += v[k].z;
            a3 += v[k].w;
        }
    }
    for (; c < nchunks; c += stride) {
        const uint4 v = rows[static_cast<uint64_t>(c) * 64];
        a0 += v.x;
        a1 += v.y;
        a2 += v.z;
        a3 += v.w;
    }
    part[wave][4 * lane] = a0;
    part[wave][4 * lane + 1] = a1;
    part[wave][4 * lane + 2] = a2;
    part[wave][4 * lane + 3] = a3;
    __syncthreads();
    if (t < 256) {
        uint64_t s = 0;
#pragma unroll
        for (uint32_t w = 0; w < kRpWaves; ++w) s += part[w][t];
        if (s)
            __hip_atomic_fetch_add(&gw[(blockIdx.x % kHistCopies) * 256 + t], static_cast<unsigned long long>(s),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();  // every add of this workgroup issued before its ticket
    if (t == 0) {
        const unsigned long long k = __hip_atomic_fetch_add(&gw[kHistCopies * 256], 1ull, __ATOMIC_ACQ_REL,
                                                            __HIP_MEMORY_SCOPE_AGENT);
        last = k == gridDim.x - 1u;
    }
    __syncthreads();
    if (!last || t >= 256) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    uint64_t tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < kHistCopies; ++k)
        tot += __hip_atomic_load(&gw[k * 256 + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&host[t], (tag << 48) | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Pass 1's result straight to pinned host memory: word b = total of bin b
// with the launch's 16-bit sequence tag in bits 48..63 (totals < 2^48). Each
// word is one 8-byte store, so the host, polling until all 256 tags match,
// needs no fence, no flag and no device-to-host copy.
__global__ __launch_bounds__(256) void k_hist_publish(const unsigned long long* __restrict__ gw,
                                                      unsigned long long* host, uint64_t tag) {
    const uint32_t t = threadIdx.x;
    uint64_t tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < kHistCopies; ++k) tot += gw[k * 256 + t];
    __hip_atomic_store(&host[t], (tag << 48) | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Pass 1's result as one device row for a collective (multi-GPU, SURVEY
// §8e): row[b] = total of bin b (b < 256), row[256] = the job's last
// min(8, n) input bytes packed little-endian, row[257] = their count. The
// all-gather of these rows (RCCL, stream-ordered after this kernel) is the
// only exchange of the sharded path; no host round trip precedes it.
__global__ __launch_bounds__(256) void k_hist_row(const unsigned long long* __restrict__ gw,
                                                  const uint8_t* __restrict__ in, uint64_t n,
                                                  long long* __restrict__ row) {
    const uint32_t t = threadIdx.x;
    uint64_t tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < kHistCopies; ++k) tot += gw[k * 256 + t];
    row[t] = static_cast<long long>(tot);
    if (t == 0) {
        const uint32_t m = n < 8 ? static_cast<uint32_t>(n) : 8u;
        uint64_t packed = 0;
        for (uint32_t i = 0; i < m; ++i) packed |= static_cast<uint64_t>(in[n - m + i]) << (8 * i);
        row[256] = static_cast<long long>(packed);
        row[257] = m;
    }
}

// bits[c] = sum_b chunk_hist[c][b] * len[b]; one wave per chunk.
__global__ __launch_bounds__(256) void k_chunk_bits(const uint32_t* __restrict__ chunk_hist, uint32_t nchunks,
                                                    CodeLens lens, uint64_t* __restrict__ bits) {
    const uint8_t* len = lens.len;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t c = blockIdx.x * 4 + wave;
    if (c >= nchunks) return;
    uint4 hv = reinterpret_cast<const uint4*>(chunk_hist + static_cast<uint64_t>(c) * 256)[lane];
    uint32_t lv = reinterpret_cast<const uint32_t*>(len)[lane];
    uint64_t s = static_cast<uint64_t>(hv.x) * (lv & 0xFF) + static_cast<uint64_t>(hv.y) * ((lv >> 8) & 0xFF) +
                 static_cast<uint64_t>(hv.z) * ((lv >> 16) & 0xFF) + static_cast<uint64_t>(hv.w) * (lv >> 24);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_down(s, d, 64);
    if (lane == 0) bits[c] = s;
}

// start[c] = base + sum_{c' < c} bits[c'], start[nchunks] = total end, in two
// launches over tiles of 1024 chunks. A chunk has at most 65536 * 57 bits <
// 2^22, so a tile's local prefix sums fit 32 bits and scan with DPP.
// k_scan_tiles: tile-local exclusive prefix -> start[], tile total -> tsum[].
__global__ __launch_bounds__(1024) void k_scan_tiles(const uint64_t* __restrict__ bits, uint32_t nchunks,
                                                     uint64_t* __restrict__ start, uint64_t* __restrict__ tsum) {
    __shared__ uint32_t wsum[16];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t i = blockIdx.x * 1024 + t;
    const uint32_t v = i < nchunks ? static_cast<uint32_t>(bits[i]) : 0u;
    const uint32_t incl = wave_scan_incl(v);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < 16; ++w) {
        pre += (w < wave) ? wsum[w] : 0u;
        tot += wsum[w];
    }
    if (i < nchunks) start[i] = pre + incl - v;
    if (t == 0) tsum[blockIdx.x] = tot;
}

// k_scan_tsum: one workgroup turns the tile totals into exclusive prefixes in
// place (tsum[tiles] = the grand total): each thread scans a run of tiles
// (the index-free decode has ~5,400 tiles per GiB: the per-tile sum over all
// earlier tiles this replaces read 15 M words)
__global__ __launch_bounds__(1024) void k_scan_tsum(uint32_t tiles, uint64_t* __restrict__ tsum) {
    __shared__ uint64_t wsum[16];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t per = (tiles + 1023) / 1024;
    const uint32_t lo = t * per < tiles ? t * per : tiles, hi = lo + per < tiles ? lo + per : tiles;
    uint64_t mine = 0;
    for (uint32_t q = lo; q < hi; ++q) mine += tsum[q];
    uint64_t incl = mine;  // wave inclusive scan (64-bit shuffles)
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t v = __shfl_up(incl, d, 64);
        if (lane >= static_cast<uint32_t>(d)) incl += v;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < 16; ++w) {
        pre += (w < wave) ? wsum[w] : 0u;
        tot += wsum[w];
    }
    uint64_t run = pre + incl - mine;
    for (uint32_t q = lo; q < hi; ++q) {
        const uint64_t v = tsum[q];
        tsum[q] = run;
        run += v;
    }
    if (t == 0) tsum[tiles] = tot;
}

// k_scan_fix_small (<= 64 tiles, the encoder's case: one launch less): add
// base + the totals of the tiles before, summed by one wave per tile; the
// last tile also writes start[nchunks]
// host: when non-null, the grand total also goes to pinned host memory as
// (tag << 48) | total (one 8-byte store), so the host polls for it instead of
// a device-to-host copy and a stream synchronisation
__device__ __forceinline__ void publish_total(unsigned long long* host, uint64_t tag, uint64_t total) {
    if (host) __hip_atomic_store(host, (tag << 48) | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(1024) void k_scan_fix_small(uint32_t nchunks, uint64_t base,
                                                         const uint64_t* __restrict__ tsum,
                                                         uint64_t* __restrict__ start,
                                                         unsigned long long* host, uint64_t tag) {
    __shared__ uint64_t off;
    const uint32_t t = threadIdx.x;
    if (t < 64) {
        uint64_t sum = t < blockIdx.x ? tsum[t] : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) sum += __shfl_down(sum, d, 64);
        if (t == 0) off = base + sum;
    }
    __syncthreads();
    const uint32_t i = blockIdx.x * 1024 + t;
    if (i < nchunks) start[i] += off;
    if (blockIdx.x == gridDim.x - 1 && t == 0) {
        const uint64_t end = off + tsum[blockIdx.x];
        start[nchunks] = end;
        publish_total(host, tag, end - base);
    }
}

// k_scan_fix: add base + the exclusive prefix of the tile totals; the last
// tile also writes start[nchunks]
__global__ __launch_bounds__(1024) void k_scan_fix(uint32_t nchunks, uint64_t base, const uint64_t* __restrict__ tsum,
                                                   uint64_t* __restrict__ start, unsigned long long* host,
                                                   uint64_t tag) {
    const uint32_t t = threadIdx.x;
    const uint64_t off = base + tsum[blockIdx.x];
    const uint32_t i = blockIdx.x * 1024 + t;
    if (i < nchunks) start[i] += off;
    if (blockIdx.x == gridDim.x - 1 && t == 0) {
        start[nchunks] = base + tsum[gridDim.x];
        publish_total(host, tag, tsum[gridDim.x]);
    }
}

// lowest index i with missing_mask[in[i]] != 0 (error path of compress_with_tree)
__global__ __launch_bounds__(256) void k_find_first(const uint8_t* __restrict__ in, uint64_t n,
                                                    const uint8_t* __restrict__ mask,
                                                    unsigned long long* __restrict__ pos) {
    __shared__ uint8_t m[256];
    m[threadIdx.x] = mask[threadIdx.x];
    __syncthreads();
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        if (m[in[i]]) {
            atomicMin(pos, static_cast<unsigned long long>(i));
            return;
        }
    }
}

}  // namespace

hipError_t launch_hist(const uint8_t* base, uint64_t lo, uint64_t hi, uint32_t nchunks, uint32_t* chunk_hist,
                       unsigned long long* gw, hipStream_t s, HistDone done) {
    if (nchunks == 0) return hipSuccess;
    if (chunk_hist) {  // per-chunk rows wanted: one-shot grid, then the row sum
        // 32 copies: 16 measured equal on uniform bytes and 20 % slower on
        // Zipf (same-address conflicts between lanes l and l + 16)
// HUFF_HIST_X2=0: k_hist1, one chunk per workgroup (A/B builds)
#ifndef HUFF_HIST_X2
#define HUFF_HIST_X2 1
#endif
        if (HUFF_HIST_X2)
            launch_k(k_hist1x2<HUFF_HIST_LOGC>, dim3((nchunks + 1) / 2), dim3(512), 0, s, base, lo, hi, nchunks,
                               chunk_hist, gw);
        else
            launch_k(k_hist1<HUFF_HIST_LOGC>, dim3(nchunks), dim3(HUFF_HIST_THREADS), 0, s, base, lo, hi,
                               chunk_hist, gw);
        if (done.host && HUFF_ROWS_PUBLISH) {
            // >= 4 rows per wave where the job has them, 128 workgroups at most
            const uint32_t want = (nchunks + 4 * kRpWaves - 1) / (4 * kRpWaves);
            const uint32_t g = want < HUFF_RP_GROUPS ? want : HUFF_RP_GROUPS;
            launch_k(k_rows_publish, dim3(g), dim3(kRpWaves * 64), 0, s, chunk_hist, nchunks, gw, done.host,
                     done.tag);
            return hipGetLastError();
        }
        const uint32_t g = nchunks < 512 ? nchunks : 512;
        launch_k(k_rows_sum, dim3(g), dim3(256), 0, s, chunk_hist, nchunks, gw);
        if (done.host) launch_k(k_hist_publish, dim3(1), dim3(256), 0, s, gw, done.host, done.tag);
        return hipGetLastError();
    }
    uint32_t grid = nchunks < 1024 ? nchunks : 1024;
    const hipError_t e = hipMemsetAsync(gw, 0, kHistCopies * 256 * 8, s);
    if (e != hipSuccess) return e;
    launch_k(k_hist, dim3(grid), dim3(kThreads), 0, s, base, lo, hi, nchunks, chunk_hist, gw);
    return hipGetLastError();
}

hipError_t launch_hist_row(const unsigned long long* gw, const uint8_t* in, uint64_t n, long long* row,
                           hipStream_t s) {
    launch_k(k_hist_row, dim3(1), dim3(256), 0, s, gw, in, n, row);
    return hipGetLastError();
}

hipError_t launch_chunk_bits(const uint32_t* chunk_hist, uint32_t nchunks, const CodeLens& len, uint64_t* bits,
                             hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    launch_k(k_chunk_bits, dim3((nchunks + 3) / 4), dim3(256), 0, s, chunk_hist, nchunks, len, bits);
    return hipGetLastError();
}

hipError_t launch_scan(const uint64_t* bits, uint32_t nchunks, uint64_t base, uint64_t* start, uint64_t* tsum,
                       hipStream_t s, HistDone done) {
    const uint32_t tiles = nchunks ? (nchunks + 1023) / 1024 : 1;
    launch_k(k_scan_tiles, dim3(tiles), dim3(1024), 0, s, bits, nchunks, start, tsum);
    if (tiles <= 64) {
        launch_k(k_scan_fix_small, dim3(tiles), dim3(1024), 0, s, nchunks, base, tsum, start, done.host,
                           done.tag);
    } else {
        launch_k(k_scan_tsum, dim3(1), dim3(1024), 0, s, tiles, tsum);
        launch_k(k_scan_fix, dim3(tiles), dim3(1024), 0, s, nchunks, base, tsum, start, done.host,
                           done.tag);
    }
    return hipGetLastError();
}

hipError_t launch_find_first(const uint8_t* in, uint64_t n, const uint8_t* missing_mask, unsigned long long* pos,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    uint32_t grid = blocks < 4096 ? static_cast<uint32_t>(blocks) : 4096;
    launch_k(k_find_first, dim3(grid), dim3(256), 0, s, in, n, missing_mask, pos);
    return hipGetLastError();
}

}  // namespace huff::dev
