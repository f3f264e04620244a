// wweights.hip — build_weights_map (weights.rs:82-123) for the wider letters:
// every distinct letter of the input with its count, ascending by letter
// value (one of the orders a Rust HashMap<L, usize> can iterate in; the
// caller builds the tree in it). Hand-written counting, no library sort:
//
//  W = 1, 2   direct bins. Each workgroup counts up to 65,535 letters into an
//             LDS histogram (W = 2: two u16 counters per dword, 128 KiB; a
//             workgroup's letters cannot overflow a u16), then adds its
//             non-zero bins to the global u64 bins; the bins ARE the answer in
//             ascending order.
//  W = 4, 8   an open-addressing table in HBM (2^k slots, linear probing,
//             key claimed by a 64-bit compare-and-swap, counts by 64-bit
//             atomic adds; the host sizes it for a guess of the distinct
//             letters and grows it when the kernel reports it too full: the
//             claims past 3/4 of the slots or a probe run past its limit set
//             the overflow word), fed through a per-workgroup LDS table of
//             2,048 slots that absorbs the repeats of frequent letters (a
//             letter whose LDS probe runs long goes straight to HBM). The
//             all-ones u64 is the empty-slot marker; that letter (W = 8) is
//             counted on the side.
//  W = 16     the same HBM table with a per-slot state word (empty, being
//             written, ready): a lane that finds a slot being written retries
//             in the next round of a wave-wide loop, so no lane waits on
//             another lane of its own wave inside one branch.
//  extract    the used slots are appended to (key, count) arrays; the host
//             sorts them by key (distinct letters only).
#include <algorithm>

#include "kernels.hpp"

namespace huff::dev {

namespace {

constexpr uint32_t kT = 256;
constexpr uint32_t kDirectPerBlock = 65535;  // letters per workgroup of the direct-bin kernels (u16 counters)
constexpr uint32_t kLdsSlots = 2048;         // per-workgroup LDS table (W = 4, 8)
constexpr uint32_t kLdsProbe = 16;           // LDS probes before a letter goes straight to HBM
constexpr uint64_t kEmpty = ~0ull;

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

template <uint32_t W>
__device__ __forceinline__ uint32_t direct_key(const uint8_t* in, uint64_t i) {
    if constexpr (W == 1) return in[i];
    else return static_cast<uint32_t>(in[2 * i]) | (static_cast<uint32_t>(in[2 * i + 1]) << 8);
}

// W = 1 / 2: LDS histogram of one workgroup's letters, then its non-zero bins
template <uint32_t W>
__global__ __launch_bounds__(kT) void k_wcount_direct(const uint8_t* __restrict__ in, uint64_t n,
                                                      unsigned long long* __restrict__ bins) {
    constexpr uint32_t nbins = 1u << (8 * W);
    constexpr uint32_t words = W == 1 ? nbins : nbins / 2;  // W = 2: two u16 counters per dword
    extern __shared__ uint32_t h[];
    for (uint32_t i = threadIdx.x; i < words; i += kT) h[i] = 0;
    __syncthreads();
    const uint64_t lo = static_cast<uint64_t>(blockIdx.x) * kDirectPerBlock;
    const uint64_t hi = lo + kDirectPerBlock < n ? lo + kDirectPerBlock : n;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += kT) {
        const uint32_t k = direct_key<W>(in, i);
        if constexpr (W == 1) atomicAdd(&h[k], 1u);
        else atomicAdd(&h[k >> 1], 1u << (16 * (k & 1)));
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < words; i += kT) {
        const uint32_t v = h[i];
        if (!v) continue;
        if constexpr (W == 1) {
            atomicAdd(&bins[i], static_cast<unsigned long long>(v));
        } else {
            if (v & 0xFFFFu) atomicAdd(&bins[2 * i], static_cast<unsigned long long>(v & 0xFFFFu));
            if (v >> 16) atomicAdd(&bins[2 * i + 1], static_cast<unsigned long long>(v >> 16));
        }
    }
}

template <uint32_t W>
__device__ __forceinline__ uint64_t key64(const uint8_t* in, uint64_t i) {
    if constexpr (W == 4) return *reinterpret_cast<const uint32_t*>(in + 4 * i);
    else return *reinterpret_cast<const uint64_t*>(in + 8 * i);
}

// the table's bookkeeping: claimed slots, overflow flag (the host grows the
// table and counts again), probe limit, the claims allowed
struct HbmTab {
    unsigned long long* used;
    unsigned int* overflow;
    uint64_t mask, max_probe, max_used;
    __device__ __forceinline__ void claimed() const {
        if (atomicAdd(used, 1ull) + 1 > max_used) atomicOr(overflow, 1u);
    }
};

// one letter (count c) into the HBM table (W <= 8)
__device__ __forceinline__ void hbm_add(unsigned long long* keys, unsigned long long* counts, const HbmTab& tab,
                                        unsigned long long* sent, uint64_t key, uint64_t c) {
    if (key == kEmpty) {
        atomicAdd(sent, static_cast<unsigned long long>(c));
        return;
    }
    uint64_t s = mix64(key) & tab.mask;
    for (uint64_t p = 0; p < tab.max_probe; ++p, s = (s + 1) & tab.mask) {
        unsigned long long k = __hip_atomic_load(keys + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == kEmpty) {
            k = atomicCAS(keys + s, kEmpty, static_cast<unsigned long long>(key));
            if (k == kEmpty) tab.claimed();
        }
        if (k == kEmpty || k == key) {
            atomicAdd(counts + s, static_cast<unsigned long long>(c));
            return;
        }
    }
    atomicOr(tab.overflow, 1u);  // a probe run this long: the table is too small
}

// W = 4 / 8: a grid-stride pass through an LDS table per workgroup
template <uint32_t W>
__global__ __launch_bounds__(kT) void k_wcount_hash(const uint8_t* __restrict__ in, uint64_t n,
                                                    unsigned long long* __restrict__ keys,
                                                    unsigned long long* __restrict__ counts, HbmTab tab,
                                                    unsigned long long* __restrict__ sent) {
    __shared__ unsigned long long lk[kLdsSlots];
    __shared__ uint32_t lc[kLdsSlots];
    for (uint32_t i = threadIdx.x; i < kLdsSlots; i += kT) {
        lk[i] = kEmpty;
        lc[i] = 0;
    }
    __syncthreads();
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kT;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kT + threadIdx.x; i < n; i += stride) {
        const uint64_t key = key64<W>(in, i);
        bool done = false;
        if (key != kEmpty) {
            uint32_t s = static_cast<uint32_t>(mix64(key)) & (kLdsSlots - 1);
            for (uint32_t p = 0; p < kLdsProbe; ++p, s = (s + 1) & (kLdsSlots - 1)) {
                unsigned long long k = lk[s];
                if (k == kEmpty) k = atomicCAS(&lk[s], kEmpty, static_cast<unsigned long long>(key));
                if (k == kEmpty || k == key) {
                    atomicAdd(&lc[s], 1u);
                    done = true;
                    break;
                }
            }
        }
        if (!done) hbm_add(keys, counts, tab, sent, key, 1);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kLdsSlots; i += kT)
        if (lc[i]) hbm_add(keys, counts, tab, sent, lk[i], lc[i]);
}

// W = 16: state 0 empty, 1 being written, 2 ready; rounds over the whole wave
__global__ __launch_bounds__(kT) void k_wcount_hash16(const uint8_t* __restrict__ in, uint64_t n,
                                                      unsigned long long* __restrict__ klo,
                                                      unsigned long long* __restrict__ khi,
                                                      unsigned int* __restrict__ state,
                                                      unsigned long long* __restrict__ counts, HbmTab tab) {
    const uint64_t mask = tab.mask;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kT;
    for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * kT; base < n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        bool pending = i < n;
        uint64_t lo = 0, hi = 0, s = 0, probes = 0;
        if (pending) {
            lo = *reinterpret_cast<const uint64_t*>(in + 16 * i);
            hi = *reinterpret_cast<const uint64_t*>(in + 16 * i + 8);
            s = mix64(lo ^ mix64(hi)) & mask;
        }
        while (__any(pending)) {
            if (pending) {
                uint32_t st = __hip_atomic_load(state + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (st == 0 && atomicCAS(state + s, 0u, 1u) == 0u) {
                    tab.claimed();
                    __hip_atomic_store(klo + s, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(khi + s, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(state + s, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    atomicAdd(counts + s, 1ull);
                    pending = false;
                } else if (st == 2) {
                    const uint64_t a = __hip_atomic_load(klo + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t b = __hip_atomic_load(khi + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (a == lo && b == hi) {
                        atomicAdd(counts + s, 1ull);
                        pending = false;
                    } else if (++probes >= tab.max_probe) {  // the table is too small: counted again, larger
                        atomicOr(tab.overflow, 1u);
                        pending = false;
                    } else {
                        s = (s + 1) & mask;
                    }
                }
                // st == 1 (or a lost claim): the same slot again next round
            }
        }
    }
}

// used slots -> (key, count) pairs, appended
__global__ __launch_bounds__(kT) void k_wextract(const unsigned long long* __restrict__ klo,
                                                 const unsigned long long* __restrict__ khi,
                                                 const unsigned long long* __restrict__ counts, uint64_t slots,
                                                 unsigned long long* __restrict__ out_lo,
                                                 unsigned long long* __restrict__ out_hi,
                                                 unsigned long long* __restrict__ out_c,
                                                 unsigned long long* __restrict__ nout, uint64_t cap) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kT;
    for (uint64_t s = static_cast<uint64_t>(blockIdx.x) * kT + threadIdx.x; s < slots; s += stride) {
        const uint64_t c = counts[s];
        if (!c) continue;
        const uint64_t j = atomicAdd(nout, 1ull);
        if (j >= cap) continue;  // counted, not stored: the host reports more used slots than claims
        out_lo[j] = klo[s];
        if (khi) out_hi[j] = khi[s];
        out_c[j] = c;
    }
}

uint32_t grid_for(uint64_t items, uint32_t per_thread, uint32_t cap) {
    const uint64_t g = (items + static_cast<uint64_t>(kT) * per_thread - 1) / (static_cast<uint64_t>(kT) * per_thread);
    return static_cast<uint32_t>(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

uint64_t wcount_slots(uint32_t width, uint64_t distinct) {
    if (width <= 2) return 1ull << (8 * width);
    uint64_t s = 1024;
    while (s < 2 * distinct) s <<= 1;
    return s;
}

hipError_t wcount_launch(const WCountArgs& a, hipStream_t st) {
    if (a.n == 0) return hipSuccess;
    // claims up to 3/4 of the slots; probe runs up to 4,096 slots (the whole
    // table when the host says this is the last size it will try)
    const HbmTab tab{a.used, a.overflow, a.slots - 1, a.unbounded ? a.slots : std::min<uint64_t>(a.slots, 4096),
                     a.unbounded ? a.slots : a.slots / 4 * 3};
    switch (a.width) {
        case 1:
            launch_k(k_wcount_direct<1>, dim3(static_cast<uint32_t>((a.n + kDirectPerBlock - 1) / kDirectPerBlock)),
                               dim3(kT), 256 * 4, st, a.in, a.n, a.counts);
            break;
        case 2: {
            static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(k_wcount_direct<2>),
                                                               hipFuncAttributeMaxDynamicSharedMemorySize, 32768 * 4);
            if (attr != hipSuccess) return attr;
            launch_k(k_wcount_direct<2>, dim3(static_cast<uint32_t>((a.n + kDirectPerBlock - 1) / kDirectPerBlock)),
                               dim3(kT), 32768 * 4, st, a.in, a.n, a.counts);
            break;
        }
        case 4:
            launch_k(k_wcount_hash<4>, dim3(grid_for(a.n, 64, 4096)), dim3(kT), 0, st, a.in, a.n, a.keys_lo,
                               a.counts, tab, a.sent);
            break;
        case 8:
            launch_k(k_wcount_hash<8>, dim3(grid_for(a.n, 64, 4096)), dim3(kT), 0, st, a.in, a.n, a.keys_lo,
                               a.counts, tab, a.sent);
            break;
        case 16:
            launch_k(k_wcount_hash16, dim3(grid_for(a.n, 16, 8192)), dim3(kT), 0, st, a.in, a.n, a.keys_lo,
                               a.keys_hi, a.state, a.counts, tab);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t wextract_launch(const WCountArgs& a, hipStream_t st) {
    if (a.n == 0 || a.width <= 2) return hipSuccess;
    launch_k(k_wextract, dim3(grid_for(a.slots, 16, 8192)), dim3(kT), 0, st, a.keys_lo,
                       a.width == 16 ? a.keys_hi : nullptr, a.counts, a.slots, a.out_lo, a.out_hi, a.out_c, a.nout, a.out_cap);
    return hipGetLastError();
}

}  // namespace huff::dev
