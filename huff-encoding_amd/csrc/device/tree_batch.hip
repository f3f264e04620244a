// tree_batch.hip — HuffTree of many small byte streams on the device in one
// launch (the case where building the tree on the host
// would dominate). Bit-exact with the host build (host/tree.cpp) and so with
// the reference: leaves in ByteWeights' iteration order (weights.rs:423-441,
// the byte-0 re-yield included), Rust std BinaryHeap with the reversed
// weight order (branch_heap.rs:18-83 over std's sift_up /
// sift_down_to_bottom; host/rust_heap.hpp), two minima popped per merge
// (tree_inner.rs:289-306), codes and as_bin in preorder (tree_inner.rs:313-
// 320, 632-663).
//
// The heap is inherently serial, so the parallelism is across streams: one
// lane per stream, kTreeLanes streams per workgroup, each stream's heap,
// joint nodes and leaf letters in LDS, interleaved by lane ([i][lane]:
// lanes at the same heap index hit distinct banks). A merge costs about two
// sift_down_to_bottom walks of LDS round trips; every stream of the batch
// runs at once (up to 256 CUs x one 32-stream workgroup).
//
//  k_hist_batch  one workgroup per stream: LDS byte histogram of the
//                stream's bytes [off[s], off[s+1]) -> hist[s][256] (u64).
//  k_tree_batch  lane = stream: heap build, merges, then one preorder walk
//                writing the as_bin bits (MSB first) and the code table.
#include "bitreader.hpp"

namespace huff::dev {

namespace {

constexpr int kTreeLanes = 16;      // streams per workgroup (one lane each): 53 KB of LDS, 3 workgroups per CU
constexpr int kHeapCap = 257;       // 256 letters + the byte-0 re-yield
constexpr uint32_t kNodeBits = 10;  // heap key = weight << 10 | node (node < 2 * 257)

// ---------------------------------------------------------------------------
// A stream longer than 2^31 bytes is counted in pieces (a u32 LDS bin could
// wrap within 2^32 bytes); each bin's piece counts add up in its thread's u64.
// A stream with d_offsets[s + 1] < d_offsets[s] counts as empty.
constexpr uint64_t kHistPiece = 1ull << 31;
__global__ __launch_bounds__(256) void k_hist_batch(const uint8_t* __restrict__ in,
                                                    const uint64_t* __restrict__ off, uint64_t* __restrict__ hist) {
    __shared__ uint32_t bins[256];
    const uint32_t s = blockIdx.x, t = threadIdx.x;
    const uint64_t lo0 = off[s], hi0 = off[s + 1] > lo0 ? off[s + 1] : lo0;
    uint64_t acc = 0;
    for (uint64_t lo = lo0; lo < hi0 || lo == lo0; lo += kHistPiece) {
        const uint64_t hi = hi0 - lo > kHistPiece ? lo + kHistPiece : hi0;
        bins[t] = 0;
        __syncthreads();
        // head bytes up to 4-B alignment, then dwords, then the tail
        const uint64_t a0 = (lo + 3) & ~3ull;
        const uint64_t mid_lo = a0 < hi ? a0 : hi;
        const uint64_t mid_hi = mid_lo + ((hi - mid_lo) & ~3ull);
        if (t < mid_lo - lo) atomicAdd(&bins[in[lo + t]], 1u);
        const uint32_t* w = reinterpret_cast<const uint32_t*>(in + mid_lo);
        const uint64_t nw = (mid_hi - mid_lo) / 4;
        for (uint64_t i = t; i < nw; i += 256) {
            const uint32_t v = w[i];
            atomicAdd(&bins[v & 0xFF], 1u);
            atomicAdd(&bins[(v >> 8) & 0xFF], 1u);
            atomicAdd(&bins[(v >> 16) & 0xFF], 1u);
            atomicAdd(&bins[v >> 24], 1u);
        }
        if (t < hi - mid_hi) atomicAdd(&bins[in[mid_hi + t]], 1u);
        __syncthreads();
        acc += bins[t];
        __syncthreads();
        if (hi >= hi0) break;
    }
    hist[static_cast<uint64_t>(s) * 256 + t] = acc;
}

// ---------------------------------------------------------------------------
// std BinaryHeap<HuffBranchHeapItem> of one lane's stream. "a <= b" under the
// reversed Ord is a.weight >= b.weight (rust_heap.hpp le); ties keep heap
// positions exactly as std does.
struct LaneHeap {
    uint64_t (*v)[kTreeLanes];
    uint32_t lane;
    uint32_t n = 0;
    __device__ static bool le(uint64_t a, uint64_t b) { return (a >> kNodeBits) >= (b >> kNodeBits); }
    __device__ uint64_t& at(uint32_t i) { return v[i][lane]; }
    __device__ void sift_up(uint32_t start, uint32_t pos) {
        const uint64_t hole = at(pos);
        while (pos > start) {
            const uint32_t parent = (pos - 1) >> 1;
            const uint64_t p = at(parent);
            if (le(hole, p)) break;
            at(pos) = p;
            pos = parent;
        }
        at(pos) = hole;
    }
    __device__ void push(uint64_t e) {
        at(n) = e;
        ++n;
        sift_up(0, n - 1);
    }
    __device__ uint64_t pop() {
        uint64_t top = at(--n);
        if (n) {
            const uint64_t root = at(0);
            at(0) = top;
            top = root;
            // sift_down_to_bottom(0), then sift_up
            const uint32_t end = n;
            uint32_t pos = 0, child = 1;
            const uint64_t hole = at(0);
            while (end >= 2 && child <= end - 2) {
                const uint64_t c0 = at(child), c1 = at(child + 1);
                const bool right = le(c0, c1);
                child += right ? 1 : 0;
                at(pos) = right ? c1 : c0;
                pos = child;
                child = 2 * pos + 1;
            }
            if (child == end - 1) {
                at(pos) = at(child);
                pos = child;
            }
            at(pos) = hole;
            sift_up(0, pos);
        }
        return top;
    }
};

// MSB-first bit writer into a stream's tree-bits bytes
struct BitOut {
    uint8_t* p;
    uint64_t acc = 0;
    uint32_t nacc = 0, nbits = 0;
    __device__ void put(uint32_t v, uint32_t len) {  // len <= 9
        acc = (acc << len) | v;
        nacc += len;
        nbits += len;
        while (nacc >= 8) {
            nacc -= 8;
            *p++ = static_cast<uint8_t>(acc >> nacc);
        }
    }
    __device__ void finish() {
        if (nacc) *p = static_cast<uint8_t>(acc << (8 - nacc));
    }
};

__global__ __launch_bounds__(kTreeLanes) void k_tree_batch(TreeBatchArgs a) {
    __shared__ uint64_t heap[kHeapCap][kTreeLanes];     // also the walk's stack afterwards
    __shared__ uint32_t joint[kHeapCap][kTreeLanes];    // joint j = node nleaves + j: left | right << 16
    __shared__ uint8_t leaf[kHeapCap + 3][kTreeLanes];  // leaf i's letter
    const uint32_t lane = threadIdx.x;
    const uint32_t s = blockIdx.x * kTreeLanes + lane;
    if (s >= a.nstreams) return;
    const uint64_t* h = a.hist + static_cast<uint64_t>(s) * 256;
    uint64_t* codes = a.codes + static_cast<uint64_t>(s) * 256;
    for (uint32_t b = 0; b < 256; ++b) codes[b] = 0;

    // leaves in ByteWeights::iter order (host/weights.cpp); the row is read
    // 16 weights at a time (independent loads in flight, not one latency per bin)
    LaneHeap hp{heap, lane};
    uint32_t nl = 0;
    int last = -1;
    uint64_t w0 = 0;
    for (uint32_t b0 = 0; b0 < 256; b0 += 16) {
        uint64_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = h[b0 + j];
        if (b0 == 0) w0 = w[0];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (w[j] == 0) continue;
            leaf[nl][lane] = static_cast<uint8_t>(b0 + j);
            hp.push((w[j] << kNodeBits) | nl);
            ++nl;
            last = static_cast<int>(b0 + j);
        }
    }
    if (w0 != 0 && last != 255) {
        leaf[nl][lane] = 0;
        hp.push((w0 << kNodeBits) | nl);
        ++nl;
    }
    // the heap keys hold weight << kNodeBits: every joint's weight (at most
    // the total) must stay below 2^54
    {
        uint64_t total = w0 != 0 && last != 255 ? w0 : 0;
        bool heavy = (total >> 54) != 0;
        for (uint32_t b = 0; b < 256; ++b) {
            const uint64_t wb = h[b];
            heavy |= (wb >> 54) != 0;
            total += heavy ? 0 : wb;
            heavy |= (total >> 54) != 0;
        }
        if (heavy) {
            a.status[s] = kTreeHeavy;
            a.tree_nbits[s] = 0;
            return;
        }
    }
    if (nl == 0) {  // tree_inner.rs:283-285
        a.status[s] = kTreeEmpty;
        a.tree_nbits[s] = 0;
        return;
    }
    // merges: min -> left (bit 0), next min -> right (bit 1)
    uint32_t next = nl;
    while (hp.n > 1) {
        const uint64_t x = hp.pop();
        const uint64_t y = hp.pop();
        const uint32_t xn = static_cast<uint32_t>(x & ((1u << kNodeBits) - 1));
        const uint32_t yn = static_cast<uint32_t>(y & ((1u << kNodeBits) - 1));
        joint[next - nl][lane] = xn | (yn << 16);
        hp.push((((x >> kNodeBits) + (y >> kNodeBits)) << kNodeBits) | next);
        ++next;
    }
    const uint32_t root = static_cast<uint32_t>(hp.pop() & ((1u << kNodeBits) - 1));

    // preorder walk (stack in the heap's storage): as_bin bits and codes
    BitOut bo{a.tree_bits + static_cast<uint64_t>(s) * a.tree_stride};
    uint32_t status = kTreeOk, maxlen = 0;
    if (root < nl) {  // a root leaf: code "0" (tree_inner.rs:313-315)
        const uint32_t l = leaf[root][lane];
        bo.put(l, 9);  // 0, then the letter
        codes[l] = (0ull << 8) | 1u;
        maxlen = 1;
    } else {
        // stack entry: node | depth << 16 | (edge bit into the node) << 32;
        // path = the current path's edge bits, MSB-first (codes of <= 64 bits)
        uint32_t sp = 0;
        heap[sp++][lane] = root;
        uint64_t path = 0;
        while (sp) {
            const uint64_t e = heap[--sp][lane];
            const uint32_t node = static_cast<uint32_t>(e & 0xFFFF);
            const uint32_t depth = static_cast<uint32_t>((e >> 16) & 0xFFFF);
            if (depth && depth <= 64) {
                const uint64_t m = 1ull << (64 - depth);
                path = (e >> 32) & 1 ? (path | m) : (path & ~m);
            }
            if (node < nl) {
                const uint32_t l = leaf[node][lane];
                bo.put(l, 9);  // 0, then the letter
                if (depth > maxlen) maxlen = depth;
                if (depth <= kTreeCodeMax) {
                    codes[l] = ((path >> (64 - depth)) << 8) | depth;  // HashMap insert: a later leaf wins
                } else {
                    codes[l] = 0;
                    status = kTreeDeep;
                }
                continue;
            }
            bo.put(1, 1);
            const uint32_t j = joint[node - nl][lane];
            heap[sp++][lane] = (j >> 16) | (static_cast<uint64_t>(depth + 1) << 16) | (1ull << 32);
            heap[sp++][lane] = (j & 0xFFFF) | (static_cast<uint64_t>(depth + 1) << 16);
        }
    }
    bo.finish();
    a.tree_nbits[s] = bo.nbits;
    a.max_len[s] = maxlen;
    a.status[s] = status;
}

}  // namespace

hipError_t launch_hist_batch(const uint8_t* in, const uint64_t* off, uint32_t nstreams, uint64_t* hist,
                             hipStream_t s) {
    if (nstreams == 0) return hipSuccess;
    launch_k(k_hist_batch, dim3(nstreams), dim3(256), 0, s, in, off, hist);
    return hipGetLastError();
}

hipError_t launch_tree_batch(const TreeBatchArgs& a, hipStream_t s) {
    if (a.nstreams == 0) return hipSuccess;
    launch_k(k_tree_batch, dim3((a.nstreams + kTreeLanes - 1) / kTreeLanes), dim3(kTreeLanes), 0, s, a);
    return hipGetLastError();
}

}  // namespace huff::dev
