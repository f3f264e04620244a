// rust_heap.hpp — the Rust std BinaryHeap algorithm, as the reference's tree
// build uses it (shared by the u8 tree and the generic-letter tree).
//
// The reference pushes leaves into a std BinaryHeap whose Ord is reversed on
// weight only (branch_heap.rs:67-71, leaf.rs:31-35) and repeatedly pops the two
// minima (tree_inner.rs:289-303). RustMaxHeap is that std heap's algorithm
// (sift_up on push; on pop the last element is swapped into the root, sifted
// down to the bottom always taking the right child on ties, then sifted up),
// keyed so that "a <= b" means a.w >= b.w.
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace huff {

struct HeapEntry {
    uint64_t w;
    int32_t node;
};

class RustMaxHeap {
public:
    explicit RustMaxHeap(size_t reserve) : v_(reserve) {}
    size_t size() const { return n_; }

    void push(HeapEntry e) {
        v_[n_++] = e;
        sift_up(0, n_ - 1);
    }

    HeapEntry pop() {
        HeapEntry top = v_[--n_];
        if (n_) {
            std::swap(top, v_[0]);
            sift_down_to_bottom(0);
        }
        return top;
    }

private:
    // "a <= b" under the reversed Ord of HuffBranchHeapItem
    static bool le(const HeapEntry& a, const HeapEntry& b) { return a.w >= b.w; }

    size_t sift_up(size_t start, size_t pos) {
        HeapEntry* v = v_.data();
        const HeapEntry hole = v[pos];
        while (pos > start) {
            const size_t parent = (pos - 1) >> 1;
            if (le(hole, v[parent])) break;
            v[pos] = v[parent];
            pos = parent;
        }
        v[pos] = hole;
        return pos;
    }

    void sift_down_to_bottom(size_t pos) {
        HeapEntry* v = v_.data();
        const size_t end = n_;
        const size_t start = pos;
        const HeapEntry hole = v[pos];
        size_t child = 2 * pos + 1;
        while (end >= 2 && child <= end - 2) {
            child += le(v[child], v[child + 1]) ? 1 : 0;
            v[pos] = v[child];
            pos = child;
            child = 2 * pos + 1;
        }
        if (child == end - 1) {
            v[pos] = v[child];
            pos = child;
        }
        v[pos] = hole;
        sift_up(start, pos);
    }

    std::vector<HeapEntry> v_;
    size_t n_ = 0;
};


// The same heap over packed keys w << 10 | node (node < 1024, every weight
// and sum < 2^54): one 8-byte load per sift step, and "a <= b" (a.w >= b.w)
// is a >= (b with its node bits cleared). Pops in exactly RustMaxHeap's
// order (the comparisons see the weights only, as there); ~25 % faster on a
// 256-leaf tree with ties (tests/test_host.cpp checks it against RustMaxHeap).
class PackedMaxHeap {
public:
    static constexpr unsigned kNodeBits = 10;
    static constexpr uint64_t kNodeMask = (1ull << kNodeBits) - 1;
    static constexpr size_t kCap = 1u << kNodeBits;
    size_t size() const { return n_; }
    void push(uint64_t w, int32_t node) {
        v_[n_++] = (w << kNodeBits) | static_cast<uint64_t>(node);
        sift_up(0, n_ - 1);
    }
    // (weight, node) of the popped entry
    void pop(uint64_t& w, int32_t& node) {
        uint64_t top = v_[--n_];
        if (n_) {
            std::swap(top, v_[0]);
            sift_down_to_bottom(0);
        }
        w = top >> kNodeBits;
        node = static_cast<int32_t>(top & kNodeMask);
    }

private:
    static bool le(uint64_t a, uint64_t b) { return a >= (b & ~kNodeMask); }
    size_t sift_up(size_t start, size_t pos) {
        const uint64_t hole = v_[pos];
        while (pos > start) {
            const size_t parent = (pos - 1) >> 1;
            if (le(hole, v_[parent])) break;
            v_[pos] = v_[parent];
            pos = parent;
        }
        v_[pos] = hole;
        return pos;
    }
    void sift_down_to_bottom(size_t pos) {
        const size_t end = n_;
        const size_t start = pos;
        const uint64_t hole = v_[pos];
        size_t child = 2 * pos + 1;
        while (end >= 2 && child <= end - 2) {
            child += le(v_[child], v_[child + 1]) ? 1 : 0;
            v_[pos] = v_[child];
            pos = child;
            child = 2 * pos + 1;
        }
        if (child == end - 1) {
            v_[pos] = v_[child];
            pos = child;
        }
        v_[pos] = hole;
        sift_up(start, pos);
    }
    uint64_t v_[kCap];
    size_t n_ = 0;
};

}  // namespace huff
