// tree.cpp — HuffTree on the host (huff_coding/src/tree/).
//
// The tree decides every output bit, so it is built with the reference's
// exact tie order: leaves go into RustMaxHeap (rust_heap.hpp) in the weights'
// iteration order and the two minima are popped repeatedly
// (tree_inner.rs:289-303).
#include <algorithm>
#include <numeric>
#include <utility>

#include "huff_coding.hpp"
#include "rust_heap.hpp"

namespace huff {


// The merges when no two items of the heap ever weigh the same: then every
// pop has one possible result whatever the heap's layout, so the sorted
// leaves and a FIFO of joints (produced in non-decreasing weight) give the
// tree RustMaxHeap gives, node for node, without its ~500 data-dependent
// sift loops (~8 of the host's ~10 us between pass 1 and pass 2). Any tie
// (equal leaves, a joint equal to a leaf or to another joint, the duplicate
// byte-0 leaf) returns false and the caller takes the heap.
static bool merge_untied(const uint64_t* weights, size_t n, std::vector<HuffNode>& nodes, int32_t& root) {
    if (n > 512) return false;
    {  // equal leaves (common: 1 GiB of uniform bytes has ~4 equal pairs of
       // counts): out before the sort, through a small open-addressing set
        uint64_t set[1024];
        bool used[1024] = {};
        for (size_t i = 0; i < n; ++i) {
            uint32_t h = static_cast<uint32_t>((weights[i] * 0x9E3779B97F4A7C15ull) >> 54);
            while (used[h]) {
                if (set[h] == weights[i]) return false;
                h = (h + 1) & 1023u;
            }
            used[h] = true;
            set[h] = weights[i];
        }
    }
    int32_t order[512];
    for (size_t i = 0; i < n; ++i) order[i] = static_cast<int32_t>(i);
    std::sort(order, order + n, [&](int32_t a, int32_t b) { return weights[a] < weights[b]; });
    struct J {
        uint64_t w;
        int32_t node;
    };
    J joints[512];
    size_t li = 0, jh = 0, jt = 0;
    // the lighter of the two queue fronts; false on a tie between them
    auto take = [&](uint64_t& w, int32_t& node) {
        const bool hl = li < n, hj = jh < jt;
        if (hl && hj && weights[order[li]] == joints[jh].w) return false;
        if (hl && (!hj || weights[order[li]] < joints[jh].w)) {
            node = order[li];
            w = weights[order[li++]];
        } else {
            node = joints[jh].node;
            w = joints[jh++].w;
        }
        return true;
    };
    for (size_t left = n; left > 1; --left) {
        uint64_t wa, wb;
        int32_t a, b;
        if (!take(wa, a) || !take(wb, b)) return false;  // min -> left, next_min -> right
        const uint64_t jw = wa + wb;
        if (jt > jh && joints[jt - 1].w == jw) return false;  // two equal joints
        HuffNode joint;
        joint.weight = jw;
        joint.left = a;
        joint.right = b;
        nodes.push_back(joint);
        joints[jt++] = J{jw, static_cast<int32_t>(nodes.size() - 1)};
    }
    uint64_t w;
    if (!take(w, root)) return false;
    return true;
}

Status HuffTree::from_leaves(const uint8_t* letters, const uint64_t* weights, size_t n, HuffTree& out) {
    if (n == 0) return Status::err(HUFF_E_EMPTY_WEIGHTS, "provided empty weights");
    out.nodes_.clear();
    out.nodes_.reserve(2 * n);
    for (size_t i = 0; i < n; ++i) {
        HuffNode leaf;
        leaf.is_leaf = true;
        leaf.letter = letters[i];
        leaf.weight = weights[i];
        out.nodes_.push_back(leaf);
    }
    if (merge_untied(weights, n, out.nodes_, out.root_)) return Status::ok();
    // a byte tree (<= 257 leaves, so < 1024 nodes) whose weights sum below
    // 2^54: the packed-key heap, same pops
    uint64_t sum = 0;
    bool small = n <= 257;
    for (size_t i = 0; small && i < n; ++i) {
        sum += weights[i];
        small = weights[i] < (1ull << 54) && sum < (1ull << 54);
    }
    if (small) {
        out.nodes_.resize(n);  // the leaves stay; merge_untied's joints go
        PackedMaxHeap heap;
        for (size_t i = 0; i < n; ++i) heap.push(weights[i], static_cast<int32_t>(i));  // branch_heap.rs:52-58
        while (heap.size() > 1) {  // tree_inner.rs:289-303
            uint64_t wa, wb;
            int32_t a, b;
            heap.pop(wa, a);  // min       -> left  (code bit 0)
            heap.pop(wb, b);  // next_min  -> right (code bit 1)
            HuffNode joint;
            joint.weight = wa + wb;
            joint.left = a;
            joint.right = b;
            out.nodes_.push_back(joint);
            heap.push(joint.weight, static_cast<int32_t>(out.nodes_.size() - 1));
        }
        uint64_t w;
        heap.pop(w, out.root_);  // tree_inner.rs:306
        return Status::ok();
    }
    out.nodes_.clear();
    RustMaxHeap heap(n + 1);
    for (size_t i = 0; i < n; ++i) {  // branch_heap.rs:52-58
        HuffNode leaf;
        leaf.is_leaf = true;
        leaf.letter = letters[i];
        leaf.weight = weights[i];
        out.nodes_.push_back(leaf);
        heap.push({weights[i], static_cast<int32_t>(out.nodes_.size() - 1)});
    }
    while (heap.size() > 1) {  // tree_inner.rs:289-303
        HeapEntry a = heap.pop();  // min       -> left  (code bit 0)
        HeapEntry b = heap.pop();  // next_min  -> right (code bit 1)
        HuffNode joint;
        joint.weight = a.w + b.w;
        joint.left = a.node;
        joint.right = b.node;
        out.nodes_.push_back(joint);
        heap.push({joint.weight, static_cast<int32_t>(out.nodes_.size() - 1)});
    }
    out.root_ = heap.pop().node;  // tree_inner.rs:306
    return Status::ok();
}

Status HuffTree::from_weights(const ByteWeights& w, HuffTree& out) {
    if (w.is_empty()) return Status::err(HUFF_E_EMPTY_WEIGHTS, "provided empty weights");
    uint8_t l[257];
    uint64_t f[257];
    size_t cnt = w.iter(l, f);  // IntoIter order, §C.1 duplicate included
    return from_leaves(l, f, cnt, out);
}

std::vector<LeafCode> HuffTree::leaves() const {
    std::vector<LeafCode> out;
    if (nodes_[root_].is_leaf) {  // tree_inner.rs:313-315: a root leaf's code is "0"
        out.push_back({nodes_[root_].letter, 1, {0}});
        return out;
    }
    struct Frame {
        int32_t node;
        uint32_t depth;
        uint8_t bit;  // bit on the edge into this node
    };
    std::vector<Frame> st;
    std::vector<uint8_t> path;
    st.push_back({nodes_[root_].right, 1, 1});
    st.push_back({nodes_[root_].left, 1, 0});
    while (!st.empty()) {
        Frame fr = st.back();
        st.pop_back();
        path.resize(fr.depth - 1);
        path.push_back(fr.bit);
        const HuffNode& nd = nodes_[fr.node];
        if (nd.is_leaf) {
            out.push_back({nd.letter, fr.depth, path});
            continue;
        }
        st.push_back({nd.right, fr.depth + 1, 1});
        st.push_back({nd.left, fr.depth + 1, 0});
    }
    return out;
}

void HuffTree::read_codes(std::array<std::vector<uint8_t>, 256>& codes) const {
    for (auto& c : codes) c.clear();
    // leaves() is in left-to-right order = the reference's insert order, so a
    // later duplicate overwrites an earlier one (HashMap::insert).
    for (const LeafCode& lc : leaves()) codes[lc.letter] = lc.bits;
}

bool HuffTree::read_codes_u64(uint64_t code[256], uint8_t len[256], uint32_t* maxlen) const {
    // read_codes (tree_inner.rs:356-440) without materialising bit vectors:
    // preorder, left before right, a later leaf of the same letter overwrites
    uint32_t true_len[256] = {};
    bool seen[256] = {};
    for (int b = 0; b < 256; ++b) {
        code[b] = 0;
        len[b] = 0;
    }
    if (nodes_[root_].is_leaf) {  // tree_inner.rs:313-315: a root leaf's code is "0"
        const uint8_t l = nodes_[root_].letter;
        len[l] = 1;
        if (maxlen) *maxlen = 1;
        return true;
    }
    struct Frame {
        int32_t node;
        uint32_t depth;
        uint64_t code;  // low 64 bits of the path (exact while depth <= 64)
    };
    Frame st[512];
    int sp = 0;
    st[sp++] = {nodes_[root_].right, 1, 1};
    st[sp++] = {nodes_[root_].left, 1, 0};
    while (sp) {
        const Frame fr = st[--sp];
        const HuffNode& nd = nodes_[fr.node];
        if (nd.is_leaf) {
            const uint8_t l = nd.letter;
            seen[l] = true;
            true_len[l] = fr.depth;
            code[l] = fr.depth <= 64 ? fr.code : 0;  // longer codes: read_codes (bit vectors)
            len[l] = static_cast<uint8_t>(fr.depth);  // <= 255 (a 256-leaf tree's depth)
            continue;
        }
        st[sp++] = {nd.right, fr.depth + 1, (fr.code << 1) | 1};
        st[sp++] = {nd.left, fr.depth + 1, fr.code << 1};
    }
    uint32_t ml = 0;
    bool ok = true;
    for (int b = 0; b < 256; ++b) {
        if (!seen[b]) continue;
        ml = std::max(ml, true_len[b]);
        ok &= true_len[b] <= 64;
    }
    if (maxlen) *maxlen = ml;
    return ok;
}

size_t HuffTree::num_leaves() const {
    size_t c = 0;
    std::vector<int32_t> st{root_};
    while (!st.empty()) {
        int32_t n = st.back();
        st.pop_back();
        if (nodes_[n].is_leaf) {
            ++c;
        } else {
            st.push_back(nodes_[n].left);
            st.push_back(nodes_[n].right);
        }
    }
    return c;
}

void HuffTree::depth_range(uint32_t* min_depth, uint32_t* max_depth, uint32_t* gcd) const {
    // leaf depths without materialising the codes (leaves() allocates a path
    // per leaf: ~20 us per call, on the host's path between the passes)
    if (nodes_[root_].is_leaf) {  // tree_inner.rs:313-315: a root leaf's code is "0"
        *min_depth = *max_depth = 1;
        if (gcd) *gcd = 1;
        return;
    }
    uint32_t lo = ~0u, hi = 0, g = 0;
    std::vector<std::pair<int32_t, uint32_t>> st;
    st.reserve(64);
    st.push_back({root_, 0});
    while (!st.empty()) {
        const auto [n, d] = st.back();
        st.pop_back();
        const HuffNode& nd = nodes_[n];
        if (nd.is_leaf) {
            lo = std::min(lo, d);
            hi = std::max(hi, d);
            g = std::gcd(g, d);
        } else {
            st.push_back({nd.right, d + 1});
            st.push_back({nd.left, d + 1});
        }
    }
    *min_depth = lo;
    *max_depth = hi;
    if (gcd) *gcd = g;
}

uint32_t HuffTree::max_depth() const {
    uint32_t lo, hi;
    depth_range(&lo, &hi);
    return hi;
}

std::vector<uint8_t> HuffTree::as_bin() const {
    // tree_inner.rs:632-663: preorder; joint -> 1, leaf -> 0 then the letter's
    // big-endian bits (8 for u8).
    std::vector<uint8_t> bits;
    std::vector<int32_t> st{root_};
    while (!st.empty()) {
        int32_t n = st.back();
        st.pop_back();
        const HuffNode& nd = nodes_[n];
        if (nd.is_leaf) {
            bits.push_back(0);
            for (int k = 7; k >= 0; --k) bits.push_back((nd.letter >> k) & 1);
        } else {
            bits.push_back(1);
            st.push_back(nd.right);
            st.push_back(nd.left);
        }
    }
    return bits;
}

Status HuffTree::try_from_bin(const std::vector<uint8_t>& bits, HuffTree& out) {
    // tree_inner.rs:526-590, iteratively: a 1 opens a joint branch whose two
    // children follow in preorder; a 0 is a letter branch + 8 letter bits.
    static const char* kSmall = "Provided BitVec is too small for an encoded HuffTree";
    static const char* kBig = "Provided BitVec is too big for an encoded HuffTree";
    out.nodes_.clear();
    struct Open {
        int32_t node;
        int filled;  // children attached so far
    };
    std::vector<Open> open;
    size_t pos = 0;
    int32_t root = -1;
    const size_t n = bits.size();
    for (;;) {
        if (pos >= n) return Status::err(HUFF_E_FROM_BIN, kSmall);
        int32_t idx;
        if (bits[pos++]) {
            out.nodes_.push_back(HuffNode{});
            idx = static_cast<int32_t>(out.nodes_.size() - 1);
        } else {
            if (n - pos < 8) return Status::err(HUFF_E_FROM_BIN, kSmall);
            uint8_t letter = 0;
            for (int k = 0; k < 8; ++k) letter = static_cast<uint8_t>((letter << 1) | bits[pos + k]);
            pos += 8;
            HuffNode leaf;
            leaf.is_leaf = true;
            leaf.letter = letter;
            out.nodes_.push_back(leaf);
            idx = static_cast<int32_t>(out.nodes_.size() - 1);
        }
        // attach to the innermost open joint
        if (open.empty()) {
            root = idx;
        } else {
            Open& o = open.back();
            if (o.filled == 0) out.nodes_[o.node].left = idx;
            else out.nodes_[o.node].right = idx;
            o.filled++;
        }
        if (!out.nodes_[idx].is_leaf) {
            open.push_back({idx, 0});
        } else {
            while (!open.empty() && open.back().filled == 2) open.pop_back();
            if (open.empty()) break;  // root complete
        }
    }
    if (pos != n) return Status::err(HUFF_E_FROM_BIN, kBig);  // tree_inner.rs:586-590
    out.root_ = root;
    return Status::ok();
}

}  // namespace huff
