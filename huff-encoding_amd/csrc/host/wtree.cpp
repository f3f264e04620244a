// wtree.cpp — HuffTree<L> for the wider integer letters (wide.hpp).
//
// Same algorithm as tree.cpp (tree_inner.rs:281-320 over the Rust std heap,
// rust_heap.hpp), with W-byte letters and an unbounded number of leaves.
#include <algorithm>

#include "rust_heap.hpp"
#include "wide.hpp"

namespace huff {

Status WideTree::from_weights(uint32_t width, const uint8_t* letters, const uint64_t* weights, size_t n,
                              WideTree& out) {
    if (!valid_width(width)) return Status::err(HUFF_E_INVALID_ARG, "letter width must be 1, 2, 4, 8 or 16 bytes");
    if (n == 0) return Status::err(HUFF_E_EMPTY_WEIGHTS, "provided empty weights");  // tree_inner.rs:283-285
    out.width_ = width;
    out.nodes_.clear();
    out.nodes_.reserve(2 * n);
    RustMaxHeap heap(n + 1);
    for (size_t i = 0; i < n; ++i) {  // branch_heap.rs:52-58, in the Weights' iteration order
        WideNode leaf;
        leaf.is_leaf = true;
        leaf.letter = load_letter(letters + i * width, width);
        leaf.weight = weights[i];
        out.nodes_.push_back(leaf);
        heap.push({weights[i], static_cast<int32_t>(out.nodes_.size() - 1)});
    }
    while (heap.size() > 1) {  // tree_inner.rs:289-303
        const HeapEntry a = heap.pop();  // min      -> left  (0)
        const HeapEntry b = heap.pop();  // next min -> right (1)
        WideNode joint;
        joint.weight = a.w + b.w;
        joint.left = a.node;
        joint.right = b.node;
        out.nodes_.push_back(joint);
        heap.push({joint.weight, static_cast<int32_t>(out.nodes_.size() - 1)});
    }
    out.root_ = heap.pop().node;
    return Status::ok();
}

Status WideTree::try_from_bin(uint32_t width, const std::vector<uint8_t>& bits, WideTree& out) {
    // tree_inner.rs:526-590, iteratively (as HuffTree::try_from_bin), W*8 letter bits
    static const char* kSmall = "Provided BitVec is too small for an encoded HuffTree";
    static const char* kBig = "Provided BitVec is too big for an encoded HuffTree";
    if (!valid_width(width)) return Status::err(HUFF_E_INVALID_ARG, "letter width must be 1, 2, 4, 8 or 16 bytes");
    const uint32_t lb = 8 * width;
    out.width_ = width;
    out.nodes_.clear();
    struct Open {
        int32_t node;
        int filled;
    };
    std::vector<Open> open;
    size_t pos = 0;
    int32_t root = -1;
    const size_t n = bits.size();
    for (;;) {
        if (pos >= n) return Status::err(HUFF_E_FROM_BIN, kSmall);  // :530-535
        int32_t idx;
        if (bits[pos++]) {
            out.nodes_.push_back(WideNode{});
        } else {
            if (n - pos < lb) return Status::err(HUFF_E_FROM_BIN, kSmall);  // :554-559
            u128 v = 0;
            for (uint32_t k = 0; k < lb; ++k) v = (v << 1) | bits[pos + k];
            pos += lb;
            WideNode leaf;
            leaf.is_leaf = true;
            leaf.letter = v;
            out.nodes_.push_back(leaf);
        }
        idx = static_cast<int32_t>(out.nodes_.size() - 1);
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
            if (open.empty()) break;
        }
    }
    if (pos != n) return Status::err(HUFF_E_FROM_BIN, kBig);  // :586-590
    out.root_ = root;
    return Status::ok();
}

std::vector<uint8_t> WideTree::as_bin() const {
    // tree_inner.rs:637-663: preorder; joint -> 1, leaf -> 0 + as_be_bytes bits
    const uint32_t lb = 8 * width_;
    std::vector<uint8_t> bits;
    std::vector<int32_t> st{root_};
    while (!st.empty()) {
        const int32_t x = st.back();
        st.pop_back();
        const WideNode& nd = nodes_[x];
        if (nd.is_leaf) {
            bits.push_back(0);
            for (uint32_t k = lb; k-- > 0;) bits.push_back(static_cast<uint8_t>((nd.letter >> k) & 1));
        } else {
            bits.push_back(1);
            st.push_back(nd.right);
            st.push_back(nd.left);
        }
    }
    return bits;
}

bool WideTree::leaves(std::vector<WideLeaf>& out) const {
    out.clear();
    if (nodes_[root_].is_leaf) {  // tree_inner.rs:313-315
        out.push_back({nodes_[root_].letter, 0, 1});
        return true;
    }
    struct Frame {
        int32_t node;
        uint32_t depth;
        uint64_t code;
    };
    bool ok = true;
    std::vector<Frame> st{{nodes_[root_].right, 1, 1}, {nodes_[root_].left, 1, 0}};
    while (!st.empty()) {
        const Frame fr = st.back();
        st.pop_back();
        const WideNode& nd = nodes_[fr.node];
        if (nd.is_leaf) {
            if (fr.depth > 64) ok = false;
            out.push_back({nd.letter, fr.code, fr.depth});
            continue;
        }
        st.push_back({nd.right, fr.depth + 1, (fr.code << 1) | 1});
        st.push_back({nd.left, fr.depth + 1, fr.code << 1});
    }
    return ok;
}

bool WideTree::read_codes(std::vector<WideLeaf>& out) const {
    std::vector<WideLeaf> lv;
    const bool ok = leaves(lv);
    // HashMap::insert in preorder: the later leaf of a letter wins
    std::vector<uint32_t> order(lv.size());
    for (uint32_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return lv[a].letter < lv[b].letter; });
    out.clear();
    for (size_t i = 0; i < order.size(); ++i) {
        if (i + 1 < order.size() && lv[order[i + 1]].letter == lv[order[i]].letter) continue;
        out.push_back(lv[order[i]]);
    }
    return ok;
}

HuffTree WideTree::shape() const {
    std::vector<HuffNode> nodes(nodes_.size());
    for (size_t i = 0; i < nodes_.size(); ++i) {
        nodes[i].left = nodes_[i].left;
        nodes[i].right = nodes_[i].right;
        nodes[i].weight = nodes_[i].weight;
        nodes[i].is_leaf = nodes_[i].is_leaf;
        nodes[i].letter = 0;
    }
    return HuffTree::from_nodes(std::move(nodes), root_);
}

size_t WideTree::num_leaves() const {
    size_t c = 0;
    for (const WideNode& nd : nodes_) c += nd.is_leaf ? 1 : 0;
    return c;
}

uint32_t WideTree::max_depth() const {
    if (nodes_[root_].is_leaf) return 1;
    uint32_t m = 0;
    std::vector<std::pair<int32_t, uint32_t>> st{{root_, 0}};
    while (!st.empty()) {
        auto [x, d] = st.back();
        st.pop_back();
        if (nodes_[x].is_leaf) {
            m = std::max(m, d);
        } else {
            st.push_back({nodes_[x].left, d + 1});
            st.push_back({nodes_[x].right, d + 1});
        }
    }
    return m;
}

Status build_wide_enc_tables(const WideTree& t, WideEncTables& out) {
    std::vector<WideLeaf> codes;
    t.read_codes(codes);
    uint32_t maxlen = 0;
    for (const WideLeaf& c : codes) maxlen = std::max(maxlen, c.len);
    if (maxlen > kWideMaxEncodeLen)
        return Status::err(HUFF_E_CODE_TOO_LONG, "code longer than 56 bits: outside the GPU encoder's range");
    const uint32_t W = t.width();
    const uint32_t KB = wide_key_bytes(W);
    out.width = W;
    out.maxlen = maxlen;
    out.distinct = codes.size();
    // buckets of 2 slots, load <= 1/2; grow (at most 16x) until every key is
    // placed. Keys of <= 8 bytes hash injectively, so they separate within
    // that; 16-byte keys fold to 64 bits first, and letters whose folds
    // collide never separate by growing: then re-seed the fold multiplier
    uint32_t lgb0 = 5;
    while ((2ull << lgb0) < 2 * codes.size()) ++lgb0;
    struct Ent {
        u128 key;
        uint64_t val;
        bool used;
    };
    std::vector<Ent> slot;
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    uint64_t fold = kWideFold0, seed = 0;
    const uint32_t lg_cap = std::min<uint32_t>(lgb0 + 4, 31);
    uint32_t lgb = lgb0;
    for (;; ++lgb) {
        if (lgb > lg_cap) {
            if (W <= 8 || ++seed > 64)
                return Status::err(HUFF_E_INVALID_ARG, "letters do not separate in the encoder's hash table");
            uint64_t z = (seed * 0x9E3779B97F4A7C15ull) ^ kWideFold0;  // splitmix64 of the seed
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            fold = (z ^ (z >> 31)) | 1u;
            lgb = lgb0;
        }
        slot.assign(size_t(2) << lgb, Ent{0, 0, false});
        bool ok = true;
        for (const WideLeaf& c : codes) {
            Ent cur{c.letter, (c.code << 8) | c.len, true};
            bool placed = false;
            for (int kick = 0; kick < 1000 && !placed; ++kick) {
                uint32_t b[2];
                wide_buckets(static_cast<uint64_t>(cur.key), static_cast<uint64_t>(cur.key >> 64), lgb, W, fold, &b[0],
                             &b[1]);
                for (int q = 0; q < 4 && !placed; ++q) {
                    Ent& e = slot[2 * b[q >> 1] + (q & 1)];
                    if (!e.used) {
                        e = cur;
                        placed = true;
                    }
                }
                if (placed) break;
                rng ^= rng << 13;
                rng ^= rng >> 7;
                rng ^= rng << 17;
                std::swap(cur, slot[2 * b[rng & 1] + ((rng >> 1) & 1)]);  // evict, re-place the evicted
            }
            if (!placed) {
                ok = false;
                break;
            }
        }
        if (ok) break;
    }
    out.log2_slots = lgb + 1;
    out.fold = fold;
    out.keys.assign(slot.size() * KB, 0);
    out.vals.assign(slot.size(), 0);
    for (size_t i = 0; i < slot.size(); ++i) {
        if (!slot[i].used) continue;
        store_letter(&out.keys[i * KB], W, slot[i].key);
        out.vals[i] = slot[i].val;
    }
    out.vals32.clear();
    if (maxlen <= 24) out.vals32.assign(out.vals.begin(), out.vals.end());
    return Status::ok();
}

Status build_wide_dec_tables(const WideTree& t, WideDecTables& out) {
    const uint32_t W = t.width();
    const auto& nodes = t.nodes();
    out.lut.clear();
    out.letters.clear();
    // leaf index = order of appearance in the walk below
    auto leaf_id = [&](int32_t x) {
        const uint32_t id = static_cast<uint32_t>(out.letters.size() / W);
        out.letters.resize(out.letters.size() + W);
        store_letter(&out.letters[id * W], W, nodes[x].letter);
        return id;
    };
    if (t.root_is_leaf()) {  // every bit decodes the root letter (comp.rs:506-509)
        out.bits = 1;
        out.maxdepth = 1;
        const uint32_t e = (1u << 24) | leaf_id(t.root());
        out.lut = {e, e};
        return Status::ok();
    }
    const uint32_t maxd = t.max_depth();
    if (maxd > kWideMaxDecodeLen)
        return Status::err(HUFF_E_CODE_TOO_LONG, "code longer than 57 bits: outside the GPU decoder's range");
    if (t.num_leaves() >= (1u << 24))
        return Status::err(HUFF_E_CODE_TOO_LONG, "more than 2^24 leaves: outside the GPU decoder's range");
    out.maxdepth = maxd;
    out.bits = std::max<uint32_t>(1, std::min<uint32_t>(maxd, kWideLutMaxBits - 1));
    out.lut.assign(1u << out.bits, 0);
    struct Job {
        int32_t x;
        uint32_t d0, tb, base;
    };
    std::vector<Job> jobs{{t.root(), 0, out.bits, 0}};
    while (!jobs.empty()) {
        const Job j = jobs.back();
        jobs.pop_back();
        struct F {
            int32_t node;
            uint32_t r, path;
        };
        std::vector<F> st{{nodes[j.x].right, 1, 1}, {nodes[j.x].left, 1, 0}};
        while (!st.empty()) {
            const F f = st.back();
            st.pop_back();
            const WideNode& nd = nodes[f.node];
            if (nd.is_leaf) {
                const uint32_t e = ((j.d0 + f.r) << 24) | leaf_id(f.node);
                const uint32_t lo = f.path << (j.tb - f.r), hi = (f.path + 1) << (j.tb - f.r);
                for (uint32_t i = lo; i < hi; ++i) out.lut[j.base + i] = e;
            } else if (f.r == j.tb) {
                const uint32_t sub = static_cast<uint32_t>(out.lut.size());
                out.lut.resize(out.lut.size() + 256, 0);
                out.lut[j.base + f.path] = kWideLutPtr | sub;
                jobs.push_back({f.node, j.d0 + j.tb, 8, sub});
            } else {
                st.push_back({nd.right, f.r + 1, (f.path << 1) | 1});
                st.push_back({nd.left, f.r + 1, f.path << 1});
            }
        }
    }
    return Status::ok();
}

}  // namespace huff
