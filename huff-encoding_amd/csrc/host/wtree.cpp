// wtree.cpp — HuffTree<L> for the wider integer letters (wide.hpp).
//
// Same algorithm as tree.cpp (tree_inner.rs:281-320 over the Rust std heap,
// rust_heap.hpp), with W-byte letters and an unbounded number of leaves.
#include <algorithm>
#include <cstring>

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
    // tree_inner.rs:632-663: preorder; joint -> 1, leaf -> 0 + as_be_bytes bits
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
    out.width = W;
    out.maxlen = maxlen;
    out.distinct = codes.size();
    out.long_codes = maxlen > kWideShortMax;
    wide_slot_layout(W, out.long_codes, &out.val_off, &out.slot_bytes);
    // shortest code (most frequent letter) first: it takes its first slot
    std::stable_sort(codes.begin(), codes.end(), [](const WideLeaf& x, const WideLeaf& y) { return x.len < y.len; });
    const size_t D = codes.size();
    std::vector<uint32_t> hk(D), s1(D), s2(D);
    std::vector<int32_t> occ;
    // load <= 4/9 (two-choice cuckoo with single-slot buckets places every
    // key below 1/2 with high probability); a failed build re-seeds the hash
    // multipliers (and the fold of wide keys), every 8th failure grows the
    // table by 1/8
    // slots: a multiple of 256 (wide_slots' s2), >= 9/4 D; 16-bit keys use
    // the narrow hash below 65,536 slots and a direct table (slot = letter)
    // from there
    auto round256 = [](uint64_t m) { return (m + 255) / 256 * 256; };
    uint64_t M = round256(std::max<uint64_t>(512, (D * 9 + 3) / 4));
    out.hash_mode = kWideHashGeneric;
    if (W <= 2) out.hash_mode = M < 65536 ? kWideHashNarrow : kWideHashDirect;
    if (out.hash_mode == kWideHashDirect) M = 65536;
    uint64_t seed = 0;
    auto mix = [](uint64_t z) {  // splitmix64
        z += 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    for (uint32_t attempt = 0;; ++attempt) {
        if (attempt == 256 || M >= (1ull << 31))
            return Status::err(HUFF_E_INVALID_ARG, "letters do not separate in the encoder's hash table");
        if (attempt && attempt % 8 == 0 && out.hash_mode != kWideHashDirect) {
            M = round256(M + M / 8);
            if (out.hash_mode == kWideHashNarrow && M >= 65536) {
                out.hash_mode = kWideHashDirect;
                M = 65536;
            }
        }
        const uint64_t z = mix(++seed);
        out.mul1 = static_cast<uint32_t>(z) | 1u;
        out.fold = attempt == 0 ? kWideFold0 : (mix(seed ^ kWideFold0) | 1u);
        out.slots = static_cast<uint32_t>(M);
        for (size_t i = 0; i < D; ++i) {
            hk[i] = wide_hkey(static_cast<uint64_t>(codes[i].letter), static_cast<uint64_t>(codes[i].letter >> 64), W,
                              out.fold);
            wide_slots(hk[i], out.mul1, out.slots, out.hash_mode, &s1[i], &s2[i]);
        }
        occ.assign(M, -1);
        bool ok = true;
        for (size_t i = 0; i < D && ok; ++i) {
            if (occ[s1[i]] < 0) {
                occ[s1[i]] = static_cast<int32_t>(i);
                continue;
            }
            if (occ[s2[i]] < 0) {
                occ[s2[i]] = static_cast<int32_t>(i);
                continue;
            }
            // evict along the walk: the evicted key moves to its other slot
            int32_t cur = static_cast<int32_t>(i);
            uint32_t pos = s1[i];
            ok = false;
            for (int kick = 0; kick < 512; ++kick) {
                std::swap(cur, occ[pos]);
                const uint32_t alt = s1[cur] == pos ? s2[cur] : s1[cur];
                if (occ[alt] < 0) {
                    occ[alt] = cur;
                    ok = true;
                    break;
                }
                pos = alt;
            }
        }
        if (ok) break;
    }
    out.table.assign((static_cast<size_t>(M) * out.slot_bytes + 15) / 16 * 16, 0);  // staged in 16-B pieces
    // the empty slots' key: the smallest value that is no letter (keys of
    // <= 2 bytes: 2^32 - 1, above every letter)
    u128 empty = ~u128(0) >> (128 - 8 * wide_key_bytes(W));
    if (W > 2) {
        std::vector<u128> ls(D);
        for (size_t i = 0; i < D; ++i) ls[i] = codes[i].letter;
        std::sort(ls.begin(), ls.end());
        empty = 0;
        for (const u128& l : ls) {
            if (l != empty) break;
            ++empty;
        }
    }
    for (uint64_t sl = 0; sl < M; ++sl) {
        if (occ[sl] < 0) {
            store_letter(&out.table[sl * out.slot_bytes], wide_key_bytes(W), empty);
            continue;
        }
        const WideLeaf& c = codes[occ[sl]];
        uint8_t* p = &out.table[sl * out.slot_bytes];
        store_letter(p, W, c.letter);  // u32 keys: bytes W..3 stay zero
        if (out.long_codes) {
            const uint64_t v = (c.code << 6) | c.len;
            std::memcpy(p + out.val_off, &v, 8);
        } else {
            const uint32_t v = static_cast<uint32_t>(c.code << (32 - c.len)) | c.len;
            std::memcpy(p + out.val_off, &v, 4);
        }
    }
    return Status::ok();
}

// The task decoder's two-level table (WideDecTables::stab): level 1 indexed
// by the first K1 = sbits bits; a window whose first code is longer points to
// a level-2 table of 2^s entries indexed by the next s bits, s = the deepest
// leaf below that node minus K1 (exact depth: no further level). Left empty
// for codes > 32 bits or more than 4 Mi entries (the long-code decoder).
static void build_wide_stab(const WideTree& t, uint32_t W, const std::vector<int64_t>& leaf_of, WideDecTables& out) {
    const auto& nodes = t.nodes();
    const uint32_t eb = 4;
    // 4-byte letters sit in the entry when they all fit its 24 bits, else the
    // entry names the leaf (the u64 entries this replaces doubled the table,
    // which for a 4,096-letter alphabet no longer fitted the LDS)
    out.w4_leaf = false;
    if (W == 4)
        for (const auto& nd : nodes)
            if (nd.is_leaf && static_cast<uint64_t>(static_cast<uint32_t>(nd.letter)) >= (1u << 24)) out.w4_leaf = true;
    std::vector<uint64_t> tab;
    auto leaf_entry = [&](int32_t x, uint32_t len, uint32_t leaf) -> uint64_t {
        if (W <= 2 || (W == 4 && !out.w4_leaf)) return (static_cast<uint64_t>(static_cast<uint32_t>(nodes[x].letter)) << 8) | len;
        return (static_cast<uint64_t>(leaf) << 8) | len;
    };
    if (t.root_is_leaf()) {  // every bit decodes the root letter (comp.rs:506-509)
        out.sbits = 1;
        const int32_t r = t.root();
        tab = {leaf_entry(r, 1, static_cast<uint32_t>(leaf_of[r])), leaf_entry(r, 1, static_cast<uint32_t>(leaf_of[r]))};
    } else {
        const uint32_t K1 = out.sbits;
        tab.assign(size_t(1) << K1, 0);
        auto depth_below = [&](int32_t x) {
            uint32_t m = 0;
            std::vector<std::pair<int32_t, uint32_t>> st{{x, 0}};
            while (!st.empty()) {
                auto [y, d] = st.back();
                st.pop_back();
                if (nodes[y].is_leaf) {
                    m = std::max(m, d);
                } else {
                    st.push_back({nodes[y].left, d + 1});
                    st.push_back({nodes[y].right, d + 1});
                }
            }
            return m;
        };
        // walk `bits` bits (MSB first) of index i from node x: the leaf and
        // its depth, or the node reached at depth `bits`
        auto walk = [&](int32_t x, uint32_t i, uint32_t bits, uint32_t* depth) {
            for (uint32_t p = 0; p < bits; ++p) {
                x = ((i >> (bits - 1 - p)) & 1u) ? nodes[x].right : nodes[x].left;
                if (nodes[x].is_leaf) {
                    *depth = p + 1;
                    return x;
                }
            }
            *depth = bits;
            return x;
        };
        for (uint32_t i = 0; i < (1u << K1); ++i) {
            uint32_t d;
            const int32_t x = walk(t.root(), i, K1, &d);
            if (nodes[x].is_leaf) {
                tab[i] = leaf_entry(x, d, static_cast<uint32_t>(leaf_of[x]));
                continue;
            }
            const uint32_t sw = depth_below(x);  // >= 1
            if (K1 + sw > 32 || tab.size() + (size_t(1) << sw) > (size_t(1) << 22)) {
                out.stab.clear();  // codes > 32 bits or a table > 4 Mi entries: the long-code decoder
                return;
            }
            const uint64_t off = tab.size();
            tab[i] = (off << 8) | 0x80u | sw;
            tab.resize(tab.size() + (size_t(1) << sw));
            for (uint32_t j = 0; j < (1u << sw); ++j) {
                uint32_t r;
                const int32_t y = walk(x, j, sw, &r);
                tab[off + j] = leaf_entry(y, K1 + r, static_cast<uint32_t>(leaf_of[y]));
            }
        }
    }
    out.stab.assign((tab.size() * eb + 15) / 16 * 16, 0);
    for (size_t i = 0; i < tab.size(); ++i) {
        const uint32_t v = static_cast<uint32_t>(tab[i]);
        std::memcpy(&out.stab[i * 4], &v, 4);
    }
}

Status build_wide_dec_tables(const WideTree& t, WideDecTables& out) {
    const uint32_t W = t.width();
    const auto& nodes = t.nodes();
    out.lut.clear();
    out.letters.clear();
    // leaf index = order of appearance in the walk below (leaf_of: a node's
    // index, for the task decoder's table)
    std::vector<int64_t> leaf_of(nodes.size(), -1);
    auto leaf_id = [&](int32_t x) {
        const uint32_t id = static_cast<uint32_t>(out.letters.size() / W);
        out.letters.resize(out.letters.size() + W);
        store_letter(&out.letters[id * W], W, nodes[x].letter);
        leaf_of[x] = id;
        return id;
    };
    if (t.root_is_leaf()) {  // every bit decodes the root letter (comp.rs:506-509)
        out.bits = 1;
        out.maxdepth = 1;
        const uint32_t e = (1u << 24) | leaf_id(t.root());
        out.lut = {e, e};
        out.sbits = 1;
        build_wide_stab(t, W, leaf_of, out);
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
// K1: 11 bits (8 KiB of level 1): W = 2 decode 0.600 -> 0.585 ms, W = 4
// 0.474 -> 0.465 against 10 bits; 12 bits measured the same as 11
// (profiles/r05/widek1/)
#ifndef HUFF_WIDE_K1
#define HUFF_WIDE_K1 11
#endif
    out.sbits = std::max<uint32_t>(1, std::min<uint32_t>(maxd, HUFF_WIDE_K1));
    build_wide_stab(t, W, leaf_of, out);
    return Status::ok();
}

}  // namespace huff
