// test_host.cpp — the reference's own tests, restated against the product's
// C++ host code (huff_coding/tests/*.rs and the weights/tree doctests).
// Host only: no GPU call.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>

#include <random>
#include <vector>

#include "host/huff_coding.hpp"
#include "host/rust_heap.hpp"

using namespace huff;

static int g_fail = 0;
#define CHECK(c)                                                    \
    do {                                                            \
        if (!(c)) {                                                 \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                               \
        }                                                           \
    } while (0)

static ByteWeights weights_of(const std::string& s) {
    uint64_t c[256] = {};
    for (unsigned char ch : s) c[ch]++;
    return ByteWeights::from_counts(c);
}

static std::string code_of(const HuffTree& t, uint8_t letter) {
    std::array<std::vector<uint8_t>, 256> codes;
    t.read_codes(codes);
    std::string s;
    for (uint8_t b : codes[letter]) s.push_back(b ? '1' : '0');
    return s;
}

// tests/tree_init.rs:8-47 (letters 0..5 stand for the six strings)
static void tree_normal_init() {
    const uint8_t letters[6] = {0, 1, 2, 3, 4, 5};
    const uint64_t w[6] = {5, 9, 12, 13, 16, 45};
    HuffTree t;
    CHECK(!HuffTree::from_leaves(letters, w, 6, t));
    CHECK(code_of(t, 0) == "1100");
    CHECK(code_of(t, 1) == "1101");
    CHECK(code_of(t, 2) == "100");
    CHECK(code_of(t, 3) == "101");
    CHECK(code_of(t, 4) == "111");
    CHECK(code_of(t, 5) == "0");
}

// tests/tree_init.rs:49-64
static void tree_single_branch() {
    const uint8_t l = 12;
    const uint64_t w = 78;
    HuffTree t;
    CHECK(!HuffTree::from_leaves(&l, &w, 1, t));
    CHECK(t.root_is_leaf());
    CHECK(code_of(t, 12) == "0");
}

// tests/tree_init.rs:66-70
static void tree_invalid_weights() {
    HuffTree t;
    Status s = HuffTree::from_weights(ByteWeights{}, t);
    CHECK(s.code == HUFF_E_EMPTY_WEIGHTS && s.msg == "provided empty weights");
}

// tests/tree_bin.rs:6-14 and :28-32
static void tree_from_bin() {
    HuffTree t;
    CHECK(!HuffTree::from_weights(weights_of("Mongo...\n    a great barbarian from the north seeking to conquer "
                                             "new lands for his kingdom.\n    Mysterio the Magnificent...\n    a "
                                             "powerful wizard questing for the secret of immortality."),
                                  t));
    HuffTree t2;
    CHECK(!HuffTree::try_from_bin(t.as_bin(), t2));
    for (int b = 0; b < 256; ++b) CHECK(code_of(t, b) == code_of(t2, b));
    HuffTree t3;
    CHECK(HuffTree::try_from_bin({}, t3).code == HUFF_E_FROM_BIN);
}

// tree_inner.rs:621-628, lib.rs (crate doc): tree bits
static void tree_bits_known_answers() {
    HuffTree t;
    CHECK(!HuffTree::from_weights(weights_of("abbccc"), t));
    std::string s;
    for (uint8_t b : t.as_bin()) s.push_back(b ? '1' : '0');
    CHECK(s == "10011000111001100001001100010");
    CHECK(code_of(t, 'c') == "0" && code_of(t, 'b') == "11" && code_of(t, 'a') == "10");
    HuffTree u;
    CHECK(!HuffTree::from_weights(weights_of("\xff\xff\xff\xaa\xaa\xcc"), u));
    s.clear();
    for (uint8_t b : u.as_bin()) s.push_back(b ? '1' : '0');
    CHECK(s == "10111111111011001100010101010");
}

// comp.rs:219-262: to_bytes of abbccc with data bits 10 11 11 0 0 | 0
static void container_known_answer() {
    HuffTree t;
    CHECK(!HuffTree::from_weights(weights_of("abbccc"), t));
    const uint8_t comp[2] = {0xbc, 0x00};
    std::vector<uint8_t> out;
    CHECK(!container_to_bytes(t, comp, 2, 7, out));
    const uint8_t want[] = {0x37, 0, 0, 0, 4, 0x98, 0xe6, 0x13, 0x10, 0xbc, 0x00};
    CHECK(out.size() == sizeof(want) && std::memcmp(out.data(), want, sizeof(want)) == 0);
    HuffTree t2;
    uint8_t pad = 0;
    size_t off = 0, len = 0;
    CHECK(!container_from_bytes(out.data(), out.size(), t2, pad, off, len));
    CHECK(pad == 7 && off == 9 && len == 2);
}

// weights.rs doctests :148-150, :156-159, :165-172
static void byte_weights_doctests() {
    ByteWeights f = weights_of("fffff");
    CHECK(f.weights['f'] == 5 && f.len == 1);
    ByteWeights z = weights_of(std::string("\x00\x01\x01\x02\x02\x02", 6));
    uint8_t l[257];
    uint64_t w[257];
    size_t n = z.iter(l, w);
    for (size_t i = 0; i < n; ++i) CHECK(l[i] == w[i] - 1);
    CHECK(n == 4);  // includes the wrap duplicate of byte 0
    ByteWeights a = weights_of("aabbb");
    a.add(weights_of("aaabbc"));
    CHECK(a.weights['a'] == 5 && a.weights['b'] == 5 && a.weights['c'] == 1);
}

// shard plan vs the single stream: random shard cuts (empty and < 8-byte
// shards included) of a random byte string
static void shard_plan_matches_single_stream() {
    uint64_t rng = 0x1234567u;
    auto next = [&] { rng = rng * 6364136223846793005ull + 1442695040888963407ull; return rng >> 33; };
    for (int trial = 0; trial < 200; ++trial) {
        const size_t n = next() % 200;
        std::vector<uint8_t> data(n);
        for (auto& x : data) x = static_cast<uint8_t>(next() % 7);
        const uint32_t world = 1 + next() % 6;
        std::vector<size_t> cut{0};
        for (uint32_t q = 1; q < world; ++q) cut.push_back(n ? next() % (n + 1) : 0);
        cut.push_back(n);
        std::sort(cut.begin(), cut.end());
        std::vector<uint64_t> hists(world * 256, 0);
        std::vector<uint8_t> tails(world * 8, 0), tl(world, 0);
        for (uint32_t q = 0; q < world; ++q) {
            for (size_t i = cut[q]; i < cut[q + 1]; ++i) ++hists[q * 256 + data[i]];
            const size_t len = std::min<size_t>(8, cut[q + 1] - cut[q]);
            tl[q] = static_cast<uint8_t>(len);
            for (size_t k = 0; k < len; ++k) tails[q * 8 + k] = data[cut[q + 1] - len + k];
        }
        const ByteWeights g = shard_weights(hists.data(), world);
        for (int b = 0; b < 256; ++b) {
            uint64_t c = 0;
            for (uint8_t x : data) c += x == b;
            CHECK(g.weights[b] == c);
        }
        uint8_t len[256];
        for (int b = 0; b < 256; ++b) len[b] = static_cast<uint8_t>(1 + b % 5);
        for (uint32_t r = 0; r < world; ++r) {
            uint64_t want = 0;
            for (size_t i = 0; i < cut[r]; ++i) want += len[data[i]];
            CHECK(shard_bit_base(hists.data(), r, len) == want);
            uint8_t prev[8];
            size_t np = 0;
            shard_prev_tail(tails.data(), tl.data(), r, prev, &np);
            CHECK(np == std::min<size_t>(8, cut[r]));
            for (size_t k = 0; k < np; ++k) CHECK(prev[8 - np + k] == data[cut[r] - np + k]);
        }
    }
}

// The untied two-queue fast path in HuffTree::from_leaves must build the very
// tree the BinaryHeap loop builds (tree.rs:148-170): same node order, same
// children, same root, on random weight sets with and without ties.
static void tree_fast_path_matches_heap() {
    std::mt19937_64 r(7);
    int bad = 0;
    for (int it = 0; it < 30000; ++it) {
        size_t n = 1 + r() % 257;
        uint8_t l[257];
        uint64_t w[257];
        uint64_t range = (it % 3 == 0) ? 20 : (it % 3 == 1) ? 100000 : (1ull << 40);
        for (size_t i = 0; i < n; ++i) {
            l[i] = (uint8_t)i;
            w[i] = 1 + r() % range;
        }
        HuffTree a;
        CHECK(HuffTree::from_leaves(l, w, n, a).code == HUFF_OK);
        std::vector<HuffNode> nodes;
        RustMaxHeap heap(n + 1);
        for (size_t i = 0; i < n; ++i) {
            HuffNode lf;
            lf.is_leaf = true;
            lf.letter = l[i];
            lf.weight = w[i];
            nodes.push_back(lf);
            heap.push({w[i], (int32_t)i});
        }
        while (heap.size() > 1) {
            auto x = heap.pop(), y = heap.pop();
            HuffNode j;
            j.weight = x.w + y.w;
            j.left = x.node;
            j.right = y.node;
            nodes.push_back(j);
            heap.push({j.weight, (int32_t)nodes.size() - 1});
        }
        int32_t root = heap.pop().node;
        bool same = root == a.root() && nodes.size() == a.nodes().size();
        for (size_t i = 0; same && i < nodes.size(); ++i)
            same = nodes[i].left == a.nodes()[i].left && nodes[i].right == a.nodes()[i].right &&
                   nodes[i].weight == a.nodes()[i].weight && nodes[i].is_leaf == a.nodes()[i].is_leaf;
        if (!same) ++bad;
    }
    CHECK(bad == 0);
}

int main() {
    shard_plan_matches_single_stream();
    tree_normal_init();
    tree_single_branch();
    tree_fast_path_matches_heap();
    tree_invalid_weights();
    tree_from_bin();
    tree_bits_known_answers();
    container_known_answer();
    byte_weights_doctests();
    if (g_fail) {
        std::printf("%d FAILED\n", g_fail);
        return 1;
    }
    std::printf("ALL OK\n");
    return 0;
}
