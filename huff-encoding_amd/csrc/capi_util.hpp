// capi_util.hpp — status -> int code + thread-local message, shared by the
// extern "C" files (capi.cpp, capi_wide.cpp). Nothing throws across the ABI.
#pragma once

#include <algorithm>
#include <cstdint>
#include <exception>
#include <new>
#include <utility>
#include <vector>

#include "common.hpp"

namespace huff::capi {

int report(const huff::Status& s);
int fail(int code, const char* msg);
const char* last_error();
uint8_t last_missing();

template <class F>
int guarded(F&& f) {
    try {
        return report(f());
    } catch (const std::bad_alloc&) {
        return fail(HUFF_E_INVALID_ARG, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(HUFF_E_INVALID_ARG, e.what());
    }
}

// HuffLeaf::code of a branch (leaf.rs:70-73): its path from the root, left
// 0 / right 1 (tree_inner.rs:422-440); the root of a tree with children has
// none (has_code false), a single-leaf root the code [0] (tree_inner.rs:
// 310-315). Node needs is_leaf, left, right.
//
// parent_links: every node's link to its parent, (parent << 1) | side, -1 for
// the root and any node not below it; built once per tree (the trees cache
// it), so a code costs O(depth) instead of a depth-first search per call
// (visiting every leaf of a large wide tree was O(nodes^2)).
template <class Node>
std::vector<int32_t> parent_links(const std::vector<Node>& nodes, int32_t root) {
    std::vector<int32_t> up(nodes.size(), -1);
    std::vector<int32_t> stack{root};
    while (!stack.empty()) {
        const int32_t v = stack.back();
        stack.pop_back();
        const Node& n = nodes[v];
        if (n.is_leaf) continue;
        up[n.left] = v << 1;
        up[n.right] = (v << 1) | 1;
        stack.push_back(n.left);
        stack.push_back(n.right);
    }
    return up;
}
// false: the branch is not below the root
template <class Node>
bool branch_path(const std::vector<Node>& nodes, const std::vector<int32_t>& up, int32_t root, int32_t branch,
                 std::vector<uint8_t>& path, bool& has_code) {
    path.clear();
    if (branch == root) {
        has_code = nodes[root].is_leaf;
        if (has_code) path.push_back(0);
        return true;
    }
    for (int32_t v = branch; v != root;) {
        const int32_t l = up[v];
        if (l < 0) return false;
        path.push_back(static_cast<uint8_t>(l & 1));
        v = l >> 1;
    }
    std::reverse(path.begin(), path.end());
    has_code = true;
    return true;
}

}  // namespace huff::capi
