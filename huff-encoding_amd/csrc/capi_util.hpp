// capi_util.hpp — status -> int code + thread-local message, shared by the
// extern "C" files (capi.cpp, capi_wide.cpp). Nothing throws across the ABI.
#pragma once

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
// 310-315). Node needs is_leaf, left, right. false: the branch is not below
// the root.
template <class Node>
bool branch_path(const std::vector<Node>& nodes, int32_t root, int32_t branch, std::vector<uint8_t>& path,
                 bool& has_code) {
    path.clear();
    if (branch == root) {
        has_code = nodes[root].is_leaf;
        if (has_code) path.push_back(0);
        return true;
    }
    // depth first from the root, left before right, keeping the path
    std::vector<std::pair<int32_t, uint8_t>> stack{{root, 0}};  // (node, next side)
    while (!stack.empty()) {
        auto& top = stack.back();
        const Node& n = nodes[top.first];
        if (n.is_leaf || top.second > 1) {
            stack.pop_back();
            if (!path.empty()) path.pop_back();
            continue;
        }
        const uint8_t side = top.second++;
        const int32_t child = side ? n.right : n.left;
        path.push_back(side);
        if (child == branch) {
            has_code = true;
            return true;
        }
        stack.push_back({child, 0});
    }
    return false;
}

}  // namespace huff::capi
