// common.hpp — status/error plumbing shared by the host and device halves.
//
// Every reference panic / Result error becomes a huff_status with the
// reference's message (see include/huffgpu.h). Errors are carried as a Status
// value inside the C++ code and turned into the thread-local last-error at the
// C ABI (capi.cpp).
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>

#include "huffgpu.h"

namespace huff {

struct Status {
    int code = HUFF_OK;
    std::string msg;
    uint8_t missing_letter = 0;

    static Status ok() { return {}; }
    static Status err(int c, std::string m) {
        Status s;
        s.code = c;
        s.msg = std::move(m);
        return s;
    }
    explicit operator bool() const { return code != HUFF_OK; }  // true == failure
};

#define HUFF_TRY(expr)                     \
    do {                                   \
        ::huff::Status _st = (expr);       \
        if (_st) return _st;               \
    } while (0)

// utils.rs:37-40 calc_padding_bits (also huff/src/utils.rs:29-32)
inline uint8_t calc_padding_bits(uint64_t bit_count) {
    uint8_t n = static_cast<uint8_t>(8 - bit_count % 8);
    return n == 8 ? 0 : n;
}

}  // namespace huff
