// capi_util.hpp — status -> int code + thread-local message, shared by the
// extern "C" files (capi.cpp, capi_wide.cpp). Nothing throws across the ABI.
#pragma once

#include <exception>
#include <new>

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

}  // namespace huff::capi
