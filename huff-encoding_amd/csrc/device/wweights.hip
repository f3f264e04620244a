// wweights.hip — build_weights_map (weights.rs:82-123) for the wider letters
// on the device: radix sort of the letters, then run-length encoding, gives
// every distinct letter with its count. rocPRIM's device-wide sort and RLE are
// plain library primitives here (as a BLAS call is for a plain GEMM); the
// order they produce (ascending letter value) is one of the orders a Rust
// HashMap<L, usize> can iterate in (RandomState makes it unspecified), and
// the caller builds the tree in it.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>

#include "kernels.hpp"

namespace huff::dev {

namespace {

template <typename T>
hipError_t sort_rle(const void* d_in, uint64_t n, void* d_sorted, void* d_uniq, uint64_t* d_counts,
                    uint64_t* d_nruns, void* d_tmp, size_t* tmp_bytes, hipStream_t s) {
    const T* in = static_cast<const T*>(d_in);
    T* sorted = static_cast<T*>(d_sorted);
    T* uniq = static_cast<T*>(d_uniq);
    auto* counts = reinterpret_cast<unsigned long long*>(d_counts);
    auto* nruns = reinterpret_cast<unsigned long long*>(d_nruns);
    size_t a = 0, b = 0;
    hipError_t e = rocprim::radix_sort_keys(nullptr, a, in, sorted, n, 0, 8 * sizeof(T), s);
    if (e != hipSuccess) return e;
    e = rocprim::run_length_encode(nullptr, b, sorted, n, uniq, counts, nruns, s);
    if (e != hipSuccess) return e;
    if (!d_tmp) {
        *tmp_bytes = a > b ? a : b;
        return hipSuccess;
    }
    e = rocprim::radix_sort_keys(d_tmp, a, in, sorted, n, 0, 8 * sizeof(T), s);
    if (e != hipSuccess) return e;
    return rocprim::run_length_encode(d_tmp, b, sorted, n, uniq, counts, nruns, s);
}

}  // namespace

hipError_t wide_weights(uint32_t width, const void* d_in, uint64_t n, void* d_sorted, void* d_uniq,
                        uint64_t* d_counts, uint64_t* d_nruns, void* d_tmp, size_t* tmp_bytes, hipStream_t s) {
    switch (width) {
        case 1: return sort_rle<uint8_t>(d_in, n, d_sorted, d_uniq, d_counts, d_nruns, d_tmp, tmp_bytes, s);
        case 2: return sort_rle<uint16_t>(d_in, n, d_sorted, d_uniq, d_counts, d_nruns, d_tmp, tmp_bytes, s);
        case 4: return sort_rle<uint32_t>(d_in, n, d_sorted, d_uniq, d_counts, d_nruns, d_tmp, tmp_bytes, s);
        case 8: return sort_rle<uint64_t>(d_in, n, d_sorted, d_uniq, d_counts, d_nruns, d_tmp, tmp_bytes, s);
        case 16:
            return sort_rle<rocprim::uint128_t>(d_in, n, d_sorted, d_uniq, d_counts, d_nruns, d_tmp, tmp_bytes, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace huff::dev
