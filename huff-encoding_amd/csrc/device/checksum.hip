// checksum.hip — letter checksums of the decoder's self-checking build
// (HUFF_DEC_VARIANT=11).
//
// The check build compares every lane's end bit with its successor's restart
// point, which sees a lane that lost its place in the stream. It cannot see a
// wrong letter whose code has the right length: the stream stays in step. So
// when the check build encodes a job, it also records per decode task of
// kTaskSym letters
//     s1 = sum of the letters, s2 = sum of (i + 1) * letter_i    (mod 2^32,
//     i = the letter's index in the task),
// and after decoding it recomputes both over the output: a wrong letter
// changes s1, two letters swapped change s2. Test builds only: one more read of
// the input at encode and of the output at decode.
#include "kernels.hpp"

namespace huff::dev {

namespace {

constexpr uint32_t kThreads = 256;  // 4 tasks per workgroup, one wave each

// the wave's sums over task `task` of x[0, n): lane l takes letters
// [64 l, 64 l + 64) of the task (16-B loads when the task is whole and x is
// 16-B aligned, bytes otherwise; letters past n count as 0 on both sides)
__device__ uint64_t task_sums(const uint8_t* __restrict__ x, uint64_t n, uint64_t task) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t l0 = task * kTaskSym + 64ull * lane;
    uint32_t s1 = 0, s2 = 0;
    const bool whole = (task + 1) * kTaskSym <= n && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        uint32_t w[4];
        if (whole) {
            const uint4 v = *reinterpret_cast<const uint4*>(x + l0 + 16 * q);
            w[0] = v.x;
            w[1] = v.y;
            w[2] = v.z;
            w[3] = v.w;
        } else {
#pragma unroll
            for (uint32_t d = 0; d < 4; ++d) {
                w[d] = 0;
                for (uint32_t b = 0; b < 4; ++b) {
                    const uint64_t i = l0 + 16 * q + 4 * d + b;
                    if (i < n) w[d] |= static_cast<uint32_t>(x[i]) << (8 * b);
                }
            }
        }
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
            // letters 4 k .. 4 k + 3 of the lane (k = 4 q + d): weights
            // 64 lane + 4 k + (1, 2, 3, 4)
            const uint32_t sd = __builtin_amdgcn_udot4(w[d], 0x01010101u, 0u, false);
            const uint32_t td = __builtin_amdgcn_udot4(w[d], 0x04030201u, 0u, false);
            s1 += sd;
            s2 += (64u * lane + 4u * (4 * q + d)) * sd + td;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        s1 += static_cast<uint32_t>(__shfl_xor(static_cast<int>(s1), o));
        s2 += static_cast<uint32_t>(__shfl_xor(static_cast<int>(s2), o));
    }
    return (static_cast<uint64_t>(s2) << 32) | s1;
}

__global__ __launch_bounds__(kThreads) void k_task_sums(const uint8_t* __restrict__ x, uint64_t n,
                                                        uint64_t* __restrict__ sums) {
    const uint64_t ntasks = (n + kTaskSym - 1) / kTaskSym;
    const uint64_t task = static_cast<uint64_t>(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6);
    if (task >= ntasks) return;  // wave-uniform
    const uint64_t s = task_sums(x, n, task);
    if ((threadIdx.x & 63) == 0) sums[task] = s;
}

// err[0] = tasks whose sums differ, err[1] = the first of them (atomic min)
__global__ __launch_bounds__(kThreads) void k_task_sums_check(const uint8_t* __restrict__ x, uint64_t n,
                                                              const uint64_t* __restrict__ sums,
                                                              unsigned int* __restrict__ err) {
    const uint64_t ntasks = (n + kTaskSym - 1) / kTaskSym;
    const uint64_t task = static_cast<uint64_t>(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6);
    if (task >= ntasks) return;
    const uint64_t s = task_sums(x, n, task);
    if ((threadIdx.x & 63) == 0 && s != sums[task]) {
        atomicAdd(err, 1u);
        atomicMin(err + 1, static_cast<unsigned int>(task < 0xFFFFFFFFull ? task : 0xFFFFFFFFull));
    }
}

uint32_t sum_blocks(uint64_t n) {
    const uint64_t ntasks = (n + kTaskSym - 1) / kTaskSym;
    return static_cast<uint32_t>((ntasks + kThreads / 64 - 1) / (kThreads / 64));
}

}  // namespace

hipError_t launch_task_sums(const uint8_t* x, uint64_t n, uint64_t* sums, hipStream_t s) {
    if (n == 0) return hipSuccess;
    launch_k(k_task_sums, dim3(sum_blocks(n)), dim3(kThreads), 0, s, x, n, sums);
    return hipGetLastError();
}

hipError_t launch_task_sums_check(const uint8_t* x, uint64_t n, const uint64_t* sums, unsigned int* err,
                                  hipStream_t s) {
    if (n == 0) return hipSuccess;
    launch_k(k_task_sums_check, dim3(sum_blocks(n)), dim3(kThreads), 0, s, x, n, sums, err);
    return hipGetLastError();
}

}  // namespace huff::dev
