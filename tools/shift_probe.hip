// shift_probe.hip — does a v_lshrrev_b64 whose shift count comes from the
// v_sub_u32 right before it ever compute a wrong result on gfx950 when many
// waves share a SIMD? Every thread runs a chain like the decoder's refill
// (count X -= entry read from LDS; window |= (w << 32) >> X), once through
// the 64-bit shift and once through 32-bit ops only, and counts differences.
//   hipcc --offload-arch=gfx950 -O3 -o tools/shift_probe tools/shift_probe.hip
//   tools/shift_probe [workgroups_per_cu] [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

__global__ __launch_bounds__(256) void k_probe(uint32_t iters, uint32_t* bad, uint32_t* first) {
    __shared__ uint16_t tab[4096];
    for (uint32_t i = threadIdx.x; i < 4096; i += 256) tab[i] = static_cast<uint16_t>((i * 2654435761u >> 16) & 0x3F1F);
    __syncthreads();
    uint32_t s = blockIdx.x * 256 + threadIdx.x;
    uint32_t w = s * 0x9E3779B9u + 1;
    uint32_t X = 40 + (s & 15);
    uint64_t acc = 0;
    uint32_t acc_hi = 0, acc_lo = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t e = tab[(w >> 20) & 4095];
        uint32_t Xn;
        uint64_t r;
        // the decoder's pair: count from a 32-bit subtraction, used at once as the 64-bit shift count
        asm volatile("v_sub_u32 %0, %2, %3\n\tv_lshrrev_b64 %1, %0, %4"
                     : "=&v"(Xn), "=&v"(r)
                     : "v"(X), "v"(e), "v"(static_cast<uint64_t>(w) << 32));
        acc ^= r;
        // the same with 32-bit operations only
        const uint32_t c = Xn & 63;
        const uint32_t hi = c >= 32 ? 0u : (w >> c);
        const uint32_t lo = c == 0 ? 0u : (c <= 32 ? (w << (32 - c)) : (w >> (c - 32)));
        acc_hi ^= hi;
        acc_lo ^= lo;
        X = (Xn & 63) | 32;
        w = w * 1664525u + 1013904223u;
    }
    if (static_cast<uint32_t>(acc >> 32) != acc_hi || static_cast<uint32_t>(acc) != acc_lo) {
        if (atomicAdd(bad, 1u) == 0) *first = s;
    }
}

int main(int argc, char** argv) {
    const int per_cu = argc > 1 ? atoi(argv[1]) : 8;
    const uint32_t iters = argc > 2 ? static_cast<uint32_t>(atoi(argv[2])) : 200000;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 2;
    uint32_t *d, h[2] = {0, 0};
    if (hipMalloc(&d, 8) != hipSuccess) return 2;
    for (int rep = 0; rep < 3; ++rep) {
        hipMemset(d, 0, 8);
        const int grid = p.multiProcessorCount * per_cu * 4;  // several dispatch waves of workgroups
        hipLaunchKernelGGL(k_probe, dim3(grid), dim3(256), 0, 0, iters, d, d + 1);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
        printf("{\"rep\": %d, \"workgroups\": %d, \"iters\": %u, \"threads_wrong\": %u, \"first\": %u}\n", rep, grid, iters, h[0], h[1]);
    }
    hipFree(d);
    return 0;
}
