// shift_probe.hip — does a v_lshrrev_b64 whose shift count comes from the
// v_sub_u32 right before it ever compute a wrong result on gfx950 when many
// waves share a SIMD? Every thread runs a chain like the decoder's refill
// (count X -= entry read from LDS; window |= (w << 32) >> X), once through
// the 64-bit shift and once through 32-bit ops only, and counts differences.
//   hipcc --offload-arch=gfx950 -O3 -o tools/shift_probe tools/shift_probe.hip
//   tools/shift_probe [workgroups_per_cu] [iters] [variant: 1 = the pair, 2 = the refill window]
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

// variant 2: the failing refill's own instruction window, registers pinned as
// in the reproducer: the shift source pair's high half is an LDS return, its
// low half a v_mov of zero, and a 64-bit shift of the window precedes it
__global__ __launch_bounds__(256) void k_probe2(uint32_t iters, uint32_t* bad, uint32_t* first) {
    __shared__ uint32_t words[4096];
    __shared__ uint16_t tab[4096];
    for (uint32_t i = threadIdx.x; i < 4096; i += 256) {
        words[i] = i * 0x9E3779B9u + 0x7F4A7C15u;
        tab[i] = static_cast<uint16_t>(((i * 2654435761u >> 16) & 0x3F00) | (1 + (i % 12)));
    }
    __syncthreads();
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    uint32_t X = 40 + (s & 15);
    uint64_t buf = static_cast<uint64_t>(s) * 0x9E3779B97F4A7C15ull;
    uint32_t wrong = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t k = (s * 7 + it * 13) & 4095;
        const uint32_t e1 = tab[(static_cast<uint32_t>(buf >> 52))];
        const uint32_t e2 = tab[(static_cast<uint32_t>(buf >> 40)) & 4095];
        const uint32_t addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
            (__attribute__((address_space(3))) uint32_t*)(&words[k])));
        uint32_t Xo = X, lo, hi, t;
        uint64_t b = buf;
        asm volatile(
            "ds_read_b32 v41, %[addr]\n\t"
            "v_or_b32 %[X], 32, %[X]\n\t"
            "v_mov_b32 v40, 0\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"
            "v_add_u32 %[t], %[e1], %[e2]\n\t"
            "v_sub_u32 %[X], %[X], %[t]\n\t"
            "v_lshlrev_b64 %[b], %[e2], %[b]\n\t"
            "v_lshrrev_b64 v[40:41], %[X], v[40:41]\n\t"
            "v_mov_b32 %[lo], v40\n\t"
            "v_mov_b32 %[hi], v41"
            : [X] "+v"(Xo), [t] "=&v"(t), [b] "+v"(b), [lo] "=&v"(lo), [hi] "=&v"(hi)
            : [addr] "v"(addr), [e1] "v"(e1), [e2] "v"(e2)
            : "v40", "v41", "memory");
        // expected, from 32-bit operations
        const uint32_t w = words[k];
        const uint32_t c = ((X | 32) - (e1 + e2)) & 63;
        const uint32_t ehi = c >= 32 ? 0u : (w >> c);
        const uint32_t elo = c == 0 ? 0u : (c <= 32 ? (w << (32 - c)) : (w >> (c - 32)));
        if (ehi != hi || elo != lo) ++wrong;
        buf = b ^ (static_cast<uint64_t>(hi) << 17) ^ lo;
        X = (Xo & 63) | 32;
    }
    if (wrong && atomicAdd(bad, 1u) == 0) *first = s;
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
        if (argc > 3 && atoi(argv[3]) == 2)
            hipLaunchKernelGGL(k_probe2, dim3(grid), dim3(256), 0, 0, iters, d, d + 1);
        else
            hipLaunchKernelGGL(k_probe, dim3(grid), dim3(256), 0, 0, iters, d, d + 1);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
        printf("{\"variant\": %d, \"rep\": %d, \"workgroups\": %d, \"iters\": %u, \"threads_wrong\": %u, \"first\": %u}\n", argc > 3 ? atoi(argv[3]) : 1, rep, grid, iters, h[0], h[1]);
    }
    hipFree(d);
    return 0;
}
