// store_war_probe.hip — is a VMEM store's data VGPR safe from a VALU write
// issued right after the store?
//
// The spilling builds of k_decode_fixed (HUFF_DEC_VARIANT 12-14) store a
// spilled VGPR and overwrite it with the next value on the very next
// instruction (`scratch_store_dword off, v4, off offset:64` then
// `v_add_u32 v4, s33, v5`). LLVM models a write-after-read hazard only for
// stores of more than 64 bits. This probe issues that pair for scratch and
// global stores, under co-resident workgroups, and reads the stored dword
// back:
//   mode 0: scratch_store_dword vD ; v_mov_b32 vD, other
//   mode 1: global_store_dword  vD ; v_mov_b32 vD, other
//   mode 2: control (s_nop 4 between the store and the overwrite)
//   hipcc --offload-arch=gfx950 -O3 tools/store_war_probe.hip -o tools/store_war_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

typedef __attribute__((address_space(5))) unsigned priv_u32;

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(unsigned* gbuf, unsigned* bad, unsigned rounds) {
    extern __shared__ unsigned lds[];
    volatile unsigned priv[16];
    priv[threadIdx.x & 15] = 0;
    unsigned nbad = 0;
    unsigned* gslot = gbuf + (blockIdx.x * 256 + threadIdx.x);
    for (unsigned r = 0; r < rounds; ++r) {
        const unsigned want = (blockIdx.x << 20) ^ (threadIdx.x << 8) ^ r;
        const unsigned other = ~want;
        unsigned d = want;
        if (MODE == 0) {
            priv_u32* p = (priv_u32*)(&priv[r & 15]);
            asm volatile(
                "scratch_store_dword %1, %0, off\n\t"
                "v_mov_b32 %0, %2\n\t"
                "s_waitcnt vmcnt(0)"
                : "+v"(d)
                : "v"(p), "v"(other)
                : "memory");
            nbad += priv[r & 15] != want;
        } else if (MODE == 1) {
            asm volatile(
                "global_store_dword %1, %0, off\n\t"
                "v_mov_b32 %0, %2\n\t"
                "s_waitcnt vmcnt(0)"
                : "+v"(d)
                : "v"(gslot), "v"(other)
                : "memory");
            nbad += __atomic_load_n(gslot, __ATOMIC_RELAXED) != want;
        } else {
            priv_u32* p = (priv_u32*)(&priv[r & 15]);
            asm volatile(
                "scratch_store_dword %1, %0, off\n\t"
                "s_nop 4\n\t"
                "v_mov_b32 %0, %2\n\t"
                "s_waitcnt vmcnt(0)"
                : "+v"(d)
                : "v"(p), "v"(other)
                : "memory");
            nbad += priv[r & 15] != want;
        }
        // LDS traffic from the co-resident workgroups
        lds[threadIdx.x] = d;
        unsigned acc = 0;
        for (int k = 0; k < 8; ++k) acc += lds[(threadIdx.x * 7 + k * 61 + r) & 255];
        if (acc == 0x12345678u) nbad += 1000000;
        __builtin_amdgcn_s_barrier();
    }
    if (nbad) atomicAdd(bad, nbad);
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned *gbuf, *bad;
    CHECK(hipMalloc(&gbuf, size_t(cus) * 8 * 256 * 4));
    CHECK(hipMalloc(&bad, 16));
    const size_t lds = 26 * 1024;
    for (int mode = 0; mode < 3; ++mode) {
        auto kern = mode == 0 ? k_probe<0> : mode == 1 ? k_probe<1> : k_probe<2>;
        for (int per_cu = 1; per_cu <= 5; per_cu += 2) {
            const unsigned grid = static_cast<unsigned>(cus * per_cu);
            unsigned h = 0;
            CHECK(hipMemset(bad, 0, 16));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, gbuf, bad, 4000u);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
            std::printf("{\"mode\": %d, \"wgs_per_cu\": %d, \"grid\": %u, \"rounds\": 4000, \"bad\": %u}\n", mode,
                        per_cu, grid, h);
        }
    }
    return 0;
}
