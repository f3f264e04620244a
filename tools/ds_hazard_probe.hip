// ds_hazard_probe.hip — is a VGPR that an issued DS write still has to read
// safe from a later VMEM load that overwrites it?
//
// The spilling builds of k_decode_fixed (HUFF_DEC_VARIANT 12-14) place a
// scratch reload into the address or data VGPR of the ds_write_b128 issued
// just before it (`ds_write_b128 v20, v[12:15]; scratch_load_dword v12, ...`)
// and decode wrong letters only when other workgroups share the CU. This
// probe issues exactly that pair in inline asm, under LDS contention from
// co-resident workgroups, and checks what landed in LDS:
//   mode 0: the load overwrites the DS write's ADDRESS register
//   mode 1: the load overwrites the first DATA register
//   mode 2: control — the load goes to an unrelated register
// Each lane writes 16 B at its own slot; the loaded dword is a marker that
// must never appear in LDS.
//   hipcc --offload-arch=gfx950 -O3 tools/ds_hazard_probe.hip -o tools/ds_hazard_probe
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

constexpr unsigned kMarker = 0xDEADBEEFu;

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(const unsigned* marker, unsigned* bad, unsigned rounds) {
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const unsigned t = threadIdx.x;
    const unsigned base = t * 16;            // byte address of this lane's slot
    unsigned nbad = 0;
    for (unsigned r = 0; r < rounds; ++r) {
        const unsigned v0 = (blockIdx.x << 16) ^ (t << 4) ^ r;
        if (MODE == 0) {  // address register v44 reloaded right after the write
            unsigned addr = 0;
            asm volatile(
                "v_mov_b32 v44, %1\n\t"
                "v_mov_b32 v40, %2\n\tv_mov_b32 v41, %3\n\tv_mov_b32 v42, %4\n\tv_mov_b32 v43, %5\n\t"
                "s_nop 4\n\t"
                "ds_write_b128 v44, v[40:43]\n\t"
                "global_load_dword v44, %6, off\n\t"
                "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
                "v_mov_b32 %0, v44"
                : "=v"(addr)
                : "v"(base), "v"(v0), "v"(v0 + 1), "v"(v0 + 2), "v"(v0 + 3), "v"(marker)
                : "v40", "v41", "v42", "v43", "v44", "memory");
            nbad += addr != kMarker;  // the load itself must have landed
        } else if (MODE == 1) {  // first data register v40 reloaded right after the write
            asm volatile(
                "v_mov_b32 v44, %0\n\t"
                "v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v42, %3\n\tv_mov_b32 v43, %4\n\t"
                "s_nop 4\n\t"
                "ds_write_b128 v44, v[40:43]\n\t"
                "global_load_dword v40, %5, off\n\t"
                "s_waitcnt vmcnt(0) lgkmcnt(0)"
                :
                : "v"(base), "v"(v0), "v"(v0 + 1), "v"(v0 + 2), "v"(v0 + 3), "v"(marker)
                : "v40", "v41", "v42", "v43", "v44", "memory");
        } else {  // control: the load goes to v45
            asm volatile(
                "v_mov_b32 v44, %0\n\t"
                "v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v42, %3\n\tv_mov_b32 v43, %4\n\t"
                "s_nop 4\n\t"
                "ds_write_b128 v44, v[40:43]\n\t"
                "global_load_dword v45, %5, off\n\t"
                "s_waitcnt vmcnt(0) lgkmcnt(0)"
                :
                : "v"(base), "v"(v0), "v"(v0 + 1), "v"(v0 + 2), "v"(v0 + 3), "v"(marker)
                : "v40", "v41", "v42", "v43", "v44", "v45", "memory");
        }
        // contention: every lane reads other lanes' slots
        const uint4 got = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(lds) + base);
        nbad += got.x != v0 || got.y != v0 + 1 || got.z != v0 + 2 || got.w != v0 + 3;
        unsigned acc = 0;
        for (int k = 0; k < 8; ++k) acc += lds[(t * 7 + k * 61 + r) & 1023];
        if (acc == kMarker) nbad += 1000000;  // never (keeps the reads)
        __builtin_amdgcn_s_barrier();
    }
    if (nbad) atomicAdd(bad, nbad);
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned *marker, *bad;
    CHECK(hipMalloc(&marker, 64));
    CHECK(hipMalloc(&bad, 16));
    const unsigned m = kMarker;
    CHECK(hipMemcpy(marker, &m, 4, hipMemcpyHostToDevice));
    const size_t lds = 26 * 1024;
    for (int mode = 0; mode < 3; ++mode) {
        auto kern = mode == 0 ? k_probe<0> : mode == 1 ? k_probe<1> : k_probe<2>;
        for (int per_cu = 1; per_cu <= 5; per_cu += 2) {
            const unsigned grid = static_cast<unsigned>(cus * per_cu);
            unsigned h = 0;
            CHECK(hipMemset(bad, 0, 16));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, marker, bad, 2000u);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
            std::printf("{\"mode\": %d, \"wgs_per_cu\": %d, \"grid\": %u, \"rounds\": 2000, \"bad\": %u}\n", mode,
                        per_cu, grid, h);
        }
    }
    return 0;
}
