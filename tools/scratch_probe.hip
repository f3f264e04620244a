// scratch_probe.hip — does private (scratch) memory survive in co-resident
// workgroups? Each lane fills a dynamically indexed private array (so it
// lives in scratch) with a pattern unique to (workgroup, wave, lane, slot),
// spins for a while so other workgroups on the CU run, then reads it back
// and counts mismatches. Launch shapes mirror k_decode_fixed: 256-thread
// workgroups, dynamic LDS, a grid of 1..4 workgroups per CU.
//   hipcc --offload-arch=gfx950 -O3 tools/scratch_probe.hip -o tools/scratch_probe
//   tools/scratch_probe            (prints one JSON line per configuration)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

constexpr int kSlots = 48;

template <int MODE>
__device__ __forceinline__ void body(unsigned* bad, unsigned* first, unsigned spin, unsigned idx_seed) {
    extern __shared__ unsigned lds[];
    volatile unsigned priv[kSlots];
    const unsigned tag = (blockIdx.x << 12) | threadIdx.x;
    for (int i = 0; i < kSlots; ++i) priv[(i * 7 + idx_seed) % kSlots] = tag * 2654435761u + i;
    lds[threadIdx.x] = tag;
    unsigned acc = 0;
    for (unsigned s = 0; s < spin; ++s) acc += lds[(threadIdx.x + s) & 255] * s;
    unsigned nbad = 0;
    for (int i = 0; i < kSlots; ++i) nbad += priv[(i * 7 + idx_seed) % kSlots] != tag * 2654435761u + i;
    if (nbad) {
        if (atomicAdd(bad, nbad) == 0) first[0] = blockIdx.x, first[1] = threadIdx.x;
    }
    if (acc == 0xFFFFFFFFu) bad[1] = acc;  // keep the spin
}

__global__ __launch_bounds__(256) void k_probe(unsigned* bad, unsigned* first, unsigned spin, unsigned seed) {
    body<0>(bad, first, spin, seed);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) void k_probe5(unsigned* bad, unsigned* first,
                                                                                          unsigned spin, unsigned seed) {
    body<1>(bad, first, spin, seed);
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned *bad, *first;
    CHECK(hipMalloc(&bad, 16));
    CHECK(hipMalloc(&first, 16));
    const size_t lds = 26 * 1024;
    for (int k = 0; k < 2; ++k) {
        auto kern = k ? k_probe5 : k_probe;
        int per_cu = 0;
        CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds));
        for (int wgs_per_cu = 1; wgs_per_cu <= 4; ++wgs_per_cu) {
            const unsigned grid = static_cast<unsigned>(cus * wgs_per_cu);
            unsigned h[2] = {0, 0}, f[2] = {0, 0};
            CHECK(hipMemset(bad, 0, 16));
            CHECK(hipMemset(first, 0, 16));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, bad, first, 20000u, 5u);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(h, bad, 8, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(f, first, 8, hipMemcpyDeviceToHost));
            std::printf("{\"kernel\": \"%s\", \"occupancy_per_cu\": %d, \"grid\": %u, \"bad_slots\": %u, "
                        "\"first_wg\": %u, \"first_thread\": %u}\n",
                        k ? "probe_waves5" : "probe", per_cu, grid, h[0], f[0], f[1]);
        }
    }
    return 0;
}
