// valu_rate.hip — issue rate of the shift forms the lane walkers use
// (tools only, not the product): 64-bit v_lshlrev_b64 against the 32-bit
// pair v_alignbit_b32 + v_lshlrev_b32, and v_add_u32 as the full-rate
// reference. Each wave runs 8 independent chains of kIters instructions;
// the grid fills every SIMD with `waves` waves. Prints cycles per
// wave-instruction per SIMD (clock from a same-run s_memtime / wall ratio is
// not needed: the ratios between forms are the result).
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate && tools/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

template <int FORM>
__global__ __launch_bounds__(256) void k_rate(unsigned* out, unsigned s) {
    unsigned a[8], b[8];
    unsigned long long q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] = threadIdx.x * 7 + k;
        b[k] = threadIdx.x * 13 + k * 3;
        q[k] = (static_cast<unsigned long long>(b[k]) << 32) | a[k];
    }
    const unsigned sh = (s + threadIdx.x) & 15;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (FORM == 0) {  // v_add_u32
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(sh));
            } else if constexpr (FORM == 1) {  // v_lshlrev_b64
                asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(q[k]) : "v"(sh));
            } else {  // v_alignbit_b32 + v_lshlrev_b32: the same 64-bit left shift in halves
                asm volatile("v_alignbit_b32 %0, %0, %1, %2\n\tv_lshlrev_b32 %1, %2, %1"
                             : "+v"(a[k]), "+v"(b[k]) : "v"(sh));
            }
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) r ^= a[k] ^ b[k] ^ static_cast<unsigned>(q[k] >> 7);
    if (r == 0x12345678u) out[threadIdx.x] = r;
}

template <int FORM>
float run(int waves_per_simd, int ninstr_per_iter) {
    unsigned* out;
    hipMalloc(&out, 4096);
    const int blocks = 256 * waves_per_simd;  // 256 CUs x 4 SIMDs x w waves = 256 w blocks of 4 waves
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_rate<FORM>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_rate<FORM>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    hipFree(out);
    // wave-instructions per SIMD: waves_per_simd waves x kIters x 8 chains x ninstr
    const double per_simd = double(waves_per_simd) * kIters * 8 * ninstr_per_iter;
    return static_cast<float>(ms * 1e-3 * 2.4e9 / per_simd);  // cycles at 2.4 GHz per wave-instruction
}

int main() {
    for (int w : {1, 2, 3, 4, 6, 8}) {
        std::printf("{\"waves_per_simd\": %d, \"cycles_per_instr_at_2.4GHz\": {\"v_add_u32\": %.2f, \"v_lshlrev_b64\": %.2f, "
                    "\"alignbit+lshl_b32 (per instr)\": %.2f}}\n",
                    w, run<0>(w, 1), run<1>(w, 1), run<2>(w, 2));
    }
    return 0;
}
