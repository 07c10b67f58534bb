// Development probe: VALU issue rate per SIMD against waves per SIMD and
// independent chains per wave (does a second wave double the plain-VALU rate?).
// hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/probe/valu_rate.hip -o tools/probe/valu_rate && ./tools/probe/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));
// KIND 3: packed fp32 chains (v_pk_fma_f32: two fmas per lane per instruction)
template <int CH>
__global__ void __launch_bounds__(64) pk_chains(float* out, int iters, float a, float b) {
    f32x2 x[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = f32x2{threadIdx.x * 1e-3f + c, threadIdx.x * 2e-3f + c};
    const f32x2 a2 = {a, a}, b2 = {b, b};
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = __builtin_elementwise_fma(x[c], a2, b2);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c].x + x[c].y;
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int CH, int KIND>
__global__ void __launch_bounds__(64) chains(float* out, int iters, float a, float b) {
    float x[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            if (KIND == 0) x[c] = __builtin_fmaf(x[c], a, b);                       // plain fma
            else if (KIND == 1) x[c] = __builtin_amdgcn_exp2f(x[c]) * a;             // trans + mul
            else x[c] = __builtin_fmaf(x[c], a, b) * __builtin_amdgcn_rcpf(x[c] + b); // mix
        }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int CH, int KIND>
void run(float* out, int waves_per_simd, int per_instr) {
    const int cus = 256, blocks = cus * 4 * waves_per_simd, iters = 4096;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto k = KIND == 3 ? (void (*)(float*, int, float, float))pk_chains<CH> : chains<CH, KIND>;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, out, 16, 0.999f, 1e-3f);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, out, iters, 0.999f, 1e-3f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions per SIMD per cycle at 2.4 GHz
    const double insts = (double)blocks * iters * CH * per_instr;
    const double per_simd_cycle = insts / (cus * 4) / (ms * 1e-3 * 2.4e9);
    printf("kind %d chains %2d waves/SIMD %d: %.3f ms, %.2f cycles per wave-instruction per SIMD\n", KIND, CH,
           waves_per_simd, ms, 1.0 / per_simd_cycle);
}

int main() {
    float* out;
    hipMalloc(&out, 256 * 4 * 8 * 64 * sizeof(float));
    for (int w : {1, 2, 3, 4, 6, 8}) run<1, 0>(out, w, 1);
    for (int w : {1, 2, 4, 8}) run<8, 0>(out, w, 1);
    for (int w : {1, 2, 4, 8}) run<8, 1>(out, w, 2);
    for (int w : {1, 2, 4, 8}) run<8, 2>(out, w, 4);
    for (int w : {1, 2, 4, 8}) run<8, 3>(out, w, 1);  // (wave-instructions: one v_pk_fma_f32 = 2 fmas per lane)
    for (int w : {1, 2, 4, 8}) run<16, 0>(out, w, 1);
    hipFree(out);
    return 0;
}
