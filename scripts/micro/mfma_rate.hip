// Micro-benchmark: issue rate of v_mfma_f32_16x16x16_bf16 vs v_mfma_f32_16x16x32_bf16 vs
// v_mfma_f32_32x32x16_bf16 (one wave per SIMD, 4 independent accumulators, operands in registers).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
constexpr int N = 4096;
__global__ __launch_bounds__(256) void k16(float* out, float seed) {
    s4 a = {(short)threadIdx.x, 1, 2, (short)(seed)}, b = a;
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < N; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
__global__ __launch_bounds__(256) void k32(float* out, float seed) {
    b8 a; for (int j = 0; j < 8; ++j) a[j] = (__bf16)(seed + j + threadIdx.x);
    b8 b = a;
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < N; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
__global__ __launch_bounds__(256) void kf32(float* out, float seed) {
    float a = seed + threadIdx.x, b = a;
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < N; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
__global__ __launch_bounds__(256) void kexp(float* out, float seed) {
    float x0 = seed + threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    for (int i = 0; i < N; ++i) {
        x0 = __builtin_amdgcn_exp2f(x0) * 0.5f; x1 = __builtin_amdgcn_exp2f(x1) * 0.5f;
        x2 = __builtin_amdgcn_exp2f(x2) * 0.5f; x3 = __builtin_amdgcn_exp2f(x3) * 0.5f;
    }
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3;
}
int main() {
    float* out; hipMalloc(&out, 256 * 256 * 4 * 8);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const char* names[] = {"16x16x16bf16", "16x16x32bf16", "16x16x4f32", "exp2+mul (4 chains)"};
    for (int k = 0; k < 4; ++k) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (k == 0) hipLaunchKernelGGL(k16, dim3(256), dim3(256), 0, 0, out, 1.f);
            if (k == 1) hipLaunchKernelGGL(k32, dim3(256), dim3(256), 0, 0, out, 1.f);
            if (k == 2) hipLaunchKernelGGL(kf32, dim3(256), dim3(256), 0, 0, out, 1.f);
            if (k == 3) hipLaunchKernelGGL(kexp, dim3(256), dim3(256), 0, 0, out, 1.f);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            // 256 workgroups x 4 waves = one wave per SIMD; 4*N instructions per wave
            double cyc = ms * 1e-3 * 2.4e9 / (4.0 * N);
            if (rep) printf("%-22s %.3f ms  -> %.2f cycles/instr per SIMD at 2.4 GHz\n", names[k], ms, cyc);
        }
    }
    return 0;
}
