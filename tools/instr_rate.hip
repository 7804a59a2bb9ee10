// Development micro-benchmark: issue rate of the instruction classes the assign kernel spends its
// time on (cycles per wave-instruction with 8 independent chains, 8 waves per SIMD).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kIters = 4096;

__global__ void k_fma(double *out, double a) {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = fma(x[i], a, 0.5);
    double s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad64(uint64_t *out, uint32_t a) {
    uint64_t x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = (uint64_t)a * (uint32_t)x[i] + (x[i] >> 32);
    uint64_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint32_t *out, uint32_t a) {
    uint32_t x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = x[i] * a;
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_xor(uint32_t *out, uint32_t a) {
    uint32_t x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = (x[i] ^ a) + 0x9E3779B9u;  // xor + add
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_div(double *out, double a) {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i + 1.0;
    for (int it = 0; it < kIters / 8; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = a / x[i] + 1.0;
    double s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_sqrt(double *out, double a) {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i + 1.0;
    for (int it = 0; it < kIters / 8; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = sqrt(x[i]) + a;
    double s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma32(float *out, float a) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = fmaf(x[i], a, 0.5f);
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ void k_pkfma(float *out, float a) {  // v_pk_fma_f32: two fp32 fmas per lane per instruction
    f32x2 x[8];
    for (int i = 0; i < 8; ++i) x[i] = (f32x2){(float)threadIdx.x + i, (float)threadIdx.x - i};
    const f32x2 av = {a, a}, h = {0.5f, 0.25f};
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], av, h);
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define RUN(name, kern, T, arg, ops)                                                                  \
    {                                                                                               \
        T *out;                                                                                     \
        hipMalloc(&out, sizeof(T) * blocks * 256);                                                  \
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, arg);                          \
        hipDeviceSynchronize();                                                                     \
        hipEventRecord(a);                                                                          \
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, arg);                          \
        hipEventRecord(b);                                                                          \
        hipEventSynchronize(b);                                                                     \
        float ms;                                                                                   \
        hipEventElapsedTime(&ms, a, b);                                                             \
        const double cyc = ms * 1e-3 * 2.4e9;                                                       \
        printf("%-8s %.3f ms  cycles per wave-instruction per SIMD: %.2f\n", name, ms,              \
               cyc / (blocks * 4.0 / 1024.0 * (ops)));                                              \
        hipFree(out);                                                                               \
    }

int main() {
    const int blocks = 256 * 8;  // 8 workgroups of 256 threads per CU: 8 waves per SIMD
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    RUN("fma_f64", k_fma, double, 1.0000001, 8.0 * kIters);
    RUN("fma_f32", k_fma32, float, 1.0000001f, 8.0 * kIters);
    RUN("pkfma_f32", k_pkfma, float, 1.0000001f, 8.0 * kIters);
    RUN("mad_u64", k_mad64, uint64_t, 0xD2511F53u, 8.0 * kIters);
    RUN("mul_lo", k_mullo, uint32_t, 0xD2511F53u, 8.0 * kIters);
    RUN("xor+add", k_xor, uint32_t, 0xD2511F53u, 16.0 * kIters);
    RUN("div_f64", k_div, double, 3.0, 8.0 * kIters / 8);
    RUN("sqrt_f64", k_sqrt, double, 3.0, 8.0 * kIters / 8);
    return 0;
}
