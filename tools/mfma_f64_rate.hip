// Development micro-benchmark: cycles per v_mfma_f64_16x16x4_f64 on one CU (4 waves, one per SIMD), one dependent
// accumulator chain per wave and four independent ones (s_memtime, the shader clock).  np8_niw_post's dense products
// run on this instruction.  Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_rate.hip -o tools/mfma_f64_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kSteps = 1024;

template <int CH>
__global__ void k(double *out, long long *cyc, double a0) {
    const int lane = threadIdx.x & 63;
    double a = a0 + lane * 1e-3, b = a0 - lane * 1e-3;
    f64x4 acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = (f64x4){0.0, 0.0, 0.0, 0.0};
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < kSteps; ++s)
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    double v = 0.0;
#pragma unroll
    for (int c = 0; c < CH; ++c) v += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = v;
    if (lane == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

template <int CH>
void run(double *out, long long *cyc) {
    hipLaunchKernelGGL(k<CH>, dim3(1), dim3(256), 0, 0, out, cyc, 1.0);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k<CH>, dim3(1), dim3(256), 0, 0, out, cyc, 1.0);
    hipDeviceSynchronize();
    printf("chains %d: %.1f cycles per MFMA per wave (wave 0: %lld cycles for %d)\n", CH,
           (double)cyc[0] / (kSteps * CH), cyc[0], kSteps * CH);
}

int main() {
    double *out;
    long long *cyc;
    hipMallocManaged(&out, sizeof(double) * 256);
    hipMallocManaged(&cyc, sizeof(long long) * 4);
    run<1>(out, cyc);
    run<2>(out, cyc);
    run<4>(out, cyc);
    return 0;
}
