// Is v_mfma_f64_16x16x4_f64 bit-for-bit a k-ordered fma chain (as the f32 form is, cdna_hip_programming.md)?
// Random operands with wide exponent spread; D = MFMA(A, B, C) against fma(a3, b3, fma(a2, b2, fma(a1, b1, fma(a0, b0, c))))
// and against a single-rounding dot product.  Prints the mismatch counts.  Build: hipcc --offload-arch=gfx950 -O2
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void k(const double *A, const double *B, const double *C, double *D, int reps) {
    const int lane = threadIdx.x;  // one wave
    for (int t = 0; t < reps; ++t) {
        // A operand: lane (row = lane & 15, k = lane >> 4); B: (col = lane & 15, k = lane >> 4); C/D: col = lane & 15,
        // rows (lane >> 4) + 4 r
        const double a = A[t * 64 + lane], b = B[t * 64 + lane];
        f64x4 c;
        for (int r = 0; r < 4; ++r) c[r] = C[t * 256 + ((lane >> 4) + 4 * r) * 16 + (lane & 15)];
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
        for (int r = 0; r < 4; ++r) D[t * 256 + ((lane >> 4) + 4 * r) * 16 + (lane & 15)] = c[r];
    }
}

int main() {
    const int reps = 4096;
    double *A, *B, *C, *D;
    hipMallocManaged(&A, sizeof(double) * 64 * reps);
    hipMallocManaged(&B, sizeof(double) * 64 * reps);
    hipMallocManaged(&C, sizeof(double) * 256 * reps);
    hipMallocManaged(&D, sizeof(double) * 256 * reps);
    srand(7);
    auto rnd = [] { return ((double)rand() / RAND_MAX - 0.5) * std::ldexp(1.0, rand() % 40 - 20); };
    for (int i = 0; i < 64 * reps; ++i) A[i] = rnd(), B[i] = rnd();
    for (int i = 0; i < 256 * reps; ++i) C[i] = rnd();
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, A, B, C, D, reps);
    hipDeviceSynchronize();
    long chain = 0, rev = 0, dot = 0, n = 0;
    for (int t = 0; t < reps; ++t)
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                // A[i][k] at lane i + 16 k, B[k][j] at lane j + 16 k
                double c = C[t * 256 + i * 16 + j], cr = c;
                for (int kk = 0; kk < 4; ++kk) c = std::fma(A[t * 64 + i + 16 * kk], B[t * 64 + j + 16 * kk], c);
                for (int kk = 3; kk >= 0; --kk) cr = std::fma(A[t * 64 + i + 16 * kk], B[t * 64 + j + 16 * kk], cr);
                long double s = C[t * 256 + i * 16 + j];
                for (int kk = 0; kk < 4; ++kk) s += (long double)A[t * 64 + i + 16 * kk] * B[t * 64 + j + 16 * kk];
                const double d = D[t * 256 + i * 16 + j];
                chain += d != c;
                rev += d != cr;
                dot += d != (double)s;
                ++n;
            }
    printf("elements %ld: differ from the k-ascending fma chain %ld, from k-descending %ld, from the long-double dot %ld\n", n,
           chain, rev, dot);
    return 0;
}
