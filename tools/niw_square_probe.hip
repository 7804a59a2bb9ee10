// Development probe: shader cycles of np8_niw_post's bound squaring (sym_square_mfma, D = 64) on one CU, the
// function as the kernel file defines it (included), on an LDS matrix, with and without a barrier per call.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I noparama_amd/csrc tools/niw_square_probe.hip
//        -o tools/niw_square_probe
#include "../noparama_amd/csrc/np8_niw.hip"

// candidate: compile-time steps, every operand loaded before the first MFMA, no masking (D a multiple of 16)
template <int NS>
__device__ __forceinline__ void sq2(int D, int LD, const double *X, double *Y) {
    const int nt = D / 16, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int il = lane & 15, kl = lane >> 4;
    for (int tt = wv; tt < nt * (nt + 1) / 2; tt += 4) {
        int ti = 0, rem = tt;
        while (rem >= nt - ti) {
            rem -= nt - ti;
            ++ti;
        }
        const int tj = ti + rem;
        double av[NS], bv[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            av[q] = X[(16 * ti + il) * LD + 4 * q + kl];
            bv[q] = X[(4 * q + kl) * LD + 16 * tj + il];
        }
        f64x4 c = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < NS; ++q) c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q], bv[q], c, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int a = 16 * ti + (lane >> 4) + 4 * r, b = 16 * tj + (lane & 15);
            Y[a * LD + b] = c[r];
            Y[b * LD + a] = c[r];
        }
    }
}

__global__ __launch_bounds__(256) void probe(double *out, long long *cyc, int D) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int LD = D + 1;
    double *X = sm, *Y = X + D * LD, *Z = Y + D * LD;
    for (int e = threadIdx.x; e < D * LD; e += blockDim.x) X[e] = 1.0 / (1.0 + (e % 7));
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < 8; ++r) {
        sym_square_mfma<true>(D, LD, (r & 1) ? Y : X, (r & 1) ? Z : Y);
        __syncthreads();
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < 8; ++r) {
        sym_square(D, LD, (r & 1) ? Y : X, (r & 1) ? Z : Y);
        __syncthreads();
    }
    long long t2 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < 8; ++r) __syncthreads();
    long long t3 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < 8; ++r) {
        sq2<16>(D, LD, (r & 1) ? Y : X, (r & 1) ? Z : Y);
        __syncthreads();
    }
    long long t4 = __builtin_amdgcn_s_memtime();
    // one panel factor (wave 0) and one forward-substitution panel (wave 1) on a diagonally dominant matrix
    for (int e = threadIdx.x; e < D * LD; e += blockDim.x) {
        const int r = e / LD, c = e - r * LD;
        X[e] = (r == c) ? 100.0 + r : 1.0 / (1.0 + r + c);
        Y[e] = 0.0;
    }
    __shared__ int skip;
    __syncthreads();
    long long t5 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x >> 6) == 0) lower_panel_factor(X, LD, D, 0, &skip);
    __syncthreads();
    long long t6 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x >> 6) == 1) forward_panel(Y, X, LD, D, 16, true);
    __syncthreads();
    long long t7 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = t2 - t1;
        cyc[2] = t3 - t2;
        cyc[3] = t4 - t3;
        cyc[4] = t6 - t5;
        cyc[5] = t7 - t6;
    }
    out[threadIdx.x] = Z[threadIdx.x];
}

int main() {
    double *out;
    long long *cyc;
    (void)hipMallocManaged(&out, sizeof(double) * 256);
    (void)hipMallocManaged(&cyc, sizeof(long long) * 8);
    const int D = 64;
    const size_t lds = sizeof(double) * 3 * D * (D + 1);
    for (int it = 0; it < 2; ++it) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(256), lds, 0, out, cyc, D);
        (void)hipDeviceSynchronize();
    }
    printf("sym_square_mfma: %.0f cycles per call; sym_square (VALU): %.0f; barrier alone: %.0f; straight-line: %.0f\n",
           cyc[0] / 8.0, cyc[1] / 8.0, cyc[2] / 8.0, cyc[3] / 8.0);
    printf("lower_panel_factor: %lld cycles per 16-column panel; forward_panel: %lld\n", cyc[4], cyc[5]);
    return 0;
}
