// fp64 MFMA peak probe: every wave issues CH independent v_mfma_f64_16x16x4_f64
// chains from registers (no memory traffic); flops = 2*16*16*4 per MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ void __launch_bounds__(256) k_peak(int iters, double *out) {
    d4 acc[CH];
    for (int i = 0; i < CH; ++i) acc[i] = d4{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < CH; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.0) out[0] = s;
}

template <int CH>
static void run(double *d, hipEvent_t a, hipEvent_t b) {
    const int iters = 80000 / CH;
    for (int blocks : {256 * 2, 256 * 4, 256 * 8}) {
        k_peak<CH><<<blocks, 256>>>(iters, d);
        (void)hipEventRecord(a);
        k_peak<CH><<<blocks, 256>>>(iters, d);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        double flops = 2.0 * 16 * 16 * 4 * (double)CH * iters * (blocks * 4.0);
        printf("chains=%d blocks=%d ms=%.3f fp64 MFMA %.2f TFLOP/s\n", CH, blocks, ms,
               flops / (ms * 1e-3) / 1e12);
    }
}

int main() {
    double *d;
    (void)hipMalloc(&d, 8);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    run<2>(d, a, b);
    run<4>(d, a, b);
    run<8>(d, a, b);
    run<16>(d, a, b);
    return 0;
}
