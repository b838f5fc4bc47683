// stream_probe.hip -- HBM calibration for the CG kernels' access mix.
// Standalone (no torch): hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o /tmp/sp
// Times, on n x ld fp64 arrays laid out like gs_er.hip's CG state:
//   flat3r2w : grid-stride, 16 B/lane: read A,B,C  write C,D   (k_cg_pq's own-row mix)
//   flat2r1w : read A,B write B                                 (k_cg_upd's own-row mix)
//   flatread : read A,B,C only
//   lane3r2w : the CG lane mapping (wave = one residue, 128 columns, rows j, j+32, ...)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);     \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void flat3r2w(const double2 *A, const double2 *B, double2 *C, double2 *D, long n2,
                         double al) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) {
        double2 a = A[i], b = B[i], c = C[i];
        c.x += al * b.x;
        c.y += al * b.y;
        C[i] = c;
        D[i] = make_double2(a.x + al * b.x, a.y + al * b.y);
    }
}

__global__ void flat2r1w(const double2 *A, double2 *B, long n2, double al) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) {
        double2 a = A[i], b = B[i];
        B[i] = make_double2(b.x - al * a.x, b.y - al * a.y);
    }
}

__global__ void flatread(const double2 *A, const double2 *B, const double2 *C, long n2, double *out) {
    double s = 0;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) {
        double2 a = A[i], b = B[i], c = C[i];
        s += a.x + b.y + c.x;
    }
    if (s == 12345.0) out[0] = s;
}

// wave = residue j of chunk t for 128 columns; 8 WGs of a (block, chunk) pair XCD-grouped
__global__ void __launch_bounds__(256) lane3r2w(const double *A, const double *B, double *C,
                                                double *D, long n, long ld, int ncb, int nch,
                                                double al) {
    const int b = blockIdx.x;
    const int grp = b >> 6, r = b & 63;
    const int sub = r & 7, part = r >> 3;
    const int pair = grp * 8 + sub;
    if (pair >= ncb * nch) return;
    const int cb = pair % ncb, t = pair / ncb;
    const int j = part * 4 + (threadIdx.x >> 6);
    const long c = (long)cb * 128 + (threadIdx.x & 63) * 2;
    const long len = (n + nch - 1) / nch, a0 = t * len;
    long a1 = a0 + len;
    if (a1 > n) a1 = n;
    for (long row = a0 + j; row < a1; row += 32) {
        const long o = row * ld + c;
        double2 av = *(const double2 *)(A + o), bv = *(const double2 *)(B + o), cv = *(double2 *)(C + o);
        cv.x += al * bv.x;
        cv.y += al * bv.y;
        *(double2 *)(C + o) = cv;
        *(double2 *)(D + o) = make_double2(av.x + al * bv.x, av.y + al * bv.y);
    }
}

// lane3r2w plus gathers of rows i-1 and i+1 of A and B (a path graph's SpMV
// recompute, as k_cg_pq does); SYNC: barrier every row step (WG lockstep)
template <bool SYNC>
__global__ void __launch_bounds__(256) lane_gather(const double *A, const double *B, double *C,
                                                   double *D, long n, long ld, int ncb, int nch,
                                                   double al) {
    const int b = blockIdx.x;
    const int grp = b >> 6, r = b & 63;
    const int sub = r & 7, part = r >> 3;
    const int pair = grp * 8 + sub;
    if (pair >= ncb * nch) return;
    const int cb = pair % ncb, t = pair / ncb;
    const int j = part * 4 + (threadIdx.x >> 6);
    const long c = (long)cb * 128 + (threadIdx.x & 63) * 2;
    const long len = (n + nch - 1) / nch, a0 = t * len;
    long a1 = a0 + len;
    if (a1 > n) a1 = n;
    const long steps = (len + 31) / 32;
    for (long s = 0; s < steps; ++s) {
        const long row = a0 + j + 32 * s;
        if (row < a1) {
            const long o = row * ld + c;
            const long om = (row > 0 ? row - 1 : row) * ld + c, op = (row + 1 < n ? row + 1 : row) * ld + c;
            double2 av = *(const double2 *)(A + o), bv = *(const double2 *)(B + o),
                    cv = *(double2 *)(C + o);
            double2 am = *(const double2 *)(A + om), bm = *(const double2 *)(B + om);
            double2 ap = *(const double2 *)(A + op), bp = *(const double2 *)(B + op);
            cv.x += al * bv.x;
            cv.y += al * bv.y;
            *(double2 *)(C + o) = cv;
            double px = av.x + al * bv.x, py = av.y + al * bv.y;
            px += (am.x + al * bm.x) * 0.25 + (ap.x + al * bp.x) * 0.5;
            py += (am.y + al * bm.y) * 0.25 + (ap.y + al * bp.y) * 0.5;
            *(double2 *)(D + o) = make_double2(px, py);
        }
        if (SYNC) __syncthreads();
    }
}

// NB gathered rows at offsets +-1, +-3 (clamped) of A and B, fold in order
template <int NB>
__global__ void __launch_bounds__(256) lane_gnb(const double *A, const double *B, double *C,
                                                double *D, long n, long ld, int ncb, int nch,
                                                double al) {
    const int b = blockIdx.x;
    const int grp = b >> 6, r = b & 63;
    const int sub = r & 7, part = r >> 3;
    const int pair = grp * 8 + sub;
    if (pair >= ncb * nch) return;
    const int cb = pair % ncb, t = pair / ncb;
    const int j = part * 4 + (threadIdx.x >> 6);
    const long c = (long)cb * 128 + (threadIdx.x & 63) * 2;
    const long len = (n + nch - 1) / nch, a0 = t * len;
    long a1 = a0 + len;
    if (a1 > n) a1 = n;
    const int offs[4] = {-1, 1, -3, 3};
    for (long row = a0 + j; row < a1; row += 32) {
        const long o = row * ld + c;
        double2 bv = *(const double2 *)(B + o), cv = *(double2 *)(C + o);
        cv.x += al * bv.x;
        cv.y += al * bv.y;
        *(double2 *)(C + o) = cv;
        double2 ga[NB + 1], gb[NB + 1];
#pragma unroll
        for (int q = 0; q <= NB; ++q) {
            long rr = q == 0 ? row : row + offs[q - 1];
            rr = rr < 0 ? 0 : (rr >= n ? n - 1 : rr);
            ga[q] = *(const double2 *)(A + rr * ld + c);
            gb[q] = *(const double2 *)(B + rr * ld + c);
        }
        double px = 0, py = 0;
#pragma unroll
        for (int q = 0; q <= NB; ++q) {
            px = px + 0.5 * (ga[q].x + al * gb[q].x);
            py = py + 0.5 * (ga[q].y + al * gb[q].y);
        }
        *(double2 *)(D + o) = make_double2(px, py);
    }
}

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : 22662;
    long k = argc > 2 ? atol(argv[2]) : 2674;
    long ld = (k + 7) / 8 * 8;
    long ncb = (k + 127) / 128;
    ld = ncb * 128 > ld ? ncb * 128 : ld;  // keep the lane kernel in bounds
    size_t bytes = (size_t)n * ld * 8;
    double *A, *B, *C, *D, *o;
    CK(hipMalloc(&A, bytes));
    CK(hipMalloc(&B, bytes));
    CK(hipMalloc(&C, bytes));
    CK(hipMalloc(&D, bytes));
    CK(hipMalloc(&o, 8));
    CK(hipMemset(A, 0, bytes));
    CK(hipMemset(B, 0, bytes));
    CK(hipMemset(C, 0, bytes));
    CK(hipMemset(D, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    long n2 = (long)n * ld / 2;
    const double algo = (double)n * k * 8;  // bytes of one n x k array
    int reps = 50;
    auto run = [&](const char *name, double arrays, auto launch) {
        for (int w = 0; w < 5; ++w) launch();
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-10s %8.4f ms  %7.1f GB/s (algorithmic, %.0f arrays of %.1f MB)\n", name, ms,
               arrays * algo / ms / 1e6, arrays, algo / 1e6);
    };
    for (int g : {1024, 2048, 4096, 8192}) {
        printf("grid %d\n", g);
        run("flat3r2w", 5, [&] { flat3r2w<<<g, 256>>>((double2 *)A, (double2 *)B, (double2 *)C, (double2 *)D, n2, 0.5); });
        run("flat2r1w", 3, [&] { flat2r1w<<<g, 256>>>((double2 *)A, (double2 *)B, n2, 0.5); });
        run("flatread", 3, [&] { flatread<<<g, 256>>>((double2 *)A, (double2 *)B, (double2 *)C, n2, o); });
    }
    int nch = 8;
    int grid = ((ncb * nch + 7) / 8) * 64;
    run("lane3r2w", 5, [&] { lane3r2w<<<grid, 256>>>(A, B, C, D, n, ld, (int)ncb, nch, 0.5); });
    run("lanegath", 5, [&] { lane_gather<false><<<grid, 256>>>(A, B, C, D, n, ld, (int)ncb, nch, 0.5); });
    run("lanegnb2", 5, [&] { lane_gnb<2><<<grid, 256>>>(A, B, C, D, n, ld, (int)ncb, nch, 0.5); });
    run("lanegnb3", 5, [&] { lane_gnb<3><<<grid, 256>>>(A, B, C, D, n, ld, (int)ncb, nch, 0.5); });
    run("lanegnb4", 5, [&] { lane_gnb<4><<<grid, 256>>>(A, B, C, D, n, ld, (int)ncb, nch, 0.5); });
    run("lanegsyn", 5, [&] { lane_gather<true><<<grid, 256>>>(A, B, C, D, n, ld, (int)ncb, nch, 0.5); });
    CK(hipDeviceSynchronize());
    return 0;
}
