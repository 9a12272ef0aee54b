// mall_probe.hip -- how fast are repeated in-place passes over a chunk that
// stays resident in the 256 MiB Infinity Cache (MALL)?
//
// The sort's passes after the first one of a level only touch keys inside
// segments of 2^(hi+1) keys, so a schedule can run several passes over one
// chunk before moving to the next.  This probe measures the rate of such a
// schedule: a 4 GiB buffer is walked chunk by chunk, each chunk gets P
// in-place read+write passes (separate launches), for chunk sizes 8..512 MiB
// and default vs non-temporal access.  Rate = P * 2 * 4 GiB / time.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mall_probe.hip -o tools/bin/mall_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                      \
    do {                                                           \
        hipError_t e = (x);                                        \
        if (e != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
            exit(1);                                               \
        }                                                          \
    } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void inplace(u32x4* a) {
    const size_t i = ((size_t)blockIdx.x * 256 * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        v[u] = NT ? __builtin_nontemporal_load(a + i + (size_t)u * 256) : a[i + (size_t)u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (NT) __builtin_nontemporal_store(v[u] ^ 1u, a + i + (size_t)u * 256);
        else a[i + (size_t)u * 256] = v[u] ^ 1u;
    }
}

template <bool NT>
double run(u32x4* a, size_t total, size_t chunk, int passes, hipGraphExec_t* gx) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t nvc = chunk / 16;
    const unsigned grid = (unsigned)(nvc / (256 * 4));
    hipGraph_t g;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (size_t off = 0; off < total; off += chunk)
        for (int p = 0; p < passes; ++p) inplace<4, NT><<<grid, 256, 0, s>>>(a + off / 16);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(gx, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipGraphLaunch(*gx, s));
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(*gx, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    CK(hipGraphExecDestroy(*gx));
    CK(hipStreamDestroy(s));
    return best;
}

int main(int argc, char** argv) {
    const size_t total = argc > 1 ? strtoull(argv[1], nullptr, 0) : (4ull << 30);
    const int passes = argc > 2 ? atoi(argv[2]) : 8;
    u32x4* a;
    CK(hipMalloc(&a, total));
    CK(hipMemset(a, 1, total));
    for (size_t mib : {8, 16, 32, 64, 128, 256, 512, 4096}) {
        const size_t chunk = mib << 20;
        if (chunk > total) continue;
        for (int nt = 0; nt < 2; ++nt) {
            hipGraphExec_t gx;
            const double ms = nt ? run<true>(a, total, chunk, passes, &gx) : run<false>(a, total, chunk, passes, &gx);
            printf("{\"chunk_MiB\": %zu, \"nt\": %d, \"passes\": %d, \"ms\": %.3f, \"GBs\": %.1f, \"ms_per_pass\": %.4f}\n",
                   mib, nt, passes, ms, passes * 2.0 * total / (ms * 1e-3) / 1e9, ms / passes);
            fflush(stdout);
        }
    }
    CK(hipFree(a));
    return 0;
}
