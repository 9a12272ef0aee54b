// hbm_shapes.hip -- in-place streaming shapes of the sort passes, timed at 4 GiB.
// Each variant reads every 16-byte vector once and writes it back once
// (a[i] ^= 1), like one sort pass.  Variants:
//   U loads per lane before the stores (U = 1, 4, 8), workgroup of T lanes;
//   cache policy: plain, non-temporal loads, non-temporal stores, both;
//   grid: one-shot (one chunk per workgroup) or persistent (grid-stride).
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_shapes.hip -o tools/bin/hbm_shapes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

template <int U, int T, bool NTL, bool NTS>
__global__ __launch_bounds__(T) void inplace(u32x4* a, size_t nchunks) {
    for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        u32x4* p = a + c * (size_t)(U * T) + threadIdx.x;
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NTL ? __builtin_nontemporal_load(p + u * T) : p[u * T];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32x4 w = v[u] ^ 1u;
            if (NTS) __builtin_nontemporal_store(w, p + u * T);
            else p[u * T] = w;
        }
    }
}

template <typename F>
static double time_ms(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

template <int U, int T, bool NTL, bool NTS>
static void run(u32x4* a, size_t bytes, const char* tag) {
    const size_t nv = bytes / 16, nchunks = nv / (U * T);
    int per_cu = 0, cus = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, inplace<U, T, NTL, NTS>, T, 0));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int persistent = 0; persistent < 2; ++persistent) {
        const size_t grid = persistent ? (size_t)per_cu * cus : nchunks;
        const double ms = time_ms([&] { inplace<U, T, NTL, NTS><<<(unsigned)grid, T>>>(a, nchunks); }, 10);
        printf("{\"shape\": \"%s\", \"U\": %d, \"T\": %d, \"nt_load\": %d, \"nt_store\": %d, "
               "\"persistent\": %d, \"ms\": %.4f, \"GBs\": %.1f}\n",
               tag, U, T, (int)NTL, (int)NTS, persistent, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    }
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : (4ull << 30));
    u32x4* a;
    CK(hipMalloc(&a, bytes));
    CK(hipMemset(a, 1, bytes));
    run<1, 256, false, false>(a, bytes, "inplace");
    run<1, 256, true, true>(a, bytes, "inplace");
    run<8, 512, false, false>(a, bytes, "tile64K");
    run<8, 512, true, false>(a, bytes, "tile64K");
    run<8, 512, false, true>(a, bytes, "tile64K");
    run<8, 512, true, true>(a, bytes, "tile64K");
    run<4, 512, false, false>(a, bytes, "tile32K");
    run<4, 512, true, true>(a, bytes, "tile32K");
    run<8, 256, false, false>(a, bytes, "tile32K_256");
    run<8, 256, true, true>(a, bytes, "tile32K_256");
    run<2, 256, false, false>(a, bytes, "u2");
    run<2, 256, true, true>(a, bytes, "u2");
    CK(hipFree(a));
    return 0;
}
