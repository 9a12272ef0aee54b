// hbm_roofline.hip -- measured HBM ceilings on this MI355X for the access
// shapes the sort passes use (16-byte lanes, 2 x bytes moved per key):
//   copy      out[i] = in[i]            (separate buffers, like the tile sort)
//   inplace   a[i] = f(a[i])            (in place, like the merge/ROWS passes)
//   read      sum(a)                    (read only)
//   write     a[i] = c                  (write only)
// Each shape is timed with hipEvents over several launches at 4 GiB, for a
// one-shot grid (one 16-byte vector x UNROLL per lane) and a persistent
// grid-stride grid.  Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_roofline.hip
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

template <int U>
__global__ void copy_oneshot(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t nv) {
    size_t i = ((size_t)blockIdx.x * blockDim.x * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = in[i + (size_t)u * blockDim.x];
#pragma unroll
    for (int u = 0; u < U; ++u) out[i + (size_t)u * blockDim.x] = v[u];
}

template <int U>
__global__ void inplace_oneshot(u32x4* a, size_t nv) {
    size_t i = ((size_t)blockIdx.x * blockDim.x * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = a[i + (size_t)u * blockDim.x];
#pragma unroll
    for (int u = 0; u < U; ++u) a[i + (size_t)u * blockDim.x] = v[u] ^ 1u;
}

__global__ void copy_persistent(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t nv) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

__global__ void read_only(const u32x4* __restrict__ a, size_t nv, unsigned* sink) {
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x)
        acc ^= a[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) *sink = 1;
}

__global__ void write_only(u32x4* a, size_t nv) {
    const u32x4 c = {1, 2, 3, 4};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x)
        a[i] = c;
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

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : (4ull << 30));
    const size_t nv = bytes / 16;
    u32x4 *a, *b;
    unsigned* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    const int reps = 10;
    auto report = [&](const char* name, double ms, double moved) {
        printf("{\"shape\": \"%s\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", name, bytes, ms,
               moved / (ms * 1e-3) / 1e9);
    };
    report("copy_u1", time_ms([&] { copy_oneshot<1><<<nv / 256, 256>>>(a, b, nv); }, reps), 2.0 * bytes);
    report("copy_u4", time_ms([&] { copy_oneshot<4><<<nv / 1024, 256>>>(a, b, nv); }, reps), 2.0 * bytes);
    report("copy_u8", time_ms([&] { copy_oneshot<8><<<nv / 2048, 256>>>(a, b, nv); }, reps), 2.0 * bytes);
    report("inplace_u1", time_ms([&] { inplace_oneshot<1><<<nv / 256, 256>>>(a, nv); }, reps), 2.0 * bytes);
    report("inplace_u4", time_ms([&] { inplace_oneshot<4><<<nv / 1024, 256>>>(a, nv); }, reps), 2.0 * bytes);
    report("inplace_u8", time_ms([&] { inplace_oneshot<8><<<nv / 2048, 256>>>(a, nv); }, reps), 2.0 * bytes);
    for (int g : {1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "copy_persistent_g%d", g);
        report(nm, time_ms([&] { copy_persistent<<<g, 256>>>(a, b, nv); }, reps), 2.0 * bytes);
    }
    report("read", time_ms([&] { read_only<<<4096, 256>>>(a, nv, sink); }, reps), 1.0 * bytes);
    report("write", time_ms([&] { write_only<<<4096, 256>>>(b, nv); }, reps), 1.0 * bytes);
    CK(hipFree(a));
    CK(hipFree(b));
    return 0;
}
