// seg_probe.hip -- rate of repeated in-place sweeps that one workgroup makes
// over its OWN segment inside a single launch (no kernel boundaries, no
// inter-workgroup sync): the access shape of a "segment-local" sort kernel
// that runs several network passes over 2^k keys between one HBM read and
// one HBM write.  Footprint = grid x segment; the sweeps hit L2/Infinity Cache
// while the footprint fits.  Rate = sweeps * 2 * footprint / time.
// Build: hipcc --offload-arch=gfx950 -O3 tools/seg_probe.hip -o tools/bin/seg_probe
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

// NT threads, each moving U 16-byte vectors per step; a segment of `seg`
// vectors is swept `sweeps` times.  Workgroup w walks segments w, w+grid, ...
template <int NT, int U>
__global__ __launch_bounds__(NT) void sweep(u32x4* a, size_t nseg, size_t seg, int sweeps) {
    for (size_t s = blockIdx.x; s < nseg; s += gridDim.x) {
        u32x4* p = a + s * seg;
        for (int r = 0; r < sweeps; ++r) {
            for (size_t i = threadIdx.x; i < seg; i += (size_t)NT * U) {
                u32x4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) v[u] = p[i + (size_t)u * NT];
#pragma unroll
                for (int u = 0; u < U; ++u) p[i + (size_t)u * NT] = v[u] ^ 1u;
            }
            __syncthreads();
        }
    }
}

int main(int argc, char** argv) {
    const size_t total = argc > 1 ? strtoull(argv[1], nullptr, 0) : (4ull << 30);
    u32x4* a;
    CK(hipMalloc(&a, total));
    CK(hipMemset(a, 1, total));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int sweeps : {1, 4, 8}) {
        for (size_t seg_kib : {64, 128, 256, 512, 1024}) {
            for (int per_cu : {1, 2, 4}) {
                const size_t seg = (seg_kib << 10) / 16, nseg = total / (seg * 16);
                const int grid = cus * per_cu;
                auto go = [&] { sweep<512, 8><<<grid, 512>>>(a, nseg, seg, sweeps); };
                go();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0));
                go();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                printf("{\"sweeps\": %d, \"seg_KiB\": %zu, \"wg_per_cu\": %d, \"footprint_MiB\": %zu, \"ms\": %.3f, "
                       "\"GBs\": %.1f}\n",
                       sweeps, seg_kib, per_cu, (size_t)grid * seg_kib / 1024, ms,
                       sweeps * 2.0 * total / (ms * 1e-3) / 1e9);
                fflush(stdout);
            }
        }
    }
    CK(hipFree(a));
    return 0;
}
