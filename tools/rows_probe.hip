// rows_probe.hip -- HBM rate of the sort passes' ACCESS SHAPES with no
// compute: every workgroup copies one 2^LT-key tile (16-byte vectors, one
// tile per workgroup, 1024 lanes x 8 vectors) from `in` to `out`.
//   contig   tile = 2^LT consecutive keys (SORT/MERGE shape)
//   rows R   tile = 2^R rows at stride 2^lo keys x 2^(LT-R) consecutive keys
//            (ROWS shape, lo = hi-R+1, hi = 29)
// Out of place (ping-pong) and in place, and three workgroup->tile maps:
//   0 identity; 1 XCD-contiguous (workgroup b -> tile (b%8)*(T/8) + b/8, so
//   each XCD streams its own 1/8 of the array, assuming round-robin dispatch);
//   2 reversed tile order for odd passes.  Rate = 2 * 4 GiB / time.
// Build: hipcc --offload-arch=gfx950 -O3 tools/rows_probe.hip -o tools/bin/rows_probe
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

constexpr int LT = 15, NT = 1024, LOADS = 8;

// virtual key e of tile `tile` -> global key index (ROWS mapping of bitonic.h)
__device__ __forceinline__ size_t gidx(size_t tile, int e, int R, int hi) {
    if (R == 0) return (tile << LT) + e;
    const int logB = LT - R, lo = hi - R + 1, sh = lo - logB;
    const size_t seg = tile >> sh, lb = tile & (((size_t)1 << sh) - 1);
    const int c = e >> logB, j = e & ((1 << logB) - 1);
    return (seg << (hi + 1)) + ((size_t)c << lo) + (lb << logB) + j;
}

template <bool NT_HINT>
__global__ __launch_bounds__(NT) void tile_copy(const unsigned* in, unsigned* out, int R, int hi, int map) {
    size_t tile = blockIdx.x;
    if (map == 1) tile = (size_t)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
    u32x4 v[LOADS];
#pragma unroll
    for (int k = 0; k < LOADS; ++k) {
        const size_t g = gidx(tile, (k * NT + threadIdx.x) * 4, R, hi);
        v[k] = NT_HINT ? __builtin_nontemporal_load((const u32x4*)(in + g)) : *(const u32x4*)(in + g);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < LOADS; ++k) {
        const size_t g = gidx(tile, (k * NT + threadIdx.x) * 4, R, hi);
        if (NT_HINT) __builtin_nontemporal_store(v[k] ^ 1u, (u32x4*)(out + g));
        else *(u32x4*)(out + g) = v[k] ^ 1u;
    }
}

int main() {
    const size_t n = (size_t)1 << 30, bytes = n * 4;
    unsigned *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned grid = (unsigned)(n >> LT);
    for (int R = 0; R <= 10; ++R) {
        for (int map = 0; map < 2; ++map) {
        for (int inplace = 0; inplace < 1; ++inplace) {
            for (int nt = 0; nt < 2; ++nt) {
                auto go = [&] {
                    if (nt) tile_copy<true><<<grid, NT>>>(a, inplace ? a : b, R, 29, map);
                    else tile_copy<false><<<grid, NT>>>(a, inplace ? a : b, R, 29, map);
                };
                go();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0));
                for (int r = 0; r < 5; ++r) go();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                ms /= 5;
                printf("{\"R\": %d, \"map\": %d, \"inplace\": %d, \"nt\": %d, \"ms\": %.4f, \"GBs\": %.1f}\n", R, map,
                       inplace, nt, ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
                fflush(stdout);
            }
        }
        }
    }
    return 0;
}
