// Measurement probe only (not product code): how fast the library radix sort
// runs on this GPU for 2^k u32 / u64 keys, as a yardstick for the local sort.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/rocprim_probe.hip -o /tmp/rp && /tmp/rp 30 4
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

template <typename K>
__global__ void fill(K* a, size_t n, uint64_t seed) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    a[i] = (K)(z ^ (z >> 31));
}

template <typename K>
int run(int lg) {
    size_t n = (size_t)1 << lg;
    K *a, *b;
    if (hipMalloc(&a, n * sizeof(K)) || hipMalloc(&b, n * sizeof(K))) return 1;
    size_t tmp = 0;
    rocprim::radix_sort_keys(nullptr, tmp, a, b, n);
    void* t;
    if (hipMalloc(&t, tmp)) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int it = 0; it < 6; ++it) {
        fill<<<(unsigned)((n + 255) / 256), 256>>>(a, n, 12345 + it);
        hipEventRecord(e0);
        rocprim::radix_sort_keys(t, tmp, a, b, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"keys\": %zu, \"key_bytes\": %zu, \"ms\": %.3f, \"gkeys_s\": %.2f}\n", n, sizeof(K), ms, n / ms / 1e6);
    }
    return 0;
}

int main(int argc, char** argv) {
    int lg = argc > 1 ? atoi(argv[1]) : 30, kb = argc > 2 ? atoi(argv[2]) : 4;
    return kb == 8 ? run<uint64_t>(lg) : run<uint32_t>(lg);
}
