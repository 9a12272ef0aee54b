// fetch_cal.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access shapes the sort's kernels use, each on a known byte count
// (MI355X_MICROARCH.md, HBM: "other access widths are uncalibrated: calibrate
// on a known byte count in your own access pattern").  One launch per shape,
// over a 2 GiB buffer (far past the 256 MiB Infinity Cache):
//   v16      16-B loads per lane, streaming (the guide's calibrated case)
//   v8       8-B loads per lane, streaming (u64 keys, u64 fences)
//   v4       4-B loads per lane, streaming (u32 merge levels)
//   lds4     global_load_lds_dword, 4 B per lane into LDS, 256 B per wave
//            instruction in rows of 512 keys (k_mergek<u32>'s row loads)
//   line128  one thread per distinct random 128-B line, 8 x 16-B loads
//            (k_bounds' line probe)
//   probe4   one thread per distinct random 128-B line, one 4-B load
//            (k_bounds' galloping / bisection probes)
//   st16     16-B non-temporal stores per lane, streaming (every pass's output)
//   st4      4-B stores per lane, streaming (chunk-edge stores)
// Every kernel name starts with "cal_" so a --pmc run can select them.
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_cal.hip -o tools/bin/fetch_cal
// Run:   rocprofv3 --pmc FETCH_SIZE -d DIR -o fetch --output-format csv -- tools/bin/fetch_cal
//        rocprofv3 --pmc WRITE_SIZE ... ; tools/fetch_cal.py DIR > profiles/fetch_cal.json
// It prints one JSON line per shape with its known bytes (the same order as the launches).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                      \
    do {                                                           \
        hipError_t e = (x);                                        \
        if (e != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
            exit(1);                                               \
        }                                                          \
    } while (0)

// streaming loads of T per lane, 8 per lane per block of 256 lanes; the xor
// of what a lane read goes to one word per block (negligible writes)
template <typename T>
__global__ __launch_bounds__(256) void cal_load(const T* __restrict__ a, uint32_t* __restrict__ sink) {
    const T* p = a + (size_t)blockIdx.x * 2048 + threadIdx.x;
    T x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = __builtin_nontemporal_load(p + u * 256);
    uint32_t s = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        if constexpr (sizeof(T) == 4) s ^= x[u];
        else if constexpr (sizeof(T) == 8) s ^= x[u].x ^ x[u].y;
        else s ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
    }
    if (s == 0x9E3779B1u) sink[blockIdx.x] = s;  // data-dependent, practically never
}

// k_mergek<u32>'s row loads: a 512-lane block fills 32 KiB of LDS with
// global_load_lds_dword, each wave 64 consecutive keys per instruction
__global__ __launch_bounds__(512) void cal_lds4(const uint32_t* __restrict__ a, uint32_t* __restrict__ sink) {
    __shared__ uint32_t t[8192];
    const int tid = threadIdx.x, w0 = __builtin_amdgcn_readfirstlane(tid & ~63);
    const uint32_t* src = a + (size_t)blockIdx.x * 8192;
#pragma unroll
    for (int j = 0; j < 16; ++j)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + j * 512 + tid),
                                         (__attribute__((address_space(3))) void*)(t + j * 512 + w0), 4, 0, 0);
    __syncthreads();
    if (t[tid * 16] == 0x9E3779B1u) sink[blockIdx.x] = tid;
}

// one thread per distinct 128-B line of the buffer (a bijection of the line
// index: odd multiplier modulo a power of two)
__device__ __forceinline__ size_t line_of(size_t i, size_t nlines) { return (i * 0x9E3779B1ull) & (nlines - 1); }

__global__ __launch_bounds__(256) void cal_line128(const u32x4* __restrict__ a, size_t nlines, size_t nprobe,
                                                   uint32_t* __restrict__ sink) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nprobe) return;
    const u32x4* p = a + line_of(i, nlines) * 8;
    u32x4 q[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) q[u] = p[u];
    uint32_t s = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) s ^= q[u].x ^ q[u].y ^ q[u].z ^ q[u].w;
    if (s == 0x9E3779B1u) sink[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void cal_probe4(const uint32_t* __restrict__ a, size_t nlines, size_t nprobe,
                                                  uint32_t* __restrict__ sink) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nprobe) return;
    const uint32_t s = a[line_of(i, nlines) * 32 + (i & 31)];
    if (s == 0x9E3779B1u) sink[blockIdx.x] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void cal_store(T* __restrict__ a) {
    T* p = a + (size_t)blockIdx.x * 2048 + threadIdx.x;
    T v{};
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        if constexpr (sizeof(T) == 16) __builtin_nontemporal_store(v, p + u * 256);
        else p[u * 256] = v;
    }
}

int main(int argc, char** argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 0) : (2ull << 30);
    char* a;
    uint32_t* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&sink, 1 << 24));
    CK(hipMemset(a, 1, bytes));
    CK(hipDeviceSynchronize());
    auto line = [](const char* shape, double rd, double wr) {
        printf("{\"shape\": \"%s\", \"read_bytes\": %.0f, \"write_bytes\": %.0f}\n", shape, rd, wr);
    };
    cal_load<u32x4><<<(unsigned)(bytes / (16 * 2048)), 256>>>((const u32x4*)a, sink);
    line("v16", (double)bytes, 0);
    cal_load<u32x2><<<(unsigned)(bytes / (8 * 2048)), 256>>>((const u32x2*)a, sink);
    line("v8", (double)bytes, 0);
    cal_load<uint32_t><<<(unsigned)(bytes / (4 * 2048)), 256>>>((const uint32_t*)a, sink);
    line("v4", (double)bytes, 0);
    cal_lds4<<<(unsigned)(bytes / (4 * 8192)), 512>>>((const uint32_t*)a, sink);
    line("lds4", (double)bytes, 0);
    const size_t nlines = bytes / 128, nprobe = nlines / 8;  // 1/8 of the lines, spread over the buffer
    cal_line128<<<(unsigned)((nprobe + 255) / 256), 256>>>((const u32x4*)a, nlines, nprobe, sink);
    line("line128", 128.0 * nprobe, 0);
    cal_probe4<<<(unsigned)((nprobe + 255) / 256), 256>>>((const uint32_t*)a, nlines, nprobe, sink);
    line("probe4", 4.0 * nprobe, 0);
    cal_store<u32x4><<<(unsigned)(bytes / (16 * 2048)), 256>>>((u32x4*)a);
    line("st16", 0, (double)bytes);
    cal_store<uint32_t><<<(unsigned)(bytes / (4 * 2048)), 256>>>((uint32_t*)a);
    line("st4", 0, (double)bytes);
    CK(hipDeviceSynchronize());
    CK(hipFree(a));
    CK(hipFree(sink));
    return 0;
}
