// valu_probe.hip -- measurement only: VALU issue rate of the compare-exchange
// instructions the SORT tile is made of (v_min_u32/v_max_u32 pairs, DPP move +
// v_med3_u32), at 1..8 waves per SIMD.  Prints SIMD cycles per wave64
// instruction (2.4 GHz assumed; 1024 SIMDs).  Decides whether the bitonic SORT
// pass is at its VALU floor (4 cycles per instruction) or can go faster (2).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int NK = 32;     // keys per lane
constexpr int ROUNDS = 256;

__device__ __forceinline__ void cx(uint32_t& a, uint32_t& b) {
    uint32_t lo, hi;
    asm volatile("v_min_u32 %0, %2, %3\n\tv_max_u32 %1, %2, %3" : "=&v"(lo), "=&v"(hi) : "v"(a), "v"(b));
    a = lo;
    b = hi;
}

// 16 independent pairs per stage, 5 stages per round (strides 16..1): 160 VALU per round
__global__ void k_cx(uint32_t* out, uint32_t seed) {
    uint32_t v[NK];
#pragma unroll
    for (int i = 0; i < NK; ++i) v[i] = (threadIdx.x * 2654435761u) ^ (seed + i * 40503u);
    for (int r = 0; r < ROUNDS; ++r) {
#pragma unroll
        for (int s = 16; s >= 1; s >>= 1)
#pragma unroll
            for (int i = 0; i < NK; ++i)
                if (!(i & s)) cx(v[i], v[i | s]);
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < NK; ++i) x ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// cross-lane stage: partner via DPP row_shr:1 style move (quad_perm swap), then
// med3(v, p, sel) -- 2 VALU per key per stage; NK independent keys per stage
__global__ void k_dpp(uint32_t* out, uint32_t seed) {
    uint32_t v[NK];
#pragma unroll
    for (int i = 0; i < NK; ++i) v[i] = (threadIdx.x * 2654435761u) ^ (seed + i * 40503u);
    const uint32_t sel = (threadIdx.x & 1) ? 0xFFFFFFFFu : 0u;
    for (int r = 0; r < ROUNDS; ++r) {
#pragma unroll
        for (int s = 0; s < 5; ++s)
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                uint32_t p;
                // quad_perm [1,0,3,2]: lanes 2k <-> 2k+1
                asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=&v"(p) : "v"(v[i]));
                uint32_t m;
                asm volatile("v_med3_u32 %0, %1, %2, %3" : "=&v"(m) : "v"(v[i]), "v"(p), "v"(sel));
                v[i] = m;
            }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < NK; ++i) x ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    uint32_t* d = nullptr;
    const int maxthreads = 256 * 8 * 4 * 64 * 2;
    CHK(hipMalloc(&d, (size_t)maxthreads * 4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const double clk = 2.4e9, simds = 1024;
    for (int kind = 0; kind < 2; ++kind) {
        const double per_wave = kind == 0 ? (double)ROUNDS * 5 * 16 * 2 : (double)ROUNDS * 5 * NK * 2;
        for (int wps = 1; wps <= 8; wps *= 2) {
            const int threads = 256;  // 4 waves per block: one per SIMD
            const int blocks = 256 * wps;
            for (int rep = 0; rep < 3; ++rep) {
                CHK(hipEventRecord(a, 0));
                if (kind == 0) k_cx<<<blocks, threads>>>(d, rep);
                else k_dpp<<<blocks, threads>>>(d, rep);
                CHK(hipEventRecord(b, 0));
                CHK(hipEventSynchronize(b));
                float ms = 0;
                CHK(hipEventElapsedTime(&ms, a, b));
                const double waves = blocks * 4.0;
                const double cyc = ms * 1e-3 * clk * simds / (waves * per_wave);
                if (rep == 2)
                    printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_valu\": %.3f}\n",
                           kind == 0 ? "min_max" : "dpp_med3", wps, ms, cyc);
            }
        }
    }
    return 0;
}
