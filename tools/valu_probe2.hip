// valu_probe2.hip -- measurement only: SIMD cycles per wave64 instruction of
// the VALU ops a compare-exchange could be built from, 8 waves per SIMD,
// 16 independent chains per lane (no dependency stalls).  Companion of
// valu_probe.hip (which found v_min/v_max_u32 at ~4.5 cycles).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int NK = 16, ROUNDS = 512;

#define KERNEL(NAME, ASM)                                                                \
    __global__ void NAME(uint32_t* out, uint32_t seed) {                                \
        uint32_t v[NK];                                                                  \
        _Pragma("unroll") for (int i = 0; i < NK; ++i) v[i] = (threadIdx.x * 2654435761u) ^ (seed + i * 40503u); \
        const uint32_t c = seed | 1u;                                                    \
        for (int r = 0; r < ROUNDS; ++r) {                                               \
            _Pragma("unroll") for (int i = 0; i < NK; ++i) asm volatile(ASM : "+v"(v[i]) : "v"(c)); \
        }                                                                                \
        uint32_t x = 0;                                                                  \
        _Pragma("unroll") for (int i = 0; i < NK; ++i) x ^= v[i];                        \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                  \
    }

KERNEL(k_min_u32, "v_min_u32 %0, %0, %1")
KERNEL(k_max_u32, "v_max_u32 %0, %0, %1")
KERNEL(k_min_i32, "v_min_i32 %0, %0, %1")
KERNEL(k_min_f32, "v_min_f32 %0, %0, %1")
KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
KERNEL(k_xor_b32, "v_xor_b32 %0, %0, %1")
KERNEL(k_mov_b32, "v_mov_b32 %0, %1")
KERNEL(k_med3_u32, "v_med3_u32 %0, %0, %1, %1")
KERNEL(k_min3_u32, "v_min3_u32 %0, %0, %1, %1")
KERNEL(k_pk_min_u16, "v_pk_min_u16 %0, %0, %1")
KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL(k_cmp_vcc, "v_cmp_lt_u32 vcc, %0, %1")
KERNEL(k_cmp_sgpr, "v_cmp_lt_u32_e64 s[40:41], %0, %1")
KERNEL(k_sub_co, "v_sub_co_u32 %0, vcc, %0, %1")
KERNEL(k_dpp_mov, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
KERNEL(k_min_dpp, "v_min_u32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    uint32_t* d = nullptr;
    const int blocks = 256 * 8, threads = 256;  // 8 waves per SIMD
    CHK(hipMalloc(&d, (size_t)blocks * threads * 4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    struct { const char* name; kfn f; } ks[] = {
        {"v_min_u32", k_min_u32}, {"v_max_u32", k_max_u32}, {"v_min_i32", k_min_i32}, {"v_min_f32", k_min_f32},
        {"v_add_u32", k_add_u32}, {"v_xor_b32", k_xor_b32}, {"v_mov_b32", k_mov_b32}, {"v_med3_u32", k_med3_u32},
        {"v_min3_u32", k_min3_u32}, {"v_pk_min_u16", k_pk_min_u16},
        {"v_cndmask_b32", k_cndmask}, {"v_cmp_lt_u32 (vcc)", k_cmp_vcc}, {"v_cmp_lt_u32_e64 (sgpr)", k_cmp_sgpr},
        {"v_sub_co_u32", k_sub_co}, {"v_mov_b32_dpp", k_dpp_mov}, {"v_min_u32_dpp", k_min_dpp}};
    const double clk = 2.4e9, simds = 1024, per_wave = (double)ROUNDS * NK;
    for (auto& k : ks) {
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            CHK(hipEventRecord(a, 0));
            k.f<<<blocks, threads>>>(d, rep + 1);
            CHK(hipEventRecord(b, 0));
            CHK(hipEventSynchronize(b));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        const double waves = blocks * 4.0;
        printf("{\"op\": \"%s\", \"waves_per_simd\": 8, \"ms\": %.4f, \"cycles_per_instr\": %.3f}\n", k.name, best,
               best * 1e-3 * clk * simds / (waves * per_wave));
    }
    return 0;
}
