// Prints the source lane each DPP control / permlane swap delivers on gfx950
// (semantics check for the in-wave bitonic stages of the SORT pass).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL, int BANK>
__global__ void k_dpp(int* out) {
    const int l = threadIdx.x;
    out[l] = __builtin_amdgcn_update_dpp(-1, l, CTRL, 0xF, BANK, false);
}
__global__ void k_pl16(int* out) {
    const int l = threadIdx.x;
    auto r = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
    out[l] = r[0];
    out[64 + l] = r[1];
}
__global__ void k_pl32(int* out) {
    const int l = threadIdx.x;
    auto r = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
    out[l] = r[0];
    out[64 + l] = r[1];
}
__global__ void k_med3(unsigned* out, unsigned a, unsigned b) {
    const unsigned l = threadIdx.x;
    const unsigned c = (l & 1) ? 0xFFFFFFFFu : 0u;
    const unsigned x = a + l, y = b;
    out[l] = max(min(x, y), min(max(x, y), c));
}

static void show(const char* name, int* d, int n) {
    int h[128];
    hipMemcpy(h, d, n * sizeof(int), hipMemcpyDeviceToHost);
    printf("%-22s", name);
    for (int i = 0; i < n; ++i) printf(" %d", h[i]);
    printf("\n");
}

int main() {
    int* d;
    hipMalloc(&d, 128 * sizeof(int));
#define RUN(C, B, NAME) k_dpp<C, B><<<1, 64>>>(d); show(NAME, d, 64);
    RUN(0xB1, 0xF, "quad_perm xor1")
    RUN(0x4E, 0xF, "quad_perm xor2")
    RUN(0x1B, 0xF, "quad_perm xor3")
    RUN(0x104, 0xF, "row_shl:4")
    RUN(0x114, 0xF, "row_shr:4")
    RUN(0x104, 0x5, "row_shl:4 banks 0,2")
    RUN(0x114, 0xA, "row_shr:4 banks 1,3")
    RUN(0x108, 0x3, "row_shl:8 banks 0,1")
    RUN(0x118, 0xC, "row_shr:8 banks 2,3")
    RUN(0x140, 0xF, "row_mirror")
    RUN(0x141, 0xF, "row_half_mirror")
    k_pl16<<<1, 64>>>(d); show("permlane16_swap", d, 128);
    k_pl32<<<1, 64>>>(d); show("permlane32_swap", d, 128);
    k_med3<<<1, 64>>>((unsigned*)d, 5, 7); show("med3 (5+l,7,odd?max:min)", d, 16);
    hipDeviceSynchronize();
    return 0;
}
