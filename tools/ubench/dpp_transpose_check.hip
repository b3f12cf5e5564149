// Checks the generated 8x8 DPP transpose (zrc4_line_loop.inc's butterflies)
// in isolation: lane l holds chunk c dword d = (l << 16) | (c << 8) | d; after
// the transpose lane 8g+i must hold in chunk slot c the chunk i of lane 8g+c.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

#define ZL_BLOCK(...) ""
#include "../../zsummerx_amd/csrc/zrc4_line_loop.inc"

__global__ void k(uint32_t *out)
{
    const uint32_t l = threadIdx.x;
    u32x32 P;
    for (int c = 0; c < 8; ++c)
        for (int d = 0; d < 4; ++d) P[4 * c + d] = (l << 16) | (c << 8) | d;
    u32x16 X;
    asm volatile("s_nop 4\n\t" ZRC4_LL_TRANSPOSE_P : "+{v[40:71]}"(P), "=&{v[104:119]}"(X) :: "vcc", "memory");
    // final chunk tuple bases are exported by the generator as ZRC4_LL_FINAL_P
    const int fin[8] = {ZRC4_LL_FINAL_P};
    for (int c = 0; c < 8; ++c) {
        const int r = fin[c];
        for (int d = 0; d < 4; ++d) {
            uint32_t v = (r >= 104) ? X[r - 104 + d] : P[r - 40 + d];
            out[(l * 8 + c) * 4 + d] = v;
        }
    }
}

int main()
{
    uint32_t *d, h[64 * 32];
    hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int c = 0; c < 8; ++c)
            for (int dd = 0; dd < 4; ++dd) {
                const uint32_t want = ((uint32_t)((l & ~7) | c) << 16) | ((uint32_t)(l & 7) << 8) | dd;
                const uint32_t got = h[(l * 8 + c) * 4 + dd];
                if (got != want && bad++ < 16)
                    printf("lane %d slot %d d %d: got lane %u chunk %u d %u, want lane %u chunk %u\n", l, c, dd,
                           got >> 16, (got >> 8) & 255, got & 255, want >> 16, (want >> 8) & 255);
            }
    printf("dpp transpose: %d mismatches\n", bad);
    return bad != 0;
}
