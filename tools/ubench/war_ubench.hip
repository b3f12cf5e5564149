// war_ubench.hip -- (1) does a VALU write to a DS instruction's address/data
// VGPR right after the DS issue corrupt the in-flight DS op on gfx950?
// (2) issue cost of ds_read_u8 / ds_write_b8 / v_add_u32_sdwa vs active lanes.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench/war_ubench.hip -o tools/ubench/war_ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint64_t memtime() { return __builtin_amdgcn_s_memtime(); }

// out[t*8 + i]: i=0 read-after-addr-overwrite, 1 same with 4 queued reads ahead,
// 2 write-after-addr-overwrite (value found at the original address),
// 3 value found at the overwritten address, 4 write-after-data-overwrite
__global__ void __launch_bounds__(64) war_kernel(uint32_t *out)
{
    __shared__ uint8_t S[65536];
    const uint32_t t = threadIdx.x;
    for (int i = t; i < 65536; i += 64) S[i] = (uint8_t)(i >> 8);   // S[(k<<8)|c] = k
    __syncthreads();
    uint32_t a = (1u << 8) | t, b = (2u << 8) | t, r, q0, q1, q2, q3;
    asm volatile("ds_read_u8 %[r], %[a]\n\tv_mov_b32 %[a], %[b]\n\ts_waitcnt lgkmcnt(0)"
                 : [r] "=&v"(r), [a] "+v"(a) : [b] "v"(b) : "memory");
    out[t * 8 + 0] = r;                                   // expect 1
    a = (1u << 8) | t;
    asm volatile("ds_read_u8 %[q0], %[b]\n\tds_read_u8 %[q1], %[b]\n\tds_read_u8 %[q2], %[b]\n\tds_read_u8 %[q3], %[b]\n\t"
                 "ds_read_u8 %[r], %[a]\n\tv_mov_b32 %[a], %[b]\n\ts_waitcnt lgkmcnt(0)"
                 : [r] "=&v"(r), [a] "+v"(a), [q0] "=&v"(q0), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3)
                 : [b] "v"(b) : "memory");
    out[t * 8 + 1] = r + 16 * (q0 + q1 + q2 + q3 - 8);   // expect 1
    a = (3u << 8) | t;
    uint32_t c = (4u << 8) | t, d = 0xAB;
    asm volatile("ds_read_u8 %[q0], %[b]\n\tds_read_u8 %[q1], %[b]\n\tds_read_u8 %[q2], %[b]\n\tds_read_u8 %[q3], %[b]\n\t"
                 "ds_write_b8 %[a], %[d]\n\tv_mov_b32 %[a], %[c]\n\tv_mov_b32 %[d], 0xCD\n\ts_waitcnt lgkmcnt(0)"
                 : [a] "+v"(a), [d] "+v"(d), [q0] "=&v"(q0), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3)
                 : [b] "v"(b), [c] "v"(c) : "memory");
    out[t * 8 + 2] = S[(3u << 8) | t];                    // expect 0xAB
    out[t * 8 + 3] = S[(4u << 8) | t];                    // expect 4
}

#define R8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define OPRD(n) "ds_read_u8 %[r" #n "], %[a]\n\t"
#define OPWR(n) "ds_write_b8 %[a], %[r" #n "] offset:" #n "\n\t"
#define OPVA(n) "v_add_u32_sdwa %[r" #n "], %[a], %[r" #n "] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_0\n\t"
#define OPVP(n) "v_add_u32 %[r" #n "], %[a], %[r" #n "]\n\t"
#define RREGS [r0] "+v"(r[0]), [r1] "+v"(r[1]), [r2] "+v"(r[2]), [r3] "+v"(r[3]), [r4] "+v"(r[4]), [r5] "+v"(r[5]), \
    [r6] "+v"(r[6]), [r7] "+v"(r[7])
template <int OP>
__global__ void __launch_bounds__(64) issue_kernel(uint64_t *cyc, int iters, int lanes)
{
    __shared__ uint8_t S[65536];
    if ((int)threadIdx.x >= lanes) return;
    uint32_t r[8];
    for (int i = 0; i < 8; ++i) r[i] = i * 7 + threadIdx.x;
    const uint32_t a = threadIdx.x * 4;
    const uint64_t t0 = memtime();
    for (int it = 0; it < iters; ++it) {
        if (OP == 0) asm volatile(R8(OPRD) R8(OPRD) "s_waitcnt lgkmcnt(0)\n\t" : RREGS : [a] "v"(a) : "memory");
        if (OP == 1) asm volatile(R8(OPWR) R8(OPWR) "s_waitcnt lgkmcnt(0)\n\t" : RREGS : [a] "v"(a) : "memory");
        if (OP == 2) asm volatile(R8(OPVA) R8(OPVA) : RREGS : [a] "v"(a) : "memory");
        if (OP == 3) asm volatile(R8(OPVP) R8(OPVP) : RREGS : [a] "v"(a) : "memory");
    }
    const uint64_t t1 = memtime();
    uint32_t acc = 0;
    for (int i = 0; i < 8; ++i) acc ^= r[i];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    if (acc == 0x12345u) S[threadIdx.x] = 1, cyc[1 << 20] = S[threadIdx.x ^ 1];
}

int main()
{
    uint32_t *d_out; uint64_t *d_cyc;
    CHECK(hipMalloc(&d_out, 64 * 8 * 4));
    CHECK(hipMalloc(&d_cyc, (1 << 20) * 8 + 8));
    CHECK(hipMemset(d_out, 0, 64 * 8 * 4));
    hipLaunchKernelGGL(war_kernel, dim3(1), dim3(64), 0, 0, d_out);
    CHECK(hipDeviceSynchronize());
    uint32_t h[64 * 8];
    CHECK(hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost));
    int bad[4] = {0, 0, 0, 0};
    const uint32_t expect[4] = {1, 1, 0xAB, 4};
    for (int t = 0; t < 64; ++t) for (int i = 0; i < 4; ++i) bad[i] += h[t * 8 + i] != expect[i];
    printf("{\n \"war\": {\"read_addr_overwrite_bad_lanes\": %d, \"queued_read_addr_overwrite_bad_lanes\": %d, "
           "\"write_addr_data_overwrite_bad_lanes\": %d, \"write_landed_elsewhere_bad_lanes\": %d, "
           "\"sample\": [%u, %u, %u, %u]},\n", bad[0], bad[1], bad[2], bad[3], h[0], h[1], h[2], h[3]);
    const char *names[4] = {"ds_read_u8", "ds_write_b8", "v_add_u32_sdwa", "v_add_u32"};
    const int lanes[5] = {64, 32, 16, 4, 1};
    const int iters = 4096;
    for (int op = 0; op < 4; ++op) {
        printf(" \"issue_%s\": {", names[op]);
        for (int li = 0; li < 5; ++li) {
            if (op == 0) hipLaunchKernelGGL(issue_kernel<0>, dim3(1), dim3(64), 0, 0, d_cyc, iters, lanes[li]);
            if (op == 1) hipLaunchKernelGGL(issue_kernel<1>, dim3(1), dim3(64), 0, 0, d_cyc, iters, lanes[li]);
            if (op == 2) hipLaunchKernelGGL(issue_kernel<2>, dim3(1), dim3(64), 0, 0, d_cyc, iters, lanes[li]);
            if (op == 3) hipLaunchKernelGGL(issue_kernel<3>, dim3(1), dim3(64), 0, 0, d_cyc, iters, lanes[li]);
            CHECK(hipDeviceSynchronize());
            uint64_t c0; CHECK(hipMemcpy(&c0, d_cyc, 8, hipMemcpyDeviceToHost));
            printf("\"lanes%d\": %.2f%s", lanes[li], (double)c0 / iters / 16, li < 4 ? ", " : "");
        }
        printf("}%s\n", op < 3 ? "," : "");
    }
    printf("}\n");
    return 0;
}
